# R/B term pairs by one byte permute of the multiply-add sums (cur) vs shifts + pack (tp0): GPU suite
# on cur first, then C5 (a third 4:4:4) and C1 (4:4:4) A/B
set -e
mkdir -p gpurun_out/r03bp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03bp/gpu.log 2>&1 || { tail -30 gpurun_out/r03bp/gpu.log; exit 1; }
tail -1 gpurun_out/r03bp/gpu.log
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bp/c5 cur tp0
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bp/c5b tp0 cur
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bp/c5c cur tp0
AB_ARGS="--config c1" bash tools/ab.sh gpurun_out/r03bp/c1 cur tp0 cur tp0
