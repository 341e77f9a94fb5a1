# Chroma terms from two 512-entry tables (cur) vs the arithmetic form (a0): GPU suite on cur first
# (test_color_exhaustive checks all 2^27 inputs), then C2 and C5 A/B
set -e
mkdir -p gpurun_out/r03bo
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03bo/gpu.log 2>&1 || { tail -30 gpurun_out/r03bo/gpu.log; exit 1; }
tail -1 gpurun_out/r03bo/gpu.log
bash tools/ab.sh gpurun_out/r03bo/c2 cur a0
bash tools/ab.sh gpurun_out/r03bo/c2b a0 cur
bash tools/ab.sh gpurun_out/r03bo/c2c cur a0
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bo/c5 cur a0 a0 cur
