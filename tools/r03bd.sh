# GPU suite on the main build (paired flush with fixed ring reads), then A/B vs ep3 (pointer-stepped record flush)
set -e
mkdir -p gpurun_out/r03bd
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03bd/gpu.log 2>&1 || { tail -30 gpurun_out/r03bd/gpu.log; exit 1; }
tail -1 gpurun_out/r03bd/gpu.log
bash tools/ab.sh gpurun_out/r03bd cur ep3
bash tools/ab.sh gpurun_out/r03bd/2 ep3 cur
bash tools/ab.sh gpurun_out/r03bd/3 cur ep3
