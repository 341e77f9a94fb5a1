set -e
mkdir -p gpurun_out/r03az
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03az/gpu.log 2>&1 || { tail -30 gpurun_out/r03az/gpu.log; exit 1; }
tail -1 gpurun_out/r03az/gpu.log
timeout -k 10 300 python -u tools/parity_sweep.py --minutes 3 --seed 34 --out gpurun_out/r03az/sweep_s34.json > gpurun_out/r03az/sweep.log 2>&1 || { tail -3 gpurun_out/r03az/sweep.log; exit 1; }
tail -1 gpurun_out/r03az/sweep.log
