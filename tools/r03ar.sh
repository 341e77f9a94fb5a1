set -e
mkdir -p gpurun_out/r03ar
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ar/tests.log 2>&1 || { tail -30 gpurun_out/r03ar/tests.log; exit 1; }
tail -1 gpurun_out/r03ar/tests.log
timeout -k 10 420 python -u tools/parity_sweep.py --minutes 3 --seed 14 --out gpurun_out/r03ar/sweep.json > gpurun_out/r03ar/sweep.log 2>&1 || { tail -3 gpurun_out/r03ar/sweep.log; exit 1; }
tail -1 gpurun_out/r03ar/sweep.log
AB_ARGS="--config c2 --steps 40" bash tools/ab.sh gpurun_out/r03ar/ab2 base cur base cur
