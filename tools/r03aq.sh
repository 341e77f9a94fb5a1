set -e
mkdir -p gpurun_out/r03aq
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03aq/tests.log 2>&1 || { tail -30 gpurun_out/r03aq/tests.log; exit 1; }
tail -1 gpurun_out/r03aq/tests.log
timeout -k 10 420 python -u tools/parity_sweep.py --minutes 5 --seed 13 --out gpurun_out/r03aq/sweep.json > gpurun_out/r03aq/sweep.log 2>&1 || { tail -3 gpurun_out/r03aq/sweep.log; exit 1; }
tail -1 gpurun_out/r03aq/sweep.log
AB_ARGS="--config c2 --steps 40" bash tools/ab.sh gpurun_out/r03aq/ab2 base cur base cur
