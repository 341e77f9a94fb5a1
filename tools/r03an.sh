set -e
mkdir -p gpurun_out/r03an
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03an/tests.log 2>&1 || { tail -30 gpurun_out/r03an/tests.log; exit 1; }
tail -1 gpurun_out/r03an/tests.log
timeout -k 10 480 python -u tools/parity_sweep.py --minutes 6 --seed 12 --out gpurun_out/r03an/sweep.json > gpurun_out/r03an/sweep.log 2>&1 || { tail -5 gpurun_out/r03an/sweep.log; exit 1; }
tail -2 gpurun_out/r03an/sweep.log
