set -e
mkdir -p gpurun_out/r03am
timeout -k 10 480 python -u tools/parity_sweep.py --minutes 6 --seed 11 --out gpurun_out/r03am/sweep.json > gpurun_out/r03am/sweep.log 2>&1 || { tail -20 gpurun_out/r03am/sweep.log; exit 1; }
tail -3 gpurun_out/r03am/sweep.log
