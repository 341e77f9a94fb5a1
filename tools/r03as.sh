set -e
mkdir -p gpurun_out/r03as
timeout -k 10 420 python -u tools/parity_sweep.py --minutes 4 --seed 15 --out gpurun_out/r03as/sweep.json > gpurun_out/r03as/sweep.log 2>&1 || { tail -3 gpurun_out/r03as/sweep.log; exit 1; }
tail -1 gpurun_out/r03as/sweep.log
timeout -k 10 420 python -u tools/parity_sweep.py --minutes 4 --seed 16 --fancy --out gpurun_out/r03as/sweep_fancy.json > gpurun_out/r03as/sweep_fancy.log 2>&1 || { tail -3 gpurun_out/r03as/sweep_fancy.log; exit 1; }
tail -1 gpurun_out/r03as/sweep_fancy.log
