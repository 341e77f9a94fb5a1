# A/B of the error-bookkeeping / DC-size-16 kernels against the previous commit, then parity sweeps
set -e
mkdir -p gpurun_out/r03av
bash tools/ab.sh gpurun_out/r03av prev cur
bash tools/ab.sh gpurun_out/r03av/2 prev cur
timeout -k 10 420 python -u tools/parity_sweep.py --minutes 5.5 --seed 31 --out gpurun_out/r03av/sweep_s31.json
timeout -k 10 300 python -u tools/parity_sweep.py --minutes 3.5 --seed 32 --fancy --out gpurun_out/r03av/sweep_s32_fancy.json
