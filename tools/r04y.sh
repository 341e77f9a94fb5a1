# Region divisor cached at parse time (host plan on the critical path between two launches):
# GPU suite, host phase times, A/B against the previous build.
set -e
mkdir -p gpurun_out/r04y
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04y/tests.log 2>&1 || { tail -30 gpurun_out/r04y/tests.log; exit 1; }
tail -2 gpurun_out/r04y/tests.log
JD_HOST_TIMING=1 timeout -k 10 200 python bench.py --steps 8 --warmup 2 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > gpurun_out/r04y/b.json 2> gpurun_out/r04y/host.log
grep -E "^plan|^host plan|^host parse" gpurun_out/r04y/host.log | tail -6
AB_REPS=3 bash tools/ab.sh gpurun_out/r04y/c2 base cur
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04y/c5 base cur
