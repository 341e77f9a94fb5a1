set -e
mkdir -p gpurun_out/r03ab && cd gpurun_out/r03ab && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d trace -o run -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 --steps 12 --warmup 3 \
  --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > bench.log 2>&1
tail -c 400 bench.log
