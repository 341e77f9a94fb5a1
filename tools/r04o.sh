# Small kernels' VALU (k_scan masks kept for the break walk, DPP block scans, uniform k_dc_sum tile
# index): GPU suite, A/B against the previous build on C2 and C5, then the SQ VALU counters of C2.
set -e
mkdir -p gpurun_out/r04o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o/tests.log 2>&1 || { tail -30 gpurun_out/r04o/tests.log; exit 1; }
tail -2 gpurun_out/r04o/tests.log
AB_REPS=3 bash tools/ab.sh gpurun_out/r04o/c2 base cur
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04o/c5 base cur
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES -d $GRAFT_REPO_ROOT/gpurun_out/r04o/pmc -o valu -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 2 --no-pipeline > $GRAFT_REPO_ROOT/gpurun_out/r04o/pmc.log 2>&1
