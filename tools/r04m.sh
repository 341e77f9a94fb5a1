# randomized parity sweep (6 min) and a kernel trace of the default pipelined C2 bench
set -e
mkdir -p gpurun_out/r04m
timeout -k 10 500 python -u tools/parity_sweep.py --minutes 6 --seed 41 --out gpurun_out/r04m/sweep.json > gpurun_out/r04m/sweep.log 2>&1 || { tail -5 gpurun_out/r04m/sweep.log; exit 1; }
tail -1 gpurun_out/r04m/sweep.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04m/tr -o cur -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04m/tr.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04m/tr -name '*kernel_trace.csv' | head -1) 8 > gpurun_out/r04m/timeline_cur.txt
