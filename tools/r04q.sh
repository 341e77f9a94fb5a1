# Round-4 closing measurements: parity sweep (3 min, seed 43), the default bench line, the round
# profile of every config (kernel stats, FETCH/WRITE_SIZE, SQ groups) and a default-pipeline trace.
set -e
mkdir -p gpurun_out/r04q
timeout -k 10 300 python -u tools/parity_sweep.py --minutes 3 --seed 43 --out gpurun_out/r04q/sweep.json > gpurun_out/r04q/sweep.log 2>&1 || { tail -5 gpurun_out/r04q/sweep.log; exit 1; }
tail -1 gpurun_out/r04q/sweep.log
timeout -k 10 400 python bench.py > gpurun_out/r04q/c2_default.json 2> gpurun_out/r04q/c2_default.err
tail -c 400 gpurun_out/r04q/c2_default.json; echo
bash tools/round_profile.sh r04q c2 c5 c1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04q/tr -o cur -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04q/tr.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04q/tr -name '*kernel_trace.csv' | head -1) 8 > gpurun_out/r04q/timeline_cur.txt
