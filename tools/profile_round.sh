#!/bin/bash
# Round profile (run on the GPU box from the repo root):
#   bash tools/profile_round.sh r01 [bench args...]
# 1. rocprofv3 --kernel-trace --stats over the bench command        -> gpurun_out/<tag>/stats/
# 2. separate PMC passes FETCH_SIZE, WRITE_SIZE (never combined with runtime traces)
# tools/profile_summary.py then writes profiles/<tag>_kernel_stats.csv and profiles/<tag>_traffic.json.
set -e
tag=$1; shift
args="$@"
out=gpurun_out/$tag
mkdir -p $out && cd $out && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d stats -o run -f csv -- python3 ../../bench.py $args > bench_stats.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d fetch -o run -f csv -- python3 ../../bench.py --steps 2 --warmup 1 --cpu-sample 0 --verify 0 > fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d write -o run -f csv -- python3 ../../bench.py --steps 2 --warmup 1 --cpu-sample 0 --verify 0 > write.log 2>&1
