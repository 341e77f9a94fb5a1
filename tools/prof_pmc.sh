#!/bin/bash
# PMC passes over a short bench run (rocprofv3, one counter group per pass, never combined with
# runtime traces).  Usage: bash tools/prof_pmc.sh OUTDIR "GROUP1" "GROUP2" ...  (run from the repo root)
# BENCH_ARGS adds bench.py arguments (e.g. "--config c3").
set -e
root=$PWD
out=$1; shift
mkdir -p gpurun_out/$out && cd gpurun_out/$out && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d p$i -o p -f csv -- python3 $root/bench.py --steps 2 --warmup 1 --cpu-sample 0 --verify 0 ${BENCH_ARGS:-} > p$i.log 2>&1
done
