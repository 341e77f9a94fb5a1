#!/bin/bash
# Bench lines for every BASELINE config that fits one GPU, each with its rocprofv3 kernel stats.
# Run on the GPU box from the repo root:  bash tools/gpu_configs.sh TAG [configs...]
#   -> gpurun_out/TAG/<config>.json (the bench line), gpurun_out/TAG/<config>_stats/ (rocprofv3)
# Each step has its own time limit and the script stops at the first failure.
set -e
tag=$1; shift
cfgs=${@:-c1 c2 c3 c5}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for c in $cfgs; do
  echo "== $c $(date +%T)"
  timeout -k 10 300 python bench.py --config $c > $out/$c.json 2> $out/$c.err
  tail -c 400 $out/$c.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${c}_stats -o run -f csv -- \
    python3 bench.py --config $c --steps 5 --warmup 1 --cpu-sample 0 --verify 0 > $out/${c}_stats.log 2>&1
done
