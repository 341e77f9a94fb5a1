#!/bin/bash
# One experiment round on the GPU box:  bash tools/gpu_exp.sh TAG [CONFIGS...]
# GPU parity suite, then A/B of the experiment build "pre" (tools/build_ref_variant.sh) against the
# shipped library per config (C2 twice, alternating order), then the ref444 latency sweep.  Every
# step has its own time limit; the script stops at the first failure.
set -e
tag=$1; shift
cfgs=${@:-c2 c5 c3}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for c in $cfgs; do
  reps=1; [ "$c" = c2 ] && reps=2
  AB_REPS=$reps AB_ARGS="--config $c" bash tools/ab.sh $out/ab_$c pre cur
done
timeout -k 10 600 python -u bench.py --config ref444 --batch 40 --sweep latency > $out/lat.json 2> $out/lat.err || { tail -20 $out/lat.err; exit 1; }
