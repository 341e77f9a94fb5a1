#!/bin/bash
# Round profile on the GPU box (run from the repo root):  bash tools/round_profile.sh TAG [configs...]
# Per config:
#   1. the bench line                                            -> gpurun_out/TAG/<cfg>.json
#   2. rocprofv3 --kernel-trace --stats over serialized steps     -> gpurun_out/TAG/<cfg>_stats/
#      (--no-pipeline: kernels of consecutive batches do not overlap, so the per-kernel averages
#      compare with the bench line's serialized hipEvent pass)
#   3. PMC passes, one counter group per run, kernel-trace only: FETCH_SIZE, WRITE_SIZE, and the SQ groups of tools/r02_sq.sh                    -> gpurun_out/TAG/<cfg>_{fetch,write,sq}/
# tools/round_summary.py then writes profiles/TAG_*.  Every step has its own time limit; the script
# stops at the first failure.
set -e
tag=$1; shift
cfgs=${@:-c1 c2 c3 c5}
root=$PWD
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
short="--steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 1 --no-pipeline"
for c in $cfgs; do
  echo "== $c $(date +%T)"
  cpu=0; [ "$c" = c2 ] && cpu=1; [ "$c" = c1 ] && cpu=1
  timeout -k 10 400 python bench.py --config $c --cpu-sample $cpu > $out/$c.json 2> $out/$c.err
  tail -c 300 $out/$c.json; echo
  (cd $out && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ${c}_stats -o run -f csv -- \
     python3 $root/bench.py --config $c --steps 5 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 \
     --copy-peak 0 --kernel-steps 1 --no-pipeline > ${c}_stats.log 2>&1)
  (cd $out && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d ${c}_fetch -o p -f csv -- \
     python3 $root/bench.py --config $c $short > ${c}_fetch.log 2>&1)
  (cd $out && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d ${c}_write -o p -f csv -- \
     python3 $root/bench.py --config $c $short > ${c}_write.log 2>&1)
  if [ "$c" = c2 ] || [ "$c" = c5 ] || [ "$c" = c3 ] || [ "$c" = c1 ]; then
    (cd $out && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU \
       SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d ${c}_sq/p1 -o p -f csv -- \
       python3 $root/bench.py --config $c $short > ${c}_sq1.log 2>&1)
    (cd $out && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
       SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d ${c}_sq/p2 -o p -f csv -- \
       python3 $root/bench.py --config $c $short > ${c}_sq2.log 2>&1)
  fi
done
echo "== done $(date +%T)"
