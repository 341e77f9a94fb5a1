#!/bin/bash
# SQ counters of experiment / ablation builds on the GPU box (one rocprofv3 --pmc pass each):
#   bash tools/abl_sq.sh OUTDIR CONFIG LIB [LIB ...]      LIB: libjdamd_<LIB>.so, "cur" = libjdamd.so
# -> OUTDIR/<LIB>/p_counter_collection.csv (serialized steps; per-dispatch SQ_INSTS_VALU etc.)
set -e
out=$1; cfg=$2; shift 2
root=$PWD
mkdir -p "$out"
export TMPDIR=/tmp
for v in "$@"; do
  lib=$root/gpu-jpeg-decoder_amd/libjdamd_$v.so; [ "$v" = cur ] && lib=$root/gpu-jpeg-decoder_amd/libjdamd.so
  export JDAMD_LIB=$lib JDAMD_ALLOW_ABI_MISMATCH=1
  (cd "$out" && timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -d "$v" -o p -f csv -- \
     python3 "$root/bench.py" --config "$cfg" --steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 \
     --kernel-steps 1 --no-pipeline > "$v.log" 2>&1)
  echo "$v done"
done
