#!/bin/bash
# Kernel timelines of pipelined bench runs on the GPU box:
#
#   bash tools/trace.sh TAG SPEC [SPEC ...]
#
# SPEC = LIB[@VAR=value,VAR=value...] as in tools/ab.sh ("cur" = the shipped libjdamd.so).
# TRACE_ARGS: extra bench.py arguments (e.g. "--config c5").  Per spec: one rocprofv3
# --kernel-trace run of 12 pipelined steps -> gpurun_out/TAG/<spec>/, its step time, and
# tools/timeline.py over the last 4 batches -> gpurun_out/TAG/<spec>.txt.
set -e
tag=$1; shift
root=$PWD
out=$root/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  v=${spec%%@*}; envs=""; [[ $spec == *@* ]] && envs=${spec#*@}
  lib=$root/gpu-jpeg-decoder_amd/libjdamd_$v.so; [ "$v" = cur ] && lib=$root/gpu-jpeg-decoder_amd/libjdamd.so
  t=$(echo "$spec" | tr '@,=/' '____')
  for kv in ${envs//,/ }; do export "$kv"; done
  (cd /tmp && JDAMD_LIB=$lib JDAMD_ALLOW_ABI_MISMATCH=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/$t" -o t -f csv -- \
     python3 "$root/bench.py" --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 \
     --kernel-steps 0 ${TRACE_ARGS:-} > "$out/$t.log" 2>&1)
  for kv in ${envs//,/ }; do unset "${kv%%=*}"; done
  python3 tools/timeline.py "$(find "$out/$t" -name '*kernel_trace.csv' | head -1)" 4 > "$out/$t.txt"
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{\"metric\"')][-1]; print(sys.argv[2], d['ms_per_step'])" "$out/$t.log" "$spec"
  tail -1 "$out/$t.txt"
done
