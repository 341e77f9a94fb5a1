#!/bin/bash
# A/B of experiment builds and environment settings on the GPU box, one bench.py line each.
#
#   bash tools/ab.sh OUTDIR SPEC [SPEC ...]
#
# SPEC = LIB[@VAR=value,VAR=value...]: LIB is an experiment build libjdamd_<LIB>.so
# (make -C gpu-jpeg-decoder_amd variant V=<LIB> VDEFS=...), "cur" = the shipped libjdamd.so; the
# optional settings are exported for that run only.  AB_ARGS: extra bench.py arguments for every
# run (e.g. "--config c5").  AB_REPS=n repeats the whole list n times (alternating order).  Each
# run has its own time limit; the script stops at the first failure.
set -e
out=$1; shift
mkdir -p "$out"
reps=${AB_REPS:-1}
for r in $(seq 1 "$reps"); do
  specs=("$@")
  if (( r % 2 == 0 )); then  # every other repetition in reverse order
    rev=(); for ((i=${#specs[@]}-1; i>=0; i--)); do rev+=("${specs[i]}"); done; specs=("${rev[@]}")
  fi
  for spec in "${specs[@]}"; do
    v=${spec%%@*}; envs=""; [[ $spec == *@* ]] && envs=${spec#*@}
    lib=gpu-jpeg-decoder_amd/libjdamd_$v.so; [ "$v" = cur ] && lib=gpu-jpeg-decoder_amd/libjdamd.so
    ver=1; case "$v" in abl*) ver=0;; esac  # ablation builds compute wrong pixels on purpose
    tag=$(echo "$spec" | tr '@,=/' '____')_$r
    env JDAMD_LIB=$PWD/$lib JDAMD_ALLOW_ABI_MISMATCH=1 ${envs//,/ } timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-sample 0 \
      --e2e-steps 0 --copy-peak 0 --verify $ver ${AB_ARGS:-} > "$out/$tag.json" 2> "$out/$tag.err" || { tail -20 "$out/$tag.err"; exit 1; }
    python - "$out/$tag.json" "$spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), {k: round(v, 3) for k, v in d.get("kernels_ms_per_step", {}).items() if v})
PY
  done
done
