#!/bin/bash
# A/B: bench with each experiment build given as an argument (libjdamd_<V>.so; "base" = libjdamd_base.so,
# "cur" = libjdamd.so).  Usage: bash tools/ab.sh OUTDIR V1 V2 ...   (AB_ARGS: extra bench.py args)
# Each run has its own time limit; the script stops at the first failure.
set -e
out=$1; shift
mkdir -p "$out"
for v in "$@"; do
  lib=gpu-jpeg-decoder_amd/libjdamd_$v.so; [ "$v" = cur ] && lib=gpu-jpeg-decoder_amd/libjdamd.so
  ver=1; case "$v" in abl*) ver=0;; esac  # ablation builds compute wrong pixels on purpose
  JDAMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 --e2e-steps 0 \
    --copy-peak 0 --verify $ver ${AB_ARGS:-} > "$out/$v.json" 2> "$out/$v.err" || { tail -20 "$out/$v.err"; exit 1; }
  python - "$out/$v.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), {k: round(v, 3) for k, v in d.get("kernels_ms_per_step", {}).items()})
PY
done
