#!/bin/bash
# A/B of environment settings on the current build: bash tools/ab_env.sh OUTDIR "NAME=ENV ..." ...
# (each argument: a label, '=', then space-separated VAR=value settings; AB_ARGS: extra bench args)
set -e
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 --e2e-steps 0 \
    --copy-peak 0 ${AB_ARGS:-} > "$out/$name.json" 2> "$out/$name.err" || { tail -20 "$out/$name.err"; exit 1; }
  python - "$out/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), {k: round(v, 3) for k, v in d.get("kernels_ms_per_step", {}).items()})
PY
done
