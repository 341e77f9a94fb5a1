#!/bin/bash
# Quick bench lines on the GPU box (no tests): bash tools/gpu_quick.sh TAG "args1" "args2" ...
# Each argument string is "[VAR=value ...] bench args" for one bench.py run (CPU baseline off).
set -e
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
i=0
for a in "$@"; do
  i=$((i+1))
  envs=(); rest=()
  for w in $a; do if [[ $w == *=* && ${#rest[@]} == 0 ]]; then envs+=("$w"); else rest+=("$w"); fi; done
  timeout -k 10 400 env "${envs[@]}" python bench.py --cpu-sample 0 "${rest[@]}" > $out/b$i.json 2> $out/b$i.err || { tail -5 $out/b$i.err; exit 1; }
  python3 - $out/b$i.json "$a" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "|", round(d["value"]), "MPix/s", round(d["ms_per_step"], 3), "ms", {k: round(v, 3) for k, v in d["kernels_ms_per_step"].items() if v})
e = d.get("e2e_h2d")
if e: print("  e2e", round(e["MPix_s"]), "MPix/s", round(e["ms_per_step"], 2), "ms h2d", round(e["pinned_h2d_GB_s"], 1), "frac", round(e["frac_of_h2d_bound"], 3), {k: round(v, 2) for k, v in e["host_ms_per_step"].items()})
PY
done
