#!/bin/bash
# Round 6: optimistic pools -- randomised parity sweep (flat images included) and the pools' peak on
# every bench config.  Run on the GPU box from the repo root.
set -e
out=gpurun_out/r06u
mkdir -p $out
timeout -k 10 420 python -u tools/parity_sweep.py --minutes 5 --seed 61 --pil --out $out/sweep.json > $out/sweep.log 2>&1 || { tail -5 $out/sweep.log; exit 1; }
tail -1 $out/sweep.log
for c in c3 c5 ref444; do
  timeout -k 10 300 python bench.py --config $c --cpu-sample 0 --e2e-steps 0 > $out/$c.json 2> $out/$c.err || { tail -5 $out/$c.err; exit 1; }
  python3 - $out/$c.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["config"], round(d["value"]), "MPix/s", round(d["ms_per_step"], 3), "ms", json.dumps(d["device_memory"]))
PY
done
