#!/bin/bash
# GPU tests, smoke, then short bench lines (no CPU baseline) for the given configs.
# Run on the GPU box from the repo root:  bash tools/gpu_check.sh TAG [configs...]
set -e
tag=$1; shift
cfgs=${@:-c2}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
for c in $cfgs; do
  timeout -k 10 300 python bench.py --config $c --cpu-sample 0 --steps 20 --warmup 3 > $out/$c.json 2> $out/$c.err
  python3 - $out/$c.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["config"], round(d["value"]), "MPix/s", round(d["ms_per_step"], 3), "ms", {k: round(v, 3) for k, v in d["kernels_ms_per_step"].items()})
PY
done
