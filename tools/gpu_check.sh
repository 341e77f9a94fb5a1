#!/bin/bash
# GPU tests, smoke, then bench lines for the given configs (c2 full default line incl. CPU baseline
# when FULL=1, else no CPU baseline).
# Run on the GPU box from the repo root:  bash tools/gpu_check.sh TAG [configs...]
set -e
tag=$1; shift
cfgs=${@:-c2}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
for c in $cfgs; do
  cpu=0; [ "${FULL:-0}" = 1 ] && cpu=1
  timeout -k 10 400 python bench.py --config $c --cpu-sample $cpu > $out/$c.json 2> $out/$c.err
  python3 - $out/$c.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["config"]["config"], round(d["value"]), "MPix/s", round(d["ms_per_step"], 3), "ms", {k: round(v, 3) for k, v in d["kernels_ms_per_step"].items()})
print("roofline", {k: d["roofline"][k] for k in ("bound", "kernel", "frac", "measured_copy_peak")})
print("e2e", json.dumps(d.get("e2e_h2d")))
print("per_rank", json.dumps(d.get("per_rank")), "mem", json.dumps(d.get("device_memory")))
PY
done
