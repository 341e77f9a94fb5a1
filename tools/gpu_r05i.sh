#!/bin/bash
# Round 5: small-batch subplan fold + kAgreed: full GPU suite, C2/C5 A/B vs the committed build, latency.
set -e
mkdir -p gpurun_out/r05i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05i/tests.log 2>&1 || { tail -30 gpurun_out/r05i/tests.log; exit 1; }
tail -2 gpurun_out/r05i/tests.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r05i/ab pre cur
timeout -k 10 600 python -u bench.py --config ref444 --batch 40 --sweep latency > gpurun_out/r05i/lat.json 2> gpurun_out/r05i/lat.err || { tail -20 gpurun_out/r05i/lat.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05i/lat.json').read().strip().splitlines()[-1])
for l in d['latency']: print(l['size'], round(l['gpu_wall_ms_median'],3), {k: round(v,3) for k,v in l['kernels_ms'].items() if v > 0.02})
"
