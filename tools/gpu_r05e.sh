#!/bin/bash
# Round 5: single-image latency per ref444 size with per-kernel times; 11-bit walk A/B.
set -e
mkdir -p gpurun_out/r05e
timeout -k 10 600 python -u bench.py --config ref444 --batch 40 --sweep latency > gpurun_out/r05e/lat.json 2> gpurun_out/r05e/lat.err || { tail -20 gpurun_out/r05e/lat.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05e/lat.json').read().strip().splitlines()[-1])
for l in d['latency']: print(l['size'], round(l['gpu_wall_ms_median'],3), {k: round(v,3) for k,v in l['kernels_ms'].items() if v > 0.02})
"
AB_REPS=2 bash tools/ab.sh gpurun_out/r05e/ab cur l11w1024
