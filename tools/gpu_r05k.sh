#!/bin/bash
# Round 5: k_chain_big for intervals over 256 pieces, dirty-chunk rounds, one-pass counts.
set -e
mkdir -p gpurun_out/r05k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05k/tests.log 2>&1 || { tail -30 gpurun_out/r05k/tests.log; exit 1; }
tail -2 gpurun_out/r05k/tests.log
timeout -k 10 600 python -u bench.py --config ref444 --batch 40 --sweep latency > gpurun_out/r05k/lat.json 2> gpurun_out/r05k/lat.err || { tail -20 gpurun_out/r05k/lat.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05k/lat.json').read().strip().splitlines()[-1])
for l in d['latency']: print(l['size'], round(l['gpu_wall_ms_median'],3), {k: round(v,3) for k,v in l['kernels_ms'].items() if v > 0.02})
"
AB_ARGS="--config c1 --steps 200 --warmup 20" bash tools/ab.sh gpurun_out/r05k/ab_c1 pre cur
AB_REPS=2 bash tools/ab.sh gpurun_out/r05k/ab pre cur
