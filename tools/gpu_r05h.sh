#!/bin/bash
# Round 5: piece plan in k_index's tail, subplan in k_compact's first workgroups: parity, A/B, trace.
set -e
mkdir -p gpurun_out/r05h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05h/tests.log 2>&1 || { tail -30 gpurun_out/r05h/tests.log; exit 1; }
tail -2 gpurun_out/r05h/tests.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r05h/ab pre cur
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r05h/ab_c5 pre cur
bash tools/trace.sh r05h cur
timeout -k 10 600 python -u bench.py --config ref444 --batch 40 --sweep latency > gpurun_out/r05h/lat.json 2> gpurun_out/r05h/lat.err || { tail -20 gpurun_out/r05h/lat.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05h/lat.json').read().strip().splitlines()[-1])
for l in d['latency']: print(l['size'], round(l['gpu_wall_ms_median'],3), {k: round(v,3) for k,v in l['kernels_ms'].items() if v > 0.02})
"
