#!/bin/bash
# Round 5: k_chain_big (big intervals) parity, then the latency sweep again.
set -e
mkdir -p gpurun_out/r05f
timeout -k 10 900 python -u -m pytest tests/test_gpu_redo.py tests/test_gpu.py tests/test_gpu_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05f/tests.log 2>&1 || { tail -30 gpurun_out/r05f/tests.log; exit 1; }
tail -2 gpurun_out/r05f/tests.log
timeout -k 10 600 python -u bench.py --config ref444 --batch 40 --sweep latency > gpurun_out/r05f/lat.json 2> gpurun_out/r05f/lat.err || { tail -20 gpurun_out/r05f/lat.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05f/lat.json').read().strip().splitlines()[-1])
for l in d['latency']: print(l['size'], round(l['gpu_wall_ms_median'],3), {k: round(v,3) for k,v in l['kernels_ms'].items() if v > 0.02})
"
bash tools/ab.sh gpurun_out/r05f/ab cur
