#!/bin/bash
# Round 5: full GPU suite on the restructured runtime, then the ref444 sweep (profiles/r05_ref_sweep.json).
set -e
mkdir -p gpurun_out/r05c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05c/tests.log 2>&1 || { tail -30 gpurun_out/r05c/tests.log; exit 1; }
tail -2 gpurun_out/r05c/tests.log
timeout -k 10 900 python -u bench.py --config ref444 --sweep > gpurun_out/r05c/ref_sweep.json 2> gpurun_out/r05c/ref_sweep.err || { tail -20 gpurun_out/r05c/ref_sweep.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05c/ref_sweep.json').read().strip().splitlines()[-1])
for b in d['batch']: print(b['images'], round(b['serial_MB_s']), round(b['kernel_MB_s']), round(b['pipelined_MB_s']))
for l in d['latency']: print(l['size'], round(l['gpu_wall_ms_median'],3), round(l['gpu_kernel_ms'],3), l['ref_cpu_ms'])
"
