#!/bin/bash
# Round 5: big-interval path restricted to small batches: parity, C2/C5/C3 A/B, latency.
set -e
mkdir -p gpurun_out/r05l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05l/tests.log 2>&1 || { tail -30 gpurun_out/r05l/tests.log; exit 1; }
tail -2 gpurun_out/r05l/tests.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r05l/ab pre cur
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r05l/ab_c5 pre cur
AB_ARGS="--config c3" bash tools/ab.sh gpurun_out/r05l/ab_c3 pre cur
timeout -k 10 600 python -u bench.py --config ref444 --batch 40 --sweep latency > gpurun_out/r05l/lat.json 2> gpurun_out/r05l/lat.err || { tail -20 gpurun_out/r05l/lat.err; exit 1; }
