#!/bin/bash
# Round-5 pipeline check: GPU batch tests, then depth 1 vs depth 2 (JD_ASYNC_DEPTH) A/B and traces.
set -e
mkdir -p gpurun_out/r05b
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05b/tests.log 2>&1 || { tail -30 gpurun_out/r05b/tests.log; exit 1; }
tail -2 gpurun_out/r05b/tests.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r05b/ab cur@JD_ASYNC_DEPTH=1 cur@JD_ASYNC_DEPTH=2
bash tools/trace.sh r05b cur@JD_ASYNC_DEPTH=1 cur@JD_ASYNC_DEPTH=2
# k_idct_color scatter ablations (wrong pixels; serialized kernel times from the bench line)
bash tools/ab.sh gpurun_out/r05b/abl cur ablsc1 ablsc2
