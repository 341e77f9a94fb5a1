#!/bin/bash
# Round 5: unrolled window-group rounds in the walk (JD_GROUP_UNROLL) A/B and parity.
set -e
mkdir -p gpurun_out/r05g
AB_REPS=2 bash tools/ab.sh gpurun_out/r05g/ab pre cur gu1
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r05g/ab_c5 pre gu1
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_gu1.so JDAMD_ALLOW_ABI_MISMATCH=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_redo.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g/tests_gu1.log 2>&1 || { tail -30 gpurun_out/r05g/tests_gu1.log; exit 1; }
tail -2 gpurun_out/r05g/tests_gu1.log
