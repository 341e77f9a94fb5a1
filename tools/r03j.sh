set -e
mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest tests/test_gpu_redo.py tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "random or redo or escape or full or 1080 or 4k" > gpurun_out/r03j/tests.log 2>&1 || { tail -30 gpurun_out/r03j/tests.log; exit 1; }
tail -2 gpurun_out/r03j/tests.log
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03j/ab2 rare1 cur rareb4 rareb16 rareb32 rare1 cur rareb4 rareb16
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03j/ab5 rare1 cur rareb4 rareb16
