set -e
mkdir -p gpurun_out/r03ai
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_redo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ai/tests.log 2>&1 || { tail -30 gpurun_out/r03ai/tests.log; exit 1; }
tail -1 gpurun_out/r03ai/tests.log
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_w16.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_redo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03ai/tests_w16.log 2>&1 || { tail -30 gpurun_out/r03ai/tests_w16.log; exit 1; }
tail -1 gpurun_out/r03ai/tests_w16.log
AB_ARGS="--config c2 --steps 60" bash tools/ab.sh gpurun_out/r03ai/ab2 cur w16 cur w16
AB_ARGS="--config c5 --steps 40" bash tools/ab.sh gpurun_out/r03ai/ab5 cur w16
