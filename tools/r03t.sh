set -e
mkdir -p gpurun_out/r03t
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_redo.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03t/tests.log 2>&1 || { tail -30 gpurun_out/r03t/tests.log; exit 1; }
tail -2 gpurun_out/r03t/tests.log
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03t/ab2 nobfi cur nobfi cur
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03t/ab5 nobfi cur
