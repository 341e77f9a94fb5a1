set -e
mkdir -p gpurun_out/r03w
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_redo.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03w/tests.log 2>&1 || { tail -30 gpurun_out/r03w/tests.log; exit 1; }
tail -2 gpurun_out/r03w/tests.log
AB_ARGS="--config c2 --steps 60" bash tools/ab.sh gpurun_out/r03w/ab2 nosync cur sync1 nosync cur sync1
AB_ARGS="--config c5 --steps 60" bash tools/ab.sh gpurun_out/r03w/ab5 nosync cur nosync cur
AB_ARGS="--config c3 --steps 40" bash tools/ab.sh gpurun_out/r03w/ab3 nosync cur
