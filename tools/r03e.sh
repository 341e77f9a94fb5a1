set -e
mkdir -p gpurun_out/r03e
timeout -k 10 300 python -u -m pytest tests/test_gpu_fancy.py tests/test_gpu_redo.py tests/test_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03e/tests.log 2>&1 || { tail -30 gpurun_out/r03e/tests.log; exit 1; }
tail -2 gpurun_out/r03e/tests.log
bash tools/gpu_quick.sh r03e '--config c2 --fancy --e2e-steps 0 --copy-peak 0'
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03e/ab cur pf0 cur pf0
