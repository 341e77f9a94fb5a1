set -e
mkdir -p gpurun_out/r03g
timeout -k 10 300 python -u -m pytest tests/test_gpu_fancy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03g/tests.log 2>&1 || { tail -30 gpurun_out/r03g/tests.log; exit 1; }
tail -2 gpurun_out/r03g/tests.log
bash tools/gpu_quick.sh r03g '--config c2 --fancy --e2e-steps 0 --copy-peak 0' '--config c5 --fancy --e2e-steps 0 --copy-peak 0'
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread -k "full_baseline" > gpurun_out/r03g/full.log 2>&1 || { tail -30 gpurun_out/r03g/full.log; exit 1; }
tail -2 gpurun_out/r03g/full.log
