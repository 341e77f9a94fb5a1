set -e
mkdir -p gpurun_out/r03h
timeout -k 10 300 python -u -m pytest tests/test_gpu_fancy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03h/tests.log 2>&1 || { tail -30 gpurun_out/r03h/tests.log; exit 1; }
tail -2 gpurun_out/r03h/tests.log
bash tools/gpu_quick.sh r03h '--config c2 --fancy --e2e-steps 0 --copy-peak 0' '--config c5 --fancy --e2e-steps 0 --copy-peak 0'
