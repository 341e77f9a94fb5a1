set -e
mkdir -p gpurun_out/r03f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03f/tests.log 2>&1 || { tail -30 gpurun_out/r03f/tests.log; exit 1; }
tail -2 gpurun_out/r03f/tests.log
bash tools/gpu_quick.sh r03f '--config c2 --fancy --e2e-steps 0 --copy-peak 0' '--config c3 --fancy --e2e-steps 0 --copy-peak 0' '--config c2 --copy-peak 0'
