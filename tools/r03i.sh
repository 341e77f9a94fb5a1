set -e
mkdir -p gpurun_out/r03i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03i/tests.log 2>&1 || { tail -30 gpurun_out/r03i/tests.log; exit 1; }
tail -2 gpurun_out/r03i/tests.log
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03i/ab2 rare1 cur rare4 rare16 rare1 cur
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03i/ab5 rare1 cur rare16
bash tools/gpu_quick.sh r03i '--config c2 --fancy --e2e-steps 0 --copy-peak 0' '--config c5 --fancy --e2e-steps 0 --copy-peak 0'
