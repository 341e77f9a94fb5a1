set -e
mkdir -p gpurun_out/r03s
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03s/tests.log 2>&1 || { tail -30 gpurun_out/r03s/tests.log; exit 1; }
tail -2 gpurun_out/r03s/tests.log
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03s/ab2 br1 cur br1 cur
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03s/ab5 br1 cur
AB_ARGS="--config c2f --e2e-steps 0" bash tools/ab.sh gpurun_out/r03s/abf cur fb16
