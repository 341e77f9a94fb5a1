set -e
mkdir -p gpurun_out/r03y
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03y/tests.log 2>&1 || { tail -30 gpurun_out/r03y/tests.log; exit 1; }
tail -2 gpurun_out/r03y/tests.log
AB_ARGS="--config c2 --steps 60" bash tools/ab.sh gpurun_out/r03y/ab2 base cur base cur
AB_ARGS="--config c5 --steps 60" bash tools/ab.sh gpurun_out/r03y/ab5 base cur
AB_ARGS="--config c3 --steps 40" bash tools/ab.sh gpurun_out/r03y/ab3 base cur
