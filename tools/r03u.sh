set -e
mkdir -p gpurun_out/r03u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03u/tests.log 2>&1 || { tail -30 gpurun_out/r03u/tests.log; exit 1; }
tail -2 gpurun_out/r03u/tests.log
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03u/ab2 nosync cur nosync cur
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03u/ab5 nosync cur
AB_ARGS="--config c3" bash tools/ab.sh gpurun_out/r03u/ab3 nosync cur
