set -e
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03l/tests.log 2>&1 || { tail -30 gpurun_out/r03l/tests.log; exit 1; }
tail -2 gpurun_out/r03l/tests.log
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03l/ab2 zr0 cur rwd2 zr0 cur rwd2
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03l/ab5 zr0 cur rwd2
