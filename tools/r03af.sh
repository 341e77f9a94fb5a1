set -e
mkdir -p gpurun_out/r03af
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03af/tests.log 2>&1 || { tail -30 gpurun_out/r03af/tests.log; exit 1; }
tail -1 gpurun_out/r03af/tests.log
AB_ARGS="--config c2 --steps 60" bash tools/ab.sh gpurun_out/r03af/ab2 base cur base cur
AB_ARGS="--config c5 --steps 40" bash tools/ab.sh gpurun_out/r03af/ab5 base cur
AB_ARGS="--config c2f --steps 30" bash tools/ab.sh gpurun_out/r03af/ab2f base cur
