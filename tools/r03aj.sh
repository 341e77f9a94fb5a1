set -e
mkdir -p gpurun_out/r03aj
timeout -k 10 300 python -u -m pytest tests/test_gpu_fancy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03aj/tests.log 2>&1 || { tail -30 gpurun_out/r03aj/tests.log; exit 1; }
tail -1 gpurun_out/r03aj/tests.log
AB_ARGS="--config c2f --steps 30" bash tools/ab.sh gpurun_out/r03aj/ab2f base nopk cur base nopk cur
