set -e
mkdir -p gpurun_out/r03l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03l/tests.log 2>&1 || { tail -30 gpurun_out/r03l/tests.log; exit 1; }
tail -2 gpurun_out/r03l/tests.log
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03l/ab2 zr0 cur rwd2 zr0 cur rwd2
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03l/ab5 zr0 cur rwd2
bash tools/gpu_quick.sh r03l 'JD_STAGE_NT=0 --config c2 --copy-peak 0' 'JD_STAGE_NT=1 --config c2 --copy-peak 0' 'JD_STAGE_NT=1 JD_STAGE_CHUNK_MB=32 --config c2 --copy-peak 0'
