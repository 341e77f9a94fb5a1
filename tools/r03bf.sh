# second emit test as one bit of lo & ~(zn2 << 1) (ep5) vs the committed build (cur); then the GPU suite on ep5
set -e
bash tools/ab.sh gpurun_out/r03bf cur ep5
bash tools/ab.sh gpurun_out/r03bf/2 ep5 cur
bash tools/ab.sh gpurun_out/r03bf/3 cur ep5
mkdir -p gpurun_out/r03bf
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_ep5.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "not sanit and not build" > gpurun_out/r03bf/gpu.log 2>&1 || { tail -30 gpurun_out/r03bf/gpu.log; exit 1; }
tail -1 gpurun_out/r03bf/gpu.log
