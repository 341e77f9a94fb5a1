# escape flag in the odd bit of ent_blk2, blocks counted by 4 (ep6) vs the committed build (cur); then the GPU suite on ep6
set -e
bash tools/ab.sh gpurun_out/r03bg cur ep6
bash tools/ab.sh gpurun_out/r03bg/2 ep6 cur
bash tools/ab.sh gpurun_out/r03bg/3 cur ep6
mkdir -p gpurun_out/r03bg
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_ep6.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "not sanit and not build" > gpurun_out/r03bg/gpu.log 2>&1 || { tail -30 gpurun_out/r03bg/gpu.log; exit 1; }
tail -1 gpurun_out/r03bg/gpu.log
