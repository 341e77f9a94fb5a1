# 4:4:4 tail lane-step as 4-pixel halves (h444) vs one more full step (h0): C5 (a third 4:4:4), C1 (4:4:4), C2;
# then the GPU suite on h444
set -e
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bl/c5 h444 h0
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bl/c5b h0 h444
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bl/c5c h444 h0
AB_ARGS="--config c1" bash tools/ab.sh gpurun_out/r03bl/c1 h444 h0 h444 h0
bash tools/ab.sh gpurun_out/r03bl/c2 h444 h0
mkdir -p gpurun_out/r03bl
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_h444.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "not sanit and not build" > gpurun_out/r03bl/gpu.log 2>&1 || { tail -30 gpurun_out/r03bl/gpu.log; exit 1; }
tail -1 gpurun_out/r03bl/gpu.log
