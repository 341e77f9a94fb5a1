# per-block counters in the fin branch + v_bfi record (ep4) vs the committed build (cur); then the GPU suite on ep4
set -e
bash tools/ab.sh gpurun_out/r03be cur ep4
bash tools/ab.sh gpurun_out/r03be/2 ep4 cur
bash tools/ab.sh gpurun_out/r03be/3 cur ep4
mkdir -p gpurun_out/r03be
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_ep4.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "not sanit and not build" > gpurun_out/r03be/gpu.log 2>&1 || { tail -30 gpurun_out/r03be/gpu.log; exit 1; }
tail -1 gpurun_out/r03be/gpu.log
