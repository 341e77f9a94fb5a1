# MCU-end reset before the table select (no tab_dc0 select) (ep7) vs the committed build (cur); then the GPU suite on ep7
set -e
bash tools/ab.sh gpurun_out/r03bh cur ep7
bash tools/ab.sh gpurun_out/r03bh/2 ep7 cur
bash tools/ab.sh gpurun_out/r03bh/3 cur ep7
mkdir -p gpurun_out/r03bh
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_ep7.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "not sanit and not build" > gpurun_out/r03bh/gpu.log 2>&1 || { tail -30 gpurun_out/r03bh/gpu.log; exit 1; }
tail -1 gpurun_out/r03bh/gpu.log
