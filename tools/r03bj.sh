# IDCT rotation (181 s + 128) >> 8 as three shift-adds (cur) vs v_mul_lo_u32 (m0); then the GPU suite on cur
set -e
bash tools/ab.sh gpurun_out/r03bj cur m0
bash tools/ab.sh gpurun_out/r03bj/2 m0 cur
bash tools/ab.sh gpurun_out/r03bj/3 cur m0
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03bj/c5 cur m0 cur m0
mkdir -p gpurun_out/r03bj
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03bj/gpu.log 2>&1 || { tail -30 gpurun_out/r03bj/gpu.log; exit 1; }
tail -1 gpurun_out/r03bj/gpu.log
