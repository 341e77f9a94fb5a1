# IDCT: rows 0/4 outputs kept for the column pass, column terms as forced v_mad_i32_i24 chains:
# the IDCT tests, then C2 / C5 A/B against the previous commit (base), then the GPU suite
set -e
mkdir -p gpurun_out/r04l
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "idct or color" -x -q --timeout 240 --timeout-method thread > gpurun_out/r04l/idct.log 2>&1 || { tail -40 gpurun_out/r04l/idct.log; exit 1; }
tail -1 gpurun_out/r04l/idct.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r04l/c2 base cur
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04l/c5 base cur
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04l/gpu.log 2>&1 || { tail -30 gpurun_out/r04l/gpu.log; exit 1; }
tail -1 gpurun_out/r04l/gpu.log
