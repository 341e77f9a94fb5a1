# co-scheduling probe: GPU suite on the new runtime, then C2 / C5 A/B of the gate, slot count and
# k_piece workgroup size (512 / 768 / 1024 lanes)
set -e
mkdir -p gpurun_out/r04a
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r04a/gpu.log 2>&1 || { tail -30 gpurun_out/r04a/gpu.log; exit 1; }
tail -1 gpurun_out/r04a/gpu.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r04a/c2 cur@JD_COSCHED=0,JD_SLOTS=2 cur cur@JD_SLOTS=2 pt768 pt768@JD_COSCHED=0 pt1024
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04a/c5 cur@JD_COSCHED=0,JD_SLOTS=2 cur pt768
