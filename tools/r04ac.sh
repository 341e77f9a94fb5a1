# Walks never overlap (each k_piece waits for the other slot's) with the fast host plan: GPU suite,
# then A/B against the shipped build (base) and the fast plan without the wait (cur@JD_WALK_WAIT=0).
set -e
mkdir -p gpurun_out/r04ac
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ac/tests.log 2>&1 || { tail -30 gpurun_out/r04ac/tests.log; exit 1; }
tail -2 gpurun_out/r04ac/tests.log
AB_REPS=4 bash tools/ab.sh gpurun_out/r04ac/c2 base cur
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04ac/c5 base cur
