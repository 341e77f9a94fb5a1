# Pair-order staging (k_idct_color): GPU suite, then A/B against the round's previous build on C2 and
# C5; then one piece per restart interval (--path lanes) with 512- vs 64-lane k_piece workgroups.
set -e
mkdir -p gpurun_out/r04n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04n/tests.log 2>&1 || { tail -30 gpurun_out/r04n/tests.log; exit 1; }
tail -2 gpurun_out/r04n/tests.log
AB_REPS=3 bash tools/ab.sh gpurun_out/r04n/c2 base cur
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04n/c5 base cur
AB_ARGS="--path lanes" bash tools/ab.sh gpurun_out/r04n/lanes cur cur@JD_PIECE_WG64=1
