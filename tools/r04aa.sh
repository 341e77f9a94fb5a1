# Paired walk scheduling (slot 0's k_piece after the other slot's colour stage, slot 1's after
# slot 0's k_piece) with the fast host plan: GPU suite, then A/B: previous build (base), fast plan
# alone (fastplan), fast plan + pairing (cur), pairing off (cur@JD_PAIR_WAIT=0).
set -e
mkdir -p gpurun_out/r04aa
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04aa/tests.log 2>&1 || { tail -30 gpurun_out/r04aa/tests.log; exit 1; }
tail -2 gpurun_out/r04aa/tests.log
AB_REPS=3 bash tools/ab.sh gpurun_out/r04aa/c2 base cur fastplan
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04aa/c5 base cur
