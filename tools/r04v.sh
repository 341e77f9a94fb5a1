# Half-window rounds in the piece walks (a round ends when every lane is past the row's first
# half; the row slides by 16 bytes): GPU suite, then A/B against whole-window rounds (JD_HALF_ROUNDS=0).
set -e
mkdir -p gpurun_out/r04v
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04v/tests.log 2>&1 || { tail -30 gpurun_out/r04v/tests.log; exit 1; }
tail -2 gpurun_out/r04v/tests.log
AB_REPS=3 bash tools/ab.sh gpurun_out/r04v/c2 whole cur
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04v/c5 whole cur
