# Warm-up length (JD_PIECE_OVERLAP_BITS) revisited with the current pipeline: 4096 (default) vs 3584 / 3072.
set -e
mkdir -p gpurun_out/r04w
AB_REPS=3 bash tools/ab.sh gpurun_out/r04w/c2 cur cur@JD_PIECE_OVERLAP_BITS=3584 cur@JD_PIECE_OVERLAP_BITS=3072
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04w/c5 cur cur@JD_PIECE_OVERLAP_BITS=3072
