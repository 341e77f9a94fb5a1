set -e
mkdir -p gpurun_out/r03v
AB_ARGS="--config c2 --steps 60" bash tools/ab.sh gpurun_out/r03v/ab2 nosync cur nosync cur nosync cur
AB_ARGS="--config c5 --steps 60" bash tools/ab.sh gpurun_out/r03v/ab5 nosync cur nosync cur
