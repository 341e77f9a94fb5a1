set -e
mkdir -p gpurun_out/r03ak
AB_ARGS="--config c2f --steps 30" bash tools/ab.sh gpurun_out/r03ak/ab2f base wrow0 cur base wrow0 cur
