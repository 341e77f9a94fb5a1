set -e
AB_ARGS="--config c2" bash tools/ab.sh gpurun_out/r03k/ab2 cur rk2 rc3e8 rc6e16 rc2e4 rare1 cur rk2 rc3e8 rc2e4
AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r03k/ab5 cur rk2 rc3e8 rc6e16 rc2e4 rare1
