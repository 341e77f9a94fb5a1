set -e
AB_ARGS="--config c2f --e2e-steps 0" bash tools/ab.sh gpurun_out/r03r/abf cur fb8 fb2 cur fb8 fb2
