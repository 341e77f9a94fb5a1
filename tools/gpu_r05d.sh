#!/bin/bash
# Round 5: colour stage on its own stream / stream priorities / async depth.
set -e
AB_REPS=2 bash tools/ab.sh gpurun_out/r05d/ab cur cur@JD_IDCT_STREAM=1 cur@JD_IDCT_STREAM=1,JD_IDCT_PRIO=-1,JD_SLOT_PRIO=1 \
  cur@JD_ASYNC_DEPTH=2,JD_IDCT_STREAM=1,JD_IDCT_PRIO=-1,JD_SLOT_PRIO=1 cur@JD_ASYNC_DEPTH=2,JD_IDCT_STREAM=1
bash tools/trace.sh r05d cur@JD_IDCT_STREAM=1,JD_IDCT_PRIO=-1,JD_SLOT_PRIO=1 cur@JD_ASYNC_DEPTH=2,JD_IDCT_STREAM=1,JD_IDCT_PRIO=-1,JD_SLOT_PRIO=1
