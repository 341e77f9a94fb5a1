#!/bin/bash
# Round-2 baseline: C2 bench line + two SQ PMC passes (kernel-trace only), summarised per kernel.
set -e
mkdir -p gpurun_out/r02a
BENCH_ARGS="--config c2" bash tools/prof_pmc.sh r02a/pmc \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
python tools/pmc_summary.py gpurun_out/r02a/pmc > gpurun_out/r02a/pmc_summary.txt
cat gpurun_out/r02a/pmc_summary.txt
