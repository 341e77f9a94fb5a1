#!/bin/bash
# SQ/GRBM counter passes (kernel-trace only, one group per pass) for one config + summary.
#   bash tools/r02_sq.sh TAG CONFIG     -> gpurun_out/TAG/sq/, profiles/TAG_sq_CONFIG.json
set -e
tag=$1; cfg=${2:-c2}
BENCH_ARGS="--config $cfg --e2e-steps 0 --copy-peak 0" bash tools/prof_pmc.sh $tag/sq \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
python tools/sq_summary.py $tag gpurun_out/$tag/sq --config $cfg
