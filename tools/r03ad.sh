set -e
mkdir -p gpurun_out/r03ad && cd gpurun_out/r03ad && export TMPDIR=/tmp
short="--config c2f --steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 1 --no-pipeline"
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU \
   SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d c2f_sq/p1 -o p -f csv -- \
   python3 $GRAFT_REPO_ROOT/bench.py $short > sq1.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
   SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d c2f_sq/p2 -o p -f csv -- \
   python3 $GRAFT_REPO_ROOT/bench.py $short > sq2.log 2>&1
echo ok
