# co-scheduling with more hardware queues (the two small-kernel chains of consecutive batches on
# distinct queues): cur vs the co-resident k_piece variants (branch cosched-exp)
set -e
mkdir -p gpurun_out/r04g
Q=GPU_MAX_HW_QUEUES=8
AB_REPS=2 bash tools/ab.sh gpurun_out/r04g/c2 cur cur@$Q cs512@JD_COSCHED=1,JD_SLOTS=3,$Q pt768w5@JD_COSCHED=1,JD_SLOTS=3,$Q co1024@JD_COSCHED=1,JD_SLOTS=3,$Q
cd /tmp && export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 JD_COSCHED=1 JD_SLOTS=3 JDAMD_LIB=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd_pt768w5.so timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04g/tr -o co -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04g/tr.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04g/tr -name '*kernel_trace.csv' | head -1) 6 > gpurun_out/r04g/timeline_pt768w5_q8.txt
