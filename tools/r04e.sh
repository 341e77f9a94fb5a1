# co-residency variants with the first-round flag and k_chain_fix at <= 128 VGPRs
set -e
mkdir -p gpurun_out/r04e
AB_REPS=2 bash tools/ab.sh gpurun_out/r04e/c2 cur cur@JD_COSCHED=1,JD_SLOTS=3 co1024@JD_COSCHED=1,JD_SLOTS=3 pt768@JD_COSCHED=1,JD_SLOTS=3 pt768w5@JD_COSCHED=1,JD_SLOTS=3
cd /tmp && export TMPDIR=/tmp
JD_COSCHED=1 JD_SLOTS=3 JDAMD_LIB=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd_pt768w5.so timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04e/tr -o co -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04e/tr.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04e/tr -name '*kernel_trace.csv' | head -1) 4 > gpurun_out/r04e/timeline_pt768w5.txt
