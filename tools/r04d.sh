# co-residency with the first-round flag: 1024-lane k_piece at 96 VGPRs beside one IDCT wave per SIMD
set -e
mkdir -p gpurun_out/r04d
AB_REPS=2 bash tools/ab.sh gpurun_out/r04d/c2 cur co1024@JD_COSCHED=1,JD_SLOTS=3 co1024p@JD_COSCHED=1,JD_SLOTS=3 cur@JD_COSCHED=1,JD_SLOTS=3
cd /tmp && export TMPDIR=/tmp
JD_COSCHED=1 JD_SLOTS=3 JDAMD_LIB=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd_co1024.so timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04d/tr -o co -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04d/tr.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04d/tr -name '*kernel_trace.csv' | head -1) 3 > gpurun_out/r04d/timeline_co1024.txt
