# Kernel trace of the default pipeline with the fast host plan (cached region divisor), to check
# where the step is lost.
set -e
mkdir -p gpurun_out/r04z
cd /tmp && export TMPDIR=/tmp
JDAMD_LIB=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd_fastplan.so timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04z/tr -o t -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04z/tr.log 2>&1
cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04z/tr -name '*kernel_trace.csv' | head -1) 8 > gpurun_out/r04z/timeline_fastplan.txt
