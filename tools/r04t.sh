# Kernel traces of the default pipeline: shipped build vs 11-bit LUT with one 1024-lane k_piece
# workgroup per CU (tools/timeline.py), to see where the latter's faster k_piece is lost.
set -e
mkdir -p gpurun_out/r04t
cd /tmp && export TMPDIR=/tmp
for v in cur l11w1024; do
  lib=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd_$v.so; [ $v = cur ] && lib=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd.so
  JDAMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04t/tr_$v -o t -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04t/tr_$v.log 2>&1
  (cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04t/tr_$v -name '*kernel_trace.csv' | head -1) 8 > gpurun_out/r04t/timeline_$v.txt)
  tail -c 200 $GRAFT_REPO_ROOT/gpurun_out/r04t/tr_$v.log; echo
done
