# Three traced runs of the default pipeline with the fast host plan (bimodal step):
# the per-two-batch period and kernel order of each, to compare the good and the bad mode.
set -e
mkdir -p gpurun_out/r04ab
cd /tmp && export TMPDIR=/tmp
for r in 1 2 3; do
  JDAMD_LIB=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd_fastplan.so timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04ab/tr$r -o t -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 3 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/r04ab/tr$r.log 2>&1
  (cd $GRAFT_REPO_ROOT && python tools/timeline.py $(find gpurun_out/r04ab/tr$r -name '*kernel_trace.csv' | head -1) 8 > gpurun_out/r04ab/timeline_$r.txt)
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{\"metric\"')][-1]; print($r, d['ms_per_step'])" $GRAFT_REPO_ROOT/gpurun_out/r04ab/tr$r.log || true
done
