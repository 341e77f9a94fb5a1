set -e
mkdir -p gpurun_out/r03aa
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_redo.py tests/test_gpu_whitebox.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03aa/tests.log 2>&1 || { tail -30 gpurun_out/r03aa/tests.log; exit 1; }
tail -1 gpurun_out/r03aa/tests.log
AB_ARGS="--config c2 --steps 60" bash tools/ab.sh gpurun_out/r03aa/ab2 base g1 g2 cur base cur
AB_ARGS="--config c5 --steps 40" bash tools/ab.sh gpurun_out/r03aa/ab5 base cur
cd gpurun_out/r03aa && export TMPDIR=/tmp
short="--steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 --kernel-steps 1 --no-pipeline"
for v in base cur; do
  lib=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd_$v.so; [ $v = cur ] && lib=$GRAFT_REPO_ROOT/gpu-jpeg-decoder_amd/libjdamd.so
  JDAMD_LIB=$lib timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d f_$v -o p -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 $short > f_$v.log 2>&1
  JDAMD_LIB=$lib timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d w_$v -o p -f csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c2 $short > w_$v.log 2>&1
done
echo pmc done
