set -e
mkdir -p gpurun_out/r03d
timeout -k 10 300 python -u -m pytest tests/test_gpu_fancy.py tests/test_gpu_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03d/tests.log 2>&1 || { tail -30 gpurun_out/r03d/tests.log; exit 1; }
tail -2 gpurun_out/r03d/tests.log
bash tools/gpu_quick.sh r03d '--config c2 --fancy --e2e-steps 0' '--config c5 --fancy --e2e-steps 0' 'JD_STAGE_CHUNK_MB=0 --config c2' 'JD_STAGE_CHUNK_MB=32 --config c2' 'JD_STAGE_CHUNK_MB=128 --config c2'
