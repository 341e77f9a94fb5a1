set -e
mkdir -p gpurun_out/r03ay
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03ay/gpu.log 2>&1 || { tail -30 gpurun_out/r03ay/gpu.log; exit 1; }
tail -1 gpurun_out/r03ay/gpu.log
timeout -k 10 300 python -u tools/parity_sweep.py --minutes 3 --seed 33 --out gpurun_out/r03ay/sweep_s33.json > gpurun_out/r03ay/sweep.log 2>&1 || { tail -3 gpurun_out/r03ay/sweep.log; exit 1; }
tail -1 gpurun_out/r03ay/sweep.log
bash tools/ab.sh gpurun_out/r03ay cur ep1
bash tools/ab.sh gpurun_out/r03ay/2 cur ep1
root=$PWD
cd gpurun_out/r03ay && export TMPDIR=/tmp
for v in ep1; do
  JDAMD_LIB=$root/gpu-jpeg-decoder_amd/libjdamd_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d w_$v -o p -f csv -- python3 $root/bench.py --steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 > w_$v.log 2>&1
  echo "$v pmc done"
done
