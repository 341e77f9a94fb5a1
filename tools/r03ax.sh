# record ring A/B: rr0 (4-byte record stores, as before), rr1 (LDS ring, conditional write), rr2 (unconditional write)
set -e
bash tools/ab.sh gpurun_out/r03ax rr0 rr1 rr2
bash tools/ab.sh gpurun_out/r03ax/2 rr0 rr1 rr2
root=$PWD
cd gpurun_out/r03ax && export TMPDIR=/tmp
for v in rr0 rr1 rr2; do
  JDAMD_LIB=$root/gpu-jpeg-decoder_amd/libjdamd_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d w_$v -o p -f csv -- python3 $root/bench.py --steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 > w_$v.log 2>&1
  echo "$v pmc done"
done
