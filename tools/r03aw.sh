# WRITE_SIZE of k_piece: current build vs no entry stores (JD_ABL=8) vs no record stores (JD_ABL=16)
set -e
root=$PWD
mkdir -p gpurun_out/r03aw && cd gpurun_out/r03aw && export TMPDIR=/tmp
for v in cur abl8 abl16; do
  lib=$root/gpu-jpeg-decoder_amd/libjdamd_$v.so; [ "$v" = cur ] && lib=$root/gpu-jpeg-decoder_amd/libjdamd.so
  JDAMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $v -o p -f csv -- python3 $root/bench.py --steps 2 --warmup 1 --cpu-sample 0 --verify 0 --e2e-steps 0 --copy-peak 0 > $v.log 2>&1
  echo "$v done"
done
