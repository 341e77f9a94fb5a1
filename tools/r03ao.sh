set -e
L=$PWD/gpu-jpeg-decoder_amd
for lib in libjdamd_old.so libjdamd_base.so libjdamd.so; do
  JDAMD_LIB=$L/$lib timeout -k 10 120 python -u tools/gray_repro.py tools/sweep_cases_r03as.json 2>&1 | grep -v Warning
done
