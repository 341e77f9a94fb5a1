set -e
A="--steps 40 --warmup 3 --e2e-steps 0 --copy-peak 0"
L=$PWD/gpu-jpeg-decoder_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_redo.py tests/test_gpu_whitebox.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1 || { tail -30 gpurun_out/r03x_tests.log; exit 1; }
tail -1 gpurun_out/r03x_tests.log
bash tools/gpu_quick.sh r03x "--config c2 $A" "JDAMD_LIB=$L/libjdamd_p12k.so --config c2 $A" "JDAMD_LIB=$L/libjdamd_p20k.so --config c2 $A" \
  "JD_PIECE_OVERLAP_BITS=3072 --config c2 $A" "JD_PIECE_OVERLAP_BITS=6144 --config c2 $A" "--config c2 $A" \
  "--config c5 $A" "JDAMD_LIB=$L/libjdamd_p12k.so --config c5 $A" "JD_PIECE_OVERLAP_BITS=3072 --config c5 $A"
