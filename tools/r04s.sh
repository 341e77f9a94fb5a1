# 11-bit Huffman index with one 1024-lane k_piece workgroup per CU (a single table copy: 4 x 16.7 KB
# + 1024 x 92 B of LDS), against 10 bits with 2 x 512 (shipped) and 10 bits with 1 x 1024.
set -e
mkdir -p gpurun_out/r04s
JDAMD_LIB=$PWD/gpu-jpeg-decoder_amd/libjdamd_l11w1024.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04s/tests_l11.log 2>&1 || { tail -30 gpurun_out/r04s/tests_l11.log; exit 1; }
tail -2 gpurun_out/r04s/tests_l11.log
AB_REPS=3 bash tools/ab.sh gpurun_out/r04s/c2 cur l11w1024 w1024
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04s/c5 cur l11w1024
