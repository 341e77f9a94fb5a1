# dense-stream tests (flat / long-code images, no spare regions), zeroing change A/B, then the GPU suite
set -e
mkdir -p gpurun_out/r04j
timeout -k 10 400 python -u -m pytest tests/test_gpu_redo.py -k dense -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j/dense.log 2>&1 || { tail -40 gpurun_out/r04j/dense.log; exit 1; }
tail -1 gpurun_out/r04j/dense.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r04j/c2 base cur
AB_REPS=1 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04j/c5 base cur
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04j/gpu.log 2>&1 || { tail -30 gpurun_out/r04j/gpu.log; exit 1; }
tail -1 gpurun_out/r04j/gpu.log
