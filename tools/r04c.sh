set -e
mkdir -p gpurun_out/r04c
timeout -k 5 60 tools/micro/cores > gpurun_out/r04c/cores.txt 2>&1
timeout -k 5 120 tools/micro/valurate > gpurun_out/r04c/valurate.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c/gpu.log 2>&1 || { tail -30 gpurun_out/r04c/gpu.log; exit 1; }
tail -2 gpurun_out/r04c/gpu.log
AB_REPS=2 bash tools/ab.sh gpurun_out/r04c/c2 base cur
AB_REPS=2 AB_ARGS="--config c5" bash tools/ab.sh gpurun_out/r04c/c5 base cur
cat gpurun_out/r04c/cores.txt
