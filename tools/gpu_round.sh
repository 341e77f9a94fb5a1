#!/bin/bash
# GPU tests (all, or the files given in TESTS), smoke, then a default C2 bench line (with the CPU
# baselines) for this round.  Run on the GPU box from the repo root:  bash tools/gpu_round.sh TAG
set -e
tag=$1
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -60 $out/tests.log; exit 1; }
tail -3 $out/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $out/bench.json 2> $out/bench.err || { tail -30 $out/bench.err; exit 1; }
tail -c 3000 $out/bench.json
