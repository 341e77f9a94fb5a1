#!/bin/bash
# Round 6: randomised parity sweeps on the final tree (after the k_scan marker-run fix), two seeds.
set -e
out=gpurun_out/r06i
mkdir -p $out
timeout -k 10 560 python -u tools/parity_sweep.py --minutes 8 --seed 64 --pil --out $out/sweep64.json > $out/sweep64.log 2>&1 || { tail -3 $out/sweep64.log; exit 1; }
tail -1 $out/sweep64.log
timeout -k 10 560 python -u tools/parity_sweep.py --minutes 8 --seed 65 --pil --out $out/sweep65.json > $out/sweep65.log 2>&1 || { tail -3 $out/sweep65.log; exit 1; }
tail -1 $out/sweep65.log
