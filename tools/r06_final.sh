#!/bin/bash
# Round 6 closing run on the GPU box (repo root): GPU suite + smoke, three driver-command bench
# lines, then randomised parity sweeps (plain with Pillow encodes, and fancy upsampling).
set -e
out=gpurun_out/r06f
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench$i.json 2> $out/bench$i.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', round(d['value']), round(d['ms_per_step'],3), d['device_memory']['decoder_pools_peak_GB'])" $out/bench$i.json
done
timeout -k 10 330 python -u tools/parity_sweep.py --minutes 4 --seed 62 --pil --out $out/sweep.json > $out/sweep.log 2>&1 || { tail -5 $out/sweep.log; exit 1; }
tail -1 $out/sweep.log
timeout -k 10 330 python -u tools/parity_sweep.py --minutes 4 --seed 63 --fancy --out $out/sweep_fancy.json > $out/sweep_fancy.log 2>&1 || { tail -5 $out/sweep_fancy.log; exit 1; }
tail -1 $out/sweep_fancy.log
