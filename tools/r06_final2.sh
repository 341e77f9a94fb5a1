#!/bin/bash
# Round 6, last GPU run on the final tree: GPU suite + smoke, one driver-command bench line, and a
# longer randomised parity sweep (Pillow encodes, flat areas).
set -e
out=gpurun_out/r06g
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', round(d['value']), round(d['ms_per_step'],3), d['device_memory']['decoder_pools_peak_GB'])" $out/bench.json
timeout -k 10 560 python -u tools/parity_sweep.py --minutes 8 --seed 64 --pil --out $out/sweep.json > $out/sweep.log 2>&1 || { tail -5 $out/sweep.log; exit 1; }
tail -1 $out/sweep.log
