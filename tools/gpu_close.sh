#!/bin/bash
# Round-closing checks on the GPU box (repo root):  bash tools/gpu_close.sh TAG [SEEDS...]
#   1. the GPU suite and smoke;
#   2. three bench lines with the driver's command (python3 bench.py --gpus 1 --steps 20 --warmup 5);
#   3. a 6-minute randomised parity sweep per seed (Pillow encodes, flat areas, bit flips), and one
#      with fancy upsampling.
# Round 6 ran these steps as separate calls: profiles/r06f_* (suite, bench x3, sweeps),
# r06u_parity_sweep_pools.json, r06i_parity_sweep_seed6{4,5}.json, r06j_parity_sweep_fancy.json.
# Each step has its own time limit; the script stops at the first failure.
set -e
tag=${1:-close}; shift || true
seeds=${@:-64}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench$i.json 2> $out/bench$i.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('bench', round(d['value']), round(d['ms_per_step'],3), d['device_memory']['decoder_pools_peak_GB'])" $out/bench$i.json
done
for s in $seeds; do
  timeout -k 10 450 python -u tools/parity_sweep.py --minutes 6 --seed $s --pil --out $out/sweep$s.json > $out/sweep$s.log 2>&1 || { tail -3 $out/sweep$s.log; exit 1; }
  tail -1 $out/sweep$s.log
done
timeout -k 10 330 python -u tools/parity_sweep.py --minutes 4 --seed 66 --fancy --out $out/sweep_fancy.json > $out/sweep_fancy.log 2>&1 || { tail -3 $out/sweep_fancy.log; exit 1; }
tail -1 $out/sweep_fancy.log
