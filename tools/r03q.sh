# Multi-rank rehearsal on the one-GPU box: two ranks (gloo counters) sharing cuda:0.
set -e
mkdir -p gpurun_out/r03q
export JD_DIST_BACKEND=gloo
timeout -k 10 900 python bench.py --gpus 2 --steps 10 --warmup 2 --cpu-sample 0 --e2e-steps 4 --copy-peak 0 \
  --kernel-steps 1 > gpurun_out/r03q/dist2.json 2> gpurun_out/r03q/dist2.err || { tail -30 gpurun_out/r03q/dist2.err; exit 1; }
python3 - gpurun_out/r03q/dist2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "world_seen", d["world_size_seen"], "backend", d["dist_backend"], round(d["value"]), "MPix/s", round(d["ms_per_step"], 2), "ms")
print("shards", d["shards"])
print("per_rank", json.dumps(d["per_rank"]))
PY
