# host-input legs (staged / registered / pinned arena) in the default bench line, the same with one
# DMA per span; then the co-scheduling variants with 8 hardware queues (tools/r04g.sh)
set -e
mkdir -p gpurun_out/r04h
timeout -k 10 600 python bench.py --cpu-sample 0 > gpurun_out/r04h/bench.json 2> gpurun_out/r04h/bench.err || { tail -20 gpurun_out/r04h/bench.err; exit 1; }
JD_STAGE_CHUNK_MB=100000 timeout -k 10 600 python bench.py --cpu-sample 0 --copy-peak 0 > gpurun_out/r04h/bench_nochunk.json 2> gpurun_out/r04h/bench_nochunk.err || { tail -20 gpurun_out/r04h/bench_nochunk.err; exit 1; }
for f in bench bench_nochunk; do python -c "
import json,sys;d=json.loads(open('gpurun_out/r04h/$f.json').read().strip().splitlines()[-1]);e=d['e2e_h2d']
print('$f', round(d['ms_per_step'],3), 'staged', round(e['ms_per_step'],2), round(e['frac_of_h2d_bound'],3), 'registered', round(e['registered']['ms_per_step'],2), round(e['registered']['frac_of_h2d_bound'],3), 'pinned', round(e['pinned_arena']['ms_per_step'],2), round(e['pinned_arena']['frac_of_h2d_bound'],3), 'h2d', round(e['pinned_h2d_GB_s'],1), e['pinned_arena']['host_ms_per_step'])"; done
bash tools/r04g.sh
