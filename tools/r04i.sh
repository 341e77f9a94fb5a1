# host-input legs with the DMAs of consecutive batches serialized (default) and not (JD_H2D_SERIAL=0);
# co-scheduling variants with 8 hardware queues
set -e
mkdir -p gpurun_out/r04i
for v in 1 0; do
JD_H2D_SERIAL=$v timeout -k 10 600 python bench.py --cpu-sample 0 --copy-peak 0 > gpurun_out/r04i/bench_s$v.json 2> gpurun_out/r04i/bench_s$v.err || { tail -20 gpurun_out/r04i/bench_s$v.err; exit 1; }
python -c "
import json,sys;d=json.loads(open('gpurun_out/r04i/bench_s$v.json').read().strip().splitlines()[-1]);e=d['e2e_h2d']
print('serial=$v', round(d['ms_per_step'],3), 'staged', round(e['ms_per_step'],2), round(e['frac_of_h2d_bound'],3), 'registered', round(e['registered']['ms_per_step'],2), round(e['registered']['frac_of_h2d_bound'],3), 'pinned', round(e['pinned_arena']['ms_per_step'],2), round(e['pinned_arena']['frac_of_h2d_bound'],3), 'h2d', round(e['pinned_h2d_GB_s'],1), e['host_ms_per_step'])"
done
bash tools/r04g.sh
