set -e
mkdir -p gpurun_out/r03al
( time timeout -k 10 600 python bench.py > gpurun_out/r03al/default.json 2> gpurun_out/r03al/default.err ) 2> gpurun_out/r03al/default.time || { tail -30 gpurun_out/r03al/default.err; exit 1; }
tail -3 gpurun_out/r03al/default.time
python3 -c "import json; d=json.loads(open('gpurun_out/r03al/default.json').read().strip().splitlines()[-1]); print(d['metric'], round(d['value']), d['unit'], d['ms_per_step'], d['config'].get('workload'), d['roofline']['kernel'], round(d['roofline']['frac'],4), d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
bash tools/r03q.sh
