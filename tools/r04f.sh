# registered host inputs: the new GPU test, the default bench line (e2e staged vs registered), the GPU suite
set -e
mkdir -p gpurun_out/r04f
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -k registered -x -q --timeout 240 --timeout-method thread > gpurun_out/r04f/reg.log 2>&1 || { tail -40 gpurun_out/r04f/reg.log; exit 1; }
tail -1 gpurun_out/r04f/reg.log
timeout -k 10 600 python bench.py > gpurun_out/r04f/bench.json 2> gpurun_out/r04f/bench.err || { tail -20 gpurun_out/r04f/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r04f/bench.json').read().strip().splitlines()[-1]);e=d['e2e_h2d'];print(d['value'],d['ms_per_step']);print({k:e[k] for k in ('MPix_s','ms_per_step','frac_of_h2d_bound','pinned_h2d_GB_s')});print(e['registered'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f/gpu.log 2>&1 || { tail -30 gpurun_out/r04f/gpu.log; exit 1; }
tail -1 gpurun_out/r04f/gpu.log
