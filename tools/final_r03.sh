# End-of-round check of HEAD: GPU suite, smoke, the default bench line (CPU baselines included), then
# the C3 / C1 bench lines again now that their SQ profiles are committed (roofline.bound from them)
set -e
bash tools/gpu_round.sh r03bn
for c in c3 c1; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/r03bn/$c.json 2> gpurun_out/r03bn/$c.err || { tail -20 gpurun_out/r03bn/$c.err; exit 1; }
done
