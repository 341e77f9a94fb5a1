# parity sweeps with Pillow-encoded images (standard and optimised Huffman tables)
set -e
mkdir -p gpurun_out/r03bb
timeout -k 10 420 python -u tools/parity_sweep.py --minutes 5 --seed 41 --pil --out gpurun_out/r03bb/sweep_pil.json > gpurun_out/r03bb/sweep_pil.log 2>&1 || { tail -3 gpurun_out/r03bb/sweep_pil.log; exit 1; }
tail -1 gpurun_out/r03bb/sweep_pil.log
timeout -k 10 300 python -u tools/parity_sweep.py --minutes 3.5 --seed 42 --pil --fancy --out gpurun_out/r03bb/sweep_pil_fancy.json > gpurun_out/r03bb/sweep_pil_fancy.log 2>&1 || { tail -3 gpurun_out/r03bb/sweep_pil_fancy.log; exit 1; }
tail -1 gpurun_out/r03bb/sweep_pil_fancy.log
