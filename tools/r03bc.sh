# paired entry flush: held quad loaded straight from the ring (ep2) vs the committed build (cur)
set -e
bash tools/ab.sh gpurun_out/r03bc cur ep2
bash tools/ab.sh gpurun_out/r03bc/2 cur ep2
bash tools/ab.sh gpurun_out/r03bc/3 ep2 cur
