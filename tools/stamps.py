"""Phase timing of k_idct_color from a JD_STAMP diagnostic build (s_memtime stamps per tile).

    JDAMD_LIB=gpu-jpeg-decoder_amd/libjdamd_stamp.so JD_STAMPS=1 python tools/stamps.py [--config c2]

Decodes one batch of the bench workload and prints, over all tiles, the mean / median cycles between
consecutive stamps (0 start, 1 loads issued + DC predicted, 2 entries scattered, 3 IDCT done,
4 colour + stores issued) and the distribution of wave lifetimes.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "gpu-jpeg-decoder_amd")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import jd_synth  # noqa: E402
import jdamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--batch", type=int, default=256)
a = ap.parse_args()
W, H, ss, rrows, _, _ = bench.CONFIGS[a.config]
datas = jd_synth.make_images(jd_synth.make_jobs(range(a.batch), W, H, 90, "4:2:0" if ss == "mixed" else ss, rrows,
                                                mixed=ss == "mixed"))
dec = jdamd.Decoder(0)
for _ in range(3):
    outs, st = dec.decode_batch(datas)
assert all(s == 0 for s in st)
s = dec.debug_fetch("stamps").astype(np.int64)
names = ["loads+dc", "scatter", "idct", "colour+stores"]
print(f"{len(s)} tiles")
for k in range(4):
    d = s[:, k + 1] - s[:, k]
    d = d[(s[:, k] > 0) & (s[:, k + 1] > 0)]
    print(f"  {names[k]:14s} mean {d.mean():9.0f}  median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f} cycles")
life = s[:, 4] - s[:, 0]
print(f"  lifetime       mean {life.mean():9.0f}  median {np.median(life):9.0f}")
span = s[:, 4].max() - s[:, 0].min()
print(f"  kernel span {span} cycles; mean resident waves = {life.sum() / span:.0f}")
