"""k_piece walk statistics from a JD_PSTAT diagnostic build (summed over the batch's waves).

    JDAMD_LIB=gpu-jpeg-decoder_amd/libjdamd_pstat.so JD_STAMPS=1 python tools/pstat.py [--config c2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "gpu-jpeg-decoder_amd")):
    sys.path.insert(0, p)
import bench  # noqa: E402
import jd_synth  # noqa: E402
import jdamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--batch", type=int, default=1024)
a = ap.parse_args()
W, H, ss, rrows, _, _ = bench.CONFIGS[a.config]
datas = jd_synth.make_images(jd_synth.make_jobs(range(a.batch), W, H, 90, "4:2:0" if ss == "mixed" else ss, rrows,
                                                mixed=ss == "mixed"))
dec = jdamd.Decoder(0)
outs, st = dec.decode_batch(datas)
assert all(s == 0 for s in st)
v = dec.debug_fetch("stamps").reshape(-1)[:10].astype(float)
names = ["write wave-its", "warm wave-its", "write lane-its", "warm lane-its", "rare lane-syms", "rare wave-its",
         "rounds", "waves", "mend-branch wave-its", "lane symbols"]
for n, x in zip(names, v):
    print(f"{n:22s} {x:14.0f}")
waves = v[7]
print(f"per wave: write its {v[0] / waves:.0f}, warm its {v[1] / waves:.0f}, rounds {v[6] / waves:.0f}")
print(f"lane utilisation: write {v[2] / (64 * v[0]):.3f}, warm {v[3] / (64 * max(v[1], 1)):.3f}")
print(f"rare wave-iteration fraction {v[5] / v[0]:.3f}; rare per lane-symbol {v[4] / v[9]:.4f}; "
      f"symbols per lane-iteration {v[9] / v[2]:.3f}; mend-branch fraction {v[8] / v[0]:.3f}")
