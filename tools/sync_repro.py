"""Piece records of one image on the "sync" path (diagnostic for a round-3 parity-sweep case)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tools", "tests", "oracle", "gpu-jpeg-decoder_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch  # noqa: F401,E402
import jdamd  # noqa: E402
import parity_sweep  # noqa: E402

p = {"seed": 16038946, "w": 366, "h": 10, "ss": "gray", "q": 100, "rows": 0, "blocks": 0, "flips": 1}
d = parity_sweep.make_image(p)
h = jdamd.parse(d)
print("ecs_offset", h.ecs_offset, "mcus", h.mcux * h.mcuy, "len", len(d))
for path in ("sync", "auto"):
    dec = jdamd.Decoder(0, path=path)
    outs, status = dec.decode_batch([d])
    f = {k: dec.debug_fetch(k) for k in ("seg_nsub", "piece_bit", "piece_end", "piece_nmcu", "piece_emcu", "piece_join", "piece_amcu")}
    n = int(f["seg_nsub"][0])
    print(path, "status", status[0], "pieces", n)
    for j in range(n):
        print(f"  {j:3d} bit {int(f['piece_bit'][j]):7d} end {int(f['piece_end'][j]):7d} nmcu {int(f['piece_nmcu'][j]):4d} "
              f"emcu {int(f['piece_emcu'][j]):11d} join {int(f['piece_join'][j]):#x} amcu {int(f['piece_amcu'][j])}")
    dec.close()
