"""Lanes-path piece records of the parity sweep's grayscale mismatches (diagnostic)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tools", "tests", "oracle", "gpu-jpeg-decoder_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import torch  # noqa: F401,E402
import numpy as np  # noqa: E402
import jdamd  # noqa: E402
import jdoracle  # noqa: E402
import parity_sweep  # noqa: E402

cases = [m["params"] for m in json.load(open(sys.argv[1]))["mismatches"]]
dec = jdamd.Decoder(0, path="lanes")
for p in cases:
    d = parity_sweep.make_image(p)
    h = jdamd.parse(d)
    outs, status = dec.decode_batch([d])
    f = {k: dec.debug_fetch(k) for k in ("seg_cstart", "seg_cend", "seg_nsub", "piece_bit", "piece_end", "piece_nmcu", "piece_emcu", "piece_nent")}
    ns = int(f["seg_nsub"][0])
    print(p["seed"], p["w"], p["h"], "q", p["q"], "mcu", h.mcux, h.mcuy, "ri", h.restart_interval, "status", status[0],
          "seg bits", (int(f["seg_cend"][0]) - int(f["seg_cstart"][0])) * 8, "nsub", ns,
          "piece0 bit/end/nmcu/emcu/nent", int(f["piece_bit"][0]), int(f["piece_end"][0]), int(f["piece_nmcu"][0]),
          int(f["piece_emcu"][0]), int(f["piece_nent"][0]), flush=True)
dec.close()
