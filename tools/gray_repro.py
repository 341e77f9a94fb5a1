"""Decodes the parity sweep's grayscale mismatches through each path and library (diagnostic)."""
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
for path in ("auto", "sync", "lanes", "full"):
    dec = jdamd.Decoder(0, path=path)
    for p in cases:
        d = parity_sweep.make_image(p)
        st, ref = jdoracle.decode(d)
        outs, status = dec.decode_batch([d])
        same = st == 0 and status[0] == 0 and np.array_equal(outs[0], ref)
        extra = ""
        if status[0] != st:
            try:
                pb = dec.debug_fetch("piece_bit"); pe = dec.debug_fetch("piece_end")
                nm = dec.debug_fetch("piece_nmcu"); em = dec.debug_fetch("piece_emcu")
                extra = f" pieces={len(pb)} bit={list(pb[:8])} end={list(pe[:8])} nmcu={list(nm[:8])} emcu={list(em[:8])}"
            except Exception as e:  # noqa: BLE001
                extra = f" (debug fetch: {e})"
        print(os.environ.get("JDAMD_LIB", "cur")[-20:], path, p["seed"], p["w"], p["h"], "oracle", st, "gpu", status[0],
              "pixels-equal" if same else "", extra, flush=True)
    dec.close()
