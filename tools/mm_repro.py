"""Repro of parity sweep r06g's one mismatch (tools/mm_r06g.jpg): status per path and pool mode."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), p) for p in ("../gpu-jpeg-decoder_amd", "../oracle")]
import torch  # noqa: F401
import jdamd, jdoracle
sys.path.insert(0, os.path.dirname(__file__)); import parity_sweep; d = parity_sweep.make_image({"seed": 64114030, "w": 318, "h": 183, "ss": "gray", "q": 75, "rows": 0, "blocks": 9, "flips": 1, "flat": True})
print("oracle", jdoracle.decode(d)[0])
for worst in (False, True):
    for path in ("auto", "sync", "lanes", "full"):
        dec = jdamd.Decoder(0, path=path, worst_case_pools=worst)
        outs, st = dec.decode_batch([d])
        ok = st[0] == 0 and __import__("numpy").array_equal(outs[0], jdoracle.decode(d)[1]) if jdoracle.decode(d)[0] == 0 else None
        print("worst" if worst else "opt", path, st, dec.stats()["retried_images"], dec.stats()["fix_intervals"], ok)
        dec.close()
