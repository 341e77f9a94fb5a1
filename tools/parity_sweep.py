"""Randomised GPU parity sweep (test infrastructure; run on the GPU box).

    python tools/parity_sweep.py --minutes 6 --seed 1 --out gpurun_out/sweep.json

Batches of synthetic JPEGs with random size (1 .. 2000 x 1 .. 1200, mostly small), sampling layout
(4:4:4 / 4:2:2 / 4:2:0 / 4:4:0 / grayscale), quality (20 .. 100), restart interval (none, MCU rows,
MCU counts), encoder (tools/jdenc.c with the Annex K tables, or Pillow with its standard or its
optimised per-image Huffman tables; Pillow has no 4:4:0) and, for about a fifth of them, bit flips in
the entropy-coded data, are decoded in one
batch call on the GPU through each entropy-decode path of the library (default, "sync": 1024-bit
pieces with most speculative starts failing, "lanes": one lane per restart interval, "full": the
full-batch piece geometry whatever the batch size; --fancy: with libjpeg fancy upsampling) and compared
with the oracle (oracle/jdoracle.c via oracle/jdoracle.py, in a process pool): per-image status, and
the pixels when the oracle decodes the image.  Any difference is written to --out with the image's
parameters and the run exits non-zero.  The oracle is the checker only; nothing here is timed.
"""
import argparse
import hashlib
import json
import os
import sys
import time
import multiprocessing
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gpu-jpeg-decoder_amd"))

LAYOUTS = ["4:4:4", "4:2:2", "4:2:0", "4:4:0", "gray"]


def make_image(args):
    """(params) -> JPEG bytes; params = dict of the image's random choices."""
    import jd_synth

    p = args
    gray = p["ss"] == "gray"
    px = jd_synth.synth_pixels(p["w"], p["h"], p["seed"], gray)
    if p.get("flat"):  # flat areas (DC-only blocks): the densest streams, which overflow the default
                       # plan's optimistic piece regions at long pieces (jd_runtime.cpp run_retries)
        rng = np.random.default_rng(p["seed"] ^ 0xF1A7)
        cell = int(rng.integers(8, 129))
        gh, gw = -(-p["h"] // cell), -(-p["w"] // cell)
        grid = rng.integers(0, 256, (gh, gw) if gray else (gh, gw, 3), dtype=np.uint8)
        px = np.ascontiguousarray(np.repeat(np.repeat(grid, cell, 0), cell, 1)[: p["h"], : p["w"]])
    enc = p.get("enc", "jdenc")  # jdenc | pil | pil-opt
    data = jd_synth.encode(px, p["q"], "4:4:4" if gray else p["ss"], p["rows"], p["blocks"],
                           optimize=enc == "pil-opt", encoder="jdenc" if enc == "jdenc" else "pil")
    if p["flips"]:
        rng = np.random.default_rng(p["seed"] ^ 0x5EED)
        d = bytearray(data)
        lo = max(2, len(d) // 3)
        for _ in range(p["flips"]):
            i = int(rng.integers(lo, len(d) - 2))
            d[i] ^= 1 << int(rng.integers(0, 8))
        data = bytes(d)
    return data


def oracle_digest(data, fancy=False):
    import jdoracle

    st, ref = jdoracle.decode(data, fancy=fancy)
    return st, (hashlib.sha256(ref.tobytes()).hexdigest() if st == 0 else None)


def oracle_digest_fancy(data):
    return oracle_digest(data, True)


def draw(rng, seed, pil=False):
    small = rng.random() < 0.85
    w = int(rng.integers(1, 400 if small else 2001))
    h = int(rng.integers(1, 300 if small else 1201))
    r = rng.random()
    rows, blocks = (0, 0) if r < 0.4 else ((int(rng.integers(1, 4)), 0) if r < 0.7 else (0, int(rng.integers(1, 12))))
    d = {"seed": int(seed), "w": w, "h": h, "ss": LAYOUTS[int(rng.integers(0, len(LAYOUTS)))],
         "q": int(rng.choice([20, 35, 50, 75, 90, 95, 100])), "rows": rows, "blocks": blocks,
         "flips": int(rng.integers(1, 4)) if rng.random() < 0.2 else 0, "flat": bool(rng.random() < 0.15)}
    if pil:
        e = rng.random()
        d["enc"] = "jdenc" if e < 0.6 or d["ss"] == "4:4:0" else ("pil" if e < 0.75 else "pil-opt")
    return d


def main():
    import torch  # noqa: F401  (torch's HIP runtime first: INTEGRATION.md)
    import jdamd

    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=5.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--batch", type=int, default=96)
    ap.add_argument("--workers", type=int, default=12)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sweep.json"))
    ap.add_argument("--fancy", action="store_true", help="libjpeg fancy upsampling (its oracle: jdoracle fancy=True)")
    ap.add_argument("--pil", action="store_true", help="also Pillow-encoded images (standard and optimised tables)")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    paths = ["auto", "sync", "lanes", "full"]
    # the workers come from a fork server started (and the pool filled) before this process
    # initialises the GPU: no worker is a fork of a process holding a HIP context
    pool = ProcessPoolExecutor(a.workers, mp_context=multiprocessing.get_context("forkserver"))
    list(pool.map(time.sleep, [0.2] * a.workers))
    decs = {p: jdamd.Decoder(0, path=p, fancy=a.fancy) for p in paths}
    t_end = time.time() + 60 * a.minutes
    n_img = n_ok = n_bad_status = 0
    fails = []
    seed = a.seed * 1000003
    with pool:
        it = 0
        while time.time() < t_end and len(fails) < 20:
            params = []
            for _ in range(a.batch):
                params.append(draw(rng, seed, a.pil))
                seed += 1
            datas = list(pool.map(make_image, params, chunksize=4))
            ref = list(pool.map(oracle_digest_fancy if a.fancy else oracle_digest, datas, chunksize=4))
            path = paths[it % len(paths)]
            outs, status = decs[path].decode_batch(datas)
            for p, d, o, s, (st, dig) in zip(params, datas, outs, status, ref):
                n_img += 1
                if s != st:
                    fails.append({"path": path, "params": p, "gpu_status": s, "oracle_status": st})
                    continue
                if st == 0:
                    n_ok += 1
                    if hashlib.sha256(np.ascontiguousarray(o).tobytes()).hexdigest() != dig:
                        fails.append({"path": path, "params": p, "pixels": "differ"})
                else:
                    n_bad_status += 1
            it += 1
            print(f"batch {it} ({path}): {n_img} images, {n_ok} decoded, {n_bad_status} corrupt (status equal), "
                  f"{len(fails)} mismatches", flush=True)
    retried = {p: d.stats()["retried_images"] for p, d in decs.items()}
    for d in decs.values():
        d.close()
    res = {"retried_images": retried, "images": n_img, "decoded_equal_or_checked": n_ok, "corrupt_status_checked": n_bad_status,
           "batches": it, "mismatches": fails, "seed": a.seed, "minutes": a.minutes, "fancy": a.fancy, "pil": a.pil,
           "paths": paths}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "mismatches"}), "mismatches:", len(fails))
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
