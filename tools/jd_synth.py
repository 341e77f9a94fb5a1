"""Deterministic synthetic JPEG inputs for tests and bench.py.

Per image i: each channel = 128 + A*sin(x*fx + y*fy + phi) + N(0, 3), with (A, fx, fy, phi) drawn
from a generator seeded by i; encoded as baseline JPEG with the standard Huffman tables
(optimize=False) at the requested quality / subsampling / restart interval.

Encoding uses the in-repo baseline encoder tools/jdenc.c by default (JD_ENCODER=pillow selects
Pillow / libjpeg-turbo; optimized-table fixtures always use Pillow).  Generation is parallel
(processes) because a 1024-image 1080p batch takes several seconds serially.
"""
from __future__ import annotations

import io
import os
from concurrent.futures import ProcessPoolExecutor
from typing import List, Optional

import numpy as np


def synth_pixels(w: int, h: int, seed: int, gray: bool = False) -> np.ndarray:
    rng = np.random.default_rng(seed)
    yy = np.arange(h, dtype=np.float32)[:, None]
    xx = np.arange(w, dtype=np.float32)[None, :]
    chans = []
    for _ in range(1 if gray else 3):
        fx, fy = (rng.uniform(1 / 80, 1 / 20, 2) * 2 * np.pi).astype(np.float32)
        phi = np.float32(rng.uniform(0, 2 * np.pi))
        amp = np.float32(rng.uniform(40, 110))
        c = 128 + amp * np.sin(xx * fx + yy * fy + phi) + rng.normal(0, 3, (h, w)).astype(np.float32)
        chans.append(np.clip(np.rint(c), 0, 255).astype(np.uint8))
    return chans[0] if gray else np.stack(chans, -1)


def default_encoder() -> str:
    return os.environ.get("JD_ENCODER", "jdenc")


def encode(pixels: np.ndarray, quality: int = 90, subsampling: str = "4:2:0", restart_rows: int = 0,
           restart_blocks: int = 0, optimize: bool = False, encoder: Optional[str] = None) -> bytes:
    encoder = encoder or default_encoder()
    if encoder == "jdenc" and not optimize:
        import jdenc

        return jdenc.encode(pixels, quality, subsampling, restart_rows, restart_blocks)
    from PIL import Image

    img = Image.fromarray(pixels, "L" if pixels.ndim == 2 else "RGB")
    kw = dict(quality=quality, optimize=optimize)
    if pixels.ndim == 3:
        kw["subsampling"] = subsampling
    if restart_rows:
        kw["restart_marker_rows"] = restart_rows
    if restart_blocks:
        kw["restart_marker_blocks"] = restart_blocks
    b = io.BytesIO()
    img.save(b, "JPEG", **kw)
    return b.getvalue()


def _one(args):
    w, h, seed, quality, subsampling, rrows, rblocks, encoder = args
    gray = subsampling == "gray"
    return encode(synth_pixels(w, h, seed, gray), quality, "4:4:4" if gray else subsampling, rrows, rblocks,
                  encoder=encoder)


MIXED_SUBSAMPLING = ("4:4:4", "4:2:2", "4:2:0")
MIXED_QUALITY = (50, 75, 90, 95)
# Bits per pixel of these synthetic images at 1080p (jdenc, standard tables), by subsampling and
# quality: the ECS-size model bench.py balances mixed shards with (measured; 480x272 images run
# about 8 % higher).
BPP_1080P = {"4:4:4": (1.594, 2.247, 3.561, 5.467), "4:2:2": (1.237, 1.726, 2.765, 4.093),
             "4:2:0": (0.972, 1.385, 2.260, 3.426)}


def mixed_params(seed: int):
    """(subsampling, quality) of image `seed` of a mixed batch (BASELINE config 5): subsampling
    cycles with the seed, quality is drawn from {50, 75, 90, 95} by it."""
    ss = MIXED_SUBSAMPLING[seed % 3]
    q = MIXED_QUALITY[int(np.random.default_rng(seed + 7777).integers(0, 4))]
    return ss, q


def estimated_bytes(w: int, h: int, subsampling: str, quality: int) -> float:
    """Model of an image's size (jdenc, standard tables) for shard balancing; 4:2:0 q90 otherwise."""
    row = BPP_1080P.get(subsampling, BPP_1080P["4:2:0"])
    qi = MIXED_QUALITY.index(quality) if quality in MIXED_QUALITY else 2
    return w * h * row[qi] / 8.0


def make_jobs(seeds, w, h, quality=90, subsampling="4:2:0", restart_rows=0, restart_blocks=0, mixed=False,
              encoder=None):
    jobs = []
    for s in seeds:
        if mixed:
            ss, q = mixed_params(int(s))
            jobs.append((w, h, int(s), q, ss, 0, 0, encoder))
        else:
            jobs.append((w, h, int(s), quality, subsampling, restart_rows, restart_blocks, encoder))
    return jobs


def make_images(jobs, workers: Optional[int] = None) -> List[bytes]:
    n = len(jobs)
    workers = workers or min(16, os.cpu_count() or 1, max(1, n))
    if workers <= 1 or n < 4:
        return [_one(j) for j in jobs]
    with ProcessPoolExecutor(workers) as ex:
        return list(ex.map(_one, jobs, chunksize=max(1, n // (workers * 4))))


def make_batch(n: int, w: int, h: int, quality: int = 90, subsampling: str = "4:2:0", restart_rows: int = 0,
               restart_blocks: int = 0, seed0: int = 0, workers: Optional[int] = None,
               mixed: bool = False, encoder: Optional[str] = None) -> List[bytes]:
    """n synthetic JPEGs of seeds seed0 .. seed0+n-1.  mixed=True: BASELINE config 5 (mixed_params
    per seed), without restart markers."""
    jobs = make_jobs(range(seed0, seed0 + n), w, h, quality, subsampling, restart_rows, restart_blocks, mixed,
                     encoder)
    return make_images(jobs, workers)
