"""Speculative-start statistics of an image at a piece geometry (CPU, pure Python).

    python tools/sync_stats.py [--size 2000] [--quality 95] [--piece 256] [--overlap 768] [--sample 600]

For a sample of the pieces of the reference's latency image (4:4:4, `bench.ref444_jobs`, no DRI)
cut as k_piece cuts them (equal shares of about `piece` bits, a warm-up of `overlap` bits before
each nominal start in the guessed state: first block of an MCU, DC next), reports how many
speculative starts land on a true MCU boundary, and for the ones that do not, the walk length
after which the wrong walk first reaches a true MCU boundary (its sync distance): the bits a
re-walk chain needs before a piece's start comes out right.  Round-based repair extends a failed
piece's walk by one piece per round, so ceil((distance - overlap) / piece) rounds is what such a
piece waits for.  The ground truth (every MCU start) comes from tools/jd_trace.py's own decoder.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import jd_synth  # noqa: E402
import jd_trace as T  # noqa: E402


def sync_distance(t, pattern, val, total, bits, start, truth, limit):
    """Walks from `start` in the guessed state; the first MCU boundary at or after nominal points
    is not needed here: returns the walk length (bits) at which an MCU boundary of the walk is a true
    MCU start, or None within `limit` bits / at a decode error past the data."""
    p, bi, k = start, 0, 0
    while p - start < limit and p < bits:
        r = T._symbol(t, pattern, val, total, p, bi, k)
        L, sym, _ = r if r else (16, 0, 0)
        p += L
        k, fin, _ = T._step(k, sym) if r else (k, False, None)
        if fin:
            bi = (bi + 1) % len(pattern)
            if bi == 0 and p in truth:
                return p - start
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=2000)
    ap.add_argument("--quality", type=int, default=95)
    ap.add_argument("--piece", type=int, default=256)
    ap.add_argument("--overlap", type=int, default=768)
    ap.add_argument("--sample", type=int, default=600)
    ap.add_argument("--limit", type=int, default=65536)
    a = ap.parse_args()
    import bench

    (d,) = jd_synth.make_images(bench.ref444_jobs([bench.REF_SIZES.index(a.size)], a.quality), workers=1)
    t = T.parse(d)
    pattern, _ = T._layout(t)
    (seg,) = T.mcu_starts(d)
    truth = set(b for b, _ in seg["starts"])
    (data,) = T.segments(d, t.ecs)
    bits = len(data) * 8
    val = int.from_bytes(data + b"\xff" * 16, "big")
    total = (len(data) + 16) * 8
    n = max(1, -(-bits // a.piece))
    plen = -(-bits // n)
    rng = np.random.default_rng(1)
    js = sorted(int(j) for j in rng.choice(np.arange(1, n), size=min(a.sample, n - 1), replace=False))
    fails, dists = 0, []
    for j in js:
        pstart = j * plen
        start = max(0, pstart - a.overlap)
        ms, _, _, _ = T._walk_scan(t, pattern, val, total, bits, start, pstart, pstart + plen)
        if ms in truth:
            continue
        fails += 1
        dists.append(sync_distance(t, pattern, val, total, bits, start, truth, a.limit))
    done = [x for x in dists if x is not None]
    rounds = [max(0, -(-(x - a.overlap) // plen)) for x in done]
    out = {"image": f"{a.size}^2 4:4:4 q{a.quality}", "bits": bits, "pieces": n, "piece_bits": plen,
           "overlap": a.overlap, "sampled": len(js), "failed_starts": fails, "fail_frac": fails / len(js),
           "sync_distance_bits": {"median": float(np.median(done)) if done else None,
                                  "p90": float(np.percentile(done, 90)) if done else None,
                                  "max": max(done) if done else None, "unsynced_within_limit": len(dists) - len(done)},
           "rounds_to_sync": {"median": float(np.median(rounds)) if rounds else None,
                              "p90": float(np.percentile(rounds, 90)) if rounds else None,
                              "max": max(rounds) if rounds else None}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
