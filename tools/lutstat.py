"""Symbols per Huffman lookup and rare-lookup rate versus the LUT index width (k_piece's table
format, jd_internal.hpp HuffLut), from a sequential decode of synthetic bench images.

    python tools/lutstat.py [n_images] [width] [height]

A lookup resolves one symbol, or two when the first is an AC symbol other than EOB that leaves its
block open and both codes + magnitudes fit the index (the second's magnitude <= 8 bits, an int9
value); codes longer than the index, AC sizes >= 10 and DC sizes > 11 are rare entries.
"""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.abspath(__file__))]
import jd_synth  # noqa: E402
import jd_trace  # noqa: E402


def symbols(d):
    """(k before the symbol, code length, magnitude size, symbol) of every symbol of a JPEG."""
    t = jd_trace.parse(d)
    pattern, nmcu = jd_trace._layout(t)
    bpm, ri = len(pattern), t.ri or nmcu
    out = []
    for si, data in enumerate(jd_trace.segments(d, t.ecs)):
        m0, m1 = si * ri, min(si * ri + ri, nmcu)
        if m0 >= nmcu:
            break
        nblk = (m1 - m0) * bpm
        val, total = int.from_bytes(data + b"\xff" * 8, "big"), (len(data) + 8) * 8
        p = bi = k = blocks = 0
        while blocks < nblk or k != 0:
            L, sym, _ = jd_trace._symbol(t, pattern, val, total, p, bi, k)
            s = sym if k == 0 else sym & 15
            out.append((k, L - s, s, sym))
            p += L
            blocks += k == 0
            k, fin, _ = jd_trace._step(k, sym)
            if fin:
                bi = 0 if bi + 1 == bpm else bi + 1
            if blocks >= nblk and k == 0:
                break
    return out


def lookups(S, W):
    i = looks = rare = 0
    while i < len(S):
        k, l, s, sym = S[i]
        looks += 1
        i += 1
        if k == 0:
            rare += l > W or s > 11
            continue
        if l > W or s >= 10:
            rare += 1
            continue
        L1 = l + s
        if sym == 0 or L1 >= W or i >= len(S):
            continue
        k2, l2, s2, _ = S[i]
        if k2 != 0 and l2 + s2 <= W - L1 and s2 <= 8:
            i += 1
    return looks, rare


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
    h = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
    S = [x for d in jd_synth.make_batch(n, w, h, 90, "4:2:0", 1, 0, seed0=3) for x in symbols(d)]
    print("symbols", len(S))
    for W in (9, 10, 11, 12):
        looks, rare = lookups(S, W)
        print(f"{W} bits: {len(S) / looks:.3f} symbols per lookup, rare {100 * rare / looks:.2f} % of lookups")
