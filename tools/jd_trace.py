"""Bit-level trace of a baseline JPEG's entropy decode (pure Python, test/debug tooling only).

For every restart interval (segment) it reports the un-stuffed data length and, for every
kSubBits-bit subsequence, the true decoder state at its first symbol (bit position, block-in-MCU,
coefficient index, AC entries of the current block) plus the counts the GPU count pass must
produce.  Used by tests/test_gpu.py to check the self-synchronising decode's intermediate arrays
(exit states, prefix sums) against an independent sequential decode.  Small images only.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

SUB_BITS = 512


@dataclass
class Tables:
    width: int = 0
    height: int = 0
    comps: List[Tuple[int, int, int, int]] = field(default_factory=list)  # (id, h, v, tq)
    td: List[int] = field(default_factory=list)
    ta: List[int] = field(default_factory=list)
    dht: Dict[Tuple[int, int], Dict[Tuple[int, int], int]] = field(default_factory=dict)  # (len, code) -> sym
    ri: int = 0
    ecs: int = 0


def parse(d: bytes) -> Tables:
    t = Tables()
    p = 2
    while True:
        while d[p + 1] == 0xFF:
            p += 1
        m = d[p + 1]
        p += 2
        if m in (0xD8, 0x01) or 0xD0 <= m <= 0xD7:
            continue
        L = struct.unpack(">H", d[p:p + 2])[0]
        s = d[p + 2:p + L]
        if m in (0xC0, 0xC1):
            t.height, t.width = struct.unpack(">HH", s[1:5])
            t.comps = [(s[6 + 3 * c], s[7 + 3 * c] >> 4, s[7 + 3 * c] & 15, s[8 + 3 * c]) for c in range(s[5])]
        elif m == 0xC4:
            q = 0
            while q < len(s):
                tc, th = s[q] >> 4, s[q] & 15
                counts = s[q + 1:q + 17]
                vals = s[q + 17:q + 17 + sum(counts)]
                code, k, table = 0, 0, {}
                for ln in range(1, 17):
                    for _ in range(counts[ln - 1]):
                        table[(ln, code)] = vals[k]
                        code += 1
                        k += 1
                    code <<= 1
                t.dht[(tc, th)] = table
                q += 17 + sum(counts)
        elif m == 0xDD:
            t.ri = struct.unpack(">H", s[:2])[0]
        elif m == 0xDA:
            ns = s[0]
            t.td = [s[2 + 2 * i] >> 4 for i in range(ns)]
            t.ta = [s[2 + 2 * i] & 15 for i in range(ns)]
            t.ecs = p + L
            return t
        p += L


def segments(d: bytes, ecs: int) -> List[bytes]:
    """Un-stuffed data of each restart interval (fill bytes before a marker excluded)."""
    segs, cur, i = [], bytearray(), ecs
    while i < len(d):
        c = d[i]
        if c == 0xFF:
            n = d[i + 1] if i + 1 < len(d) else 0xD9
            if n == 0x00:
                cur.append(0xFF)
                i += 2
                continue
            if n == 0xFF:
                i += 1
                continue
            if 0xD0 <= n <= 0xD7:
                segs.append(bytes(cur))
                cur = bytearray()
                i += 2
                continue
            break
        cur.append(c)
        i += 1
    segs.append(bytes(cur))
    return segs


def trace(d: bytes, sub_bits: int = SUB_BITS):
    """Returns a list (per segment) of dicts: bits, nsub, entry[j] = (p, bi, k, ncur),
    counts[j] = (blocks, entries, dc0, dc1, dc2)."""
    t = parse(d)
    nc = len(t.comps)
    if nc == 1:
        hs, vs = [1], [1]
    else:
        hs = [c[1] for c in t.comps]
        vs = [c[2] for c in t.comps]
    hmax, vmax = max(hs), max(vs)
    mcux = (t.width + 8 * hmax - 1) // (8 * hmax)
    mcuy = (t.height + 8 * vmax - 1) // (8 * vmax)
    pattern = [c for c in range(nc) for _ in range(hs[c] * vs[c])]
    bpm = len(pattern)
    nmcu = mcux * mcuy
    ri = t.ri or nmcu
    out = []
    for si, data in enumerate(segments(d, t.ecs)):
        m0 = si * ri
        m1 = min(m0 + ri, nmcu)
        if m0 >= nmcu:
            break
        nblk = (m1 - m0) * bpm
        bits = len(data) * 8
        val = int.from_bytes(data + b"\xff" * 8, "big")
        total = (len(data) + 8) * 8

        def peek(p, n):
            return (val >> (total - p - n)) & ((1 << n) - 1)

        states = []  # (p, bi, k, ncur) before every symbol, and the symbol's effect
        p, bi, k, ncur, blocks = 0, 0, 0, 0, 0
        while blocks < nblk or k != 0:
            comp = pattern[bi]
            tab = t.dht[(0, t.td[comp])] if k == 0 else t.dht[(1, t.ta[comp])]
            sym = None
            for ln in range(1, 17):
                if (ln, peek(p, ln)) in tab:
                    sym = tab[(ln, peek(p, ln))]
                    break
            assert sym is not None, "bad code"
            s = sym if k == 0 else sym & 15
            v = peek(p + ln, s) if s else 0
            if s and v < (1 << (s - 1)):
                v -= (1 << s) - 1
            states.append((p, bi, k, ncur, comp, sym, v))
            p += ln + s
            if k == 0:
                blocks += 1
                k, ncur = 1, 0
            elif sym == 0:
                k = 64
            else:
                k += sym >> 4
                if k < 64:
                    if sym & 15:
                        ncur += 1
                    k += 1
            if k >= 64:
                bi = 0 if bi + 1 == bpm else bi + 1
                k = 0
            if blocks >= nblk and k == 0:
                break
        nsub = max(1, -(-bits // sub_bits))
        entry, counts = [], []
        si_ = 0
        for j in range(nsub):
            lo, hi = j * sub_bits, (j + 1) * sub_bits
            while si_ < len(states) and states[si_][0] < lo:
                si_ += 1
            if si_ < len(states):
                entry.append(states[si_][:4])
            else:
                entry.append((p, bi, k, ncur))
            b = e = 0
            dc = [0, 0, 0]
            q = si_
            while q < len(states) and (states[q][0] < hi or j == nsub - 1):
                sp, sbi, sk, sn, comp, sym, v = states[q]
                if sk == 0:
                    b += 1
                    dc[comp] += v
                elif sym != 0 and (sym & 15) and sk + (sym >> 4) < 64:
                    e += 1
                q += 1
            counts.append((b, e, dc[0], dc[1], dc[2]))
        out.append({"bits": bits, "nsub": nsub, "nblk": nblk, "entry": entry, "counts": counts, "end": p})
    return out


def _layout(t: Tables):
    nc = len(t.comps)
    hs = [1] if nc == 1 else [c[1] for c in t.comps]
    vs = [1] if nc == 1 else [c[2] for c in t.comps]
    hmax, vmax = max(hs), max(vs)
    mcux = (t.width + 8 * hmax - 1) // (8 * hmax)
    mcuy = (t.height + 8 * vmax - 1) // (8 * vmax)
    pattern = [c for c in range(nc) for _ in range(hs[c] * vs[c])]
    return pattern, mcux * mcuy


def _decode_range(t, pattern, val, total, p, bi, k, ncur, end, mode, nblk=0, blk=0, ent=0, pred=None,
                  entries=None, blocks=None):
    """The GPU decode_run (jd_kernels.hip) restated: decode symbols that start before `end`.
    mode 0/1: exit (+ counts); mode 2: also writes entries[ent..] and blocks[blk] = (start, cnt, dc)."""
    bpm = len(pattern)
    comp = pattern[bi]
    nblocks = nent = 0
    dcs = [0, 0, 0]
    pred = list(pred or [0, 0, 0])
    cur_blk = blk - 1
    ent_blk = ent - ncur
    dc = pred[comp]

    def peek(q, n):
        if n == 0:
            return 0
        return (val >> (total - q - n)) & ((1 << n) - 1) if q + n <= total else 0

    while p < end:
        if mode == 2 and k == 0 and blk >= nblk:
            break
        tab = t.dht[(0, t.td[comp])] if k == 0 else t.dht[(1, t.ta[comp])]
        sym, ln = 0, 16
        for L in range(1, 17):
            if (L, peek(p, L)) in tab:
                sym, ln = tab[(L, peek(p, L))], L
                break
        s = min(sym if k == 0 else sym & 15, 16)
        v = peek(p + ln, s)
        if s and v < (1 << (s - 1)):
            v -= (1 << s) - 1
        p += ln + s
        if k == 0:
            nblocks += 1
            dcs[comp] += v
            if mode == 2:
                pred[comp] += v
                dc = pred[comp]
                cur_blk = blk
                blk += 1
                ent_blk = ent
            k, ncur = 1, 0
        elif sym == 0:
            k = 64
        else:
            k += sym >> 4
            if k < 64:
                if sym & 15:
                    ncur += 1
                    nent += 1
                    if mode == 2:
                        entries[ent] = (k, v)
                        ent += 1
                k += 1
        if k >= 64:
            if mode == 2:
                blocks[cur_blk] = (ent_blk, ent - ent_blk, dc)
            bi = 0 if bi + 1 == bpm else bi + 1
            comp = pattern[bi]
            k = 0
    return (p, bi, k, ncur), (nblocks, nent, dcs), blk


def emulate(d: bytes, sub_bits: int = SUB_BITS):
    """Runs spec -> count -> chain -> write exactly as the GPU does; returns per-block
    (dc, [(zz, value)...]) in scan order and the number of chain re-decodes."""
    t = parse(d)
    pattern, nmcu = _layout(t)
    bpm = len(pattern)
    ri = t.ri or nmcu
    result = []
    redecodes = 0
    for si, data in enumerate(segments(d, t.ecs)):
        m0 = si * ri
        if m0 >= nmcu:
            break
        nblk = (min(m0 + ri, nmcu) - m0) * bpm
        bits = len(data) * 8
        val = int.from_bytes(data + b"\xff" * 16, "big")
        total = (len(data) + 16) * 8
        n = max(1, -(-bits // sub_bits))

        def end(j):
            return bits if j == n - 1 else (j + 1) * sub_bits

        spec = [_decode_range(t, pattern, val, total, j * sub_bits, 0, 0, 0, end(j), 0)[0] for j in range(n)]
        used = [(0, 0, 0, 0)] + spec[:-1]
        cnt = [_decode_range(t, pattern, val, total, *used[j], end(j), 1)[:2] for j in range(n)]
        true_entry = [(0, 0, 0, 0)]
        for j in range(1, n):  # chain: verify, re-decode broken links
            te = cnt[j - 1][0]
            true_entry.append(te)
            if te != used[j]:
                redecodes += 1
                cnt[j] = _decode_range(t, pattern, val, total, *te, end(j), 1)[:2]
        entries, blocks = {}, {}
        blk, ent, pred = 0, 0, [0, 0, 0]
        for j in range(n):  # write pass from verified entries + prefix sums
            _decode_range(t, pattern, val, total, *true_entry[j], bits + 64 if j == n - 1 else end(j), 2, nblk,
                          blk, ent, pred, entries, blocks)
            c = cnt[j][1]
            blk += c[0]
            ent += c[1]
            pred = [pred[q] + c[2][q] for q in range(3)]
        for b in range(nblk):
            st, n_e, dc = blocks.get(b, (0, 0, None))
            result.append((dc, [entries.get(st + i) for i in range(n_e)]))
    return result, redecodes
