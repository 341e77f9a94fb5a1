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


def _symbol(t, pattern, val, total, p, bi, k):
    """Decodes the symbol at bit p in state (bi, k): (code+magnitude bits, symbol, value) or None."""
    comp = pattern[bi]
    tab = t.dht[(0, t.td[comp])] if k == 0 else t.dht[(1, t.ta[comp])]

    def peek(q, n):
        if n == 0:
            return 0
        return (val >> (total - q - n)) & ((1 << n) - 1) if q + n <= total else 0

    for ln in range(1, 17):
        if (ln, peek(p, ln)) in tab:
            sym = tab[(ln, peek(p, ln))]
            s = sym if k == 0 else sym & 15
            v = peek(p + ln, s)
            if s and v < (1 << (s - 1)):
                v -= (1 << s) - 1
            return ln + s, sym, v
    return None


def _step(k, sym):
    """(next k, block finished, coefficient index emitted or None) — parser.cpp:114-134."""
    if k == 0:
        return 1, False, None
    if sym == 0:
        return 0, True, None
    knew = k + (sym >> 4)
    emit = knew if (sym & 15) and knew < 64 else None
    kn = knew + 1 if knew < 64 else knew
    return (0, True, emit) if kn >= 64 else (kn, False, emit)


def mcu_starts(d: bytes):
    """Per interval: [(bit, AC entries before)] of every MCU start (ground truth for the pieces)."""
    t = parse(d)
    pattern, nmcu = _layout(t)
    ri = t.ri or nmcu
    out = []
    for si, data in enumerate(segments(d, t.ecs)):
        m0 = si * ri
        if m0 >= nmcu:
            break
        n = min(m0 + ri, nmcu) - m0
        val = int.from_bytes(data + b"\xff" * 16, "big")
        total = (len(data) + 16) * 8
        p, bi, k, ents, starts = 0, 0, 0, 0, [(0, 0)]
        while len(starts) <= n:
            L, sym, _ = _symbol(t, pattern, val, total, p, bi, k)
            p += L
            k, fin, emit = _step(k, sym)
            ents += emit is not None
            if fin:
                bi = (bi + 1) % len(pattern)
                if bi == 0:
                    starts.append((p, ents))
        out.append({"bits": len(data) * 8, "starts": starts[:n + 1]})
    return out


def _walk_scan(t, pattern, val, total, bits, start, warm_to, stop_at):
    """The GPU's walk<kWalkScan> (jd_kernels.hip) restated: (m_start, m_end, mcus, entries)."""
    p, bi, k = start, 0, 0
    counting = warm_to == start
    m_start = start if counting else None
    mcus = ents = 0
    if counting and (start + 8 > bits or start >= stop_at):  # at the data end / past its share: empty
        return start, start, 0, 0
    while True:
        r = _symbol(t, pattern, val, total, p, bi, k)
        L, sym, _ = r if r else (16, 0, 0)
        p += L
        k, fin, emit = _step(k, sym) if r else (k, False, None)
        if counting and emit is not None:
            ents += 1
        mcu_end = fin and (bi + 1) % len(pattern) == 0
        if fin:
            bi = (bi + 1) % len(pattern)
        if not counting and mcu_end and p >= warm_to:
            counting, m_start = True, p
            if p + 8 > bits or p >= stop_at:  # no MCU begins in the piece's share: empty
                return m_start, p, 0, 0
        elif counting and mcu_end:
            mcus += 1
            if p >= stop_at or p + 8 > bits:
                return m_start, p, mcus, ents
        if p > bits or (counting and r is None):
            return m_start, p, mcus, ents


def emulate(d: bytes, piece_bits: int = 8192, overlap: int = 4096):
    """Runs scan -> chain -> write as the GPU does; returns per-block (dc, [(zz, value)...]) in
    scan order (DC already predicted) and the number of chain re-scans."""
    t = parse(d)
    pattern, nmcu = _layout(t)
    bpm = len(pattern)
    ri = t.ri or nmcu
    result, rescans = [], 0
    for si, data in enumerate(segments(d, t.ecs)):
        m0 = si * ri
        if m0 >= nmcu:
            break
        nm = min(m0 + ri, nmcu) - m0
        bits = len(data) * 8
        val = int.from_bytes(data + b"\xff" * 16, "big")
        total = (len(data) + 16) * 8
        n = max(1, -(-bits // piece_bits))
        plen = -(-bits // n)  # equal shares (jd_kernels.hip piece_len)
        big = 1 << 40
        pcs = []
        for j in range(n):  # scan
            pstart = j * plen
            warm_to = 0 if j == 0 else min(pstart, bits)
            start = 0 if pstart <= overlap else min(pstart - overlap, warm_to)
            stop_at = big if j == n - 1 else pstart + plen
            ms, me, mc, en = _walk_scan(t, pattern, val, total, bits, start, warm_to, stop_at)
            pcs.append([0 if j == 0 else ms, me, mc, en])
        for j in range(1, n):  # chain: verify, re-scan from the verified boundary
            if pcs[j][0] != pcs[j - 1][1]:
                rescans += 1
                st = pcs[j - 1][1]
                stop_at = big if j == n - 1 else (j + 1) * plen
                ms, me, mc, en = _walk_scan(t, pattern, val, total, bits, st, st, stop_at)
                pcs[j] = [st, me, mc, en]
        blocks = []
        pred = [0, 0, 0]
        mcu_run = 0
        for j in range(n):  # write
            cnt = pcs[j][2] if j < n - 1 else nm - mcu_run
            mcu_run += cnt
            p, bi, k = pcs[j][0], 0, 0
            ents = []
            for _ in range(cnt * bpm):
                while True:
                    L, sym, v = _symbol(t, pattern, val, total, p, bi, k)
                    p += L
                    if k == 0:
                        c = pattern[bi]
                        pred[c] += v
                        dc, ents = pred[c], []
                    k, fin, emit = _step(k, sym)
                    if emit is not None:
                        ents.append((emit, v))
                    if fin:
                        bi = (bi + 1) % bpm
                        blocks.append((dc, ents))
                        break
        result.extend(blocks)
    return result, rescans
