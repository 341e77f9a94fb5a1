"""Re-encode a baseline JPEG's entropy-coded data under other Huffman tables (test inputs only).

    retable(data, dc_len=4, ac_len=8) -> bytes

Every symbol of the file (DC size / AC run-size, with its magnitude bits) is decoded with the
file's own tables and written again with canonical tables in which every DC symbol has a
`dc_len`-bit code and every AC symbol an `ac_len`-bit code; the DHT segments are replaced and
everything else (headers, restart markers, the coefficients) is kept.  With 4-bit DC and 8-bit AC
codes no block or entry takes fewer than 8 walk bits per region word, so the GPU's region divisor
(jd_plan.cpp region_divisor) is at its maximum, 8 (the tight case of the region bound).
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import jd_trace


def _canonical(syms: List[int], length: int) -> Tuple[bytes, Dict[int, Tuple[int, int]]]:
    """DHT body (16 counts + values) giving every symbol a `length`-bit code, and sym -> (len, code)."""
    assert len(syms) < (1 << length), "too many symbols for that code length"
    counts = [0] * 16
    counts[length - 1] = len(syms)
    return bytes(counts) + bytes(syms), {s: (length, i) for i, s in enumerate(syms)}


class _Reader:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def bit(self) -> int:
        b = (self.d[self.p >> 3] >> (7 - (self.p & 7))) & 1 if (self.p >> 3) < len(self.d) else 1
        self.p += 1
        return b

    def bits(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bit()
        return v

    def sym(self, table: Dict[Tuple[int, int], int]) -> int:
        code = 0
        for ln in range(1, 17):
            code = (code << 1) | self.bit()
            if (ln, code) in table:
                return table[(ln, code)]
        raise ValueError("bad Huffman code")


class _Writer:
    def __init__(self):
        self.out, self.acc, self.n = bytearray(), 0, 0

    def put(self, v: int, n: int) -> None:
        for k in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> k) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)
                self.acc, self.n = 0, 0

    def flush(self) -> bytes:
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)  # 1-bit padding
        return bytes(self.out)


def retable(data: bytes, dc_len: int = 4, ac_len: int = 8) -> bytes:
    t = jd_trace.parse(data)
    nc = len(t.comps)
    hs = [c[1] for c in t.comps] if nc > 1 else [1]
    vs = [c[2] for c in t.comps] if nc > 1 else [1]
    mcux = (t.width + 8 * max(hs) - 1) // (8 * max(hs))
    mcuy = (t.height + 8 * max(vs) - 1) // (8 * max(vs))
    pattern = [c for c in range(nc) for _ in range(hs[c] * vs[c])]
    nmcu = mcux * mcuy
    ri = t.ri or nmcu
    new_codes, dht = {}, b""
    for (tc, th), table in sorted(t.dht.items()):
        syms = sorted(set(table.values()))
        body, codes = _canonical(syms, dc_len if tc == 0 else ac_len)
        new_codes[(tc, th)] = codes
        dht += bytes([(tc << 4) | th]) + body
    segs_out = []
    for si, seg in enumerate(jd_trace.segments(data, t.ecs)):
        m0 = si * ri
        if m0 >= nmcu:
            break
        r, w = _Reader(seg), _Writer()
        for _ in range(m0, min(m0 + ri, nmcu)):
            for c in pattern:
                dct, act = t.dht[(0, t.td[c])], t.dht[(1, t.ta[c])]
                dcc, acc = new_codes[(0, t.td[c])], new_codes[(1, t.ta[c])]
                s = r.sym(dct)
                w.put(dcc[s][1], dcc[s][0])
                w.put(r.bits(s), s)
                k = 1
                while k < 64:
                    s = r.sym(act)
                    w.put(acc[s][1], acc[s][0])
                    if s == 0:
                        break
                    w.put(r.bits(s & 15), s & 15)
                    k += (s >> 4) + 1
        segs_out.append(w.flush())
    # headers up to SOS with the DHT segments replaced by one, then the scan
    out, p = bytearray(data[:2]), 2
    while True:
        m = data[p + 1]
        L = struct.unpack(">H", data[p + 2:p + 4])[0]
        if m == 0xDA:
            out += b"\xff\xc4" + struct.pack(">H", len(dht) + 2) + dht
            out += data[p:p + 2 + L]
            break
        if m != 0xC4:
            out += data[p:p + 2 + L]
        p += 2 + L
    for i, s in enumerate(segs_out):
        out += s
        if i + 1 < len(segs_out):
            out += bytes([0xFF, 0xD0 + (i & 7)])
    out += b"\xff\xd9"
    return bytes(out)
