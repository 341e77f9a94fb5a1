"""White-box checks of the piece-parallel Huffman decode (GPU): intermediate arrays of the last
batch (jd_debug_fetch) against an independent sequential bit-level trace (tools/jd_trace.py).
The decoder uses 1024-bit pieces here (path="sync"), so many pieces start speculatively and
some need the chain's re-scan.

  seg_cstart/seg_cend          -> un-stuffed interval lengths
  piece_bit/mcu0/abase         -> every piece starts on a true MCU boundary, with the right MCU
                                  index; its blocks come from its own region (or a spare one)
  blocks                       -> per-block AC-entry counts and DC differences vs the oracle
                                  (the DC predictor itself runs inside k_idct_color)
"""
import os
import sys

import numpy as np
import pytest

import jdamd
import jdoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import jd_trace  # noqa: E402

pytestmark = pytest.mark.gpu

CASES = ["ref/1_320x240.jpg", "ref/3_120x120.jpg", "ref/2_400x400.jpg", "gen/g055_64x48_444_q75_blocks3.jpg",
         "gen/g058_64x48_422_q75_blocks3.jpg", "gen/g061_64x48_420_q75_blocks3.jpg"]


def _load(name):
    with open(os.path.join(ROOT, "tests", "golden", name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name", CASES)
def test_intervals_and_piece_starts(sync_decoder, name):
    data = _load(name)
    try:
        sync_decoder.decode(data)
    except Exception:
        pass  # inspect the intermediate state even when the decode reports an error
    truth = jd_trace.mcu_starts(data)
    cs = sync_decoder.debug_fetch("seg_cstart")
    ce = sync_decoder.debug_fetch("seg_cend")
    ssb = sync_decoder.debug_fetch("seg_sub_base")
    nsub = sync_decoder.debug_fetch("seg_nsub")
    pbit = sync_decoder.debug_fetch("piece_bit")
    pm0 = sync_decoder.debug_fetch("piece_mcu0")
    pnm = sync_decoder.debug_fetch("piece_nmcu")
    pab = sync_decoder.debug_fetch("piece_abase")
    pjoin = sync_decoder.debug_fetch("piece_join")
    sent = sync_decoder.debug_fetch("seg_ent")
    div = int(sync_decoder.debug_fetch("rw_div")[0])  # jd_plan.hpp region_sizing of the image
    slack = int(sync_decoder.debug_fetch("rw_slack")[0])
    assert 2 <= div <= 8 and slack <= 1040
    errs = []
    for s, seg in enumerate(truth):
        if (int(ce[s]) - int(cs[s])) * 8 != seg["bits"]:
            errs.append(f"seg {s}: bits gpu {(int(ce[s]) - int(cs[s])) * 8} want {seg['bits']}")
            continue
        want_n = max(1, -(-seg["bits"] // 1024))
        if int(nsub[s]) != want_n:
            errs.append(f"seg {s}: pieces gpu {nsub[s]} want {want_n}")
            continue
        plen = -(-seg["bits"] // want_n)
        rw = ((plen + div - 1) // div + slack + 7) // 8 * 8  # jd_internal.hpp region_words (kRegionAlign 8)
        starts = {b: (m, e) for m, (b, e) in enumerate(seg["starts"])}
        nm = 0
        for j in range(want_n):
            u = int(ssb[s]) + j
            b = int(pbit[u])
            if b not in starts:
                errs.append(f"seg {s} piece {j}: bit {b} is not an MCU boundary")
                continue
            m, e = starts[b]
            if int(pm0[u]) != m and not (j == want_n - 1 and int(pnm[u]) == 0):
                errs.append(f"seg {s} piece {j}: mcu0 gpu {pm0[u]} want {m}")
            # segment A: the piece's own region, or (re-walked) a spare region past every own one
            own = int(sent[s]) + j * rw
            if int(pab[u]) != own and int(pab[u]) < own + rw:
                errs.append(f"seg {s} piece {j}: region {int(pab[u])} overlaps own {own}")
            if (int(pjoin[u]) & 0xFFFF) > ((int(pjoin[u]) >> 16) & 0xFF):
                errs.append(f"seg {s} piece {j}: joined checkpoint {int(pjoin[u]) & 0xFFFF} of {(int(pjoin[u]) >> 16) & 0xFF}")
            nm += int(pnm[u])
        if nm != len(seg["starts"]) - 1:
            errs.append(f"seg {s}: MCUs gpu {nm} want {len(seg['starts']) - 1}")
        if len(errs) > 20:
            break
    assert not errs, "\n".join(errs[:20])


@pytest.mark.parametrize("name", CASES)
def test_scan_checkpoints(sync_decoder, name):
    """Checkpoints (k_piece) sit on true MCU boundaries with the MCU and AC-entry counts from the
    piece start, for every piece whose speculative start synchronised (the join relies on both),
    and record no error in the segment before them (kNoError; the images are valid)."""
    data = _load(name)
    try:
        sync_decoder.decode(data)
    except Exception:
        pass
    truth = jd_trace.mcu_starts(data)
    ssb = sync_decoder.debug_fetch("seg_sub_base")
    nsub = sync_decoder.debug_fetch("seg_nsub")
    pbit = sync_decoder.debug_fetch("piece_bit")
    cp = sync_decoder.debug_fetch("piece_cp").reshape(-1, 9, 4)
    pjoin = sync_decoder.debug_fetch("piece_join")
    checked = bad = 0
    for s, seg in enumerate(truth):
        starts = {b: (m, e) for m, (b, e) in enumerate(seg["starts"])}
        for j in range(int(nsub[s])):
            u = int(ssb[s]) + j
            ncp = (int(pjoin[u]) >> 16) & 0xFF  # (tail count << 24 | checkpoints << 16)
            assert ncp <= 8
            b0 = int(pbit[u])
            if b0 not in starts or ncp == 0:
                continue
            m0, e0 = starts[b0]
            for c in range(ncp):
                bit, mcus, ents, err = (int(x) for x in cp[u, c])
                if bit in starts and (starts[bit][0] - m0, starts[bit][1] - e0) == (mcus, ents) and err == 0xFFFFFFFF:
                    checked += 1
                else:
                    bad += 1
    # a piece whose speculative start did not synchronise records its checkpoints on a wrong
    # trajectory (k_redo ignores them unless it meets one at an MCU boundary)
    assert checked > 0 and bad <= checked // 20, (checked, bad)


def _s16(x):
    return ((x + 0x8000) & 0xFFFF) - 0x8000


def dc_differences(data, dc):
    """The oracle's absolute DCs (MCU-interleaved block order) as the differences the write pass
    stores: per component, the predictor restarts at 0 at every restart interval
    (parser.cpp:106-111)."""
    h = jdamd.parse(data)
    comp_of = [c for c in range(h.ncomp) for _ in range(h.h[c] * h.v[c])]
    out = np.zeros_like(dc)
    pred = [0, 0, 0, 0]
    for i in range(dc.shape[0]):
        mcu, bb = divmod(i, h.blocks_per_mcu)
        if bb == 0 and h.restart_interval and mcu % h.restart_interval == 0:
            pred = [0, 0, 0, 0]
        c = comp_of[bb]
        out[i] = dc[i] - pred[c]
        pred[c] = int(dc[i])
    return out


@pytest.mark.parametrize("name", CASES)
def test_block_coefficients(sync_decoder, name):
    data = _load(name)
    sync_decoder.decode(data)
    blocks = sync_decoder.debug_fetch("blocks")
    entries = sync_decoder.debug_fetch("entries")
    st, coef = jdoracle.decode_coefs(data)
    assert st == 0
    coef = coef.copy()
    coef[:, 0] = dc_differences(data, coef[:, 0].astype(np.int64))
    nb = coef.shape[0]
    bad = []
    slots = entries.view(np.uint16)  # 16-bit AC-entry slots (jd_internal.hpp BlockInfo)
    for i in range(nb):
        start, cd = int(blocks[i, 0]), int(blocks[i, 1])
        cnt, dc = cd >> 25, ((cd & 0xFFFFFF) ^ 0x800000) - 0x800000  # 7-bit slot count, 24-bit DC
        got = np.zeros(64, np.int32)
        got[0] = dc
        k = start
        while k < start + cnt:
            h = int(slots[k])
            v = _s16(h) >> 6
            if (h & 0xFFC0) == 0x8000:  # escape: the value in the next slot
                k += 1
                v = _s16(int(slots[k]))
            got[h & 63] = v
            k += 1
        if not np.array_equal(got, coef[i]):
            bad.append(i)
    assert not bad, f"{len(bad)} of {nb} blocks differ, first {bad[:10]}"
