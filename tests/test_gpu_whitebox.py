"""White-box checks of the self-synchronising decode (GPU): intermediate arrays of the last batch
(jd_debug_fetch) against an independent sequential bit-level trace (tools/jd_trace.py).

  seg_cstart/seg_cend  -> un-stuffed interval lengths
  sub_entry            -> true entry state of every subsequence + block / DC prefix sums
  blocks               -> per-block AC-entry counts and DC values vs the oracle's coefficients
"""
import os
import sys

import numpy as np
import pytest

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
def test_intervals_and_entry_states(sync_decoder, name):
    data = _load(name)
    try:
        sync_decoder.decode(data)
    except Exception:
        pass  # inspect the intermediate state even when the decode reports an error
    tr = jd_trace.trace(data, jd_trace.SUB_BITS)
    cs = sync_decoder.debug_fetch("seg_cstart")
    ce = sync_decoder.debug_fetch("seg_cend")
    ssb = sync_decoder.debug_fetch("seg_sub_base")
    nsub = sync_decoder.debug_fetch("seg_nsub")
    ent = sync_decoder.debug_fetch("sub_entry")
    errs = []
    for s, seg in enumerate(tr):
        if (int(ce[s]) - int(cs[s])) * 8 != seg["bits"]:
            errs.append(f"seg {s}: bits gpu {(int(ce[s]) - int(cs[s])) * 8} want {seg['bits']}")
            continue
        if int(nsub[s]) != seg["nsub"]:
            errs.append(f"seg {s}: nsub gpu {nsub[s]} want {seg['nsub']}")
            continue
        blk = 0
        dc = [0, 0, 0]
        for j in range(seg["nsub"]):
            e = ent[int(ssb[s]) + j]
            p, sk = int(e[0]) & 0xFFFFFFFF, int(e[1]) & 0xFFFFFFFF
            got = (p, sk >> 16, (sk >> 8) & 0xFF, sk & 0xFF)
            want = seg["entry"][j]
            if got != tuple(want):
                errs.append(f"seg {s} sub {j}: entry gpu {got} want {want}")
            if int(e[2]) != blk or [int(x) for x in e[4:7]] != dc:
                errs.append(f"seg {s} sub {j}: blk/pred gpu {int(e[2])} {list(e[4:7])} want {blk} {dc}")
            c = seg["counts"][j]
            blk += c[0]
            dc = [dc[0] + c[2], dc[1] + c[3], dc[2] + c[4]]
        if len(errs) > 20:
            break
    assert not errs, "\n".join(errs[:20])


def _s16(x):
    return ((x + 0x8000) & 0xFFFF) - 0x8000


@pytest.mark.parametrize("name", CASES)
def test_block_coefficients(sync_decoder, name):
    data = _load(name)
    sync_decoder.decode(data)
    blocks = sync_decoder.debug_fetch("blocks")
    entries = sync_decoder.debug_fetch("entries")
    st, coef = jdoracle.decode_coefs(data)
    assert st == 0
    nb = coef.shape[0]
    bad = []
    for i in range(nb):
        start, cd = int(blocks[i, 0]), int(blocks[i, 1])
        cnt, dc = cd >> 16, _s16(cd & 0xFFFF)
        got = np.zeros(64, np.int32)
        got[0] = dc
        for e in entries[start:start + cnt]:
            got[int(e) & 63] = _s16((int(e) >> 16) & 0xFFFF)
        if not np.array_equal(got, coef[i]):
            bad.append(i)
    assert not bad, f"{len(bad)} of {nb} blocks differ, first {bad[:10]}"
