"""Re-walk paths of the fused Huffman pass (GPU), against the oracle.

With a short warm-up (JD_PIECE_OVERLAP_BITS) most speculative piece starts are wrong, so k_redo
re-walks them and k_chain_fix walks the intervals where a re-walked piece's predecessor was itself
re-walked.  With JD_SPARE_PIECES=0 no spare region is left: every re-walk writes over its own region
and cannot join the speculative walk (jd_kernels.hip redo_piece); with the default spare regions it
joins at a checkpoint and the piece's blocks come from two segments (k_gather).  The re-walks read
the Huffman tables from global memory (each table set's LUTs in BatchDev::set_luts); the grayscale
image adds a second table set.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import jd_synth  # noqa: E402
import jdamd  # noqa: E402
import jdoracle  # noqa: E402

pytestmark = pytest.mark.gpu

IMAGES = [  # (w, h, subsampling, restart_rows, quality)
    (1920, 1080, "4:2:0", 0, 90),
    (1920, 1080, "4:2:0", 1, 75),
    (1024, 768, "4:4:4", 0, 95),
    (1280, 720, "4:2:2", 2, 50),
    (333, 251, "4:2:0", 0, 90),
    (640, 480, "4:4:4", 0, 100),  # quality 100: AC values beyond +-511 take escaped 16-bit entry slots
    (1280, 720, "gray", 0, 85),   # a second table set (one component): k_redo / k_chain_fix read
                                  # their tables at a nonzero offset of BatchDev::set_luts
]


@pytest.fixture(scope="module")
def batch():
    datas = [jd_synth.encode(jd_synth.synth_pixels(w, h, 5 + i, ss == "gray"), q, "4:4:4" if ss == "gray" else ss, rr)
             for i, (w, h, ss, rr, q) in enumerate(IMAGES)]
    refs = []
    for d in datas:
        st, ref = jdoracle.decode(d)
        assert st == 0
        refs.append(ref)
    return datas, refs


@pytest.mark.parametrize("spare", ["0", "default"])
@pytest.mark.parametrize("overlap,path", [("256", "sync"), ("512", "full"), ("64", "auto")])
def test_rewalks_vs_oracle(monkeypatch, batch, spare, overlap, path):
    datas, refs = batch
    monkeypatch.setenv("JD_PIECE_OVERLAP_BITS", overlap)
    if spare != "default":
        monkeypatch.setenv("JD_SPARE_PIECES", spare)
    dec = jdamd.Decoder(0, path=path)
    try:
        outs, status = dec.decode_batch(datas)
        valid = dec.debug_fetch("sub_seg") != 0xFFFFFFFF  # padding slots hold stale scratch
        joins = (dec.debug_fetch("piece_join") & 0xFFFF)[valid]
    finally:
        dec.close()
    assert status == [0] * len(datas), status
    for i, (o, r) in enumerate(zip(outs, refs)):
        assert o.shape == r.shape and np.array_equal(o, r), f"image {i} differs ({IMAGES[i]})"
    if spare == "0":  # in place: a re-walk never joins
        assert not np.any(joins), "a re-walk joined without a spare region"
    else:  # the short warm-up makes re-walks common: some must have joined
        assert np.any(joins), "no re-walk joined its speculative walk"


def test_escaped_entries_vs_oracle():
    """Quality 100 on noisy pixels: many AC values need the two-slot escape (jd_internal.hpp)."""
    rng = np.random.default_rng(3)
    px = rng.integers(0, 256, (256, 384, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:256, 0:384]
    px[:128] = np.where(((xx + yy) & 1)[:128, :, None] == 1, 255, 0).astype(np.uint8)  # high AC values
    px[128:, :192] = np.where(((xx // 2) & 1)[128:, :192, None] == 1, 255, 0).astype(np.uint8)
    data = jd_synth.encode(px, 100, "4:4:4")
    st, ref = jdoracle.decode(data)
    assert st == 0
    dec = jdamd.Decoder(0)
    try:
        out = dec.decode(data)
        esc = (dec.debug_fetch("blocks")[:, 1] >> 24) & 1
    finally:
        dec.close()
    assert np.any(esc), "no block used an escaped entry"
    assert np.array_equal(out, ref)


@pytest.fixture(scope="module")
def dense_batch():
    """the densest streams the region bound allows.  Flat images are all DC-only
    blocks (Annex K tables: a 2-bit DC code plus a 2-bit chroma EOB, exactly the divisor-4 bound);
    re-tabled files (tools/jd_retable.py: 4-bit DC, 8-bit AC codes) sit at the divisor's maximum, 8."""
    import jd_retable

    datas = []
    for i, (w, h, ss, rr) in enumerate([(1920, 1080, "4:2:0", 0), (1280, 720, "4:4:4", 1), (777, 333, "4:2:2", 0),
                                        (640, 480, "4:2:0", 2), (1024, 768, "gray", 0)]):
        gray = ss == "gray"
        px = np.full((h, w) if gray else (h, w, 3), 37 + 40 * i, np.uint8)
        datas.append(jd_synth.encode(px, 90, "4:4:4" if gray else ss, rr))
    for i, (w, h, ss, rr) in enumerate([(1280, 720, "4:2:0", 1), (640, 480, "4:4:4", 0), (333, 251, "4:2:2", 0)]):
        datas.append(jd_retable.retable(jd_synth.encode(jd_synth.synth_pixels(w, h, 40 + i), 90, ss, rr)))
    refs = []
    for d in datas:
        st, ref = jdoracle.decode(d)
        assert st == 0
        refs.append(ref)
    return datas, refs


@pytest.mark.parametrize("path", ["auto", "sync", "lanes", "full"])
def test_dense_streams_without_spare_regions(monkeypatch, dense_batch, path):
    """Flat (DC-only) and long-code images on every piece geometry with JD_SPARE_PIECES=0 (re-walks
    over their own regions), with worst-case pools (tests/test_gpu_pools.py: the default optimistic
    ones): bit-exact, and the re-tabled images planned with region divisor 8."""
    datas, refs = dense_batch
    monkeypatch.setenv("JD_SPARE_PIECES", "0")
    monkeypatch.setenv("JD_WORST_CASE_POOLS", "1")
    dec = jdamd.Decoder(0, path=path)
    try:
        outs, status = dec.decode_batch(datas)
        assert status == [0] * len(datas)
        for i, (o, r) in enumerate(zip(outs, refs)):
            assert np.array_equal(o, r), i
        assert list(dec.debug_fetch("rw_div")[5:]) == [8, 8, 8]
        assert list(dec.debug_fetch("rw_div")[:5]) == [4, 4, 4, 4, 4]
    finally:
        dec.close()


@pytest.mark.parametrize("overlap,spare", [("1024", "default"), ("256", "default"), ("64", "0")])
def test_big_interval_rounds_vs_oracle(monkeypatch, overlap, spare):
    """One image without DRI in a batch of its own: a single interval of ~45 K 512-bit pieces, which
    k_chain leaves to k_chain_big (re-walk rounds, then the counts by prefix sums).  A short warm-up
    makes runs of consecutive failed starts; with a 64-bit warm-up and no spare regions (no joins)
    they are long, and each is re-walked by one lane in one round (there is no serial fallback)."""
    import bench

    (data,) = jd_synth.make_images(bench.ref444_jobs([bench.REF_SIZES.index(2000)], 95), workers=1)
    st, ref = jdoracle.decode(data)
    assert st == 0
    monkeypatch.setenv("JD_PIECE_OVERLAP_BITS", overlap)
    if spare != "default":
        monkeypatch.setenv("JD_SPARE_PIECES", spare)
    dec = jdamd.Decoder(0, timing=True)
    try:
        out = dec.decode(data)
        nsub = int((dec.debug_fetch("sub_seg") != 0xFFFFFFFF).sum())
        assert nsub > 4096  # one interval of thousands of pieces (kBigInterval = 256)
        assert np.array_equal(out, ref)
        s = dec.stats()
        assert s["redo_pieces"] > 0 and s["fix_early"] == 0  # (a valid image: no early stop)
    finally:
        dec.close()


def _decode_timed(dec, data, reps=3):
    """(pixels, best wall time in s) of `reps` blocking decodes after one untimed decode (pools)."""
    import time
    out = dec.decode(data)
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        out = dec.decode(data)
        best = min(best, time.perf_counter() - t0)
    return out, best


def test_big_interval_short_pieces_bounded(monkeypatch):
    """the geometry of round 5's silent latency run (r05ac, a variant build):
    256-bit pieces with a 768-bit warm-up on the 2 000 x 2 000 4:4:4 q95 image, ~90 K pieces in one
    interval.  Its cause: a 4:4:4 q95 MCU takes ~450 bits, more than a piece, and a piece in whose
    share no MCU begins walked one MCU anyway, so nearly every start after it disagreed and
    k_chain_big, after 32 rounds, left the interval to one lane.  Such a piece is now empty, and
    k_chain_big has no serial fallback: parity with the oracle, the rounds counted (jd_stats), and a
    wall bound."""
    import bench

    (data,) = jd_synth.make_images(bench.ref444_jobs([bench.REF_SIZES.index(2000)], 95), workers=1)
    st, ref = jdoracle.decode(data)
    assert st == 0
    monkeypatch.setenv("JD_MIN_PIECE_BITS", "256")
    monkeypatch.setenv("JD_PIECE_OVERLAP_BITS", "768")
    dec = jdamd.Decoder(0)
    try:
        dec.reset_stats()
        out, wall = _decode_timed(dec, data)
        nsub = int((dec.debug_fetch("sub_seg") != 0xFFFFFFFF).sum())
        s = dec.stats()
        per = {k: s[k] / s["batches"] for k in ("redo_pieces", "fix_intervals", "fix_rounds", "fix_rewalks", "fix_early")}
        print(f"\n2000^2 4:4:4 q95, 256-bit pieces, 768-bit warm-up: {nsub} pieces, {wall * 1e3:.2f} ms, per decode {per}")
        assert nsub > 80_000
        assert np.array_equal(out, ref)
        assert per["fix_early"] == 0
        assert per["fix_rounds"] <= 32
        assert wall < 0.020
    finally:
        dec.close()


@pytest.mark.parametrize("damage", ["ones", "truncate"])
def test_big_interval_corrupt_bounded(monkeypatch, damage):
    """a corrupt image without DRI in a batch of its own (one interval of tens of
    thousands of short pieces).  Past the damage no start agrees with anything, so k_chain_big's
    rounds would chase garbage; they stop at the first right piece with an error instead.  The
    status must be the oracle's, and the decode must stay within a wall bound."""
    import bench

    (data,) = jd_synth.make_images(bench.ref444_jobs([bench.REF_SIZES.index(2000)], 95), workers=1)
    h = jdamd.parse(data)
    b = bytearray(data)
    if damage == "ones":  # 256 one-bits (stuffed FF bytes) mid-scan: no Huffman code is all ones
        m = h.ecs_offset + (len(b) - h.ecs_offset) // 2
        b[m:m + 64] = b"\xff\x00" * 32
    else:  # the scan cut at two thirds, EOI appended
        b = b[: h.ecs_offset + 2 * (len(b) - h.ecs_offset) // 3] + b"\xff\xd9"
    data = bytes(b)
    st, _ = jdoracle.decode(data)
    monkeypatch.setenv("JD_PIECE_OVERLAP_BITS", "256")  # many failed starts
    dec = jdamd.Decoder(0)
    try:
        import time
        _, status = dec.decode_batch([data])  # (pools)
        assert status == [st] and st == jdamd.JD_ERR_CORRUPT
        dec.reset_stats()
        t0 = time.perf_counter()
        _, status = dec.decode_batch([data])
        wall = time.perf_counter() - t0
        s = dec.stats()
        print(f"\ncorrupt ({damage}): {wall * 1e3:.2f} ms, rounds {s['fix_rounds']:.0f}, early stops {s['fix_early']:.0f}, "
              f"re-walks {s['fix_rewalks']:.0f} + {s['redo_pieces']:.0f}")
        assert status == [st]
        assert wall < 0.050
    finally:
        dec.close()


@pytest.mark.parametrize("overlap", ["default", "256"])
def test_big_intervals_with_dri_vs_oracle(monkeypatch, overlap):
    """Several big intervals in one image (2000 x 2000 4:4:4 q95, an RSTn every 50 MCU rows: five
    intervals of ~14 K 512-bit pieces): k_chain_big's rounds and counts on intervals that end at an
    RSTn (every piece counts, the last one takes the rest) as well as the final one (bytes after its
    last MCU ignored), with re-walk rounds forced by a short warm-up."""
    px = jd_synth.synth_pixels(2000, 2000, 4242)
    data = jd_synth.encode(px, 95, "4:4:4", restart_rows=50)
    h = jdamd.parse(data)
    assert h.restart_interval and -(-h.mcux * h.mcuy // h.restart_interval) == 5
    st, ref = jdoracle.decode(data)
    assert st == 0
    if overlap != "default":
        monkeypatch.setenv("JD_PIECE_OVERLAP_BITS", overlap)
    dec = jdamd.Decoder(0)
    try:
        out = dec.decode(data)
        nsub = int((dec.debug_fetch("sub_seg") != 0xFFFFFFFF).sum())
        assert nsub > 5 * 1024  # intervals of thousands of pieces each (kBigInterval = 256)
        assert np.array_equal(out, ref)
    finally:
        dec.close()
