"""GPU parity tests: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bar: bit-exact RGB (integer/byte work).  Oracle = oracle/liboracle.so, pinned to the reference by
tests/test_oracle.py; golden digests from tests/golden/make_golden.py.
"""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

import jdamd
import jdoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import jd_synth  # noqa: E402

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint8).tobytes()).hexdigest()


def test_golden_single(decoder, golden):
    bad = []
    for e in golden:
        if e["status"] != 0:
            with pytest.raises(jdamd.JDError) as ei:
                decoder.decode(e["data"])
            assert ei.value.status == e["status"], e["file"]
            continue
        out = decoder.decode(e["data"])
        if sha(out) != e["sha256"]:
            st, ref = jdoracle.decode(e["data"])
            diff = np.abs(out.astype(int) - ref.astype(int))
            bad.append((e["file"], int(diff.max()), int((diff > 0).sum())))
    assert not bad, bad


def test_golden_batch(decoder, golden):
    """All fixtures in one batch: mixed sizes, sampling factors, table sets, RST / no RST."""
    outs, status = decoder.decode_batch([e["data"] for e in golden])
    for e, o, s in zip(golden, outs, status):
        assert s == e["status"], e["file"]
        if s == 0:
            assert sha(o) == e["sha256"], e["file"]


def test_device_resident_batch(decoder, golden):
    """Inputs already in HBM, outputs left in HBM (the bench path)."""
    ok = [e for e in golden if e["status"] == 0]
    hosts = [np.frombuffer(e["data"], np.uint8).copy() for e in ok]
    offs, total = [], 0
    for h in hosts:
        offs.append(total)
        total += (h.nbytes + 255) // 256 * 256
    din = decoder.alloc(total)
    for h, o in zip(hosts, offs):
        din.upload(h, o)
    sizes = [e["width"] * e["height"] * 3 for e in ok]
    ooffs, ototal = [], 0
    for s in sizes:
        ooffs.append(ototal)
        ototal += (s + 255) // 256 * 256
    dout = decoder.alloc(ototal)
    status = decoder.decode_batch_device(hosts, [din.ptr + o for o in offs], [dout.ptr + o for o in ooffs])
    assert all(s == 0 for s in status)
    for e, o, s in zip(ok, ooffs, sizes):
        img = dout.download(np.empty(s, np.uint8), o)
        assert sha(img) == e["sha256"], e["file"]


def test_pipelined_batches(decoder, golden):
    """jd_decode_batch_async: three device-resident batches launched back to back (each call
    collects the one before), then jd_decode_wait; every result and pixel as the blocking call."""
    ok = [e for e in golden if e["status"] == 0]
    groups = [ok[0::3], ok[1::3], ok[2::3]]
    bufs, batches = [], []
    for g in groups:
        hosts = [np.frombuffer(e["data"], np.uint8).copy() for e in g]
        offs, total = [], 0
        for h in hosts:
            offs.append(total)
            total += (h.nbytes + 255) // 256 * 256
        din = decoder.alloc(total)
        for h, o in zip(hosts, offs):
            din.upload(h, o)
        sizes = [e["width"] * e["height"] * 3 for e in g]
        ooffs, ototal = [], 0
        for sz in sizes:
            ooffs.append(ototal)
            ototal += (sz + 255) // 256 * 256
        dout = decoder.alloc(ototal)
        bufs.append((din, dout, ooffs, sizes, hosts))
        batches.append(decoder.make_batch(hosts, [din.ptr + o for o in offs], [dout.ptr + o for o in ooffs]))
    for bt in batches:
        decoder.decode_prepared(bt, pipelined=True)
    decoder.wait()
    for g, bt, (din, dout, ooffs, sizes, hosts) in zip(groups, batches, bufs):
        assert [r.status for r in bt[1]] == [0] * len(g)
        assert [(r.width, r.height) for r in bt[1]] == [(e["width"], e["height"]) for e in g]
        for e, o, sz in zip(g, ooffs, sizes):
            assert sha(dout.download(np.empty(sz, np.uint8), o)) == e["sha256"], e["file"]


@pytest.mark.parametrize("w,h,ss,rows,blocks,q", [
    (1920, 1080, "4:2:0", 1, 0, 90),   # BASELINE config 2 shape
    (1920, 1080, "4:2:0", 0, 0, 90),   # no DRI: single segment
    (1920, 1080, "4:4:4", 0, 0, 90),
    (1280, 720, "4:2:2", 0, 7, 75),
    (3840, 2160, "4:2:0", 1, 0, 90),   # BASELINE config 3 shape
    (1920, 1080, "4:4:0", 1, 0, 90),   # vertically subsampled chroma only: row pairs, per-pixel terms
    (333, 217, "4:4:0", 0, 0, 50),
    (333, 217, "4:2:2", 0, 3, 50),
])
def test_full_size_vs_oracle(decoder, w, h, ss, rows, blocks, q):
    data = jd_synth.encode(jd_synth.synth_pixels(w, h, 42), q, ss, rows, blocks)
    st, ref = jdoracle.decode(data)
    assert st == 0
    out = decoder.decode(data)
    assert np.array_equal(out, ref)


def test_c1_exact_image_vs_oracle(decoder):
    """BASELINE config 1 exactly as bench.py --config c1 builds it: 512 x 512 4:4:4 q90, no DRI,
    seed 0."""
    import bench

    W, H, ss, rows, _, _ = bench.CONFIGS["c1"]
    (job,) = jd_synth.make_jobs([0], W, H, 90, ss, rows, 0)
    (data,) = jd_synth.make_images([job], workers=1)
    assert data == jd_synth.encode(jd_synth.synth_pixels(512, 512, 0), 90, "4:4:4")
    st, ref = jdoracle.decode(data)
    assert st == 0
    assert np.array_equal(decoder.decode(data), ref)


@pytest.mark.parametrize("size", [200, 1000, 2000])
def test_ref444_sizes_vs_oracle(decoder, size):
    """The reference's own benchmark format (4:4:4 q95, data_preprocessing/image_converter.py:6,18)
    at its latency-benchmark sizes (cuda-decoder/benchmark/benchmark.cu:87), as bench.py
    --config ref444 builds them."""
    import bench

    (data,) = jd_synth.make_images(bench.ref444_jobs([bench.REF_SIZES.index(size)], 95), workers=1)
    assert jdamd.parse(data).width == size
    st, ref = jdoracle.decode(data)
    assert st == 0
    assert np.array_equal(decoder.decode(data), ref)


def test_rst_invariance_full_size(decoder):
    px = jd_synth.synth_pixels(1920, 1080, 7)
    a = decoder.decode(jd_synth.encode(px, 90, "4:2:0"))
    b = decoder.decode(jd_synth.encode(px, 90, "4:2:0", restart_rows=1))
    c = decoder.decode(jd_synth.encode(px, 90, "4:2:0", restart_blocks=5))
    assert np.array_equal(a, b) and np.array_equal(a, c)


def test_idct_kat(decoder):
    rng = np.random.default_rng(1)
    blocks = []
    # DC-only sweep across the whole dequantised DC range
    dc = np.zeros((4096, 64), np.int32)
    dc[:, 0] = np.arange(-32768, 32768, 16)[:4096]
    blocks.append(dc)
    # sparse realistic blocks and dense random blocks
    sp = np.zeros((20000, 64), np.int32)
    for k in range(20000):
        n = rng.integers(0, 12)
        idx = rng.integers(0, 64, n)
        sp[k, idx] = rng.integers(-1024, 1024, n) * rng.integers(1, 40, n)
    blocks.append(sp)
    blocks.append(rng.integers(-2048, 2048, (20000, 64), dtype=np.int32))
    # the int16 fast form's corners (v_dot2_i32_i16 row pass: every input within int16)
    corner = np.where(rng.random((4096, 64)) < 0.5, 32767, -32768).astype(np.int32)
    corner[2048:][rng.random((2048, 64)) < 0.7] = 0
    blocks.append(corner)
    a = np.concatenate(blocks)
    got = decoder.test_idct(a)
    want = jdoracle.idct(a)
    assert np.array_equal(got, want)


def test_idct_both_forms_over_int32(decoder):
    """The decode path's forms against the oracle, at and beyond the fast form's range: the fast form
    (int16 dot2 row pass + 24-bit column pass, taken when every input fits int16) and the exact
    form (the reference's formulas and DC-only shortcuts, any int32 input; the oracle wraps like the
    GPU, -fwrapv)."""
    rng = np.random.default_rng(2)
    n = 40000
    edge = rng.integers(-65536, 65537, (n, 64)).astype(np.int32)          # fast form, dense
    edge[: n // 2][rng.random((n // 2, 64)) < 0.85] = 0
    edge[:64] = np.where(rng.random((64, 64)) < 0.5, 65536, -65536)      # the range's corners
    wide = rng.integers(-2**31, 2**31, (n, 64), dtype=np.int64).astype(np.int32)
    wide[: n // 2][rng.random((n // 2, 64)) < 0.9] = 0                    # exact form, shortcuts
    dc = np.zeros((4096, 64), np.int32)
    dc[:, 0] = rng.integers(-2**31, 2**31, 4096, dtype=np.int64)          # DC-only rows and columns
    wrap = np.zeros((64, 64), np.int32)
    wrap[:, 14] = (np.arange(64) - 32) * (1 << 21)                         # block[4] << 11 wraps to 0
    wrap[:, 0] = rng.integers(-5000, 5000, 64)
    a = np.concatenate([edge, wide, dc, wrap])
    want = jdoracle.idct(a)
    assert np.array_equal(decoder.test_idct(a), want)
    assert np.array_equal(decoder.test_idct(a, exact_only=True), want)


def test_color_exhaustive(decoder):
    """All 2^27 (Y, Cb, Cr) in [-256, 255]^3 against utils/color.cpp's double/float formula
    (restated in numpy, float32/float64 exactly as the reference rounds)."""
    cb, cr = np.meshgrid(np.arange(-256, 256, dtype=np.int32), np.arange(-256, 256, dtype=np.int32),
                         indexing="ij")
    cb = cb.ravel()
    cr = cr.ravel()
    bad = 0
    for y0 in range(-256, 256, 16):
        ys = np.repeat(np.arange(y0, y0 + 16, dtype=np.int32), cb.size)
        cbs = np.tile(cb, 16)
        crs = np.tile(cr, 16)
        ycc = np.stack([ys, cbs, crs], -1)
        got = decoder.test_color(ycc)
        yd = ys.astype(np.float64)
        r = (crs * (2 - 2 * 0.299) + yd).astype(np.float32)
        b = (cbs * (2 - 2 * 0.114) + yd).astype(np.float32)
        g = ((yd - 0.114 * b.astype(np.float64) - 0.299 * r.astype(np.float64)) / 0.587).astype(np.float32)
        want = np.stack([np.clip((r + np.float32(128)).astype(np.int32), 0, 255),
                         np.clip((g + np.float32(128)).astype(np.int32), 0, 255),
                         np.clip((b + np.float32(128)).astype(np.int32), 0, 255)], -1).astype(np.uint8)
        bad += int((got != want).any(-1).sum())
    assert bad == 0


def test_corrupt_inputs_do_not_poison_batch(decoder, golden):
    good = next(e for e in golden if e["file"].endswith("2_400x400.jpg"))
    d = good["data"]
    trunc = d[: len(d) // 2]                                # ECS cut short -> overrun
    garbage = d[:700] + bytes(np.random.default_rng(3).integers(0, 256, 4000, dtype=np.uint8)) + b"\xff\xd9"
    noheader = b"\xff\xd8\xff\xd9"
    outs, status = decoder.decode_batch([d, trunc, garbage, noheader, d])
    assert status[0] == 0 and status[4] == 0
    assert sha(outs[0]) == good["sha256"] and sha(outs[4]) == good["sha256"]
    assert status[1] != 0 and status[3] != 0
    for data, s in ((trunc, status[1]), (garbage, status[2])):
        ost, _ = jdoracle.decode(data)
        assert (ost == 0) == (s == 0)


def test_cli_array_matches_reference_format(tmp_path, golden):
    exe = os.path.join(ROOT, "gpu-jpeg-decoder_amd", "decoder")
    img = os.path.join(ROOT, "tests", "golden", "ref", "3_120x120.jpg")
    subprocess.run([exe, img, str(tmp_path)], check=True)
    got = open(tmp_path / "3_120x120.array", "rb").read()
    want = open(os.path.join(ROOT, "tests", "golden", "ref", "3_120x120.array"), "rb").read()
    assert got == want


def _dc_ramp_jpeg(nblocks: int, dri: int) -> bytes:
    """A grayscale 8 x 8*nblocks baseline JPEG whose every block has DC difference +2047 and no AC
    (one-symbol DC and AC tables, unit quantisation): the DC leaves int16 after 17 blocks unless
    restart intervals of `dri` MCUs reset the predictor first."""
    bits = []

    def put(v, n):
        bits.extend((v >> (n - 1 - k)) & 1 for k in range(n))

    ecs = bytearray()

    def flush():
        while len(bits) % 8:
            bits.append(1)
        for i in range(0, len(bits), 8):
            byte = int("".join(map(str, bits[i:i + 8])), 2)
            ecs.append(byte)
            if byte == 0xFF:
                ecs.append(0)
        bits.clear()

    for k in range(nblocks):
        if dri and k and k % dri == 0:
            flush()
            ecs += bytes([0xFF, 0xD0 + (k // dri - 1) % 8])
        put(0, 1)          # DC code '0' -> size 11
        put(2047, 11)      # +2047
        put(0, 1)          # AC code '0' -> EOB
    flush()
    seg = lambda m, body: bytes([0xFF, m]) + (len(body) + 2).to_bytes(2, "big") + body
    out = b"\xff\xd8" + seg(0xDB, b"\x00" + bytes([1] * 64))
    out += seg(0xC0, b"\x08" + (8).to_bytes(2, "big") + (8 * nblocks).to_bytes(2, "big") + b"\x01\x01\x11\x00")
    out += seg(0xC4, b"\x00" + bytes([1] + [0] * 15) + b"\x0b")  # DC table 0: one 1-bit code, symbol 11
    out += seg(0xC4, b"\x10" + bytes([1] + [0] * 15) + b"\x00")  # AC table 0: one 1-bit code, EOB
    if dri:
        out += seg(0xDD, dri.to_bytes(2, "big"))
    out += seg(0xDA, b"\x01\x01\x00\x00\x3f\x00") + bytes(ecs) + b"\xff\xd9"
    return out


@pytest.mark.parametrize("nblocks,dri", [(20, 0), (16, 0), (20, 8), (150, 5), (150, 16), (150, 17)])
def test_dc_prediction_beyond_int16_and_resets(decoder, nblocks, dri):
    """DC predictor values beyond int16 decode with the reference's int arithmetic (its
    predictor and dequantisation are int, parser.cpp:106-111), and the predictor restarts at
    every restart interval, including intervals that start inside an IDCT tile."""
    data = _dc_ramp_jpeg(nblocks, dri)
    ost, ref = jdoracle.decode(data)
    assert ost == 0
    assert np.array_equal(decoder.decode(data), ref)


def _cut_interval(jpeg, seg, nmcu):
    """seg cut right after its first nmcu MCUs (tools/jd_trace.py decodes the symbols), the last
    byte padded with 1-bits (and a stuffed zero after an FF); seg itself when it ends earlier."""
    import jd_trace

    t = jd_trace.parse(jpeg)
    pattern, _ = jd_trace._layout(t)
    val, total = int.from_bytes(seg, "big"), len(seg) * 8
    p, k = 0, 0
    for _ in range(nmcu):
        for bi in range(len(pattern)):
            while True:
                r = jd_trace._symbol(t, pattern, val, total, p, bi, k)
                if r is None or p + r[0] > total:
                    return seg
                p += r[0]
                k, fin, _ = jd_trace._step(k, r[1])
                if fin:
                    break
    nb = (p + 7) // 8
    out = bytearray(seg[:nb])
    if p % 8:
        out[-1] |= (1 << (8 - p % 8)) - 1
    if out and out[-1] == 0xFF:
        out.append(0)
    return bytes(out)


# Bit flips in the entropy data of images with restart intervals that leave whole bytes between an
# interval's last MCU and its RSTn (found by tools/parity_sweep.py): the oracle's restart finds no
# marker at the byte-aligned position (status CORRUPT); the interval's last piece must not accept an
# error after its last counted MCU (jd_kernels.hip piece_take).
@pytest.mark.parametrize("params", [
    {"seed": 11004573, "w": 133, "h": 12, "ss": "4:4:4", "q": 50, "rows": 0, "blocks": 2, "flips": 1},
    {"seed": 11002742, "w": 119, "h": 34, "ss": "4:2:2", "q": 90, "rows": 0, "blocks": 2, "flips": 3},
    {"seed": 11005497, "w": 36, "h": 238, "ss": "4:2:0", "q": 95, "rows": 2, "blocks": 0, "flips": 3},
    {"seed": 11006876, "w": 35, "h": 157, "ss": "4:4:0", "q": 90, "rows": 0, "blocks": 10, "flips": 3},
    {"seed": 11009965, "w": 28, "h": 100, "ss": "4:4:0", "q": 100, "rows": 0, "blocks": 2, "flips": 1},
    {"seed": 11000078, "w": 22, "h": 250, "ss": "4:4:0", "q": 90, "rows": 0, "blocks": 5, "flips": 2},
])
def test_bytes_left_before_rst_is_corrupt(decoder, params):
    import parity_sweep

    data = parity_sweep.make_image(params)
    st, ref = jdoracle.decode(data)
    assert st == jdamd.JD_ERR_CORRUPT
    out, status = decoder.decode_batch([data])
    assert status == [st]
    clean = parity_sweep.make_image(dict(params, flips=0))  # the unflipped image decodes
    st0, ref0 = jdoracle.decode(clean)
    out0, status0 = decoder.decode_batch([clean])
    assert st0 == 0 and status0 == [0] and np.array_equal(out0[0], ref0)


# Grayscale images whose last MCU (one block: DC "00" + EOB "1010", 6 bits) lies inside the last
# byte of the entropy data or of a restart interval (found by tools/parity_sweep.py): the walk must
# decode it instead of taking the byte for padding (jd_kernels.hip walk_piece, mbeg).
@pytest.mark.parametrize("params", [
    {"seed": 12011017, "w": 73, "h": 193, "ss": "gray", "q": 75, "rows": 0, "blocks": 0, "flips": 0},
    {"seed": 12020118, "w": 385, "h": 225, "ss": "gray", "q": 50, "rows": 3, "blocks": 0, "flips": 1},
    {"seed": 12072936, "w": 281, "h": 83, "ss": "gray", "q": 35, "rows": 3, "blocks": 0, "flips": 0},
    {"seed": 12083853, "w": 274, "h": 106, "ss": "gray", "q": 20, "rows": 0, "blocks": 0, "flips": 0},
])
def test_mcu_inside_the_last_byte(decoder, params):
    import parity_sweep

    data = parity_sweep.make_image(params)
    st, ref = jdoracle.decode(data)
    assert st == 0
    out, status = decoder.decode_batch([data])
    assert status == [0] and np.array_equal(out[0], ref)


# Corrupt streams found by tools/parity_sweep.py, through every piece geometry:
#  - 16033655: a flip leaves an interval's last MCU ending in its last byte, and the leftover bits
#    complete one more (short, grayscale) MCU, which the oracle never reads (it decodes the
#    interval's count, then finds RSTn): status 0 (jd_kernels.hip piece_take, the tail count);
#  - 16038946: on 1024-bit pieces, a piece re-walked from its true start joins its speculative
#    walk, which had hit a garbage code before synchronising and a real one after the joined
#    checkpoint: the real one must count (status corrupt; redo_piece, per-checkpoint errors);
#  - 16045274: a flip turns the chroma DC table's first symbol into 16 (DC size 16, decoded by the
#    reference and the oracle: jd_internal.hpp lut_entry);
#  - 64114030 (round 6, a flat-area image): a flip turns the byte before a stuffed FF 00 into FF,
#    and the run FF FF 00 is a marker at its first FF, where the oracle's reader stops (status
#    corrupt: the interval overruns it and no RSTn follows; jd_kernels.hip k_scan).
@pytest.mark.parametrize("params", [
    {"seed": 16033655, "w": 74, "h": 179, "ss": "gray", "q": 35, "rows": 0, "blocks": 2, "flips": 1},
    {"seed": 16038946, "w": 366, "h": 10, "ss": "gray", "q": 100, "rows": 0, "blocks": 0, "flips": 1},
    {"seed": 16045274, "w": 11, "h": 68, "ss": "4:4:4", "q": 90, "rows": 0, "blocks": 0, "flips": 3},
    {"seed": 64114030, "w": 318, "h": 183, "ss": "gray", "q": 75, "rows": 0, "blocks": 9, "flips": 1, "flat": True},
])
def test_sweep_cases_every_path(params):
    import parity_sweep

    data = parity_sweep.make_image(params)
    st, ref = jdoracle.decode(data)
    for path in ("auto", "sync", "lanes", "full"):
        dec = jdamd.Decoder(0, path=path)
        try:
            out, status = dec.decode_batch([data])
        finally:
            dec.close()
        assert status == [st], path
        if st == 0:
            assert np.array_equal(out[0], ref), path


def _dht_values_offset(data, tc, th):
    """Byte offset of the symbol values of DHT table (tc, th) in a JPEG."""
    i = 2
    while i + 4 <= len(data):
        m, L = data[i + 1], (data[i + 2] << 8) | data[i + 3]
        if m == 0xC4:
            q = i + 4
            while q < i + 2 + L:
                tot = sum(data[q + 1:q + 17])
                if (data[q] >> 4, data[q] & 15) == (tc, th):
                    return q + 17
                q += 17 + tot
        if m == 0xDA:
            break
        i += 2 + L
    raise ValueError("no such table")


@pytest.mark.parametrize("w,h,ss,q,rst", [(8, 8, "gray", 90, 0), (16, 16, "4:2:0", 50, 0), (24, 16, "4:4:4", 95, 0),
                                          (64, 48, "4:2:2", 75, 0), (32, 32, "4:2:0", 90, 1), (40, 16, "4:4:4", 75, 2),
                                          (256, 256, "gray", 90, 0), (128, 128, "4:2:0", 75, 0),
                                          (64, 32, "gray", 75, "dc16"), (48, 32, "4:2:0", 50, "dc16"),
                                          (40, 16, "4:4:4", 90, "dc16r2")])
def test_random_entropy_data_vs_oracle(decoder, w, h, ss, q, rst):
    """Random entropy-coded bytes behind valid headers: every symbol the tables allow, in any
    order (runs past index 63, ZRL, codes longer than the LUT, magnitudes whose dequantised values
    need the exact IDCT form, paired and unpaired lookups).  Status (decoded or not) and pixels
    must match the oracle, image by image, in one batch.  rst > 0: restart intervals of rst MCUs,
    each its own random bytes followed by the expected RSTn (trailing bytes before an RSTn are
    corrupt, trailing bytes before EOI are not).
    "dc16[rN]": luma DC symbols rewritten to DC sizes 16, 12, 15 and (the longest code) 17 (beyond
    baseline's 11: the reference reads up to 16 magnitude bits, parser.cpp:106-108, the oracle
    flags a size above 16, jdoracle.c decode_block; 16 gives differences of +-32768..65535,
    jd_kernels.hip block_rec's 17-bit DC), restart intervals of N MCUs with "rN"."""
    dcs = isinstance(rst, str)
    if dcs:
        rst = int(rst[5:]) if len(rst) > 4 else 0
    rng = np.random.default_rng(w * 10007 + h * 101 + q + rst + (7 if dcs else 0))
    hdr = jd_synth.encode(jd_synth.synth_pixels(w, h, 1, ss == "gray"), q, "4:4:4" if ss == "gray" else ss,
                          restart_blocks=rst)
    if dcs:  # the standard luma DC table: codes 00, 010, 011, ..., 111111110 for symbols 0 .. 11
        hdr = bytearray(hdr)
        o = _dht_values_offset(hdr, 0, 0)
        hdr[o:o + 3] = bytes([16, 12, 15])
        hdr[o + 11] = 17
        hdr = bytes(hdr)
    hd = jdamd.parse(hdr)
    head = hdr[:hd.ecs_offset]
    nseg = -(-hd.mcux * hd.mcuy // rst) if rst else 1
    files = []
    for i in range(96):
        segs = []
        for k in range(nseg):
            n = (w * h // 64) * 2 * int(rng.integers(8, 40)) // nseg  # about 16-80 bytes per block
            ecs = rng.integers(0, 256, max(n, 1), dtype=np.uint8)
            ecs[ecs == 0xFF] = 0xFE  # no markers inside an interval
            seg = ecs.tobytes()
            if k + 1 < nseg and i % 4:  # 3 of 4: cut the interval where its MCUs end, 1-padded
                seg = _cut_interval(hdr, seg, rst)
            segs.append(seg + (bytes([0xFF, 0xD0 + k % 8]) if k + 1 < nseg else b""))
        files.append(head + b"".join(segs) + b"\xff\xd9")
    outs, status = decoder.decode_batch(files)
    decoded = 0
    for i, data in enumerate(files):
        ost, ref = jdoracle.decode(data)
        assert (ost == 0) == (status[i] == 0), i
        if ost == 0:
            assert np.array_equal(outs[i], ref), i
            decoded += 1
    assert decoded > 0
