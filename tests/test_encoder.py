"""CPU tests of the in-repo baseline encoder (tools/jdenc.c) that makes the
bench and test inputs.  It is input tooling, not the decode path: these tests check that its files
are valid baseline JPEGs with the standard tables, that every decoder we trust reads them, and
that its output is deterministic."""
import hashlib
import io
import os
import sys
import tempfile

import numpy as np
import pytest

import jdoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import jd_synth  # noqa: E402
import jdenc  # noqa: E402


def segments(data: bytes, marker: int):
    out, i = [], 2
    while i < len(data):
        mk, ln = data[i + 1], data[i + 2] << 8 | data[i + 3]
        if mk == marker:
            out.append(data[i + 4:i + 2 + ln])
        if mk == 0xDA:
            break
        i += 2 + ln
    return out


@pytest.mark.parametrize("ss", ["4:4:4", "4:2:2", "4:2:0", "4:4:0"])
@pytest.mark.parametrize("rows", [0, 1])
def test_roundtrip_through_oracle(ss, rows):
    px = jd_synth.synth_pixels(203, 91, 7)
    data = jdenc.encode(px, 85, ss, restart_rows=rows)
    st, rgb = jdoracle.decode(data)
    assert st == 0
    err = np.abs(rgb.astype(int) - px.astype(int))
    assert err.mean() < 6.0 and err.max() < 80, (err.mean(), err.max())


def test_restart_intervals_do_not_change_pixels():
    px = jd_synth.synth_pixels(160, 120, 3)
    base = jdoracle.decode(jdenc.encode(px, 90, "4:2:0"))[1]
    for kw in ({"restart_rows": 1}, {"restart_blocks": 1}, {"restart_blocks": 7}):
        st, rgb = jdoracle.decode(jdenc.encode(px, 90, "4:2:0", **kw))
        assert st == 0 and np.array_equal(rgb, base), kw


def test_grayscale():
    px = jd_synth.synth_pixels(77, 50, 9, gray=True)
    st, rgb = jdoracle.decode(jdenc.encode(px, 80))
    assert st == 0 and np.abs(rgb[..., 0].astype(int) - px.astype(int)).mean() < 4


def test_deterministic_digest():
    """A pure function of pixels and parameters (integer colour, -ffp-contract=off AAN DCT)."""
    px = jd_synth.synth_pixels(64, 48, 0)
    a = jdenc.encode(px, 90, "4:2:0", restart_rows=1)
    assert a == jdenc.encode(px, 90, "4:2:0", restart_rows=1)
    assert hashlib.sha256(a).hexdigest()[:16] == "a931b32775637ee9"


def test_standard_tables_match_pillow():
    pytest.importorskip("PIL")
    px = jd_synth.synth_pixels(96, 64, 1)
    ours = jdenc.encode(px, 75, "4:2:0")
    pil = jd_synth.encode(px, 75, "4:2:0", encoder="pillow")
    assert sorted(segments(ours, 0xC4)) == sorted(segments(pil, 0xC4))  # Annex K.3 Huffman tables
    assert segments(ours, 0xDB) == segments(pil, 0xDB)                  # IJG-scaled Annex K.1 tables


def test_pillow_reads_our_files():
    PIL = pytest.importorskip("PIL.Image")
    px = jd_synth.synth_pixels(250, 130, 11)
    for ss in ("4:4:4", "4:2:2", "4:2:0"):
        got = np.asarray(PIL.open(io.BytesIO(jdenc.encode(px, 90, ss, restart_rows=2))).convert("RGB"))
        assert np.abs(got.astype(int) - px.astype(int)).mean() < 5, ss


@pytest.mark.skipif(not jdoracle.ref_available(), reason="oracle/_ref/decoder not built")
def test_reference_decoder_reads_our_444_files():
    """4:4:4 without DRI is the reference's supported subset: its own decoder equals the oracle."""
    with tempfile.TemporaryDirectory() as td:
        for i, (w, h, q) in enumerate([(64, 64, 90), (123, 45, 50), (200, 160, 100)]):
            data = jdenc.encode(jd_synth.synth_pixels(w, h, 50 + i), q, "4:4:4")
            p = os.path.join(td, f"e{i}.jpg")
            with open(p, "wb") as f:
                f.write(data)
            ref = jdoracle.ref_decode(p, td)
            st, rgb = jdoracle.decode(data)
            assert st == 0 and np.array_equal(ref, rgb)


def test_rejects_bad_arguments():
    with pytest.raises(ValueError):
        jdenc.encode(np.zeros((0, 8, 3), np.uint8))
