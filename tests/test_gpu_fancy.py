"""GPU parity of the fancy (triangular) chroma upsampling option, JD_FLAG_FANCY_UPSAMPLING.

Oracle: jdoracle.decode(fancy=True), the restatement of libjpeg's h2v1 / h2v2 / h1v2 filters on
the reference's samples (oracle/jdoracle.c fancy_sample).  That restatement is parity-unpinned by
the reference (which has no subsampled chroma); tests/test_oracle.py::test_fancy_close_to_pillow
anchors it to libjpeg-turbo within the reference's own IDCT/colour difference.  Bar: bit-exact.
"""
import os
import sys

import numpy as np
import pytest

import jdamd
import jdoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import jd_synth  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fancy_decoder():
    dec = jdamd.Decoder(0, timing=True, fancy=True)
    yield dec
    dec.close()


@pytest.mark.parametrize("w,h,ss,rows", [
    (1920, 1080, "4:2:0", 1), (333, 217, "4:2:0", 0), (333, 217, "4:2:2", 2), (333, 217, "4:4:0", 0),
    (129, 65, "4:4:4", 0), (17, 9, "4:2:0", 0), (1, 1, "4:2:0", 0), (2, 3, "4:2:0", 0), (9, 3, "4:2:2", 0),
    (3, 9, "4:4:0", 1), (16, 16, "4:2:0", 1), (250, 1, "4:2:2", 0),
    # k_colour_fancy's 128 x 16 bands: widths and heights just across band and window edges
    (257, 35, "4:2:0", 0), (130, 33, "4:2:2", 1), (300, 47, "4:4:0", 0), (383, 17, "4:2:0", 2), (128, 16, "4:2:0", 0),
])
def test_fancy_vs_oracle(fancy_decoder, w, h, ss, rows):
    data = jd_synth.encode(jd_synth.synth_pixels(w, h, 5), 90, ss, rows)
    st, ref = jdoracle.decode(data, fancy=True)
    assert st == 0
    assert np.array_equal(fancy_decoder.decode(data), ref)


def test_fancy_gray_and_batch(fancy_decoder):
    datas = [jd_synth.encode(jd_synth.synth_pixels(97, 45, 1, gray=True), 80)]
    datas += [jd_synth.encode(jd_synth.synth_pixels(200 + 3 * i, 120 - i, 10 + i), 85, ss, i % 2)
              for i, ss in enumerate(["4:2:0", "4:2:2", "4:4:4", "4:4:0", "4:2:0"])]
    outs, status = fancy_decoder.decode_batch(datas)
    for d, o, s in zip(datas, outs, status):
        st, ref = jdoracle.decode(d, fancy=True)
        assert s == 0 and st == 0 and np.array_equal(o, ref)


def test_fancy_timed_kernel(fancy_decoder):
    fancy_decoder.reset_stats()
    fancy_decoder.decode(jd_synth.encode(jd_synth.synth_pixels(640, 480, 3), 90, "4:2:0"))
    k = fancy_decoder.stats()["kernels"]
    assert k["k_colour_fancy"]["launches"] == 1 and k["k_colour_fancy"]["bytes"] > 0
