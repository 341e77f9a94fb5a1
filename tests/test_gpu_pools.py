"""Optimistic device pools and their retry (GPU), against the oracle.

By default a batch's piece regions are sized for 8 walk bits per 32-bit word plus the image's
largest MCU (jd_plan.hpp region_sizing), and its scan break lists for the batch's most restart
intervals + 16 (jd_runtime.cpp build_plan).  A denser stream fills a region: the walk stops at the
region guard and flags its image kStOverflow (jd_kernels.hip walk_piece); a chunk that held more
breaks before the ECS end than its slots flags it too (k_index).  The host then decodes the image
again with worst-case pools before reporting its batch (jd_runtime.cpp run_retries), from the
headers and device bytes kept with the batch.  Results must be the same as with worst-case pools
(JD_FLAG_WORST_CASE_POOLS), which never retry.

Flat (DC-only) images are the densest streams the Annex K tables allow (5.3 walk bits per word in
4:2:0): at full-size pieces (path "full") or one piece per interval ("lanes") their regions
overflow; at the short pieces of a small batch ("auto", "sync") the per-piece slack holds them.
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


def _flat(w, h, ss, rr, v):
    px = np.full((h, w, 3), v, np.uint8)
    px[:, : w // 3] = (v + 60) % 256  # two flat areas: DC differences at the edge only
    return jd_synth.encode(px, 90, ss, rr)


@pytest.fixture(scope="module")
def mixed_batch():
    """Flat images (overflow at full-size pieces) between ordinary synthetic ones (never)."""
    datas = [_flat(1920, 1080, "4:2:0", 0, 40), jd_synth.encode(jd_synth.synth_pixels(1280, 720, 61), 90, "4:2:0", 1),
             _flat(1280, 720, "4:4:4", 0, 90), _flat(1920, 1080, "4:2:0", 2, 140),
             jd_synth.encode(jd_synth.synth_pixels(640, 480, 62), 75, "4:2:2", 0), _flat(777, 333, "4:2:2", 0, 200)]
    refs = []
    for d in datas:
        st, ref = jdoracle.decode(d)
        assert st == 0
        refs.append(ref)
    return datas, refs


@pytest.mark.parametrize("path", ["auto", "sync", "lanes", "full"])
def test_optimistic_pools_retry_bit_exact(mixed_batch, path):
    datas, refs = mixed_batch
    for worst in (False, True):
        dec = jdamd.Decoder(0, path=path, worst_case_pools=worst)
        try:
            outs, status = dec.decode_batch(datas)
            assert status == [0] * len(datas), (path, worst)
            for i, (o, r) in enumerate(zip(outs, refs)):
                assert np.array_equal(o, r), (path, worst, i)
            retried = dec.stats()["retried_images"]
            if worst:
                assert retried == 0
            elif path in ("lanes", "full"):
                assert 1 <= retried <= 4, retried  # the flat images only
        finally:
            dec.close()


@pytest.mark.parametrize("depth", [1, 2])
def test_retry_of_pipelined_batches(depth):
    """Overflowing images inside pipelined batches (jd_decode_batch_async): a batch is retried when
    a later call collects it.  Host-staged inputs are clobbered as soon as each call returns, so the
    retry can only read the slot's device copy (depth 1); at depth 2 such a batch is planned with
    worst-case pools instead.  Device inputs alternate with host inputs."""
    import torch

    sets = []
    for k in range(4):
        sets.append([_flat(1920, 1080, "4:2:0", 0, 30 + 50 * k),
                     jd_synth.encode(jd_synth.synth_pixels(1280, 720, 70 + k), 90, "4:2:0", 1),
                     _flat(1024, 768, "4:4:4", 0, 20 + 30 * k)])
    dec = jdamd.Decoder(0, path="full", async_depth=depth)
    keep = []
    try:
        for k, datas in enumerate(sets):
            hdrs = [jdamd.parse(d) for d in datas]
            ooffs, otot = [], 0
            for h in hdrs:
                ooffs.append(otot)
                otot += (h.width * h.height * 3 + 255) // 256 * 256
            out = torch.zeros(otot, dtype=torch.uint8, device="cuda:0")
            hosts = [np.frombuffer(d, np.uint8).copy() for d in datas]
            if k % 2 == 0:  # device inputs
                offs, tot = [], 0
                for h in hosts:
                    offs.append(tot)
                    tot += (h.nbytes + 64 + 255) // 256 * 256
                din = dec.alloc(tot)
                flat = np.zeros(tot, np.uint8)
                for h, o in zip(hosts, offs):
                    flat[o:o + h.nbytes] = h
                din.upload(flat)
                dev = [din.ptr + o for o in offs]
            else:  # host inputs, staged
                din, dev = None, [None] * len(datas)
            bt = dec.make_batch(hosts, dev, [out.data_ptr() + o for o in ooffs])
            dec.decode_prepared(bt, pipelined=True)
            if din is None:
                for h in hosts:  # staged already: clobber the caller's bytes
                    h[:] = 0
            keep.append((bt, out, hdrs, ooffs, datas, din, hosts))
        dec.wait()
        for bt, out, hdrs, ooffs, datas, din, hosts in keep:
            assert [r.status for r in bt[1]] == [0] * len(datas)
            flatout = out.cpu().numpy()
            for i, (d, h) in enumerate(zip(datas, hdrs)):
                got = flatout[ooffs[i]:ooffs[i] + h.width * h.height * 3].reshape(h.height, h.width, 3)
                assert np.array_equal(got, jdoracle.decode(d)[1]), i
        retried = dec.stats()["retried_images"]
        if depth == 1:
            assert retried >= 4 * 2, retried  # both flat images of every batch
        else:
            assert 4 <= retried <= 6, retried  # the device-input batches' flat images only
    finally:
        for bt, out, hdrs, ooffs, datas, din, hosts in keep:
            if din is not None:
                din.free()
        dec.close()


def test_break_list_overflow_retried(monkeypatch):
    """JD_BRK_CAP=1: one break slot per scan chunk in the optimistic plan.  An image with several
    RSTn in one chunk before its EOI is flagged by k_index and decoded again with kScanCap slots;
    an image without DRI stores its EOI in its one slot and is not retried."""
    monkeypatch.setenv("JD_BRK_CAP", "1")
    datas = jd_synth.make_batch(3, 1280, 720, 90, "4:2:0", 1, 0, seed0=9910)  # RSTn every MCU row
    datas += jd_synth.make_batch(3, 1280, 720, 90, "4:2:0", 0, 0, seed0=9920)  # no DRI
    dec = jdamd.Decoder(0)
    try:
        outs, status = dec.decode_batch(datas)
        assert status == [0] * len(datas)
        for i, (d, o) in enumerate(zip(datas, outs)):
            assert np.array_equal(o, jdoracle.decode(d)[1]), i
        assert dec.stats()["retried_images"] == 3
    finally:
        dec.close()


def test_corrupt_image_not_retried_forever():
    """A truncated flat image overflows in the optimistic plan, is retried once with worst-case
    pools, and reported corrupt; the rest of its batch decodes."""
    good = jd_synth.encode(jd_synth.synth_pixels(640, 480, 80), 90, "4:2:0", 1)
    flat = _flat(1920, 1080, "4:2:0", 0, 77)
    bad = flat[: len(flat) * 2 // 3] + b"\xff\xd9"
    dec = jdamd.Decoder(0, path="full")
    try:
        outs, status = dec.decode_batch([good, bad, good])
        assert status[0] == 0 and status[2] == 0 and status[1] == jdoracle.decode(bad)[0] != 0
        assert np.array_equal(outs[0], jdoracle.decode(good)[1])
        assert dec.stats()["retried_images"] <= 1
    finally:
        dec.close()


def test_optimistic_pools_smaller_than_worst_case():
    """The pools of a C2-shaped batch (1080p 4:2:0 q90, DRI = one MCU row) at most 0.7x the
    worst-case ones, with no retry."""
    datas = jd_synth.make_batch(48, 1920, 1080, 90, "4:2:0", 1, 0, seed0=9950)
    peaks = {}
    for worst in (False, True):
        dec = jdamd.Decoder(0, worst_case_pools=worst)
        try:
            _, status = dec.decode_batch(datas)
            assert status == [0] * len(datas)
            assert dec.stats()["retried_images"] == 0
            peaks[worst] = dec.device_bytes()[1]
        finally:
            dec.close()
    assert peaks[False] <= 0.7 * peaks[True], peaks


def test_synchronize_runs_pending_retries():
    """jd_synchronize collects a pipelined batch and decodes its overflowed images again before it
    returns, like jd_decode_wait."""
    import torch

    datas = [_flat(1920, 1080, "4:2:0", 0, 99), jd_synth.encode(jd_synth.synth_pixels(640, 480, 90), 90, "4:2:0", 1)]
    hdrs = [jdamd.parse(d) for d in datas]
    ooffs, otot = [], 0
    for h in hdrs:
        ooffs.append(otot)
        otot += (h.width * h.height * 3 + 255) // 256 * 256
    dec = jdamd.Decoder(0, path="full")
    try:
        out = torch.zeros(otot, dtype=torch.uint8, device="cuda:0")
        hosts = [np.frombuffer(d, np.uint8).copy() for d in datas]
        bt = dec.make_batch(hosts, [None] * len(datas), [out.data_ptr() + o for o in ooffs])
        dec.decode_prepared(bt, pipelined=True)
        dec.synchronize()
        assert [r.status for r in bt[1]] == [0, 0]
        assert dec.stats()["retried_images"] == 1
        flat = out.cpu().numpy()
        for i, (d, h) in enumerate(zip(datas, hdrs)):
            got = flat[ooffs[i]:ooffs[i] + h.width * h.height * 3].reshape(h.height, h.width, 3)
            assert np.array_equal(got, jdoracle.decode(d)[1]), i
    finally:
        dec.close()


def _async_host_batch(dec, datas):
    """A pipelined batch of host-staged inputs with device outputs; the caller's host bytes are
    clobbered once the call returns (only the slot's device copy can produce the pixels)."""
    import torch

    hdrs = [jdamd.parse(d) for d in datas]
    ooffs, otot = [], 0
    for h in hdrs:
        ooffs.append(otot)
        otot += (h.width * h.height * 3 + 255) // 256 * 256
    out = torch.zeros(otot, dtype=torch.uint8, device="cuda:0")
    hosts = [np.frombuffer(d, np.uint8).copy() for d in datas]
    bt = dec.make_batch(hosts, [None] * len(datas), [out.data_ptr() + o for o in ooffs])
    dec.decode_prepared(bt, pipelined=True)
    for h in hosts:
        h[:] = 0
    return bt, out, hdrs, ooffs, hosts


def _check_async(bt, out, hdrs, ooffs, datas):
    assert [r.status for r in bt[1]] == [0] * len(datas)
    flat = out.cpu().numpy()
    for i, (d, h) in enumerate(zip(datas, hdrs)):
        got = flat[ooffs[i]:ooffs[i] + h.width * h.height * 3].reshape(h.height, h.width, 3)
        assert np.array_equal(got, jdoracle.decode(d)[1]), i


def test_retry_before_a_host_output_call_reuses_the_slot():
    """A pipelined batch with an overflowing host-staged image, then a blocking call with host
    outputs: that call collects the pipelined batch first, and its retry must run before the
    call's own launch reuses a slot (and its device input pool)."""
    a = [_flat(1920, 1080, "4:2:0", 0, 11), _flat(1024, 768, "4:4:4", 0, 222)]
    b = [_flat(1280, 720, "4:2:0", 0, 66), jd_synth.encode(jd_synth.synth_pixels(640, 480, 91), 90, "4:2:0", 1)]
    dec = jdamd.Decoder(0, path="full")
    try:
        ka = _async_host_batch(dec, a)
        outs, status = dec.decode_batch(b)  # host outputs
        assert status == [0, 0]
        for d, o in zip(b, outs):
            assert np.array_equal(o, jdoracle.decode(d)[1])
        _check_async(*ka[:4], a)
        assert dec.stats()["retried_images"] >= 3
    finally:
        dec.close()


def test_retry_between_sub_batches(monkeypatch):
    """A pipelined call split into sub-batches (JD_MAX_BATCH_IMAGES=2): a sub-batch collected
    inside the call is retried before the next sub-batch reuses its slot."""
    monkeypatch.setenv("JD_MAX_BATCH_IMAGES", "2")
    sets = [[_flat(1920, 1080, "4:2:0", 0, 17 + 40 * k), _flat(1024, 768, "4:4:4", 0, 5 + 30 * k),
             jd_synth.encode(jd_synth.synth_pixels(800, 600, 93 + k), 90, "4:2:0", 1),
             _flat(1280, 720, "4:2:2", 0, 150 + 20 * k), _flat(640, 480, "4:2:0", 0, 77 + k)] for k in range(2)]
    dec = jdamd.Decoder(0, path="full")
    try:
        runs = [_async_host_batch(dec, s) for s in sets]
        dec.wait()
        for (bt, out, hdrs, ooffs, _), s in zip(runs, sets):
            _check_async(bt, out, hdrs, ooffs, s)
        assert dec.stats()["retried_images"] >= 6
    finally:
        dec.close()


def test_large_batch_overflow_retried():
    """A batch large enough for the device piece plan (k_pieceplan: full-size pieces grown to fill
    the resident lanes, k_chain_fix, LDS-free re-walk tables) with flat images among C2-shaped
    ones: the flat images overflow their regions, are retried, and every image is bit-exact."""
    datas = jd_synth.make_batch(224, 1920, 1080, 90, "4:2:0", 1, 0, seed0=12000)
    flats = [_flat(1920, 1080, "4:2:0", 0, 9 + 29 * k) for k in range(4)] + \
            [_flat(1920, 1080, "4:4:4", 1, 200 - 31 * k) for k in range(4)]
    for k, f in enumerate(flats):
        datas.insert(17 + 25 * k, f)
    dec = jdamd.Decoder(0, timing=True)
    try:
        outs, status = dec.decode_batch(datas)
        assert status == [0] * len(datas)
        st = dec.stats()
        assert st["retried_images"] >= 4, st["retried_images"]  # at least the 4:2:0 flat images
        for i, (d, o) in enumerate(zip(datas, outs)):
            if d in flats or i % 16 == 0:
                assert np.array_equal(o, jdoracle.decode(d)[1]), i
    finally:
        dec.close()
