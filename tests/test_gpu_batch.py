"""GPU parity of large and split batches (round-2 additions).

* A BASELINE-config-5-shaped batch (1024 mixed 4:4:4 / 4:2:2 / 4:2:0 1080p, q in {50,75,90,95}, no
  DRI) is decoded as ONE launch; its AC-entry slots pass 2^32, so the tail images' image-relative
  entry indices sit on a 64-bit ImgDesc::entry_base beyond 2^32.  Head, middle and tail images
  are checked bit-exact against the oracle.
* A batch forced into three sub-batches (JD_MAX_BATCH_ENTRIES) with host inputs and host outputs:
  every image bit-exact (the sub-batches share the staging and output pools).
* A batch of mutated headers / entropy data: per-image status and pixels equal the oracle's.

Reference path replaced: batchDecodeKernel (cuda-decoder/src/parser.cu:663-682).
"""
import os
import sys

import numpy as np
import pytest

import jdamd
import jdoracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import jd_synth  # noqa: E402

pytestmark = pytest.mark.gpu


def entry_slots(h):
    """AC-entry slots of one image (jd_runtime.cpp entry_slots_per_mcu: 63 per block + 3 per MCU)."""
    return h.mcux * h.mcuy * (63 * h.blocks_per_mcu + 3)


def _device_batch(dec, datas):
    hosts = [np.frombuffer(d, np.uint8).copy() for d in datas]
    hdrs = [jdamd.parse(d) for d in datas]
    offs, tot = [], 0
    for h in hosts:
        offs.append(tot)
        tot += (h.nbytes + 64 + 255) // 256 * 256
    ooffs, otot = [], 0
    for h in hdrs:
        ooffs.append(otot)
        otot += (h.width * h.height * 3 + 255) // 256 * 256
    din, dout = dec.alloc(tot), dec.alloc(otot)
    flat = np.zeros(tot, np.uint8)
    for h, o in zip(hosts, offs):
        flat[o:o + h.nbytes] = h
    din.upload(flat)
    return hosts, hdrs, din, dout, offs, ooffs


def test_mixed_batch_tail_beyond_2_32_entry_slots():
    n = 1024
    datas = jd_synth.make_batch(n, 1920, 1080, mixed=True, seed0=500000)
    dec = jdamd.Decoder(0)
    try:
        hosts, hdrs, din, dout, offs, ooffs = _device_batch(dec, datas)
        bases, run = [], 0
        for h in hdrs:
            bases.append(run)
            run += entry_slots(h)
        tail = [i for i in range(n) if bases[i] >= 1 << 32]
        assert tail and tail[-1] == n - 1, "the batch must put its tail past 2^32 entry slots"
        status = dec.decode_batch_device(hosts, [din.ptr + o for o in offs], [dout.ptr + o for o in ooffs])
        assert status == [0] * n
        check = sorted({0, 1, n // 2, tail[0], tail[len(tail) // 2], n - 2, n - 1})
        for i in check:
            h = hdrs[i]
            got = dout.download(np.empty((h.height, h.width, 3), np.uint8), ooffs[i])
            st, ref = jdoracle.decode(datas[i])
            assert st == 0 and np.array_equal(got, ref), (i, bases[i])
        din.free()
        dout.free()
    finally:
        dec.close()


def test_forced_split_host_inputs_and_outputs(monkeypatch):
    """sub-batches of one call reuse the pinned input staging and the output
    pool; each must be collected before the next is launched."""
    datas = jd_synth.make_batch(24, 640, 480, 90, "4:2:0", 1, 0, seed0=7000)
    datas += jd_synth.make_batch(12, 800, 600, 75, "4:4:4", 0, 0, seed0=8000)
    per = entry_slots(jdamd.parse(datas[0]))
    monkeypatch.setenv("JD_MAX_BATCH_ENTRIES", str(per * 64 * 14 // 63))  # ~14 images of the first kind
    dec = jdamd.Decoder(0)
    try:
        outs, status = dec.decode_batch(datas)
        assert status == [0] * len(datas)
        for d, o in zip(datas, outs):
            st, ref = jdoracle.decode(d)
            assert st == 0 and np.array_equal(o, ref)
        stats = dec.stats()
        assert stats["batches"] >= 3, stats["batches"]  # really split
    finally:
        dec.close()


def test_async_then_blocking_call_on_another_stream():
    """a pending jd_decode_batch_async batch on the context stream, then a
    blocking call on another stream: the scratch pools must not be overwritten under it."""
    import torch

    datas = jd_synth.make_batch(16, 1280, 720, 90, "4:2:0", 1, 0, seed0=9100)
    dec = jdamd.Decoder(0)
    try:
        hosts, hdrs, din, dout, offs, ooffs = _device_batch(dec, datas)
        bt = dec.make_batch(hosts, [din.ptr + o for o in offs], [dout.ptr + o for o in ooffs])
        dec.decode_prepared(bt, pipelined=True)
        other = torch.cuda.Stream(device=0)
        small = jd_synth.make_batch(4, 320, 240, 90, "4:2:2", 0, 0, seed0=9200)
        h2, d2, din2, dout2, o2, oo2 = _device_batch(dec, small)
        st2 = dec.decode_batch_device(h2, [din2.ptr + o for o in o2], [dout2.ptr + o for o in oo2],
                                      stream=other.cuda_stream)
        dec.wait()
        assert [r.status for r in bt[1]] == [0] * len(datas) and st2 == [0] * len(small)
        for i, h in enumerate(hdrs):
            got = dout.download(np.empty((h.height, h.width, 3), np.uint8), ooffs[i])
            assert np.array_equal(got, jdoracle.decode(datas[i])[1]), i
        for i, h in enumerate(d2):
            got = dout2.download(np.empty((h.height, h.width, 3), np.uint8), oo2[i])
            assert np.array_equal(got, jdoracle.decode(small[i])[1]), i
    finally:
        dec.close()


def test_mutated_files_batch_matches_oracle_status_and_pixels():
    """Header and entropy mutations of the golden corpus in one batch: every image's status class
    and (when decodable) pixels equal the oracle's; corrupt images never poison the batch."""
    from test_abi import _fuzz_corpus, mutate

    rng = np.random.default_rng(5150)
    corpus = _fuzz_corpus()
    datas = []
    for it in range(240):
        d = mutate(corpus[it % len(corpus)], rng)
        if it % 3 == 0 and len(d) > 200:  # plus an entropy-segment byte flip
            d = bytearray(d)
            i = int(rng.integers(len(d) // 2, len(d) - 2))
            d[i] ^= 1 << int(rng.integers(0, 8))
            d = bytes(d)
        st, info = jdoracle.info(d)
        if st == 0 and info.width * info.height > 1 << 22:  # a mutated SOF size: keep memory bounded
            continue
        datas.append(d)
    dec = jdamd.Decoder(0)
    try:
        outs, status = dec.decode_batch(datas)
        n_ok = 0
        for i, (d, o, s) in enumerate(zip(datas, outs, status)):
            st, ref = jdoracle.decode(d)
            assert s == st, (i, s, st)
            if st == 0:
                n_ok += 1
                assert np.array_equal(o, ref), i
        assert n_ok >= 10
    finally:
        dec.close()
