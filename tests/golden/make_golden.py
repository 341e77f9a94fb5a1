#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (run in the build container).

Inputs and what pins each expected output:
  ref/*.jpg     the reference's own test images (/root/reference/testing/images, data files).
                Expected RGB = SHA-256 of the reference's ground truth
                (/root/reference/testing/ground_truth/*.array, which is byte-identical to the
                reference C++ decoder's output).  "pinned_by": "reference_ground_truth".
                4_800x600 has no committed ground truth (missing blob); its expected digest comes
                from the reference C++ decoder built by oracle/Makefile ("reference_decoder").
  gen/*.jpg     small Pillow (libjpeg-turbo) encodes of seeded synthetic images covering the
                hot-path configurations.  Expected RGB = our oracle (oracle/liboracle.so), and
                  - 4:4:4 without DRI: oracle == reference decoder on the same file
                    ("reference_decoder"),
                  - with DRI: oracle output == oracle output of the same pixels encoded without
                    DRI ("rst_invariance"; restart intervals do not change the coefficients),
                  - other sampling factors: defined semantics, sanity-checked
                    against Pillow within a tolerance ("semantics+tolerance"; parity unpinned by
                    the reference, which decodes these files to garbage).
Writes golden.json.
"""
import hashlib
import io
import json
import os
import shutil
import sys
import tempfile

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import jdoracle  # noqa: E402

REF_TESTING = "/root/reference/testing"


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint8).tobytes()).hexdigest()


def synth(w, h, seed, gray=False):
    """SURVEY.md §8(d) synthetic content: 128 + A sin(x fx + y fy + phi) + N(0, 3) per channel."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    chans = []
    for _ in range(1 if gray else 3):
        fx, fy = rng.uniform(1 / 80, 1 / 20, 2) * 2 * np.pi
        phi = rng.uniform(0, 2 * np.pi)
        amp = rng.uniform(40, 110)
        c = 128 + amp * np.sin(x * fx + y * fy + phi) + rng.normal(0, 3, (h, w))
        chans.append(np.clip(np.rint(c), 0, 255).astype(np.uint8))
    a = chans[0] if gray else np.stack(chans, -1)
    return Image.fromarray(a, "L" if gray else "RGB")


def encode(img, **kw):
    b = io.BytesIO()
    img.save(b, "JPEG", **kw)
    return b.getvalue()


def main():
    os.makedirs(os.path.join(HERE, "ref"), exist_ok=True)
    os.makedirs(os.path.join(HERE, "gen"), exist_ok=True)
    entries = []
    work = tempfile.mkdtemp()
    have_ref = jdoracle.ref_available()

    # ---- the reference's own fixtures --------------------------------------------------------
    for fn in sorted(os.listdir(os.path.join(REF_TESTING, "images"))) + ["image.jpeg"]:
        src = os.path.join(REF_TESTING, "images", fn) if fn != "image.jpeg" else os.path.join(REF_TESTING, fn)
        dst = os.path.join(HERE, "ref", fn)
        shutil.copyfile(src, dst)
        data = open(dst, "rb").read()
        st, rgb = jdoracle.decode(data)
        name = os.path.splitext(fn)[0]
        gt = os.path.join(REF_TESTING, "ground_truth", name + ".array")
        e = {"file": "ref/" + fn, "status": st, "width": int(rgb.shape[1]), "height": int(rgb.shape[0]),
             "sha256": sha(rgb)}
        if os.path.exists(gt):
            g = jdoracle.read_array(gt)
            assert sha(g) == e["sha256"], f"oracle != reference ground truth on {fn}"
            e["pinned_by"] = "reference_ground_truth"
        elif fn == "image.jpeg":
            e["pinned_by"] = "semantics+tolerance"  # 4:2:0: the reference decodes it to garbage
        elif have_ref:
            r = jdoracle.ref_decode(dst, work)
            assert sha(r) == e["sha256"], f"oracle != reference decoder on {fn}"
            e["pinned_by"] = "reference_decoder"
        entries.append(e)

    # ---- generated configurations ------------------------------------------------------------
    sizes = [(1, 1), (7, 5), (8, 8), (16, 16), (33, 17), (64, 48), (100, 75), (127, 129), (256, 192)]
    subs = ["4:4:4", "4:2:2", "4:2:0"]
    cases = []
    seed = 0
    for (w, h) in sizes:
        for ss in subs:
            for q in (50, 90):
                cases.append(dict(w=w, h=h, ss=ss, q=q, seed=seed, rst=None, opt=False, gray=False))
                seed += 1
    for (w, h) in [(64, 48), (127, 129), (256, 192), (200, 200)]:
        for ss in subs:
            for rst in ({"restart_marker_blocks": 1}, {"restart_marker_blocks": 3}, {"restart_marker_rows": 1}):
                cases.append(dict(w=w, h=h, ss=ss, q=75, seed=seed, rst=rst, opt=False, gray=False))
                seed += 1
    for (w, h) in [(64, 48), (123, 77)]:
        for ss in subs:
            cases.append(dict(w=w, h=h, ss=ss, q=95, seed=seed, rst=None, opt=True, gray=False))
            cases.append(dict(w=w, h=h, ss=ss, q=100, seed=seed + 1, rst=None, opt=False, gray=False))
            seed += 2
    for (w, h) in [(33, 17), (128, 96)]:
        cases.append(dict(w=w, h=h, ss="4:4:4", q=80, seed=seed, rst=None, opt=False, gray=True))
        cases.append(dict(w=w, h=h, ss="4:4:4", q=80, seed=seed + 1, rst={"restart_marker_blocks": 2}, opt=False,
                          gray=True))
        seed += 2

    for c in cases:
        img = synth(c["w"], c["h"], c["seed"], c["gray"])
        kw = dict(quality=c["q"], optimize=c["opt"])
        if not c["gray"]:
            kw["subsampling"] = c["ss"]
        base = encode(img, **kw)
        data = encode(img, **kw, **(c["rst"] or {}))
        tag = "gray" if c["gray"] else c["ss"].replace(":", "")
        rtag = "" if not c["rst"] else "_" + "_".join(f"{k.split('_')[-1]}{v}" for k, v in c["rst"].items())
        fn = f"g{c['seed']:03d}_{c['w']}x{c['h']}_{tag}_q{c['q']}{'_opt' if c['opt'] else ''}{rtag}.jpg"
        with open(os.path.join(HERE, "gen", fn), "wb") as f:
            f.write(data)
        st, rgb = jdoracle.decode(data)
        assert st == 0, (fn, st)
        e = {"file": "gen/" + fn, "status": st, "width": c["w"], "height": c["h"], "sha256": sha(rgb),
             "subsampling": tag, "quality": c["q"], "restart": c["rst"] or {}}
        if c["rst"]:
            st0, rgb0 = jdoracle.decode(base)
            assert st0 == 0 and np.array_equal(rgb0, rgb), f"RST invariance broken on {fn}"
            e["pinned_by"] = "rst_invariance"
        elif tag == "444" and have_ref:
            p = os.path.join(work, fn)
            with open(p, "wb") as f:
                f.write(data)
            r = jdoracle.ref_decode(p, work)
            assert np.array_equal(r, rgb), f"oracle != reference decoder on {fn}"
            e["pinned_by"] = "reference_decoder"
        else:
            e["pinned_by"] = "semantics+tolerance"
        pil = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
        e["max_abs_vs_pillow"] = int(np.abs(pil.astype(int) - rgb.astype(int)).max())
        e["mean_abs_vs_pillow"] = float(np.abs(pil.astype(int) - rgb.astype(int)).mean())
        entries.append(e)

    # ---- unsupported variants (status only) --------------------------------------------------
    img = synth(48, 40, 999)
    for fn, data, want in [("u_progressive.jpg", encode(img, quality=90, progressive=True), 3)]:
        with open(os.path.join(HERE, "gen", fn), "wb") as f:
            f.write(data)
        st, _ = jdoracle.decode(data)
        assert st == want, (fn, st)
        entries.append({"file": "gen/" + fn, "status": st, "pinned_by": "status"})

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "entries": entries}, f, indent=1)
    shutil.rmtree(work, ignore_errors=True)
    print(f"{len(entries)} golden entries")


if __name__ == "__main__":
    main()
