"""Shared fixtures.  `-m "not gpu"` runs on CPU; `-m gpu` tests need a MI355X (gfx950)."""
import json
import os
import sys

import pytest

# PyTorch-ROCm bundles its own libamdhip64.so.7 and libjdamd.so links the system one under the same
# soname: whichever loads first serves the process.  torch must come first (a torch that finds the
# system runtime already loaded reports "No HIP GPUs are available"), so the GPU tests that also use
# torch streams / tensors run in any order and selection.
import torch  # noqa: E402,F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-jpeg-decoder_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a MI355X GPU (run with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        entries = json.load(f)["entries"]
    for e in entries:
        with open(os.path.join(GOLDEN, e["file"]), "rb") as f:
            e["data"] = f.read()
    return entries


@pytest.fixture(scope="session", params=["auto", "sync", "lanes", "full"])
def decoder(request):
    """A decoder per entropy-decode path: default selection (small batches: short pieces), every
    image through 1024-bit pieces, every image one lane per restart interval, and the full-batch
    geometry (8192-bit pieces, 4096-bit warm-up) whatever the batch size."""
    import jdamd

    dec = jdamd.Decoder(0, timing=True, path=request.param)
    yield dec
    dec.close()


@pytest.fixture(scope="session")
def sync_decoder():
    import jdamd

    dec = jdamd.Decoder(0, timing=True, path="sync")
    yield dec
    dec.close()
