"""H2D copy rates by host-memory kind (DESIGN.md §4.5 host inputs): pageable, registered
(jd_host_register = hipHostRegister of a caller buffer) and allocated pinned (torch pin_memory =
hipHostMalloc), through the library's jd_memcpy_h2d, for one batch-sized buffer and in 128 MiB chunks.

    python tools/h2d_rates.py [MiB]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gpu-jpeg-decoder_amd"))


def rate(dec, dst, src_ptr, n, chunk, reps=3):
    lib = dec.lib
    best = 0.0
    for _ in range(reps):
        t = time.perf_counter()
        for o in range(0, n, chunk):
            lib.jd_memcpy_h2d(dec.ctx, dst + o, src_ptr + o, min(chunk, n - o))
        dec.synchronize()
        best = max(best, n / (time.perf_counter() - t) / 1e9)
    return best


def main():
    import torch
    import jdamd

    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 640
    n = mib << 20
    dec = jdamd.Decoder(0)
    dst = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    page = np.ones(n, np.uint8)
    reg = np.ones(n, np.uint8)
    pin = torch.ones(n, dtype=torch.uint8).pin_memory()
    t = time.perf_counter()
    dec.register_host(reg)
    t_reg = time.perf_counter() - t
    out = {"MiB": mib, "register_ms": round(t_reg * 1e3, 2)}
    for name, ptr in (("pageable", page.ctypes.data), ("registered", reg.ctypes.data), ("pinned_alloc", pin.data_ptr())):
        for chunk in (n, 128 << 20, 16 << 20):
            out[f"{name}_chunk{chunk >> 20}MiB_GB_s"] = round(rate(dec, dst.data_ptr(), ptr, n, chunk), 2)
    dec.unregister_host(reg)
    dec.close()
    print(out)


if __name__ == "__main__":
    main()
