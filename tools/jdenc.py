"""ctypes binding of tools/libjdenc.so, the in-repo deterministic baseline JPEG encoder (jdenc.c).

Used by jd_synth (bench and test inputs); not part of the decode path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libjdenc.so")
_lib = None

# luma sampling factors (h, v) per subsampling name; chroma is 1x1
SAMPLING = {"4:4:4": (1, 1), "4:2:2": (2, 1), "4:2:0": (2, 2), "4:4:0": (1, 2)}


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "libjdenc.so"], check=True, capture_output=True)
        L = ctypes.CDLL(LIB)
        L.jdenc_encode.restype = ctypes.c_long
        L.jdenc_encode.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        L.jdenc_bound.restype = ctypes.c_size_t
        L.jdenc_bound.argtypes = [ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def encode(pixels: np.ndarray, quality: int = 90, subsampling: str = "4:2:0", restart_rows: int = 0,
           restart_blocks: int = 0) -> bytes:
    """Baseline JPEG of uint8 pixels ([H, W, 3] RGB or [H, W] gray).  restart_rows = MCU rows per
    restart interval, restart_blocks = MCUs per interval (as Pillow's restart_marker_* options)."""
    px = np.ascontiguousarray(pixels, dtype=np.uint8)
    h, w = px.shape[:2]
    gray = px.ndim == 2
    hs, vs = (1, 1) if gray else SAMPLING[subsampling]
    mcux = (w + 8 * hs - 1) // (8 * hs)
    restart = restart_blocks or restart_rows * mcux
    L = lib()
    cap = L.jdenc_bound(w, h)
    out = np.empty(cap, np.uint8)
    n = L.jdenc_encode(px.ctypes.data, w, h, 1 if gray else 3, quality, hs, vs, restart, out.ctypes.data, cap)
    if n < 0:
        raise ValueError(f"jdenc_encode failed ({n})")
    return out[:n].tobytes()
