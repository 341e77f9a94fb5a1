"""ctypes binding of oracle/liboracle.so — the CPU restatement of the reference decoder.

TEST INFRASTRUCTURE ONLY: imported by tests/, by __graft_entry__.smoke() (as the checker) and by
bench.py's cpu_baseline leg.  The product (gpu-jpeg-decoder_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_DECODER = os.path.join(HERE, "_ref", "decoder")
REF_BENCH = os.path.join(HERE, "_ref", "ref_bench")

_lib = None


class _Info(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("ncomp", ctypes.c_int),
                ("hmax", ctypes.c_int), ("vmax", ctypes.c_int), ("mcux", ctypes.c_int), ("mcuy", ctypes.c_int),
                ("blocks_per_mcu", ctypes.c_int), ("restart_interval", ctypes.c_int),
                ("h", ctypes.c_int * 4), ("v", ctypes.c_int * 4), ("tq", ctypes.c_int * 4),
                ("ecs_offset", ctypes.c_size_t)]


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE, "oracle"], check=True, capture_output=True)
        L = ctypes.CDLL(LIB)
        L.jdo_parse.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(_Info)]
        L.jdo_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_int)]
        L.jdo_decode_ex.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int), ctypes.c_uint]
        L.jdo_decode_coefs.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.jdo_idct_ref.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.jdo_color_ref.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.jdo_decode_many.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_void_p]
        L.jdo_decode_many.restype = ctypes.c_double
        L.jdo_decode_fast.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                      ctypes.POINTER(ctypes.c_int)]
        L.jdo_decode_many_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_int]
        L.jdo_decode_many_ex.restype = ctypes.c_double
        _lib = L
    return _lib


def info(data: bytes) -> Tuple[int, _Info]:
    i = _Info()
    st = lib().jdo_parse(data, len(data), ctypes.byref(i))
    return st, i


FANCY_UPSAMPLING = 8  # == JD_FLAG_FANCY_UPSAMPLING


def decode(data: bytes, fancy: bool = False) -> Tuple[int, Optional[np.ndarray]]:
    """(status, RGB uint8 [H,W,3] or None).  Mirrors JPEGParser extract()+decode(); fancy=True
    selects libjpeg's triangular chroma upsampling (an option beyond the reference)."""
    st, i = info(data)
    if st != 0:
        return st, None
    out = np.empty((i.height, i.width, 3), np.uint8)
    w, h = ctypes.c_int(), ctypes.c_int()
    st = lib().jdo_decode_ex(data, len(data), out.ctypes.data, ctypes.byref(w), ctypes.byref(h),
                             FANCY_UPSAMPLING if fancy else 0)
    return st, out


def decode_coefs(data: bytes) -> Tuple[int, Optional[np.ndarray]]:
    st, i = info(data)
    if st != 0:
        return st, None
    out = np.zeros((i.mcux * i.mcuy * i.blocks_per_mcu, 64), np.int32)
    st = lib().jdo_decode_coefs(data, len(data), out.ctypes.data)
    return st, out


def idct(zz_dequant: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(zz_dequant, dtype=np.int32).reshape(-1, 64)
    out = np.empty_like(a)
    L = lib()
    for k in range(a.shape[0]):
        L.jdo_idct_ref(a[k].ctypes.data, out[k].ctypes.data)
    return out


def color(y: int, cb: int, cr: int) -> Tuple[int, int, int]:
    o = (ctypes.c_uint8 * 3)()
    lib().jdo_color_ref(y, cb, cr, o)
    return o[0], o[1], o[2]


def decode_fast(data: bytes) -> Tuple[int, Optional[np.ndarray]]:
    """The "fast" CPU mode (jdo_decode_fast: LUT Huffman, integer colour terms): a CPU baseline
    with decode()'s status and pixels."""
    st, i = info(data)
    if st != 0:
        return st, None
    out = np.empty((i.height, i.width, 3), np.uint8)
    st = lib().jdo_decode_fast(data, len(data), out.ctypes.data, None, None)
    return st, out


def decode_many(datas: Sequence[np.ndarray], threads: int = 1, want_rgb: bool = False, fast: bool = False):
    """Times jdo_decode (fast: jdo_decode_fast) over a list of uint8 arrays.  Returns (seconds,
    statuses, rgbs or None)."""
    n = len(datas)
    ptrs = (ctypes.c_void_p * n)(*[d.ctypes.data for d in datas])
    lens = (ctypes.c_size_t * n)(*[d.nbytes for d in datas])
    status = (ctypes.c_int * n)()
    rgbs = None
    rgb_ptrs = None
    if want_rgb:
        rgbs = []
        for d in datas:
            st, i = info(d.tobytes())
            rgbs.append(np.empty((i.height, i.width, 3), np.uint8))
        rgb_ptrs = (ctypes.c_void_p * n)(*[r.ctypes.data for r in rgbs])
    secs = lib().jdo_decode_many_ex(ptrs, lens, n, rgb_ptrs, threads, status, 1 if fast else 0)
    return secs, list(status), rgbs


def ref_available() -> bool:
    return os.path.exists(REF_DECODER)


def ref_decode(path: str, workdir: str) -> np.ndarray:
    """Runs the reference C++ decoder (built from /root/reference by oracle/Makefile) on `path`.
    The reference writes ../testing/cpp_output_arrays/<name>.array relative to its cwd
    (cpp-decoder/src/parser.cpp:199), so it runs inside a scratch tree."""
    run = os.path.join(workdir, "run")
    arr_dir = os.path.join(workdir, "testing", "cpp_output_arrays")
    os.makedirs(run, exist_ok=True)
    os.makedirs(arr_dir, exist_ok=True)
    subprocess.run([REF_DECODER, os.path.abspath(path)], cwd=run, check=True, capture_output=True)
    name = os.path.splitext(os.path.basename(path))[0] + ".array"
    return read_array(os.path.join(arr_dir, name))


def read_array(path: str) -> np.ndarray:
    """Reads the reference's `.array` text format into uint8 [H, W, 3]."""
    with open(path) as f:
        h, w = map(int, f.readline().split())
        planes = [np.array(f.readline().split(), dtype=np.int64) for _ in range(3)]
    return np.stack([p.reshape(h, w) for p in planes], -1).astype(np.uint8)
