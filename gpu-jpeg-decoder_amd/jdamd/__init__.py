"""jdamd — ctypes binding of libjdamd.so (the C ABI in include/jd.h).

This is the binding a Python caller of the reference's decode path would add:
the reference itself is reached from Python only through a subprocess + `.array` files
(/root/reference/testing/compare.py:37-64); here the same path is a direct call.

No CPU fallback exists: if libjdamd.so is missing or no GPU is present, the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import warnings
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libjdamd.so")

JD_OK = 0
JD_ERR_INVALID_ARG = 1
JD_ERR_CORRUPT = 2
JD_ERR_UNSUPPORTED = 3
JD_ERR_TRUNCATED = 4
JD_ERR_HIP = 5
JD_ERR_NOMEM = 6
JD_ERR_CAPACITY = 7
JD_ERR_IO = 8
JD_FLAG_TIMING = 1
JD_FLAG_FORCE_SYNC = 2
JD_FLAG_FORCE_LANES = 4
JD_FLAG_FANCY_UPSAMPLING = 8
JD_FLAG_FULL_PIECES = 16
JD_FLAG_ASYNC_DEPTH2 = 32
JD_FLAG_WORST_CASE_POOLS = 64
PATHS = {"auto": 0, "sync": JD_FLAG_FORCE_SYNC, "lanes": JD_FLAG_FORCE_LANES, "full": JD_FLAG_FULL_PIECES}
JD_ABI_VERSION = 8
JD_NUM_KERNELS = 11
KERNEL_NAMES = ["k_scan", "k_index", "k_compact", "k_subplan", "k_piece", "k_redo", "k_chain",
                "k_gather", "k_dc_pred", "k_idct_color", "k_colour_fancy"]


class JDError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {status_str(status)} ({status})" if what else status_str(status))


class _Header(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int), ("height", ctypes.c_int), ("ncomp", ctypes.c_int),
        ("h", ctypes.c_int * 4), ("v", ctypes.c_int * 4), ("tq", ctypes.c_int * 4),
        ("hmax", ctypes.c_int), ("vmax", ctypes.c_int), ("mcux", ctypes.c_int), ("mcuy", ctypes.c_int),
        ("blocks_per_mcu", ctypes.c_int), ("restart_interval", ctypes.c_int), ("subsampling", ctypes.c_int),
        ("ecs_offset", ctypes.c_uint64),
    ]


class _Opts(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint), ("parse_threads", ctypes.c_int)]


class _Item(ctypes.Structure):
    _fields_ = [("jpeg", ctypes.c_void_p), ("jpeg_dev", ctypes.c_void_p), ("len", ctypes.c_size_t),
                ("rgb", ctypes.c_void_p)]


class _Result(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int), ("width", ctypes.c_int), ("height", ctypes.c_int)]


class _Stats(ctypes.Structure):
    _fields_ = [("launches", ctypes.c_int * JD_NUM_KERNELS), ("total_ms", ctypes.c_double * JD_NUM_KERNELS),
                ("bytes", ctypes.c_double * JD_NUM_KERNELS), ("batches", ctypes.c_double),
                ("images", ctypes.c_double), ("pixels", ctypes.c_double), ("ecs_bytes", ctypes.c_double),
                ("blocks", ctypes.c_double), ("segments", ctypes.c_double), ("subsequences", ctypes.c_double),
                ("host_ms", ctypes.c_double * 4), ("h2d_bytes", ctypes.c_double),
                ("h2d_registered_bytes", ctypes.c_double), ("redo_pieces", ctypes.c_double),
                ("fix_intervals", ctypes.c_double), ("fix_rounds", ctypes.c_double), ("fix_rewalks", ctypes.c_double),
                ("fix_early", ctypes.c_double), ("retried_images", ctypes.c_double)]


# Every symbol include/jd.h and include/jd_test.h declare (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = [
    "jd_ctx_create", "jd_ctx_destroy", "jd_parse", "jd_decode", "jd_decode_file", "jd_decode_batch",
    "jd_decode_batch_async", "jd_decode_wait", "jd_write_array", "jd_write_ppm", "jd_status_str", "jd_abi_version", "jd_device_alloc", "jd_device_free",
    "jd_memcpy_h2d", "jd_memcpy_d2h", "jd_synchronize", "jd_get_stats", "jd_reset_stats",
    "jd_kernel_name", "jd_test_idct", "jd_test_idct_exact", "jd_test_color", "jd_debug_fetch", "jd_ctx_last_error",
    "jd_test_copy_peak", "jd_device_bytes", "jd_host_register", "jd_host_unregister",
    "jd_host_alloc", "jd_host_free",
]

_lib = None


def _abi_mismatch_allowed() -> bool:
    """JDAMD_ALLOW_ABI_MISMATCH=1 (set by tools/ab.sh and tools/trace.sh for experiment builds
    from older trees): skip the ABI-version check and tolerate missing entry points."""
    return os.environ.get("JDAMD_ALLOW_ABI_MISMATCH") == "1"


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libjdamd.so (in-tree build).  Raises if it is absent: there is no fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("JDAMD_LIB") or LIB_PATH  # JDAMD_LIB: an experiment build
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} not built: run `make -C gpu-jpeg-decoder_amd` or __graft_entry__.build()")
    lib = ctypes.CDLL(p)
    c_void_p, c_int, c_size_t = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    sig = {
        "jd_ctx_create": (c_int, [ctypes.POINTER(c_void_p), c_int, ctypes.POINTER(_Opts)]),
        "jd_ctx_destroy": (c_int, [c_void_p]),
        "jd_parse": (c_int, [c_void_p, c_size_t, ctypes.POINTER(_Header)]),
        "jd_decode": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p, c_int, ctypes.POINTER(c_int),
                              ctypes.POINTER(c_int)]),
        "jd_decode_file": (c_int, [c_void_p, ctypes.c_char_p, c_void_p, c_size_t, c_int, ctypes.POINTER(c_int),
                                   ctypes.POINTER(c_int)]),
        "jd_decode_batch": (c_int, [c_void_p, ctypes.POINTER(_Item), c_int, ctypes.POINTER(_Result), c_int,
                                    c_void_p]),
        "jd_decode_batch_async": (c_int, [c_void_p, ctypes.POINTER(_Item), c_int, ctypes.POINTER(_Result), c_void_p]),
        "jd_decode_wait": (c_int, [c_void_p]),
        "jd_write_array": (c_int, [ctypes.c_char_p, c_void_p, c_int, c_int]),
        "jd_write_ppm": (c_int, [ctypes.c_char_p, c_void_p, c_int, c_int]),
        "jd_status_str": (ctypes.c_char_p, [c_int]),
        "jd_abi_version": (c_int, []),
        "jd_device_alloc": (c_int, [c_void_p, c_size_t, ctypes.POINTER(c_void_p)]),
        "jd_device_free": (c_int, [c_void_p, c_void_p]),
        "jd_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
        "jd_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
        "jd_synchronize": (c_int, [c_void_p]),
        "jd_get_stats": (c_int, [c_void_p, ctypes.POINTER(_Stats)]),
        "jd_reset_stats": (c_int, [c_void_p]),
        "jd_kernel_name": (ctypes.c_char_p, [c_int]),
        "jd_test_idct": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
        "jd_test_idct_exact": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
        "jd_test_color": (c_int, [c_void_p, c_void_p, c_void_p, c_int]),
        "jd_debug_fetch": (c_int, [c_void_p, c_int, c_void_p, c_size_t, ctypes.POINTER(c_size_t)]),
        "jd_ctx_last_error": (ctypes.c_char_p, [c_void_p]),
        "jd_device_bytes": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "jd_test_copy_peak": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, ctypes.POINTER(ctypes.c_double)]),
        "jd_host_register": (c_int, [c_void_p, c_void_p, c_size_t]),
        "jd_host_unregister": (c_int, [c_void_p, c_void_p]),
        "jd_host_alloc": (c_int, [c_void_p, c_size_t, ctypes.POINTER(c_void_p)]),
        "jd_host_free": (c_int, [c_void_p, c_void_p]),
    }
    # an A/B build from an older tree may lack newer entry points: tolerated only on explicit opt-in
    experiment = p != LIB_PATH and _abi_mismatch_allowed()
    for name, (res, args) in sig.items():
        if experiment and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def status_str(st: int) -> str:
    try:
        return load_library().jd_status_str(st).decode()
    except (OSError, FileNotFoundError):
        return f"status {st}"


@dataclass
class Header:
    width: int
    height: int
    ncomp: int
    h: List[int]
    v: List[int]
    tq: List[int]
    hmax: int
    vmax: int
    mcux: int
    mcuy: int
    blocks_per_mcu: int
    restart_interval: int
    subsampling: int
    ecs_offset: int


def parse(data: bytes) -> Header:
    """Header parse only (host).  Mirrors JPEGParser::extract() (cpp-decoder/src/parser.cpp:24-103)."""
    lib = load_library()
    h = _Header()
    st = lib.jd_parse(data, len(data), ctypes.byref(h))
    if st != JD_OK:
        raise JDError(st, "jd_parse")
    return Header(h.width, h.height, h.ncomp, list(h.h), list(h.v), list(h.tq), h.hmax, h.vmax, h.mcux, h.mcuy,
                  h.blocks_per_mcu, h.restart_interval, h.subsampling, h.ecs_offset)


def write_array(path: str, rgb: np.ndarray) -> None:
    """`.array` writer, byte-identical to JPEGParser::write() (cpp-decoder/src/parser.cpp:197-209)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    st = load_library().jd_write_array(path.encode(), rgb.ctypes.data, rgb.shape[1], rgb.shape[0])
    if st != JD_OK:
        raise JDError(st, "jd_write_array")


def write_ppm(path: str, rgb: np.ndarray) -> None:
    """Binary PPM (P6), the format of the reference's libjpeg comparison outputs
    (testing/jpeglib_output_ppm/, read by jpeglib-implementation/process_ppm.py)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    st = load_library().jd_write_ppm(path.encode(), rgb.ctypes.data, rgb.shape[1], rgb.shape[0])
    if st != JD_OK:
        raise JDError(st, "jd_write_ppm")


class DeviceBuffer:
    """A device allocation owned by a Decoder (for callers without their own allocator)."""

    def __init__(self, dec: "Decoder", nbytes: int):
        self.dec = dec
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        st = dec.lib.jd_device_alloc(dec.ctx, self.nbytes, ctypes.byref(p))
        if st != JD_OK:
            raise JDError(st, "jd_device_alloc")
        self.ptr = p.value

    def upload(self, arr: np.ndarray, offset: int = 0) -> None:
        a = np.ascontiguousarray(arr)
        assert offset + a.nbytes <= self.nbytes
        st = self.dec.lib.jd_memcpy_h2d(self.dec.ctx, self.ptr + offset, a.ctypes.data, a.nbytes)
        if st != JD_OK:
            raise JDError(st, "jd_memcpy_h2d")

    def download(self, out: np.ndarray, offset: int = 0) -> np.ndarray:
        assert out.flags["C_CONTIGUOUS"] and offset + out.nbytes <= self.nbytes
        st = self.dec.lib.jd_memcpy_d2h(self.dec.ctx, out.ctypes.data, self.ptr + offset, out.nbytes)
        if st != JD_OK:
            raise JDError(st, "jd_memcpy_d2h")
        return out

    def free(self) -> None:
        if self.ptr:
            self.dec.lib.jd_device_free(self.dec.ctx, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if self.ptr and self.dec.ctx:
                self.free()
        except Exception:
            pass


class Decoder:
    """One jd_ctx on one HIP device.  Mirrors the reference's allocate()/decode/clean() lifecycle
    (cuda-decoder/src/parser.cu:324-358, 577-700) as a context object."""

    def __init__(self, device: int = 0, timing: bool = False, parse_threads: int = 0, path: str = "auto",
                 fancy: bool = False, async_depth: int = 1, worst_case_pools: bool = False):
        """fancy=True: libjpeg's triangular chroma upsampling instead of replication
        (JD_FLAG_FANCY_UPSAMPLING; an option beyond the reference, see include/jd.h).
        async_depth=2: pipelined calls leave two batches in flight (JD_FLAG_ASYNC_DEPTH2).
        worst_case_pools=True: device pools sized for the densest stream the tables allow, so no
        image is ever decoded twice (JD_FLAG_WORST_CASE_POOLS; about twice the device memory)."""
        if async_depth not in (1, 2):
            raise ValueError("async_depth: 1 or 2")
        self.lib = load_library()
        abi = self.lib.jd_abi_version()
        if abi != JD_ABI_VERSION:
            if not _abi_mismatch_allowed():
                raise JDError(JD_ERR_INVALID_ARG, f"libjdamd ABI {abi} != {JD_ABI_VERSION}: rebuild")
            warnings.warn(f"libjdamd ABI {abi} != {JD_ABI_VERSION}: loaded anyway (JDAMD_ALLOW_ABI_MISMATCH=1)")
        self._arenas = {}  # pointer -> registered numpy arena (kept alive while registered)
        self.ctx = ctypes.c_void_p()
        opts = _Opts((JD_FLAG_TIMING if timing else 0) | PATHS[path] | (JD_FLAG_FANCY_UPSAMPLING if fancy else 0) |
                     (JD_FLAG_ASYNC_DEPTH2 if async_depth == 2 else 0) |
                     (JD_FLAG_WORST_CASE_POOLS if worst_case_pools else 0), parse_threads)
        st = self.lib.jd_ctx_create(ctypes.byref(self.ctx), device, ctypes.byref(opts))
        if st != JD_OK:
            raise JDError(st, "jd_ctx_create")

    def close(self) -> None:
        if self.ctx:
            self.lib.jd_ctx_destroy(self.ctx)  # unregisters the arenas still registered
            self.ctx = ctypes.c_void_p()
        self._arenas = {}

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- single image -----------------------------------------------------------------------
    def decode(self, data: bytes) -> np.ndarray:
        """decode(bitstream) -> RGB uint8 [H, W, 3]."""
        hdr = parse(data)
        out = np.empty((hdr.height, hdr.width, 3), np.uint8)
        w, h = ctypes.c_int(), ctypes.c_int()
        st = self.lib.jd_decode(self.ctx, data, len(data), out.ctypes.data, 0, ctypes.byref(w), ctypes.byref(h))
        if st != JD_OK:
            raise JDError(st, "jd_decode " + (self.last_error() if st == JD_ERR_HIP else ""))
        return out

    def decode_file(self, path: str) -> np.ndarray:
        w, h = ctypes.c_int(), ctypes.c_int()
        st = self.lib.jd_decode_file(self.ctx, path.encode(), None, 0, 0, ctypes.byref(w), ctypes.byref(h))
        if st != JD_OK:
            raise JDError(st, "jd_decode_file")
        out = np.empty((h.value, w.value, 3), np.uint8)
        st = self.lib.jd_decode_file(self.ctx, path.encode(), out.ctypes.data, out.nbytes, 0, ctypes.byref(w),
                                     ctypes.byref(h))
        if st != JD_OK:
            raise JDError(st, "jd_decode_file")
        return out

    # -- batches ----------------------------------------------------------------------------
    def decode_batch(self, datas: Sequence[bytes]):
        """Host in, host out.  Returns (list of arrays or None, list of status)."""
        n = len(datas)
        items = (_Item * n)()
        results = (_Result * n)()
        outs: List[Optional[np.ndarray]] = []
        keep = []
        for i, d in enumerate(datas):
            buf = ctypes.create_string_buffer(bytes(d), len(d))
            keep.append(buf)
            try:
                hdr = parse(d)
                o = np.empty((hdr.height, hdr.width, 3), np.uint8)
            except JDError:
                o = None
            outs.append(o)
            items[i] = _Item(ctypes.addressof(buf), None, len(d), o.ctypes.data if o is not None else None)
        st = self.lib.jd_decode_batch(self.ctx, items, n, results, 0, None)
        if st != JD_OK:
            raise JDError(st, "jd_decode_batch")
        status = [results[i].status for i in range(n)]
        return [o if s == JD_OK else None for o, s in zip(outs, status)], status

    def decode_batch_device(self, host_datas: Sequence[bytes], dev_ptrs: Sequence[int], rgb_ptrs: Sequence[int],
                            stream: Optional[int] = None, _keep=None):
        """Inputs already resident in HBM (dev_ptrs), outputs written to device rgb_ptrs.
        host_datas are the same bytes on the host (headers are parsed on the host)."""
        n = len(host_datas)
        items = (_Item * n)()
        results = (_Result * n)()
        for i in range(n):
            items[i] = _Item(_addr_of(host_datas[i]), dev_ptrs[i], len(host_datas[i]), rgb_ptrs[i])
        st = self.lib.jd_decode_batch(self.ctx, items, n, results, 1, stream)
        if st != JD_OK:
            raise JDError(st, "jd_decode_batch")
        return [results[i].status for i in range(n)]

    def make_batch(self, host_datas: Sequence, dev_ptrs: Sequence[int], rgb_ptrs: Sequence[int]):
        """Pre-builds the ctypes item array for repeated decode_prepared() calls (benchmarks)."""
        n = len(host_datas)
        items = (_Item * n)()
        for i in range(n):
            items[i] = _Item(_addr_of(host_datas[i]), dev_ptrs[i], len(host_datas[i]), rgb_ptrs[i])
        return items, (_Result * n)()

    def decode_prepared(self, batch, stream: Optional[int] = None, pipelined: bool = False) -> None:
        """Decode a make_batch() batch.  pipelined=True: jd_decode_batch_async (returns once the
        batch is launched and the previous one collected; call wait() after the last)."""
        items, results = batch
        if pipelined:
            st = self.lib.jd_decode_batch_async(self.ctx, items, len(items), results, stream)
        else:
            st = self.lib.jd_decode_batch(self.ctx, items, len(items), results, 1, stream)
        if st != JD_OK:
            raise JDError(st, "jd_decode_batch " + (self.last_error() if st == JD_ERR_HIP else ""))

    def wait(self) -> None:
        """Collect every pipelined batch (jd_decode_wait)."""
        st = self.lib.jd_decode_wait(self.ctx)
        if st != JD_OK:
            raise JDError(st, "jd_decode_wait " + (self.last_error() if st == JD_ERR_HIP else ""))

    def register_host(self, arena: np.ndarray) -> None:
        """jd_host_register: page-lock a caller-owned input arena (a contiguous numpy array) so that
        batch items whose bytes lie in it are uploaded straight from it (no staging copy).  The
        arena must stay unchanged while batches reading it are in flight; the Decoder keeps a
        reference to it until unregister_host() or close(), so it cannot be freed while registered."""
        if not isinstance(arena, np.ndarray) or not arena.flags["C_CONTIGUOUS"]:
            raise JDError(JD_ERR_INVALID_ARG, "jd_host_register: the arena must be a C-contiguous numpy array")
        st = self.lib.jd_host_register(self.ctx, arena.ctypes.data, arena.nbytes)
        if st != JD_OK:
            raise JDError(st, "jd_host_register " + (self.last_error() if st == JD_ERR_HIP else ""))
        self._arenas[arena.ctypes.data] = arena

    def unregister_host(self, arena: np.ndarray) -> None:
        """jd_host_unregister (waits for the context's in-flight batches first)."""
        st = self.lib.jd_host_unregister(self.ctx, arena.ctypes.data)
        if st != JD_OK:
            raise JDError(st, "jd_host_unregister " + (self.last_error() if st == JD_ERR_HIP else ""))
        self._arenas.pop(arena.ctypes.data, None)

    def host_alloc(self, nbytes: int) -> np.ndarray:
        """jd_host_alloc: a pinned input arena (hipHostMalloc) owned by the context, as a numpy
        uint8 array; batch items whose bytes lie in it are uploaded straight from it.  Free it with
        host_free() (or let close() do it); the array must not be used afterwards."""
        p = ctypes.c_void_p()
        st = self.lib.jd_host_alloc(self.ctx, nbytes, ctypes.byref(p))
        if st != JD_OK:
            raise JDError(st, "jd_host_alloc " + (self.last_error() if st == JD_ERR_HIP else ""))
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))

    def host_free(self, arena: np.ndarray) -> None:
        st = self.lib.jd_host_free(self.ctx, arena.ctypes.data)
        if st != JD_OK:
            raise JDError(st, "jd_host_free")

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def synchronize(self) -> None:
        st = self.lib.jd_synchronize(self.ctx)
        if st != JD_OK:
            raise JDError(st, "jd_synchronize")

    # -- stats / test hooks -----------------------------------------------------------------
    def stats(self) -> dict:
        s = _Stats()
        self.lib.jd_get_stats(self.ctx, ctypes.byref(s))
        return {
            "kernels": {KERNEL_NAMES[k]: {"launches": s.launches[k], "total_ms": s.total_ms[k], "bytes": s.bytes[k]}
                        for k in range(JD_NUM_KERNELS)},
            "batches": s.batches, "images": s.images, "pixels": s.pixels, "ecs_bytes": s.ecs_bytes,
            "blocks": s.blocks, "segments": s.segments, "subsequences": s.subsequences,
            "host_ms": {"parse": s.host_ms[0], "plan": s.host_ms[1], "stage_inputs": s.host_ms[2],
                        "wait": s.host_ms[3]},
            "h2d_bytes": s.h2d_bytes, "h2d_registered_bytes": s.h2d_registered_bytes,
            # speculative decode: k_redo's re-walks; intervals k_chain_fix / k_chain_big fixed, their
            # rounds, re-walked pieces, early stops
            "redo_pieces": s.redo_pieces, "fix_intervals": s.fix_intervals, "fix_rounds": s.fix_rounds,
            "fix_rewalks": s.fix_rewalks, "fix_early": s.fix_early,
            # images decoded again with worst-case pools after overflowing an optimistic one
            "retried_images": s.retried_images,
        }

    def device_bytes(self):
        """(bytes the context's device pools hold now, their high-water mark)."""
        cur, peak = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.jd_device_bytes(self.ctx, ctypes.byref(cur), ctypes.byref(peak))
        return cur.value, peak.value

    def last_error(self) -> str:
        return (self.lib.jd_ctx_last_error(self.ctx) or b"").decode()

    def reset_stats(self) -> None:
        self.lib.jd_reset_stats(self.ctx)

    DEBUG_ARRAYS = {"blocks": (0, np.uint32, 2), "seg_cstart": (1, np.uint32, 1), "seg_cend": (2, np.uint32, 1),
                    "seg_sub_base": (3, np.uint32, 1), "seg_nsub": (4, np.uint32, 1), "piece_bit": (5, np.uint32, 1),
                    "piece_end": (6, np.uint32, 1), "piece_nmcu": (7, np.uint32, 1), "piece_nent": (8, np.uint32, 1),
                    "sub_seg": (9, np.uint32, 1), "status": (10, np.uint32, 1), "entries": (11, np.uint32, 1),
                    "piece_mcu0": (12, np.uint32, 1), "piece_abase": (13, np.uint32, 1),
                    "piece_cp": (14, np.uint32, 36), "stamps": (15, np.uint64, 8), "piece_emcu": (16, np.uint32, 1),
                    "piece_amcu": (17, np.uint32, 1), "piece_join": (18, np.uint32, 1), "seg_ent": (19, np.uint32, 1),
                    "entry_base": (20, np.uint64, 1), "rw_div": (21, np.uint32, 1),
                    "rw_slack": (22, np.uint32, 1)}

    def debug_fetch(self, name: str) -> np.ndarray:
        """Internal array of the most recent batch (white-box tests and debugging)."""
        what, dt, width = self.DEBUG_ARRAYS[name]
        n = ctypes.c_size_t()
        st = self.lib.jd_debug_fetch(self.ctx, what, None, 0, ctypes.byref(n))
        if st != JD_OK:
            raise JDError(st, "jd_debug_fetch " + self.last_error())
        out = np.empty(n.value // np.dtype(dt).itemsize, dt)
        st = self.lib.jd_debug_fetch(self.ctx, what, out.ctypes.data, out.nbytes, ctypes.byref(n))
        if st != JD_OK:
            raise JDError(st, "jd_debug_fetch " + self.last_error())
        return out.reshape(-1, width) if width > 1 else out

    def test_idct(self, zz_dequant: np.ndarray, exact_only: bool = False) -> np.ndarray:
        """The device IDCT on dequantised zig-zag blocks: the decode path's per-block choice of form,
        or (exact_only) the exact form whatever the inputs."""
        a = np.ascontiguousarray(zz_dequant, dtype=np.int32).reshape(-1, 64)
        n = a.shape[0]
        din, dout = self.alloc(a.nbytes), self.alloc(a.nbytes)
        din.upload(a)
        fn = self.lib.jd_test_idct_exact if exact_only else self.lib.jd_test_idct
        st = fn(self.ctx, din.ptr, dout.ptr, n)
        if st != JD_OK:
            raise JDError(st, "jd_test_idct")
        out = dout.download(np.empty((n, 64), np.int32))
        din.free()
        dout.free()
        return out

    def copy_peak(self, src_ptr: int, dst_ptr: int, nbytes: int, reps: int = 5) -> float:
        """HBM copy peak in GB/s (read + write bytes): the library's 16-byte-per-lane copy kernel
        over caller device buffers (jd_test_copy_peak)."""
        g = ctypes.c_double()
        st = self.lib.jd_test_copy_peak(self.ctx, src_ptr, dst_ptr, nbytes, reps, ctypes.byref(g))
        if st != JD_OK:
            raise JDError(st, "jd_test_copy_peak " + self.last_error())
        return g.value

    def test_color(self, ycc: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(ycc, dtype=np.int32).reshape(-1, 3)
        n = a.shape[0]
        din, dout = self.alloc(a.nbytes), self.alloc(n * 3)
        din.upload(a)
        st = self.lib.jd_test_color(self.ctx, din.ptr, dout.ptr, n)
        if st != JD_OK:
            raise JDError(st, "jd_test_color")
        out = dout.download(np.empty((n, 3), np.uint8))
        din.free()
        dout.free()
        return out


def _addr_of(b) -> int:
    """Address of a bytes-like object's buffer (numpy array or ctypes buffer)."""
    if isinstance(b, np.ndarray):
        return b.ctypes.data
    if isinstance(b, ctypes.Array):
        return ctypes.addressof(b)
    raise TypeError("pass numpy uint8 arrays or ctypes buffers for zero-copy batch items")
