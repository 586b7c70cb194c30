"""ctypes binding of oracle/liboracle.so (TEST INFRASTRUCTURE: the checker,
never the thing measured or shipped). Builds it on first use if missing."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_SO = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True)
        l = ctypes.CDLL(_SO)
        vp, u32, u64, sz, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int
        for name, res, args in [
            ("oracle_crc32", u32, [vp, sz]),
            ("oracle_crc32_update_state", u32, [u32, vp, sz]),
            ("oracle_crc32_provider", u32, [u32, vp, sz]),
            ("oracle_crc32_shift", u32, [u32, u64]),
            ("oracle_crc32_combine", u32, [u32, u32, u64]),
            ("oracle_build_data_frame", sz, [vp, u32, u64, i32, vp, sz]),
            ("oracle_crc32_frames", None, [vp, vp, vp, u64, vp, vp, i32]),
            ("oracle_crc32_frames_strided", None, [vp, u64, u32, u64, vp, vp, i32]),
            ("oracle_verify_frames", u64, [vp, vp, vp, u64, vp, i32]),
        ]:
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def _arr(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)


def crc32(data) -> int:
    a = _arr(data)
    return int(lib().oracle_crc32(a.ctypes.data, a.size))


def update_state(state: int, data) -> int:
    a = _arr(data)
    return int(lib().oracle_crc32_update_state(state & 0xFFFFFFFF, a.ctypes.data, a.size))


def provider(seed: int, data) -> int:
    a = _arr(data)
    return int(lib().oracle_crc32_provider(seed & 0xFFFFFFFF, a.ctypes.data, a.size))


def shift(state: int, nbytes: int) -> int:
    return int(lib().oracle_crc32_shift(state & 0xFFFFFFFF, nbytes))


def combine(a: int, b: int, len_b: int) -> int:
    return int(lib().oracle_crc32_combine(a & 0xFFFFFFFF, b & 0xFFFFFFFF, len_b))


def build_data_frame(payload, offset: int, include_offset: bool) -> bytes:
    p = _arr(payload)
    out = np.zeros(p.size + 8 + 8 + 4 + 16, dtype=np.uint8)
    w = lib().oracle_build_data_frame(p.ctypes.data if p.size else None, p.size, offset, int(include_offset),
                                      out.ctypes.data, out.size)
    return bytes(out[:w])


def frames(base, off, length, header=False, nthreads=1):
    base = _arr(base)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    n = off.size
    crc = np.zeros(n, dtype=np.uint32)
    hdr = np.zeros(n, dtype=np.uint32) if header else None
    lib().oracle_crc32_frames(base.ctypes.data, off.ctypes.data, length.ctypes.data, n, crc.ctypes.data,
                              hdr.ctypes.data if header else None, nthreads)
    return (crc, hdr) if header else crc


def frames_strided(base, stride: int, flen: int, n: int, header=False, nthreads=1):
    base = _arr(base)
    crc = np.zeros(n, dtype=np.uint32)
    hdr = np.zeros(n, dtype=np.uint32) if header else None
    lib().oracle_crc32_frames_strided(base.ctypes.data, stride, flen, n, crc.ctypes.data,
                                      hdr.ctypes.data if header else None, nthreads)
    return (crc, hdr) if header else crc


def verify_frames(base, off, length, nthreads=1):
    base = _arr(base)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    ok = np.zeros(off.size, dtype=np.uint8)
    bad = lib().oracle_verify_frames(base.ctypes.data, off.ctypes.data, length.ctypes.data, off.size,
                                     ok.ctypes.data, nthreads)
    return ok, int(bad)
