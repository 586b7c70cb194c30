"""Host framing helpers (C implementation in csrc/val_wire.c).

``build_data_batch`` lays out a window of DATA frames the way the reference
sender emits them one by one (src/val_core.c:733-834); ``scan_frames`` walks a
received byte stream into descriptors for batch verify
(src/val_core.c:893-921).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .crc import ValError, _check, lib

HEADER = 8
TRAILER = 4
VAL_PKT_DATA = 5
VAL_DATA_OFFSET_PRESENT = 1


def serialize_header(ptype: int, flags: int, content_len: int, type_data: int) -> bytes:
    out = (ctypes.c_uint8 * 8)()
    lib().val_serialize_frame_header(ptype, flags, content_len, type_data, out)
    return bytes(out)


def deserialize_header(hdr: bytes):
    buf = (ctypes.c_uint8 * 8).from_buffer_copy(hdr[:8])
    t, f = ctypes.c_uint8(), ctypes.c_uint8()
    cl, td = ctypes.c_uint16(), ctypes.c_uint32()
    lib().val_deserialize_frame_header(buf, ctypes.byref(t), ctypes.byref(f), ctypes.byref(cl), ctypes.byref(td))
    return t.value, f.value, cl.value, td.value


def build_data_batch(payload: np.ndarray, pay_off, pay_len, file_off, include_offset=None):
    """Returns (stream uint8, frame_off uint64, crc_len uint32); trailers zero."""
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    pay_off = np.ascontiguousarray(pay_off, dtype=np.uint64)
    pay_len = np.ascontiguousarray(pay_len, dtype=np.uint32)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
    n = pay_len.size
    inc = None
    if include_offset is not None:
        inc = np.ascontiguousarray(include_offset, dtype=np.uint8)
    cap = int(pay_len.sum()) + n * (HEADER + 8 + TRAILER)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    frame_off = np.zeros(n, dtype=np.uint64)
    crc_len = np.zeros(n, dtype=np.uint32)
    used = ctypes.c_size_t(0)
    st = lib().val_frame_data_batch(payload.ctypes.data if payload.size else None, pay_off.ctypes.data,
                                    pay_len.ctypes.data, file_off.ctypes.data,
                                    inc.ctypes.data if inc is not None else None, n, out.ctypes.data, out.size,
                                    frame_off.ctypes.data, crc_len.ctypes.data, ctypes.byref(used))
    _check(st, "val_frame_data_batch")
    return out[: used.value], frame_off, crc_len


def put_trailers(stream: np.ndarray, frame_off, crc_len, crc) -> None:
    frame_off = np.ascontiguousarray(frame_off, dtype=np.uint64)
    crc_len = np.ascontiguousarray(crc_len, dtype=np.uint32)
    crc = np.ascontiguousarray(crc, dtype=np.uint32)
    lib().val_frame_put_trailers(stream.ctypes.data, frame_off.ctypes.data, crc_len.ctypes.data, crc.ctypes.data,
                                 crc.size)


def scan_frames(stream: np.ndarray, mtu: int, max_frames: int = 1 << 30):
    """Returns (status, frame_off, crc_len, consumed)."""
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    cap = min(max_frames, stream.size // (HEADER + TRAILER) + 1)
    frame_off = np.zeros(cap, dtype=np.uint64)
    crc_len = np.zeros(cap, dtype=np.uint32)
    nf = ctypes.c_uint32(0)
    used = ctypes.c_size_t(0)
    st = lib().val_frame_scan(stream.ctypes.data, stream.size, mtu, cap, frame_off.ctypes.data, crc_len.ctypes.data,
                              ctypes.byref(nf), ctypes.byref(used))
    return st, frame_off[: nf.value], crc_len[: nf.value], used.value


def payload_lens(stream: np.ndarray, frame_off, crc_len) -> np.ndarray:
    """Payload bytes of each frame (val_frame_payload_lens)."""
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    frame_off = np.ascontiguousarray(frame_off, dtype=np.uint64)
    crc_len = np.ascontiguousarray(crc_len, dtype=np.uint32)
    out = np.zeros(crc_len.size, dtype=np.uint32)
    lib().val_frame_payload_lens(stream.ctypes.data, frame_off.ctypes.data, crc_len.ctypes.data, crc_len.size,
                                 out.ctypes.data)
    return out


# val_frame_data_offsets sentinels (val_wire.h)
OFFSET_IMPLIED = (1 << 64) - 1
OFFSET_NOT_DATA = (1 << 64) - 2


def data_offsets(stream: np.ndarray, frame_off, crc_len) -> np.ndarray:
    """File offset of each frame as the receiver reads it (val_frame_data_offsets):
    explicit offset, OFFSET_IMPLIED or OFFSET_NOT_DATA."""
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    frame_off = np.ascontiguousarray(frame_off, dtype=np.uint64)
    crc_len = np.ascontiguousarray(crc_len, dtype=np.uint32)
    out = np.zeros(crc_len.size, dtype=np.uint64)
    lib().val_frame_data_offsets(stream.ctypes.data, frame_off.ctypes.data, crc_len.ctypes.data, crc_len.size,
                                 out.ctypes.data)
    return out


__all__ = ["serialize_header", "deserialize_header", "build_data_batch", "put_trailers", "scan_frames", "payload_lens",
           "data_offsets", "OFFSET_IMPLIED", "OFFSET_NOT_DATA", "ValError"]
