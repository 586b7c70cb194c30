"""numpy restatement of oracle/prng.h (TEST INFRASTRUCTURE) plus synthetic
DATA-frame streams shaped like the reference sender's output
(type 5, flags OFFSET_PRESENT, LE16 content_len, type_data 0, LE64 offset,
payload, LE32 trailer; src/val_core.c:733-834)."""
from __future__ import annotations

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, k: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (k.astype(np.uint64) + np.uint64(1)) * _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def prng_bytes(seed: int, n: int) -> np.ndarray:
    words = (n + 7) // 8
    z = splitmix64(seed, np.arange(words, dtype=np.uint64))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def data_header(content_len: int, explicit: bool = True) -> np.ndarray:
    h = np.zeros(8, dtype=np.uint8)
    h[0] = 5
    h[1] = 1 if explicit else 0
    h[2] = content_len & 0xFF
    h[3] = (content_len >> 8) & 0xFF
    return h


def frames_stream(n: int, payload: int, stride_pad: int = 0, seed: int = 0x56414C00, explicit: bool = True):
    """n DATA frames of `payload` bytes back to back (plus stride_pad bytes of
    zeros after each trailer). Trailers are left zero."""
    content = payload + (8 if explicit else 0)
    flen = 8 + content
    stride = flen + 4 + stride_pad
    buf = np.zeros((n, stride), dtype=np.uint8)
    buf[:, :8] = data_header(content, explicit)
    col = 8
    if explicit:
        offs = (np.arange(n, dtype=np.uint64) * np.uint64(payload)).astype("<u8")
        buf[:, 8:16] = offs.view(np.uint8).reshape(n, 8)
        col = 16
    buf[:, col:col + payload] = prng_bytes(seed, n * payload).reshape(n, payload)
    return buf.reshape(-1)
