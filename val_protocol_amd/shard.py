"""Multi-GPU sharding of the CRC path.

Frames are independent, so a batch is split into contiguous frame ranges, one
per rank, balanced by CRC-input bytes; each rank hashes its slice on its own
GPU and writes a disjoint range of the output. No collective touches the data
path. A long verify window is split into byte ranges whose raw partial states
fold on the host with the GF(2) combine (val_crc32_fold_partials).
Both the split and the fold are the product's C host code (libval_crc_hip.so).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np


def shard_frames(n: int, world: int, rank: int, lengths: Optional[np.ndarray] = None) -> Tuple[int, int]:
    """[start, start+count) of the frames rank `rank` owns: the product's
    val_shard_frames (the split its *_host_multi calls use)."""
    import ctypes

    from .crc import lib

    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    ln = None
    if lengths is not None:
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        if ln.size != n:
            raise ValueError("lengths must have n entries")
    s, c = ctypes.c_uint32(0), ctypes.c_uint32(0)
    lib().val_shard_frames(n, ln.ctypes.data if ln is not None else None, world, rank, ctypes.byref(s), ctypes.byref(c))
    return int(s.value), int(c.value)


def shard_region(length: int, world: int, rank: int, align: int = 4096) -> Tuple[int, int]:
    """Byte range [start, start+count) of a long window for rank `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per = -(-length // world)
    per = -(-per // align) * align
    start = min(rank * per, length)
    return start, min(per, length - start)


def fold_partials(parts: Sequence[Tuple[int, int]]) -> int:
    """Fold raw register partials [(state_r, len_r)] in rank order into one
    with the product's val_crc32_fold_partials. Rank 0's partial carries the
    initial register; the others start from 0."""
    from .crc import lib

    st = np.array([p[0] for p in parts], dtype=np.uint32)
    nb = np.array([p[1] for p in parts], dtype=np.uint64)
    return int(lib().val_crc32_fold_partials(st.ctypes.data, nb.ctypes.data, st.size))


__all__: List[str] = ["shard_frames", "shard_region", "fold_partials"]
