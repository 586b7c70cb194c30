"""Multi-GPU sharding of the CRC path.

Frames are independent, so a batch is split into contiguous frame ranges, one
per rank, balanced by CRC-input bytes; each rank hashes its slice on its own
GPU and writes a disjoint range of the output. No collective touches the data
path. A long verify window is split into byte ranges whose raw partial states
fold on the host with the GF(2) combine (val_crc32_shift).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np


def shard_frames(n: int, world: int, rank: int, lengths: Optional[np.ndarray] = None) -> Tuple[int, int]:
    """[start, start+count) of the frames rank `rank` owns."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    if lengths is None:
        base, extra = divmod(n, world)
        start = rank * base + min(rank, extra)
        return start, base + (1 if rank < extra else 0)
    lengths = np.asarray(lengths, dtype=np.uint64)
    if lengths.size != n:
        raise ValueError("lengths must have n entries")
    csum = np.concatenate([[0], np.cumsum(lengths, dtype=np.uint64)])
    total = int(csum[-1])
    cuts = [int(np.searchsorted(csum, (total * r) // world, side="left")) for r in range(world + 1)]
    cuts[0], cuts[-1] = 0, n
    for i in range(1, world + 1):
        cuts[i] = max(cuts[i], cuts[i - 1])
    return cuts[rank], cuts[rank + 1] - cuts[rank]


def shard_region(length: int, world: int, rank: int, align: int = 4096) -> Tuple[int, int]:
    """Byte range [start, start+count) of a long window for rank `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    per = -(-length // world)
    per = -(-per // align) * align
    start = min(rank * per, length)
    return start, min(per, length - start)


def fold_partials(parts: Sequence[Tuple[int, int]], shift) -> int:
    """Fold raw register partials [(state_r, len_r)] in rank order into one.

    Rank 0's partial carries the initial register; the others start from 0.
    ``shift(state, nbytes)`` is the GF(2) advance (val_crc32_shift).
    """
    acc = 0
    for state, nbytes in parts:
        acc = shift(acc, nbytes) ^ state
    return acc


__all__: List[str] = ["shard_frames", "shard_region", "fold_partials"]
