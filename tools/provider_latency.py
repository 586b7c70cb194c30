#!/usr/bin/env python3
"""Per-call latency of the scalar hooks (val_gpu_crc32_provider) by size,
host memory in, finished CRC out (diagnostic)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402

vc.init(0)
for L in (16, 1024, 16400, 65543, 1 << 20, 8 << 20):
    data = np.random.default_rng(L).integers(0, 256, L, dtype=np.uint8)
    vc.crc32_provider(0xFFFFFFFF, data)
    reps = 300 if L <= 65543 else 30
    t0 = time.perf_counter()
    for _ in range(reps):
        vc.crc32_provider(0xFFFFFFFF, data)
    us = (time.perf_counter() - t0) / reps * 1e6
    print(f"provider L={L:8d}: {us:8.1f} us/call  {L / us / 1e3:8.2f} GB/s", flush=True)
