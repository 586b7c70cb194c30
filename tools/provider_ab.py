#!/usr/bin/env python3
"""Per-call latency of the scalar provider hook for two or more builds of the
library in one process, interleaved (tooling only).
usage: provider_ab.py LIB_A LIB_B [...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import load  # noqa: E402

libs = [load(p) for p in sys.argv[1:]]
for l in libs:
    assert l.val_gpu_init(0) == 0
for L in (16, 1024, 16400, 65543, 1 << 20):
    data = np.random.default_rng(L).integers(0, 256, L, dtype=np.uint8)
    reps = 300 if L <= 65543 else 30
    res = [[] for _ in libs]
    outs = []
    for rep in range(3):
        for i, l in enumerate(libs):
            vc._lib = l
            outs.append(vc.crc32_provider(0xFFFFFFFF, data))
            t0 = time.perf_counter()
            for _ in range(reps):
                vc.crc32_provider(0xFFFFFFFF, data)
            res[i].append((time.perf_counter() - t0) / reps * 1e6)
    line = f"provider L={L:8d}:"
    for i in range(len(libs)):
        line += f"  {chr(65 + i)} {np.median(res[i]):7.1f} us"
    print(line, " same:", len(set(outs)) == 1, flush=True)
