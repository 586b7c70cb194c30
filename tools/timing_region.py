#!/usr/bin/env python3
"""Per-wave timeline of one k_region launch from a -DVCRC_TIMING build:
stamps 0 start, 1 frame loads issued (prologue writes begin), 2 after the
prologue barrier, 3 after the chunk hash. usage: timing_region.py LIB BYTES..."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import load  # noqa: E402

vc._lib = load(sys.argv[1])
vc._lib.vcrc_debug_times.argtypes = [ctypes.c_void_p]
vc._lib.vcrc_debug_times.restype = ctypes.c_int
vc.init(0)
dev = torch.device("cuda:0")
sizes = [int(x) for x in sys.argv[2:]]
big = torch.randint(0, 256, (max(sizes),), dtype=torch.uint8, device=dev)
for size in sizes:
    buf = np.zeros(4096 * 4, np.uint64)
    for rep in range(3):
        vc._lib.vcrc_debug_times(buf.ctypes.data)  # (reset not needed: stamps overwrite)
        vc.region(big[:size])
        torch.cuda.synchronize()
    assert vc._lib.vcrc_debug_times(buf.ctypes.data) == 0
    t = buf.reshape(4096, 4).astype(np.int64)
    k = 12
    while (4096 << k) < size:
        k += 1
    nwg = -(-(-(-size // (1 << k))) // 16)
    used = (np.arange(4096) < nwg * 16) & (t[:, 0] > 0)
    nw = int(used.sum())
    t0 = t[used, 0].min()
    us = (t - t0) / 100.0
    pct = lambda a: " ".join(f"{np.percentile(a, q):6.2f}" for q in (0, 50, 100))
    print(f"region {size} B: waves stamped {nw}")
    for k, name in enumerate(("start", "issued", "barrier", "hashed")):
        print(f"  {name:9s}", pct(us[used, k]))
    hashed = us[used, 3]
    print("  hashed percentiles 10/25/75/90:", " ".join(f"{np.percentile(hashed, q):6.2f}" for q in (10, 25, 75, 90)))
