#!/usr/bin/env python3
"""A/B of region (K4) builds: interleaved GPU-event timing of back-to-back
val_crc32_region_dev calls per window size (tooling only; diagnostic builds
may return wrong CRCs). usage: ab_region.py LIB... """
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402

libs = []
for path in sys.argv[1:]:
    l = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    vc._declare(l, strict=False)
    assert l.val_gpu_init(0) == 0
    libs.append((os.path.basename(path), l))
dev = torch.device("cuda:0")
big = torch.randint(0, 256, (64 << 20,), dtype=torch.uint8, device=dev)
out = torch.empty(1, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
for size in (256 << 10, 1 << 20, 8 << 20, 64 << 20):
    res = {n: [] for n, _ in libs}
    for rep in range(5):
        for name, l in libs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(100):
                l.val_crc32_region_dev(ctypes.c_void_p(big.data_ptr()), size, 0xFFFFFFFF,
                                       ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s.cuda_stream))
            b.record(s)
            torch.cuda.synchronize()
            res[name].append(a.elapsed_time(b) * 10.0)  # us per call
    print(size, {n: round(sorted(v)[2], 2) for n, v in res.items()}, flush=True)
