#!/usr/bin/env python3
"""A/B of region (K4) builds: interleaved GPU-event timing of back-to-back
val_crc32_region_dev calls per window size (tooling only; diagnostic builds
may return wrong CRCs). Each size cycles over distinct windows spanning at
least 1 GiB (or 128 windows for sizes under 1 MiB), as bench.py's verify
windows do, so calls read from HBM, not from the 256 MiB Infinity Cache; the
registers of every library are compared on the first window.
usage: ab_region.py LIB... [SIZE...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402

libs = []
sizes = [int(a) for a in sys.argv[1:] if not a.endswith(".so")] or [256 << 10, 1 << 20, 8 << 20, 64 << 20, 256 << 20]
for path in [a for a in sys.argv[1:] if a.endswith(".so")]:
    l = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    vc._declare(l, strict=False)
    assert l.val_gpu_init(0) == 0
    libs.append((os.path.basename(path), l))
dev = torch.device("cuda:0")
span = max(1 << 30, max(sizes))
big = torch.randint(0, 256, (span,), dtype=torch.uint8, device=dev)
out = torch.empty(1, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
for size in sizes:
    if size >= (1 << 20):
        starts = [j * size for j in range(max(1, span // size))]
    else:
        gap = max(size, (span - size) // 128)
        starts = [j * gap for j in range(128)]
    calls = max(len(starts), 64 if size >= (64 << 20) else 200)
    res = {n: [] for n, _ in libs}
    regs = {}
    for rep in range(5):
        for name, l in libs:
            call = lambda o: l.val_crc32_region_dev(ctypes.c_void_p(big.data_ptr() + o), size, 0xFFFFFFFF,  # noqa: E731
                                                    ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s.cuda_stream))
            if rep == 0:
                call(starts[0])
                torch.cuda.synchronize()
                regs[name] = int(out.item()) & 0xFFFFFFFF
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for k in range(calls):
                call(starts[k % len(starts)])
            b.record(s)
            torch.cuda.synchronize()
            res[name].append(a.elapsed_time(b) * 1e3 / calls)  # us per call
    same = len(set(regs.values())) == 1
    print(size, {n: round(sorted(v)[2], 2) for n, v in res.items()}, "same" if same else f"DIFFER {regs}", flush=True)
