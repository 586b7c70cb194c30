#!/usr/bin/env python3
"""Tail of a ragged launch from a -DVCRC_TIMING build: for each wave, the end
time and the start, class and frame length of its last item (tooling only).
usage: timing_ragged_tail.py LIB [workload]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import load, workload  # noqa: E402

vc._lib = load(sys.argv[1])
for fn in ("vcrc_debug_times", "vcrc_debug_info"):
    getattr(vc._lib, fn).argtypes = [ctypes.c_void_p]
    getattr(vc._lib, fn).restype = ctypes.c_int
name = sys.argv[2] if len(sys.argv) > 2 else "cfg5log"
dev = torch.device("cuda:0")
vc.init(0)
w, nbytes = workload(name, dev)
out = torch.empty(w["length"].numel(), dtype=torch.int32, device=dev)
t = np.zeros(4096 * 4, np.uint64)
info = np.zeros(4096, np.uint32)
for rep in range(4):
    vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out, len_hint=w["len_hint"])
    torch.cuda.synchronize()
    assert vc._lib.vcrc_debug_times(t.ctypes.data) == 0 and vc._lib.vcrc_debug_info(info.ctypes.data) == 0
t = t.reshape(4096, 4).astype(np.int64)
used = (t[:, 0] > 0) & (t[:, 2] > 0) & (t[:, 3] > 0)
t0 = t[used, 0].min()
us = (t[used] - t0) / 100.0
end, last = us[:, 2], us[:, 3]
cls, L = info[used] >> 16, (info[used] & 0xFFFF) * 64
order = np.argsort(end)
pct = lambda a: " ".join(f"{np.percentile(a, q):7.1f}" for q in (0, 10, 50, 90, 100))
print(f"{name}: waves={used.sum()} end {pct(end)}")
print("  last-item duration", pct(end - last))
print("  prologue (LDS fill) end", pct(us[:, 1]))
for c in range(4):
    m = cls == c
    if m.any():
        print(f"  last item class {c}: waves {m.sum():5d}  end {pct(end[m])}  dur {pct(end[m] - last[m])}  L~{pct(L[m])}")
print("  the 40 latest waves (end, last start, class, L, slot):")
for i in order[-40:]:
    wv = np.nonzero(used)[0][i]
    print(f"    {end[i]:7.1f} {last[i]:7.1f} c{cls[i]} L~{L[i]:6d} slot {wv % 16:2d} blk%8 {(wv // 16) % 8}")
