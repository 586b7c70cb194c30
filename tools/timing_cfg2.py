#!/usr/bin/env python3
"""Per-wave timeline of one frames launch from a -DVCRC_TIMING build
(tools/build_rev.sh WT build/libval_T.so -DVCRC_TIMING): start, after the LDS
prologue, end (s_memrealtime, 100 MHz). usage: timing_cfg2.py LIB [workload G]."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import load, workload  # noqa: E402

vc._lib = load(sys.argv[1])
vc._lib.vcrc_debug_times.argtypes = [ctypes.c_void_p]
vc._lib.vcrc_debug_times.restype = ctypes.c_int
name = sys.argv[2] if len(sys.argv) > 2 else "cfg2"
G = int(sys.argv[3]) if len(sys.argv) > 3 else 0
dev = torch.device("cuda:0")
vc.init(0)
w, nbytes = workload(name, dev)
out = torch.empty(w.get("n") or w["length"].numel(), dtype=torch.int32, device=dev)
vc.set_geometry(G)
buf = np.zeros(4096 * 4, np.uint64)
for rep in range(4):
    if "off" in w:
        vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out, len_hint=w["len_hint"])
    else:
        vc.frames(w["buf"], stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out)
    torch.cuda.synchronize()
    assert vc._lib.vcrc_debug_times(buf.ctypes.data) == 0
t = buf.reshape(4096, 4)[:, :3].astype(np.int64)
used = (t[:, 0] > 0) & (t[:, 2] > 0)
t = t[used]
t0 = t[:, 0].min()
us = (t - t0) / 100.0  # 100 MHz -> us
pct = lambda a: " ".join(f"{np.percentile(a, q):6.2f}" for q in (0, 10, 50, 90, 100))
print(f"{name} G={G or 'auto'} waves={used.sum()}  (percentiles 0/10/50/90/100, us from first wave start)")
print("  start     ", pct(us[:, 0]))
print("  prologue  ", pct(us[:, 1]))
print("  end       ", pct(us[:, 2]))
print("  prologue dur", pct(us[:, 1] - us[:, 0]), " hash dur", pct(us[:, 2] - us[:, 1]))
# where the late waves are: by XCD (block % 8), by wave slot in the block
blk = np.nonzero(used)[0] // 16
end = us[:, 2]
print("  end by blockIdx%8 (median us):", " ".join(f"{np.median(end[blk % 8 == x]):7.1f}" for x in range(8)))
print("  start by blockIdx%8 (median us):", " ".join(f"{np.median(us[blk % 8 == x, 0]):7.2f}" for x in range(8)))
print("  prologue end by blockIdx%8 (median us):", " ".join(f"{np.median(us[blk % 8 == x, 1]):7.2f}" for x in range(8)))
print("  start by block (first 16 blocks, us):", " ".join(f"{us[blk == b, 0].min():5.2f}" for b in range(16)))
slot = np.nonzero(used)[0] % 16
print("  end by wave slot (median us):  ", " ".join(f"{np.median(end[slot == k]):6.0f}" for k in range(16)))
per_block = np.array([end[blk == b].max() for b in np.unique(blk)])
print("  per-block max end percentiles:", pct(per_block))
print("  within-block spread (max-min) median:", np.median([end[blk == b].max() - end[blk == b].min() for b in np.unique(blk)]))
