#!/usr/bin/env python3
"""Profiling target for the ragged path.
usage: prof_ragged.py MODE [LIB]   MODE: strided57 | ragged57 | mix3 | mix3aligned
LIB: optional other build of libval_crc_hip.so (A/B under the profiler)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda:0")
if len(sys.argv) > 2:
    from tools.ab_libs import load  # noqa: E402

    vc._lib = load(sys.argv[2])
vc.init(0)
rng = np.random.default_rng(1)
if mode in ("strided57", "ragged57"):
    lens = np.full(56508, 57000, np.int64)
elif mode == "mix3":
    lens = np.exp(rng.uniform(np.log(49152), np.log(65532), 60000)).astype(np.int64)
else:  # mix3aligned: same lengths rounded to a multiple of 16 (all frame starts 16-B aligned incl. 4-B trailer gap)
    lens = (np.exp(rng.uniform(np.log(49152), np.log(65532), 60000)).astype(np.int64) // 16) * 16 + 12
wire = lens + 4
off = np.concatenate([[0], np.cumsum(wire)[:-1]]).astype(np.int64)
buf = torch.randint(0, 256, (int(wire.sum()),), dtype=torch.uint8, device=dev)
d_off, d_len = torch.from_numpy(off).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev)
crc = torch.empty(lens.size, dtype=torch.int32, device=dev)
for _ in range(3):
    if mode == "strided57":
        vc.frames(buf, stride=57004, flen=57000, n=lens.size, out_crc=crc)
    else:
        vc.frames(buf, off=d_off, length=d_len, out_crc=crc, len_hint=0)
torch.cuda.synchronize()
print(mode, "done")
