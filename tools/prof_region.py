#!/usr/bin/env python3
"""Profiling target: N back-to-back region calls of one size (run under
rocprofv3). usage: prof_region.py BYTES [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
vc.init(0)
d = torch.randint(0, 256, (size,), dtype=torch.uint8, device="cuda:0")
out = torch.empty(1, dtype=torch.int32, device="cuda:0")
torch.cuda.synchronize()
for _ in range(reps):
    vc.region(d, out=out)
torch.cuda.synchronize()
print("done", size, reps)
