#!/usr/bin/env python3
"""Minimal profiling target: builds the cfg workload once and launches the
frames kernel `reps` times (run under rocprofv3). Usage: prof_target.py [cfg] [reps] [verify]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import val_protocol_amd.crc as vc  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
verify = len(sys.argv) > 3 and sys.argv[3] == "verify"
dev = torch.device("cuda:0")
vc.init(0)
n, payload, explicit, header = bench.CONFIGS[cfg]
buf, flen, stride = bench.make_frames(torch, dev, n, payload, explicit, 0, 11)
flat = buf.view(-1)
crc = torch.empty(n, dtype=torch.int32, device=dev)
hdr = torch.empty(n, dtype=torch.int32, device=dev) if header else None
if verify:
    vc.frames(flat, stride=stride, flen=flen, n=n, out_crc=crc)
    buf[:, flen:flen + 4] = crc.view(torch.uint8).view(n, 4)
torch.cuda.synchronize()
for _ in range(reps):
    if verify:
        vc.verify_frames(flat, stride=stride, flen=flen, n=n, out_hdr=hdr)
    else:
        vc.frames(flat, stride=stride, flen=flen, n=n, out_crc=crc, out_hdr=hdr)
torch.cuda.synchronize()
print(f"{cfg}: {reps} launches of {n} frames x {flen} B CRC input, lanes/frame {vc.lanes_per_frame(flen)}")
