#!/usr/bin/env python3
"""Minimal profiling target: builds the cfg workload once and launches the
frames kernel `reps` times (run under rocprofv3). Usage: prof_target.py [cfg] [reps] [verify] [nohdr]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import val_protocol_amd.crc as vc  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
verify = "verify" in sys.argv[3:]
nohdr = "nohdr" in sys.argv[3:]  # diagnostic: no header_crc output
dev = torch.device("cuda:0")
vc.init(0)
n, payload, explicit, header = bench.CONFIGS[cfg]
crc = torch.empty(n, dtype=torch.int32, device=dev)
hdr = torch.empty(n, dtype=torch.int32, device=dev) if header and not nohdr else None
if cfg == "cfg5":  # ragged descriptor batch, binned on the device (len_hint 0)
    flat, d_off, d_len = bench.make_ragged_frames(torch, dev, n, seed=1234)  # = bench.py rank 0
    kw = dict(off=d_off, length=d_len, len_hint=0)
    alg = int(d_len.long().sum().item())
else:
    buf, flen, stride = bench.make_frames(torch, dev, n, payload, explicit, 0, 11)
    flat = buf.view(-1)
    kw = dict(stride=stride, flen=flen, n=n)
    alg = n * flen
if verify:
    vc.frames(flat, out_crc=crc, **kw)
    if cfg == "cfg5":
        tidx = ((d_off + d_len.long())[:, None] + torch.arange(4, device=dev)[None, :]).reshape(-1)
        flat[tidx] = crc.view(torch.uint8)
    else:
        buf[:, flen:flen + 4] = crc.view(torch.uint8).view(n, 4)
torch.cuda.synchronize()
for _ in range(reps):
    if verify:
        vc.verify_frames(flat, out_hdr=hdr, **kw)
    else:
        vc.frames(flat, out_crc=crc, out_hdr=hdr, **kw)
torch.cuda.synchronize()
print(f"{cfg}: {reps} launches of {n} frames, algorithmic_bytes_per_launch {alg}")
