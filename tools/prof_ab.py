#!/usr/bin/env python3
"""Profiling target: 3 launches of one tools/ab_libs.py workload.
usage: prof_ab.py WORKLOAD [LIB]   (WORKLOAD: cfg3 | cfg3b | cfg5 | u57)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import load, workload  # noqa: E402

dev = torch.device("cuda:0")
if len(sys.argv) > 2:
    vc._lib = load(sys.argv[2])
vc.init(0)
w, _ = workload(sys.argv[1], dev)
out = torch.empty(w.get("n") or w["length"].numel(), dtype=torch.int32, device=dev)
for _ in range(3):
    if "off" in w:
        vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out, len_hint=w["len_hint"])
    else:
        vc.frames(w["buf"], stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out)
torch.cuda.synchronize()
print(sys.argv[1], "done")
