#!/usr/bin/env python3
"""Profiling target for rocprofv3 passes over the A/B workloads of
tools/ab_libs.py (u1100d, s1100, cfg3b, cfg5log, ...): builds the workload
once, launches the frames kernel `reps` times through the product library.
Usage: prof_wl.py WORKLOAD [reps]  (tooling only; PROF_LIB=path profiles
another build of the library, e.g. build/libval_B.so)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import workload  # noqa: E402

if os.environ.get("PROF_LIB"):
    vc.LIB_PATH = os.path.abspath(os.environ["PROF_LIB"])
name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
vc.init(0)
w, nbytes = workload(name, dev)
n = w.get("n") or w["length"].numel()
out = torch.empty(n, dtype=torch.int32, device=dev)
if "off" in w:
    fn = lambda: vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out, len_hint=w["len_hint"])
else:
    fn = lambda: vc.frames(w["buf"], stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out)
fn()
torch.cuda.synchronize()
for _ in range(reps):
    fn()
torch.cuda.synchronize()
print(f"{name}: {reps} launches, {n} frames, algorithmic_bytes_per_launch {nbytes}", flush=True)
