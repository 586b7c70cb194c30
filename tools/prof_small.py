#!/usr/bin/env python3
"""Profiling target for small batches (run under rocprofv3 --kernel-trace):
for each workload x geometry, REPS launches with a sync after each.
usage: [VCRC_LIB=lib.so] prof_small.py REPS name:G:PF ...   (G 0 / PF -1 = automatic). Tooling only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import load, workload  # noqa: E402

if os.environ.get("VCRC_LIB"):  # another build of the library (A/B)
    vc._lib = load(os.environ["VCRC_LIB"])

reps = int(sys.argv[1])
dev = torch.device("cuda:0")
vc.init(0)
cache = {}
for spec in sys.argv[2:]:
    name, G, PF = spec.split(":")
    if name not in cache:
        cache[name] = workload(name, dev)
    w, nbytes = cache[name]
    out = torch.empty(w.get("n") or w["length"].numel(), dtype=torch.int32, device=dev)
    vc.set_geometry(int(G), int(PF))
    for _ in range(reps):
        if "off" in w:
            vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out, len_hint=w["len_hint"])
        else:
            vc.frames(w["buf"], stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out)
        torch.cuda.synchronize()
    print(spec, nbytes, flush=True)
vc.set_geometry()
