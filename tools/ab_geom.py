#!/usr/bin/env python3
"""Same-box A/B of geometries in one library: interleaved timing of
val_crc32_frames_dev under val_gpu_set_lanes_per_frame / val_gpu_set_prefetch
settings (tooling only).
usage: ab_geom.py WORKLOAD G:PF [G:PF ...]   (0:-1 = the library's own choice)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import workload  # noqa: E402
from tools.sweep_geometry import time_it  # noqa: E402


def main():
    name = sys.argv[1]
    geoms = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]]
    dev = torch.device("cuda:0")
    vc.init(0)
    w, nbytes = workload(name, dev)
    n = w.get("n") or w["length"].numel()
    out = torch.empty(n, dtype=torch.int32, device=dev)
    if "off" in w:
        fn = lambda: vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out, len_hint=w["len_hint"])
    else:
        fn = lambda: vc.frames(w["buf"], stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out)
    res = [[] for _ in geoms]
    ref = None
    for rep in range(4):
        for i, (g, pf) in enumerate(geoms):
            vc.set_geometry(g, pf)
            med, _ = time_it(fn, reps=10)
            res[i].append(med)
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), (g, pf)
    vc.set_geometry()
    a = np.median(res[0])
    line = f"{name}: {geoms[0]} {a:.4f} ms ({nbytes / a / 1e6:.0f} GB/s)"
    for i in range(1, len(geoms)):
        b = np.median(res[i])
        line += f"  {geoms[i]} {b:.4f} ms speed {a / b:.3f}"
    print(line, flush=True)


if __name__ == "__main__":
    main()
