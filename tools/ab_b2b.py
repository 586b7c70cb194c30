#!/usr/bin/env python3
"""A/B of library builds on back-to-back launches (tooling only): each
library hashes K launches in a row over rotating copies of a workload
(tools/ab_libs.py names), two events bracketing the K launches, as bench.py
times its steps; libraries interleaved, median of rounds. Separates the
kernel from the host submission path: a host path slower than the kernel
shows up here and not in ab_libs.py's single-launch timing.
usage: ab_b2b.py LIB_A LIB_B [...] [workload ...] (K=200 launches)"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import workload  # noqa: E402


def main():
    paths = [a for a in sys.argv[1:] if a.endswith(".so")]
    names = [a for a in sys.argv[1:] if not a.endswith(".so")] or ["cfg2"]
    libs = []
    for p in paths:
        l = ctypes.CDLL(os.path.abspath(p), mode=ctypes.RTLD_LOCAL)
        vc._declare(l, strict=False)
        assert l.val_gpu_init(0) == 0
        libs.append(l)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    K = int(os.environ.get("B2B_K", "200"))
    for name in names:
        w, nbytes = workload(name, dev)
        n = w.get("n") or w["length"].numel()
        rot = max(1, min(16, -(-(1 << 30) // w["buf"].numel())))
        bufs = [w["buf"]] + [w["buf"].clone() for _ in range(rot - 1)]
        out = torch.empty(n, dtype=torch.int32, device=dev)
        res = [[] for _ in libs]
        for rep in range(5):
            for i, l in enumerate(libs):
                vc._lib = l
                def go(b):
                    if "off" in w:
                        vc.frames(b, off=w["off"], length=w["length"], out_crc=out, len_hint=w["len_hint"])
                    else:
                        vc.frames(b, stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out)
                for k in range(20):
                    go(bufs[k % rot])
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                for k in range(K):
                    go(bufs[k % rot])
                b.record(s)
                torch.cuda.synchronize()
                res[i].append(a.elapsed_time(b) / K * 1e3)
        base = np.median(res[0])
        line = f"{name}: A {base:.2f} us/launch ({nbytes / base / 1e3:.0f} GB/s)"
        for i in range(1, len(libs)):
            m = np.median(res[i])
            line += f"  {chr(65 + i)} {m:.2f} us speed {base / m:.3f}"
        print(line, " ", [["%.2f" % x for x in r] for r in res], flush=True)


if __name__ == "__main__":
    main()
