#!/usr/bin/env python3
"""Cost of the header_crc output (K3) per workload: the same call with and
without out_hdr, interleaved in one process (tooling only, not the product).
usage: hdr_cost.py [cfg5log|cfg3b|cfg4d|...]..."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import workload  # noqa: E402
from tools.sweep_geometry import time_it  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    vc.init(0)
    for name in sys.argv[1:] or ["cfg5log", "cfg3b"]:
        w, nbytes = workload(name, dev)
        n = w.get("n") or w["length"].numel()
        out = torch.empty(n, dtype=torch.int32, device=dev)
        hdr = torch.empty(n, dtype=torch.int32, device=dev)
        res = {False: [], True: []}
        for rep in range(4):
            for h in (False, True):
                if "off" in w:
                    fn = lambda: vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out,
                                           out_hdr=hdr if h else None, len_hint=w["len_hint"])
                else:
                    fn = lambda: vc.frames(w["buf"], stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out,
                                           out_hdr=hdr if h else None)
                res[h].append(time_it(fn, reps=10)[0])
        a, b = np.median(res[False]), np.median(res[True])
        print(f"{name}: no hdr {a:.4f} ms ({nbytes / a / 1e6:.0f} GB/s)  hdr {b:.4f} ms ({nbytes / b / 1e6:.0f} GB/s)"
              f"  cost {100 * (b / a - 1):+.1f}%", flush=True)


if __name__ == "__main__":
    main()
