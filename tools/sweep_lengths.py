#!/usr/bin/env python3
"""Best lanes-per-frame per frame length: uniform strided batches of ~3.4 GB
at each CRC-input length, every G. Diagnostic only (feeds lanes_per_frame)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.ab_libs import time_it  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    vc.init(0)
    lengths = [int(x) for x in os.environ.get("SWEEP_LENGTHS", "300,600,1100,2100,4200,8300,16500,33000,65540").split(",")]
    total = 3 << 30
    for L in lengths:
        stride = L + 4
        n = total // stride
        buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev)
        crc = torch.empty(n, dtype=torch.int32, device=dev)
        row = []
        for G in (1, 2, 4, 8, 16, 32, 64):
            vc.set_geometry(G, 1)
            med, _ = time_it(lambda: vc.frames(buf, stride=stride, flen=L, n=n, out_crc=crc), reps=5)
            row.append((G, n * L / (med * 1e-3) / 1e9))
        best = max(row, key=lambda t: t[1])
        print(f"L={L:6d} n={n:8d} " + " ".join(f"G{g}:{r:6.0f}" for g, r in row) + f"  best G={best[0]}", flush=True)
        vc.set_geometry()
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
