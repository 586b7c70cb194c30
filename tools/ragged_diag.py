#!/usr/bin/env python3
"""Ragged-path diagnostics: the binned kernel on uniform-length descriptor
batches vs the strided kernel, and on single-class log-uniform mixes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402
from tools.sweep_geometry import time_it  # noqa: E402


def run(name, lens, dev):
    lens = np.asarray(lens, np.int64)
    wire = lens + 4
    off = np.concatenate([[0], np.cumsum(wire)[:-1]]).astype(np.int64)
    total = int(wire.sum())
    buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    d_off = torch.from_numpy(off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    crc = torch.empty(lens.size, dtype=torch.int32, device=dev)
    nbytes = int(lens.sum())
    med, _ = time_it(lambda: vc.frames(buf, off=d_off, length=d_len, out_crc=crc, len_hint=0), reps=5)
    line = f"{name:28s} n={lens.size:7d} {nbytes / 1e9:5.2f} GB ragged {med:7.3f} ms {nbytes / med / 1e6:7.1f} GB/s"
    if np.all(lens == lens[0]):
        L = int(lens[0])
        med2, _ = time_it(lambda: vc.frames(buf, stride=L + 4, flen=L, n=lens.size, out_crc=crc), reps=5)
        med3, _ = time_it(lambda: vc.frames(buf, off=d_off, length=d_len, out_crc=crc, len_hint=L), reps=5)
        line += f" | strided {med2:7.3f} ms {nbytes / med2 / 1e6:7.1f} | desc-uniform {med3:7.3f} ms {nbytes / med3 / 1e6:7.1f}"
    print(line, flush=True)
    del buf
    torch.cuda.empty_cache()


def main():
    dev = torch.device("cuda:0")
    vc.init(0)
    rng = np.random.default_rng(1)
    for L in (600, 4200, 16400, 57000):
        run(f"uniform L={L}", np.full((3 << 30) // (L + 4), L), dev)

    def logu(lo, hi, n):
        return np.exp(rng.uniform(np.log(lo), np.log(hi), n)).astype(np.int64)

    run("cfg5 mix 520..65532", logu(520, 65532, 262144), dev)
    run("class3 only 49152..65532", logu(49152, 65532, 60000), dev)
    run("class2 only 8192..49151", logu(8192, 49151, 150000), dev)
    run("class1 only 1024..8191", logu(1024, 8191, 600000), dev)
    run("narrow 16000..16800", rng.integers(16000, 16800, 200000), dev)


if __name__ == "__main__":
    main()
