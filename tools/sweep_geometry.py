#!/usr/bin/env python3
"""Times the frames kernel for every lanes-per-frame geometry on the BASELINE
shapes (device-resident, HIP events on the launch stream). Diagnostic only."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import val_protocol_amd.crc as vc  # noqa: E402


def time_it(fn, reps=10):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(np.min(ts))


def main():
    dev = torch.device("cuda:0")
    vc.init(0)
    cfgs = sys.argv[1:] or ["cfg3", "cfg2", "cfg4"]
    for name in cfgs:
        n, payload, explicit, header = bench.CONFIGS[name]
        buf, flen, stride = bench.make_frames(torch, dev, n, payload, explicit, 0, 7)
        flat = buf.view(-1)
        crc = torch.empty(n, dtype=torch.int32, device=dev)
        hdr = torch.empty(n, dtype=torch.int32, device=dev) if header else None
        ref = None
        for G in [1, 2, 4, 8, 16, 32, 64]:
            vc.set_lanes_per_frame(G)
            med, best = time_it(lambda: vc.frames(flat, stride=stride, flen=flen, n=n, out_crc=crc, out_hdr=hdr))
            out = crc.clone()
            same = True if ref is None else bool(torch.equal(out, ref))
            ref = out if ref is None else ref
            gbs = n * flen / (med * 1e-3) / 1e9
            print(f"{name} G={G:2d}: median {med:.3f} ms best {best:.3f} ms  {gbs:7.1f} GB/s  same={same}", flush=True)
        vc.set_lanes_per_frame(0)
        del buf, flat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
