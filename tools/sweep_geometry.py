#!/usr/bin/env python3
"""Times the frames kernel for kernel geometries on the BASELINE shapes
(device-resident, HIP events on the launch stream). Diagnostic only.

SWEEP_COMBOS="G:PF,..." overrides the default list."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import val_protocol_amd.crc as vc  # noqa: E402

DEFAULT = {
    "cfg3": [(g, p) for g in (4, 8, 16, 32) for p in (0, 1)],
    "cfg4": [(g, p) for g in (8, 16, 32, 64) for p in (0, 1)],
    "cfg2": [(g, p) for g in (1, 2, 4, 8) for p in (0, 1)],
}


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
    cfgs = sys.argv[1:] or ["cfg3", "cfg4", "cfg2"]
    env = os.environ.get("SWEEP_COMBOS")
    for name in cfgs:
        combos = [tuple(int(x) for x in c.split(":")) for c in env.split(",")] if env else DEFAULT[name]
        n, payload, explicit, header = bench.CONFIGS[name]
        buf, flen, stride = bench.make_frames(torch, dev, n, payload, explicit, 0, 7)
        flat = buf.view(-1)
        crc = torch.empty(n, dtype=torch.int32, device=dev)
        hdr = torch.empty(n, dtype=torch.int32, device=dev) if header else None
        vc.set_geometry()
        vc.frames(flat, stride=stride, flen=flen, n=n, out_crc=crc, out_hdr=hdr)
        ref = crc.clone()
        rounds = int(os.environ.get("SWEEP_ROUNDS", "1"))  # >1: combos interleaved, median of round medians
        res = {c: [] for c in combos}
        for _ in range(rounds):
            for G, PF in combos:
                vc.set_geometry(G, PF)
                med, best = time_it(lambda: vc.frames(flat, stride=stride, flen=flen, n=n, out_crc=crc, out_hdr=hdr))
                res[(G, PF)].append((med, best, bool(torch.equal(crc, ref))))
        for G, PF in combos:
            med = float(np.median([r[0] for r in res[(G, PF)]]))
            best = min(r[1] for r in res[(G, PF)])
            same = all(r[2] for r in res[(G, PF)])
            gbs = n * flen / (med * 1e-3) / 1e9
            print(f"{name} G={G:2d} PF={PF}: median {med:.3f} ms best {best:.3f} ms "
                  f"{gbs:7.1f} GB/s same={same}", flush=True)
        vc.set_geometry()
        del buf, flat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
