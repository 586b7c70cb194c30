#!/usr/bin/env python3
"""Does the 128-B line layout of cfg3 frames cost time? 1 M frames of 16,400
B CRC input through the product's descriptor path (uniform hint), in three
layouts of the same bytes per frame (tooling only):
  packed     stride 16,404 (the bench: frames share their boundary lines,
             rounds straddle lines)
  end_align  stride 16,512, each frame's END on a 128-B line (rounds, which
             are anchored at the end, never straddle a line; no line is
             shared by two frames; 112 B of gap per frame is read with the
             first line)
  start_align stride 16,512, each frame's START on a line (no shared lines,
             rounds straddle)
Timed like bench.py (W untimed launches, K back to back between events),
alternating, and the plain read roof of each buffer.
usage: layout_probe.py [--steps 20] [--warmup 10] [--reps 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    import bench
    import val_protocol_amd.crc as vc

    dev = torch.device("cuda:0")
    vc.init(0)
    n, L = 1 << 20, 16400
    stream = torch.cuda.current_stream()
    cases = {}
    for name, stride, first in (("packed", 16404, 0), ("end_align", 16512, 112), ("start_align", 16512, 0)):
        g = torch.Generator(device=dev).manual_seed(stride + first)
        buf = torch.randint(0, 256, (n * stride + 256,), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(n, device=dev, dtype=torch.int64) * stride + first
        ln = torch.full((n,), L, dtype=torch.int32, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = (lambda b, o, l, c: lambda: vc.frames(b, off=o, length=l, len_hint=L, out_crc=c))(buf, off, ln, out)
        cases[name] = (buf, fn)
        del buf
    times = {k: [] for k in cases}
    for rep in range(args.reps):
        for name in (list(cases) if rep % 2 == 0 else list(cases)[::-1]):
            _, km = bench.timed_steps(torch, dist, 1, cases[name][1], args.steps, args.warmup, stream)
            times[name].append(round(km, 4))
    for name, (buf, _) in cases.items():
        roof = bench.read_roof(torch, buf, stream)
        best = min(times[name])
        print(json.dumps({"layout": name, "kernel_ms": times[name], "best_ms": best,
                          "alg_GBs": round(n * L / (best * 1e-3) / 1e9, 1), "buffer_read_roof_GBs": round(roof, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
