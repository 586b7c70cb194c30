#!/usr/bin/env python3
"""Strided against descriptor mode on the same uniform buffers (tooling
only): cfg3's 1 M x 16,400 B at stride 16,404 and cfg4's 131,113 x 65,532 B
at stride 65,536, each hashed through val_crc32_frames_dev in strided mode
and in descriptor mode with the uniform length hint, timed like bench.py,
alternating. usage: desc_probe.py [--steps 20] [--warmup 10] [--reps 3]"""
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
    stream = torch.cuda.current_stream()
    for name, n, L in (("cfg3", 1 << 20, 16400), ("cfg4", 131113, 65532)):
        stride = L + 4
        g = torch.Generator(device=dev).manual_seed(n)
        buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(n, device=dev, dtype=torch.int64) * stride
        ln = torch.full((n,), L, dtype=torch.int32, device=dev)
        a = torch.empty(n, dtype=torch.int32, device=dev)
        b = torch.empty(n, dtype=torch.int32, device=dev)
        fns = {"strided": lambda: vc.frames(buf, stride=stride, flen=L, n=n, out_crc=a),
               "descriptor": lambda: vc.frames(buf, off=off, length=ln, len_hint=L, out_crc=b)}
        times = {k: [] for k in fns}
        for rep in range(args.reps):
            for k in (list(fns) if rep % 2 == 0 else list(fns)[::-1]):
                _, km = bench.timed_steps(torch, dist, 1, fns[k], args.steps, args.warmup, stream)
                times[k].append(round(km, 4))
        torch.cuda.synchronize()
        print(json.dumps({"workload": name, "same_outputs": bool(torch.equal(a, b)), "kernel_ms": times,
                          "best_ms": {k: min(v) for k, v in times.items()}}), flush=True)
        del buf, off, ln, a, b, fns
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
