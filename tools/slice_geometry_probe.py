#!/usr/bin/env python3
"""Lanes per frame for the cfg4 proxy's slices (tooling only): a 1/8, 1/4
and 1/2 slice of bench.py's cfg4 file (64 KiB frames, descriptor batches with
the uniform hint, as the proxy times them) and the whole file, each hashed at
the automatic geometry (16 lanes: one 4-frame group per wave for an eighth)
and forced to 32 and 64 lanes (2 and 4 groups per wave, so the dynamic
queue evens out the waves' ends), timed like bench.py in alternating order,
outputs compared across geometries.
usage: slice_geometry_probe.py [--steps 20] [--warmup 10] [--reps 3]"""
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
    from val_protocol_amd.shard import shard_frames

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    vc.init(0)
    w = bench.build_workload(torch, dev, "cfg4", 0, 1, False, vc)
    stream = torch.cuda.current_stream()
    n, stride, flen = w["n"], w["stride"], w["flen"]
    slices = {"eighth_0": shard_frames(n, 8, 0), "eighth_7": shard_frames(n, 8, 7),
              "quarter_3": shard_frames(n, 4, 3), "half_1": shard_frames(n, 2, 1), "whole": (0, n)}
    for name, (first, cnt) in slices.items():
        view = w["flat"][first * stride:(first + cnt) * stride]
        ln = w["d_len"][first:first + cnt]
        off = w["d_off"][:cnt]
        nbytes = int(ln.long().sum().item())
        outs, times = {}, {}
        geoms = (0, 32, 64)
        for g in geoms:
            outs[g] = torch.empty(cnt, dtype=torch.int32, device=dev)
            times[g] = []
        for rep in range(args.reps):
            for g in (geoms if rep % 2 == 0 else geoms[::-1]):
                vc.set_geometry(g)
                try:
                    fn = (lambda o: lambda: vc.frames(view, off=off, length=ln, n=cnt, len_hint=flen, out_crc=o))(outs[g])
                    _, km = bench.timed_steps(torch, dist, 1, fn, args.steps, args.warmup, stream)
                finally:
                    vc.set_geometry()
                times[g].append(round(km, 4))
        torch.cuda.synchronize()
        same = all(torch.equal(outs[0], outs[g]) for g in geoms)
        best = {("auto" if g == 0 else str(g)): min(v) for g, v in times.items()}
        print(json.dumps({"slice": name, "frames": cnt, "bytes": nbytes, "auto_lanes": vc.lanes_per_frame(flen),
                          "same_outputs": same, "kernel_ms": {("auto" if g == 0 else str(g)): v for g, v in times.items()},
                          "best_ms": best, "GiB_s": {k: round(nbytes / (v * 1e-3) / 2**30, 1) for k, v in best.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
