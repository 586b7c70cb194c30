#!/usr/bin/env python3
"""Where the cfg4 slices' time goes (bench.py's cfg4_strong_proxy showed the
last rank's slice 2-6% slower than rank 0's, and 1 GiB slices at 80% of the
whole file's per-GPU rate). On one GPU, over bench.py's own cfg4 buffer:
each case is timed like the bench (W untimed launches, K launches between
two events on the launch stream), in an interleaved order, twice:

  first_half / second_half        frames [0, n/2) / [n/2, n) (the 816-B frame last)
  second_half_no_tail             [n/2, n-1): the same bytes without the tail frame
  second_half_strided             [n/2, n-1) through the strided (no descriptor) path
  eighth_<r>                      rank r's 1/8 slice, r = 0 and 7
  whole                           the file in one launch

plus the plain read roof (bench/roof.hip) of each half's bytes. Prints one
JSON line per case.  python tools/slice_probe.py [--steps 20] [--warmup 5]"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
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
    h = n // 2

    def desc_case(first, cnt, hint=flen):
        view = w["flat"][first * stride:(first + cnt) * stride]
        ln = w["d_len"][first:first + cnt]
        off = w["d_off"][:cnt]
        crc = torch.empty(cnt, dtype=torch.int32, device=dev)
        return view, (lambda: vc.frames(view, off=off, length=ln, n=cnt, len_hint=hint, out_crc=crc)), \
            int(ln.long().sum().item())

    def strided_case(first, cnt):
        view = w["flat"][first * stride:(first + cnt) * stride]
        crc = torch.empty(cnt, dtype=torch.int32, device=dev)
        return view, (lambda: vc.frames(view, stride=stride, flen=flen, n=cnt, out_crc=crc)), cnt * flen

    s8 = [shard_frames(n, 8, r) for r in range(8)]
    cases = {
        "first_half": desc_case(0, h),
        "second_half": desc_case(h, n - h),
        "second_half_no_tail": desc_case(h, n - h - 1),
        "second_half_strided": strided_case(h, n - h - 1),
        "first_half_strided": strided_case(0, n - h - 1),
        "eighth_0": desc_case(*s8[0]),
        "eighth_7": desc_case(*s8[7]),
        "eighth_7_no_tail": desc_case(s8[7][0], s8[7][1] - 1),
        "whole": (w["flat"], (lambda: vc.frames(w["flat"], out_crc=w["crc"], **w["kw"])), w["bytes_per_launch"]),
    }
    for rep in range(2):
        order = list(cases) if rep == 0 else list(reversed(list(cases)))
        for name in order:
            view, fn, nbytes = cases[name]
            _, km = bench.timed_steps(torch, dist, 1, fn, args.steps, args.warmup, stream)
            # per-launch spread
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in evs:
                a.record(stream)
                fn()
                b.record(stream)
            torch.cuda.synchronize()
            roof = bench.read_roof(torch, view, stream) if rep == 0 and "strided" not in name else None
            print(json.dumps({"case": name, "rep": rep, "bytes": nbytes, "kernel_ms": round(km, 4),
                              "GiB_s": round(nbytes / (km * 1e-3) / 2**30, 1),
                              "per_launch_ms": [round(a.elapsed_time(b), 4) for a, b in evs],
                              "read_roof_GBs": round(roof, 1) if roof else None,
                              "lanes": vc.lanes_per_frame(flen)}), flush=True)


if __name__ == "__main__":
    main()
