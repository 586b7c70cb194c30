#!/usr/bin/env python3
"""Crossover of the host-memory batch calls (tooling).
For windows of W DATA frames at VAL's MTUs, host memory in and CRCs out,
times val_crc32_frames_host on the GPU path (threshold 0; pageable and pinned
input) against the library's CPU engine on 1 thread and on the process's
effective CPU count (threshold 2^62, val_gpu_set_host_cpu_threads), every
output checked equal. Prints one JSON line per (MTU, W) and a summary line
with the smallest window where the GPU path beats one CPU thread.
usage: host_crossover.py [max_bytes] [--fine]
--fine: windows of 16, 24, ..., 72 MiB of CRC input at each MTU (the band
where the crossover lies), instead of W = 16 .. 65,535 frames."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import val_protocol_amd.crc as vc  # noqa: E402


def t_call(fn, budget_s=0.4, max_reps=200):
    fn()
    ts = []
    t_end = time.perf_counter() + budget_s
    while len(ts) < 3 or (time.perf_counter() < t_end and len(ts) < max_reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e6


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    fine = "--fine" in sys.argv
    max_bytes = int(args[0]) if args else (1 << 30)
    vc.init(0)
    _, eff = bench.effective_cpus()
    rows = []
    rng = np.random.default_rng(5)
    for mtu in (1024, 16404, 65536):
        flen = mtu - 4
        ws = ([max(1, (m << 20) // flen) for m in range(16, 73, 8)] if fine
              else (16, 64, 256, 1024, 4096, 16384, 65535))
        for W in ws:
            if W * mtu > max_bytes:
                continue
            stream = rng.integers(0, 256, W * mtu, dtype=np.uint8)
            pinned = vc.PinnedBuffer(stream.size)
            pinned.array[:] = stream
            kw = dict(stride=mtu, flen=flen, n=W)
            vc.set_host_batch_min_bytes(0)
            ref = vc.frames_host(stream, **kw)
            gpu = t_call(lambda: vc.frames_host(stream, **kw))
            gpu_p = t_call(lambda: vc.frames_host(pinned.array, **kw))
            vc.set_host_batch_min_bytes(1 << 62)
            out = {}
            for t in (1, eff):
                vc.set_host_cpu_threads(t)
                got = vc.frames_host(stream, **kw)
                assert np.array_equal(got, ref), (mtu, W, t)
                out[t] = t_call(lambda: vc.frames_host(stream, **kw))
            vc.set_host_cpu_threads(1)
            vc.set_host_batch_min_bytes(-1)
            pinned.free()
            r = {"mtu": mtu, "frames": W, "crc_bytes": W * flen, "gpu_pageable_us": round(gpu, 1),
                 "gpu_pinned_us": round(gpu_p, 1), "cpu_1thread_us": round(out[1], 1),
                 f"cpu_{eff}threads_us": round(out[eff], 1), "cpu_threads_effective": eff,
                 "gpu_beats_1thread": gpu < out[1], "gpu_beats_all_threads": gpu < out[eff]}
            rows.append(r)
            print(json.dumps(r), flush=True)
    summary = {}
    for mtu in (1024, 16404, 65536):
        wins = [r["crc_bytes"] for r in rows if r["mtu"] == mtu and r["gpu_beats_1thread"]]
        summary[str(mtu)] = min(wins) if wins else None
    print(json.dumps({"summary": "smallest crc_bytes where the pageable GPU path beats 1 CPU thread, per MTU",
                      "crossover_bytes": summary}), flush=True)


if __name__ == "__main__":
    main()
