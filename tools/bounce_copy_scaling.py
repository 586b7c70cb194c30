#!/usr/bin/env python3
"""Host half of the N-device crossover: the pageable
bounce copies alone, with no device work. For 1, 2, 4 and 8 concurrent copy
streams (the shards of a *_host_multi call over that many GPUs), each copying
64 MiB chunks (the host path's chunk) from resident pageable memory into its
own page-locked bounce buffer through the library's own bounce copy and its
thread policy (val_gpu_host_copy_probe, val_gpu_host_copy_threads), prints
one JSON line per case: aggregate GB/s and the threads each copy used.

  python tools/bounce_copy_scaling.py [--pinned 1] [--reps 8] > out.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pinned", type=int, default=1, help="1: hipHostMalloc bounce buffers (needs a GPU box)")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--copies", default="1,2,4,8")
    args = ap.parse_args()
    import val_protocol_amd.crc as vc
    from bench import effective_cpus

    nbytes = args.chunk_mib << 20
    visible, budget = effective_cpus()
    for k in [int(x) for x in args.copies.split(",")]:
        runs = [vc.host_copy_probe(k, nbytes, args.reps, bool(args.pinned)) for _ in range(3)]
        print(json.dumps({"copies": k, "chunk_bytes": nbytes, "reps": args.reps, "pinned_dst": bool(args.pinned),
                          "threads_per_copy": int(vc.lib().val_gpu_host_copy_threads(nbytes, k)),
                          "cpu_budget": budget, "cpus_visible": visible,
                          "aggregate_GBs": round(max(runs), 2), "runs_GBs": [round(r, 2) for r in runs]}),
              flush=True)


if __name__ == "__main__":
    main()
