#!/usr/bin/env python3
"""Wall time of the reference's own loopback transfer (oracle/_ref/
provider_harness: val_send_files -> val_receive_files over an in-memory pipe,
the reference's src/ compiled here) with the reference's built-in CRC, with
the product's provider, and with the window batcher in its modes (build
container; CPU engine unless VAL_GPU_HOST_BATCH_MIN_BYTES says otherwise).
Median of REPS runs per case; the harness's wall_ms is the transfer only.
usage: session_timing.py [BYTES MTU WINDOW [REPS]]"""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H = os.path.join(ROOT, "oracle", "_ref", "provider_harness")
L = os.path.join(ROOT, "val_protocol_amd", "libval_crc_hip.so")
nbytes, mtu, window = (int(a) for a in (sys.argv[1:4] if len(sys.argv) >= 4 else (64 << 20, 1024, 64)))
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
CASES = [  # name, library, mode, harness environment
    ("reference built-in CRC", "none", "loopback", {}),
    ("product provider", L, "loopback", {}),
    ("batcher AUTO (attach default)", L, "loopback-batched", {"VAL_HARNESS_BATCH_MODE": "auto"}),
    ("batcher ALWAYS, TX and RX", L, "loopback-batched", {}),
    ("batcher ALWAYS, TX only", L, "loopback-batched", {"VAL_HARNESS_BATCH": "tx"}),
    ("batcher ALWAYS, RX only", L, "loopback-batched", {"VAL_HARNESS_BATCH": "rx"}),
    ("batcher ALWAYS, RX only, max_frames 8", L, "loopback-batched",
     {"VAL_HARNESS_BATCH": "rx", "VAL_HARNESS_BATCH_FRAMES": "8"}),
]
print(json.dumps({"bytes": nbytes, "mtu": mtu, "window": window, "reps": reps,
                  "host_batch_min_bytes": os.environ.get("VAL_GPU_HOST_BATCH_MIN_BYTES", "library default")}))
for name, lib, mode, extra in CASES:
    env = dict(os.environ, **extra)
    walls, last = [], None
    for _ in range(reps):
        out = subprocess.run([H, lib, mode, str(nbytes), str(mtu), str(window)], capture_output=True, text=True,
                             env=env, timeout=600, check=True).stdout
        last = json.loads(out.strip().splitlines()[-1])
        assert last["equal"] == 1 and last["tx_status"] == 0 and last["rx_status"] == 0, last
        walls.append(last["wall_ms"])
    med = statistics.median(walls)
    rec = {"case": name, "median_ms": med, "MiB_s": round(nbytes / 2**20 / (med / 1e3), 1), "wall_ms": walls}
    if "batch" in last:
        rec["batches"] = {e["end"]: [e["tx_batches"], e["rx_batches"]] for e in last["batch"]}
    print(json.dumps(rec), flush=True)
