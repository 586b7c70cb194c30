"""Verify-window (K4) latency: back-to-back val_crc32_region_dev calls per
window size, timed with HIP events on the launch stream (GPU time per call)
and the host wall clock (submission cost per call). Each result is checked
against the oracle once. Run under rocprofv3 --kernel-trace --stats for the
kernel durations alone."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import val_protocol_amd.crc as vc  # noqa: E402
from tests import _oracle  # noqa: E402

vc.init(0)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(7)
big = torch.randint(0, 256, (256 << 20,), dtype=torch.uint8, device=dev, generator=g)
stream = torch.cuda.current_stream()
out = torch.empty(1, dtype=torch.int32, device=dev)
rows = []
for size in (1 << 10, 4 << 10, 8 << 10, (8 << 10) + 1, 16 << 10, (16 << 10) + 1, 32 << 10, 64 << 10, 1 << 20, 8 << 20, 64 << 20, 256 << 20):
    win = big[:size]
    vc.region(win, out=out)
    torch.cuda.synchronize()
    ok = (int(out.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == _oracle.crc32(win.cpu().numpy())
    reps = 200 if size <= (8 << 20) else 50
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    t0 = time.perf_counter()
    for _ in range(reps):
        vc.region(win, out=out)
    t1 = time.perf_counter()
    b.record(stream)
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    rows.append({"bytes": size, "gpu_us_per_call": round(us, 2), "host_us_per_call": round((t1 - t0) * 1e6 / reps, 2),
                 "GiB_s": round(size / (us * 1e-6) / (1 << 30), 1), "crc_ok": ok})
for r in rows:
    print(json.dumps(r))
