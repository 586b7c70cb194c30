#!/usr/bin/env python3
"""PCIe-inclusive rate of the TX CRC path for cfg3: frames start in pinned host
memory, are copied H2D in chunks on a copy stream while the previous chunk is
hashed on a compute stream, and the CRCs come back D2H. This is the number
DESIGN.md reports beside the device-resident one (never bench.py's value)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import val_protocol_amd.crc as vc  # noqa: E402
from tests import _oracle  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    vc.init(0)
    n, payload, explicit, _ = bench.CONFIGS["cfg3"]
    n = n // 4  # 256 Ki frames = 4.3 GB of pinned host memory
    buf, flen, stride = bench.make_frames(torch, dev, n, payload, explicit, 0, 5)
    host = buf.cpu().pin_memory()
    del buf
    chunk = 16384  # frames per chunk (269 MB)
    nchunks = (n + chunk - 1) // chunk
    dbuf = [torch.empty((chunk, stride), dtype=torch.uint8, device=dev) for _ in range(2)]
    dcrc = torch.empty(n, dtype=torch.int32, device=dev)
    hcrc = torch.empty(n, dtype=torch.int32).pin_memory()
    copy_s, comp_s = torch.cuda.Stream(), torch.cuda.Stream()
    done = [torch.cuda.Event() for _ in range(2)]
    ready = [torch.cuda.Event() for _ in range(2)]

    def run():
        for i in range(nchunks):
            s = i % 2
            lo, hi = i * chunk, min(n, (i + 1) * chunk)
            with torch.cuda.stream(copy_s):
                copy_s.wait_event(done[s])
                dbuf[s][: hi - lo].copy_(host[lo:hi], non_blocking=True)
                ready[s].record(copy_s)
            with torch.cuda.stream(comp_s):
                comp_s.wait_event(ready[s])
                vc.frames(dbuf[s].view(-1), stride=stride, flen=flen, n=hi - lo, out_crc=dcrc[lo:hi], stream=comp_s)
                done[s].record(comp_s)
        with torch.cuda.stream(comp_s):
            hcrc.copy_(dcrc, non_blocking=True)
        torch.cuda.synchronize()

    run()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    gib = n * flen / dt / (1 << 30)
    h2d = n * stride / dt / 1e9
    idx = np.random.default_rng(0).choice(n, 200, replace=False)
    rows = host[torch.from_numpy(idx)].numpy().reshape(-1)
    ok = np.array_equal(hcrc.numpy().view(np.uint32)[idx], _oracle.frames_strided(rows, stride, flen, idx.size))
    print(f"host-inclusive cfg3 ({n} frames, pinned, {chunk}-frame chunks, 2 streams): {gib:.1f} GiB/s CRC input, "
          f"{h2d:.1f} GB/s H2D wire bytes, {dt * 1e3:.1f} ms per pass, parity={ok}", flush=True)

    # The product's own host API (C ABI, native chunked pipeline): pinned
    # buffer from val_gpu_host_alloc (DMA in place) and a pageable copy
    # (pinned bounce buffers, host memcpy threads).
    want = hcrc.numpy().view(np.uint32).copy()
    pb = vc.PinnedBuffer(n * stride)
    pb.array[:] = host.numpy().reshape(-1)
    pageable = np.array(host.numpy().reshape(-1))
    del host
    for name, arr in (("pinned (val_gpu_host_alloc)", pb.array), ("pageable", pageable)):
        vc.frames_host(arr, stride=stride, flen=flen, n=n)
        t0 = time.perf_counter()
        for _ in range(reps):
            got = vc.frames_host(arr, stride=stride, flen=flen, n=n)
        dt = (time.perf_counter() - t0) / reps
        print(f"C-ABI val_crc32_frames_host cfg3 ({n} frames, {name}): {n * flen / dt / (1 << 30):.1f} GiB/s CRC input, "
              f"{n * stride / dt / 1e9:.1f} GB/s wire, {dt * 1e3:.1f} ms per call, parity={np.array_equal(got, want)}",
              flush=True)
    pb.free()


if __name__ == "__main__":
    main()
