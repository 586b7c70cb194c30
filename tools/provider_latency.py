#!/usr/bin/env python3
"""Per-call latency of the scalar hooks by size, host memory in, finished CRC
out (diagnostic; DESIGN.md section 1 takes the provider threshold from it).

Columns, per input length:
  gpu      val_gpu_crc32_provider forced onto the GPU (threshold 0)
  cpu      the library's CPU engine (best this host has) through the provider
  s16      the CPU engine's slice-by-16 (val_crc32_cpu_update_state engine 1)
  ref      the reference's own val_crc32 (oracle/_ref/libval_ref.so, the code
           the provider replaces), when built
  default  the provider with its built-in threshold
The crossover is the shortest length from which the GPU column stays below the
cpu column."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import val_protocol_amd.crc as vc  # noqa: E402

vc.init(0)
lib = vc.lib()
ref_path = os.path.join(ROOT, "oracle", "_ref", "libval_ref.so")
ref = None
if os.path.exists(ref_path):
    ref = ctypes.CDLL(ref_path)
    ref.val_crc32.restype = ctypes.c_uint32
    ref.val_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]


def per_call(fn, L):
    fn()
    reps = max(5, min(2000, int(2e8 / (L + 2000))))
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


sizes = [16, 1024, 16400, 65543, 262144, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30]
print(f"cpu engine {vc.cpu_engine()}; built-in threshold {vc.provider_min_bytes()} B "
      f"(env VAL_GPU_PROVIDER_MIN_BYTES={os.environ.get('VAL_GPU_PROVIDER_MIN_BYTES')})", flush=True)
print(f"{'L':>10} {'gpu_us':>9} {'cpu_us':>9} {'s16_us':>9} {'ref_us':>9} {'default_us':>10}  gpu GB/s  cpu GB/s",
      flush=True)
rows = []
for L in sizes:
    data = np.random.default_rng(L).integers(0, 256, L, dtype=np.uint8)
    p = ctypes.c_void_p(data.ctypes.data)
    want = vc.cpu_update_state(0xFFFFFFFF, data) ^ 0xFFFFFFFF
    vc.set_provider_min_bytes(0)
    assert lib.val_gpu_crc32_provider(0xFFFFFFFF, p, L) == want and vc.last_hook_path() == vc.HOOK_GPU
    gpu = per_call(lambda: lib.val_gpu_crc32_provider(0xFFFFFFFF, p, L), L)
    vc.set_provider_min_bytes(1 << 62)
    assert lib.val_gpu_crc32_provider(0xFFFFFFFF, p, L) == want and vc.last_hook_path() == vc.HOOK_CPU
    cpu = per_call(lambda: lib.val_gpu_crc32_provider(0xFFFFFFFF, p, L), L)
    s16 = per_call(lambda: lib.val_crc32_cpu_update_state(0xFFFFFFFF, p, L, 1), L) if L <= (64 << 20) else float("nan")
    r = float("nan")
    if ref is not None and L <= (16 << 20):
        assert ref.val_crc32(p, L) == want
        r = per_call(lambda: ref.val_crc32(p, L), L)
    vc.set_provider_min_bytes(-1)
    dflt = per_call(lambda: lib.val_gpu_crc32_provider(0xFFFFFFFF, p, L), L)
    rows.append((L, gpu, cpu))
    print(f"{L:10d} {gpu:9.2f} {cpu:9.2f} {s16:9.2f} {r:9.2f} {dflt:10.2f}  {L / gpu / 1e3:8.2f}  {L / cpu / 1e3:8.2f}",
          flush=True)
cross = None
for i, (L, gpu, cpu) in enumerate(rows):
    if all(g < c for _, g, c in rows[i:]):
        cross = L
        break
print(f"crossover (GPU faster from here on): {cross}", flush=True)
