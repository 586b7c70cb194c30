#!/usr/bin/env python3
"""A/B two builds of libval_crc_hip.so in one process on the same inputs:
interleaved timing of val_crc32_frames_dev (tooling only, not the product).
usage: ab_libs.py LIB_A LIB_B [cfg3|cfg3b|cfg5|cfg5log|u57]..."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import val_protocol_amd.crc as vc  # noqa: E402


def load(path):
    l = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    vc._declare(l, strict=False)
    return l


def time_it(fn, reps=10):
    """(median, min) ms of fn on the current stream, one event pair per call."""
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(np.min(ts))


def workload(name, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    if name in ("cfg2", "cfg4", "w256"):  # bench layouts: 64 K x 1,040 B; 131,113 x 65,532 B; 256-frame window
        n, L = {"cfg2": (1 << 16, 1040), "cfg4": (131113, 65532), "w256": (256, 1040)}[name]
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        return dict(buf=buf, stride=L + 4, flen=L, n=n), n * L
    if name == "cfg3d":  # cfg3's layout (1 M x 16,400 B at stride 16,404) through descriptors with the hint
        n, L = 1 << 20, 16400
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(n, device=dev, dtype=torch.int64) * (L + 4)
        return dict(buf=buf, off=off, length=torch.full((n,), L, dtype=torch.int32, device=dev), len_hint=L), n * L
    if name == "cfg4d":  # cfg4 as bench.py launches it: descriptors with the uniform length hint
        n, L = 131113, 65532
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(n, device=dev, dtype=torch.int64) * (L + 4)
        return dict(buf=buf, off=off, length=torch.full((n,), L, dtype=torch.int32, device=dev), len_hint=L), n * L
    if name.startswith("t") and name[1:].isdigit():  # tNNNNN: a cfg4 slice, NNNNN x 65,532 B, the last 816 B,
        n, L = int(name[1:]), 65532                    # descriptors with the uniform hint (bench.py's slices)
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(n, device=dev, dtype=torch.int64) * (L + 4)
        length = torch.full((n,), L, dtype=torch.int32, device=dev)
        length[-1] = 816
        return dict(buf=buf, off=off, length=length, len_hint=L), int(length.long().sum().item())
    if name in ("cfg3", "cfg3b"):  # cfg3b: the bench layout (flen 16400, stride 16404)
        n, L = 1 << 20, (16384 - 4 if name == "cfg3" else 16400)
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        return dict(buf=buf, stride=L + 4, flen=L, n=n), n * L
    if name.startswith("w") and "x" in name:  # wNNNxLLLLL: a window of NNN strided frames of LLLLL CRC bytes
        n, L = (int(v) for v in name[1:].split("x"))
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        return dict(buf=buf, stride=L + 4, flen=L, n=n), n * L
    if name.startswith("d") and "x" in name:  # dNNNxLLLLL: NNN frames of LLLLL CRC bytes, descriptors with the hint
        n, L = (int(v) for v in name[1:].split("x"))
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        off = torch.arange(n, device=dev, dtype=torch.int64) * (L + 4)
        return dict(buf=buf, off=off, length=torch.full((n,), L, dtype=torch.int32, device=dev), len_hint=L), n * L
    if name.startswith("s") and name[1:].isdigit():  # sNNNNN: 1 M strided frames of NNNNN CRC bytes, stride +4
        n, L = 1 << 20, int(name[1:])
        buf = torch.randint(0, 256, (n * (L + 4),), dtype=torch.uint8, device=dev, generator=g)
        return dict(buf=buf, stride=L + 4, flen=L, n=n), n * L
    if name == "cfg5log":  # bench.py cfg5: log-uniform payloads with DATA headers (rank 0 sample)
        import bench

        buf, off, length = bench.make_ragged_frames(torch, dev, bench.CONFIGS["cfg5"][0], seed=1234)
        return dict(buf=buf, off=off, length=length, len_hint=0), int(length.long().sum().item())
    rng = np.random.default_rng(1)
    if name == "cfg5":
        lens = rng.integers(520, 65533, 262144)
    elif name == "u57":
        lens = np.full(56508, 57000)
    elif name in ("c2h", "c2s"):  # c2's lengths through the uniform kernels (len_hint 16384), or sorted in memory
        lens = np.exp(rng.uniform(np.log(8192), np.log(49151), 150000)).astype(np.int64)
        if name == "c2s":
            lens = np.sort(lens)[::-1].copy()
    elif name in ("c2", "c2a", "c2b", "c2d"):  # class-2 log-uniform mix, variants by alignment:
        # c2a: L = 12 mod 16 (frame starts 16-B aligned, units 12 mod 16, no tail bytes);
        # c2b: L = 0 mod 4 (no tail bytes, units at random 16-B phase);
        # c2d: as c2a with the stream shifted by 4 B (units 16-B aligned, no tail bytes)
        lens = np.exp(rng.uniform(np.log(8192), np.log(49151), 150000)).astype(np.int64)
        if name in ("c2a", "c2d"):
            lens = (lens // 16) * 16 + 12
        elif name == "c2b":
            lens = (lens // 4) * 4
    elif name.startswith("u") and name.rstrip("d")[1:].isdigit():  # uNNNN: uniform length NNNN, ragged path;
        L = int(name.rstrip("d")[1:])                              # uNNNNd: same, descriptor-uniform (len_hint)
        lens = np.full(max(1, (3 << 30) // (L + 4)), L)
    else:
        raise SystemExit(name)
    wire = lens + 4
    off = np.concatenate([[0], np.cumsum(wire)[:-1]]) + (4 if name == "c2d" else 0)
    buf = torch.randint(0, 256, (int(wire.sum()) + 4,), dtype=torch.uint8, device=dev, generator=g)
    return dict(buf=buf, off=torch.from_numpy(off.astype(np.int64)).to(dev),
                length=torch.from_numpy(lens.astype(np.int32)).to(dev),
                len_hint=16384 if name == "c2h" else int(lens[0]) if name.endswith("d") else 0), int(lens.sum())


def main():
    """usage: ab_libs.py LIB_A LIB_B [LIB_C ...] [workload ...]: B, C, ... against A."""
    dev = torch.device("cuda:0")
    paths = [a for a in sys.argv[1:] if a.endswith(".so")]
    names = [a for a in sys.argv[1:] if not a.endswith(".so")]
    libs = [load(p) for p in paths]
    for l in libs:
        assert l.val_gpu_init(0) == 0
    for name in names or ["cfg3", "cfg5"]:
        w, nbytes = workload(name, dev)
        outs = []
        res = [[] for _ in libs]
        for rep in range(4):
            for i, l in enumerate(libs):
                vc._lib = l
                out = torch.empty(w.get("n") or w["length"].numel(), dtype=torch.int32, device=dev)
                hdr = torch.empty_like(out) if os.environ.get("AB_HDR") == "1" else None  # header_crc too
                if "off" in w:
                    fn = lambda: vc.frames(w["buf"], off=w["off"], length=w["length"], out_crc=out, out_hdr=hdr,
                                           len_hint=w["len_hint"])
                else:
                    fn = lambda: vc.frames(w["buf"], stride=w["stride"], flen=w["flen"], n=w["n"], out_crc=out,
                                           out_hdr=hdr)
                med, _ = time_it(fn, reps=10)
                res[i].append(med)
                if rep == 0:
                    outs.append(out.clone() if hdr is None else torch.cat([out, hdr]))
        a = np.median(res[0])
        line = f"{name}: A {a:.4f} ms ({nbytes / a / 1e6:.0f} GB/s)"
        for i in range(1, len(libs)):
            b = np.median(res[i])
            line += (f"  {chr(65 + i)} {b:.4f} ms speed {a / b:.3f} same={bool(torch.equal(outs[0], outs[i]))}")
        print(line, " ", [["%.3f" % x for x in r] for r in res], flush=True)


if __name__ == "__main__":
    main()
