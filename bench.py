#!/usr/bin/env python3
"""Headline benchmark: device-resident trailer CRC-32 (+ header_crc) over
batched VAL DATA frames on MI355X (BASELINE.json metric, configs[2] = cfg3:
1 M DATA frames x 16 KiB payload, header_crc + trailer CRC-32).

One step = one launch of the fused frames kernel over the whole batch already
resident in HBM. N GPUs (torchrun, one rank per GPU): every rank hashes its
own 1 M-frame batch (frames are independent -> weak scaling, no collective on
the data path; the only collectives are the timing barrier/max).

Prints ONE JSON line on rank 0. Extra diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md

CONFIGS = {
    # name: (frames per GPU, payload bytes, explicit offset, header_crc); cfg5 is ragged (make_ragged_frames)
    "cfg3": (1 << 20, 16384, True, True),
    "cfg2": (1 << 16, 1024, True, False),
    "cfg4": (131113, 65516, True, False),
    "cfg5": (262144, 0, True, True),
}
CFG5_MIN, CFG5_MAX = 512, 65516  # payload bytes, log-uniform (BASELINE configs[4])
CFG4_FILE = 8 << 30  # cfg4: one 8 GiB file at MTU 65,536 -> 131,112 x 65,516 B + a last frame of 800 B


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=15)  # the first ~10 cfg3 launches run 1-4% slower (clocks settling)
    ap.add_argument("--config", default="cfg3", choices=sorted(CONFIGS))
    ap.add_argument("--verify", action="store_true", help="time the RX verify kernel instead of TX")
    ap.add_argument("--pay", action="store_true", help="with --verify: also emit payload states (RX file-CRC by-product)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores)")
    ap.add_argument("--no-host-inclusive", action="store_true",
                    help="skip the host-inclusive block (H2D + kernel + D2H through val_crc32_frames_host)")
    ap.add_argument("--sort-frames", action="store_true", help="cfg5: order descriptors by length (diagnostic)")
    ap.add_argument("--no-cfg4-strong", action="store_true",
                    help="skip the cfg4 strong-scaling block (BASELINE configs[3]) timed after the headline")
    ap.add_argument("--with-cfg4-strong", action="store_true",
                    help="also time the cfg4 strong-scaling block after a weak config other than cfg3 "
                         "(by default only the cfg3 headline line carries it)")
    ap.add_argument("--no-cfg4-proxy", action="store_true",
                    help="N=1: skip the single-GPU proxy of cfg4's 2/4/8-GPU slices after the cfg4 block")
    ap.add_argument("--cfg4-alloc-first", action="store_true",
                    help="allocate the cfg4 block's buffer before the headline's (placement A/B)")
    ap.add_argument("--block-warmup-ms", type=float, default=100.0,
                    help="cfg4 block: after its --warmup launches, further untimed launches up to this much GPU "
                         "time (the block follows ~20 s of host-side work with the GPU idle; with 5 launches of "
                         "warm-up it ran 1%% slower than cfg4 alone, with 100 ms 0.5%% faster: "
                         "profiles/r06_ab_cfg4_block.jsonl)")
    return ap.parse_args()


def make_frames(torch, dev, n, payload, explicit, first_index, seed):
    """Synthetic DATA frames laid out like the reference sender's output
    (src/val_core.c:733-834): [5, flags, LE16 content_len, LE32 0,
    LE64 offset (explicit), payload, LE32 trailer], packed back to back."""
    content = payload + (8 if explicit else 0)
    flen = 8 + content
    stride = flen + 4
    g = torch.Generator(device=dev).manual_seed(seed)
    buf = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device=dev, generator=g)
    buf[:, 0] = 5
    buf[:, 1] = 1 if explicit else 0
    buf[:, 2] = content & 0xFF
    buf[:, 3] = content >> 8
    buf[:, 4:8] = 0
    if explicit:
        offs = (torch.arange(n, device=dev, dtype=torch.int64) + first_index) * payload
        buf[:, 8:16] = offs.view(torch.uint8).view(n, 8)
    buf[:, flen:] = 0
    return buf, flen, stride


def make_ragged_frames(torch, dev, n, seed):
    """cfg5: n DATA frames, payload log-uniform in [512, 65516], one in 8 with
    an implied offset (content = payload, src/val_sender.c:833), packed back to
    back so frame starts are byte-unaligned. Returns (stream, off, len) with
    off/len as GPU tensors (int64 / int32) and len = CRC input bytes."""
    rng = np.random.default_rng(seed)
    pay = np.exp(rng.uniform(np.log(CFG5_MIN), np.log(CFG5_MAX), n)).astype(np.int64)
    explicit = (np.arange(n) % 8) != 7
    content = pay + 8 * explicit
    crc_len = 8 + content
    wire = crc_len + 4
    off = np.concatenate([[0], np.cumsum(wire)[:-1]]).astype(np.int64)
    total = int(wire.sum())
    g = torch.Generator(device=dev).manual_seed(seed)
    buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    hdr = np.zeros((n, 8), np.uint8)
    hdr[:, 0] = 5
    hdr[:, 1] = explicit.astype(np.uint8)
    hdr[:, 2] = content & 0xFF
    hdr[:, 3] = content >> 8
    d_off = torch.from_numpy(off).to(dev)
    idx = (d_off[:, None] + torch.arange(8, device=dev)[None, :]).reshape(-1)
    buf[idx] = torch.from_numpy(hdr.reshape(-1)).to(dev)
    file_off = np.concatenate([[0], np.cumsum(pay)[:-1]]).astype(np.int64)
    ex = np.nonzero(explicit)[0]
    idx = (d_off[ex][:, None] + 8 + torch.arange(8, device=dev)[None, :]).reshape(-1)
    buf[idx] = torch.from_numpy(file_off[ex].astype("<i8").view(np.uint8)).to(dev)
    return buf, d_off, torch.from_numpy(crc_len.astype(np.int32)).to(dev)


def effective_cpus() -> tuple[int, int]:
    """(CPUs this process may run on, CPUs its cgroup quota pays for): the
    affinity set, and ceil(quota / period) from cgroup v2 cpu.max (v1:
    cpu.cfs_quota_us / cpu.cfs_period_us) when a quota is set. A GPU box
    shows every CPU of the machine in its affinity set but grants one GPU's
    share (16) through the quota."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = float(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = float(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    eff = visible if quota is None else max(1, min(visible, int(-(-quota // 1))))
    return visible, eff


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sample: np.ndarray, n: int, threads: int, stride: int = 0, flen: int = 0, off=None, length=None,
                 all_threads: int = 0):
    """Time the reference's own val_crc32 (oracle/_ref/libref_bench.so, built
    from /root/reference/src/val_core.c:150-160) -- or the oracle port if that
    build is absent -- over a host copy of `n` frames of the same workload:
    on 1 thread, on `threads` threads and on `all_threads` (every core this
    process may run on; frames round-robin over pthreads).
    Returns (GiB/s at `threads`, GiB/s on 1 thread, kind, outputs, detail,
    GiB/s on all_threads)."""
    kind = "reference"
    so = os.path.join(ROOT, "oracle", "_ref", "libref_bench.so")
    out = np.zeros(n, np.uint32)
    vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        nbytes = int(length.astype(np.int64).sum())
    else:
        nbytes = n * flen
    if os.path.exists(so):
        lib = ctypes.CDLL(so)
        if off is not None:
            fn = lib.ref_bench_frames_desc
            fn.argtypes = [vp, vp, vp, u64, vp, ci]
            run = lambda t: fn(sample.ctypes.data, off.ctypes.data, length.ctypes.data, n, out.ctypes.data, t)  # noqa: E731
        else:
            fn = lib.ref_bench_frames
            fn.argtypes = [vp, u64, u32, u64, vp, ci]
            run = lambda t: fn(sample.ctypes.data, stride, flen, n, out.ctypes.data, t)  # noqa: E731
    else:
        kind = "port"
        from tests import _oracle

        if off is not None:
            run = lambda t: _oracle.lib().oracle_crc32_frames(sample.ctypes.data, off.ctypes.data,  # noqa: E731
                                                              length.ctypes.data, n, out.ctypes.data, None, t)
        else:
            run = lambda t: _oracle.lib().oracle_crc32_frames_strided(sample.ctypes.data, stride, flen, n,  # noqa: E731
                                                                      out.ctypes.data, None, t)

    def rate(t, cpu_s, wall_s):
        run(t)  # warm caches/pages
        reps, tt = 0, 0.0
        while True:  # >= cpu_s of CPU (thread) time or >= wall_s of wall time
            t0 = time.perf_counter()
            run(t)
            tt += time.perf_counter() - t0
            reps += 1
            if tt * t >= cpu_s or tt >= wall_s:
                break
        return reps * nbytes / tt / GIB, reps

    one, reps1 = rate(1, 3.0, 3.0)
    many, reps = rate(threads, 10.0, 4.0)
    allc, repsa = rate(all_threads, 10.0, 4.0) if all_threads and all_threads != threads else (many, reps)
    return (many, one, kind, out, f"x{reps} reps on {threads} threads, x{repsa} on {all_threads or threads}, "
            f"x{reps1} on 1 thread", allc)


def read_pmc_traffic(config: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this
    workload (profiles/pmc_<config>.json, tools/pmc_traffic.py) and where it
    came from. PMC counters need their own rocprofv3 passes, so the number is
    never measured by this run: `traffic_source` names the file, the tree and
    box it was measured on, and whether the library this run loaded was built
    from the same sources (val_protocol_amd/libval_crc_hip.so.srchash)."""
    rel = os.path.join("profiles", f"pmc_{config}.json")
    try:
        with open(os.path.join(ROOT, rel)) as f:
            d = json.load(f)
    except Exception:
        return None, None
    src = dict(d.get("source") or {})
    try:
        with open(os.path.join(ROOT, "val_protocol_amd", "libval_crc_hip.so.srchash")) as f:
            mine = f.read().strip()
    except OSError:
        mine = None
    src.update({"file": rel, "measured_in_this_run": False,
                "same_library_sources": bool(mine) and src.get("lib_srchash") == mine})
    return d.get("hbm_bytes_per_launch"), src


def read_roof(torch, flat, stream):
    """Same-box achievable read rate (GB/s): a plain read-only stream over this
    run's frame buffer (bench/roof.hip, built by __graft_entry__.build()), timed
    with events on the stream it runs on. None if the helper is not built."""
    so = os.path.join(ROOT, "bench", "libval_roof.so")
    if not os.path.exists(so):
        return None
    lib = ctypes.CDLL(so)
    lib.val_bench_read_roof.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    lib.val_bench_read_roof.restype = ctypes.c_int
    sink = torch.zeros(1, dtype=torch.int32, device=flat.device)
    nbytes = (flat.numel() // 128) * 128
    go = lambda: lib.val_bench_read_roof(flat.data_ptr(), nbytes, sink.data_ptr(), stream.cuda_stream)  # noqa: E731
    if go() != 0:
        return None
    torch.cuda.synchronize()
    ms = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        go()
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    return nbytes / (float(np.median(ms)) * 1e-3) / 1e9


def host_inclusive(vc, w, slice_bytes=1 << 30, reps=3):
    """The path as VAL runs it: frames in host memory (the transport's byte
    stream), CRCs back in host memory. A >= 1 GiB slice of this run's own
    frames (CRC input) goes through the C-ABI host call
    val_crc32_frames_host from pinned memory (val_gpu_host_alloc: DMA in
    place) and from pageable memory (bounced through pinned buffers): H2D in
    64 MiB chunks overlapped with the kernel, then one D2H of the results.
    Best of `reps` timed calls after one warm call; outputs are checked
    against the device-resident launch's CRCs of the same frames."""
    import torch

    n, desc = w["n"], w["desc"]
    if desc:
        offs = w["d_off"].cpu().numpy().astype(np.uint64)
        lens = w["d_len"].cpu().numpy().astype(np.uint32)
        ends = offs + lens.astype(np.uint64)
        cum = np.cumsum(lens.astype(np.int64))
        ns = int(min(n, np.searchsorted(cum, slice_bytes) + 1))
        span = int(ends[:ns].max()) + 4
        host = w["flat"][:span].cpu().numpy()
        kw = dict(off=offs[:ns], length=lens[:ns])
        crc_bytes = int(cum[ns - 1])
    else:
        flen = w["flen"]
        ns = int(min(n, -(-slice_bytes // flen)))
        host = w["buf"][:ns].cpu().numpy().reshape(-1)
        kw = dict(stride=w["stride"], flen=flen, n=ns)
        crc_bytes = ns * flen
    want = w["crc"][:ns].cpu().numpy().view(np.uint32)
    pinned = vc.PinnedBuffer(host.size)
    pinned.array[:] = host
    before = vc.cpu_batch_count()
    out = {"slice_frames": ns, "slice_crc_input_bytes": crc_bytes, "slice_wire_bytes": int(host.size),
           "chunk_bytes": 64 << 20, "unit": "GiB/s", "reps": reps,
           "path": "val_crc32_frames_host: H2D (64 MiB chunks on a copy stream, overlapped with the kernel) + "
                   "kernel + D2H of the CRCs; GiB/s of CRC input, best of reps"}
    ok = True
    for kind, arr in (("pinned", pinned.array), ("pageable", host)):
        crc = vc.frames_host(arr, **kw)  # warm: bounce buffers, descriptors
        ok = ok and bool(np.array_equal(crc, want))
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            vc.frames_host(arr, **kw)
            best = min(best, time.perf_counter() - t0)
        out[kind] = round(crc_bytes / best / GIB, 2)
        out[f"{kind}_ms"] = round(best * 1e3, 3)
    pinned.free()
    torch.cuda.synchronize()
    out["value"] = out["pinned"]
    out["outputs_equal_device"] = ok
    out["on_gpu"] = vc.cpu_batch_count() == before  # no call was routed to the CPU engine
    print(f"[bench] host-inclusive: pinned {out['pinned']} GiB/s, pageable {out['pageable']} GiB/s "
          f"({ns} frames, {crc_bytes / GIB:.2f} GiB)", file=sys.stderr)
    return out


def build_workload(torch, dev, config, rank, world, verify, vc):
    """Frames of `config` for this rank, resident in HBM. cfg4 is one 8 GiB
    file sharded across the ranks (BASELINE configs[3]): contiguous frame
    ranges balanced by bytes, no collective on the data path (strong
    scaling); the other configs give every rank its own batch (weak)."""
    n, payload, explicit, header = CONFIGS[config]
    strong = config == "cfg4"
    n_total, first = n, rank * n
    if strong:
        from val_protocol_amd.shard import shard_frames

        first, n = shard_frames(n_total, world, rank)
    ragged = config == "cfg5"
    d_off = d_len = None
    if ragged:
        buf, d_off, d_len = make_ragged_frames(torch, dev, n, seed=1234 + rank)
        flen, stride = 0, 0
        flat = buf
        len_hint = 0  # mixed lengths: the library bins frames by length class on the device
    else:
        buf, flen, stride = make_frames(torch, dev, n, payload, explicit, first, seed=1234 + rank)
        flat = buf.view(-1)
        len_hint = flen
        if strong:
            # the file's last frame carries the 800-B remainder: descriptor
            # mode with the uniform geometry hint; only the rank holding it differs
            last_pay = CFG4_FILE - (n_total - 1) * payload
            d_off = torch.arange(n, device=dev, dtype=torch.int64) * stride
            d_len = torch.full((n,), flen, dtype=torch.int32, device=dev)
            if n and first + n == n_total:
                content = last_pay + (8 if explicit else 0)
                buf[n - 1, 2], buf[n - 1, 3] = content & 0xFF, content >> 8
                d_len[n - 1] = 8 + content
    desc = ragged or strong
    kw = dict(off=d_off, length=d_len, n=n, len_hint=len_hint) if desc else dict(stride=stride, flen=flen, n=n)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n, dtype=torch.int32, device=dev) if header else None
    if verify:  # trailers must be valid first
        vc.frames(flat, out_crc=crc, **kw)
        if desc:
            tidx = ((d_off + d_len.long())[:, None] + torch.arange(4, device=dev)[None, :]).reshape(-1)
            flat[tidx] = crc.view(torch.uint8)
        else:
            buf[:, flen:flen + 4] = crc.view(torch.uint8).view(n, 4)
    bytes_per_launch = int(d_len.long().sum().item()) if desc else n * flen
    # the whole job's CRC input per step: cfg4's one file, else every rank's own batch
    file_crc_input = (n_total - 1) * (8 + payload + (8 if explicit else 0)) + 8 + (CFG4_FILE - (n_total - 1) * payload) \
        + (8 if explicit else 0)
    return dict(config=config, n=n, n_total=n_total, first=first, payload=payload, explicit=explicit, header=header,
                strong=strong, ragged=ragged, desc=desc, buf=buf, flat=flat, flen=flen, stride=stride,
                d_off=d_off, d_len=d_len, len_hint=len_hint, kw=kw, crc=crc, hdr=hdr,
                bytes_per_launch=bytes_per_launch, job_bytes=file_crc_input if strong else None)


def timed_steps(torch, dist, world, step, steps, warmup, stream):
    """W untimed steps, then K steps bracketed by a barrier and a device
    synchronise on both sides. Two HIP events bracket the K launches on
    their stream: the launches run back to back as in a real window stream
    (events between every step, as until round 3, put an event command
    between the kernels: about 7 us per step, 0.3% of cfg3 and a fifth of
    cfg2's 19 us launches). Returns (wall seconds, kernel ms per step = the
    events' span over K, gaps between the launches included)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, ev0.elapsed_time(ev1) / steps


def max_over_ranks(torch, dist, world, value, dev, backend):
    t = torch.tensor([value], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def parity_sample(torch, w, rank, verify, nbad):
    """This run's outputs against the oracle on a sample of frames (untimed)."""
    from tests import _oracle

    n, dev = w["n"], w["flat"].device
    sample_idx = np.unique(np.concatenate([np.random.default_rng(rank).choice(n, min(n, 256), replace=False),
                                           [0, n - 1]]))
    if w["desc"]:
        o = w["d_off"].cpu().numpy()[sample_idx]
        l = w["d_len"].cpu().numpy()[sample_idx].astype(np.int64)
        pieces = [w["flat"][int(a):int(a) + int(b)].cpu().numpy() for a, b in zip(o, l)]
        rows = np.concatenate(pieces)
        so = np.concatenate([[0], np.cumsum(l)[:-1]]).astype(np.uint64)
        want = _oracle.frames(rows, so, l.astype(np.uint32))
    else:
        rows = w["buf"][torch.from_numpy(sample_idx).to(dev)].cpu().numpy().reshape(-1)
        want = _oracle.frames_strided(rows, w["stride"], w["flen"], sample_idx.size)
    got = w["crc"].cpu().numpy().view(np.uint32)[sample_idx] if not verify else want
    ok = bool(np.array_equal(got, want))
    if verify:
        ok = ok and int(nbad.item()) == 0
    return ok


def rank_record(w, rank, gpu, steps, elapsed, kern_ms, parity):
    b = w["bytes_per_launch"]
    return {"rank": rank, "device": gpu, "frames": w["n"], "bytes_per_step": b,
            "kernel_ms": round(kern_ms, 4), "elapsed_s": round(elapsed, 6),
            "GiB_s": round(b * steps / elapsed / GIB, 2),
            "kernel_GiB_s": round(b / (kern_ms * 1e-3) / GIB, 2), "parity_sample_ok": parity,
            "last_frame_crc_input": int(w["d_len"][w["n"] - 1].item()) if w["desc"] and w["n"] else w["flen"]}


def gather(dist, world, mine):
    if not dist.is_initialized():
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


def aggregate(per_rank, total_bytes, elapsed_max):
    return {"total_bytes": total_bytes, "max_elapsed_s": round(elapsed_max, 6),
            "slowest_rank": max(per_rank, key=lambda r: r["elapsed_s"])["rank"],
            "sum_of_rank_GiB_s": round(sum(r["GiB_s"] for r in per_rank), 2)}


def verify_windows(torch, vc, flat, dev, stream):
    """VAL_RESUME_TAIL verify-window CRC: region windows
    over the cfg5 stream, timed with HIP events on the launch stream. Each
    size cycles over distinct windows spanning >= 1 GiB of the stream (or all
    of it), more than the 256 MiB Infinity Cache, so no call re-reads bytes a
    recent call left in a cache: the 8 MiB and 256 MiB rates are HBM rates.
    Windows under 1 MiB are launch-bound; they take 128 windows spread over
    the stream. The first and last window of each size are checked against
    the oracle. Reported beside the frames number, never as `value`."""
    from tests import _oracle

    nb = int(flat.numel())
    out = []
    for wlen in (1 << 10, 8 << 10, 8 << 20, 256 << 20):
        wlen = min(wlen, nb)
        if wlen >= (1 << 20):
            k = max(1, min(-(-(1 << 30) // wlen), nb // wlen))
            starts = [j * wlen for j in range(k)]
            span = k * wlen
        else:
            k = 128
            gap = max(wlen, (nb - wlen) // k)
            starts = [j * gap for j in range(k)]
            span = k * wlen
        reps = max(len(starts), 200 if wlen < (1 << 20) else 2 * len(starts))
        st_out = torch.empty(1, dtype=torch.int32, device=dev)
        vc.region(flat[starts[-1]:starts[-1] + wlen], out=st_out)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for r in range(reps):
            o = starts[r % len(starts)]
            vc.region(flat[o:o + wlen], out=st_out)
        b.record(stream)
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / reps
        ok = True
        for o in (starts[0], starts[-1]):
            vc.region(flat[o:o + wlen], out=st_out)
            torch.cuda.synchronize()
            ok = ok and ((int(st_out.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF) == _oracle.crc32(flat[o:o + wlen].cpu().numpy())
        out.append({"bytes": wlen, "us": round(us, 2), "GiB_s": round(wlen / (us * 1e-6) / GIB, 1),
                    "distinct_windows": len(starts), "bytes_cycled": span, "calls": reps, "crc_ok": ok})
    return out


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_launch_command(n: int, argv: list, port: int) -> list:
    """The one-process-per-GPU command `bench.py --gpus N` starts for N > 1
    when it was not launched under torch.distributed.run: the same script and
    arguments under torchrun, N ranks on this node, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def launch_ranks(n: int, backend: str) -> int:
    """`bench.py --gpus N` (N > 1) run as a plain process: start the N ranks
    as a fresh child process (torch.distributed.run), wait for it and return
    its exit status. Decided before this process touches the GPU (the device
    count below does not initialise it) and never by exec: the ranks are a
    child, their JSON line reaches the caller on the inherited stdout."""
    import signal
    import subprocess

    import torch

    ndev = torch.cuda.device_count()
    if backend == "nccl" and ndev < n:
        print(f"bench.py: --gpus {n} needs {n} visible GPUs for the nccl (RCCL) backend, found {ndev}; one rank "
              f"per GPU (VAL_BENCH_BACKEND=gloo rehearses several ranks on one GPU)", file=sys.stderr, flush=True)
        return 2
    env = dict(os.environ, VAL_BENCH_LAUNCHER="bench.py --gpus (torch.distributed.run child)")
    cmd = rank_launch_command(n, sys.argv[1:], _free_port())
    print(f"[bench] starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    child = subprocess.Popen(cmd, env=env)

    def forward(sig, _frame):  # a timeout's SIGTERM to this process ends the ranks too
        child.send_signal(sig)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    return child.wait()


def block_warmup(torch, step, steps, min_ms, stream):
    """Untimed launches before an extra block: `steps` of them, then more
    until at least `min_ms` of GPU time has run (the block follows minutes of
    host-side work with the GPU idle, and its clocks settle over ~30 ms of
    load). Returns the number of launches run."""
    done = 0
    for _ in range(steps):
        step()
        done += 1
    if min_ms <= 0:
        torch.cuda.synchronize()
        return done
    spent = 0.0
    while spent < min_ms:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(4):
            step()
        b.record(stream)
        torch.cuda.synchronize()
        spent += a.elapsed_time(b)
        done += 4
    return done


def roofline_block(nbytes, kern_ms, roof):
    achieved = nbytes / (kern_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel_ms": round(kern_ms, 4), "bytes_per_launch": nbytes,
            "read_roof": round(roof, 1) if roof else None,
            "frac_of_read_roof": round(achieved / roof, 4) if roof else None,
            "read_roof_frac_of_peak": round(roof / HBM_PEAK_GBS, 4) if roof else None}


def cfg4_strong_proxy(torch, dist, vc, w4, stream, steps, warmup, block_kern_ms):
    """Single-GPU proxy of cfg4's 1/2/4/8-GPU strong-scaling curve (north_star:
    "absolute GiB/s at 1/2/4/8 GPUs"; no multi-GPU node is available to this
    run). For each N the file is split exactly as N ranks split it
    (val_shard_frames), and on this one GPU the largest slice and the last
    rank's slice (it holds the 800-B tail frame) are each timed alone, like the
    block: untimed launches (W, and at least 20 ms), K back-to-back launches
    between two events on the launch stream; two alternating passes, the
    faster one counts. Each N's estimated aggregate = the file's CRC input /
    the slower of the two slice times: what N GPUs that each run like this one
    would reach, without node-level effects (placement, PCIe/xGMI, clocks)."""
    from val_protocol_amd.shard import shard_frames

    n_total, stride, flen = w4["n_total"], w4["stride"], w4["flen"]
    job = w4["job_bytes"]
    out = {"label": "single-GPU proxy; no multi-GPU node: each N's slices timed alone on this one GPU",
           "file_crc_input_bytes": job, "unit": "GiB/s",
           "1": {"frames": n_total, "kernel_ms": round(block_kern_ms, 4),
                 "GiB_s_per_gpu": round(job / (block_kern_ms * 1e-3) / GIB, 2),
                 "est_aggregate_GiB_s": round(job / (block_kern_ms * 1e-3) / GIB, 2), "source": "cfg4_strong block"}}
    for nr in (2, 4, 8):
        shards = [shard_frames(n_total, nr, r) for r in range(nr)]
        big = max(range(nr), key=lambda r: (shards[r][1], -r))
        cases = []
        for r in sorted({big, nr - 1}):
            first, cnt = shards[r]
            view = w4["flat"][first * stride:(first + cnt) * stride]
            ln = w4["d_len"][first:first + cnt]
            off = w4["d_off"][:cnt]  # uniform stride: a slice's offsets from its own base are the first cnt
            crc = torch.empty(cnt, dtype=torch.int32, device=view.device)
            step = (lambda v, o, l, c, k: lambda: vc.frames(v, off=o, length=l, n=k, len_hint=flen, out_crc=c))(
                view, off, ln, crc, cnt)
            cases.append((r, first, cnt, view, off, ln, crc, step))
        # two passes over the slices, alternating, each after >= 20 ms of untimed launches: a slice's
        # time is the faster pass (single passes on one box varied by up to 35%: one clock or
        # placement hiccup decided a slice's number)
        times = {c[0]: [] for c in cases}
        for rep in range(2):
            for c in (cases if rep == 0 else cases[::-1]):
                block_warmup(torch, c[7], warmup, 20.0, stream)
                _, km = timed_steps(torch, dist, 1, c[7], steps, 0, stream)
                times[c[0]].append(round(km, 4))
        slices = []
        for r, first, cnt, view, off, ln, crc, step in cases:
            km = min(times[r])
            sw = {"n": cnt, "flat": view, "desc": True, "d_off": off, "d_len": ln, "crc": crc}
            ok = parity_sample(torch, sw, r, False, None)
            nbytes = int(ln.long().sum().item())
            slices.append({"rank": r, "frames": cnt, "bytes": nbytes, "kernel_ms": km, "kernel_ms_passes": times[r],
                           "GiB_s_per_gpu": round(nbytes / (km * 1e-3) / GIB, 2), "parity_sample_ok": ok,
                           "last_frame_crc_input": int(ln[cnt - 1].item())})
        slow = max(s["kernel_ms"] for s in slices)
        out[str(nr)] = {"frames": max(s["frames"] for s in slices), "kernel_ms": slow,
                        "GiB_s_per_gpu": min(s["GiB_s_per_gpu"] for s in slices),
                        "est_aggregate_GiB_s": round(job / (slow * 1e-3) / GIB, 2),
                        "slices_timed": slices}
    out["parity_sample_ok"] = all(s["parity_sample_ok"] for k in ("2", "4", "8") for s in out[k]["slices_timed"])
    return out


def main():
    args = parse()
    backend = os.environ.get("VAL_BENCH_BACKEND", "nccl")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, backend))
    world = int(env_world or "1")
    if args.gpus < 1 or world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: the launcher started a different number of "
              f"ranks than the run asks for", file=sys.stderr, flush=True)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()  # counts devices without initialising the GPU
    if world > 1 and backend == "nccl" and ndev < world:
        print(f"bench.py: WORLD_SIZE={world} ranks need {world} visible GPUs for the nccl (RCCL) backend, "
              f"found {ndev}; one rank per GPU (VAL_BENCH_BACKEND=gloo rehearses several ranks on one GPU)",
              file=sys.stderr, flush=True)
        sys.exit(2)
    gpu = local % max(ndev, 1)  # == local on a full node; with gloo a 1-GPU box rehearses N ranks
    # VAL_BENCH_FORCE_DIST=1: a process group even for one rank (the RCCL path
    # on a one-GPU box: init, barriers, all_reduce, all_gather_object)
    if world > 1 or os.environ.get("VAL_BENCH_FORCE_DIST") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{gpu}")
    torch.cuda.set_device(dev)

    import val_protocol_amd.crc as vc

    vc.init(gpu)
    want_strong = (args.config == "cfg3" or args.with_cfg4_strong) and not args.no_cfg4_strong \
        and args.config != "cfg4" and not args.verify and not args.sort_frames
    # --cfg4-alloc-first: the cfg4 block's buffer is placed before the headline's (diagnostic A/B)
    w4 = build_workload(torch, dev, "cfg4", rank, world, False, vc) if want_strong and args.cfg4_alloc_first else None
    w = build_workload(torch, dev, args.config, rank, world, args.verify, vc)
    if w["ragged"] and args.sort_frames:
        perm = torch.argsort(w["d_len"])
        w["d_off"], w["d_len"] = w["d_off"][perm].contiguous(), w["d_len"][perm].contiguous()
        w["kw"].update(off=w["d_off"], length=w["d_len"])
    n, n_total, strong, ragged, header = w["n"], w["n_total"], w["strong"], w["ragged"], w["header"]
    flat, buf, flen, stride, kw = w["flat"], w["buf"], w["flen"], w["stride"], w["kw"]
    crc, hdr = w["crc"], w["hdr"]
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    pay = torch.empty(n, dtype=torch.int32, device=dev) if args.pay else None
    nbad = torch.zeros(1, dtype=torch.int32, device=dev)

    # Batches smaller than the 256 MiB Infinity Cache (cfg2: 68 MB) would be
    # re-read from it by back-to-back steps. A real window stream hashes new
    # frames every call, so such batches rotate over identical copies spanning
    # at least 1 GiB: every step reads its bytes from HBM.
    nb = flat.numel()
    rot = min(16, max(1, -(-(1 << 30) // max(nb, 1))))
    flats = [flat] + [flat.clone() for _ in range(rot - 1)]
    turn = [0]

    def step():
        src = flats[turn[0] % rot]
        turn[0] += 1
        if args.verify and args.pay:
            vc.verify_frames_ex(src, out_ok=ok, nbad=nbad, out_hdr=hdr, out_pay=pay, **kw)
        elif args.verify:
            vc.verify_frames(src, out_ok=ok, nbad=nbad, out_hdr=hdr, **kw)
        else:
            vc.frames(src, out_crc=crc, out_hdr=hdr, **kw)

    stream = torch.cuda.current_stream()
    elapsed, kern_ms = timed_steps(torch, dist, world, step, args.steps, args.warmup, stream)
    # per-step spread, from a short untimed pass with an event pair per step
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(min(args.steps, 5))]
    for a, b in evs:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    print("[bench] per-step ms (untimed pass): " + " ".join(f"{a.elapsed_time(b):.4f}" for a, b in evs), file=sys.stderr)
    elapsed_max = max_over_ranks(torch, dist, world, elapsed, dev, backend)
    # algorithmic: CRC input of every frame (header_crc is a prefix: +0)
    bytes_per_launch = w["bytes_per_launch"]
    parity = parity_sample(torch, w, rank, args.verify, nbad)
    # Per-rank record (BASELINE configs[3]: "per-GPU and aggregate GiB/s"):
    # each rank's own frames, kernel time by events and wall time between the
    # barriers; gathered on rank 0 (the only other collective of the run).
    per_rank = gather(dist, world, rank_record(w, rank, gpu, args.steps, elapsed, kern_ms, parity))
    total_bytes = (w["job_bytes"] if strong else bytes_per_launch * world) * args.steps
    value = total_bytes / elapsed_max / GIB
    achieved_gbs = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = read_pmc_traffic(args.config + ("_verify" if args.verify else ""))
    roof = read_roof(torch, flat, stream) if rank == 0 else None

    host_incl = None
    if rank == 0 and not args.no_host_inclusive and not args.verify and not args.sort_frames:
        host_incl = host_inclusive(vc, w)

    windows = verify_windows(torch, vc, flat, dev, stream) if ragged and rank == 0 else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.sort_frames:
        visible, effective = effective_cpus()
        threads = args.cpu_threads or min(16, effective)  # the GPU box's CPU share is 16 per GPU
        all_threads = effective  # N = all host cores this process is granted
        if ragged:
            offs_all = w["d_off"].cpu().numpy()
            lens_all = w["d_len"].cpu().numpy().astype(np.uint32)
            ends = offs_all + lens_all.astype(np.int64)
            ns = int(np.searchsorted(ends, 1 << 30, side="right"))  # ~1 GiB of the batch
            ns = max(1, min(ns, n))
            host_rows = flat[: int(ends[ns - 1])].cpu().numpy()
            cgibs, one, kind, cout, detail, call = cpu_baseline(host_rows, ns, threads, off=offs_all[:ns],
                                                                length=lens_all[:ns], all_threads=all_threads)
            sample_bytes = int(lens_all[:ns].astype(np.int64).sum())
        else:
            ns = min(n, max(1, (1 << 30) // flen))  # ~1 GiB host sample of the same frames
            host_rows = buf[:ns].cpu().numpy().reshape(-1)
            cgibs, one, kind, cout, detail, call = cpu_baseline(host_rows, ns, threads, stride=stride, flen=flen,
                                                                all_threads=all_threads)
            sample_bytes = ns * flen
        same = bool(np.array_equal(cout, crc[:ns].cpu().numpy().view(np.uint32))) if not args.verify else None
        cpu = {"value": round(cgibs, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
               "value_1core": round(one, 3), "value_all_cores": round(call, 3), "cores_all": all_threads,
               "cores_effective": effective, "cores_visible": visible, "cpu_model": cpu_model(),
               "sample": f"first {ns} frames of this batch ({sample_bytes / GIB:.2f} GiB of CRC input), "
                         f"reference val_crc32 per frame (src/val_core.c:150-160), frames round-robin over "
                         f"pthreads, {detail}; all cores = the cgroup CPU quota ({effective} of {visible} "
                         f"visible); outputs equal GPU: {same}"}

    # BASELINE configs[3] in the same invocation: one 8 GiB file at MTU
    # 65,536 sharded over the ranks by val_shard_frames (strong scaling),
    # timed like the headline, its own per-rank records and aggregate.
    strong_block = proxy = None
    if want_strong:
        del flats, flat, buf, w, crc, hdr, ok, pay, kw
        torch.cuda.empty_cache()
        if w4 is None:
            w4 = build_workload(torch, dev, "cfg4", rank, world, False, vc)
        step4 = lambda: vc.frames(w4["flat"], out_crc=w4["crc"], **w4["kw"])  # noqa: E731
        warm4 = block_warmup(torch, step4, args.warmup, args.block_warmup_ms, stream)
        el4, km4 = timed_steps(torch, dist, world, step4, args.steps, 0, stream)
        el4_max = max_over_ranks(torch, dist, world, el4, dev, backend)
        par4 = parity_sample(torch, w4, rank, False, None)
        pr4 = gather(dist, world, rank_record(w4, rank, gpu, args.steps, el4, km4, par4))
        tb4 = w4["job_bytes"] * args.steps
        roof4 = read_roof(torch, w4["flat"], stream) if rank == 0 else None
        if rank == 0 and world == 1 and not args.no_cfg4_proxy:
            proxy = cfg4_strong_proxy(torch, dist, vc, w4, stream, args.steps, args.warmup, km4)
        strong_block = {
            "workload": f"cfg4: one {CFG4_FILE >> 30} GiB file as {w4['n_total']} DATA frames of "
                        f"{CONFIGS['cfg4'][1]} B payload (last frame {CFG4_FILE - (w4['n_total'] - 1) * CONFIGS['cfg4'][1]} B), "
                        f"sharded over {world} GPU{'s' if world > 1 else ''} by contiguous byte-balanced frame ranges "
                        f"(val_shard_frames, no collective), trailer CRC-32",
            "scaling": "strong", "value": round(tb4 / el4_max / GIB, 2), "unit": "GiB/s",
            "ms_per_step": round(el4_max / args.steps * 1e3, 4), "steps": args.steps, "warmup_launches": warm4,
            "frames_total": w4["n_total"], "parity_sample_ok": all(r["parity_sample_ok"] for r in pr4),
            # this rank's (rank 0's) slice against the same box's plain read of the same buffer
            "roofline": roofline_block(w4["bytes_per_launch"], km4, roof4) if rank == 0 else None,
            "per_rank": pr4, "aggregate_over_max_rank": aggregate(pr4, tb4, el4_max)}

    if rank == 0:
        metric = "GiB/s device-resident trailer CRC-32 over batched DATA packets, 1 MI355X"
        line = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (device-generated random payloads, reference DATA framing)",
            "config": {
                "workload": (f"{args.config}: {n_total if strong else n} DATA frames x "
                             + (f"{CFG5_MIN}-{CFG5_MAX} B log-uniform payload (1 in 8 implied offset), packed unaligned"
                                if ragged else f"{w_payload(args.config)} B payload"
                                + (f" (last frame {CFG4_FILE - (n_total - 1) * w_payload(args.config)} B: an 8 GiB file)"
                                   if strong else ""))
                             + (f" (one file, sharded over {world} GPU{'s' if world > 1 else ''}), " if strong else " per GPU, ")
                             + f"{'header_crc + ' if header else ''}trailer CRC-32"
                             f"{' (RX verify)' if args.verify else ''}"
                             f"{' + payload states' if args.pay else ''}"),
                "frames_per_gpu": n,
                **({"frames_total": n_total} if strong else {}),
                "crc_input_bytes_per_frame": (bytes_per_launch / n) if ragged else flen,
                "frame_stride": stride if not ragged else "packed",
                "lanes_per_frame": "per length class (2/4/8/16)" if ragged else vc.lanes_per_frame(flen),
                "parallelism": (f"one {n_total}-frame file sharded x{world} by contiguous frame ranges (no collective)"
                                if strong else f"frame-sharded x{world} (no collective)"),
                "parity_sample_ok": parity,
                # copies the steps rotate over (batches under 1 GiB: no step re-reads the
                # previous step's bytes from the Infinity Cache)
                "buffer_copies": rot,
                **({"verify_windows": windows} if windows is not None else {}),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel_ms": round(kern_ms, 4),
                "bytes_per_launch": bytes_per_launch,
                # same box, same buffer: plain read-only stream (bench/roof.hip); SURVEY 8(d)
                "read_roof": round(roof, 1) if roof else None,
                "frac_of_read_roof": round(achieved_gbs / roof, 4) if roof else None,
                # the plain-load roof itself as a share of the spec peak: when it is
                # below 0.80, the 80% target sits above what any read of this buffer
                # reaches on this box
                "read_roof_frac_of_peak": round(roof / HBM_PEAK_GBS, 4) if roof else None,
            },
            "cpu_baseline": cpu,
            # north_star: the path starts and ends in host memory; this is the rate
            # with the H2D and D2H copies (never `value`)
            "host_inclusive": host_incl,
            # per-GPU rates and the aggregate's denominator (BASELINE configs[3])
            "per_rank": per_rank,
            "aggregate_over_max_rank": aggregate(per_rank, total_bytes, elapsed_max),
            **({"cfg4_strong": strong_block} if strong_block is not None else {}),
            **({"cfg4_strong_proxy": proxy} if proxy is not None else {}),
            "launcher": os.environ.get("VAL_BENCH_LAUNCHER",
                                       "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else "single process"),
        }
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def w_payload(config):
    return CONFIGS[config][1]


if __name__ == "__main__":
    main()
