"""World-size-2 runs of the N > 1 paths on one GPU (both ranks on cuda:0,
gloo for the host-side collectives), with every CRC computed by the product:
  * bench.py under torch.distributed.run, as the driver launches it for
    --gpus N: weak scaling (cfg2, each rank its own batch) and strong scaling
    (cfg4, one 8 GiB file sharded by contiguous frame ranges, the last frame
    800 B on the last rank);
  * a window split into per-rank byte ranges (val_protocol_amd.shard, the
    product's val_shard_region rule), each rank's partial register computed by
    val_crc32_region_dev on the GPU, gathered over gloo and folded with the
    product's val_crc32_fold_partials, against the oracle.
And bench.py's RCCL path (nccl backend) with one rank on the box's GPU.
SURVEY 8(e); reference window fill src/val_sender.c:822-841."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench_two_ranks(config: str, *extra: str, ranks: int = 2, timeout: int = 240) -> dict:
    env = dict(os.environ, VAL_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(ranks), "--config", config, "--steps", "2", "--warmup", "1", "--no-cpu-baseline", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints exactly one line
    return json.loads(lines[0])


def test_bench_two_ranks_weak_cfg2():
    # (the cfg3 headline carries the cfg4 block by default; cfg2 asks for it, to stay small)
    line = _bench_two_ranks("cfg2", "--with-cfg4-strong")
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["parity_sample_ok"] is True
    assert line["config"]["frames_per_gpu"] == 65536
    assert line["value"] > 0 and line["cpu_baseline"] is None
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1]
    assert all(r["frames"] == 65536 and r["parity_sample_ok"] and r["GiB_s"] > 0 and r["kernel_ms"] > 0 for r in pr)
    agg = line["aggregate_over_max_rank"]
    assert agg["max_elapsed_s"] == max(r["elapsed_s"] for r in pr)
    assert agg["total_bytes"] == 2 * 2 * 65536 * (8 + 8 + 1024)  # 2 ranks x 2 steps
    assert abs(line["value"] - agg["total_bytes"] / agg["max_elapsed_s"] / 2**30) / line["value"] < 0.01
    # BASELINE configs[3] timed in the same invocation: the 8 GiB file sharded over the ranks
    st = line["cfg4_strong"]
    assert st["scaling"] == "strong" and st["frames_total"] == 131113 and st["parity_sample_ok"] is True
    spr = st["per_rank"]
    assert [r["rank"] for r in spr] == [0, 1] and sum(r["frames"] for r in spr) == 131113
    assert spr[0]["frames"] in (65556, 65557)
    # the file's 800-B remainder lands on the last rank
    assert spr[-1]["last_frame_crc_input"] == 8 + 8 + 800 and spr[0]["last_frame_crc_input"] == 8 + 8 + 65516
    file_crc_input = 131112 * (8 + 8 + 65516) + 8 + 8 + 800
    assert st["aggregate_over_max_rank"]["total_bytes"] == 2 * file_crc_input  # 2 steps
    assert st["value"] > 0


def test_bench_eight_ranks_driver_command():
    """The driver's 8-GPU invocation, literally: `python3 bench.py --gpus 8 ...`
    with no torchrun around it. bench.py starts the 8 ranks itself (a
    torch.distributed.run child process, decided before any GPU call), here
    rehearsed on one GPU (gloo for the host-side collectives, all ranks on
    cuda:0): cfg2 weak plus the cfg4 strong block, the 8 GiB file's 131,113
    frames split byte-balanced (~16,389 per rank, no collective on the data),
    the 816-B last frame on rank 7, the aggregate over the slowest rank, and
    every rank's parity sample against the oracle."""
    env = dict(os.environ, VAL_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--config", "cfg2", "--with-cfg4-strong",
           "--no-host-inclusive", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints exactly one line, through the parent's stdout
    line = json.loads(lines[0])
    assert line["launcher"].startswith("bench.py --gpus")
    assert line["n_gpus"] == 8 and line["scaling"] == "weak" and line["config"]["parity_sample_ok"] is True
    assert line["cpu_baseline"] is None and "cfg4_strong_proxy" not in line  # N > 1: measured ranks, no proxy
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == list(range(8)) and all(r["parity_sample_ok"] for r in pr)
    assert line["aggregate_over_max_rank"]["total_bytes"] == 8 * 2 * 65536 * (8 + 8 + 1024)
    st = line["cfg4_strong"]
    spr = st["per_rank"]
    assert st["parity_sample_ok"] is True and [r["rank"] for r in spr] == list(range(8))
    assert sum(r["frames"] for r in spr) == 131113
    assert all(16387 <= r["frames"] <= 16391 for r in spr), [r["frames"] for r in spr]
    assert spr[7]["last_frame_crc_input"] == 8 + 8 + 800
    assert all(r["last_frame_crc_input"] == 8 + 8 + 65516 for r in spr[:7])
    file_crc_input = 131112 * (8 + 8 + 65516) + 8 + 8 + 800
    agg = st["aggregate_over_max_rank"]
    assert agg["total_bytes"] == 2 * file_crc_input
    assert agg["max_elapsed_s"] == max(r["elapsed_s"] for r in spr)
    assert abs(st["value"] - agg["total_bytes"] / agg["max_elapsed_s"] / 2**30) / st["value"] < 0.01
    assert st["roofline"]["frac"] > 0 and st["roofline"]["bytes_per_launch"] == spr[0]["bytes_per_step"]


def test_bench_cfg4_proxy_at_one_gpu():
    """N = 1: after the cfg4 block, the single-GPU proxy of the 2/4/8-GPU
    strong-scaling curve: for each N the largest slice and the last rank's
    slice (the 816-B frame) of the file as N ranks split it, each timed alone
    and parity-sampled against the oracle."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "cfg2", "--with-cfg4-strong",
           "--no-host-inclusive", "--no-cpu-baseline", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    px = line["cfg4_strong_proxy"]
    assert px["parity_sample_ok"] is True and "single-GPU proxy" in px["label"]
    file_crc_input = 131112 * (8 + 8 + 65516) + 8 + 8 + 800
    assert px["file_crc_input_bytes"] == file_crc_input
    assert px["1"]["frames"] == 131113
    for n in (2, 4, 8):
        sl = px[str(n)]["slices_timed"]
        assert sl[-1]["rank"] == n - 1 and sl[-1]["last_frame_crc_input"] == 8 + 8 + 800
        assert all(s["parity_sample_ok"] and s["kernel_ms"] > 0 for s in sl)
        assert 131113 // n - 2 <= max(s["frames"] for s in sl) <= 131113 // n + 2
        assert px[str(n)]["est_aggregate_GiB_s"] > 0
    rf = line["cfg4_strong"]["roofline"]
    assert rf["bytes_per_launch"] == file_crc_input and rf["read_roof"] and rf["frac_of_read_roof"] > 0


def test_bench_rccl_process_group_one_rank():
    """The RCCL (nccl backend) code path of bench.py on real hardware: one rank
    under torch.distributed.run with a process group forced on, so the nccl
    init with device_id, the barriers around the timed region, the GPU-tensor
    all_reduce(MAX) and all_gather_object run through RCCL exactly as on the
    driver's 8-GPU node (where each rank has its own GPU)."""
    env = dict(os.environ, VAL_BENCH_BACKEND="nccl", VAL_BENCH_FORCE_DIST="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--config", "cfg2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--with-cfg4-strong"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["config"]["parity_sample_ok"] is True and line["value"] > 0
    # the host-inclusive block (north_star: H2D + kernel + D2H through the C ABI)
    hi = line["host_inclusive"]
    assert hi["outputs_equal_device"] is True and hi["on_gpu"] is True, hi
    assert hi["pinned"] > 0 and hi["pageable"] > 0 and hi["slice_frames"] == 65536
    assert [x["rank"] for x in line["per_rank"]] == [0]
    st = line["cfg4_strong"]
    assert st["parity_sample_ok"] is True and st["per_rank"][0]["frames"] == 131113


def test_bench_two_ranks_strong_cfg4():
    line = _bench_two_ranks("cfg4")
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["parity_sample_ok"] is True
    assert line["config"]["frames_total"] == 131113
    assert line["config"]["frames_per_gpu"] in (65556, 65557)  # rank 0's byte-balanced share
    pr = line["per_rank"]
    assert sum(r["frames"] for r in pr) == 131113 and all(r["parity_sample_ok"] for r in pr)
    # the file's 800-B remainder is the last rank's last frame; every other frame is a full one
    assert pr[-1]["last_frame_crc_input"] == 8 + 8 + 800 and pr[0]["last_frame_crc_input"] == 8 + 8 + 65516


def _region_worker(rank, world, port, data, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import val_protocol_amd.crc as vc
    from val_protocol_amd.shard import fold_partials, shard_region

    vc.init(0)
    dev = torch.device("cuda:0")
    start, cnt = shard_region(data.size, world, rank, align=64)
    d = torch.from_numpy(np.ascontiguousarray(data[start:start + cnt])).to(dev)
    st = int(vc.region(d, state_in=0xFFFFFFFF if rank == 0 else 0).item()) & 0xFFFFFFFF
    torch.cuda.synchronize()
    t = torch.tensor([st, cnt], dtype=torch.int64)
    out = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, t)
    if rank == 0:
        q.put((fold_partials([(int(o[0]), int(o[1])) for o in out]) ^ 0xFFFFFFFF, vc.cpu_fallback_count()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("nbytes", [1_000_003, 9 << 20])
def test_region_split_fold_gpu_ranks(nbytes):
    import torch.multiprocessing as mp

    from tests import _oracle, _prng

    data = _prng.prng_bytes(0xD16 + nbytes, nbytes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_region_worker, args=(r, 2, port, data, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    got, fallbacks = q.get(timeout=10)
    assert fallbacks == 0
    assert got == _oracle.crc32(data)
