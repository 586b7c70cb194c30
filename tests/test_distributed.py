"""World-size-2 gloo run of the sharding logic used by bench.py --gpus N and
by the product's *_host_multi calls: frames split by bytes with no overlap or
gap (the product's val_shard_frames), and a long window split into byte
ranges whose partial states fold with the product's val_crc32_fold_partials to
the oracle CRC. Without a GPU the per-rank partial states come from the
oracle; tests/test_gpu_multi.py runs the same split and fold with partial
states the GPU computed."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from val_protocol_amd.shard import fold_partials, shard_frames, shard_region

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_frames_partition():
    for n, w in [(0, 2), (1, 2), (7, 3), (1048576, 8), (131113, 8)]:
        spans = [shard_frames(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == n
        for (s0, c0), (s1, _) in zip(spans, spans[1:]):
            assert s0 + c0 == s1
    lens = np.random.default_rng(3).integers(520, 65532, 1000).astype(np.uint64)
    spans = [shard_frames(1000, 4, r, lens) for r in range(4)]
    assert sum(c for _, c in spans) == 1000
    per = [int(lens[s:s + c].sum()) for s, c in spans]
    assert max(per) - min(per) <= 2 * 65532


def _worker(rank, world, port, data, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests import _oracle

    start, cnt = shard_region(data.size, world, rank, align=64)
    st = _oracle.update_state(0xFFFFFFFF if rank == 0 else 0, data[start:start + cnt])
    t = torch.tensor([st, cnt], dtype=torch.int64)
    out = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(out, t)  # host-side metadata only (2 words per rank)
    if rank == 0:
        parts = [(int(o[0]), int(o[1])) for o in out]
        q.put(fold_partials(parts) ^ 0xFFFFFFFF)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_region_split_fold_gloo(world):
    from tests import _oracle, _prng

    data = _prng.prng_bytes(0xD15, 1_000_003)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) == _oracle.crc32(data)


def test_fold_partials_matches_oracle_any_split():
    """The product's host fold over uneven splits (including empty ranges)."""
    from tests import _oracle, _prng

    data = _prng.prng_bytes(0xF01D, 300_001)
    for cuts in ([0, 300_001], [0, 1, 300_001], [0, 4096, 4096, 150_000, 300_001], [0, 299_999, 300_001]):
        parts = [(_oracle.update_state(0xFFFFFFFF if k == 0 else 0, data[a:b]), b - a)
                 for k, (a, b) in enumerate(zip(cuts, cuts[1:]))]
        assert fold_partials(parts) ^ 0xFFFFFFFF == _oracle.crc32(data)


def test_shard_frames_matches_reference_split_rule():
    """val_shard_frames cut r = first frame whose byte prefix reaches total*r/world."""
    rng = np.random.default_rng(9)
    for n, w in [(1, 8), (5, 8), (1000, 3), (262144, 8)]:
        lens = rng.integers(0, 65532, n).astype(np.uint64)
        csum = np.concatenate([[0], np.cumsum(lens)])
        total = int(csum[-1])
        for r in range(w):
            s, c = shard_frames(n, w, r, lens)
            want_s = 0 if r == 0 else int(np.searchsorted(csum, (total * r) // w, side="left"))
            want_e = n if r == w - 1 else int(np.searchsorted(csum, (total * (r + 1)) // w, side="left"))
            assert (s, s + c) == (want_s, max(want_s, want_e))


def test_fold_payload_states_host():
    """The product's host fold of payload states (f4) with oracle states: the
    rolling CRC over the concatenated payloads, stopping at the first
    rejected frame."""
    import val_protocol_amd.crc as vc
    from tests import _oracle, _prng

    rng = np.random.default_rng(4)
    lens = np.concatenate([rng.integers(0, 3000, 200), [0, 0, 65516, 1, 65516]]).astype(np.uint32)
    data = _prng.prng_bytes(41, int(lens.sum()))
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    states = np.array([_oracle.update_state(0, data[offs[i]:offs[i + 1]]) for i in range(lens.size)], np.uint32)
    st, nf = vc.fold_payload_states(0xFFFFFFFF, states, lens)
    assert nf == lens.size and st ^ 0xFFFFFFFF == _oracle.crc32(data)
    ok = np.ones(lens.size, np.uint8)
    ok[150] = 0
    st, nf = vc.fold_payload_states(0x1234, states, lens, ok)
    assert nf == 150 and st == _oracle.update_state(0x1234, data[:offs[150]])


def test_bench_refuses_more_ranks_than_gpus():
    """bench.py under the driver's torchrun with the nccl (RCCL) backend and
    fewer visible GPUs than ranks: exits non-zero with a clear message before
    any GPU call or rendezvous (no GPU in this container: 0 < 2)."""
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    env.pop("VAL_BENCH_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-1000:])
    assert "need 2 visible GPUs" in r.stderr and r.stdout == ""


def test_bench_refuses_a_world_size_other_than_gpus():
    """A launcher that started a different number of ranks than --gpus asks
    for: bench.py exits non-zero with a message before importing torch."""
    import subprocess
    import sys

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29999")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-1000:])
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_bench_gpus_n_starts_ranks_itself():
    """`bench.py --gpus N` without torchrun: the ranks are started as a fresh
    child process (torch.distributed.run over 127.0.0.1, the same script and
    arguments), decided before any GPU call; with the nccl backend and fewer
    visible GPUs than N (none here) the parent refuses with exit 2 first."""
    import subprocess
    import sys

    sys.path.insert(0, ROOT)
    import bench

    cmd = bench.rank_launch_command(8, ["--gpus", "8", "--steps", "3"], 29500)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8" and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29500"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "VAL_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-1000:])
    assert "--gpus 8 needs 8 visible GPUs" in r.stderr and r.stdout == ""
