"""Host-memory batches below the host-batch crossover are answered by the
library's CPU engine (val_crc32_hip.hip cpu_frames):
the same outputs as the kernels, pinned here to the reference-written
fixtures without a GPU. The windows, TX frames, RX verdicts and the 1 MiB
loopback frame log in tests/golden/dropin_vectors.json were produced by the
reference's own protocol code (src/val_core.c:718-1073, src/val_sender.c:
258-315,822-841; oracle/provider_harness.c fixtures); header_crc and the
payload states are checked against the oracle. The GPU suite forces the
threshold to 0, so tests/test_gpu_dropin.py replays the same fixtures on the
GPU path."""
import json
import os

import numpy as np
import pytest

import val_protocol_amd.crc as vc
import val_protocol_amd.wire as wire
from tests import _oracle, _prng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAL_OK, VAL_ERR_CRC = 0, -6


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(ROOT, "tests", "golden", "dropin_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(params=[1, 4], ids=["1thread", "4threads"])
def cpu_routed(request):
    """Every host batch below 2^62 bytes on the CPU engine, on 1 or 4 threads."""
    vc.set_host_batch_min_bytes(1 << 62)
    vc.set_host_cpu_threads(request.param)
    before = vc.cpu_batch_count()
    yield before
    vc.set_host_batch_min_bytes(-1)
    vc.set_host_cpu_threads(1)


def _window(w):
    file = _prng.prng_bytes(w["file_seed"], w["file_size"])
    fr = np.array(w["frames"], dtype=np.uint64)
    return wire.build_data_batch(file, fr[:, 0], fr[:, 1].astype(np.uint32), fr[:, 0], fr[:, 2].astype(np.uint8))


@pytest.mark.parametrize("k", range(5))
def test_windows_match_reference(fx, cpu_routed, k):
    w = fx["windows"][k]
    stream, fo, cl = _window(w)
    crc, hdr = vc.frames_host(stream, off=fo, length=cl, header=True)
    assert crc.tolist() == w["trailers"]
    assert np.array_equal(hdr, _oracle.frames(stream, fo, cl, header=True)[1])
    wire.put_trailers(stream, fo, cl, crc)
    assert _oracle.crc32(stream) == w["wire_crc"]
    for _, pos, mask in w["corrupt"]:
        stream[pos] ^= mask
    st, fo2, cl2, consumed = wire.scan_frames(stream, w["mtu"])
    assert st == VAL_OK and consumed == stream.size
    vst, ok, nbad = vc.verify_frames_host(stream, off=fo2, length=cl2)
    assert [bool(x) for x in ok] == [rc == VAL_OK for rc in w["ref_rc"]]
    assert nbad == w["ref_crc_errors"] and vst == (VAL_ERR_CRC if nbad else VAL_OK)
    assert vc.cpu_batch_count() - cpu_routed == 2


def test_tx_frames_and_loopback_log(fx, cpu_routed):
    frames, want = [], []
    for r in fx["tx"]:
        content = r["payload_len"] + (8 if r["include_offset"] else 0)
        if content > 0xFFFF:
            continue  # the reference's u16-wrapped frames (the product framer refuses them)
        payload = _prng.prng_bytes(r["seed"], r["payload_len"])
        stream, fo, cl = wire.build_data_batch(payload, [0], [payload.size], [r["offset"]], [r["include_offset"]])
        frames.append(stream[:int(cl[0])])
        want.append(r["trailer"])
    off = np.concatenate([[0], np.cumsum([f.size + 4 for f in frames])[:-1]]).astype(np.uint64)
    buf = np.zeros(int(off[-1]) + frames[-1].size + 4, dtype=np.uint8)
    for o, f in zip(off, frames):
        buf[int(o):int(o) + f.size] = f
    assert vc.frames_host(buf, off=off, length=np.array([f.size for f in frames], np.uint32)).tolist() == want
    # BASELINE configs[0]: both sessions of the 1 MiB / MTU 1024 loopback
    lb = fx["loopback"]
    file = _prng.prng_bytes(lb["file_seed"], lb["bytes"])
    for side in ("tx", "rx"):
        parts, offs, lens, trailers, pos = [], [], [], [], 0
        for ptype, wire_len, trailer, foff, prefix in lb[f"{side}_frames"]:
            head = np.frombuffer(bytes.fromhex(prefix), dtype=np.uint8)
            body = np.concatenate([head, file[foff:foff + wire_len - 4 - head.size]]) if ptype == 5 else head
            parts += [body, np.frombuffer(int(trailer).to_bytes(4, "little"), dtype=np.uint8)]
            offs.append(pos)
            lens.append(body.size)
            trailers.append(trailer)
            pos += wire_len
        stream = np.concatenate(parts)
        offs, lens = np.array(offs, np.uint64), np.array(lens, np.uint32)
        assert vc.frames_host(stream, off=offs, length=lens).tolist() == trailers
        st, ok, nbad = vc.verify_frames_host(stream, off=offs, length=lens)
        assert st == VAL_OK and nbad == 0 and ok.all()


def test_strided_and_payload_states(cpu_routed):
    """Strided batches and the RX payload-state by-product (f4) against the
    oracle, including frames shorter than their prefix."""
    n, flen, stride = 300, 1040, 1044
    sb = _prng.prng_bytes(91, n * stride)
    assert np.array_equal(vc.frames_host(sb, stride=stride, flen=flen, n=n), _oracle.frames_strided(sb, stride, flen, n))
    rng = np.random.default_rng(92)
    lens = rng.integers(0, 3000, 500).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 4)[:-1]]).astype(np.uint64)
    base = _prng.prng_bytes(93, int(offs[-1]) + int(lens[-1]) + 4)
    base[offs[::2].astype(np.int64) + 1] |= 1  # half the frames say "offset present" (16-B prefix)
    base[offs[1::2].astype(np.int64) + 1] &= 0xFE
    want = _oracle.frames(base, offs, lens)
    for i, (o, L) in enumerate(zip(offs, lens)):
        base[int(o) + int(L):int(o) + int(L) + 4] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    base[int(offs[7]) + 2] ^= 0x10
    st, ok, nbad, pay = vc.verify_frames_ex_host(base, off=offs, length=lens)
    assert st == VAL_ERR_CRC and nbad == (1 if lens[7] > 2 else 0)
    for i, (o, L) in enumerate(zip(offs, lens)):
        f = base[int(o):int(o) + int(L)]
        pre = (16 if f[1] & 1 else 8) if L >= 8 else None
        exp = _oracle.update_state(0, f[pre:]) if pre is not None and L >= pre else 0
        assert int(pay[i]) == exp, i


def test_helper_threads_large_batches(cpu_routed):
    """Batches of >= 16 MiB of CRC input, where the 4-thread parametrization
    really starts helper threads (one per 4 MiB): strided, descriptor (mixed
    lengths, so the byte-balanced cuts differ from count cuts) and verify with
    corruption on both sides of a cut, against the oracle."""
    n, flen, stride = 16400, 1040, 1044  # 17.1 MB of CRC input
    sb = _prng.prng_bytes(94, n * stride)
    want = _oracle.frames_strided(sb, stride, flen, n)
    assert np.array_equal(vc.frames_host(sb, stride=stride, flen=flen, n=n), want)
    rng = np.random.default_rng(95)
    lens = rng.integers(1, 9000, 4000).astype(np.uint32)  # ~18 MB
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 4)[:-1]]).astype(np.uint64)
    base = _prng.prng_bytes(96, int(offs[-1]) + int(lens[-1]) + 4)
    want = _oracle.frames(base, offs, lens)
    assert np.array_equal(vc.frames_host(base, off=offs, length=lens), want)
    for i, (o, L) in enumerate(zip(offs, lens)):
        base[int(o) + int(L):int(o) + int(L) + 4] = np.frombuffer(int(want[i]).to_bytes(4, "little"), np.uint8)
    bad = [3, 1999, 2000, 3999]
    for i in bad:
        base[int(offs[i])] ^= 0x40
    st, ok, nbad = vc.verify_frames_host(base, off=offs, length=lens)
    assert st == VAL_ERR_CRC and nbad == len(bad)
    assert np.nonzero(ok == 0)[0].tolist() == bad
    assert vc.cpu_batch_count() - cpu_routed == 3


def _cpu_budget() -> int:
    """The library's CPU budget: the affinity set capped by the cgroup quota."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except OSError:
        pass
    return n


def _n_eff_x16(n: int, pinned: bool) -> int:
    """The N-device rule restated: pinned input
    scales with N; pageable input is capped by the host bounce copies, which
    all shards share within the CPU budget: one copy thread ~14 GB/s, all
    copies together ~135 GB/s, against ~53 GB/s per GPU's pageable path
    (profiles/r06_bounce_copy_scaling.jsonl)."""
    if pinned:
        return 16 * n
    per_copy = max(1, min(8, max(1, _cpu_budget() // n), 16))  # val_gpu_host_copy_threads(64 MiB, n)
    assert per_copy == vc.lib().val_gpu_host_copy_threads(64 << 20, n)
    copy = min(min(_cpu_budget(), n * per_copy) * 14000, 135000)
    return max(16, min(16 * n, copy * 16 // 53000))


def test_multi_decides_once_for_the_whole_batch():
    """val_crc32_*_host_multi choose CPU or GPU once per batch against a
    crossover that scales with the distinct devices and the CPU threads
    (C1 * T / N_eff; N_eff = N for pinned input, capped by the shared host
    bounce copies for pageable input), never per shard; below it the batch
    needs no device (this container has none) and the helper threads stay
    within the CPU budget."""
    vc.set_host_batch_min_bytes(64 << 20)  # the built-in single-GPU crossover (conftest exports 0)
    c1 = 64 << 20
    try:
        assert vc.host_multi_min_bytes(1) == c1
        for n in (1, 2, 4, 8):
            assert vc.host_multi_min_bytes(n, pinned=True) == c1 // n
            assert vc.host_multi_min_bytes(n, pinned=False) == c1 * 16 // _n_eff_x16(n, False), n
            assert vc.host_multi_min_bytes(n) == vc.host_multi_min_bytes(n, pinned=False)
        # pageable shards never reach more devices' worth of GPU than the copies feed
        assert vc.host_multi_min_bytes(8, pinned=False) >= vc.host_multi_min_bytes(8, pinned=True)
        if _cpu_budget() >= 16:  # the GPU box's share: N_eff 2.55 from 4 devices on
            assert _n_eff_x16(8, False) == 40 and _n_eff_x16(2, False) == 32
        vc.set_host_cpu_threads(4)
        assert vc.host_multi_min_bytes(8, pinned=True) == min(4, _cpu_budget()) * (c1 // 8)
        vc.set_host_cpu_threads(1)
        n, flen, stride = 2000, 1040, 1044
        sb = _prng.prng_bytes(97, n * stride)
        before = vc.cpu_batch_count()
        for ndev in (0, 1, 3, 8):
            got = vc.frames_host_multi(sb, stride=stride, flen=flen, n=n, ndev=ndev)
            assert np.array_equal(got, _oracle.frames_strided(sb, stride, flen, n)), ndev
        data = _prng.prng_bytes(98, (9 << 20) + 77)
        vc.set_host_cpu_threads(4)  # 9 MiB: two ranges at most (one per 4 MiB)
        for ndev in (1, 8):
            assert vc.region_host_multi(data, ndev=ndev) == _oracle.update_state(0xFFFFFFFF, data)
        assert vc.cpu_batch_count() - before == 6
    finally:
        vc.set_host_batch_min_bytes(-1)
        vc.set_host_cpu_threads(1)


def test_threshold_knob():
    vc.set_host_batch_min_bytes(12345)
    assert vc.host_batch_min_bytes() == 12345
    vc.set_host_batch_min_bytes(-1)
    # the suite's conftest exports VAL_GPU_HOST_BATCH_MIN_BYTES=0 before the library loads
    assert vc.host_batch_min_bytes() == int(os.environ.get("VAL_GPU_HOST_BATCH_MIN_BYTES", vc.host_batch_min_bytes()))


CHECK = os.path.join(ROOT, "oracle", "host_runtime_check")


@pytest.mark.parametrize("gpu", [pytest.param(False, id="cpu_engine"), pytest.param(True, id="gpu", marks=pytest.mark.gpu)])
def test_host_runtime_threads_of_random_batches(gpu):
    """oracle/host_runtime_check (checker, built by `make -C oracle oracle`):
    four threads at once, each with random packed unaligned batches of up to
    3,000 frames and ~49 MiB, through val_crc32_frames_host,
    val_crc32_verify_frames_ex_host (every 97th trailer corrupted; ok flags,
    nbad, payload states), val_crc32_frames_host_multi (8 shards),
    val_crc32_region_host_multi and the scalar hooks, every output against the
    oracle. CPU variant: the library's thresholds with the CPU engine's helper
    threads on (4 per call). GPU variant: thresholds at 0, so every call of
    every thread goes through the GPU host path at once. The same program
    under AddressSanitizer/UBSan and ThreadSanitizer: tools/
    sanitize_host_runtime.sh (profiles/r05_sanitize_host_runtime.txt)."""
    import subprocess

    if not os.path.exists(CHECK):
        pytest.skip("oracle/host_runtime_check not built (make -C oracle oracle)")
    env = dict(os.environ)
    if gpu:
        env.update(VAL_GPU_HOST_BATCH_MIN_BYTES="0", VAL_GPU_PROVIDER_MIN_BYTES="0")
    else:
        env.pop("VAL_GPU_HOST_BATCH_MIN_BYTES", None)
        env.pop("VAL_GPU_PROVIDER_MIN_BYTES", None)
    r = subprocess.run([CHECK, "4", "6", "11"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["bad"] == 0 and out["frames_checked"] > 20000 and out["cpu_fallbacks"] == 0, out
    if gpu:
        assert out["devices"] >= 1 and out["cpu_batches"] == 0, out
    else:
        assert out["cpu_batches"] >= 4 * 6 * 2, out
