"""Several GPUs from one process: the *_host_multi calls split a
batch into contiguous frame ranges balanced by bytes (val_shard_frames), one
host thread per range, each bound to device (range % device count); a long
window is split into byte ranges whose GPU-computed partial states fold with
the GF(2) shift. On a 1-GPU box the ranges are logical shards sharing the
device; the results must equal the single-call path and the oracle bit for
bit. Reference: src/val_sender.c:822-841 (the window being sharded)."""
import threading

import numpy as np
import pytest

from tests import _oracle, _prng

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import val_protocol_amd.crc as m

    m.init(0)
    m.set_geometry()
    return m


def _ragged(seed, n, lo, hi):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 4)[:-1]]).astype(np.uint64)
    base = _prng.prng_bytes(seed, int(offs[-1]) + int(lens[-1]) + 4)
    return base, offs, lens


def test_devices_and_binding(vc):
    assert vc.init_devices(0) >= 1
    assert vc.current_device() == 0
    vc.set_device(0)
    with pytest.raises(vc.ValError):
        vc.set_device(vc.device_count() + 5)


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_frames_host_multi_equals_oracle(vc, ndev):
    base, offs, lens = _ragged(31 + ndev, 3000, 0, 70000)
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    crc, hdr = vc.frames_host_multi(base, off=offs, length=lens, header=True, ndev=ndev)
    assert np.array_equal(crc, want) and np.array_equal(hdr, want_h)
    # strided mode
    n, flen, stride = 5000, 1040, 1044
    sb = _prng.prng_bytes(77, n * stride)
    assert np.array_equal(vc.frames_host_multi(sb, stride=stride, flen=flen, n=n, ndev=ndev),
                          _oracle.frames_strided(sb, stride, flen, n))


@pytest.mark.parametrize("ndev", [2, 4])
def test_verify_frames_host_multi(vc, ndev):
    base, offs, lens = _ragged(55, 2000, 8, 20000)
    crc = _oracle.frames(base, offs, lens)
    for o, l, c in zip(offs, lens, crc):
        base[int(o) + int(l):int(o) + int(l) + 4] = np.frombuffer(int(c).to_bytes(4, "little"), np.uint8)
    st, ok, nbad = vc.verify_frames_host_multi(base, off=offs, length=lens, ndev=ndev)
    assert st == vc.VAL_OK and nbad == 0 and ok.all()
    bad = [3, 999, 1000, 1999]
    for i in bad:
        base[int(offs[i]) + int(lens[i]) // 2] ^= 1
    st, ok, nbad = vc.verify_frames_host_multi(base, off=offs, length=lens, ndev=ndev)
    assert st == vc.VAL_ERR_CRC and nbad == len(bad) and np.nonzero(ok == 0)[0].tolist() == bad


@pytest.mark.parametrize("ndev", [2, 3, 8])
@pytest.mark.parametrize("length", [1, 4096, 1_000_003, 40 << 20])
def test_region_host_multi(vc, ndev, length):
    data = _prng.prng_bytes(length + ndev, length)
    got = vc.region_host_multi(data, 0xFFFFFFFF, ndev=ndev) ^ 0xFFFFFFFF
    assert got == _oracle.crc32(data)


def test_multi_at_default_thresholds_reaches_the_gpu(vc):
    """At the library's built-in crossover (64 MiB for one GPU and one CPU
    thread; the suite normally forces 0) a 256 MiB batch split over ndev = 8
    shards is decided once for the whole batch, goes to the GPU (the CPU
    counter does not move; each 32 MiB shard alone is below the single-GPU
    crossover and used to be answered on the CPU) and is bit-exact."""
    vc.set_host_batch_min_bytes(64 << 20)
    try:
        n, flen, stride = 16384, 16400, 16404  # 268.7 MB of CRC input
        sb = _prng.prng_bytes(0x256, n * stride)
        want = _oracle.frames_strided(sb, stride, flen, n, nthreads=8)
        before = vc.cpu_batch_count()
        for ndev in (8, 0):
            assert np.array_equal(vc.frames_host_multi(sb, stride=stride, flen=flen, n=n, ndev=ndev), want)
        data = sb[: 200 << 20]
        assert vc.region_host_multi(data, 0xFFFFFFFF, ndev=8) ^ 0xFFFFFFFF == _oracle.crc32(data)
        assert vc.cpu_batch_count() == before
        assert vc.host_multi_min_bytes(vc.device_count()) <= 64 << 20
    finally:
        vc.set_host_batch_min_bytes(-1)


def test_scalar_hooks_from_many_threads(vc):
    """The provider is called from several sessions' threads at once
    (reference include/val_protocol.h:231-233): reentrant, every CRC exact."""
    bad = []

    def worker(k):
        for i in range(60):
            ln = (k * 7919 + i * 104729) % 70000
            d = _prng.prng_bytes(k * 1000 + i, ln)
            if vc.crc32_provider(0xFFFFFFFF, d.tobytes()) != _oracle.crc32(d):
                bad.append((k, i, ln))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not bad
