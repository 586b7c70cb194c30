"""GPU parity of this round's kernel paths, through the C ABI against the
oracle (bit-exact):
  * unit 0 read inside its frame's first line (four dwordx4 loads and a select
    network) at G = 2 and 4: descriptor batches in shuffled memory order,
    frames at the very start of the buffer, every start alignment, header_crc
    and verify, and a batch long enough for the dynamic-tail queue (these
    tests were written for the carried-frames kernel, measured and removed
    this round; they pin the same paths of k_frames);
  * the ragged path's single-bucket batches (k_bin_scatter skips the scatter,
    the kernel takes frame i at sorted position i), alternated with
    multi-bucket batches on the same stream (scratch state carried between
    launches), and its one-ahead item queue."""
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
    yield m
    m.set_geometry()


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda:0")


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _shuffled(seed, n, L, gap_max=7, first_at_zero=True):
    """n frames of L CRC bytes laid out with random gaps, the descriptors in a
    random order (frame i of the batch is not frame i in memory)."""
    rng = np.random.default_rng(seed)
    gaps = rng.integers(0, gap_max + 1, n)
    if first_at_zero:
        gaps[0] = 0
    offs = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        offs[i] = pos
        pos += L + 4
    base = _prng.prng_bytes(seed, pos + 16)
    perm = rng.permutation(n)
    return base, offs[perm].copy(), np.full(n, L, np.uint32)


def _frames(vc, dev, base, offs, lens, hint, header=True):
    d = torch.from_numpy(base).to(dev)
    crc = torch.empty(offs.size, dtype=torch.int32, device=dev)
    hdr = torch.empty(offs.size, dtype=torch.int32, device=dev) if header else None
    vc.frames(d, off=torch.from_numpy(offs.view(np.int64)).to(dev), length=torch.from_numpy(lens.view(np.int32)).to(dev),
              out_crc=crc, out_hdr=hdr, len_hint=hint)
    torch.cuda.synchronize()
    return _u32(crc), (_u32(hdr) if header else None)


@pytest.mark.parametrize("L", [60, 64, 65, 127, 128, 129, 600, 1023, 1100, 4200, 8191])
def test_short_shuffled_descriptors(vc, dev, L):
    vc.set_geometry()  # the measured geometry: G = 2, 4 or 8 below 8 KiB
    base, offs, lens = _shuffled(1000 + L, 3000, L)
    got, got_h = _frames(vc, dev, base, offs, lens, hint=L)
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    assert np.array_equal(got, want)
    assert np.array_equal(got_h, want_h)


@pytest.mark.parametrize("G", [2, 4])
@pytest.mark.parametrize("shift", range(8))
def test_short_every_start_alignment(vc, dev, G, shift):
    # frames at byte offsets shift, shift + stride, ... with the first frame
    # near the buffer start: unit 0 starts before the buffer for small shifts
    vc.set_geometry(G, 1)
    L = 700 + 13 * shift
    stride = L + 4 + shift
    n = 2048 + 3
    base = _prng.prng_bytes(2000 + shift, shift + n * stride + 8)
    offs = (shift + np.arange(n, dtype=np.uint64) * stride).astype(np.uint64)
    lens = np.full(n, L, np.uint32)
    got, got_h = _frames(vc, dev, base, offs, lens, hint=L)
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    assert np.array_equal(got, want)
    assert np.array_equal(got_h, want_h)
    vc.set_geometry()


def test_short_verify_detects_corruption(vc, dev):
    vc.set_geometry()
    base, offs, lens = _shuffled(3001, 5000, 1100)
    crc = _oracle.frames(base, offs, lens)
    for o, l, c in zip(offs, lens, crc):
        base[int(o) + int(l):int(o) + int(l) + 4] = np.frombuffer(int(c).to_bytes(4, "little"), np.uint8)
    bad = np.random.default_rng(5).choice(5000, 17, replace=False)
    for i in bad:
        base[int(offs[i]) + int(i % 1100)] ^= 0x10
    ok, nbad = vc.verify_frames(torch.from_numpy(base).to(dev), off=torch.from_numpy(offs.view(np.int64)).to(dev),
                                length=torch.from_numpy(lens.view(np.int32)).to(dev), len_hint=1100)
    torch.cuda.synchronize()
    assert int(nbad.item()) == 17
    assert set(np.flatnonzero(ok.cpu().numpy() == 0).tolist()) == set(bad.tolist())


def test_short_dynamic_tail_every_frame(vc, dev):
    # long enough for the partitioned dynamic-tail queue (>= 4 group rounds of
    # 16 KiB+ descriptor groups): 300,000 x 1,100 B, strided and descriptor,
    # twice on one stream (the last wave out re-zeroes the queue)
    vc.set_geometry()
    n, L = 300000, 1100
    stride = L + 4
    base = _prng.prng_bytes(4001, n * stride + 8)
    d = torch.from_numpy(base).to(dev)
    want = _oracle.frames_strided(base, stride, L, n, nthreads=8)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * stride
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    for _ in range(2):
        crc = vc.frames(d, stride=stride, flen=L, n=n)
        torch.cuda.synchronize()
        assert np.array_equal(_u32(crc), want)
        crc = vc.frames(d, off=offs, length=lens, len_hint=L)
        torch.cuda.synchronize()
        assert np.array_equal(_u32(crc), want)


@pytest.fixture
def binned_always(vc):
    vc.set_ragged_min_frames(1)


@pytest.mark.parametrize("lo,hi", [(16400, 16400), (16385, 16896), (600, 600), (0, 0), (65000, 65536)])
def test_ragged_one_bucket_identity(vc, dev, binned_always, lo, hi):
    vc.set_geometry()
    rng = np.random.default_rng(lo)
    n = 5000
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 4 + rng.integers(0, 5, n - 1))]).astype(np.uint64)
    base = _prng.prng_bytes(lo + 7, int(offs[-1]) + int(lens[-1]) + 16)
    perm = rng.permutation(n)
    offs, lens = offs[perm].copy(), lens[perm].copy()
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    # one bucket, then two buckets, then one again on the same stream
    got, got_h = _frames(vc, dev, base, offs, lens, hint=0)
    assert np.array_equal(got, want) and np.array_equal(got_h, want_h)
    lens2 = lens.copy()
    lens2[::2] //= 2
    got2, _ = _frames(vc, dev, base, offs, lens2, hint=0)
    assert np.array_equal(got2, _oracle.frames(base, offs, lens2))
    got3, got3_h = _frames(vc, dev, base, offs, lens, hint=0)
    assert np.array_equal(got3, want) and np.array_equal(got3_h, want_h)


def test_ragged_queue_many_items(vc, dev, binned_always):
    # more items than waves, across all four length classes: the one-ahead
    # queue hands out every item exactly once
    rng = np.random.default_rng(77)
    n = 120000
    lens = np.exp(rng.uniform(np.log(40), np.log(20000), n)).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 4)]).astype(np.uint64)
    base = _prng.prng_bytes(78, int(offs[-1]) + int(lens[-1]) + 8)
    got, _ = _frames(vc, dev, base, offs, lens, hint=0, header=False)
    assert np.array_equal(got, _oracle.frames(base, offs, lens, nthreads=8))
