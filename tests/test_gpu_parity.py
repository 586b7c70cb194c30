"""GPU parity: the HIP path (through the C ABI) against the oracle and the
reference-derived golden vectors. Bit-exact everywhere (integer work)."""
import os

import numpy as np
import pytest

from tests import _oracle, _prng

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GEOMS = [1, 2, 4, 8, 16, 32, 64]
# register prefetch depths of the frames kernel (0 = off; -2, -3: in-place
# rings, G = 2 and 4)
VARIANTS = [(0,), (1,), (2,), (4,), (-2,), (-3,)]


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


# ---- scalar hooks (host memory) ---------------------------------------------
def test_kat(vc, golden):
    assert vc.val_crc32(b"123456789") == 0xCBF43926 == golden["kat_123456789"]
    assert vc.val_crc32(b"") == 0
    assert vc.crc32_provider(0xFFFFFFFF, b"123456789") == 0xCBF43926


def test_single_bytes(vc, golden):
    assert [vc.val_crc32(bytes([b])) for b in range(256)] == golden["single_bytes"]


def test_length_sweep(vc, golden):
    data = _prng.prng_bytes(golden["sweep_seed"], 70000)
    got = [vc.val_crc32(data[:L]) for L in range(0, 4097)]
    assert got == golden["sweep_0_4096"]
    for L, want in golden["sweep_special"].items():
        assert vc.val_crc32(data[: int(L)]) == want


def test_state_and_provider_semantics(vc, golden):
    data = _prng.prng_bytes(golden["sweep_seed"], 70000)
    for v in golden["state_vectors"]:
        assert vc.val_crc32_update_state(v["seed"], data[: v["len"]]) == v["state"]
        assert vc.crc32_provider(v["seed"], data[: v["len"]]) == v["final"]


def test_regions_host(vc, golden):
    data = _prng.prng_bytes(golden["region_seed"], 8 << 20)
    for r in golden["regions"]:
        L, c = r["len"], r["chunk"]
        st = vc.val_crc32_init_state()
        for o in range(0, L, c):
            st = vc.val_crc32_update_state(st, data[o:min(L, o + c)])
        assert vc.val_crc32_finalize_state(st) == r["crc"]
        assert vc.val_crc32(data[:L]) == r["oneshot"]


# ---- region (device) ---------------------------------------------------------
@pytest.mark.parametrize("L", [0, 1, 2, 3, 4, 5, 7, 8, 63, 64, 65, 127, 128, 4095, 4096, 4097, 8191, 8192, 8193, 16384, 16385, 32768, 65535, 65536,
                               65537, 69632, 69633, 1_000_003, (16 << 20) - 1, 16 << 20, (16 << 20) + 1,
                               (64 << 20) + 7, 16 * 4096 * 4096 + 4096 * 17 + 3])
def test_region_dev(vc, dev, L):
    data = _prng.prng_bytes(0xAB00 + L % 977, L)
    d = torch.from_numpy(data).to(dev)
    for state_in in (0xFFFFFFFF, 0, 0x1234ABCD):
        out = vc.region(d, state_in)
        torch.cuda.synchronize()
        assert int(_u32(out)[0]) == _oracle.update_state(state_in, data)


@pytest.mark.parametrize("shift", [1, 2, 3, 5, 17])
@pytest.mark.parametrize("L", [16385, 69633, 1_000_003, (16 << 20) + 9])
def test_region_dev_misaligned(vc, dev, L, shift):
    """k_region chunks are anchored at the window end; windows starting at any
    byte (a resume window inside a file buffer) hash the same."""
    data = _prng.prng_bytes(0xA11 + L + shift, L + shift)
    d = torch.from_numpy(data).to(dev)
    for state_in in (0xFFFFFFFF, 0x0BADCAFE):
        out = vc.region(d[shift:], state_in)
        torch.cuda.synchronize()
        assert int(_u32(out)[0]) == _oracle.update_state(state_in, data[shift:])


@pytest.mark.parametrize("piece", [65537, 1 << 20, 3 << 20])
def test_region_chained_pieces(vc, dev, piece, monkeypatch):
    """Windows longer than one k_region launch covers (2^43 B) are chained
    pieces, each seeded from the previous result in device memory; the piece
    size is lowered here so the chaining runs."""
    import subprocess
    import sys

    code = f"""
import sys; sys.path.insert(0, {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r})
import numpy as np, torch
import val_protocol_amd.crc as vc
from tests import _oracle, _prng
vc.init(0)
data = _prng.prng_bytes(0xC4A1, 10_000_019)
d = torch.from_numpy(data).to('cuda:0')
for s in (0xFFFFFFFF, 0x1234ABCD):
    out = vc.region(d, s)
    torch.cuda.synchronize()
    assert (int(out.item()) & 0xFFFFFFFF) == _oracle.update_state(s, data), s
print('ok')
"""
    env = dict(os.environ, VAL_GPU_REGION_MAX_PIECE=str(piece))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_region_2gib_window(vc, dev):
    """W = 512 KiB chunks, 4,096 of them: the full oracle over 2 GiB + 3."""
    L = (2 << 30) + 3
    g = torch.Generator(device=dev).manual_seed(0x2618)
    d = torch.randint(0, 256, (L,), dtype=torch.uint8, device=dev, generator=g)
    out = vc.region(d, 0x0BADF00D)
    torch.cuda.synchronize()
    assert int(_u32(out)[0]) == _oracle.update_state(0x0BADF00D, d.cpu().numpy())


def test_region_256mib_window(vc, dev):
    # Largest resume tail-verify window (reference src/val_receiver.c:161).
    L = 256 << 20
    data = _prng.prng_bytes(0x256, L)
    d = torch.from_numpy(data).to(dev)
    out = vc.region(d, 0xFFFFFFFF)
    torch.cuda.synchronize()
    assert int(_u32(out)[0]) ^ 0xFFFFFFFF == _oracle.crc32(data)


# ---- batch frames ----------------------------------------------------------
@pytest.mark.parametrize("G", GEOMS)
@pytest.mark.parametrize("payload,explicit", [(1024, True), (1004, True), (16384, True), (400, False), (65516, True)])
def test_frames_strided(vc, dev, G, payload, explicit):
    n = 96 if payload > 20000 else 600
    stream = _prng.frames_stream(n, payload, stride_pad=3, seed=0x51 ^ payload, explicit=explicit)
    flen = 8 + payload + (8 if explicit else 0)
    stride = flen + 4 + 3
    vc.set_geometry(G, *VARIANTS[G % len(VARIANTS)])
    d = torch.from_numpy(stream).to(dev)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n, dtype=torch.int32, device=dev)
    vc.frames(d, stride=stride, flen=flen, n=n, out_crc=crc, out_hdr=hdr)
    torch.cuda.synchronize()
    want, want_h = _oracle.frames_strided(stream, stride, flen, n, header=True)
    assert np.array_equal(_u32(crc), want)
    assert np.array_equal(_u32(hdr), want_h)


def _ragged(seed, n, lo, hi):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    gaps = rng.integers(0, 7, n)  # byte-unaligned starts
    offs = np.zeros(n, np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        offs[i] = pos
        pos += int(lens[i]) + 4
    base = _prng.prng_bytes(seed, pos + 16)
    return base, offs, lens


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("G", GEOMS)
def test_frames_ragged_descriptors(vc, dev, G, variant):
    base, offs, lens = _ragged(100 + G, 700, 0, 70000)
    lens[:40] = np.arange(40)  # tiny frames incl. 0..3 (byte path) and 4..39
    vc.set_geometry(G, *variant)
    d = torch.from_numpy(base).to(dev)
    do = torch.from_numpy(offs.view(np.int64)).to(dev)
    dl = torch.from_numpy(lens.view(np.int32)).to(dev)
    crc = torch.empty(offs.size, dtype=torch.int32, device=dev)
    hdr = torch.empty(offs.size, dtype=torch.int32, device=dev)
    vc.frames(d, off=do, length=dl, out_crc=crc, out_hdr=hdr)
    torch.cuda.synchronize()
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    assert np.array_equal(_u32(crc), want)
    assert np.array_equal(_u32(hdr), want_h)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("G", GEOMS)
def test_every_length_0_to_600(vc, dev, G, variant):
    lens = np.arange(601, dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 5)]).astype(np.uint64)
    base = _prng.prng_bytes(77, int(offs[-1]) + 700)
    vc.set_geometry(G, *variant)
    d = torch.from_numpy(base).to(dev)
    crc = vc.frames(d, off=torch.from_numpy(offs.view(np.int64)).to(dev),
                    length=torch.from_numpy(lens.view(np.int32)).to(dev))
    torch.cuda.synchronize()
    assert np.array_equal(_u32(crc), _oracle.frames(base, offs, lens))


def _with_trailers(base, offs, lens):
    crc = _oracle.frames(base, offs, lens)
    for o, l, c in zip(offs, lens, crc):
        base[int(o) + int(l):int(o) + int(l) + 4] = np.frombuffer(int(c).to_bytes(4, "little"), np.uint8)
    return base


@pytest.mark.parametrize("G", [1, 8, 64])
def test_verify_detects_corruption(vc, dev, G):
    base, offs, lens = _ragged(900 + G, 500, 8, 20000)
    base = _with_trailers(base, offs, lens)
    rng = np.random.default_rng(G)
    bad = rng.choice(500, 23, replace=False)
    for k, i in enumerate(bad):
        o, l = int(offs[i]), int(lens[i])
        pos = o + l + 3 if k % 3 == 0 else o + int(rng.integers(0, l))  # trailer byte or payload/header bit
        base[pos] ^= np.uint8(1 << (k % 8))
    want_ok, want_bad = _oracle.verify_frames(base, offs, lens)
    assert want_bad == 23
    vc.set_geometry(G, *VARIANTS[G % len(VARIANTS)])
    d = torch.from_numpy(base).to(dev)
    ok, nbad = vc.verify_frames(d, off=torch.from_numpy(offs.view(np.int64)).to(dev),
                                length=torch.from_numpy(lens.view(np.int32)).to(dev))
    torch.cuda.synchronize()
    assert int(nbad.item()) == 23
    assert np.array_equal(ok.cpu().numpy(), want_ok)


def test_reference_tx_frames_verify_on_gpu(vc, dev, golden):
    # Frames produced by the reference TX path (golden, full wire bytes).
    frames = [bytes.fromhex(f["wire"]) for f in golden["frames"] if "wire" in f]
    offs, lens, blob = [], [], b""
    for w in frames:
        offs.append(len(blob))
        lens.append(len(w) - 4)
        blob += w
    base = np.frombuffer(blob, np.uint8).copy()
    ok, nbad = vc.verify_frames(torch.from_numpy(base).to(dev),
                                off=torch.tensor(offs, dtype=torch.int64, device=dev),
                                length=torch.tensor(lens, dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    assert int(nbad.item()) == 0 and bool(ok.all())


def test_host_batch_api(vc):
    vc.set_geometry()
    base, offs, lens = _ragged(31, 300, 0, 40000)
    crc, hdr = vc.frames_host(base, offs, lens, header=True)
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    assert np.array_equal(crc, want) and np.array_equal(hdr, want_h)
    base = _with_trailers(base, offs, lens)
    st, ok, nbad = vc.verify_frames_host(base, offs, lens)
    assert st == vc.VAL_OK and nbad == 0 and ok.all()
    base[int(offs[5]) + 1] ^= 0x10
    st, ok, nbad = vc.verify_frames_host(base, offs, lens)
    assert st == vc.VAL_ERR_CRC and nbad == 1 and ok[5] == 0
    with pytest.raises(vc.ValError) as e:  # frame overruns the buffer
        vc.frames_host(base[:100], np.array([90], np.uint64), np.array([20], np.uint32))
    assert e.value.status == vc.VAL_ERR_INVALID_ARG


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("n,lo,hi", [(1, 0, 3), (16, 1000, 1100), (40, 0, 6000), (3, 60000, 65547)])
def test_host_small_window_zero_copy(vc, pinned, n, lo, hi):
    """Windows up to 256 KiB take the one-launch zero-copy host path: strided,
    packed descriptors (with a non-zero first offset), shuffled descriptors,
    header_crc, and verify with a corrupted frame."""
    vc.set_geometry()
    base, offs, lens = _ragged(77 + n, n, lo, hi)
    pad = 37  # first frame not at the buffer start
    base = np.concatenate([np.full(pad, 0xEE, np.uint8), base])
    offs = offs + np.uint64(pad)

    def host(a):
        if not pinned:
            return a
        pb = vc.PinnedBuffer(a.size)
        pb.array[:] = a
        keep.append(pb)
        return pb.array

    keep = []
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    crc, hdr = vc.frames_host(host(base), offs, lens, header=True)
    assert np.array_equal(crc, want) and np.array_equal(hdr, want_h)
    perm = np.random.default_rng(n).permutation(n)
    assert np.array_equal(vc.frames_host(host(base), offs[perm], lens[perm]), want[perm])
    tr = _with_trailers(base.copy(), offs, lens)
    st, ok, nbad = vc.verify_frames_host(host(tr), offs, lens)
    assert st == vc.VAL_OK and nbad == 0 and ok.all()
    k = n // 2
    tr[int(offs[k]) + int(lens[k]) + 1] ^= 0x08  # trailer byte
    st, ok, nbad = vc.verify_frames_host(host(tr), offs, lens)
    assert st == vc.VAL_ERR_CRC and nbad == 1 and ok[k] == 0
    stream = _prng.frames_stream(n, 1024, stride_pad=0, seed=0x99)
    assert np.array_equal(vc.frames_host(host(stream), stride=1044, flen=1040, n=n),
                          _oracle.frames_strided(stream, 1044, 1040, n))


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("chunk", [0, 1 << 16, 200_003])
def test_host_pipeline_chunks(vc, pinned, chunk):
    """Host-memory batches through the chunked H2D pipeline: strided,
    packed-descriptor (chunked), shuffled-descriptor (one span) and verify,
    from pageable (bounce buffers) and pinned (DMA in place) memory, with
    chunks from 64 KiB (one frame can exceed it) to the default."""
    vc.set_geometry()
    vc.set_host_chunk_bytes(chunk)
    try:
        base, offs, lens = _ragged(41, 400, 0, 70000)
        if pinned:
            pb = vc.PinnedBuffer(base.size)
            pb.array[:] = base
            host = pb.array
        else:
            host = base
        want, want_h = _oracle.frames(base, offs, lens, header=True)
        crc, hdr = vc.frames_host(host, offs, lens, header=True)
        assert np.array_equal(crc, want) and np.array_equal(hdr, want_h)
        perm = np.random.default_rng(5).permutation(offs.size)  # non-monotone offsets: one span
        crc = vc.frames_host(host, offs[perm], lens[perm])
        assert np.array_equal(crc, want[perm])
        stride, flen, n = 1044, 1040, 900
        strided = _prng.frames_stream(n, 1024, stride_pad=0, seed=0x77)
        if pinned:
            ps = vc.PinnedBuffer(strided.size)
            ps.array[:] = strided
            sh = ps.array
        else:
            sh = strided
        assert np.array_equal(vc.frames_host(sh, stride=stride, flen=flen, n=n),
                              _oracle.frames_strided(strided, stride, flen, n))
        tr = _with_trailers(base.copy(), offs, lens)
        tr[int(offs[7]) + 3] ^= 0x01
        if pinned:
            pb.array[:] = tr
            tr = pb.array
        st, ok, nbad = vc.verify_frames_host(tr, offs, lens)
        assert st == vc.VAL_ERR_CRC and nbad == 1 and ok[7] == 0 and ok.sum() == offs.size - 1
    finally:
        vc.set_host_chunk_bytes(0)


def test_concurrent_streams_share_scratch(vc, dev, monkeypatch):
    """Region and ragged calls on four streams at once: each stream has its own
    scratch (kept per stream handle), every result bit-exact. The frame
    batches take the device-binned path (its bucket totals are re-zeroed by
    each batch's last kernel for the next one) and differ in size, so the bin
    scratch also grows between calls."""
    vc.set_ragged_min_frames(1)
    vc.set_geometry()
    streams = [torch.cuda.Stream() for _ in range(4)]
    regions, frames = [], []
    for k, st in enumerate(streams):
        data = _prng.prng_bytes(900 + k, 3_000_000 + 77_777 * k)
        base, offs, lens = _ragged(950 + k, 300 + 1200 * k, 0, 70000)
        regions.append((torch.from_numpy(data).to(dev), data))
        frames.append((torch.from_numpy(base).to(dev), torch.from_numpy(offs.view(np.int64)).to(dev),
                       torch.from_numpy(lens.view(np.int32)).to(dev), base, offs, lens))
    torch.cuda.synchronize()
    outs = []
    for rep in range(3):
        for k, st in enumerate(streams):
            with torch.cuda.stream(st):
                r = vc.region(regions[k][0], stream=st)
                c = vc.frames(frames[k][0], off=frames[k][1], length=frames[k][2], stream=st)
                outs.append((k, r, c))
    torch.cuda.synchronize()
    for k, r, c in outs:
        assert (int(r.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == _oracle.crc32(regions[k][1])
        _, _, _, base, offs, lens = frames[k]
        assert np.array_equal(_u32(c), _oracle.frames(base, offs, lens))


def test_cfg3_full_size_properties(vc, dev):
    """1 M x 16 KiB explicit-offset DATA frames (BASELINE cfg3, 17.2 GB).
    Size-independent checks: trailer write -> verify round trip has zero
    mismatches, exactly the corrupted frames fail, and a random sample of
    frames is bit-exact against the oracle."""
    vc.set_geometry()
    n, payload = 1 << 20, 16384
    flen, stride = 8 + 8 + payload, 8 + 8 + payload + 4
    g = torch.Generator(device=dev).manual_seed(3)
    buf = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device=dev, generator=g)
    buf[:, 0], buf[:, 1], buf[:, 2], buf[:, 3] = 5, 1, (payload + 8) & 0xFF, (payload + 8) >> 8
    buf[:, 4:8] = 0
    offs = torch.arange(n, device=dev, dtype=torch.int64) * payload
    buf[:, 8:16] = offs.view(torch.uint8).view(n, 8)
    flat = buf.view(-1)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    hdr = torch.empty(n, dtype=torch.int32, device=dev)
    vc.frames(flat, stride=stride, flen=flen, n=n, out_crc=crc, out_hdr=hdr)
    buf[:, flen:flen + 4] = crc.view(torch.uint8).view(n, 4)
    ok, nbad = vc.verify_frames(flat, stride=stride, flen=flen, n=n)
    torch.cuda.synchronize()
    assert int(nbad.item()) == 0 and bool(ok.all())
    hot = [0, 1, n // 2, n - 1]
    for i in hot[:3]:
        buf[i, 100 + i % 7] ^= 0x01
    ok, nbad = vc.verify_frames(flat, stride=stride, flen=flen, n=n)
    torch.cuda.synchronize()
    assert int(nbad.item()) == 3
    bad_idx = torch.nonzero(ok == 0).flatten().cpu().tolist()
    assert bad_idx == hot[:3]
    for i in hot[:3]:
        buf[i, 100 + i % 7] ^= 0x01
    rng = np.random.default_rng(5)
    sample = np.unique(np.concatenate([rng.choice(n, 1500, replace=False), hot]))
    rows = buf[torch.from_numpy(sample).to(dev)].cpu().numpy().reshape(-1)
    want, want_h = _oracle.frames_strided(rows, stride, flen, sample.size, header=True)
    assert np.array_equal(_u32(crc)[sample], want)
    assert np.array_equal(_u32(hdr)[sample], want_h)
    h0 = _u32(hdr)
    assert np.all(h0 == h0[0])  # every header is identical in this stream
    # The same 17.2 GB through the descriptor paths (u64 offsets past 4 GiB):
    # uniform (len_hint) and device-binned ragged (len_hint 0) equal strided.
    d_off = torch.arange(n, device=dev, dtype=torch.int64) * stride
    d_len = torch.full((n,), flen, dtype=torch.int32, device=dev)
    for hint in (flen, 0):
        c2 = vc.frames(flat, off=d_off, length=d_len, len_hint=hint)
        torch.cuda.synchronize()
        assert torch.equal(c2, crc), hint


def test_no_cpu_fallback_symbols_loaded(vc):
    # The product library must be the one mapped in this process.
    maps = open("/proc/self/maps").read()
    assert os.path.basename(vc.LIB_PATH) in maps


# ---- ragged path: device binning by length class + grouped launch ------------
@pytest.fixture
def binned_always(vc):
    """Pin the device-binned path even for batches below its size threshold."""
    vc.set_ragged_min_frames(1)


def _run_ragged(vc, dev, base, offs, lens, header=False):
    vc.set_geometry()  # automatic geometry: len_hint == 0 selects the binned path
    d = torch.from_numpy(base).to(dev)
    crc = torch.empty(offs.size, dtype=torch.int32, device=dev)
    hdr = torch.empty(offs.size, dtype=torch.int32, device=dev) if header else None
    vc.frames(d, off=torch.from_numpy(offs.view(np.int64)).to(dev),
              length=torch.from_numpy(lens.view(np.int32)).to(dev), out_crc=crc, out_hdr=hdr, len_hint=0)
    torch.cuda.synchronize()
    return _u32(crc), (_u32(hdr) if header else None)


@pytest.mark.parametrize("seed,n,lo,hi", [(1, 1, 5, 5), (2, 3, 0, 2000), (3, 700, 0, 70000), (4, 5000, 8, 1023),
                                          (5, 4000, 50000, 66000), (6, 20000, 0, 70000)])
@pytest.mark.parametrize("binned", [True, False])
def test_ragged_binned(vc, dev, seed, n, lo, hi, binned, monkeypatch):
    if binned:
        vc.set_ragged_min_frames(1)
    base, offs, lens = _ragged(seed, n, lo, hi)
    got, got_h = _run_ragged(vc, dev, base, offs, lens, header=True)
    want, want_h = _oracle.frames(base, offs, lens, header=True)
    assert np.array_equal(got, want)
    assert np.array_equal(got_h, want_h)


def test_ragged_log_uniform_cfg5_shape(vc, dev, binned_always):
    rng = np.random.default_rng(55)
    n = 3000
    lens = (np.exp(rng.uniform(np.log(520), np.log(65532), n))).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 4)[:-1]]).astype(np.uint64)
    base = _prng.prng_bytes(56, int(offs[-1]) + int(lens[-1]) + 8)
    got, _ = _run_ragged(vc, dev, base, offs, lens)
    assert np.array_equal(got, _oracle.frames(base, offs, lens))


@pytest.mark.parametrize("binned", [True, False])
def test_ragged_every_length_and_verify(vc, dev, binned, monkeypatch):
    if binned:
        vc.set_ragged_min_frames(1)
    lens = np.arange(0, 2500, dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 4)]).astype(np.uint64)
    base = _prng.prng_bytes(57, int(offs[-1]) + 2600)
    got, _ = _run_ragged(vc, dev, base, offs, lens)
    assert np.array_equal(got, _oracle.frames(base, offs, lens))
    base = _with_trailers(base, offs, lens)
    base[int(offs[1234]) + 3] ^= 0x40
    ok, nbad = vc.verify_frames(torch.from_numpy(base).to(dev), off=torch.from_numpy(offs.view(np.int64)).to(dev),
                                length=torch.from_numpy(lens.view(np.int32)).to(dev), len_hint=0)
    torch.cuda.synchronize()
    assert int(nbad.item()) == 1 and int(ok.cpu().numpy().argmin()) == 1234


def test_empty_batches(vc, dev):
    d = torch.zeros(16, dtype=torch.uint8, device=dev)
    e64 = torch.zeros(0, dtype=torch.int64, device=dev)
    e32 = torch.zeros(0, dtype=torch.int32, device=dev)
    out = vc.frames(d, off=e64, length=e32, len_hint=0)
    out2 = vc.frames(d, stride=4, flen=4, n=0)
    torch.cuda.synchronize()
    assert out.numel() == 0 and out2.numel() == 0


# Batches whose frame groups leave a partial last wave-round (256 CUs x 16
# waves on MI355X): the library re-cuts those frames with more lanes per frame
# in a second launch. Strided and descriptor mode, header_crc, verify with a
# corrupted frame inside the tail, and a byte-misaligned base.
@pytest.mark.parametrize("L,extra", [(60000, 37), (1000, 1000), (16400, 4097), (4200, 1)])
def test_wave_round_tail(vc, dev, L, extra):
    per = 64 // vc.lanes_per_frame(L)
    n = 256 * 16 * per + extra
    stride = L + 4
    g = torch.Generator(device=dev).manual_seed(L + extra)
    raw = torch.randint(0, 256, (n * stride + 3,), dtype=torch.uint8, device=dev, generator=g)
    buf = raw[3:]
    host = buf.cpu().numpy()
    want, want_h = _oracle.frames_strided(host, stride, L, n, header=True, nthreads=16)
    hdr = torch.empty(n, dtype=torch.int32, device=dev)
    crc = vc.frames(buf, stride=stride, flen=L, n=n, out_hdr=hdr)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * stride
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    crc_d = vc.frames(buf, off=offs, length=lens, len_hint=L)
    torch.cuda.synchronize()
    assert np.array_equal(_u32(crc), want)
    assert np.array_equal(_u32(hdr), want_h)
    assert np.array_equal(_u32(crc_d), want)
    buf.view(n, stride)[:, L:L + 4] = crc.view(torch.uint8).view(n, 4)
    bad = n - 2
    buf[bad * stride + L // 2] ^= 0x10
    ok, nbad = vc.verify_frames(buf, stride=stride, flen=L, n=n)
    torch.cuda.synchronize()
    okh = ok.cpu().numpy()
    assert int(nbad.item()) == 1 and int(okh.argmin()) == bad and int(okh.sum()) == n - 1


@pytest.mark.parametrize("strided,payload,per", [
    (True, 16384, 8),    # strided groups of 8 x 16 KiB: one queue word
    (False, 65516, 4),   # descriptor groups of 4 x 64 KiB: one queue word
    (True, 4184, 8),     # strided groups of 8 x 4.2 KiB (34 KB): 64 queue partitions
    (False, 4184, 8),    # descriptor groups of 8 x 4.2 KiB: 64 queue partitions
    (False, 1084, 16),   # descriptor groups of 16 x 1.1 KiB: 64 queue partitions, dequeued one group ahead
])
def test_dynamic_tail_every_frame(vc, dev, strided, payload, per):
    """Launches long enough for the dynamic tail (k_frames: the last half of
    the group rounds come from a queue, one word for long groups, 64
    partitions for shorter ones): 4 full rounds of the machine plus a partial
    one, every frame checked against the oracle, then the same batch again
    (the queue must have been re-zeroed by the previous launch)."""
    vc.set_geometry()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = cus * 16 * per * 4 + 777
    flen = 8 + 8 + payload
    stride = flen + 4
    assert vc.lanes_per_frame(flen) == 64 // per
    g = torch.Generator(device=dev).manual_seed(11)
    buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=dev, generator=g)
    kw = dict(stride=stride, flen=flen, n=n) if strided else dict(
        off=torch.arange(n, device=dev, dtype=torch.int64) * stride,
        length=torch.full((n,), flen, dtype=torch.int32, device=dev), len_hint=flen)
    host = buf.cpu().numpy()
    offs = np.arange(n, dtype=np.uint64) * np.uint64(stride)
    want = _oracle.frames(host, offs, np.full(n, flen, np.uint32), nthreads=16)
    for _ in range(2):
        crc = vc.frames(buf, **kw)
        torch.cuda.synchronize()
        assert np.array_equal(_u32(crc), want)


@pytest.mark.parametrize("G,depth", [(2, -1), (4, -1), (2, -2), (4, -3), (2, 1), (4, 1)])
def test_ring_prefetch_multi_pass(vc, dev, G, depth):
    """Multi-pass batches at 2 and 4 lanes per frame hash each round in its
    registers and refill them in place (rings of 3 and 2 rounds by default):
    mixed lengths 0..3,000 B (1 to 24 rounds, so frames longer than the ring
    refill it), unaligned starts, against the oracle, with the automatic depth
    (-1), the other ring, and the copy-and-refill loop."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = cus * 16 * (64 // G) * 3 + 555  # three passes of the machine and a partial one
    base, offs, lens = _ragged_fast(0x71 + G, n, 0, 3000)
    vc.set_geometry(G, depth)
    try:
        d = torch.from_numpy(base).to(dev)
        crc = vc.frames(d, off=torch.from_numpy(offs.view(np.int64)).to(dev),
                        length=torch.from_numpy(lens.view(np.int32)).to(dev), len_hint=1500)
        torch.cuda.synchronize()
    finally:
        vc.set_geometry()
    assert np.array_equal(_u32(crc), _oracle.frames(base, offs, lens, nthreads=16))


@pytest.mark.parametrize("G,depth", [(2, -1), (4, -1), (2, -2), (4, -3)])
def test_ring_prefetch_verify_and_header(vc, dev, G, depth):
    """The in-place rings on the verify kernel with header_crc (multi-pass):
    trailers written by the oracle, 97 frames corrupted (trailer bytes and
    frame bytes in every round position), verdicts, mismatch count, the
    computed CRCs and header_crcs against the oracle."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = cus * 16 * (64 // G) * 2 + 333
    base, offs, lens = _ragged_fast(0x91 + G, n, 8, 2500)
    crc_want, hdr_want = _oracle.frames(base, offs, lens, header=True, nthreads=16)
    tr = np.frombuffer(crc_want.astype("<u4").tobytes(), np.uint8).reshape(-1, 4)
    idx = (offs + lens.astype(np.uint64)).astype(np.int64)
    for k in range(4):
        base[idx + k] = tr[:, k]
    rng = np.random.default_rng(G)
    bad = rng.choice(n, 97, replace=False)
    for k, i in enumerate(bad):
        o, l = int(offs[i]), int(lens[i])
        pos = o + l + (k % 4) if k % 3 == 0 else o + int(rng.integers(0, l))
        base[pos] ^= np.uint8(1 << (k % 8))
    want_ok, want_bad = _oracle.verify_frames(base, offs, lens, nthreads=16)
    assert want_bad == 97
    vc.set_geometry(G, depth)
    try:
        d = torch.from_numpy(base).to(dev)
        crc = torch.empty(n, dtype=torch.int32, device=dev)
        hdr = torch.empty(n, dtype=torch.int32, device=dev)
        ok, nbad = vc.verify_frames(d, off=torch.from_numpy(offs.view(np.int64)).to(dev),
                                    length=torch.from_numpy(lens.view(np.int32)).to(dev), out_crc=crc, out_hdr=hdr,
                                    len_hint=1200)
        torch.cuda.synchronize()
    finally:
        vc.set_geometry()
    assert int(nbad.item()) == 97
    assert np.array_equal(ok.cpu().numpy(), want_ok)
    crc2, hdr2 = _oracle.frames(base, offs, lens, header=True, nthreads=16)
    assert np.array_equal(_u32(crc), crc2) and np.array_equal(_u32(hdr), hdr2)


def _ragged_fast(seed, n, lo, hi):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.cumsum(lens.astype(np.uint64) + 4 + rng.integers(0, 7, n).astype(np.uint64)) - lens - 4
    base = rng.integers(0, 256, int(offs[-1]) + int(lens[-1]) + 16, dtype=np.uint8)
    return base, offs.astype(np.uint64), lens
