"""BASELINE configs at full size on the GPU, generated exactly as bench.py
generates them (cfg1, the 1 MiB loopback, is tests/test_gpu_dropin.py::
test_loopback_1mib_frame_log; cfg3 is test_gpu_parity.py::
test_cfg3_full_size_properties). Bit-exact against the oracle on every frame
where the oracle finishes in seconds (cfg2, cfg5), on samples plus
size-independent properties (write -> verify round trip, exactly the
corrupted frames rejected, sharded == whole) where it would not (cfg4)."""
import numpy as np
import pytest

import bench
from tests import _oracle

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


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda:0")


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def test_cfg2_full_batch_bit_exact(vc, dev):
    """64 K DATA frames x 1 KiB payload, trailer only (BASELINE configs[1]):
    every one of the 65,536 trailers against the oracle, then RX verify."""
    n, payload, explicit, _ = bench.CONFIGS["cfg2"]
    buf, flen, stride = bench.make_frames(torch, dev, n, payload, explicit, 0, seed=2)
    flat = buf.view(-1)
    crc = vc.frames(flat, stride=stride, flen=flen, n=n)
    torch.cuda.synchronize()
    host = flat.cpu().numpy()
    assert np.array_equal(_u32(crc), _oracle.frames_strided(host, stride, flen, n, nthreads=16))
    buf[:, flen:flen + 4] = crc.view(torch.uint8).view(n, 4)
    buf[4321, 500] ^= 0x80
    ok, nbad = vc.verify_frames(flat, stride=stride, flen=flen, n=n)
    torch.cuda.synchronize()
    okh = ok.cpu().numpy()
    assert int(nbad.item()) == 1 and int(okh.argmin()) == 4321 and int(okh.sum()) == n - 1


def _cfg4(dev):
    """The 8 GiB file framed at MTU 65,536: 131,112 frames of 65,516 B payload
    and a last frame of 800 B (BASELINE configs[3])."""
    n, payload, explicit, _ = bench.CONFIGS["cfg4"]
    buf, flen, stride = bench.make_frames(torch, dev, n, payload, explicit, 0, seed=4)
    last_pay = (8 << 30) - (n - 1) * payload
    assert last_pay == 800
    last_content = last_pay + 8
    buf[n - 1, 2], buf[n - 1, 3] = last_content & 0xFF, last_content >> 8
    d_off = torch.arange(n, device=dev, dtype=torch.int64) * stride
    d_len = torch.full((n,), flen, dtype=torch.int32, device=dev)
    d_len[n - 1] = 8 + last_content
    return buf, flen, stride, d_off, d_len


def test_cfg4_8gib_file_sharded(vc, dev):
    buf, flen, stride, d_off, d_len = _cfg4(dev)
    n = d_off.numel()
    flat = buf.view(-1)
    whole = vc.frames(flat, off=d_off, length=d_len, len_hint=flen)
    # two logical shards (the split bench.py --gpus 2 uses), each its own launch
    from val_protocol_amd.shard import shard_frames

    lens = d_len.cpu().numpy().astype(np.uint32)
    parts = []
    for r in range(2):
        s, c = shard_frames(n, 2, r, lens)
        parts.append(vc.frames(flat, off=d_off[s:s + c].contiguous(), length=d_len[s:s + c].contiguous(),
                               len_hint=flen))
    torch.cuda.synchronize()
    assert torch.equal(torch.cat(parts), whole)
    # sample against the oracle, including the 816-B last frame
    rng = np.random.default_rng(4)
    sample = np.unique(np.concatenate([rng.choice(n, 200, replace=False), [0, n - 2, n - 1]]))
    offs = d_off.cpu().numpy()
    pieces = [flat[int(offs[i]):int(offs[i]) + int(lens[i])].cpu().numpy() for i in sample]
    so = np.concatenate([[0], np.cumsum([p.size for p in pieces])[:-1]]).astype(np.uint64)
    want = _oracle.frames(np.concatenate(pieces), so, lens[sample])
    assert np.array_equal(_u32(whole)[sample], want)
    # trailers written -> verify accepts all, rejects exactly the corrupted ones
    tidx = ((d_off + d_len.long())[:, None] + torch.arange(4, device=dev)[None, :]).reshape(-1)
    flat[tidx] = whole.view(torch.uint8)
    bad = [7, n // 2, n - 1]
    for i in bad:
        flat[int(offs[i]) + 100] ^= 0x04
    ok, nbad = vc.verify_frames(flat, off=d_off, length=d_len, len_hint=flen)
    torch.cuda.synchronize()
    assert int(nbad.item()) == 3
    assert torch.nonzero(ok == 0).flatten().cpu().tolist() == bad


def test_cfg5_mixed_mtu_full_batch_and_windows(vc, dev):
    """262,144 frames, payload log-uniform in [512, 65,516], one in 8 with an
    implied offset, packed byte-unaligned (BASELINE configs[4]): every trailer
    and header_crc through the device-binned ragged path against the oracle;
    then the VAL_RESUME_TAIL verify windows {1 KiB, 8 KiB, 8 MiB, 256 MiB} over
    the same stream (src/val_receiver.c:158-181)."""
    n = bench.CONFIGS["cfg5"][0]
    buf, d_off, d_len = bench.make_ragged_frames(torch, dev, n, seed=5)
    hdr = torch.empty(n, dtype=torch.int32, device=dev)
    crc = vc.frames(buf, off=d_off, length=d_len, out_hdr=hdr, len_hint=0)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    offs = d_off.cpu().numpy().astype(np.uint64)
    lens = d_len.cpu().numpy().astype(np.uint32)
    want, want_h = _oracle.frames(host, offs, lens, header=True, nthreads=16)
    assert np.array_equal(_u32(crc), want)
    assert np.array_equal(_u32(hdr), want_h)
    for wlen in (1 << 10, 8 << 10, 8 << 20, 256 << 20):
        st = vc.region(buf[:wlen])
        torch.cuda.synchronize()
        assert (int(st.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == _oracle.crc32(host[:wlen]), wlen
