"""k_frames_split (small batches of long frames, one workgroup per frame):
bit-exact against the oracle (reference src/val_core.c:150-160, framing
:718-834, RX compare :963-974) for strided and descriptor batches, frames of
one chunk group and of many (the front-to-back group fold), short and empty
frames inside a split batch, unaligned offsets, header_crc, verify with
corruption, and region windows that take the split path (the seed)."""
import numpy as np
import pytest
import torch

from tests import _oracle, _prng

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def vc():
    import val_protocol_amd.crc as vc

    vc.init(0)
    return vc


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,payload", [(1, 8192), (3, 16384), (17, 16384), (256, 65516), (300, 8176), (64, 65520)])
def test_strided_long_frames(vc, n, payload):
    stream = _prng.frames_stream(n, payload, seed=0x5B + n + payload)
    flen = 16 + payload
    stride = flen + 4
    d = torch.from_numpy(stream).to(DEV)
    crc = torch.zeros(n, dtype=torch.int32, device=DEV)
    hdr = torch.zeros(n, dtype=torch.int32, device=DEV)
    vc.frames(d, stride=stride, flen=flen, n=n, out_crc=crc, out_hdr=hdr)
    want, want_h = _oracle.frames_strided(stream, stride, flen, n, header=True)
    assert np.array_equal(_u32(crc), want)
    assert np.array_equal(_u32(hdr), want_h)


@pytest.mark.parametrize("hint,lo,hi", [(8192, 0, 110_000), (16400, 16000, 16800), (65532, 60000, 65540)])
def test_descriptor_long_frames(vc, hint, lo, hi):
    """Frames longer than 16 chunks of the hint's W fold several groups; short
    and empty frames ride in the same batch."""
    rng = np.random.default_rng(hint)
    n = 200
    lens = rng.integers(lo, hi, n).astype(np.uint32)
    lens[:4] = [0, 1, 3, 7]
    wire = lens.astype(np.int64) + 4 + rng.integers(0, 3, n)
    off = np.concatenate([[1], 1 + np.cumsum(wire)[:-1]]).astype(np.uint64)
    buf = _prng.prng_bytes(hint ^ 0x51, int(off[-1]) + int(wire[-1]) + 4)
    d = torch.from_numpy(buf).to(DEV)
    d_off = torch.from_numpy(off.astype(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(DEV)
    crc = torch.zeros(n, dtype=torch.int32, device=DEV)
    hdr = torch.zeros(n, dtype=torch.int32, device=DEV)
    vc.frames(d, off=d_off, length=d_len, out_crc=crc, out_hdr=hdr, len_hint=hint)
    want, want_h = _oracle.frames(buf, off, lens, header=True)
    assert np.array_equal(_u32(crc), want)
    assert np.array_equal(_u32(hdr), want_h)


def test_verify_long_frames_with_corruption(vc):
    n, payload = 120, 32768
    stream = _prng.frames_stream(n, payload, seed=0x7E)
    flen = 16 + payload
    stride = flen + 4
    want = _oracle.frames_strided(stream, stride, flen, n)
    rows = stream.reshape(n, stride)
    rows[:, flen:] = want.astype("<u4").view(np.uint8).reshape(n, 4)
    rng = np.random.default_rng(5)
    bad = rng.choice(n, 9, replace=False)
    for i in bad:
        rows[i, int(rng.integers(0, flen + 4))] ^= 0x10
    d = torch.from_numpy(rows.reshape(-1).copy()).to(DEV)
    ok, nbad = vc.verify_frames(d, stride=stride, flen=flen, n=n)
    got = ok.cpu().numpy()
    assert int(nbad.item()) == 9
    assert set(np.nonzero(got == 0)[0]) == set(bad)


@pytest.mark.parametrize("L", [8192, 8191])
def test_region_windows_through_split(vc, L):
    """Windows up to 8 KiB are one frame of the frames path; at 8 KiB that
    frame takes the split kernel, with the caller's state as its seed."""
    data = _prng.prng_bytes(0xE9 + L, L)
    d = torch.from_numpy(data).to(DEV)
    for st in (0xFFFFFFFF, 0x12345678, 0):
        out = vc.region(d, state_in=st)
        assert int(out.item()) & 0xFFFFFFFF == _oracle.update_state(st, data)
