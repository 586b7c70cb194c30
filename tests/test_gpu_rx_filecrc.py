"""the receiver's rolling file CRC as a by-product of the
batched RX verify (reference src/val_receiver.c:794,891,1004-1005: for every
in-order DATA frame, crc_state = val_crc32_update_state(crc_state, payload)).
The verify kernel writes each frame's payload register from zero; the host
folds them with val_crc32_fold_payload_states. Checked against the oracle's
update_state over the payload bytes, and against the reference's own file CRC
of the 1 MiB loopback transfer (tests/golden/dropin_vectors.json)."""
import json
import os

import numpy as np
import pytest

from tests import _oracle, _prng

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def vc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import val_protocol_amd.crc as m

    m.init(0)
    m.set_geometry()
    return m


def _stream(seed, n, lo, hi, explicit_every=3):
    """DATA frames with random payload sizes, some implied-offset, plus trailers."""
    import val_protocol_amd.wire as w

    rng = np.random.default_rng(seed)
    pay_len = rng.integers(lo, hi + 1, n).astype(np.uint32)
    inc = (np.arange(n) % explicit_every != 1).astype(np.uint8)
    file = _prng.prng_bytes(seed, int(pay_len.sum()) + 1)
    pay_off = np.concatenate([[0], np.cumsum(pay_len.astype(np.uint64))[:-1]]).astype(np.uint64)
    stream, fo, cl = w.build_data_batch(file, pay_off, pay_len, pay_off, inc)
    crc = _oracle.frames(stream, fo, cl)
    w.put_trailers(stream, fo, cl, crc)
    return stream, fo, cl, pay_len, inc, file


def _want_states(file, pay_len):
    offs = np.concatenate([[0], np.cumsum(pay_len.astype(np.uint64))]).astype(np.int64)
    return np.array([_oracle.update_state(0, file[offs[i]:offs[i + 1]]) for i in range(pay_len.size)], np.uint32)


@pytest.mark.parametrize("hint", ["ragged", "uniform"])
@pytest.mark.parametrize("seed,n,lo,hi", [(1, 5000, 0, 1200), (2, 700, 0, 65516), (3, 40, 65000, 65516)])
def test_payload_states_device(vc, hint, seed, n, lo, hi, monkeypatch):
    import val_protocol_amd.wire as w

    if hint == "ragged":
        vc.set_ragged_min_frames(1)
    stream, fo, cl, pay_len, inc, file = _stream(seed, n, lo, hi)
    assert np.array_equal(w.payload_lens(stream, fo, cl), pay_len)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(stream).to(dev)
    ok, nbad, pay = vc.verify_frames_ex(d, off=torch.from_numpy(fo.astype(np.int64)).to(dev),
                                        length=torch.from_numpy(cl.astype(np.int32)).to(dev),
                                        len_hint=0 if hint == "ragged" else int(cl.max()))
    torch.cuda.synchronize()
    assert int(nbad.item()) == 0 and bool(ok.all())
    assert np.array_equal(pay.cpu().numpy().view(np.uint32), _want_states(file, pay_len))


@pytest.mark.parametrize("G", [1, 8, 64])
def test_payload_states_strided_and_geometries(vc, G):
    """Strided batches at forced geometries (unit grid, tiny frames, tails)."""
    n, payload = 3000, 333
    stream = _prng.frames_stream(n, payload, stride_pad=1, seed=9)
    flen, stride = 8 + 8 + payload, 8 + 8 + payload + 4 + 1
    crc = _oracle.frames_strided(stream, stride, flen, n)
    rows = stream.reshape(n, stride)
    rows[:, flen:flen + 4] = crc.view(np.uint8).reshape(n, 4)
    vc.set_lanes_per_frame(G)
    try:
        dev = torch.device("cuda:0")
        d = torch.from_numpy(stream).to(dev)
        ok, nbad, pay = vc.verify_frames_ex(d, stride=stride, flen=flen, n=n)
        torch.cuda.synchronize()
    finally:
        vc.set_lanes_per_frame(0)
    assert int(nbad.item()) == 0
    want = np.array([_oracle.update_state(0, rows[i, 16:flen]) for i in range(n)], np.uint32)
    assert np.array_equal(pay.cpu().numpy().view(np.uint32), want)


def test_short_frames_and_control_frames(vc):
    """Frames shorter than their prefix carry no payload (state 0); frames
    without OFFSET_PRESENT hash everything after the 8-byte header."""
    lens = np.array([0, 3, 7, 8, 9, 15, 16, 17, 40], np.uint32)
    base = _prng.prng_bytes(12, 400)
    offs = (np.arange(lens.size, dtype=np.uint64) * 40).astype(np.uint64)
    for i, o in enumerate(offs):
        base[int(o) + 1] = 1 if i % 2 else 0
        c = _oracle.crc32(base[int(o):int(o) + int(lens[i])])
        base[int(o) + int(lens[i]):int(o) + int(lens[i]) + 4] = np.frombuffer(c.to_bytes(4, "little"), np.uint8)
    st, ok, nbad, pay = vc.verify_frames_ex_host(base, off=offs, length=lens)
    assert st == vc.VAL_OK and nbad == 0
    for i, (o, L) in enumerate(zip(offs, lens)):
        pre = 16 if (L >= 8 and base[int(o) + 1] & 1) else 8
        want = _oracle.update_state(0, base[int(o) + pre:int(o) + int(L)]) if L >= pre else 0
        assert pay[i] == want, (i, L)


def test_loopback_rx_rolling_crc_equals_file_crc(vc):
    """The 1 MiB / MTU 1024 transfer (BASELINE configs[0]): the receiver's
    DATA frames, verified in one batch; their folded payload states are the
    reference's file CRC (ts_file_crc32, unit_tests/support/test_support.c:
    1458-1472)."""
    import val_protocol_amd.wire as w

    with open(os.path.join(ROOT, "tests", "golden", "dropin_vectors.json")) as f:
        lb = json.load(f)["loopback"]
    file = _prng.prng_bytes(lb["file_seed"], lb["bytes"])
    parts, off, lens, pos = [], [], [], 0
    for ptype, wire_len, trailer, foff, prefix in lb["tx_frames"]:
        if ptype != 5:
            continue
        head = np.frombuffer(bytes.fromhex(prefix), np.uint8)
        body = np.concatenate([head, file[foff:foff + wire_len - 4 - head.size]])
        parts += [body, np.frombuffer(int(trailer).to_bytes(4, "little"), np.uint8)]
        off.append(pos)
        lens.append(body.size)
        pos += wire_len
    stream = np.concatenate(parts)
    off, lens = np.array(off, np.uint64), np.array(lens, np.uint32)
    st, ok, nbad, pay = vc.verify_frames_ex_host(stream, off=off, length=lens)
    assert st == vc.VAL_OK and nbad == 0
    state, nf = vc.fold_payload_states(0xFFFFFFFF, pay, w.payload_lens(stream, off, lens), ok)
    assert nf == 1045 and state ^ 0xFFFFFFFF == lb["file_crc"]


def test_fold_stops_at_first_rejected_frame(vc):
    import val_protocol_amd.wire as w

    stream, fo, cl, pay_len, inc, file = _stream(7, 300, 100, 3000)
    stream[int(fo[123]) + 30] ^= 0x08
    st, ok, nbad, pay = vc.verify_frames_ex_host(stream, off=fo, length=cl)
    assert st == vc.VAL_ERR_CRC and nbad == 1 and ok[123] == 0
    state, nf = vc.fold_payload_states(0xFFFFFFFF, pay, w.payload_lens(stream, fo, cl), ok)
    assert nf == 123
    assert state == _oracle.update_state(0xFFFFFFFF, file[:int(pay_len[:123].sum())])
