"""Real reference sessions replayed through the product on the GPU
(tests/golden/session_vectors.json, recorded by `oracle/_ref/provider_harness
none sessions` from the reference's own val_send_files / val_receive_files):

* windowed transfers (tx_flow.window_cap_packets = 64, MTU 1,024 and 16,404):
  every window fill of the real sender, with the include_offset pattern it
  produced, is rebuilt by val_frame_data_batch and CRC'd in one
  val_crc32_frames_host call and one val_crc32_frames_dev launch; the
  stream must equal the frames the reference put on the wire, byte for byte,
  and one batched verify per window must accept all of them;
* resumed VAL_RESUME_TAIL transfers: the tail-window CRCs that crossed the
  wire (the receiver's RESUME_RESP over its partial file, the sender's VERIFY
  request over its own file, the receiver's VERIFY response) must equal
  val_crc32_region_dev over the same windows in HBM.

Reference: src/val_sender.c:205-252,822-841; src/val_receiver.c:158-181,
431-444."""
import numpy as np
import pytest

from tests import _sessions

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
VAL_OK = 0


@pytest.fixture(scope="module")
def vc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import val_protocol_amd.crc as m

    m.init(0)
    m.set_geometry()
    return m


@pytest.fixture(scope="module")
def sessions():
    return _sessions.load()


@pytest.mark.parametrize("name", ["window64_mtu1024", "window64_mtu16404", "resume_tail_cap8m", "resume_tail_cap1k"])
def test_session_windows_replayed(vc, sessions, name):
    import val_protocol_amd.wire as wire

    s = sessions[name]
    file = _sessions.input_file(s)
    dev = torch.device("cuda:0")
    data_recs = [r for r in s["tx_frames"] if r[0] == _sessions.PKT_DATA]
    k = 0
    for pay_off, pay_len, inc, trailers in _sessions.windows(s):
        stream, fo, cl = wire.build_data_batch(file, pay_off, pay_len, pay_off, inc)
        crc = vc.frames_host(stream, off=fo, length=cl)  # one host batch per window fill
        assert np.array_equal(crc, trailers), (name, k)
        d = torch.from_numpy(stream).to(dev)
        d_off = torch.from_numpy(fo.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(cl.astype(np.int32)).to(dev)
        c_dev = vc.frames(d, off=d_off, length=d_len, len_hint=0)  # one device launch per window
        torch.cuda.synchronize()
        assert np.array_equal(c_dev.cpu().numpy().view(np.uint32), trailers), (name, k)
        wire.put_trailers(stream, fo, cl, crc)
        assert np.array_equal(stream, _sessions.wire_stream(data_recs[k:k + len(trailers)], file)), (name, k)
        st, ok, nbad = vc.verify_frames_host(stream, off=fo, length=cl)
        assert st == VAL_OK and nbad == 0 and ok.all()
        k += len(trailers)
    assert k == len(data_recs)


@pytest.mark.parametrize("name,cap", [("resume_tail_cap8m", 8 << 20), ("resume_tail_cap1k", 1024),
                                      ("resume_tail_mismatch", 8192)])
def test_resume_verify_window_on_gpu(vc, sessions, name, cap):
    s = sessions[name]
    c = _sessions.control(s, vc.lib())
    dev = torch.device("cuda:0")
    part = torch.from_numpy(_sessions.receiver_existing(s)).to(dev)
    src = torch.from_numpy(_sessions.input_file(s)).to(dev)
    vlen = int(c["resp_verify_length"])
    assert vlen == min(s["existing"], cap)
    recv = vc.region(part[s["existing"] - vlen:s["existing"]])  # the receiver's tail window (RESUME_RESP)
    send = vc.region(src[c["req_offset"]:c["req_offset"] + c["req_length"]])  # the sender's VERIFY request window
    torch.cuda.synchronize()
    fin = lambda t: (int(t.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF  # noqa: E731
    assert fin(recv) == c["resp_verify_crc"] == c["receiver_crc"]
    assert fin(send) == c["req_crc"]
    assert (c["result"] == VAL_OK) == (fin(recv) == fin(send))
