"""Recorded reference sessions (tests/golden/session_vectors.json, written by
`oracle/_ref/provider_harness none sessions`): windowed transfers with
tx_flow.window_cap_packets = 64 at MTU 1,024 and 16,404, and resumed
VAL_RESUME_TAIL transfers over a partial receiver file at the default 8 MiB
cap, at 1 KiB, and with a corrupted tail. Checked here without a GPU: the
recording is self-consistent against the oracle, the sender's windows have
the reference's include_offset pattern, and the product's CPU-routed host
batch path (below the host-batch crossover) reproduces every window byte
for byte. tests/test_gpu_sessions.py replays the same on the GPU.
Reference: src/val_sender.c:205-252,822-841; src/val_receiver.c:158-181,
431-444; window negotiation src/val_core.c:1755,1810-1834."""
import numpy as np
import pytest

import val_protocol_amd.crc as vc
import val_protocol_amd.wire as wire
from tests import _oracle, _sessions

VAL_OK, VAL_ERR_RESUME_VERIFY = 0, -7


@pytest.fixture(scope="module")
def sessions():
    return _sessions.load()


def test_sessions_ran_clean(sessions):
    assert set(sessions) == {"window64_mtu1024", "window64_mtu16404", "resume_tail_cap8m", "resume_tail_cap1k",
                             "resume_tail_mismatch"}
    for s in sessions.values():
        assert s["tx_status"] == VAL_OK and s["rx_status"] == VAL_OK and s["equal"] == 1, s["name"]
        assert s["tx_crc_errors"] == 0 and s["rx_crc_errors"] == 0
        file = _sessions.input_file(s)
        assert _oracle.crc32(file) == s["file_crc"]
        for side in ("tx_frames", "rx_frames"):
            for rec in s[side]:  # every trailer on the wire = the reference CRC of its frame
                assert _oracle.crc32(_sessions.frame_bytes(rec, file)) == rec[2], (s["name"], side, rec[:4])


@pytest.mark.parametrize("name", ["window64_mtu1024", "window64_mtu16404"])
def test_window_fills_and_include_offset(sessions, name):
    """The real sender fills windows of up to 64 frames, and only the first
    frame of each fill carries an explicit offset (next_to_send == last_acked:
    every earlier frame is acknowledged before the next fill)."""
    s = sessions[name]
    ws = _sessions.windows(s)
    assert max(len(w[0]) for w in ws) == 64 and len(ws) >= 3
    total = 0
    for pay_off, pay_len, inc, _ in ws:
        assert inc[0] == 1 and not inc[1:].any()
        assert np.array_equal(pay_off[1:], pay_off[:-1] + pay_len[:-1])  # contiguous file ranges
        total += int(pay_len.sum())
    assert total == s["bytes"]
    maxp = s["mtu"] - 12
    assert all(int(l) <= maxp - 8 * int(i) for w in ws for l, i in zip(w[1], w[2]))


@pytest.fixture
def cpu_routed():
    vc.set_host_batch_min_bytes(1 << 62)
    yield
    vc.set_host_batch_min_bytes(-1)


@pytest.mark.parametrize("name", ["window64_mtu1024", "window64_mtu16404", "resume_tail_cap8m"])
def test_windows_replayed_cpu_routed(sessions, name, cpu_routed):
    """Each window fill rebuilt by the product's framer and CRC'd by the host
    batch call (CPU engine below the crossover) equals the recorded frames."""
    s = sessions[name]
    file = _sessions.input_file(s)
    data_recs = [r for r in s["tx_frames"] if r[0] == _sessions.PKT_DATA]
    k = 0
    for pay_off, pay_len, inc, trailers in _sessions.windows(s):
        stream, fo, cl = wire.build_data_batch(file, pay_off, pay_len, pay_off, inc)
        crc = vc.frames_host(stream, off=fo, length=cl)
        assert np.array_equal(crc, trailers)
        wire.put_trailers(stream, fo, cl, crc)
        want = _sessions.wire_stream(data_recs[k:k + len(trailers)], file)
        assert np.array_equal(stream, want)
        st, ok, nbad = vc.verify_frames_host(stream, off=fo, length=cl)
        assert st == VAL_OK and nbad == 0 and ok.all()
        k += len(trailers)
    assert k == len(data_recs)


@pytest.mark.parametrize("name,cap", [("resume_tail_cap8m", 8 << 20), ("resume_tail_cap1k", 1024),
                                      ("resume_tail_mismatch", 8192)])
def test_resume_verify_crcs_against_oracle(sessions, name, cap):
    """The tail-window CRCs that crossed the wire: the receiver's over the last
    min(existing, cap) bytes of its partial file (RESUME_RESP), the sender's
    over the same window of its own file (VERIFY request), and the verdict."""
    s = sessions[name]
    c = _sessions.control(s, vc.lib())
    part, file = _sessions.receiver_existing(s), _sessions.input_file(s)
    vlen = min(s["existing"], cap)
    assert c["action"] == 2 and c["resume_offset"] == s["existing"]  # VAL_RESUME_VERIFY_FIRST
    assert c["resp_verify_length"] == vlen and c["req_length"] == vlen
    assert c["req_offset"] == s["existing"] - vlen
    assert c["resp_verify_crc"] == _oracle.crc32(part[-vlen:])
    assert c["req_crc"] == _oracle.crc32(file[s["existing"] - vlen:s["existing"]])
    assert c["receiver_crc"] == c["resp_verify_crc"]
    if s["flip"] < 0:
        assert c["result"] == VAL_OK and c["req_crc"] == c["resp_verify_crc"]
    else:
        assert c["result"] == VAL_ERR_RESUME_VERIFY and c["req_crc"] != c["resp_verify_crc"]
