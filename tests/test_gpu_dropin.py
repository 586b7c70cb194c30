"""Drop-in witness on the GPU box, from committed reference fixtures.

`tests/golden/dropin_vectors.json` was written in the build container by
`oracle/_ref/provider_harness none fixtures` (oracle/Makefile `golden`): the
reference's own protocol code (/root/reference/src, compiled with gcc, built-in
CRC) framing DATA packets (src/val_core.c:718-866), verifying them
(src/val_core.c:880-1073), framing TX windows as the sender does
(src/val_sender.c:258-315,822-841) and running the 1 MiB / MTU 1024 loopback
transfer of BASELINE configs[0] (unit_tests/send_receive/test_single_file.c:
9-11,155-161), whose every transport.send is logged.

Here the same bytes are rebuilt (payloads are oracle/prng.h streams,
tests/_prng.py) and pushed through the product: the crc32_func_t hook
`val_gpu_crc32_provider`, `val_crc32_frames_host`, `val_crc32_verify_frames_host`
and the device entry points. Every trailer and every accept/reject verdict must
equal the reference's. No reference code runs here.
"""
import json
import os

import numpy as np
import pytest

from tests import _oracle, _prng

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAL_OK, VAL_ERR_CRC, VAL_ERR_INVALID_ARG = 0, -6, -1


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(ROOT, "tests", "golden", "dropin_vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def vc():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import val_protocol_amd.crc as m

    m.init(0)
    return m


@pytest.fixture(scope="module")
def wire(vc):
    import val_protocol_amd.wire as w

    return w


def _le32(b) -> int:
    return int.from_bytes(bytes(b[:4]), "little")


def _data_frame(wire, payload, offset, include_offset):
    """One DATA frame built by the product's batch framer (trailer zero)."""
    stream, fo, cl = wire.build_data_batch(payload, [0], [payload.size], [offset], [1 if include_offset else 0])
    return stream, int(cl[0])


# ---- TX: val_internal_send_packet_ex frames -------------------------------------
def test_tx_frames_match_reference(vc, wire, fx):
    frames, lens, want = [], [], []
    for r in fx["tx"]:
        assert r["rc"] == 0, r
        payload = _prng.prng_bytes(r["seed"], r["payload_len"])
        prefix = bytes.fromhex(r["prefix"])
        content = r["payload_len"] + (8 if r["include_offset"] else 0)
        if content > 0xFFFF:
            # the reference wraps content_len to u16 (src/val_core.c:747); the
            # product framer refuses such a frame ...
            with pytest.raises(vc.ValError) as e:
                wire.build_data_batch(payload, [0], [payload.size], [r["offset"]], [r["include_offset"]])
            assert e.value.status == VAL_ERR_INVALID_ARG
            # ... and the CRC of the bytes the reference did put on the wire matches
            frame = np.frombuffer(prefix, dtype=np.uint8)
            assert r["wire_len"] == frame.size + 4
        else:
            stream, clen = _data_frame(wire, payload, r["offset"], r["include_offset"])
            assert stream.size == r["wire_len"] and clen == r["wire_len"] - 4
            assert bytes(stream[: len(prefix)]) == prefix, r
            frame = stream[:clen]
        got = vc.crc32_provider(0xFFFFFFFF, frame.tobytes())  # the crc32_func_t hook
        assert got == r["trailer"], (r["payload_len"], r["include_offset"], hex(got), hex(r["trailer"]))
        frames.append(frame)
        lens.append(frame.size)
        want.append(r["trailer"])
    # the same frames as one host batch (descriptor mode, ragged lengths)
    off = np.concatenate([[0], np.cumsum([f.size + 4 for f in frames])[:-1]]).astype(np.uint64)
    buf = np.zeros(int(off[-1]) + frames[-1].size + 4, dtype=np.uint8)
    for o, f in zip(off, frames):
        buf[int(o):int(o) + f.size] = f
    crc = vc.frames_host(buf, off=off, length=np.array(lens, dtype=np.uint32))
    assert crc.tolist() == want


# ---- RX: val_internal_recv_packet verdicts ------------------------------------------
def test_rx_verdicts_match_reference(vc, wire, fx):
    crc_errors = 0
    for r in fx["rx"]:
        payload = _prng.prng_bytes(r["seed"], r["payload_len"])
        stream, clen = _data_frame(wire, payload, r["offset"], True)
        stream[clen:clen + 4] = np.frombuffer(r["trailer"].to_bytes(4, "little"), dtype=np.uint8)
        if r["corrupt"]:
            stream[r["pos"]] ^= r["mask"]
        # the reference compares provider(frame) with the LE32 trailer (src/val_core.c:963-974)
        hook_ok = vc.crc32_provider(0xFFFFFFFF, stream[:clen].tobytes()) == _le32(stream[clen:])
        st, ok, nbad = vc.verify_frames_host(stream, off=np.array([0], np.uint64), length=np.array([clen], np.uint32))
        want_ok = r["rc"] == VAL_OK
        assert hook_ok == want_ok and bool(ok[0]) == want_ok, r
        assert st == (VAL_OK if want_ok else VAL_ERR_CRC) and nbad == (0 if want_ok else 1)
        crc_errors += nbad
        assert crc_errors == r["crc_errors"], r  # metrics.crc_errors++ per rejected frame


# ---- TX window batching and RX batch verify ----------------------
def _window(wire, w):
    file = _prng.prng_bytes(w["file_seed"], w["file_size"])
    fr = np.array(w["frames"], dtype=np.uint64)
    stream, fo, cl = wire.build_data_batch(file, fr[:, 0], fr[:, 1].astype(np.uint32), fr[:, 0],
                                           fr[:, 2].astype(np.uint8))
    return stream, fo, cl


@pytest.mark.parametrize("k", range(5))
def test_window_batching_matches_reference(vc, wire, fx, k):
    w = fx["windows"][k]
    stream, fo, cl = _window(wire, w)
    assert stream.size == w["wire_bytes"]
    # f1: one batched launch fills every trailer; the stream equals the reference TX stream
    crc = vc.frames_host(stream, off=fo, length=cl)
    assert crc.tolist() == w["trailers"]
    wire.put_trailers(stream, fo, cl, crc)
    assert vc.val_crc32(stream.tobytes()) == w["wire_crc"]
    # f2: corrupt the reference's frames, scan the byte stream, one batched verify
    for _, pos, mask in w["corrupt"]:
        stream[pos] ^= mask
    st, fo2, cl2, consumed = wire.scan_frames(stream, w["mtu"])
    assert st == VAL_OK and consumed == stream.size and fo2.tolist() == fo.tolist()
    vst, ok, nbad = vc.verify_frames_host(stream, off=fo2, length=cl2)
    want_ok = [rc == VAL_OK for rc in w["ref_rc"]]
    assert [bool(x) for x in ok] == want_ok
    assert nbad == w["ref_crc_errors"] == len(w["corrupt"])
    assert vst == (VAL_ERR_CRC if nbad else VAL_OK)


@pytest.mark.parametrize("k", range(5))
def test_window_verify_device_resident(vc, wire, fx, k):
    """The same corrupted windows verified from HBM (descriptor mode, ragged
    and len_hint paths), with header_crc checked against the oracle."""
    import torch

    w = fx["windows"][k]
    stream, fo, cl = _window(wire, w)
    crc = np.array(w["trailers"], dtype=np.uint32)
    wire.put_trailers(stream, fo, cl, crc)
    for _, pos, mask in w["corrupt"]:
        stream[pos] ^= mask
    dev = torch.device("cuda:0")
    d = torch.from_numpy(stream).to(dev)
    d_off = torch.from_numpy(fo.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(cl.astype(np.int32)).to(dev)
    want_ok = np.array([rc == VAL_OK for rc in w["ref_rc"]], dtype=np.uint8)
    _, want_hdr = _oracle.frames(stream, fo, cl, header=True)
    for hint in (0, int(cl.max())):
        hdr = torch.empty(len(cl), dtype=torch.int32, device=dev)
        ok, nbad = vc.verify_frames(d, off=d_off, length=d_len, out_hdr=hdr, len_hint=hint)
        torch.cuda.synchronize()
        assert np.array_equal(ok.cpu().numpy(), want_ok)
        assert int(nbad.item()) == w["ref_crc_errors"]
        assert np.array_equal(hdr.cpu().numpy().view(np.uint32), want_hdr)


# ---- BASELINE configs[0]: the 1 MiB / MTU 1024 loopback frame log (F6) -------------
def _rebuild(log, file):
    """Wire stream of one session's transport.send calls, from the F6 log."""
    parts, off, lens, trailers = [], [], [], []
    pos = 0
    for ptype, wire_len, trailer, foff, prefix in log:
        head = np.frombuffer(bytes.fromhex(prefix), dtype=np.uint8)
        body = head
        if ptype == 5:  # DATA: prefix is header (+ offset), payload is file[foff:]
            plen = wire_len - 4 - head.size
            body = np.concatenate([head, file[foff:foff + plen]])
        assert body.size == wire_len - 4
        parts.append(body)
        parts.append(np.frombuffer(int(trailer).to_bytes(4, "little"), dtype=np.uint8))
        off.append(pos)
        lens.append(body.size)
        trailers.append(trailer)
        pos += wire_len
    return np.concatenate(parts), np.array(off, np.uint64), np.array(lens, np.uint32), trailers


def test_loopback_1mib_frame_log(vc, fx):
    lb = fx["loopback"]
    file = _prng.prng_bytes(lb["file_seed"], lb["bytes"])
    assert lb["tx_crc_errors"] == 0 and lb["rx_crc_errors"] == 0
    # ts_file_crc32 of the transferred file (unit_tests/support/test_support.c:1458-1472)
    assert vc.val_crc32(file.tobytes()) == lb["file_crc"]
    nd = 0
    for side in ("tx", "rx"):
        log = lb[f"{side}_frames"]
        stream, off, lens, trailers = _rebuild(log, file)
        # every transport.send of the session, digested as the harness did
        assert vc.val_crc32(stream.tobytes()) == lb[f"{side}_digest"]
        # TX path: the crc32_func_t hook on every frame (what val_internal_crc32 calls)
        got = [vc.crc32_provider(0xFFFFFFFF, stream[int(o):int(o) + int(n)].tobytes()) for o, n in zip(off, lens)]
        assert got == trailers
        # batched: all frames of the session in one launch, and one verify
        assert vc.frames_host(stream, off=off, length=lens).tolist() == trailers
        st, ok, nbad = vc.verify_frames_host(stream, off=off, length=lens)
        assert st == VAL_OK and nbad == 0 and ok.all()
        nd += sum(1 for f in log if f[0] == 5)
    assert nd == 1045  # DATA frames of the transfer


# ---- the scalar hook under stress (pageable, reused, misaligned buffers) -------------
@pytest.mark.parametrize("seed,lo,hi,n", [(21, 1, 300000, 1500), (22, 2049, 70000, 1500), (23, 1, 64, 2000)])
def test_provider_stress_random_lengths(vc, seed, lo, hi, n):
    """Random lengths, alignments and data from ONE reused pageable buffer
    through val_gpu_crc32_provider, against the oracle. Pins the pinned
    staging and the context scratch arenas: pageable hipMemcpyAsync and
    per-call hipMallocAsync once gave ~7% wrong CRCs here."""
    import ctypes

    buf = np.zeros(hi + 64, dtype=np.uint8)
    base = buf.ctypes.data
    bad = []
    for i in range(n):
        r = (seed * 0x9E3779B97F4A7C15 + i * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF
        r ^= r >> 31
        ln = lo + r % (hi - lo + 1)
        al = (r >> 40) & 15
        buf[al:al + ln] = _prng.prng_bytes(r, ln)
        want = _oracle.crc32(buf[al:al + ln])
        got = int(vc.lib().val_gpu_crc32_provider(0xFFFFFFFF, ctypes.c_void_p(base + al), ln))
        if got != want:
            bad.append((i, ln, al, hex(got), hex(want)))
    assert not bad, bad[:10]
