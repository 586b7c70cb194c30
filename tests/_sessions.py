"""Helpers for tests/golden/session_vectors.json: real reference sessions
recorded by `oracle/_ref/provider_harness none sessions` (oracle/Makefile
`sessions`; the reference's own val_send_files / val_receive_files with its
built-in CRC). Each frame record is [type, wire_len, trailer, file_off,
prefix_hex, epoch]: DATA frames carry their 8- or 16-byte prefix and the file
offset of their payload, every other frame all of its bytes but the trailer;
epoch = the end's transport.recv calls before the send, so DATA frames of one
epoch are one window fill of the sender (src/val_sender.c:822-841).
Payload bytes are oracle/prng.h streams (tests/_prng.py). Test data only."""
from __future__ import annotations

import ctypes
import json
import os

import numpy as np

from tests import _prng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKT_RESUME_RESP, PKT_DATA, PKT_VERIFY = 4, 5, 7


def load() -> dict:
    with open(os.path.join(ROOT, "tests", "golden", "session_vectors.json")) as f:
        return {s["name"]: s for s in json.load(f)["sessions"]}


def input_file(s) -> np.ndarray:
    return _prng.prng_bytes(s["file_seed"], s["bytes"])


def receiver_existing(s) -> np.ndarray:
    """The receiver's output file before the session (a prefix of the input,
    one byte XOR 0x5A when flip >= 0)."""
    part = input_file(s)[: s["existing"]].copy()
    if s["flip"] >= 0:
        part[s["flip"]] ^= 0x5A
    return part


def frame_bytes(rec, file: np.ndarray) -> np.ndarray:
    """The CRC input of a logged frame (everything but its trailer)."""
    ptype, wire_len, _, foff, prefix = rec[:5]
    head = np.frombuffer(bytes.fromhex(prefix), dtype=np.uint8)
    if ptype != PKT_DATA:
        return head
    return np.concatenate([head, file[foff:foff + wire_len - 4 - head.size]])


def wire_stream(log, file: np.ndarray) -> np.ndarray:
    """Every transport.send of one end, back to back (frames + LE32 trailers)."""
    parts = []
    for rec in log:
        parts.append(frame_bytes(rec, file))
        parts.append(np.frombuffer(int(rec[2]).to_bytes(4, "little"), dtype=np.uint8))
    return np.concatenate(parts)


def windows(s):
    """The sender's DATA frames grouped by window fill: a list of
    (pay_off, pay_len, include_offset, trailers) arrays, one per window."""
    groups = {}
    for rec in s["tx_frames"]:
        if rec[0] != PKT_DATA:
            continue
        head = bytes.fromhex(rec[4])
        inc = head[1] & 1
        plen = rec[1] - 4 - (16 if inc else 8)
        groups.setdefault(rec[5], []).append((rec[3], plen, inc, rec[2]))
    out = []
    for ep in sorted(groups):
        g = np.array(groups[ep], dtype=np.uint64)
        out.append((g[:, 0], g[:, 1].astype(np.uint32), g[:, 2].astype(np.uint8), g[:, 3].astype(np.uint32)))
    return out


class ResumeResp(ctypes.Structure):  # val_resume_resp_t (include/val_protocol.h)
    _fields_ = [("action", ctypes.c_int), ("resume_offset", ctypes.c_uint64), ("verify_crc", ctypes.c_uint32),
                ("verify_length", ctypes.c_uint64)]


def control(s, lib):
    """The resume handshake as it crossed the wire, decoded with the product's
    own codecs (include/val_wire.h): the receiver's RESUME_RESP, the sender's
    VERIFY request and the receiver's VERIFY response."""
    def payload(log, ptype, size):
        recs = [r for r in log if r[0] == ptype and r[1] - 12 == size]
        assert len(recs) == 1, (ptype, size, len(recs))
        return (ctypes.c_uint8 * size).from_buffer_copy(bytes.fromhex(recs[0][4])[8:])

    # every argument is a pointer and passed as one; no argtypes are set on the
    # shared library object, so other tests' calls are unaffected
    rr = ResumeResp()
    lib.val_deserialize_resume_resp(payload(s["rx_frames"], PKT_RESUME_RESP, 24), ctypes.byref(rr))
    off, crc, ln = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
    lib.val_deserialize_verify_request(payload(s["tx_frames"], PKT_VERIFY, 16), ctypes.byref(off), ctypes.byref(crc),
                                       ctypes.byref(ln))
    res, rcrc = ctypes.c_int(), ctypes.c_uint32()
    lib.val_deserialize_verify_response(payload(s["rx_frames"], PKT_VERIFY, 8), ctypes.byref(res), ctypes.byref(rcrc))
    return {"action": rr.action, "resume_offset": rr.resume_offset, "resp_verify_crc": rr.verify_crc,
            "resp_verify_length": rr.verify_length, "req_offset": off.value, "req_crc": crc.value,
            "req_length": ln.value, "result": res.value, "receiver_crc": rcrc.value}
