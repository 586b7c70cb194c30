"""Pins the CPU oracle against golden vectors produced by the reference
library itself (oracle/gen_golden.c linked against /root/reference/src)."""
import os

import numpy as np
import pytest

from tests import _oracle, _prng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_kat(golden):
    assert golden["kat_123456789"] == 0xCBF43926
    assert _oracle.crc32(b"123456789") == golden["kat_123456789"]
    assert _oracle.crc32(b"") == golden["kat_empty"] == 0


def test_single_bytes(golden):
    got = [_oracle.crc32(bytes([b])) for b in range(256)]
    assert got == golden["single_bytes"]


def test_length_sweep(golden):
    data = _prng.prng_bytes(golden["sweep_seed"], 70000)
    got = [_oracle.crc32(data[:L]) for L in range(4097)]
    assert got == golden["sweep_0_4096"]
    for L, want in golden["sweep_special"].items():
        assert _oracle.crc32(data[: int(L)]) == want


def test_state_semantics(golden):
    data = _prng.prng_bytes(golden["sweep_seed"], 70000)
    for v in golden["state_vectors"]:
        st = _oracle.update_state(v["seed"], data[: v["len"]])
        assert st == v["state"]
        assert _oracle.provider(v["seed"], data[: v["len"]]) == v["final"]


def test_region_chunking(golden):
    data = _prng.prng_bytes(golden["region_seed"], 8 << 20)
    for r in golden["regions"]:
        L, c = r["len"], r["chunk"]
        st = 0xFFFFFFFF
        for o in range(0, L, c):
            st = _oracle.update_state(st, data[o:min(L, o + c)])
        assert st ^ 0xFFFFFFFF == r["crc"] == r["oneshot"]
        assert _oracle.crc32(data[:L]) == r["oneshot"]


def test_combine(golden):
    for la, lb, ca, cb, cab in golden["combine"]:
        assert _oracle.combine(ca, cb, lb) == cab


def test_frames(golden):
    for fr in golden["frames"]:
        pl = fr["payload_len"]
        payload = _prng.prng_bytes(golden["frames_payload_seed_base"] ^ (pl << 8), pl)
        w = _oracle.build_data_frame(payload, fr["offset"], bool(fr["include_offset"]))
        assert len(w) == fr["wire_len"], fr
        assert w[:8].hex() == fr["header"]
        assert w[-4:].hex() == fr["trailer"]
        assert _oracle.crc32(w[:-4]) == fr["crc_input_crc"]
        if "wire" in fr:
            assert w.hex() == fr["wire"]


def test_truncation_cases_recorded(golden):
    # The reference wraps content_len to 16 bits (src/val_core.c:747): a
    # 65,528-byte payload with explicit offset leaves a 12-byte frame.
    wl = {(f["payload_len"], f["include_offset"]): f["wire_len"] for f in golden["frames"]}
    assert wl[(65528, 1)] == 12 and wl[(65536, 0)] == 12 and wl[(65536, 1)] == 20
    assert wl[(65527, 1)] == 65547


_REF = os.path.join(ROOT, "oracle", "_ref", "libval_ref.so")


@pytest.mark.skipif(not os.path.exists(_REF), reason="reference build only exists in the build container")
def test_oracle_matches_reference_library():
    import ctypes

    ref = ctypes.CDLL(_REF)
    ref.val_crc32.restype = ctypes.c_uint32
    ref.val_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    rng = np.random.default_rng(7)
    for L in list(range(0, 80)) + [1020, 1040, 16400, 65532, 200001]:
        d = rng.integers(0, 256, L, dtype=np.uint8)
        assert ref.val_crc32(d.ctypes.data, L) == _oracle.crc32(d)
