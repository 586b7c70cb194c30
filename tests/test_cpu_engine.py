"""The scalar hooks' CPU side ("val_gpu_crc32_provider
(CPU below a size threshold)"), pinned on the CPU, no GPU needed.

* Each engine of the library's own CPU CRC (cpu_crc32.c: slice-by-16,
  PCLMULQDQ folding, VPCLMULQDQ folding) reproduces the reference-generated
  goldens (tests/golden/ref_vectors.json: KAT, 256 single bytes, lengths
  0..4096 and the special lengths, seeded states) and the oracle on random
  lengths and alignments.
* Below the provider threshold the three hooks answer on the CPU
  (last_hook_path HOOK_CPU, counted by cpu_small_count, never by the failure
  fallback count) with the reference's results; the threshold's knob and
  environment variable behave as documented.
* The receiver's ordered payload fold (val_crc32_fold_payload_states_at)
  follows src/val_receiver.c:871-891: duplicates, gaps, rejected and control
  frames are not folded.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import val_protocol_amd.crc as vc
from tests import _oracle, _prng

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINES = (1, 2, 3)  # slice-by-16, PCLMULQDQ, VPCLMULQDQ (a missing one runs the next simpler)


@pytest.mark.parametrize("engine", ENGINES)
def test_engine_goldens(golden, engine):
    assert vc.cpu_update_state(0xFFFFFFFF, b"123456789", engine) ^ 0xFFFFFFFF == golden["kat_123456789"]
    assert vc.cpu_update_state(0xFFFFFFFF, b"", engine) ^ 0xFFFFFFFF == golden["kat_empty"]
    assert [vc.cpu_update_state(0xFFFFFFFF, bytes([b]), engine) ^ 0xFFFFFFFF for b in range(256)] == \
        golden["single_bytes"]
    data = _prng.prng_bytes(golden["sweep_seed"], 70000)
    got = [vc.cpu_update_state(0xFFFFFFFF, data[:L], engine) ^ 0xFFFFFFFF for L in range(4097)]
    assert got == golden["sweep_0_4096"]
    for L, want in golden["sweep_special"].items():
        assert vc.cpu_update_state(0xFFFFFFFF, data[: int(L)], engine) ^ 0xFFFFFFFF == want
    for v in golden["state_vectors"]:
        assert vc.cpu_update_state(v["seed"], data[: v["len"]], engine) == v["state"]


@pytest.mark.parametrize("engine", ENGINES)
def test_engine_random_lengths_and_alignments(engine):
    rng = np.random.default_rng(engine)
    buf = _prng.prng_bytes(0xC0DE, 3 << 20)
    lens = list(rng.integers(0, 70000, 300)) + [63, 64, 65, 127, 128, 255, 256, 257, 511, 512, 1 << 20, (3 << 20) - 7]
    for L in lens:
        a = int(rng.integers(0, 7))
        L = int(min(L, buf.size - a))
        seed = int(rng.integers(0, 1 << 32))
        assert vc.cpu_update_state(seed, buf[a:a + L], engine) == _oracle.update_state(seed, buf[a:a + L]), (L, a)


def test_engines_agree_on_this_host():
    assert vc.cpu_engine() in (1, 2, 3)
    data = _prng.prng_bytes(5, 100_003)
    ref = vc.cpu_update_state(0x1234, data, 1)
    assert all(vc.cpu_update_state(0x1234, data, e) == ref for e in (0, 2, 3))


def test_hooks_below_threshold_answer_on_cpu(golden):
    lib = vc.lib()
    data = _prng.prng_bytes(golden["sweep_seed"], 70000)
    p = ctypes.c_void_p(data.ctypes.data)
    vc.set_provider_min_bytes(1 << 40)
    try:
        small0, fb0 = vc.cpu_small_count(), vc.cpu_fallback_count()
        for L in list(range(0, 300)) + [1020, 1040, 16400, 65524, 65535, 65543]:
            want = golden["sweep_0_4096"][L] if L <= 4096 else golden["sweep_special"][str(L)]
            assert lib.val_gpu_crc32_provider(0xFFFFFFFF, p, L) == want
            assert vc.last_hook_path() == vc.HOOK_CPU
            assert lib.val_crc32(p, L) == want
            assert lib.val_crc32_update_state(0xFFFFFFFF, p, L) ^ 0xFFFFFFFF == want
        # the Python API accepts a below-threshold answer (it is not a failure)
        assert vc.crc32_provider(0xFFFFFFFF, b"123456789") == 0xCBF43926
        assert vc.val_crc32(data[:1040]) == golden["sweep_special"]["1040"]
        assert vc.cpu_small_count() - small0 == 306 * 3 + 2
        assert vc.cpu_fallback_count() == fb0
    finally:
        vc.set_provider_min_bytes(-1)


def test_threshold_knob_and_environment():
    code = r"""
import sys; sys.path.insert(0, {root!r})
import val_protocol_amd.crc as vc
print(vc.provider_min_bytes())
vc.set_provider_min_bytes(123); print(vc.provider_min_bytes())
vc.set_provider_min_bytes(-1); print(vc.provider_min_bytes())
""".format(root=ROOT)
    env = {k: v for k, v in os.environ.items() if k != "VAL_GPU_PROVIDER_MIN_BYTES"}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         timeout=300).stdout.split()
    default = int(out[0])
    assert default > 0 and out[1:] == ["123", str(default)]
    env["VAL_GPU_PROVIDER_MIN_BYTES"] = "4096"
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, check=True,
                         timeout=300).stdout.split()
    assert out == ["4096", "123", "4096"]


# ---- receiver ordering of the payload fold -------------------------------------
def _window(payloads, offsets, explicit, types=None):
    """A byte stream of frames: DATA frames carry payloads[i] at file offset
    offsets[i] (explicit or implied); types[i] != 5 makes a control frame."""
    parts, fo, cl = [], [], []
    pos = 0
    for i, pl in enumerate(payloads):
        t = 5 if types is None else types[i]
        content = (int(offsets[i]).to_bytes(8, "little") if explicit[i] and t == 5 else b"") + bytes(pl)
        hdr = bytes([t, 1 if (explicit[i] and t == 5) else 0]) + len(content).to_bytes(2, "little") + b"\0" * 4
        fr = hdr + content
        fr += _oracle.crc32(fr).to_bytes(4, "little")
        parts.append(fr)
        fo.append(pos)
        cl.append(8 + len(content))
        pos += len(fr)
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy(), np.array(fo, np.uint64), np.array(cl, np.uint32)


def _pay_states(stream, fo, cl):
    from val_protocol_amd import wire

    pl = wire.payload_lens(stream, fo, cl)
    ps = np.array([_oracle.update_state(0, stream[int(o) + int(c) - int(p):int(o) + int(c)])
                   for o, c, p in zip(fo, cl, pl)], dtype=np.uint32)
    return ps, pl


def test_fold_at_follows_the_receiver():
    from val_protocol_amd import wire

    rng = np.random.default_rng(9)
    file = _prng.prng_bytes(77, 6000)
    # in order 0..1000, a duplicate of the first frame, in order, a gap, an
    # implied-offset frame (in order), a control frame, a rejected frame, in order
    cuts = [(0, 1000), (0, 1000), (1000, 2500), (4000, 4500), (2500, 3000), (None, None), (3000, 3500), (3500, 4000)]
    payloads, offs, expl, types = [], [], [], []
    for a, b in cuts:
        if a is None:
            payloads.append(bytes(rng.integers(0, 256, 20, dtype=np.uint8)))
            offs.append(0)
            expl.append(False)
            types.append(6)  # DATA_ACK
        else:
            payloads.append(file[a:b].tobytes())
            offs.append(a)
            expl.append(a != 2500)
            types.append(5)
    stream, fo, cl = _window(payloads, offs, expl, types)
    ps, pl = _pay_states(stream, fo, cl)
    file_off = wire.data_offsets(stream, fo, cl)
    assert int(file_off[4]) == wire.OFFSET_IMPLIED and int(file_off[5]) == wire.OFFSET_NOT_DATA
    ok = np.ones(len(cuts), np.uint8)
    ok[6] = 0  # frame 6 (3000..3500) failed its trailer check: the next one becomes a gap
    state, written, nf = vc.fold_payload_states_at(0xFFFFFFFF, ps, pl, file_off, 0, ok)
    assert (written, nf) == (3000, 3)
    assert state == _oracle.update_state(0xFFFFFFFF, file[:3000])
    # the retransmitted frame arrives: the rest folds on
    state2, written2, nf2 = vc.fold_payload_states_at(state, ps[6:], pl[6:], file_off[6:], written)
    assert (written2, nf2) == (4000, 2)
    assert state2 == _oracle.update_state(0xFFFFFFFF, file[:4000])


def test_fold_at_on_the_loopback_log():
    """The F6 loopback frames (reference RX order, every DATA frame once): the
    ordered fold equals the reference's file CRC."""
    import json

    from val_protocol_amd import wire

    lb = json.load(open(os.path.join(ROOT, "tests", "golden", "dropin_vectors.json")))["loopback"]
    file = _prng.prng_bytes(lb["file_seed"], lb["bytes"])
    payloads, offs, expl = [], [], []
    for t, wl, _tr, off, *_ in lb["tx_frames"]:
        if t == 5:
            pl = wl - 12 - 8
            payloads.append(file[off:off + pl].tobytes())
            offs.append(off)
            expl.append(True)
    stream, fo, cl = _window(payloads, offs, expl)
    ps, pl = _pay_states(stream, fo, cl)
    state, written, nf = vc.fold_payload_states_at(0xFFFFFFFF, ps, pl, wire.data_offsets(stream, fo, cl), 0)
    assert written == lb["bytes"] and nf == len(payloads)
    assert state ^ 0xFFFFFFFF == lb["file_crc"]
