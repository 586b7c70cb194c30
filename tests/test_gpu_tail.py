"""In-launch tail pieces of the uniform frames kernel (crc_kernels.hpp
tail_pieces, val_crc32_hip.hip launch_uniform): a uniform batch whose frame
groups do not fill the last round of the persistent grid hashes the frames
past the last full round in 1-4 KiB pieces inside the same launch, each
piece's register advanced over the bytes after it and folded into its frame
by device atomics. Bit-exact against the oracle (reference src/val_core.c:
150-160, framing :718-834, RX compare :963-974) with the path on and off,
for strided and descriptor batches, one or several full rounds (with the
dynamic tail), frames of 8-64 KiB at 8 and 16 lanes, a short and an empty
frame among the tail frames, unaligned offsets, header_crc, verify with
corrupted tail frames, and the same batch twice (the accumulators must be
re-zeroed by the launch that used them)."""
import numpy as np
import pytest
import torch

from tests import _oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def vc():
    import val_protocol_amd.crc as vc

    vc.init(0)
    yield vc
    vc.lib().val_gpu_set_tail_pieces(-1)
    vc.set_geometry()


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _waves():
    return torch.cuda.get_device_properties(0).multi_processor_count * 16


def _run_both(vc, fn):
    """fn() with the in-launch tail on, then off; returns both results and
    whether the on-run used the path."""
    lib = vc.lib()
    lib.val_gpu_set_tail_pieces(1)
    before = lib.val_gpu_tail_piece_launches()
    on = fn()
    torch.cuda.synchronize()
    used = lib.val_gpu_tail_piece_launches() - before
    lib.val_gpu_set_tail_pieces(0)
    off = fn()
    torch.cuda.synchronize()
    lib.val_gpu_set_tail_pieces(-1)
    return on, off, used


@pytest.mark.parametrize("flen,rounds,tail", [
    (65532, 1, 6),      # a 1 GiB eighth of the cfg4 file: one round and 6 frames
    (65532, 1, 1024),   # the most tail frames at 16 lanes: 4 KiB pieces (1-2 KiB ones need more groups than waves)
    (65532, 2, 41),
    (16400, 1, 100),    # 8 lanes, 17 pieces of 1 KiB per frame (the front one 16 B)
    (8192, 1, 3),       # the shortest frames that take the path: 8 pieces
    (24580, 4, 777),    # with the dynamic tail (four rounds)
])
def test_strided_tail_every_frame(vc, flen, rounds, tail):
    G = vc.lanes_per_frame(flen)
    assert G in (8, 16)
    n = _waves() * (64 // G) * rounds + tail
    stride = flen + 4
    g = torch.Generator(device=DEV).manual_seed(flen + tail)
    buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=DEV, generator=g)
    hdr_on = torch.empty(n, dtype=torch.int32, device=DEV)
    hdr_off = torch.empty(n, dtype=torch.int32, device=DEV)
    outs = []

    def fn():
        h = hdr_on if not outs else hdr_off
        outs.append(0)
        return vc.frames(buf, stride=stride, flen=flen, n=n, out_hdr=h).clone()

    on, off, used = _run_both(vc, fn)
    assert used == 1
    host = buf.cpu().numpy()
    want, want_h = _oracle.frames_strided(host, stride, flen, n, header=True, nthreads=16)
    assert np.array_equal(_u32(on), want)
    assert np.array_equal(_u32(off), want)
    assert np.array_equal(_u32(hdr_on), want_h) and np.array_equal(_u32(hdr_off), want_h)
    # again, path on: the accumulators were re-zeroed by the first launch
    vc.lib().val_gpu_set_tail_pieces(1)
    again = vc.frames(buf, stride=stride, flen=flen, n=n)
    torch.cuda.synchronize()
    vc.lib().val_gpu_set_tail_pieces(-1)
    assert np.array_equal(_u32(again), want)


@pytest.mark.parametrize("hint,rounds,tail", [(65532, 1, 6), (65532, 8, 41), (16400, 1, 33)])
def test_descriptor_tail_short_and_empty_frames(vc, hint, rounds, tail):
    """Descriptor batches with the uniform length hint, as bench.py's cfg4
    slices: the file's last frame (816 B) and an empty frame among the tail
    frames, frame starts unaligned (odd gaps), one frame longer than the hint
    (its front piece absorbs the excess)."""
    G = vc.lanes_per_frame(hint)
    n = _waves() * (64 // G) * rounds + tail
    rng = np.random.default_rng(hint + tail)
    lens = np.full(n, hint, np.uint32)
    lens[-1] = 816
    lens[-3] = 0
    lens[-2] = hint + 5000
    lens[n - tail] = 7
    gaps = rng.integers(4, 7, n)
    wire = lens.astype(np.int64) + gaps
    offs = np.concatenate([[3], 3 + np.cumsum(wire)[:-1]]).astype(np.uint64)
    total = int(offs[-1]) + int(wire[-1]) + 8
    g = torch.Generator(device=DEV).manual_seed(hint ^ tail)
    buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device=DEV, generator=g)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    hdr = torch.empty(n, dtype=torch.int32, device=DEV)

    def fn():
        return vc.frames(buf, off=d_off, length=d_len, len_hint=hint, out_hdr=hdr).clone(), hdr.clone()

    (on, hon), (off, hoff), used = _run_both(vc, fn)
    assert used == 1
    host = buf.cpu().numpy()
    want, want_h = _oracle.frames(host, offs, lens, header=True, nthreads=16)
    assert np.array_equal(_u32(on), want) and np.array_equal(_u32(off), want)
    assert np.array_equal(_u32(hon), want_h) and np.array_equal(_u32(hoff), want_h)


def test_verify_tail_with_corruption(vc):
    """RX verify through the in-launch tail: trailers written from the oracle,
    frames corrupted in the main rounds and among the tail frames (payload
    bytes and trailer bytes): verdicts and the mismatch count."""
    flen, tail = 32784, 57
    G = vc.lanes_per_frame(flen)
    n = _waves() * (64 // G) + tail
    stride = flen + 4
    g = torch.Generator(device=DEV).manual_seed(5)
    buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=DEV, generator=g)
    host = buf.cpu().numpy()
    want = _oracle.frames_strided(host, stride, flen, n, nthreads=16)
    rows = host.reshape(n, stride)
    rows[:, flen:] = want.astype("<u4").view(np.uint8).reshape(n, 4)
    rng = np.random.default_rng(9)
    bad = np.concatenate([rng.choice(n - tail, 20, replace=False), n - tail + rng.choice(tail, 11, replace=False)])
    for k, i in enumerate(bad):
        rows[i, flen + (k % 4) if k % 2 else int(rng.integers(0, flen))] ^= np.uint8(1 << (k % 8))
    d = torch.from_numpy(rows.reshape(-1).copy()).to(DEV)

    def fn():
        ok, nbad = vc.verify_frames(d, stride=stride, flen=flen, n=n)
        return ok.cpu().numpy(), int(nbad.item())

    (ok_on, nb_on), (ok_off, nb_off), used = _run_both(vc, fn)
    assert used == 1
    want_ok = np.ones(n, np.uint8)
    want_ok[bad] = 0
    assert nb_on == nb_off == bad.size
    assert np.array_equal(ok_on, want_ok) and np.array_equal(ok_off, want_ok)


def test_forced_lanes_and_the_path_off_for_others(vc):
    """Forced 8 or 16 lanes take the path; 32 lanes and payload states do
    not (their kernels do not carry it) and still hash every frame right."""
    flen, tail = 65532, 9
    stride = flen + 4
    for G, expect in ((8, 1), (16, 1), (32, 0)):
        n = _waves() * (64 // G) + tail
        g = torch.Generator(device=DEV).manual_seed(G)
        buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=DEV, generator=g)
        vc.set_geometry(G)
        try:
            on, off, used = _run_both(vc, lambda: vc.frames(buf, stride=stride, flen=flen, n=n).clone())
        finally:
            vc.set_geometry()
        assert used == expect, G
        want = _oracle.frames_strided(buf.cpu().numpy(), stride, flen, n, nthreads=16)
        assert np.array_equal(_u32(on), want) and np.array_equal(_u32(off), want), G


def test_tail_fuzz(vc):
    """Random uniform batches around the path's edges, each bit-exact against
    the oracle with the path on and off: frame length 8-64 KiB, 1-3 full
    rounds, 1 .. one round minus one tail frames, strided or descriptor
    (unaligned start, one short and one empty frame among the tail frames),
    header_crc, then verify with one corrupted tail frame. TAIL_FUZZ_CASES and
    TAIL_FUZZ_SEED scale and reseed it."""
    import os

    cases = int(os.environ.get("TAIL_FUZZ_CASES", "4"))
    rng = np.random.default_rng(int(os.environ.get("TAIL_FUZZ_SEED", "20261018")))
    used_total = 0
    for c in range(cases):
        flen = int(rng.integers(8192, 65537))
        G = vc.lanes_per_frame(flen)
        assert G in (8, 16), flen
        per_round = _waves() * (64 // G)
        rounds = int(rng.integers(1, 4)) if flen <= 32768 else int(rng.integers(1, 3))
        tail = int(rng.integers(1, per_round))
        n = per_round * rounds + tail
        case = f"case {c}: flen {flen} G {G} rounds {rounds} tail {tail}"
        stride = flen + 4
        g = torch.Generator(device=DEV).manual_seed(int(rng.integers(1 << 62)))
        strided = bool(rng.random() < 0.5)
        case += " strided" if strided else " descriptor"
        if strided:
            buf = torch.randint(0, 256, (n * stride,), dtype=torch.uint8, device=DEV, generator=g)
            hdr = torch.empty(n, dtype=torch.int32, device=DEV)

            def fn():
                return vc.frames(buf, stride=stride, flen=flen, n=n, out_hdr=hdr).clone(), hdr.clone()

            host = buf.cpu().numpy()
            want, want_h = _oracle.frames_strided(host, stride, flen, n, header=True, nthreads=16)
            offs = np.arange(n, dtype=np.uint64) * stride
            lens = np.full(n, flen, np.uint32)
        else:
            lens = np.full(n, flen, np.uint32)
            lens[n - 1 - int(rng.integers(0, tail))] = int(rng.integers(1, flen))
            lens[n - 1 - int(rng.integers(0, tail))] = 0
            wire = lens.astype(np.int64) + 4 + rng.integers(0, 3, n)
            first = int(rng.integers(0, 16))
            offs = np.concatenate([[first], first + np.cumsum(wire)[:-1]]).astype(np.uint64)
            buf = torch.randint(0, 256, (int(offs[-1]) + int(wire[-1]) + 8,), dtype=torch.uint8, device=DEV,
                                generator=g)
            d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
            d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
            hdr = torch.empty(n, dtype=torch.int32, device=DEV)

            def fn():
                return vc.frames(buf, off=d_off, length=d_len, len_hint=flen, out_hdr=hdr).clone(), hdr.clone()

            host = buf.cpu().numpy()
            want, want_h = _oracle.frames(host, offs, lens, header=True, nthreads=16)
        (on, hon), (off_, hoff), used = _run_both(vc, fn)
        used_total += used
        assert np.array_equal(_u32(on), want) and np.array_equal(_u32(off_), want), case
        assert np.array_equal(_u32(hon), want_h) and np.array_equal(_u32(hoff), want_h), case
        # verify: trailers from the oracle, one tail frame with a flipped bit
        for o, L, w in zip(offs[n - tail:], lens[n - tail:], want[n - tail:]):
            host[int(o) + int(L):int(o) + int(L) + 4] = np.frombuffer(int(w).to_bytes(4, "little"), np.uint8)
        # the main rounds' trailers too, vectorised for the strided layout
        if strided:
            rows = host[:(n - tail) * stride].reshape(n - tail, stride)
            rows[:, flen:] = want[:n - tail].astype("<u4").view(np.uint8).reshape(n - tail, 4)
        else:
            for o, L, w in zip(offs[:n - tail], lens[:n - tail], want[:n - tail]):
                host[int(o) + int(L):int(o) + int(L) + 4] = np.frombuffer(int(w).to_bytes(4, "little"), np.uint8)
        bad = n - tail + int(rng.integers(0, tail))
        host[int(offs[bad]) + int(rng.integers(0, int(lens[bad]) + 4))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        d = torch.from_numpy(host).to(DEV)
        d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
        d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)

        def vfn():
            ok, nbad = vc.verify_frames(d, off=d_off, length=d_len, len_hint=flen)
            return ok.cpu().numpy(), int(nbad.item())

        (ok_on, nb_on), (ok_off, nb_off), vused = _run_both(vc, vfn)
        used_total += vused
        want_ok = np.ones(n, np.uint8)
        want_ok[bad] = 0
        assert nb_on == nb_off == 1, case + " verify"
        assert np.array_equal(ok_on, want_ok) and np.array_equal(ok_off, want_ok), case + " verify"
        print(f"{case}: tail-piece launches {used}+{vused}", flush=True)
        del buf, d, host
        torch.cuda.empty_cache()
    assert used_total >= 1 or cases < 3  # about half the cases take the path (tails under ~half a round)
