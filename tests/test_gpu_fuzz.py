"""Randomised parity across every batch entry point (device and host memory,
strided / descriptor-uniform / binned ragged / zero-copy / chunked, TX and
verify, payload states, several logical GPUs, regions with random seeds),
each call checked bit-exact against the oracle. Seeded, so a
failure names a reproducible case; FUZZ_ROUNDS scales it and FUZZ_SEED
reseeds it."""
import os

import numpy as np
import pytest

from tests import _oracle, _prng

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROUNDS = int(os.environ.get("FUZZ_ROUNDS", "40"))


@pytest.fixture(scope="module")
def vc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import val_protocol_amd.crc as m

    m.init(0)
    yield m
    m.set_geometry()
    m.set_host_chunk_bytes(0)


def _batch(rng):
    kind = rng.choice(["tiny", "small", "mtu", "mixed"])
    n = int({"tiny": rng.integers(1, 40), "small": rng.integers(1, 600), "mtu": rng.integers(1, 3000),
             "mixed": rng.integers(1, 6000)}[kind])
    hi = {"tiny": 80, "small": 3000, "mtu": 65547, "mixed": 70000}[kind]
    if kind == "mtu":  # one length for the whole window except a short last frame
        L = int(rng.integers(8, hi))
        lens = np.full(n, L, np.uint32)
        lens[-1] = int(rng.integers(0, L + 1))
    else:
        lens = rng.integers(0, hi + 1, n).astype(np.uint32)
    gaps = rng.integers(0, 9, n) if rng.random() < 0.7 else np.zeros(n, np.int64)
    offs = np.zeros(n, np.uint64)
    pos = int(rng.integers(0, 64))
    for i in range(n):
        pos += int(gaps[i])
        offs[i] = pos
        pos += int(lens[i]) + 4
    base = _prng.prng_bytes(int(rng.integers(1 << 30)), pos + 8)
    return base, offs, lens


def test_fuzz_batches(vc, monkeypatch):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(int(os.environ.get("FUZZ_SEED", "20261016")))
    for r in range(ROUNDS):
        base, offs, lens = _batch(rng)
        n = offs.size
        want, want_h = _oracle.frames(base, offs, lens, header=True)
        case = f"round {r} n={n} lens {int(lens.min())}..{int(lens.max())}"
        if r % 50 == 0:
            print(case, flush=True)
        vc.set_geometry(int(rng.choice([0, 0, 0, 1, 2, 4, 8, 16, 32, 64])), int(rng.choice([-1, -1, 0, 1, 2])))
        vc.set_host_chunk_bytes(int(rng.choice([0, 0, 1 << 16, 1 << 20])))
        if rng.random() < 0.5:
            vc.set_ragged_min_frames(1)
        else:
            vc.set_ragged_min_frames(-1)
        # device memory
        d = torch.from_numpy(base).to(dev)
        do = torch.from_numpy(offs.view(np.int64)).to(dev)
        dl = torch.from_numpy(lens.view(np.int32)).to(dev)
        hint = int(lens.max()) if (rng.random() < 0.3 and lens.min() == lens.max()) else 0
        hdr = torch.empty(n, dtype=torch.int32, device=dev)
        crc = vc.frames(d, off=do, length=dl, out_hdr=hdr, len_hint=hint)
        torch.cuda.synchronize()
        assert np.array_equal(crc.cpu().numpy().view(np.uint32), want), case
        assert np.array_equal(hdr.cpu().numpy().view(np.uint32), want_h), case
        # host memory (zero-copy or chunked pipeline by size), pageable or pinned
        hb = base
        if rng.random() < 0.5:
            pb = vc.PinnedBuffer(base.size)
            pb.array[:] = base
            hb = pb.array
        got, got_h = vc.frames_host(hb, offs, lens, header=True)
        assert np.array_equal(got, want) and np.array_equal(got_h, want_h), case + " host"
        # verify: trailers written, up to 3 frames corrupted
        tr = base.copy()
        for o, l, c in zip(offs, lens, want):
            tr[int(o) + int(l):int(o) + int(l) + 4] = np.frombuffer(int(c).to_bytes(4, "little"), np.uint8)
        bad = rng.choice(n, size=min(n, int(rng.integers(0, 4))), replace=False)
        for i in bad:
            span = int(lens[i]) + 4
            tr[int(offs[i]) + int(rng.integers(0, span))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        st, ok, nbad = vc.verify_frames_host(tr, offs, lens)
        want_ok, want_bad = _oracle.verify_frames(tr, offs, lens)
        assert nbad == want_bad == len(bad) and np.array_equal(ok, want_ok), case + " verify"
        ok_d, nbad_d = vc.verify_frames(torch.from_numpy(tr).to(dev), off=do, length=dl, len_hint=hint)
        torch.cuda.synchronize()
        assert int(nbad_d.item()) == want_bad and np.array_equal(ok_d.cpu().numpy(), want_ok), case + " verify dev"
        # payload states (f4): raw zero-init register of each frame's payload
        # (after the 8-B header and, when flags bit 0 is set, the 8-B offset)
        ok_x, nbad_x, pay = vc.verify_frames_ex(torch.from_numpy(tr).to(dev), off=do, length=dl, len_hint=hint)
        st_h, ok_h, nbad_h, pay_h = vc.verify_frames_ex_host(tr, offs, lens)
        torch.cuda.synchronize()
        want_pay = np.zeros(n, np.uint32)
        for i, (o, L) in enumerate(zip(offs, lens)):
            o, L = int(o), int(L)
            pre = 16 if (L >= 8 and tr[o + 1] & 1) else 8
            want_pay[i] = _oracle.update_state(0, tr[o + pre:o + L]) if L >= pre else 0
        assert np.array_equal(pay.cpu().numpy().view(np.uint32), want_pay), case + " pay dev"
        assert np.array_equal(pay_h, want_pay) and nbad_h == want_bad, case + " pay host"
        assert int(nbad_x.item()) == want_bad and np.array_equal(ok_x.cpu().numpy(), want_ok), case + " verify ex"
        # several logical GPUs from one process
        ndev = int(rng.integers(2, 5))
        assert np.array_equal(vc.frames_host_multi(base, offs, lens, ndev=ndev), want), case + f" multi {ndev}"
        # region over a random slice, device and host, random seed
        a = int(rng.integers(0, base.size))
        b = int(rng.integers(a, base.size + 1))
        seg = base[a:b]
        want_r = _oracle.crc32(seg)
        assert (int(vc.region(d[a:b]).item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == want_r, case + f" region {a}:{b}"
        assert vc.val_crc32(seg) == want_r, case + f" host region {a}:{b}"
        s0 = int(rng.integers(0, 1 << 32))
        assert (int(vc.region(d[a:b], s0).item()) & 0xFFFFFFFF) == _oracle.update_state(s0, seg), case + " region seed"
        assert vc.region_host_multi(seg, s0, ndev=ndev) == _oracle.update_state(s0, seg), case + " region multi"
