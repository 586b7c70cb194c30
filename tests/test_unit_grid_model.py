"""CPU model of the frame decomposition `hash_frame` runs on the GPU
(val_protocol_amd/csrc/crc_kernels.hpp), checked against the oracle.

The kernel anchors its unit grid at floor4(frame end): the first Lg = L - tb
bytes (tb = (address of the frame end) mod 4) are cut into U = ceil(Lg/64)
units counted from that point, so every unit is dword-aligned whatever the
frame's byte alignment; unit 0 is front-padded with pad = 64U - Lg virtual
zero bytes (free: the register is still 0 there). It XORs the seed into frame
bytes 0..3, hashes lane g's units u0+g+G*k (u0 = U - G*R) with a gap shift of
64(G-1) bytes between rounds, merges the lanes with shifts of 64*2^j bytes,
then feeds the tb bytes past the grid with byte steps. Frames with Lg < 4 take
the byte path. This
restates that algebra byte-wise in Python (raw register updates via zlib), so
the decomposition is proven on CPU for every length, alignment and lane
count; the GPU tests prove the kernel.
"""
import zlib

import numpy as np
import pytest

from tests import _oracle

M = 0xFFFFFFFF
POLY = 0xEDB88320
ONE = 0x80000000  # x^0, reflected


def gf2_mul(a: int, b: int) -> int:
    prod = 0
    for i in range(31, -1, -1):
        if (a >> i) & 1:
            prod ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return prod


def gf2_pow(x: int, n: int) -> int:
    r = ONE
    while n:
        if n & 1:
            r = gf2_mul(r, x)
        x = gf2_mul(x, x)
        n >>= 1
    return r


X8 = 0x00800000  # x^8


def raw_update(reg: int, data: bytes) -> int:
    """Raw (no pre/post inversion) register update, via zlib's finished CRC."""
    return (~zlib.crc32(data, (~reg) & M)) & M


def model_frame(mem: bytes, fp: int, L: int, G: int, seed: int = M, xorout: int = M) -> int:
    tb = min((fp + L) % 4, L)  # mem index = device address mod 4 (allocations are 4-aligned)
    Lg = L - tb
    if Lg < 4:  # byte path
        return raw_update(seed, mem[fp:fp + L]) ^ xorout
    U = -(-Lg // 64)
    R = -(-U // G)
    pad = 64 * U - Lg
    frame = bytearray(mem[fp:fp + Lg])
    for j in range(4):  # seed XORed into frame bytes 0..3
        frame[j] ^= (seed >> (8 * j)) & 0xFF
    grid = bytes(pad) + bytes(frame)  # unit 0 front-padded with zeros
    assert len(grid) == 64 * U
    gap = gf2_pow(X8, 64 * (G - 1))
    lanes = []
    for g in range(G):
        acc = 0
        for k in range(R):
            u = U - G * R + g + G * k
            if k > 0:
                acc = gf2_mul(acc, gap)
            if u >= 0:
                acc = raw_update(acc, grid[64 * u:64 * u + 64])
        lanes.append(acc)
    # merge tree: level j joins blocks of 2^j lanes, left advanced by 64*2^j bytes
    width = 1
    while width < G:
        sh = gf2_pow(X8, 64 * width)
        lanes = [gf2_mul(lanes[i], sh) ^ lanes[i + 1] for i in range(0, len(lanes), 2)]
        width *= 2
    return raw_update(lanes[0], mem[fp + Lg:fp + L]) ^ xorout


@pytest.mark.parametrize("G", [1, 2, 4, 16])
def test_grid_model_matches_oracle(G):
    rng = np.random.default_rng(G)
    mem = rng.integers(0, 256, 4096, dtype=np.uint8).tobytes()
    for L in list(range(0, 70)) + [127, 128, 129, 191, 300, 1000, 1100]:
        for fp in (128, 129, 130, 131, 187, 188, 189, 190, 191, 128 + 61):
            want = _oracle.frames(np.frombuffer(mem[fp:fp + L], np.uint8), np.array([0], np.uint64),
                                  np.array([L], np.uint32))[0]
            assert model_frame(mem, fp, L, G) == int(want), (L, fp, G)


def test_grid_model_seeded_raw_state():
    """Region chunks: seed = state_in, xorout 0 -> the raw register."""
    rng = np.random.default_rng(7)
    mem = rng.integers(0, 256, 2048, dtype=np.uint8).tobytes()
    for seed in (0, 1, 0xDEADBEEF, M):
        for L in (4, 5, 63, 64, 65, 700):
            for fp in (256, 257, 300):
                want = raw_update(seed, mem[fp:fp + L])
                assert model_frame(mem, fp, L, 4, seed=seed, xorout=0) == want
