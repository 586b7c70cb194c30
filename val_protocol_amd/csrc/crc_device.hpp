// crc_device.hpp -- gfx950 device building blocks of the CRC-32 kernels:
// LDS table layout, the slice-by-4 step, the gap step and the GF(2)
// bit-matrix. Included by val_crc32_hip.hip only.
//
// LDS image (one per workgroup, 144 KiB, built in the prologue):
//   [0, 128 KiB)      slice tables T3|T2 (pair 0) and T1|T0 (pair 1):
//                     row = byte value * 256 B, half = 128 B, 32 bank replicas
//                     of 4 B, so the 32 lanes of a half-wave read 32 banks.
//   [128, 160 KiB)    gap maps as 8 nibble tables x 16 rows: one map with 32
//                     replicas (uniform kernel, 16 KiB) or four maps with 16
//                     replicas (ragged kernel, 4 x 8 KiB; lanes l and l+16
//                     share a replica, so a gap lookup is at most 2-way).
// T_k[b] = b * x^(8(k+1)) mod P (T_0 = the classic table of the reference,
// src/val_core.c:133-148).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf2_crc32.h"

namespace vcrc {

constexpr int kUnit = 64;              // bytes a lane hashes per round
constexpr int kWords = kUnit / 4;
constexpr int kBlock = 1024;           // threads per workgroup (16 waves, 1 workgroup per CU)
constexpr int kWavesPerBlock = kBlock / 64;
constexpr uint32_t kLdsS4 = 0;
constexpr uint32_t kLdsGap = 131072;
constexpr uint32_t kLdsWords = (131072 + 32768) / 4;  // 160 KiB: the whole LDS of a CU
constexpr int kMaxTree = 6;            // log2(64 lanes)

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));

__shared__ uint32_t s_lds[kLdsWords];

__device__ __forceinline__ uint32_t lds_read(uint32_t byte_addr)
{
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_lds) + byte_addr);
}

__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const u32u *>(p); }

// Per-lane LDS bases of the slice tables (T3 consumes the first byte of a word).
struct SliceBases {
    uint32_t t3, t2, t1, t0;
};

__device__ __forceinline__ SliceBases slice_bases(uint32_t lo4)
{
    return SliceBases{kLdsS4 + lo4, kLdsS4 + 128u + lo4, kLdsS4 + 65536u + lo4, kLdsS4 + 65536u + 128u + lo4};
}

// v_perm_b32 builds [base.b0 | y.byte_k | base.b2 | 0] = the table address.
__device__ __forceinline__ uint32_t tab_addr(uint32_t y, uint32_t base, int k)
{
    return __builtin_amdgcn_perm(y, base, 0x0C020400u + ((uint32_t)k << 8));
}

// Feed one little-endian word into raw register c (slice-by-4).
__device__ __forceinline__ uint32_t s4_step(uint32_t c, uint32_t w, const SliceBases &b)
{
    const uint32_t y = c ^ w;
    return lds_read(tab_addr(y, b.t3, 0)) ^ lds_read(tab_addr(y, b.t2, 1)) ^ lds_read(tab_addr(y, b.t1, 2)) ^
           lds_read(tab_addr(y, b.t0, 3));
}

// Classic byte step c = T0[(c ^ byte) & 0xff] ^ (c >> 8) (reference val_core.c:157).
__device__ __forceinline__ uint32_t byte_step(uint32_t c, uint32_t byte, const SliceBases &b)
{
    return lds_read(tab_addr(c ^ byte, b.t0, 0)) ^ (c >> 8);
}

// Advance a register over the bytes other lanes own between two of this
// lane's units: 8 nibble lookups in a gap map with REPL replicas per row,
// based at `base` (byte address); lane_off = (lane % REPL) * 4.
template <int REPL>
__device__ __forceinline__ uint32_t gap_step(uint32_t a, uint32_t base, uint32_t lane_off)
{
    constexpr uint32_t kRow = REPL * 4, kTab = 16 * kRow;
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= lds_read(base + (uint32_t)k * kTab + ((a >> (4 * k)) & 15u) * kRow + lane_off);
    return r;
}

// r = M v for a 32x32 GF(2) matrix given by its columns (wave-uniform, SGPRs).
__device__ __forceinline__ uint32_t bitmatrix_apply(uint32_t v, const uint32_t *col)
{
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) r ^= (0u - ((v >> i) & 1u)) & col[i];
    return r;
}

// Prologue, slice tables: T_k from x^(8(k+1)) (xtab), 32 bank replicas.
__device__ __forceinline__ void build_slice_tables(const uint32_t (&xtab)[4])
{
    const int t = threadIdx.x;  // thread t: T_k[b], k = t >> 8, b = t & 255
    const int k = t >> 8, b = t & 255;
    // constant indices: a per-thread index would spill the kernel arguments to scratch
    const uint32_t xk = k == 0 ? xtab[0] : k == 1 ? xtab[1] : k == 2 ? xtab[2] : xtab[3];
    const uint32_t v = gf2_mul(xk, (uint32_t)b);
    const int slot = 3 - k;
    uint4 *row = reinterpret_cast<uint4 *>(
        s_lds + (kLdsS4 + (uint32_t)(slot >> 1) * 65536u + (uint32_t)b * 256u + (uint32_t)(slot & 1) * 128u) / 4);
    const uint4 vv = make_uint4(v, v, v, v);
#pragma unroll
    for (int r = 0; r < 8; r++) row[r] = vv;
}

// Prologue, one gap map "advance by gap bytes" (xgap = x^(8 gap)) at `base`
// with REPL replicas: threads 0..127 each build one (table, nibble) row.
template <int REPL>
__device__ __forceinline__ void build_gap_table(uint32_t xgap, uint32_t base)
{
    const int t = threadIdx.x;
    if (t < 128) {  // NT_k[n] = gap(n << 4k)
        const int k = t >> 4, nib = t & 15;
        const uint32_t v = gf2_mul(xgap, (uint32_t)nib << (4 * k));
        uint4 *row = reinterpret_cast<uint4 *>(s_lds + (base + (uint32_t)k * (16u * REPL * 4u) + (uint32_t)nib * (REPL * 4u)) / 4);
        const uint4 vv = make_uint4(v, v, v, v);
#pragma unroll
        for (int r = 0; r < REPL / 4; r++) row[r] = vv;
    }
}

}  // namespace vcrc
