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

// Device constant blob (u32 words, built once per device at init from
// gf2_crc32.h and kept in HBM; every launch's prologue copies it into LDS, an
// L2 hit after the first workgroup):
//   [kConstSlice, +1024)   T_k[b] at k * 256 + b
//   [kConstGap,   +7*128)  nibble map "advance (G - 1) * 64 bytes" for G = 2^i,
//                          entry k * 16 + n = image of n << 4k
//   [kConstTree,  +6*128)  nibble map "advance 64 * 2^j bytes" (merge level j)
constexpr uint32_t kConstSlice = 0, kConstGap = 1024, kConstTree = 1024 + 7 * 128;
constexpr uint32_t kConstWords = kConstTree + kMaxTree * 128;
constexpr uint32_t kLdsTree = kLdsGap + 16384;  // uniform kernel: 6 x 512 B merge maps after the gap map

// Prologue: the LDS image is written in 16-B chunks, chunk c = r * 1024 + t
// for thread t, so the 64 lanes of a ds_write_b128 fill 1 KiB contiguously
// (bank-conflict free; writing each thread's own 128-B table row instead put
// all lanes 256 B apart and cost 3.4 us per launch). Every thread issues all
// of its loads from the constant blob before it waits on any of them, so the
// launch pays one memory latency.
//   slice tables (128 KiB, 32 bank replicas): chunk c is row c >> 4 (pair =
//     row >> 8, byte = row & 255), half (c >> 3) & 1 -> T_{3 - (2 pair + half)}[byte];
//   gap maps: NMAPS maps of 16 x 8 rows (entry k * 16 + n) with REPL replicas,
//     map m (G = 2^gi[m]) at base + m * 64 * REPL (= its size);
//   merge maps: thread t < 128 * levels copies one word (one copy each: a
//     lookup of nibble k reads 16 consecutive words, so lanes never share a bank).
template <int NMAPS, int REPL>
__device__ __forceinline__ void build_lds_tables(const uint32_t *consts, const int (&gi)[NMAPS], uint32_t base,
                                                 int tree_levels)
{
    const uint32_t t = threadIdx.x;
    constexpr uint32_t kMapBytes = 128u * REPL * 4u;              // 128 entries x REPL words
    constexpr uint32_t kGapChunks = NMAPS * kMapBytes / 16u;      // per workgroup
    constexpr int kGapPer = (int)((kGapChunks + kBlock - 1) / kBlock);
    uint32_t v[8], vg[kGapPer];
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const uint32_t c = (uint32_t)r * kBlock + t, row = c >> 4;
        const uint32_t slot = (row >> 8) * 2u + ((c >> 3) & 1u);
        v[r] = consts[kConstSlice + (3u - slot) * 256u + (row & 255u)];
    }
#pragma unroll
    for (int r = 0; r < kGapPer; r++) {
        const uint32_t c = (uint32_t)r * kBlock + t;
        const uint32_t m = c / (kMapBytes / 16u), entry = (c % (kMapBytes / 16u)) / (REPL / 4u);
        int g = gi[0];
#pragma unroll
        for (int q = 1; q < NMAPS; q++) g = m == (uint32_t)q ? gi[q] : g;
        vg[r] = c < kGapChunks ? consts[kConstGap + (uint32_t)g * 128u + entry] : 0u;
    }
    const bool has_tree = t < (uint32_t)tree_levels * 128u;
    const uint32_t vt = has_tree ? consts[kConstTree + t] : 0u;
    uint4 *lds4 = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
    for (int r = 0; r < 8; r++) lds4[(kLdsS4 / 16u) + (uint32_t)r * kBlock + t] = make_uint4(v[r], v[r], v[r], v[r]);
#pragma unroll
    for (int r = 0; r < kGapPer; r++) {
        const uint32_t c = (uint32_t)r * kBlock + t;
        if (c < kGapChunks) lds4[base / 16u + c] = make_uint4(vg[r], vg[r], vg[r], vg[r]);
    }
    if (has_tree) s_lds[kLdsTree / 4 + t] = vt;
}

// Advance register a by 64 * 2^j bytes: 8 nibble lookups in merge map j.
__device__ __forceinline__ uint32_t tree_step(uint32_t a, int j)
{
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= lds_read(kLdsTree + (uint32_t)j * 512u + (uint32_t)k * 64u + ((a >> (4 * k)) & 15u) * 4u);
    return r;
}

// Host: fill the constant blob (kConstWords u32).
__host__ inline void fill_const_blob(uint32_t *w)
{
    for (int k = 0; k < 4; k++) {
        const uint32_t xk = gf2_x8n((uint64_t)(k + 1));
        for (int b = 0; b < 256; b++) w[kConstSlice + k * 256 + b] = gf2_mul(xk, (uint32_t)b);
    }
    for (int gi = 0; gi < 7; gi++) {
        const uint32_t x = gf2_x8n((uint64_t)((1u << gi) - 1u) * kUnit);
        for (int t = 0; t < 128; t++) w[kConstGap + gi * 128 + t] = gf2_mul(x, (uint32_t)(t & 15) << (4 * (t >> 4)));
    }
    for (int j = 0; j < kMaxTree; j++) {
        const uint32_t x = gf2_x8n((uint64_t)kUnit << j);
        for (int t = 0; t < 128; t++) w[kConstTree + j * 128 + t] = gf2_mul(x, (uint32_t)(t & 15) << (4 * (t >> 4)));
    }
}

__host__ __device__ constexpr int ilog2(int g) { return g <= 1 ? 0 : 1 + ilog2(g >> 1); }

}  // namespace vcrc
