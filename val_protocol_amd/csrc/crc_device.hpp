// crc_device.hpp -- gfx950 device building blocks of the CRC-32 kernels:
// LDS table layout, the slice-by-4 step, the gap step and the GF(2)
// bit-matrix. Included by val_crc32_hip.hip only.
//
// LDS image (one per workgroup, built in the prologue from the device
// constant blob):
//   [0, 128 KiB)        slice tables T3|T2 (pair 0) and T1|T0 (pair 1):
//                       row = byte value * 256 B, half = 128 B, 32 bank replicas
//                       of 4 B, so the 32 lanes of a half-wave read 32 banks.
//   [128 KiB, +6.5 KiB) 13 nibble maps of 512 B, one copy each: gap maps
//                       "advance (G - 1) * 64 bytes" for G = 2^0..2^6, then
//                       merge maps "advance 64 * 2^j bytes", j = 0..5. A map is
//                       8 tables x 16 words; a lookup of nibble k reads one of
//                       16 consecutive words, so lanes either share a word
//                       (broadcast) or hit distinct banks: no replicas needed.
//   [134.5 KiB, +8 KiB) 16 nibble maps "advance 2^(k0+i) bytes", i = 0..15:
//                       k0 = 0 for the variable shift of the RX payload-state
//                       by-product, k0 = log2(chunk) for the region fold
//                       (filled only by launches that use them).
// T_k[b] = b * x^(8(k+1)) mod P (T_0 = the classic table of the reference,
// src/val_core.c:133-148).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf2_crc32.h"

// Switches that make the kernels return wrong CRCs (A/B diagnostics of the
// load schedule, the prologue and the region fold) exist only in builds that
// say so: val_gpu_build_flags() then reports VCRC_DIAG_BUILD, and
// tests/test_build.py asserts the shipped library reports nothing.
#if (defined(VCRC_DIAG_NOHASH) || defined(VCRC_NO_LDS_FILL) || defined(VCRC_REGION_HASHONLY) || \
     defined(VCRC_REGION_NOATOMIC)) &&                                                             \
    !defined(VCRC_DIAG_BUILD)
#error "wrong-result diagnostic switches need -DVCRC_DIAG_BUILD (never a product build)"
#endif

namespace vcrc {

constexpr int kUnit = 64;              // bytes a lane hashes per round
constexpr int kWords = kUnit / 4;
constexpr int kBlock = 1024;           // threads per workgroup (16 waves, 1 workgroup per CU)
constexpr int kWavesPerBlock = kBlock / 64;
constexpr uint32_t kLdsS4 = 0;
constexpr uint32_t kLdsMaps = 131072;
constexpr uint32_t kNumMaps = 7 + 6;   // gap maps G = 2^0..2^6, merge maps j = 0..5
constexpr uint32_t kNumPowMaps = 16;   // LDS slots of "advance 2^(k0+i) bytes"
constexpr uint32_t kBlobPowMaps = 48;  // blob maps "advance 2^k bytes", k = 0..47
constexpr uint32_t kLdsPow = kLdsMaps + kNumMaps * 512;
constexpr uint32_t kLdsWords = (kLdsPow + kNumPowMaps * 512) / 4;
constexpr int kMaxTree = 6;            // log2(64 lanes)

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));  // unit loads are dword-aligned
typedef uint32_t u32u __attribute__((aligned(1)));
// Frame bytes are read through global-address-space pointers: from a generic
// pointer hipcc emitted flat loads for some kernel shapes (a flat load counts
// in both vmcnt and lgkmcnt and is waited for with both at zero).
typedef const uint8_t __attribute__((address_space(1))) gu8;
typedef const u32x4u __attribute__((address_space(1))) gu32x4u;
typedef const u32u __attribute__((address_space(1))) gu32u;
typedef const uint32_t __attribute__((address_space(1))) gu32;
__device__ __forceinline__ gu8 *gptr(const uint8_t *p) { return (gu8 *)p; }

__shared__ uint32_t s_lds[kLdsWords];

__device__ __forceinline__ uint32_t lds_read(uint32_t byte_addr)
{
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_lds) + byte_addr);
}

__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const u32u *>(p); }
__device__ __forceinline__ uint32_t ld32(gu8 *p) { return *reinterpret_cast<gu32u *>(p); }

// Per-lane LDS bases of the slice tables (T3 consumes the first byte of a
// word): the pair bases T3 and T1; T2 and T0 sit 128 B above them (the half),
// reached through the ds_read offset field, so two VGPRs hold all four.
struct SliceBases {
    uint32_t t3, t1;
};

__device__ __forceinline__ SliceBases slice_bases(uint32_t lo4)
{
    return SliceBases{kLdsS4 + lo4, kLdsS4 + 65536u + lo4};
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
#ifdef VCRC_DIAG_NOHASH  // diagnostic A/B builds only (wrong CRCs): the load schedule without the table work
    return y + b.t1;
#endif
    return lds_read(tab_addr(y, b.t3, 0)) ^ lds_read(tab_addr(y, b.t3, 1) + 128u) ^ lds_read(tab_addr(y, b.t1, 2)) ^
           lds_read(tab_addr(y, b.t1, 3) + 128u);
}

// Classic byte step c = T0[(c ^ byte) & 0xff] ^ (c >> 8) (reference val_core.c:157).
__device__ __forceinline__ uint32_t byte_step(uint32_t c, uint32_t byte, const SliceBases &b)
{
    return lds_read(tab_addr(c ^ byte, b.t1, 0) + 128u) ^ (c >> 8);
}

// Advance register a by the distance of the nibble map at byte address
// `map`: 8 lookups (table k holds the images of n << 4k).
__device__ __forceinline__ uint32_t map_apply(uint32_t a, uint32_t map)
{
#ifdef VCRC_DIAG_NOHASH
    return a ^ map;
#endif
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= lds_read(map + (uint32_t)k * 64u + ((a >> (4 * k)) & 15u) * 4u);
    return r;
}
__host__ __device__ constexpr uint32_t gap_map(int gi) { return kLdsMaps + (uint32_t)gi * 512u; }
__host__ __device__ constexpr uint32_t tree_map(int j) { return kLdsMaps + (7u + (uint32_t)j) * 512u; }
__host__ __device__ constexpr uint32_t pow_map(int k) { return kLdsPow + (uint32_t)k * 512u; }

// Device constant blob (u32 words, built once per device at init from
// gf2_crc32.h and kept in HBM; every launch's prologue copies it into LDS, an
// L2 hit after the first workgroup):
//   [kConstSlice, +1024)   T_k[b] at k * 256 + b
//   [kConstGap,   +7*128)  nibble map "advance (G - 1) * 64 bytes" for G = 2^i,
//                          entry k * 16 + n = image of n << 4k
//   [kConstTree,  +6*128)  nibble map "advance 64 * 2^j bytes" (merge level j)
//   [kConstPow,  +48*128)  nibble map "advance 2^k bytes", k = 0..47
//   [kConstPowHi,    +16)  x^(8 * 2^k) mod P for k = 16..31 (shifts past 64 KiB, VALU)
//   [kConstXpow,     +48)  x^(8 * 2^k) mod P for k = 0..47 (VALU shifts by any distance)
//   [kConstPieceMul, +4*128) x^(8 * j * 2^k0) mod P for k0 = 10..13, j = 0..127: one VALU
//                          product per piece for k_frames' in-launch tail pieces
// The maps are contiguous, in LDS order.
constexpr uint32_t kConstSlice = 0, kConstGap = 1024, kConstTree = 1024 + 7 * 128;
constexpr uint32_t kConstPow = kConstTree + kMaxTree * 128;
constexpr uint32_t kConstPowHi = kConstPow + kBlobPowMaps * 128;
constexpr uint32_t kConstXpow = kConstPowHi + 16;
constexpr uint32_t kPieceK0Min = 10, kPieceK0Max = 13, kPieceMulJ = 128;
constexpr uint32_t kConstPieceMul = kConstXpow + 48;
constexpr uint32_t kConstWords = kConstPieceMul + (kPieceK0Max - kPieceK0Min + 1) * kPieceMulJ;

// Prologue: the slice tables are written in 16-B chunks, chunk c = r * 1024 + t
// for thread t, so the 64 lanes of a ds_write_b128 fill 1 KiB contiguously
// (bank-conflict free; writing each thread's own 128-B table row instead put
// all lanes 256 B apart and cost 3.4 us per launch). Chunk c is row c >> 4
// (pair = row >> 8, byte = row & 255), half (c >> 3) & 1 ->
// T_{3 - (2 pair + half)}[byte]. The maps are copied word for word. Every
// thread issues all of its loads from the constant blob before it waits on any
// of them, so the launch pays one memory latency. The prologue is split in
// two so a kernel can issue its first frame loads between the halves: the
// blob loads go first (loads complete in issue order, so waiting for them
// does not wait for the frame data), and the HBM latency of the first round
// runs under the LDS fill and the barrier instead of after them (with no
// LDS-DMA in flight, __syncthreads() is a bare s_barrier: plain loads stay
// outstanding across it).
// NT = threads of the workgroup that fills the tables (1,024, or 512 for the
// eight-wave short-frame kernels): each thread holds 8192 / NT table chunks and
// 2048 / NT map words.
template <int NT = kBlock>
struct LdsImageT {
    uint32_t v[8 * kBlock / NT], vm[2 * kBlock / NT];
};
using LdsImage = LdsImageT<kBlock>;

template <int NT>
__device__ __forceinline__ void lds_tables_issue(const uint32_t *consts, LdsImageT<NT> &im)
{
    const uint32_t t = threadIdx.x;
    constexpr uint32_t kMapWords = kNumMaps * 128u;
#pragma unroll
    for (int r = 0; r < 8 * kBlock / NT; r++) {
        const uint32_t c = (uint32_t)r * NT + t, row = c >> 4;
        const uint32_t slot = (row >> 8) * 2u + ((c >> 3) & 1u);
        im.v[r] = consts[kConstSlice + (3u - slot) * 256u + (row & 255u)];
    }
#pragma unroll
    for (int r = 0; r < 2 * kBlock / NT; r++) {
        const uint32_t i = (uint32_t)r * NT + t;
        im.vm[r] = i < kMapWords ? consts[kConstGap + i] : 0u;
    }
}

template <int NT>
__device__ __forceinline__ void lds_tables_write(const LdsImageT<NT> &im)
{
    const uint32_t t = threadIdx.x;
    constexpr uint32_t kMapWords = kNumMaps * 128u;
    uint4 *lds4 = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
    for (int r = 0; r < 8 * kBlock / NT; r++)
        lds4[(kLdsS4 / 16u) + (uint32_t)r * NT + t] = make_uint4(im.v[r], im.v[r], im.v[r], im.v[r]);
#pragma unroll
    for (int r = 0; r < 2 * kBlock / NT; r++) {
        const uint32_t i = (uint32_t)r * NT + t;
        if (i < kMapWords) s_lds[kLdsMaps / 4u + i] = im.vm[r];
    }
}

__device__ __forceinline__ void build_lds_tables(const uint32_t *consts)
{
    LdsImage im;
    lds_tables_issue(consts, im);
    lds_tables_write(im);
}

// The 16 maps "advance 2^(k0+i) bytes" into the LDS pow slots (2 words per
// thread), in two halves like the tables: issue the loads early (before any
// frame load, so waiting for them never waits for frame data), write them in
// the prologue; the caller's barrier publishes them.
struct PowImage {
    uint32_t v[2];
};
__device__ __forceinline__ void lds_pow_issue(const uint32_t *consts, uint32_t k0, PowImage &im)
{
    static_assert(kNumPowMaps * 128u == 2 * kBlock, "two pow-map words per thread");
#pragma unroll
    for (int r = 0; r < 2; r++) im.v[r] = consts[kConstPow + k0 * 128u + (uint32_t)r * kBlock + threadIdx.x];
}
__device__ __forceinline__ void lds_pow_write(const PowImage &im)
{
#pragma unroll
    for (int r = 0; r < 2; r++) s_lds[kLdsPow / 4u + (uint32_t)r * kBlock + threadIdx.x] = im.v[r];
}
__device__ __forceinline__ void lds_pow_maps(const uint32_t *consts, uint32_t k0 = 0)
{
    PowImage im;
    lds_pow_issue(consts, k0, im);
    lds_pow_write(im);
}

// Advance raw register v over n zero bytes: one LDS nibble map (8 lookups) per
// set bit below 2^16, a VALU GF(2) multiply per set bit above.
__device__ __forceinline__ uint32_t shift_bytes(uint32_t v, uint32_t n, const uint32_t *consts)
{
#pragma unroll
    for (int k = 0; k < (int)kNumPowMaps; k++)
        if ((n >> k) & 1u) v = map_apply(v, pow_map(k));
    for (int k = 16; k < 32; k++)
        if ((n >> k) & 1u) v = gf2_mul(consts[kConstPowHi + (uint32_t)(k - 16)], v);
    return v;
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
    for (int k = 0; k < (int)kBlobPowMaps; k++) {
        const uint32_t x = gf2_x8n((uint64_t)1 << k);
        for (int t = 0; t < 128; t++) w[kConstPow + k * 128 + t] = gf2_mul(x, (uint32_t)(t & 15) << (4 * (t >> 4)));
    }
    for (int k = 16; k < 32; k++) w[kConstPowHi + k - 16] = gf2_x8n((uint64_t)1 << k);
    for (int k = 0; k < 48; k++) w[kConstXpow + k] = gf2_x8n((uint64_t)1 << k);
    for (uint32_t k0 = kPieceK0Min; k0 <= kPieceK0Max; k0++)
        for (uint32_t j = 0; j < kPieceMulJ; j++)
            w[kConstPieceMul + (k0 - kPieceK0Min) * kPieceMulJ + j] = gf2_x8n((uint64_t)j << k0);
}

// Advance raw register v over n zero bytes with VALU multiplies only (one
// GF(2) product per set bit of n, constants from the blob): no LDS maps, for
// the rare shifts of launches that do not fill the pow slots.
__device__ __forceinline__ uint32_t shift_bytes_valu(uint32_t v, uint64_t n, const uint32_t *consts)
{
    while (n) {
        const int k = __builtin_ctzll(n);
        v = gf2_mul(consts[kConstXpow + (uint32_t)k], v);
        n &= n - 1;
    }
    return v;
}

__host__ __device__ constexpr int ilog2(int g) { return g <= 1 ? 0 : 1 + ilog2(g >> 1); }

}  // namespace vcrc
