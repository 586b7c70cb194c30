// crc_kernels.hpp -- the CRC-32 kernels (gfx950). Included by val_crc32_hip.hip.
//
// k_frames<G, PF>      K1/K2/K3: per-frame trailer CRC, header_crc, verify;
//                      persistent grid, G lanes per frame, uniform geometry.
// k_bin_* + k_frames_ragged<PF>
//                      K5: ragged descriptor batches. Frames are counting-
//                      sorted by length on the device (512-B buckets, longest
//                      first), each length class runs its measured lanes per
//                      frame; a persistent grid walks the sorted items
//                      longest first. No host round trip.
// k_region             K4: long region CRC in one launch (chunk states folded
//                      per workgroup, then across workgroups by atomics).
//
// Frame algorithm (all GF(2)-linear):
//   A frame's L bytes of CRC input are cut into 64-B units counted from the
//   frame END; unit 0 is front-padded with zeros (free: a zero register stays
//   zero over zero bytes) and carries the seed XORed into the first 4 real
//   bytes. Lane g of the G lanes owns units g, g+G, g+2G, ...: a contiguous
//   64-B read per lane per round, G*64 contiguous bytes per frame per round.
//   Between its units a lane advances its register over the (G-1)*64 bytes
//   the other lanes own (gap step); a log2(G) __shfl_xor tree merges lanes.
#pragma once

#include "crc_device.hpp"

namespace vcrc {

// Length classes of the ragged path and their lanes per frame, measured on
// MI355X with uniform 3 GB batches (tools/sweep_lengths.py,
// profiles/r01_length_sweep.log).
constexpr int kClasses = 4;
#ifndef VCRC_CLASS_LANES  // A/B builds may override, e.g. -DVCRC_CLASS_LANES=4,8,16,16 (each >= the default: a
#define VCRC_CLASS_LANES 2, 4, 8, 16  // bucket must stay inside one round of its class)
#endif
constexpr int kClassLanes[kClasses] = {VCRC_CLASS_LANES};
__host__ __device__ constexpr int class_lanes(int c) { return c == 0 ? kClassLanes[0] : c == 1 ? kClassLanes[1] : c == 2 ? kClassLanes[2] : kClassLanes[3]; }
__host__ __device__ inline int length_class(uint32_t L)
{
    return L < 1024u ? 0 : L < 8192u ? 1 : L < 49152u ? 2 : 3;
}

// Work-queue partitions: the ragged kernel's item queue (kQueueParts) and the
// uniform kernel's dynamic tail (kDynParts), one head word each, 64 B apart;
// the host sizes both scratch blocks from these.
#ifndef VCRC_RAGGED_PARTS  // A/B builds may override
#define VCRC_RAGGED_PARTS 64  // 1, 2, 4 partitions: slower (u1100 up to 2.8x); 8 -> 64: +1.5-3% (r02_ab_ragged_parts.log)
#endif
#ifndef VCRC_DYN_PARTS  // A/B builds may override (the host picks 1 or this per launch)
#define VCRC_DYN_PARTS 64
#endif
constexpr uint32_t kQueueParts = VCRC_RAGGED_PARTS, kDynParts = VCRC_DYN_PARTS;
static_assert(kQueueParts >= 1 && kQueueParts <= 64 && kDynParts >= 1 && kDynParts <= 64, "queue partitions");
constexpr uint32_t kDynQueueBytes = (kDynParts + 1u) * 64u;  // heads, then the exit counter

struct FrameParams {
    const uint8_t *base;
    const uint64_t *off;     // descriptor mode (NULL: strided mode)
    const uint32_t *len;
    uint64_t stride;         // strided mode
    uint32_t flen;
    uint32_t last_len;       // strided mode: length of frame n-1
    uint32_t n;
    uint32_t seed0;          // initial register of frame 0
    uint32_t seed_rest;      // initial register of frames 1..n-1
    uint32_t xorout;         // XORed into every output (0xFFFFFFFF = finished CRC)
    uint32_t *out_crc;
    uint32_t *out_hdr;
    uint8_t *out_ok;
    uint32_t *nbad;
    uint32_t verify;
    const uint32_t *order;   // grouped mode: class-sorted frame indices
    const uint32_t *plan;    // ragged mode: class table {cstart[4], ccount[4], istart[5]}
    uint32_t *heads;         // ragged mode: 8 work-queue heads, 64 B apart, zero on entry
    uint32_t *bin_counts;    // ragged mode: k_bin_count's bucket totals, re-zeroed here for the next batch
    const uint32_t *consts;  // device constant blob (crc_device.hpp): tables and maps
    uint32_t *out_pay;       // RX by-product: raw zero-init register of each frame's payload (nullable)
    uint32_t *qhead;         // uniform mode: dynamic-tail queue, kDynQueueBytes (zero on entry, re-zeroed), nullable
    uint32_t static_rounds;  // with qhead: group rounds dealt statically before the queue
    uint32_t qparts;         // with qhead: queue partitions, 1..kDynParts
    // uniform mode, G >= 8: frames [n, n + tail_n) hashed in pieces inside this launch (tail_pieces)
    uint32_t tail_n;         // 0: none
    uint32_t tail_units;     // pieces per tail frame
    uint32_t tail_k0;        // piece bytes W = 2^tail_k0
    uint32_t tail_last_len;  // strided mode: length of the last tail frame
    uint32_t *tail_acc;      // {register, arrivals} per tail frame (zero on entry, re-zeroed)
};

// Bytes before a DATA frame's payload: the 8-B header, plus the 8-B file
// offset when flags (byte 1) has VAL_DATA_OFFSET_PRESENT (reference
// include/val_wire.h:45, src/val_core.c:743-766).
__device__ __forceinline__ uint32_t payload_prefix(uint32_t hdr_word0) { return (hdr_word0 & 0x100u) ? 16u : 8u; }

// A full 64-B unit at a dword-aligned address: four dwordx4 loads. Every
// unit is dword-aligned by construction (hash_frame anchors the unit grid at
// floor4(frame end)); a dword-aligned load never crosses a page, so nothing
// outside the buffer's pages is touched.
__device__ __forceinline__ void load_full(uint32_t (&w)[kWords], gu8 *up)
{
#pragma unroll
    for (int q = 0; q < kWords / 4; q++) {
        const u32x4u v = *reinterpret_cast<gu32x4u *>(up + 16 * q);
        w[4 * q + 0] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
}

// Unit 0 through its frame's first line. Unit 0 starts pad bytes before the
// frame, so read whole it can reach into the previous 128-B line (the previous
// frame's end, which that frame reads a group-time later: 1,100-B frames read
// 1.30x their bytes that way, against 1.12x when only the frame's own line is
// touched). Sixteen clamped dword loads (round 2) issued sixteen memory
// instructions and needed sixteen addresses. Here the 64 B are read from
// A = max(unit start, the frame's first line) by four dwordx4 loads, never
// outside that line (A is dword-aligned and A + 64 stays in the line), and
// moved up by the s = (A - unit start) / 4 words skipped: a four-stage select
// network. The words before the frame are masked later (unit0_finish). A line
// never crosses a page, so the read is safe even for a frame at the very start
// of its buffer. (Uniform 1,100-B ragged batches +3.5%, cfg5 +0.9%:
// profiles/r03_ab_unit0_line.log.)
// (The loads are issued by load_unit0, the words moved by unit0_line_shift
// where they are used: the shift amount is recomputed, so nothing extra stays
// live in between.)
__device__ __forceinline__ uint32_t unit0_line_skip(gu8 *fp, uint32_t pad)  // bytes of unit 0 before fp's line
{
    const uint32_t in_line = (uint32_t)((uintptr_t)fp & 127u);
    return pad > in_line ? pad - in_line : 0u;
}
__device__ __forceinline__ void unit0_line_shift(uint32_t (&w)[kWords], gu8 *fp, uint32_t pad)
{
    const uint32_t sh = unit0_line_skip(fp, pad) >> 2;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const int d = 1 << b;
        const bool on = (sh >> b) & 1u;
#pragma unroll
        for (int i = kWords - 1; i >= 0; i--) w[i] = on ? (i >= d ? w[i - d] : 0u) : w[i];
    }
}

// Words of a lane's round-0 unit u: u > 0 a full unit; u == 0 the front-padded
// first unit, with the seed in frame bytes 0..3; u < 0 nothing. Lg = bytes on
// the unit grid; Lg < 4 frames take the byte path (tiny). Loads only, into
// registers left undefined for lanes without a unit; unit 0's words are moved
// into place (unit0_line_shift) and the masks and the seed applied
// (unit0_finish) where the words are first used. hipcc waits for every
// outstanding load at the first use of a loaded value, and at the end of a
// branch whose loads feed a value defined on the other path too: with the
// masks next to the loads (and zeros on the other path) the loads of unit 0
// ran one memory round trip after another, behind round 1's prefetch.
// Unit u starts at fp + 64u - pad, dword-aligned (the grid ends at
// floor4(frame end)); unit 0 is read from inside the frame's first line
// (unit0_line_skip). In k_frames (multi-pass launches) and the ragged kernel
// every round-0 unit is read by four dwordx4 loads: one load shape on every
// path. With two shapes (round 2: sixteen clamped dword
// loads for unit 0 beside whole-unit loads; round 3 briefly: the line loads
// beside them) the results met in copies at the join, which waited for the
// loads there, and the LDS fill stopped overlapping the first memory latency
// (one-pass windows of 64-1024 frames +1.7 us per call,
// profiles/r03_ab_round0_shape.log).
// BF (k_region, k_frames_split): branch-free, every lane issues the loads; a
// lane without a unit reads 64 B of `dummy` (the constant blob, an L1/L2
// hit); whole units by dwordx4, the window's unit 0 by clamped dword loads
// (the line loads cost these one-pass launches about 2 us per call:
// profiles/r03_summary.json ab_region). Behind a skippable branch, the waitcnt pass could not count them, and
// the prologue's waits for the constant-blob loads (issued first) then also
// waited for most of the frame loads (region launches: prologue 7.7 us;
// tools/timing_region.py).
// Otherwise (k_frames, ragged): only lanes with a unit issue them; measured
// faster on frame batches (the dummy loads cost cfg2 3%, a 256-frame window 9%).
// C0 (k_frames launches that are one pass of the grid: windows, cfg2): round
// 2's sixteen dword loads per round-0 unit, unit 0's clamped to the frame's
// first dword (a word wholly before the frame reads that dword and is masked
// to zero). The line loads above are faster on batches of many group rounds
// (1,100-B frames +4-7%) and slower on one-pass launches, where round 0 is the
// whole wait (windows of 64-1024 frames -10%, cfg2 -3.4%;
// profiles/r03_ab_round0_shape.log), so both are kept and the host picks.
template <bool BF, bool C0 = false>
__device__ __forceinline__ void load_unit0(uint32_t (&w)[kWords], int u, gu8 *fp, uint32_t Lg, uint32_t pad, gu8 *dummy)
{
    const bool has = u >= 0 && Lg >= 4;
    if (C0 && !BF) {
        if (has) {
            gu8 *const base = fp + ((int64_t)u * kUnit - pad);
            const uint32_t lo = u == 0 ? (pad & ~3u) : 0u;
#pragma unroll
            for (int i = 0; i < kWords; i++) w[i] = *reinterpret_cast<gu32 *>(base + max(4u * (uint32_t)i, lo));
        }
        return;
    }
    if (BF) {  // k_region, k_frames_split: every unit but a window's first is whole
        gu8 *const base = has ? fp + ((int64_t)u * kUnit - pad) : dummy;
        const uint32_t lo = (has && u == 0) ? (pad & ~3u) : 0u;
        if (lo == 0) {
            load_full(w, base);
        } else {
#pragma unroll
            for (int i = 0; i < kWords; i++) w[i] = *reinterpret_cast<gu32 *>(base + max(4u * (uint32_t)i, lo));
        }
        return;
    }
    if (has) load_full(w, fp + ((int64_t)u * kUnit - pad) + (u == 0 ? unit0_line_skip(fp, pad) : 0u));
}

// 16-B interleaved loads of rounds >= 1 at G = 2 and 4 (round 4): a round's
// G x 64-B span is read by four dwordx4 instructions, instruction q covering
// the span's bytes [16 G q, 16 G (q + 1)) with lane g at 16 g, so one
// instruction reads G x 16 contiguous bytes of each frame (the unit layout
// reads 16 B at a 64-B lane stride: 32 B of each line per instruction). Lanes
// then swap chunks inside their frame's lane group (DPP quad permutes: the G
// lanes of a frame are one quad or one pair) so that each holds its own 64-B
// unit again and the hash is unchanged. Lane g's register q holds span chunk
// q G + g; unit g is chunks 4 g .. 4 g + 3. Same box against the unit
// loads (profiles/r04_ab_ilv16.log, r04_ab_ilv16_ragged.log): u1100d
// +1.7-2.7%, u600d +2.2%, u2000d +2.1%, s1100 0 to +0.8%; one-pass launches
// lost (cfg2 -3%), so the C0 kernels keep the unit loads. -DVCRC_ILV16=0
// builds the unit loads everywhere (A/B).
#ifndef VCRC_ILV16
#define VCRC_ILV16 1
#endif
template <int GT>
constexpr bool ilv_lanes() { return VCRC_ILV16 && (GT == 2 || GT == 4); }
// Not in the ragged kernel (run-time G per length class): choosing the load
// shape per item (wave-uniform branches in the round loop) cost the ragged
// path 4-11% (u1100 ragged -11%, u600 -4%, cfg5 -10%;
// profiles/r04_ab_ilv16_ragged.log).

__device__ __forceinline__ void load_ilv(uint32_t (&w)[kWords], gu8 *span_lane, int G)  // span_lane = span + 16 g
{
#pragma unroll
    for (int q = 0; q < kWords / 4; q++) {
        const u32x4u v = *reinterpret_cast<gu32x4u *>(span_lane + 16 * G * q);
        w[4 * q + 0] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
}

template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

template <int GT>
__device__ __forceinline__ void ilv_to_units(uint32_t (&w)[kWords], int g)
{
    constexpr int kSwap1 = 0xB1, kSwap2 = 0x4E;  // quad_perm [1,0,3,2] and [2,3,0,1]
    if (GT == 4) {
        // 4 x 4 transpose of 16-B chunks in the quad: two butterfly stages
        const bool o1 = g & 1, o2 = g & 2;
#pragma unroll
        for (int q = 0; q < 4; q += 2)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t r = quad_perm<kSwap1>(o1 ? w[4 * q + i] : w[4 * (q + 1) + i]);
                if (o1) w[4 * q + i] = r;
                else w[4 * (q + 1) + i] = r;
            }
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t r = quad_perm<kSwap2>(o2 ? w[4 * q + i] : w[4 * (q + 2) + i]);
                if (o2) w[4 * q + i] = r;
                else w[4 * (q + 2) + i] = r;
            }
    } else if (GT == 2) {
        // lane 0's unit = L0.R0 L1.R0 L0.R1 L1.R1; lane 1's = L0.R2 L1.R2 L0.R3 L1.R3
        const bool o = g & 1;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t a = quad_perm<kSwap1>(o ? w[i] : w[8 + i]);
            const uint32_t b = quad_perm<kSwap1>(o ? w[4 + i] : w[12 + i]);
            const uint32_t r0 = w[i], r1 = w[4 + i], r2 = w[8 + i], r3 = w[12 + i];
            w[i] = o ? a : r0;
            w[4 + i] = o ? r2 : a;
            w[8 + i] = o ? b : r1;
            w[12 + i] = o ? r3 : b;
        }
    }
}

// Mask and seed of unit-0 word i (frame offset q = 4i - pad): bytes before the
// frame are zero and the seed is XORed into frame bytes 0..3.
__device__ __forceinline__ uint32_t unit0_word(uint32_t x, int q, uint32_t seed)
{
    if (q <= -4) return 0u;
    if (q < 0) return (x & (~0u << (8 * -q))) ^ (seed << (8 * -q));
    return q < 4 ? x ^ (seed >> (8 * q)) : x;
}

__device__ __forceinline__ void unit0_finish(uint32_t (&w)[kWords], int u, uint32_t Lg, uint32_t pad, uint32_t seed)
{
    const bool has = u >= 0 && Lg >= 4;
#pragma unroll
    for (int i = 0; i < kWords; i++) {
        const uint32_t x = u == 0 ? unit0_word(w[i], 4 * i - (int)pad, seed) : w[i];
        w[i] = has ? x : 0u;
    }
    // Seed bytes that did not fit in a unit 0 holding < 4 real bytes.
    if (u == 1 && pad > kUnit - 4) w[0] ^= seed >> (8 * (kUnit - pad));
}

// Kernel arguments the first memory accesses depend on, fetched together: an
// empty asm that needs them in SGPRs makes the compiler issue their scalar
// loads up front and wait once. Left to itself it loaded the constant-blob
// pointer, waited, then loaded the frame base, lengths and stride and waited
// again: two kernarg round trips before the first frame load.
#ifndef VCRC_NO_KARG_EARLY  // diagnostic A/B builds only
#define VCRC_KARG_EARLY(...) asm volatile("" ::__VA_ARGS__)
#else
#define VCRC_KARG_EARLY(...) \
    do {                     \
    } while (0)
#endif

// Descriptor of frame f (offset and CRC-input length).
__device__ __forceinline__ void frame_desc(const FrameParams &p, uint64_t f, uint64_t &off, uint32_t &L)
{
    if (p.off) {
        off = p.off[f];
        L = p.len[f];
    } else {
        // select values, not kernel-argument lvalues: `cond ? p.last_len : p.flen`
        // made hipcc spill both to scratch, and a scratch-using kernel launches
        // its waves several us slower
        const uint32_t flen = p.flen, last = p.last_len;
        off = f * p.stride;
        L = (f + 1 == p.n) ? last : flen;
    }
}

// Register after feeding words first..15 of w into a zero register
// (first is wave-uniform: a scalar jump into the unrolled steps).
__device__ __forceinline__ uint32_t s4_words_from(int first, const uint32_t (&w)[kWords], const SliceBases &sb)
{
    uint32_t acc = 0;
    switch (first) {
#define VCRC_STEP(i) \
    case i: acc = s4_step(acc, w[i], sb); [[fallthrough]];
        VCRC_STEP(0) VCRC_STEP(1) VCRC_STEP(2) VCRC_STEP(3) VCRC_STEP(4) VCRC_STEP(5) VCRC_STEP(6) VCRC_STEP(7)
        VCRC_STEP(8) VCRC_STEP(9) VCRC_STEP(10) VCRC_STEP(11) VCRC_STEP(12) VCRC_STEP(13) VCRC_STEP(14) VCRC_STEP(15)
#undef VCRC_STEP
    default: break;
    }
    return acc;
}

// Hash frame f (at base + off, L bytes) with the G lanes of this lane's group
// (g = 0..G-1). All 64 lanes of the wave must call this together (the merge
// tree shuffles); inactive lanes pass L = 0.
// PF = rounds whose 64 B sit in registers ahead of the one being hashed: 1 on
// long batches (measured best); 2 or 4 when the whole batch is one pass of the
// grid (small windows: every round's load is issued before the first returns,
// so a wave pays one HBM latency instead of R - 1).
// GT = 0: G is the runtime value Gr (the ragged kernel: one code path for
// every length class, half the registers of four inlined instances).
// pre() runs once this frame's first loads are issued and before the first
// LDS read: a launch's first call passes the LDS fill and the barrier, so the
// latency of round 0 runs under them.
// PAY: also write the payload state (p.out_pay); a separate instantiation so
// the TX and plain verify kernels carry none of its registers.
// BF: branch-free round-0 loads (load_unit0); k_region only.
// mid() runs once round 0 is hashed (all 64 lanes, wave-uniform): the ragged
// kernel fetches its next item's descriptors there.
struct NoMid {
    __device__ void operator()() const {}
};
template <int GT, int PF, bool PAY, bool BF, bool C0 = false, typename Pre, typename Mid = NoMid>
__device__ __forceinline__ uint32_t hash_frame(const FrameParams &p, uint64_t f, bool active, uint64_t off, uint32_t L, int g,
                                           const SliceBases &sb, int Gr, Pre &&pre, Mid &&mid = Mid{})
{
    // PF < 0 (burst): rounds 1..-PF are all issued with round 0 and hashed in
    // place, never refilled; rounds past them (frames longer than the burst)
    // are loaded one at a time after it.
    constexpr bool BURST = PF < 0;
    constexpr int D = PF > 0 ? PF : (BURST ? -PF : 1);
    const int G = GT ? GT : Gr;
    const uint32_t gmap = gap_map(GT ? ilog2(GT) : __builtin_ctz((unsigned)Gr));
    gu8 *fp = gptr(p.base) + off;
    const uint32_t seed = (f == 0) ? p.seed0 : p.seed_rest;
    // The unit grid ends at floor4(frame end), so every unit is dword-aligned
    // whatever the frame's byte alignment; the tb <= 3 bytes past it are fed
    // by byte steps after the merge.
    const uint32_t tb = min((uint32_t)((uintptr_t)(fp + L) & 3u), L);
    const uint32_t Lg = L - tb;
    const uint32_t U = Lg ? (Lg + kUnit - 1) / kUnit : 1u;
    const uint32_t R = active ? (U + G - 1) >> (GT ? ilog2(GT) : __builtin_ctz((unsigned)Gr)) : 0u;
    const uint32_t pad = U * kUnit - Lg;
    const int u0 = (int)U - G * (int)R + g;  // this lane's unit in round 0
    gu8 *up = fp + ((int64_t)u0 + G) * kUnit - pad;  // its unit in round 1
    const uint64_t kStep = (uint64_t)G * kUnit;                // bytes between a lane's rounds
    // Round 0 is issued before the prefetched rounds: loads complete in issue
    // order, so hashing it never waits for them.
    uint32_t w0[kWords];
    const bool tiny = u0 == 0 && Lg < 4;
    gu8 *const dummy = gptr(reinterpret_cast<const uint8_t *>(p.consts));
    load_unit0<BF, C0>(w0, u0, fp, Lg, pad, dummy);
    // header_crc: by the lane holding unit 0, from the frame's first line,
    // which round 0 reads anyway (read after the merge, the line had left the
    // caches: +0.4% HBM traffic on cfg3).
    const bool hdr = R > 0 && u0 == 0 && p.out_hdr;
    uint32_t h0, h1;
    if (BF || (hdr && L >= 8)) {
        gu8 *hp = (hdr && L >= 8) ? fp : dummy;
        h0 = ld32(hp);
        h1 = ld32(hp + 4);
    }
    constexpr bool ILV = ilv_lanes<GT>() && !BF && !C0;
    gu8 *const ilv_up = up - 48 * g;  // round 1's span + 16 g (ILV)
    uint32_t nxt[D][kWords];
    if (PF != 0) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            if (ILV) {
                if (R > 1u + d) load_ilv(nxt[d], ilv_up + d * kStep, G);
            } else if (BF || R > 1u + d) {
                load_full(nxt[d], R > 1u + d ? up + d * kStep : dummy);
            }
        }
    }
    uint32_t acc = 0;
    // Round 0's leading zero words (unit 0's front padding, lanes without a
    // unit) leave the zero register unchanged: the wave starts at the first
    // word any lane needs (e.g. 16,400-B frames: 257 units, round 0 = one
    // unit holding 16 real bytes -> 4 steps instead of 16).
    int first = (R == 0 || u0 < 0) ? kWords : (u0 == 0 ? (int)(pad >> 2) : 0);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) first = min(first, __shfl_xor(first, o));
    first = __builtin_amdgcn_readfirstlane(first);
    pre();
    if (hdr) {
        uint32_t h = seed;
        if (L >= 8) {
            h = s4_step(h, h0, sb);
            h = s4_step(h, h1, sb);
        } else {
            for (uint32_t i = 0; i < L; i++) h = byte_step(h, fp[i], sb);
        }
        p.out_hdr[f] = h ^ p.xorout;
    }
    if (R > 0) {
        // Round 0 alone can hold unit 0 (padding, seed, tiny frames) or no
        // unit; the register is still zero, so no gap step.
        if (u0 == 0 && Lg >= 4 && !BF && !C0) unit0_line_shift(w0, fp, pad);
        unit0_finish(w0, u0, Lg, pad, seed);
        acc = s4_words_from(first, w0, sb);
        if (tiny) {  // Lg < 4: state of all L bytes straight from the seed
            acc = seed;
            for (uint32_t i = 0; i < L; i++) acc = byte_step(acc, fp[i], sb);
        }
    }
    mid();
    // Seed bytes past a unit 0 with < 4 real bytes land in unit 1 (lane 0, round 1).
    const bool seed_spill = g == 0 && pad > kUnit - 4 && (int)U - G * (int)(R - 1) == 1;
    if (PF == 0) {
        for (uint32_t k = 1; k < R; k++, up += kStep) {
            uint32_t w[kWords];
            if (ILV) {
                load_ilv(w, up - 48 * g, G);
                ilv_to_units<GT>(w, g);
            } else {
                load_full(w, up);
            }
            if (k == 1 && seed_spill) w[0] ^= seed >> (8 * (kUnit - pad));
            if (G > 1) acc = map_apply(acc, gmap);
#pragma unroll
            for (int i = 0; i < kWords; i++) acc = s4_step(acc, w[i], sb);
        }
    } else if (BURST) {
        // ring in place: round k sits in nxt[(k - 1) % D], is hashed there, and
        // its registers are then refilled with round k + D (no copy, so the
        // D - 1 rounds after it stay in flight while it is hashed)
        for (uint32_t k = 1; k < R; k += D) {
#pragma unroll
            for (int d = 0; d < D; d++) {
                const uint32_t kk = k + d;
                if (kk < R) {
                    if (ILV) ilv_to_units<GT>(nxt[d], g);
                    if (kk == 1 && seed_spill) nxt[d][0] ^= seed >> (8 * (kUnit - pad));
                    if (G > 1) acc = map_apply(acc, gmap);
#pragma unroll
                    for (int i = 0; i < kWords; i++) acc = s4_step(acc, nxt[d][i], sb);
                    if (kk + D < R) {
                        if (ILV) load_ilv(nxt[d], ilv_up + (uint64_t)(kk + D - 1) * kStep, G);
                        else load_full(nxt[d], up + (uint64_t)(kk + D - 1) * kStep);
                    }
                }
            }
        }
    } else {
        // nxt[d] holds round k + d; once consumed it is refilled with round k + d + D.
        for (uint32_t k = 1; k < R; k += D) {
#pragma unroll
            for (int d = 0; d < D; d++) {
                const uint32_t kk = k + d;
                if (kk < R) {
                    uint32_t w[kWords];
#pragma unroll
                    for (int i = 0; i < kWords; i++) w[i] = nxt[d][i];
                    if (kk + D < R) {
                        if (ILV) load_ilv(nxt[d], ilv_up + (uint64_t)(kk + D - 1) * kStep, G);
                        else load_full(nxt[d], up + (uint64_t)(kk + D - 1) * kStep);
                    }
                    if (ILV) ilv_to_units<GT>(w, g);
                    if (kk == 1 && seed_spill) w[0] ^= seed >> (8 * (kUnit - pad));
                    if (G > 1) acc = map_apply(acc, gmap);
#pragma unroll
                    for (int i = 0; i < kWords; i++) acc = s4_step(acc, w[i], sb);
                }
            }
        }
    }
    // The tb <= 3 bytes past the grid and, on verify, the stored trailer: all
    // issued before the merge, which hides their round trip (a byte loop after
    // it waited once per byte).
    // (One dword-aligned load for the tail bytes instead of three byte loads
    // measured the same: cfg5 -0.2%, 1,101-B frames +0.2%;
    // profiles/r04_ab_tail_dword.log.)
    uint32_t tail[3] = {0, 0, 0}, trailer = 0, pw[4] = {0, 0, 0, 0};
    if (active && g == G - 1) {
        if (tb && Lg >= 4) {
#pragma unroll
            for (uint32_t j = 0; j < 3; j++) tail[j] = fp[Lg + min(j, tb - 1)];
        }
        if (p.verify) trailer = ld32(fp + L);
        // payload by-product: the frame's first 16 bytes (L1/L2 hits: the
        // unit-0 lane read them in round 0)
        if (PAY && L >= 8) {
            pw[0] = ld32(fp);
            pw[1] = ld32(fp + 4);
            if (L >= 16) {
                pw[2] = ld32(fp + 8);
                pw[3] = ld32(fp + 12);
            }
        }
    }
    // Merge: level j joins blocks of 2^j lanes, the left one advanced by 64 * 2^j
    // bytes (LDS nibble map: 8 lookups, where a bit-matrix product costs 96 VALU).
#pragma unroll
    for (int j = 0; j < kMaxTree; j++) {
        if ((1 << j) >= G) break;
        const uint32_t other = __shfl_xor(acc, 1 << j);
        const bool right = (g >> j) & 1;
        const uint32_t left = right ? other : acc;
        acc = map_apply(left, tree_map(j)) ^ (right ? acc : other);
    }
    if (active && g == G - 1) {
        if (Lg >= 4) {  // the bytes past the unit grid (tiny frames already fed all L)
#pragma unroll
            for (uint32_t j = 0; j < 3; j++)
                if (j < tb) acc = byte_step(acc, tail[j], sb);
        }
        const uint32_t crc = acc ^ p.xorout;
        if (p.out_crc) p.out_crc[f] = crc;
        if (PAY) {
            // RX rolling file CRC by-product (reference src/val_receiver.c:794,
            // 891): payload register from zero = frame register ^ (register
            // after the prefix, advanced over the payload's length), by
            // linearity. Frames shorter than their prefix carry no payload.
            const uint32_t pre = L >= 8 ? payload_prefix(pw[0]) : 0xFFFFFFFFu;
            uint32_t pay = 0;
            if (L >= 8 && L >= pre) {
                uint32_t h = s4_step(s4_step(seed, pw[0], sb), pw[1], sb);
                if (pre == 16u) h = s4_step(s4_step(h, pw[2], sb), pw[3], sb);
                pay = acc ^ shift_bytes(h, L - pre, p.consts);
            }
            p.out_pay[f] = pay;
        }
        if (p.verify) {
            const bool good = (crc == trailer);
            if (p.out_ok) p.out_ok[f] = good ? 1u : 0u;
            if (!good && p.nbad) atomicAdd(p.nbad, 1u);
        }
    }
    return acc;  // lane G - 1: the frame's raw register (before xorout)
}

#ifdef VCRC_TIMING  // diagnostic builds only (tools/timing_cfg2.py): per-wave s_memrealtime stamps
__device__ uint64_t g_vcrc_time[4096 * 4];
__device__ uint32_t g_vcrc_info[4096];  // ragged: class << 16 | (L >> 6) of lane 0's frame in the wave's last item
#define VCRC_LAST_ITEM(c_, L_)                                                                                  \
    do {                                                                                                        \
        const uint64_t w_ = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;                                 \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                                   \
        const uint32_t l_ = __shfl((uint32_t)(L_), 0);                                                          \
        if ((threadIdx.x & 63) == 0 && w_ < 4096) {                                                             \
            g_vcrc_time[w_ * 4 + 3] = t_;                                                                       \
            g_vcrc_info[w_] = ((uint32_t)(c_) << 16) | (l_ >> 6);                                               \
        }                                                                                                       \
    } while (0)
#define VCRC_STAMP(k)                                                                                      \
    do {                                                                                                   \
        const uint64_t w_ = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;                            \
        if ((threadIdx.x & 63) == 0 && w_ < 4096) g_vcrc_time[w_ * 4 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define VCRC_STAMP(k) \
    do {              \
    } while (0)
#define VCRC_LAST_ITEM(c_, L_) \
    do {                       \
    } while (0)
#endif

// Uniform geometry: persistent grid, each wave hashes 64/G frames per step;
// wave w takes groups w, w + nwaves, ... The four waves of a SIMD finish in
// age order (cfg3: 2.59 / 2.62 / 2.71 / 2.88 ms, the oldest issues first), but
// a dynamic work queue that evened them out measured 3-5% slower on cfg3,
// cfg4 and unaligned uniform batches (profiles/r01_ab_dynamic_uniform.log):
// the static deal is kept.
// One frame group of a uniform wave: hash group f.., fetch the next group's
// descriptors meanwhile, advance.
template <int G, int PF, bool PAY, bool C0, typename Pre>
__device__ __forceinline__ void group_pass(const FrameParams &p, uint64_t &f, uint64_t &off, uint32_t &L, uint64_t &fb,
                                           uint64_t step, int lane, const SliceBases &sb, Pre &&pre)
{
    const uint64_t fn = f + step;
    uint64_t off_n = 0;
    uint32_t L_n = 0;
    if (fn < p.n) frame_desc(p, fn, off_n, L_n);
    hash_frame<G, PF, PAY, false, C0>(p, f, f < p.n, off, L, lane % G, sb, G, pre);
    f = fn;
    off = off_n;
    L = L_n;
    fb += step;
}

// In-launch tail of a uniform launch (launch_uniform). A batch whose frame
// groups do not fill the last wave-round (131,113 x 64 KiB frames: 8 rounds
// and 41 frames; a 1 GiB eighth of that file: one round and 6 frames) used to
// hash those frames in a second small launch after this one: a launch boundary
// and a 12-14 us latency-bound kernel on 6-41 CUs, 9% of a 1 GiB step. Here
// they are cut into pieces that the waves hash as one extra frame group each,
// after their own groups, the oldest waves first (a SIMD's oldest waves
// finish first, see above): piece j of a tail frame of L bytes covers
// [L - (j+1) W, L - j W) (W = 2^tail_k0, 1 KiB unless the pieces would need
// more groups than there are waves), the front piece everything before
// it, and the piece holding the frame's first byte carries the seed. Each
// piece's register is advanced over the j W bytes after it and XORed into the
// frame's accumulator (device-scope atomics, each returned before the next is
// issued, as k_region folds); the frame's last piece to count in writes its
// outputs (trailer CRC, header_crc, verify) and re-zeroes the accumulator.
__device__ __forceinline__ void tail_desc(const FrameParams &p, uint32_t t, uint64_t &off, uint32_t &L)
{
    const uint64_t f = (uint64_t)p.n + t;
    if (p.off) {
        off = p.off[f];
        L = p.len[f];
    } else {
        const uint32_t flen = p.flen, last = p.tail_last_len;
        off = f * p.stride;
        L = (t + 1 == p.tail_n) ? last : flen;
    }
}

// Instances that carry the path: 8 and 16 lanes per frame (2-48 KiB and longer
// frames), the default round depth; in the others its registers made the
// 32- and 64-lane one-pass kernels spill.
template <int G, int PF, bool PAY, int BT>
constexpr bool kTailPieces = (G == 8 || G == 16) && PF == 1 && !PAY && BT == kBlock;

template <int G, int PF, bool C0>
__device__ __forceinline__ void tail_pieces(const FrameParams &p, int lane, const SliceBases &sb)
{
    constexpr int kGroups = 64 / G;
    const uint32_t total = p.tail_n * p.tail_units;
    const uint32_t wg = (uint32_t)(threadIdx.x >> 6) * gridDim.x + blockIdx.x;  // oldest waves first
    if (wg * (uint32_t)kGroups >= total) return;                                // wave-uniform
    const uint32_t u = wg * (uint32_t)kGroups + (uint32_t)(lane / G);
    const bool real = u < total;
    const uint32_t t = real ? u / p.tail_units : 0u, j = real ? u % p.tail_units : 0u;
    uint64_t off = 0;
    uint32_t L = 0;
    if (real) tail_desc(p, t, off, L);
    const uint64_t after = (uint64_t)j << p.tail_k0;  // bytes of the frame after this piece
    const uint32_t W = 1u << p.tail_k0;
    const uint32_t hi = (uint64_t)L > after ? (uint32_t)((uint64_t)L - after) : 0u;
    const uint32_t lo = (j + 1u == p.tail_units || hi <= W) ? 0u : hi - W;
    const bool carrier = real && lo == 0u && (hi > 0u || j == 0u);  // holds byte 0 (or is an empty frame's piece 0)
    const bool act = real && (hi > lo || carrier);
    FrameParams q{};
    q.base = p.base;
    q.consts = p.consts;
    q.seed0 = p.seed_rest;  // a tail frame is never frame 0 of the batch
    const uint32_t st = hash_frame<G, PF, false, false, C0>(q, carrier ? 0u : 1u, act, off + lo, act ? hi - lo : 0u,
                                                         lane % G, sb, G, [] {});
    if (!real || lane % G != G - 1) return;
    uint32_t v = 0;
    if (act) {  // one product from the blob's piece table (any other distance: a product per set bit)
        const bool tab = p.tail_k0 >= kPieceK0Min && p.tail_k0 <= kPieceK0Max && j < kPieceMulJ;
        v = tab ? gf2_mul(p.consts[kConstPieceMul + (p.tail_k0 - kPieceK0Min) * kPieceMulJ + j], st)
                : shift_bytes_valu(st, after, p.consts);
    }
    uint32_t *a = p.tail_acc + 2u * t;
    const uint32_t old = atomicXor(&a[0], v);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");
    const uint32_t arrived = atomicAdd(&a[1], 1u);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(arrived) : "memory");
    if (arrived + 1u != p.tail_units) return;
    const uint32_t crc = atomicExch(&a[0], 0u) ^ p.xorout;
    atomicExch(&a[1], 0u);
    const uint64_t f = (uint64_t)p.n + t;
    gu8 *fp = gptr(p.base) + off;
    if (p.out_crc) p.out_crc[f] = crc;
    if (p.out_hdr) {
        uint32_t h = p.seed_rest;
        if (L >= 8) {
            h = s4_step(h, ld32(fp), sb);
            h = s4_step(h, ld32(fp + 4), sb);
        } else {
            for (uint32_t i = 0; i < L; i++) h = byte_step(h, fp[i], sb);
        }
        p.out_hdr[f] = h ^ p.xorout;
    }
    if (p.verify) {
        const bool good = crc == ld32(fp + L);
        if (p.out_ok) p.out_ok[f] = good ? 1u : 0u;
        if (!good && p.nbad) atomicAdd(p.nbad, 1u);
    }
}

// BT: threads per workgroup. 1,024 (16 waves, 128 VGPRs) everywhere, or 512
// (8 waves, up to 256 VGPRs: deeper rings for short frames; an A/B that lost
// 10-24%, val_crc32_hip.hip VCRC_W8_PF).
template <int G, int PF, bool PAY, bool C0 = false, int BT = kBlock>
__global__ __launch_bounds__(BT) void k_frames(const FrameParams p)
{
    VCRC_STAMP(0);
    VCRC_KARG_EARLY("s"(p.consts), "s"(p.base), "s"(p.off), "s"(p.len), "s"(p.stride), "s"(p.flen), "s"(p.last_len),
                    "s"(p.n), "s"(p.seed0), "s"(p.seed_rest), "s"(gridDim.x));
    constexpr int kGroups = 64 / G;
    const int lane = threadIdx.x & 63;
    const SliceBases sb = slice_bases((uint32_t)(lane & 31) << 2);
    static_assert(BT == kBlock || !PAY, "payload states need the 1,024-thread pow-map fill");
    const uint64_t wave = ((uint64_t)blockIdx.x * BT + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * BT) >> 6;
    LdsImageT<BT> im;
    lds_tables_issue(p.consts, im);
    PowImage pim;
    if constexpr (PAY) lds_pow_issue(p.consts, 0, pim);
    // Descriptors of the next frame group are fetched while this one hashes.
    // (Loading the first group's descriptors branch-free before the blob, so
    // the prologue overlaps the first frame loads exactly, measured slower:
    // cfg2 -3%, 256-frame windows -9%, cfg3 -1%.)
    uint64_t fb = wave * kGroups, f = fb + (uint64_t)(lane / G), off = 0;
    uint32_t L = 0;
    if (f < p.n) frame_desc(p, f, off, L);
    // Every wave runs the first pass (lanes past the batch hash nothing): the
    // LDS fill and the barrier sit in its hash_frame call, after the frame
    // loads are issued. Peeled, so the LDS image's registers are dead in the
    // loop.
    const LdsImageT<BT> &cim = im;
    const PowImage &cpim = pim;
    group_pass<G, PF, PAY, C0>(p, f, off, L, fb, nwaves * kGroups, lane, sb, [&cim, &cpim] {
#ifndef VCRC_NO_LDS_FILL  // diagnostic A/B builds only (wrong CRCs): the prologue's share of small launches
        lds_tables_write(cim);
#endif
        if (PAY) lds_pow_write(cpim);
        __syncthreads();
        VCRC_STAMP(1);
    });
    if (!p.qhead) {
        while (fb < p.n) group_pass<G, PF, PAY, C0>(p, f, off, L, fb, nwaves * kGroups, lane, sb, [] {});
        if constexpr (kTailPieces<G, PF, PAY, BT>) {
            if (p.tail_n) tail_pieces<G, PF, C0>(p, lane, sb);
        }
        VCRC_STAMP(2);
        return;
    }
    // Dynamic tail: the first static_rounds group rounds are dealt as above,
    // the rest are pulled one group at a time from a queue, so waves that run
    // ahead (the oldest of a SIMD issue first) take more of the end. Short
    // groups split the queue into P interleaved partitions (group part + P * k
    // of the dynamic range), one head word each, keyed by blockIdx % P as in the
    // ragged kernel (every partition has a workgroup: P <= gridDim.x); long
    // groups keep one word, which evens the end out better. The last wave out
    // re-zeroes the heads for the next launch on this stream.
    const uint64_t dyn = (uint64_t)p.static_rounds * nwaves * kGroups;  // first frame of the queue
    while (fb < p.n && fb < dyn) group_pass<G, PF, PAY, C0>(p, f, off, L, fb, nwaves * kGroups, lane, sb, [] {});
    const uint32_t P = min(min(p.qparts, kDynParts), gridDim.x), part = blockIdx.x % P;
    // the lane id again from mbcnt: kept live from the entry, it was the one
    // value k_frames<16/32, 1> spilled to scratch (a scratch kernel's waves
    // launch later)
    // Short groups (P > 1 partitions), one group ahead: each group's dequeue is
    // issued when the previous group starts, and its descriptors are fetched once that group's round 0 is
    // hashed (the mid() hook, as the ragged kernel does), so a group's first
    // loads no longer wait for an atomic and then for its descriptors: two
    // dependent round trips per group, which short groups (1,100-B frames:
    // five rounds) could not hide (u1100d +3.0-3.7%, profiles/r03_ab_dyn_one_ahead_gated.log).
    // Every wave still ends on one failed dequeue, so the exit count below is
    // unchanged.
    const int ql = (int)__lane_id();
    if (P == 1u) {  // long groups: dequeue at each group's start (one ahead lost cfg4 2.5%, cfg3 0.7%: a wave
                    // then holds a reserved long group while others run dry)
        for (;;) {
            uint32_t k = 0;
#ifdef VCRC_DYN_PRECHECK
            if (ql == 0) {
                k = __hip_atomic_load(&p.qhead[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (dyn + (uint64_t)k * kGroups < p.n) k = atomicAdd(&p.qhead[0], 1u);
            }
#else
            if (ql == 0) k = atomicAdd(&p.qhead[0], 1u);
#endif
            k = __builtin_amdgcn_readfirstlane(k);
            const uint64_t gb = dyn + (uint64_t)k * kGroups;
            if (gb >= p.n) break;
            const uint64_t fd = gb + (uint64_t)(ql / G);
            uint64_t od = 0;
            uint32_t Ld = 0;
            if (fd < p.n) frame_desc(p, fd, od, Ld);
            hash_frame<G, PF, PAY, false, C0>(p, fd, fd < p.n, od, Ld, ql % G, sb, G, [] {});
        }
    }
    uint32_t k = 0;
    if (P > 1u && ql == 0) k = atomicAdd(&p.qhead[part * 16u], 1u);
    // (Runs of 4 or 16 consecutive groups per partition, as the ragged kernel
    // deals one-bucket batches, measured neutral here: -0.4 to +0.4%;
    // profiles/r04_ab_dyn_tail_runs.log.)
    uint64_t gb = P == 1u ? p.n : dyn + ((uint64_t)part + (uint64_t)P * __builtin_amdgcn_readfirstlane(k)) * kGroups;
    uint64_t fd = gb + (uint64_t)(ql / G), od = 0;
    uint32_t Ld = 0;
    if (fd < p.n) frame_desc(p, fd, od, Ld);
    while (gb < p.n) {
        uint32_t kn = 0;
        if (ql == 0) kn = atomicAdd(&p.qhead[part * 16u], 1u);
        uint64_t gb_n = 0, fd_n = 0, od_n = 0;
        uint32_t Ld_n = 0;
        hash_frame<G, PF, PAY, false, C0>(p, fd, fd < p.n, od, Ld, ql % G, sb, G, [] {}, [&] {
            gb_n = dyn + ((uint64_t)part + (uint64_t)P * __builtin_amdgcn_readfirstlane(kn)) * kGroups;
            fd_n = gb_n + (uint64_t)(ql / G);
            if (fd_n < p.n) frame_desc(p, fd_n, od_n, Ld_n);
        });
        gb = gb_n;
        fd = fd_n;
        od = od_n;
        Ld = Ld_n;
    }
    if constexpr (kTailPieces<G, PF, PAY, BT>) {
        if (p.tail_n) tail_pieces<G, PF, C0>(p, ql, sb);
    }
    VCRC_STAMP(2);
    // Exits are counted per workgroup, after a barrier: one atomic per CU. One
    // per wave (4,096 on one word, serialised at its atomic unit) added tens of
    // microseconds to the end of short launches, where the waves all finish
    // together.
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t out = atomicAdd(&p.qhead[kDynParts * 16u], 1u);
        if (out == gridDim.x - 1u) {  // every wave is past its last dequeue
            for (uint32_t i = 0; i < P; i++) atomicExch(&p.qhead[i * 16u], 0u);
            atomicExch(&p.qhead[kDynParts * 16u], 0u);
        }
    }
}

// ---- ragged path ------------------------------------------------------------
// Frames are counting-sorted by length bucket, longest first, so the 64/G
// frames a wave hashes together need the same number of rounds, and the
// sorted order is cut into geometry classes (contiguous bucket ranges). A
// bucket is one round of its class (G * 64 bytes): within a bucket every
// frame has R = ceil(L / (64 G)) rounds, so no lane idles behind a longer
// neighbour (round 0 is partial, and nearly free: s4_words_from).
//   class 0 (G=2,  128 B rounds): L in [0, 1024)       buckets 0..7
//   class 1 (G=4,  256 B rounds): L in [1024, 8192)    buckets 8..36
//   class 2 (G=8,  512 B rounds): L in [8192, 49152)   buckets 37..117
//   class 3 (G=16, 1 KiB rounds): L in [49152, 65536]  buckets 118..134, longer 135
// (Buckets of two rounds for classes 1 and 2, so that an item's frames lie
// closer together in memory at the price of one idle round for some lanes,
// measured neutral: cfg5 0 / -0.2%, class-2 mix +0.5%;
// profiles/r04_ab_ragged_two_round_buckets.log.)
constexpr int kBuckets = 136;
__host__ __device__ inline int length_bucket(uint32_t L)
{
    if (L < 1024u) return L <= 128u ? 0 : (int)((L - 1u) / 128u);
    if (L < 8192u) return 8 + (int)((L - 1u) / 256u) - 3;
    if (L < 49152u) return 37 + (int)((L - 1u) / 512u) - 15;
    const uint32_t r = (L - 1u) / 1024u;  // 47.. for L >= 49152
    return r < 64u ? 118 + (int)r - 47 : kBuckets - 1;
}
__host__ __device__ inline int bucket_class(int b) { return b < 8 ? 0 : b < 37 ? 1 : b < 118 ? 2 : 3; }
constexpr int kClassFirstBucket[kClasses + 1] = {0, 8, 37, 118, kBuckets};

// A wave's lanes that all hold the same bucket (uniform batches) reserve
// their slots with one LDS atomic; mixed waves use one atomic per lane.
// Returns this lane's slot offset from cnt[b] (v: the lane holds an element).
__device__ __forceinline__ uint32_t bucket_slot(uint32_t *cnt, int b, bool v)
{
    const int lane = threadIdx.x & 63;
    const uint64_t act = __ballot(v);
    if (act == 0) return 0;
    const int leader = __ffsll((long long)act) - 1;
    const int b0 = __shfl(b, leader);
    if (__ballot(v && b != b0) == 0) {
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&cnt[b0], (uint32_t)__popcll(act));
        base = __shfl(base, leader);
        return base + (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
    }
    return v ? atomicAdd(&cnt[b], 1u) : 0u;
}

// Lengths of a binning workgroup's slice are read kBinBatch per thread before
// any is used: one memory latency per batch instead of one per 256 frames
// (a dependent load -> atomic loop made each binning pass ~8 us).
constexpr int kBinThreads = 256, kBinBatch = 8;

template <typename F>
__device__ __forceinline__ void for_each_bucket(const uint32_t *len, uint64_t lo, uint64_t hi, F &&f)
{
    for (uint64_t base = lo; base < hi; base += (uint64_t)kBinThreads * kBinBatch) {
        uint32_t lv[kBinBatch];
#pragma unroll
        for (int k = 0; k < kBinBatch; k++) {
            const uint64_t i = base + (uint64_t)k * kBinThreads + threadIdx.x;
            lv[k] = i < hi ? len[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < kBinBatch; k++) {
            const uint64_t i = base + (uint64_t)k * kBinThreads + threadIdx.x;
            if (base + (uint64_t)k * kBinThreads >= hi) break;  // workgroup-uniform
            f(i, i < hi, length_bucket(lv[k]));
        }
    }
}

// Pass 1: per-workgroup bucket counts; each workgroup reserves its slice of
// every non-empty bucket with one atomic (offsets within the bucket).
// gcount must be zero on entry (k_frames_ragged re-zeroes it for the next
// batch once pass 2 has consumed it).
__global__ __launch_bounds__(kBinThreads) void k_bin_count(const uint32_t *len, uint32_t n, uint32_t chunk,
                                                           uint32_t *gcount, uint32_t *blockoff)
{
    __shared__ uint32_t cnt[kBuckets];
    for (int b = threadIdx.x; b < kBuckets; b += blockDim.x) cnt[b] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = min((uint64_t)n, lo + chunk);
    for_each_bucket(len, lo, hi, [&](uint64_t, bool v, int b) { (void)bucket_slot(cnt, v ? b : 0, v); });
    __syncthreads();
    for (int b = threadIdx.x; b < kBuckets; b += blockDim.x)
        blockoff[(size_t)blockIdx.x * kBuckets + b] = cnt[b] ? atomicAdd(&gcount[b], cnt[b]) : 0u;
}

// Bucket starts in sorted order (longest bucket first), by a prefix scan in
// one wave, into bstart (LDS). Returns (in every lane) whether one bucket
// holds all n frames.
__device__ __forceinline__ bool bin_starts_wave(const uint32_t *gcount, uint32_t *bstart, uint32_t n)
{
    constexpr int kPer = (kBuckets + 63) / 64;
    const int l = threadIdx.x & 63;
    uint32_t c[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int r = l * kPer + k;  // rank r = bucket kBuckets-1-r
        c[k] = r < kBuckets ? gcount[kBuckets - 1 - r] : 0u;
        sum += c[k];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (l >= o) inc += t;
    }
    uint32_t pos = inc - sum;
    bool one = false;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const int r = l * kPer + k;
        if (r < kBuckets) bstart[kBuckets - 1 - r] = pos;
        pos += c[k];
        one = one || c[k] == n;
    }
    return __ballot(one) != 0;
}

// Pass 2: the plan (every workgroup scans the 136 bucket counts itself;
// workgroup 0 also writes the class table and zeroes the work-queue heads),
// then the frame indices are scattered into sorted order (order within a
// bucket is unspecified; every output is written at its frame's own index).
// When one bucket holds the whole batch (uniform lengths sent without a
// length hint) any order is sorted: nothing is scattered, and ctab[13] tells
// k_frames_ragged to take frame i at sorted position i.
__global__ __launch_bounds__(kBinThreads) void k_bin_scatter(const uint32_t *len, uint32_t n, uint32_t chunk,
                                                             const uint32_t *gcount, const uint32_t *blockoff,
                                                             uint32_t *ctab, uint32_t *heads, uint32_t *order)
{
    __shared__ uint32_t cur[kBuckets];
    __shared__ uint32_t s_one;
    if (threadIdx.x < 64) {
        const bool one = bin_starts_wave(gcount, cur, n);
        if (threadIdx.x == 0) s_one = one ? 1u : 0u;
    }
    __syncthreads();
    const bool one = s_one != 0;
    if (blockIdx.x == 0) {
        for (uint32_t i = threadIdx.x; i < kQueueParts * 16u; i += blockDim.x) heads[i] = 0u;
        if (threadIdx.x == 0) {
            // class cc = the sorted range from its longest bucket's start to the
            // next shorter class's (class 0 ends at n: every frame has a bucket);
            // items are numbered longest class first
            uint32_t item = 0;
            for (int cc = kClasses - 1; cc >= 0; cc--) {
                const uint32_t cstart = cur[kClassFirstBucket[cc + 1] - 1];
                const uint32_t cend = cc > 0 ? cur[kClassFirstBucket[cc] - 1] : n;
                const uint32_t ccount = cend - cstart, per = 64u / (uint32_t)class_lanes(cc);
                ctab[8 + cc] = item;
                item += (ccount + per - 1) / per;
                ctab[cc] = ccount ? cstart : 0u;
                ctab[4 + cc] = ccount;
            }
            ctab[12] = item;  // total items
            ctab[13] = one ? 1u : 0u;
        }
    }
    if (one) return;  // workgroup-uniform
    __syncthreads();
    for (int b = threadIdx.x; b < kBuckets; b += blockDim.x) cur[b] += blockoff[(size_t)blockIdx.x * kBuckets + b];
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = min((uint64_t)n, lo + chunk);
    for_each_bucket(len, lo, hi, [&](uint64_t i, bool v, int b) {
        const uint32_t slot = bucket_slot(cur, v ? b : 0, v);
        if (v) order[slot] = (uint32_t)i;
    });
}

// Item `it` of the ragged plan: its class and sorted-order range.
struct Item {
    int c;
    uint32_t first, end;
};

__device__ __forceinline__ Item ragged_item(const uint32_t *ctab, uint32_t it)
{
    // items are numbered class 3 (longest) first
    const int c = it >= ctab[8 + 2] ? (it >= ctab[8 + 1] ? (it >= ctab[8 + 0] ? 0 : 1) : 2) : 3;
    const uint32_t per = 64u / (uint32_t)(c == 0 ? class_lanes(0) : c == 1 ? class_lanes(1) : c == 2 ? class_lanes(2) : class_lanes(3));
    const uint32_t cstart = c == 0 ? ctab[0] : c == 1 ? ctab[1] : c == 2 ? ctab[2] : ctab[3];
    const uint32_t ccount = c == 0 ? ctab[4] : c == 1 ? ctab[5] : c == 2 ? ctab[6] : ctab[7];
    const uint32_t istart = c == 0 ? ctab[8] : c == 1 ? ctab[9] : c == 2 ? ctab[10] : ctab[11];
    return Item{c, cstart + (it - istart) * per, cstart + ccount};
}

// This lane's frame of an item (lane / G-th frame) and its descriptor.
__device__ __forceinline__ void item_frame(const FrameParams &p, const Item &t, int lane, uint64_t &f, bool &active,
                                           uint64_t &off, uint32_t &L, bool ident)
{
    const int G = class_lanes(t.c == 0 ? 0 : t.c == 1 ? 1 : t.c == 2 ? 2 : 3);
    const uint32_t i = t.first + (uint32_t)(lane / G);
    active = i < t.end;
    f = active ? (ident ? i : p.order[i]) : 0u;  // ident: one bucket, sorted order = batch order
    off = 0;
    L = 0;
    if (active) frame_desc(p, f, off, L);
}

// Ragged batches: persistent grid; waves pull items (64/G frames of one
// class, longest first) from a work queue, so the launch ends about one item
// after the bytes run out (longest-processing-time-first: a static cyclic deal
// gave wave 0 the longest item of every round). The queue is split into
// P <= kQueueParts (64) interleaved partitions (item = part + P * k), one head
// word each, keyed by blockIdx % P: a head is pulled by the 64 waves of four
// workgroups on one XCD (one word saturates near 88 dequeues/us; 8 heads, one
// per XCD, measured 1.5-3% slower on every mix and one head up to 2.8x).
// Every partition has at least one workgroup (P <= gridDim.x), so every item
// is hashed exactly once whatever the placement. A wave's first two items are
// static; item i + 2 is dequeued while item i hashes and item i + 1's
// descriptors load, so neither latency is exposed. All four classes' gap maps
// stay in LDS: waves never synchronise after the prologue.
template <int PF, bool PAY>
__global__ __launch_bounds__(kBlock) void k_frames_ragged(const FrameParams p)
{
    VCRC_STAMP(0);
    if (blockIdx.x == 0 && threadIdx.x < kBuckets) p.bin_counts[threadIdx.x] = 0u;  // consumed by k_bin_scatter
    // The first item's frame loads wait on three dependent reads (plan, sorted
    // order, descriptors), so the LDS fill is not overlapped with them here:
    // its registers would be live through the loop (a spill at 128 VGPRs).
#ifndef VCRC_NO_LDS_FILL  // diagnostic A/B builds only (wrong CRCs): the upper bound of overlapping the fill
    build_lds_tables(p.consts);
#endif
    if (PAY) lds_pow_maps(p.consts);
    __syncthreads();
    VCRC_STAMP(1);
    const uint32_t *ctab = p.plan;
    const uint32_t items = ctab[12];
    const bool ident = ctab[13] != 0;
    const int lane = threadIdx.x & 63;
    const SliceBases sb = slice_bases((uint32_t)(lane & 31) << 2);
    const uint32_t P = min(kQueueParts, gridDim.x);
    const uint32_t part = blockIdx.x % P;
    const uint32_t nwp = ((gridDim.x - part + P - 1) / P) * kWavesPerBlock;  // waves of this partition
    uint32_t *head = p.heads + part * 16u;  // 64 B apart
    const uint32_t k0 = (blockIdx.x / P) * kWavesPerBlock + (threadIdx.x >> 6);
    // (Dealing the first half or three quarters of every wave's items
    // statically, as the uniform kernel does, lost on mixes: cfg5 -1.2% and
    // -3.1%, class-2 mix -0.7% and -2%; uniform 16,400-B frames +1.3% and
    // +0.7%; profiles/r04_ab_ragged_static_prefix.log.)
    // Partition part's idx-th item. A one-bucket batch (uniform lengths without
    // a length hint, identity order) deals its items to the partitions in runs
    // of 4 consecutive items, so a partition's waves (one XCD) hash neighbouring
    // frames: u16400 +2.8%, u600 +1.4% through this path. Mixes keep runs of 1:
    // there runs of 4 measured -0.1 to -0.4% and runs of 16 -1.5 to -2.6%
    // (profiles/r04_ab_ragged_item_runs.log).
    const uint32_t lgch = ident ? 2u : 0u;
    auto item_of = [&](uint32_t idx) {
        return (((idx >> lgch) * P + part) << lgch) + (idx & ((1u << lgch) - 1u));
    };
    uint32_t it = item_of(k0);
    if (it >= items) return;
    Item cur = ragged_item(ctab, it);
    uint64_t f, off;
    uint32_t L;
    bool active;
    item_frame(p, cur, lane, f, active, off, L, ident);
    // One item ahead: the next item is dequeued when this one starts, and its
    // descriptors are fetched once this one's round 0 is hashed (the atomic
    // has long returned). When the queue runs dry each wave has one item left
    // to hash, not two (a two-ahead queue left up to two items per wave).
    while (true) {
        uint32_t k_n = 0;
        if (lane == 0) k_n = atomicAdd(head, 1u);
        Item nx{0, 0, 0};
        uint32_t it_n = items;
        uint64_t f_n = 0, off_n = 0;
        uint32_t L_n = 0;
        bool active_n = false;
        const int G = class_lanes(cur.c);
        VCRC_LAST_ITEM(cur.c, L);
        // (One compile-time-G hash_frame instance per class instead, switched per
        // item, spilled 6-8 VGPRs and ran 1.5-16% slower: cfg5 -1.5%, class-2 mix
        // -2.4%, 1,100-B frames -16%; with the unit loads -0.3 to -7%;
        // profiles/r04_ab_ragged_compile_time_lanes.log.)
        hash_frame<0, PF, PAY, false>(p, f, active, off, L, lane & (G - 1), sb, G, [] {}, [&] {
            it_n = item_of(__builtin_amdgcn_readfirstlane(k_n) + nwp);
            if (it_n < items) {
                nx = ragged_item(ctab, it_n);
                item_frame(p, nx, lane, f_n, active_n, off_n, L_n, ident);
            }
        });
        if (it_n >= items) {
            VCRC_STAMP(2);
            break;
        }
        it = it_n;
        cur = nx;
        f = f_n;
        off = off_n;
        L = L_n;
        active = active_n;
    }
}

// ---- K1/K2 for small batches of long frames: one workgroup per frame --------
// A batch of a few long frames leaves most of the machine idle even at one
// wave per frame, and each wave walks its frame one 4 KiB round after
// another (256 x 64 KiB: 16 rounds, ~40 us). Here a workgroup takes a whole
// frame: the frame is cut into chunks of W = 2^k0 bytes anchored at its end
// (only chunk 0 can be short; it carries the seed), the 16 waves hash 16
// chunks at a time as k_region's waves do (hash_frame at 64 lanes), wave 0
// folds their registers (4-level shuffle tree, LDS maps "advance W * 2^j"),
// and a frame longer than 16 W folds its 16-chunk groups front to back
// ("advance 16 W"). A padded chunk holds zeros, which are inert. Lane 15 of
// wave 0 writes the trailer CRC and, on verify, compares the stored LE32; it
// also hashes the frame's first 8 bytes for header_crc (chunk 0 can be
// shorter than the header). Uniform and descriptor batches alike (any length
// per frame).
__global__ __launch_bounds__(kBlock) void k_frames_split(const FrameParams p, const uint32_t k0)
{
    __shared__ uint32_t s_fold[kWavesPerBlock];
    LdsImage im;
    lds_tables_issue(p.consts, im);
    PowImage pim;
    lds_pow_issue(p.consts, k0, pim);
    lds_tables_write(im);
    lds_pow_write(pim);
    __syncthreads();
    const int lane = threadIdx.x & 63, wi = threadIdx.x >> 6;
    const SliceBases sb = slice_bases((uint32_t)(lane & 31) << 2);
    const uint64_t W = (uint64_t)1 << k0;
    for (uint64_t f = blockIdx.x; f < p.n; f += gridDim.x) {
        uint64_t off = 0;
        uint32_t L = 0;
        frame_desc(p, f, off, L);
        const uint64_t C = L ? ((uint64_t)L + W - 1) >> k0 : 1u;  // chunks
        const uint64_t groups = (C + kWavesPerBlock - 1) / kWavesPerBlock;
        FrameParams q{};
        q.base = p.base;
        q.n = (uint32_t)C;
        q.seed0 = f == 0 ? p.seed0 : p.seed_rest;
        q.seed_rest = 0;
        q.xorout = p.xorout;  // finishes header_crc; the chunk registers come back raw (no out_crc)
        q.consts = p.consts;
        uint32_t facc = 0;  // wave 0, lane 15: the frame's register over the groups so far
        for (uint64_t g = 0; g < groups; g++) {
            // group g: chunks C - (groups - g) * 16 + wi, the first group padded at the front
            const int64_t cp = (int64_t)C - (int64_t)(groups - g) * kWavesPerBlock + wi;
            const bool real = cp >= 0;
            const uint64_t c = real ? (uint64_t)cp : 0u;
            const uint64_t hi = (uint64_t)L - (C - 1u - c) * W;
            const uint64_t lo = hi > W ? hi - W : 0u;
            const uint32_t st = hash_frame<64, 1, false, true>(q, c, real, off + lo, real ? (uint32_t)(hi - lo) : 0u,
                                                             lane, sb, 64, [] {});
            if (lane == 63) s_fold[wi] = real ? st : 0u;
            __syncthreads();
            if (wi == 0) {
                uint32_t v = lane < kWavesPerBlock ? s_fold[lane] : 0u;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t other = __shfl_xor(v, 1 << j);
                    const bool right = (lane >> j) & 1;
                    const uint32_t left = right ? other : v;
                    v = map_apply(left, pow_map(j)) ^ (right ? v : other);
                }
                facc = g ? map_apply(facc, pow_map(4)) ^ v : v;  // a later group is 16 W bytes long
            }
            __syncthreads();  // s_fold is reused by the next group
        }
        if (wi == 0 && lane == kWavesPerBlock - 1) {
            const uint32_t crc = facc ^ p.xorout;
            if (p.out_crc) p.out_crc[f] = crc;
            if (p.out_hdr) {
                gu8 *fp = gptr(p.base) + off;
                uint32_t h = q.seed0;
                if (L >= 8) {
                    h = s4_step(h, ld32(fp), sb);
                    h = s4_step(h, ld32(fp + 4), sb);
                } else {
                    for (uint32_t i = 0; i < L; i++) h = byte_step(h, fp[i], sb);
                }
                p.out_hdr[f] = h ^ p.xorout;
            }
            if (p.verify) {
                const bool good = crc == ld32(gptr(p.base) + off + L);
                if (p.out_ok) p.out_ok[f] = good ? 1u : 0u;
                if (!good && p.nbad) atomicAdd(p.nbad, 1u);
            }
        }
    }
}

// ---- K4: region CRC, one launch --------------------------------------------
// A long window of len bytes is cut into C chunks of W = 2^k0 bytes (k0 >= 12)
// anchored at the window END: chunk c covers [len - (C-c) W, len - (C-c-1) W),
// so only chunk 0 can be short. One wave hashes one chunk (hash_frame at 64
// lanes; chunk 0 carries state_in, the others start from zero), so every
// combine below advances a left state over whole right subtrees of full
// chunks, W * 2^j bytes: LDS maps "advance 2^(k0+j) bytes" from the constant
// blob, nothing built at run time. Chunks are numbered in a padded space of
// 16 * nwg with the real ones at the end (zero states in front are inert).
//   workgroup b: its 16 chunk states -> one state S_b (4-level shuffle tree);
//   S_b advanced over the (nwg - 1 - b) * 16 W bytes after it is atomically
//   XORed into an accumulator (the fold is linear); the last workgroup to
//   count in (device-scope atomics, each returned before the next is issued)
//   takes the accumulator, writes the result and re-zeroes the scratch.
// Replaces a chunk-state kernel + a single-workgroup combine launch that
// built its maps with gf2_mul on every call (26 us for an 8 MiB window).
struct RegionParams {
    const uint8_t *base;
    uint64_t len;
    uint64_t W;               // chunk bytes, 2^k0
    uint32_t C;               // chunks
    uint32_t nwg;             // workgroups = ceil(C / 16)
    uint32_t k0;              // log2(W)
    uint32_t seed;            // state_in (unless seed_dev)
    const uint32_t *seed_dev; // state_in read from device memory (chained pieces), nullable
    uint32_t *out;            // raw register of the window
    uint32_t *acc;            // scratch: acc[0] accumulator, acc[16] arrival count (zero on entry, re-zeroed)
    const uint32_t *consts;
};
constexpr uint32_t kRegionMaxChunks = 4096;  // nwg <= 256: 8 levels of workgroup fold

__global__ __launch_bounds__(kBlock) void k_region(const RegionParams rp)
{
    __shared__ uint32_t s_fold[kWavesPerBlock];
    VCRC_STAMP(0);
    VCRC_KARG_EARLY("s"(rp.consts), "s"(rp.base), "s"(rp.len), "s"(rp.W), "s"(rp.C), "s"(rp.nwg), "s"(rp.k0),
                    "s"(rp.seed), "s"(rp.seed_dev));
    LdsImage im;
    lds_tables_issue(rp.consts, im);
    PowImage pim;
    lds_pow_issue(rp.consts, rp.k0, pim);
    const int lane = threadIdx.x & 63, wi = threadIdx.x >> 6;
    const SliceBases sb = slice_bases((uint32_t)(lane & 31) << 2);
    const uint32_t pad = rp.nwg * kWavesPerBlock - rp.C;
    const uint32_t cp = blockIdx.x * kWavesPerBlock + (uint32_t)wi;  // padded chunk index
    const bool real = cp >= pad;
    const uint32_t c = real ? cp - pad : 0u;
    const uint64_t hi = rp.len - (uint64_t)(rp.C - 1u - c) * rp.W;
    const uint64_t lo = hi > rp.W ? hi - rp.W : 0u;
    FrameParams p{};
    p.base = rp.base;
    p.n = rp.C;
    p.seed0 = rp.seed_dev ? *rp.seed_dev : rp.seed;
    p.seed_rest = 0;
    p.consts = rp.consts;
    const LdsImage &cim = im;
    const PowImage &cpim = pim;
    const uint32_t st = hash_frame<64, 1, false, true>(p, c, real, lo, real ? (uint32_t)(hi - lo) : 0u, lane, sb, 64,
                                                 [&cim, &cpim] {
                                                     VCRC_STAMP(1);
                                                     lds_tables_write(cim);
                                                     lds_pow_write(cpim);
                                                     __syncthreads();
                                                     VCRC_STAMP(2);
                                                 });
    VCRC_STAMP(3);
#ifdef VCRC_REGION_HASHONLY  // diagnostic A/B builds only
    if (lane == 63 && wi == 0) *rp.out = st;
    return;
#endif
    if (lane == 63) s_fold[wi] = real ? st : 0u;
    __syncthreads();
    if (wi != 0) return;
    // 16 chunk states -> S_b: level j advances the left half by W * 2^j
    uint32_t v = lane < kWavesPerBlock ? s_fold[lane] : 0u;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t other = __shfl_xor(v, 1 << j);
        const bool right = (lane >> j) & 1;
        const uint32_t left = right ? other : v;
        v = map_apply(left, pow_map(j)) ^ (right ? v : other);
    }
    if (lane != kWavesPerBlock - 1) return;
    // advance over the (nwg - 1 - b) later workgroups: 16 W * 2^i per set bit i
    const uint32_t d = rp.nwg - 1u - blockIdx.x;
    for (int i = 0; i < 12; i++)
        if ((d >> i) & 1u) v = map_apply(v, pow_map(4 + i));
#ifdef VCRC_REGION_NOATOMIC  // diagnostic A/B builds only
    *rp.out = v;
    return;
#endif
    const uint32_t old = atomicXor(&rp.acc[0], v);
    // the XOR has been performed (its value returned) before this workgroup counts in
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");
    const uint32_t arrived = atomicAdd(&rp.acc[16], 1u);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(arrived) : "memory");
    if (arrived == rp.nwg - 1u) {
        const uint32_t total = atomicExch(&rp.acc[0], 0u);
        atomicExch(&rp.acc[16], 0u);
        *rp.out = total;
    }
}

}  // namespace vcrc
