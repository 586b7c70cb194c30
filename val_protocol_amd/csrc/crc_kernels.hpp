// crc_kernels.hpp -- the CRC-32 kernels (gfx950). Included by val_crc32_hip.hip.
//
// k_frames<G, PF>      K1/K2/K3: per-frame trailer CRC, header_crc, verify;
//                      persistent grid, G lanes per frame, uniform geometry.
// k_bin_* + k_frames_grouped<PF>
//                      K5: ragged descriptor batches. Frames are binned by
//                      length class on the device (stable), each class gets its
//                      measured lanes-per-frame, and workgroups are planned in
//                      proportion to each class's bytes. No host round trip.
// k_combine            K4 stage 2: fold per-chunk raw states of a long region.
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
__host__ __device__ constexpr int class_lanes(int c) { return c == 0 ? 2 : c == 1 ? 4 : c == 2 ? 8 : 16; }
__host__ __device__ inline int length_class(uint32_t L)
{
    return L < 1024u ? 0 : L < 8192u ? 1 : L < 49152u ? 2 : 3;
}

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
    const uint32_t *plan;    // grouped mode: {class, begin, end} per workgroup
    uint32_t xtab[4];        // x^(8(k+1)): slice table T_k
    uint32_t xgap[kClasses]; // x^(8 (G-1) 64) per geometry (index 0 in uniform mode)
    uint32_t tree[kMaxTree][32];  // columns of "advance 64 * 2^j bytes"
};

// Words of a lane's round-0 unit u: u > 0 a full unit; u == 0 the front-padded
// first unit, assembled word by word with the seed in frame bytes 0..3;
// u < 0 nothing. L < 4 frames take the byte path (tiny).
__device__ __forceinline__ void load_unit0(uint32_t (&w)[kWords], int u, const uint8_t *fp, uint32_t L, uint32_t pad,
                                           uint32_t seed, bool &tiny)
{
    tiny = false;
    if (u > 0) {
        const uint8_t *up = fp + (uint64_t)u * kUnit - pad;
#pragma unroll
        for (int q = 0; q < kWords / 4; q++) {
            const u32x4u v = *reinterpret_cast<const u32x4u *>(up + 16 * q);
            w[4 * q + 0] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
        // Seed bytes that did not fit in a unit 0 holding < 4 real bytes.
        if (u == 1 && pad > kUnit - 4) w[0] ^= seed >> (8 * (kUnit - pad));
    } else if (u == 0 && L >= 4) {
#pragma unroll
        for (int i = 0; i < kWords; i++) {
            const int q = 4 * i - (int)pad;  // frame offset of this word
            uint32_t x = 0;
            if (q >= 0) {
                x = ld32(fp + q);
                if (q < 4) x ^= seed >> (8 * q);
            } else if (q > -4) {
                x = (ld32(fp) ^ seed) << (8 * (-q));
            }
            w[i] = x;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kWords; i++) w[i] = 0;
        tiny = (u == 0);
    }
}

__device__ __forceinline__ void load_full(uint32_t (&w)[kWords], const uint8_t *up)
{
#pragma unroll
    for (int q = 0; q < kWords / 4; q++) {
        const u32x4u v = *reinterpret_cast<const u32x4u *>(up + 16 * q);
        w[4 * q + 0] = v.x;
        w[4 * q + 1] = v.y;
        w[4 * q + 2] = v.z;
        w[4 * q + 3] = v.w;
    }
}

// Hash frame f with the G lanes of this lane's group (g = 0..G-1). All 64
// lanes of the wave must call this together (the merge tree shuffles).
template <int G, bool PF>
__device__ __forceinline__ void hash_frame(const FrameParams &p, uint64_t f, bool active, int g, uint32_t lo4,
                                           const SliceBases &sb)
{
    uint64_t off = 0;
    uint32_t L = 0;
    if (active) {
        if (p.off) {
            off = p.off[f];
            L = p.len[f];
        } else {
            off = f * p.stride;
            L = (f + 1 == p.n) ? p.last_len : p.flen;
        }
    }
    const uint8_t *fp = p.base + off;
    const uint32_t seed = (f == 0) ? p.seed0 : p.seed_rest;
    const uint32_t U = L ? (L + kUnit - 1) / kUnit : 1u;
    const uint32_t R = active ? (U + G - 1) / G : 0u;
    const uint32_t pad = U * kUnit - L;
    const int u0 = (int)U - G * (int)R + g;  // this lane's unit in round 0
    const uint8_t *up = fp + ((int64_t)u0 + G) * kUnit - pad;  // its unit in round 1
    uint32_t nxt[kWords];
    if (PF && R > 1) load_full(nxt, up);
    uint32_t acc = 0;
    if (R > 0) {
        // Round 0 alone can hold unit 0 (padding, seed, tiny frames) or no
        // unit; the register is still zero, so no gap step.
        uint32_t w[kWords];
        bool tiny;
        load_unit0(w, u0, fp, L, pad, seed, tiny);
#pragma unroll
        for (int i = 0; i < kWords; i++) acc = s4_step(acc, w[i], sb);
        if (tiny) {  // L < 4: state of the few bytes straight from the seed
            acc = seed;
            for (uint32_t i = 0; i < L; i++) acc = byte_step(acc, fp[i], sb);
        }
    }
    // Steady state: every lane has a full unit (u >= 1) in rounds 1..R-1.
    for (uint32_t k = 1; k < R; k++, up += (uint64_t)G * kUnit) {
        uint32_t w[kWords];
        if (PF) {
#pragma unroll
            for (int i = 0; i < kWords; i++) w[i] = nxt[i];
            if (k + 1 < R) load_full(nxt, up + (uint64_t)G * kUnit);
        } else {
            load_full(w, up);
        }
        // Seed bytes past a unit 0 with < 4 real bytes land in unit 1 (lane 0, k == 1).
        if (k == 1 && g == 0 && pad > kUnit - 4 && (int)U - G * (int)(R - 1) == 1) w[0] ^= seed >> (8 * (kUnit - pad));
        if (G > 1) acc = gap_step(acc, lo4);
#pragma unroll
        for (int i = 0; i < kWords; i++) acc = s4_step(acc, w[i], sb);
    }
    // Merge: level j joins blocks of 2^j lanes, the left one advanced by 64 * 2^j bytes.
#pragma unroll
    for (int j = 0; (1 << j) < G; j++) {
        const uint32_t other = __shfl_xor(acc, 1 << j);
        const bool right = (g >> j) & 1;
        acc = bitmatrix_apply(right ? other : acc, p.tree[j]) ^ (right ? acc : other);
    }
    if (active && g == G - 1) {
        const uint32_t crc = acc ^ p.xorout;
        if (p.out_crc) p.out_crc[f] = crc;
        if (p.verify) {
            const bool good = (crc == ld32(fp + L));
            if (p.out_ok) p.out_ok[f] = good ? 1u : 0u;
            if (!good && p.nbad) atomicAdd(p.nbad, 1u);
        }
    }
    if (active && g == 0 && p.out_hdr) {
        uint32_t h = seed;
        if (L >= 8) {
            h = s4_step(h, ld32(fp), sb);
            h = s4_step(h, ld32(fp + 4), sb);
        } else {
            for (uint32_t i = 0; i < L; i++) h = byte_step(h, fp[i], sb);
        }
        p.out_hdr[f] = h ^ p.xorout;
    }
}

// Uniform geometry: persistent grid, each wave hashes 64/G frames per step.
template <int G, bool PF>
__global__ __launch_bounds__(kBlock) void k_frames(const FrameParams p)
{
    build_tables(p.xtab, p.xgap[0], G > 1);
    constexpr int kGroups = 64 / G;
    const int lane = threadIdx.x & 63;
    const uint32_t lo4 = (uint32_t)(lane & 31) << 2;
    const SliceBases sb = slice_bases(lo4);
    const uint64_t wave = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * kBlock) >> 6;
    for (uint64_t fb = wave * kGroups; fb < p.n; fb += nwaves * kGroups) {
        const uint64_t f = fb + (uint64_t)(lane / G);
        hash_frame<G, PF>(p, f, f < p.n, lane % G, lo4, sb);
    }
}

// ---- ragged path ------------------------------------------------------------
// Pass 1: per-workgroup counts and bytes of each length class.
__global__ __launch_bounds__(256) void k_bin_count(const uint32_t *len, uint32_t n, uint32_t chunk, uint32_t *hist,
                                                   unsigned long long *hbytes)
{
    __shared__ uint32_t cnt[kClasses];
    __shared__ unsigned long long bytes[kClasses];
    if (threadIdx.x < kClasses) {
        cnt[threadIdx.x] = 0;
        bytes[threadIdx.x] = 0;
    }
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = min((uint64_t)n, lo + chunk);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const uint32_t L = len[i];
        const int c = length_class(L);
        atomicAdd(&cnt[c], 1u);
        atomicAdd(&bytes[c], (unsigned long long)L);
    }
    __syncthreads();
    if (threadIdx.x < kClasses) {
        hist[blockIdx.x * kClasses + threadIdx.x] = cnt[threadIdx.x];
        hbytes[blockIdx.x * kClasses + threadIdx.x] = bytes[threadIdx.x];
    }
}

// Pass 2 (one workgroup): class starts, per-(block, class) scatter bases and
// the workgroup plan {class, begin, end} (workgroups per class in proportion
// to its bytes, >= 1 for a non-empty class; unused plan entries are empty).
__global__ __launch_bounds__(64) void k_bin_plan(const uint32_t *hist, const unsigned long long *hbytes, uint32_t nbin,
                                                 uint32_t *base, uint32_t *plan, uint32_t nplan)
{
    __shared__ uint32_t count[kClasses], start[kClasses], nblk[kClasses];
    __shared__ unsigned long long cbytes[kClasses];
    const int c = threadIdx.x;
    if (c < kClasses) {
        uint32_t s = 0;
        unsigned long long b = 0;
        for (uint32_t k = 0; k < nbin; k++) {
            base[k * kClasses + c] = s;  // relative to the class start, fixed below
            s += hist[k * kClasses + c];
            b += hbytes[k * kClasses + c];
        }
        count[c] = s;
        cbytes[c] = b;
    }
    __syncthreads();
    if (c == 0) {
        unsigned long long total = 0;
        uint32_t s = 0;
        for (int k = 0; k < kClasses; k++) {
            start[k] = s;
            s += count[k];
            total += cbytes[k];
        }
        const uint32_t budget = nplan - kClasses;  // room for the ">= 1" rounding
        for (int k = 0; k < kClasses; k++) {
            uint32_t nb = 0;
            if (count[k]) {
                nb = total ? (uint32_t)((double)budget * (double)cbytes[k] / (double)total) : 1u;
                if (nb < 1) nb = 1;
                if (nb > count[k]) nb = count[k];
            }
            nblk[k] = nb;
        }
    }
    __syncthreads();
    if (c < kClasses) {
        for (uint32_t k = 0; k < nbin; k++) base[k * kClasses + c] += start[c];
        uint32_t first = 0;
        for (int k = 0; k < c; k++) first += nblk[k];
        for (uint32_t b = 0; b < nblk[c]; b++) {
            plan[3 * (first + b) + 0] = (uint32_t)c;
            plan[3 * (first + b) + 1] = start[c] + (uint32_t)((uint64_t)count[c] * b / nblk[c]);
            plan[3 * (first + b) + 2] = start[c] + (uint32_t)((uint64_t)count[c] * (b + 1) / nblk[c]);
        }
        if (c == kClasses - 1) {
            for (uint32_t b = first + nblk[c]; b < nplan; b++) {
                plan[3 * b + 0] = 0;
                plan[3 * b + 1] = 0;
                plan[3 * b + 2] = 0;
            }
        }
    }
}

// Pass 3: stable scatter of frame indices into class order.
__global__ __launch_bounds__(256) void k_bin_scatter(const uint32_t *len, uint32_t n, uint32_t chunk,
                                                     const uint32_t *base, uint32_t *order)
{
    __shared__ uint32_t wave_cnt[4][kClasses];
    __shared__ uint32_t run[kClasses];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x < kClasses) run[threadIdx.x] = base[blockIdx.x * kClasses + threadIdx.x];
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = min((uint64_t)n, lo + chunk);
    for (uint64_t t0 = lo; t0 < hi; t0 += blockDim.x) {
        const uint64_t i = t0 + threadIdx.x;
        const bool valid = i < hi;
        const int c = valid ? length_class(len[i]) : -1;
        uint32_t rank = 0;
#pragma unroll
        for (int k = 0; k < kClasses; k++) {
            const unsigned long long m = __ballot(c == k);
            if (c == k) rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (lane == 0) wave_cnt[wv][k] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        if (valid) {
            uint32_t before = run[c];
            for (int w = 0; w < wv; w++) before += wave_cnt[w][c];
            order[before + rank] = (uint32_t)i;
        }
        __syncthreads();
        if (threadIdx.x < kClasses) {
            uint32_t add = 0;
            for (int w = 0; w < 4; w++) add += wave_cnt[w][threadIdx.x];
            run[threadIdx.x] += add;
        }
        __syncthreads();
    }
}

template <int G, bool PF>
__device__ __forceinline__ void hash_range(const FrameParams &p, uint32_t begin, uint32_t end, uint32_t lo4,
                                           const SliceBases &sb)
{
    constexpr int kGroups = 64 / G;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t i0 = begin + (uint32_t)wv * kGroups; i0 < end; i0 += (uint32_t)kWavesPerBlock * kGroups) {
        const uint32_t i = i0 + (uint32_t)(lane / G);
        const bool active = i < end;
        const uint64_t f = active ? p.order[i] : 0u;
        hash_frame<G, PF>(p, f, active, lane % G, lo4, sb);
    }
}

// Ragged batches: workgroup b hashes the class-sorted frames plan[b] with the
// class's lanes per frame.
template <bool PF>
__global__ __launch_bounds__(kBlock) void k_frames_grouped(const FrameParams p)
{
    const uint32_t cls = p.plan[3 * blockIdx.x], begin = p.plan[3 * blockIdx.x + 1], end = p.plan[3 * blockIdx.x + 2];
    if (begin >= end) return;
    // Constant indices only: a runtime index into the kernel arguments would
    // copy them to scratch.
    const uint32_t xgap = cls == 0 ? p.xgap[0] : cls == 1 ? p.xgap[1] : cls == 2 ? p.xgap[2] : p.xgap[3];
    build_tables(p.xtab, xgap, true);
    const uint32_t lo4 = (uint32_t)(threadIdx.x & 31) << 2;
    const SliceBases sb = slice_bases(lo4);
    switch (cls) {
    case 0: hash_range<class_lanes(0), PF>(p, begin, end, lo4, sb); break;
    case 1: hash_range<class_lanes(1), PF>(p, begin, end, lo4, sb); break;
    case 2: hash_range<class_lanes(2), PF>(p, begin, end, lo4, sb); break;
    default: hash_range<class_lanes(3), PF>(p, begin, end, lo4, sb); break;
    }
}

// ---- region stage 2 -----------------------------------------------------------
// Fold per-chunk raw states: chunks 0..n-2 are `clen` bytes, chunk n-1 is
// `last_len`. One workgroup, pairwise GF(2) tree in LDS.
constexpr int kMaxChunks = 16384;
struct CombineParams {
    const uint32_t *states;
    uint32_t n;
    uint32_t *out;
    uint32_t levels;          // ceil(log2(n-1)) levels of "advance clen * 2^j"
    uint32_t col[15][32];     // level maps
    uint32_t last_col[32];    // advance last_len bytes
};

__global__ __launch_bounds__(1024) void k_combine(const CombineParams p)
{
    __shared__ uint32_t v[kMaxChunks];
    const uint32_t m = p.n - 1;          // equal-length chunks
    const uint32_t P = 1u << p.levels;   // padded to a power of two, zeros in front
    for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) v[i] = (i >= P - m) ? p.states[i - (P - m)] : 0u;
    __syncthreads();
    uint32_t width = P;
    for (uint32_t lv = 0; lv < p.levels; lv++) {
        const uint32_t half = width >> 1;
        uint32_t tmp[kMaxChunks / 2 / 1024];
        int cnt = 0;
        for (uint32_t i = threadIdx.x; i < half; i += blockDim.x) tmp[cnt++] = bitmatrix_apply(v[2 * i], p.col[lv]) ^ v[2 * i + 1];
        __syncthreads();
        cnt = 0;
        for (uint32_t i = threadIdx.x; i < half; i += blockDim.x) v[i] = tmp[cnt++];
        __syncthreads();
        width = half;
    }
    if (threadIdx.x == 0) {
        const uint32_t head = (m > 0) ? v[0] : 0u;
        *p.out = bitmatrix_apply(head, p.last_col) ^ p.states[p.n - 1];
    }
}

}  // namespace vcrc
