// val_crc32_hip.hip -- CDNA4 (gfx950) kernels and the C ABI of the VAL CRC-32
// integrity path. See DESIGN.md for the roofline argument; reference call
// sites are cited per entry point in include/val_crc32_gpu.h.
//
// Algorithm (no carry-less multiply on gfx950, no MFMA: this is GF(2) table
// work, not a dense contraction):
//   * A frame's CRC input of L bytes is cut into UNIT-byte units counted from
//     the END of the frame; the first unit is front-padded with zeros (free:
//     a zero register stays zero over zero bytes). The initial register
//     ("seed", 0xFFFFFFFF for VAL) is XORed into the first four real bytes,
//     which equals starting the register at the seed for L >= 4.
//   * G lanes share a frame. Lane g owns units g, g+G, g+2G, ... counted so
//     that lane G-1 owns the last unit. Each lane keeps one raw register and
//     runs slice-by-4 over its units (4 LDS lookups per 4 bytes); between its
//     units it advances the register over the (G-1)*UNIT bytes owned by the
//     other lanes with 8 nibble-table lookups (the "gap" map).
//   * A log2(G)-step __shfl_xor tree merges the G registers; step j advances
//     the left half by UNIT*2^j bytes (32x32 GF(2) bit-matrix in SGPRs).
//   * LDS holds the four slice tables replicated 32x across banks so the
//     per-lane lookups of a half-wave never conflict (128 KiB), plus the gap
//     nibble tables (16 KiB). One 1024-thread workgroup per CU.
//   * Loads are per-lane contiguous 64-byte units (4 x dwordx4, unaligned
//     addresses allowed): measured on MI355X this pattern streams faster than
//     1 KiB-contiguous wave loads (bench/micro/mb1.hip).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>

#include "gf2_crc32.h"
#include "val_crc32_gpu.h"
#include "val_protocol.h"

namespace vcrc {

constexpr int kBlock = 1024;   // threads per workgroup (16 waves)
constexpr uint32_t kLdsS4 = 0;          // 2 table pairs x 256 rows x 256 B
constexpr uint32_t kLdsGap = 131072;    // 8 nibble tables x 16 rows x 128 B
constexpr uint32_t kLdsWords = (131072 + 16384) / 4;
constexpr int kMaxTree = 7;    // log2(max virtual lanes = 128)

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));

struct FrameParams {
    const uint8_t *base;
    const uint64_t *off;   // NULL: strided mode
    const uint32_t *len;
    uint64_t stride;
    uint32_t flen;
    uint32_t last_len;     // strided mode: length of frame n-1
    uint32_t n;
    uint32_t seed0;        // initial register of frame 0
    uint32_t seed_rest;    // initial register of frames 1..n-1
    uint32_t xorout;       // XORed into every output (0xFFFFFFFF = finalized CRC)
    uint32_t *out_crc;
    uint32_t *out_hdr;
    uint8_t *out_ok;
    uint32_t *nbad;
    uint32_t verify;
    uint32_t xtab[4];      // x^(8(k+1)) defining slice table T_k
    uint32_t xgap;         // x^(8 (G-1) UNIT)
    uint32_t tree[kMaxTree][32];  // bit-matrix columns of "advance UNIT*2^j bytes"
};

__shared__ uint32_t s_lds[kLdsWords];

__device__ __forceinline__ uint32_t lds_read(uint32_t byte_addr)
{
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_lds) + byte_addr);
}

// Per-lane LDS base of each slice table: pair * 64 KiB + half * 128 + bank*4.
// T3 (first byte of a word) -> pair 0 half 0, T2 -> 0/1, T1 -> 1/0, T0 -> 1/1.
struct SliceBases {
    uint32_t t3, t2, t1, t0;
};

__device__ __forceinline__ SliceBases slice_bases(uint32_t lo4)
{
    SliceBases b;
    b.t3 = kLdsS4 + lo4;
    b.t2 = kLdsS4 + 128u + lo4;
    b.t1 = kLdsS4 + 65536u + lo4;
    b.t0 = kLdsS4 + 65536u + 128u + lo4;
    return b;
}

// v_perm_b32 builds the LDS address [base.b0 | y.byte_k | base.b2 | 0] in one
// instruction: row = byte value * 256, column = half*128 + bank*4.
__device__ __forceinline__ uint32_t tab_addr(uint32_t y, uint32_t base, int k)
{
    return __builtin_amdgcn_perm(y, base, 0x0C020400u + ((uint32_t)k << 8));
}

// One slice-by-4 step: feed the LE word w into raw register c.
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

// Advance a register over the (G-1)*UNIT bytes between a lane's units.
__device__ __forceinline__ uint32_t gap_step(uint32_t a, uint32_t lo4)
{
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= lds_read(kLdsGap + (uint32_t)k * 2048u + (((a >> (4 * k)) & 15u) << 7) + lo4);
    return r;
}

__device__ __forceinline__ uint32_t bitmatrix_apply(uint32_t v, const uint32_t *col)
{
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) r ^= (0u - ((v >> i) & 1u)) & col[i];
    return r;
}

__device__ __forceinline__ uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const u32u *>(p); }

template <int G>
__device__ void build_tables(const FrameParams &p)
{
    const int t = threadIdx.x;
    {   // slice tables: thread t builds T_k[b], k = t>>8, b = t&255, 32 bank replicas
        const int k = t >> 8, b = t & 255;
        const uint32_t v = gf2_mul(p.xtab[k], (uint32_t)b);
        const int slot = 3 - k;  // T3 -> slot 0 ... T0 -> slot 3
        uint32_t *row = s_lds + (kLdsS4 + (uint32_t)(slot >> 1) * 65536u + (uint32_t)b * 256u + (uint32_t)(slot & 1) * 128u) / 4;
        const uint4 vv = make_uint4(v, v, v, v);
#pragma unroll
        for (int r = 0; r < 8; r++) reinterpret_cast<uint4 *>(row)[r] = vv;
    }
    if (G > 1 && t < 128) {  // gap nibble tables: NT_k[n] = gap(n << 4k)
        const int k = t >> 4, nib = t & 15;
        const uint32_t v = gf2_mul(p.xgap, (uint32_t)nib << (4 * k));
        uint32_t *row = s_lds + (kLdsGap + (uint32_t)k * 2048u + (uint32_t)nib * 128u) / 4;
        const uint4 vv = make_uint4(v, v, v, v);
#pragma unroll
        for (int r = 0; r < 8; r++) reinterpret_cast<uint4 *>(row)[r] = vv;
    }
    __syncthreads();
}

// Words of one virtual lane's unit for round 0 (see header comment):
// u > 0: a full unit of unaligned dwordx4 loads; u == 0: the front-padded
// first unit, assembled word by word with the seed XORed into frame bytes
// 0..3; u < 0: nothing (zeros keep a zero register zero). Frames shorter than
// 4 bytes take the byte path instead (tiny = true).
template <int UNIT>
__device__ __forceinline__ void load_unit(uint32_t (&w)[UNIT / 4], int u, const uint8_t *fp, uint32_t L, uint32_t pad,
                                          uint32_t seed, bool &tiny)
{
    tiny = false;
    if (u > 0) {
        const uint8_t *up = fp + (uint64_t)u * UNIT - pad;
#pragma unroll
        for (int q = 0; q < UNIT / 16; q++) {
            const u32x4u v = *reinterpret_cast<const u32x4u *>(up + 16 * q);
            w[4 * q + 0] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
        // Seed bytes that did not fit in a unit 0 holding < 4 real bytes.
        if (u == 1 && pad > UNIT - 4) w[0] ^= seed >> (8 * (UNIT - pad));
    } else if (u == 0 && L >= 4) {
#pragma unroll
        for (int i = 0; i < UNIT / 4; i++) {
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
        for (int i = 0; i < UNIT / 4; i++) w[i] = 0;
        tiny = (u == 0);
    }
}

template <int CH, int G, int UNIT>
__device__ __forceinline__ void load_round(uint32_t (&w)[CH][UNIT / 4], const uint8_t *up)
{
#pragma unroll
    for (int c = 0; c < CH; c++) {
#pragma unroll
        for (int q = 0; q < UNIT / 16; q++) {
            const u32x4u v = *reinterpret_cast<const u32x4u *>(up + (uint64_t)G * UNIT * c + 16 * q);
            w[c][4 * q + 0] = v.x;
            w[c][4 * q + 1] = v.y;
            w[c][4 * q + 2] = v.z;
            w[c][4 * q + 3] = v.w;
        }
    }
}

// K1/K2/K3 fused: per-frame CRC (trailer), optional header_crc and verify.
// G lanes per frame, CH independent chains per lane -> V = G*CH virtual lanes;
// virtual lane v = g + G*c owns units v, v+V, v+2V, ... (counted so virtual
// lane V-1 owns the last unit). UNIT bytes per unit. PF: load the next
// round's units before hashing the current one (register double buffer).
template <int G, int CH, int UNIT, bool PF>
__global__ __launch_bounds__(kBlock) void k_frames(const FrameParams p)
{
    constexpr int V = G * CH;
    constexpr int W = UNIT / 4;
    build_tables<V>(p);
    constexpr int kGroups = 64 / G;
    const int lane = threadIdx.x & 63;
    const uint32_t lo4 = (uint32_t)(lane & 31) << 2;
    const SliceBases sb = slice_bases(lo4);
    const int g = lane % G;
    const int grp = lane / G;
    const uint64_t wave = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * kBlock) >> 6;

    for (uint64_t fb = wave * kGroups; fb < p.n; fb += nwaves * kGroups) {
        const uint64_t f = fb + (uint64_t)grp;
        const bool active = f < p.n;
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
        const uint32_t U = L ? (L + UNIT - 1) / UNIT : 1u;
        const uint32_t R = active ? (U + V - 1) / V : 0u;
        const uint32_t pad = U * UNIT - L;
        // Steady-state cursor: this lane's chain-0 unit of round 1.
        const uint8_t *up = fp + ((uint64_t)((int)U - V * (int)R + g) + V) * UNIT - pad;
        uint32_t nxt[PF ? CH : 1][PF ? W : 1];
        if (PF && R > 1) load_round<CH, G, UNIT>(reinterpret_cast<uint32_t(&)[CH][W]>(nxt), up);
        uint32_t acc[CH];
#pragma unroll
        for (int c = 0; c < CH; c++) acc[c] = 0;
        if (R > 0) {
            // Round 0 is the only one that can hold a virtual lane's unit 0
            // (front padding, seed, tiny frames) or no unit at all; registers
            // are still zero, so no gap step. Chains run one after another
            // here to keep register pressure low.
#pragma unroll
            for (int c = 0; c < CH; c++) {
                uint32_t w[W];
                bool tiny;
                load_unit<UNIT>(w, (int)U - V * (int)R + g + G * c, fp, L, pad, seed, tiny);
                uint32_t a = 0;
#pragma unroll
                for (int i = 0; i < W; i++) a = s4_step(a, w[i], sb);
                if (tiny) {  // L < 4: crc state of the few bytes straight from the seed
                    a = seed;
                    for (uint32_t i = 0; i < L; i++) a = byte_step(a, fp[i], sb);
                }
                acc[c] = a;
            }
        }
        // Steady state: every virtual lane has a full unit u >= 1 in rounds 1..R-1.
        for (uint32_t k = 1; k < R; k++, up += (uint64_t)V * UNIT) {
            uint32_t w[CH][W];
            if (PF) {
#pragma unroll
                for (int c = 0; c < CH; c++)
#pragma unroll
                    for (int i = 0; i < W; i++) w[c][i] = nxt[PF ? c : 0][PF ? i : 0];
                if (k + 1 < R) load_round<CH, G, UNIT>(reinterpret_cast<uint32_t(&)[CH][W]>(nxt), up + (uint64_t)V * UNIT);
            } else {
                load_round<CH, G, UNIT>(w, up);
            }
            // Seed bytes that did not fit in a unit 0 holding < 4 real bytes
            // land in the first word of unit 1 (k == 1, virtual lane 0).
            if (k == 1 && g == 0 && pad > UNIT - 4 && (int)U - V * (int)(R - 1) == 1)
                w[0][0] ^= seed >> (8 * (UNIT - pad));
            if (V > 1) {
#pragma unroll
                for (int c = 0; c < CH; c++) acc[c] = gap_step(acc[c], lo4);
            }
#pragma unroll
            for (int i = 0; i < W; i++) {
#pragma unroll
                for (int c = 0; c < CH; c++) acc[c] = s4_step(acc[c], w[c][i], sb);
            }
        }
        // Merge virtual lanes: level j joins blocks of 2^j virtual lanes, the
        // left one advanced by UNIT * 2^j bytes. Levels below log2(G) cross
        // lanes (__shfl_xor); the rest combine the chains inside a lane.
#pragma unroll
        for (int j = 0; (1 << j) < G; j++) {
            const bool right = (g >> j) & 1;
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const uint32_t other = __shfl_xor(acc[c], 1 << j);
                const uint32_t left = right ? other : acc[c];
                const uint32_t rgt = right ? acc[c] : other;
                acc[c] = bitmatrix_apply(left, p.tree[j]) ^ rgt;
            }
        }
        constexpr int kLaneLevels = (G >= 64) ? 6 : (G >= 32) ? 5 : (G >= 16) ? 4 : (G >= 8) ? 3 : (G >= 4) ? 2 : (G >= 2) ? 1 : 0;
#pragma unroll
        for (int span = 1, lvl = kLaneLevels; span < CH; span <<= 1, lvl++) {
#pragma unroll
            for (int c = 0; c + span < CH; c += 2 * span) acc[c] = bitmatrix_apply(acc[c], p.tree[lvl]) ^ acc[c + span];
        }
        const uint32_t total = acc[0];
        if (active && g == G - 1) {
            const uint32_t crc = total ^ p.xorout;
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
}

// Region stage 2: fold per-chunk raw states. Chunks 0..n-2 are `clen` bytes,
// chunk n-1 is `last_len`. One workgroup, pairwise tree in LDS.
constexpr int kMaxChunks = 16384;
struct CombineParams {
    const uint32_t *states;
    uint32_t n;
    uint32_t *out;
    uint32_t levels;                 // ceil(log2(n-1)) levels of "advance clen*2^j"
    uint32_t col[15][32];            // level maps
    uint32_t last_col[32];           // advance last_len bytes
};

__global__ __launch_bounds__(1024) void k_combine(const CombineParams p)
{
    __shared__ uint32_t v[kMaxChunks];
    const uint32_t m = p.n - 1;                // equal-length chunks
    const uint32_t P = 1u << p.levels;         // padded to a power of two, zeros in front
    for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) v[i] = (i >= P - m) ? p.states[i - (P - m)] : 0u;
    __syncthreads();
    uint32_t width = P;
    for (uint32_t lv = 0; lv < p.levels; lv++) {
        const uint32_t half = width >> 1;
        uint32_t tmp[kMaxChunks / 2 / 1024 > 0 ? kMaxChunks / 2 / 1024 : 1];
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

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
struct Ctx {
    std::recursive_mutex mu;
    bool ready = false;
    int device = -1;
    int cus = 0;
    hipStream_t stream = nullptr;
    uint8_t *d_stage = nullptr;   // host-API staging (frames, region input)
    size_t d_stage_cap = 0;
    uint8_t *d_small = nullptr;   // descriptors / outputs for host APIs
    size_t d_small_cap = 0;
};
Ctx g_ctx;
thread_local std::string t_err;

val_status_t fail(val_status_t st, const char *what, hipError_t e = hipSuccess)
{
    char buf[256];
    if (e != hipSuccess)
        snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else
        snprintf(buf, sizeof buf, "%s", what);
    t_err = buf;
    return st;
}

#define VCRC_HIP(call, what)                                   \
    do {                                                       \
        hipError_t e_ = (call);                                \
        if (e_ != hipSuccess) return fail(VAL_ERR_IO, what, e_); \
    } while (0)

val_status_t ensure_init(int device)
{
    std::lock_guard<std::recursive_mutex> lk(g_ctx.mu);
    if (g_ctx.ready && (device < 0 || device == g_ctx.device)) return VAL_OK;
    if (g_ctx.ready) return fail(VAL_ERR_INVALID_ARG, "val_gpu_init: already bound to another device");
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) return fail(VAL_ERR_IO, "val_gpu_init: no HIP device", e);
    if (device < 0) device = 0;
    if (device >= count) return fail(VAL_ERR_INVALID_ARG, "val_gpu_init: device index out of range");
    VCRC_HIP(hipSetDevice(device), "hipSetDevice");
    hipDeviceProp_t prop;
    VCRC_HIP(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return fail(VAL_ERR_IO, "val_gpu_init: device is not gfx950");
    VCRC_HIP(hipStreamCreateWithFlags(&g_ctx.stream, hipStreamNonBlocking), "hipStreamCreate");
    g_ctx.device = device;
    g_ctx.cus = prop.multiProcessorCount;
    g_ctx.ready = true;
    return VAL_OK;
}

val_status_t bind_thread()
{
    val_status_t st = ensure_init(-1);
    if (st != VAL_OK) return st;
    VCRC_HIP(hipSetDevice(g_ctx.device), "hipSetDevice");  // device is per host thread in HIP
    return VAL_OK;
}

bool valid_lanes(uint32_t g) { return g == 1 || g == 2 || g == 4 || g == 8 || g == 16 || g == 32 || g == 64; }
bool valid_chains(uint32_t c) { return c == 1 || c == 2; }

std::atomic<uint32_t> g_forced_lanes{0};
std::atomic<uint32_t> g_forced_chains{0};

uint32_t env_u32(const char *name)
{
    const char *e = getenv(name);
    return e ? (uint32_t)atoi(e) : 0u;
}

// Lanes that share one frame (G). Short frames share a wave (64/G frames per
// wave); long frames spread over more lanes so every lane hashes a few KiB.
uint32_t lanes_per_frame(uint32_t len)
{
    static const uint32_t env_g = env_u32("VAL_GPU_LANES_PER_FRAME");
    const uint32_t forced = g_forced_lanes.load(std::memory_order_relaxed);
    if (valid_lanes(forced)) return forced;
    if (valid_lanes(env_g)) return env_g;
    // Measured on MI355X (tools/sweep_geometry.py): ~2 KiB of CRC input per
    // lane, at least 4 and at most 32 lanes per frame.
    uint32_t g = 4;
    while (g < 32 && (uint64_t)len >= (uint64_t)g * 2u * 2048u) g <<= 1;
    return g;
}

// Independent CRC chains per lane (CH): more loads and LDS lookups in flight.
uint32_t chains_per_lane(uint32_t len)
{
    static const uint32_t env_c = env_u32("VAL_GPU_CHAINS_PER_LANE");
    const uint32_t forced = g_forced_chains.load(std::memory_order_relaxed);
    if (valid_chains(forced)) return forced;
    if (valid_chains(env_c)) return env_c;
    (void)len;
    return 1;
}

bool valid_unit(uint32_t u) { return u == 64 || u == 128; }
std::atomic<uint32_t> g_forced_unit{0};
std::atomic<int> g_forced_prefetch{-1};

// Bytes a lane hashes per round.
uint32_t unit_bytes(uint32_t len)
{
    static const uint32_t env_u = env_u32("VAL_GPU_UNIT");
    const uint32_t forced = g_forced_unit.load(std::memory_order_relaxed);
    if (valid_unit(forced)) return forced;
    if (valid_unit(env_u)) return env_u;
    (void)len;
    return 64;
}

bool prefetch_on(uint32_t len)
{
    static const int env_p = getenv("VAL_GPU_PREFETCH") ? atoi(getenv("VAL_GPU_PREFETCH")) : -1;
    const int forced = g_forced_prefetch.load(std::memory_order_relaxed);
    if (forced >= 0) return forced != 0;
    if (env_p >= 0) return env_p != 0;
    (void)len;
    return true;
}

void fill_geometry(FrameParams &p, uint32_t V, uint32_t unit)
{
    for (int k = 0; k < 4; k++) p.xtab[k] = gf2_x8n((uint64_t)(k + 1));
    p.xgap = gf2_x8n((uint64_t)(V - 1) * unit);
    for (int j = 0; j < kMaxTree; j++) gf2_shift_columns((uint64_t)unit << j, p.tree[j]);
}

template <int G, int UNIT, bool PF>
void launch_gup(uint32_t CH, dim3 grid, dim3 block, hipStream_t s, const FrameParams &p)
{
    if (CH == 2) hipLaunchKernelGGL((k_frames<G, 2, UNIT, PF>), grid, block, 0, s, p);
    else hipLaunchKernelGGL((k_frames<G, 1, UNIT, PF>), grid, block, 0, s, p);
}

template <int G>
void launch_g(uint32_t CH, uint32_t unit, bool pf, dim3 grid, dim3 block, hipStream_t s, const FrameParams &p)
{
    if (unit == 128) {
        if (pf) launch_gup<G, 128, true>(CH, grid, block, s, p);
        else launch_gup<G, 128, false>(CH, grid, block, s, p);
    } else {
        if (pf) launch_gup<G, 64, true>(CH, grid, block, s, p);
        else launch_gup<G, 64, false>(CH, grid, block, s, p);
    }
}

val_status_t launch_frames(FrameParams &p, uint32_t typical_len, hipStream_t s)
{
    if (p.n == 0) return VAL_OK;
    const uint32_t G = lanes_per_frame(typical_len);
    const uint32_t CH = chains_per_lane(typical_len);
    const uint32_t unit = unit_bytes(typical_len);
    const bool pf = prefetch_on(typical_len);
    fill_geometry(p, G * CH, unit);
    const uint64_t groups_per_block = (uint64_t)(kBlock / 64) * (64 / G);
    uint64_t blocks = (p.n + groups_per_block - 1) / groups_per_block;
    blocks = std::min<uint64_t>(blocks, (uint64_t)g_ctx.cus);  // one 144 KiB-LDS workgroup per CU, persistent
    if (blocks == 0) blocks = 1;
    dim3 grid((unsigned)blocks), block(kBlock);
    switch (G) {
    case 1: launch_g<1>(CH, unit, pf, grid, block, s, p); break;
    case 2: launch_g<2>(CH, unit, pf, grid, block, s, p); break;
    case 4: launch_g<4>(CH, unit, pf, grid, block, s, p); break;
    case 8: launch_g<8>(CH, unit, pf, grid, block, s, p); break;
    case 16: launch_g<16>(CH, unit, pf, grid, block, s, p); break;
    case 32: launch_g<32>(CH, unit, pf, grid, block, s, p); break;
    case 64: launch_g<64>(CH, unit, pf, grid, block, s, p); break;
    default: return fail(VAL_ERR_INVALID_ARG, "bad lanes-per-frame");
    }
    VCRC_HIP(hipGetLastError(), "k_frames launch");
    return VAL_OK;
}

// NULL selects the HIP default (null) stream, as in every HIP API.
hipStream_t pick_stream(void *stream) { return (hipStream_t)stream; }

// Chunking of a long region into "frames" for stage 1.
void region_geometry(uint64_t len, uint64_t *clen, uint32_t *nchunks)
{
    uint64_t c = 4096;
    while ((len + c - 1) / c > (uint64_t)kMaxChunks) c <<= 1;
    // Prefer >= 8192 chunks of work when the region is large enough.
    while (c < 65536 && (len + 2 * c - 1) / (2 * c) >= 8192) c <<= 1;
    *clen = c;
    *nchunks = (uint32_t)(len ? (len + c - 1) / c : 1);
}

val_status_t region_dev(const uint8_t *d_ptr, uint64_t len, uint32_t state_in, uint32_t *d_out, hipStream_t s)
{
    uint64_t clen;
    uint32_t n;
    region_geometry(len, &clen, &n);
    if (n == 1) {
        FrameParams p{};
        p.base = d_ptr;
        p.stride = clen;
        p.flen = (uint32_t)len;
        p.last_len = (uint32_t)len;
        p.n = 1;
        p.seed0 = p.seed_rest = state_in;
        p.xorout = 0;
        p.out_crc = d_out;
        return launch_frames(p, (uint32_t)len, s);
    }
    uint32_t *d_states = nullptr;
    VCRC_HIP(hipMallocAsync((void **)&d_states, (size_t)n * 4u, s), "hipMallocAsync(region scratch)");
    FrameParams p{};
    p.base = d_ptr;
    p.stride = clen;
    p.flen = (uint32_t)clen;
    p.last_len = (uint32_t)(len - (uint64_t)(n - 1) * clen);
    p.n = n;
    p.seed0 = state_in;
    p.seed_rest = 0;
    p.xorout = 0;
    p.out_crc = d_states;
    val_status_t st = launch_frames(p, (uint32_t)clen, s);
    if (st != VAL_OK) {
        (void)hipFreeAsync(d_states, s);
        return st;
    }
    CombineParams cp{};
    cp.states = d_states;
    cp.n = n;
    cp.out = d_out;
    uint32_t m = n - 1, levels = 0;
    while ((1u << levels) < m) levels++;
    cp.levels = levels;
    for (uint32_t j = 0; j < levels; j++) gf2_shift_columns(clen << j, cp.col[j]);
    gf2_shift_columns(p.last_len, cp.last_col);
    hipLaunchKernelGGL(k_combine, dim3(1), dim3(1024), 0, s, cp);
    hipError_t e = hipGetLastError();
    (void)hipFreeAsync(d_states, s);
    if (e != hipSuccess) return fail(VAL_ERR_IO, "k_combine launch", e);
    return VAL_OK;
}

val_status_t grow(uint8_t **buf, size_t *cap, size_t need)
{
    if (*cap >= need) return VAL_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    size_t sz = std::max<size_t>(need, 1u << 20);
    hipError_t e = hipMalloc((void **)buf, sz);
    if (e != hipSuccess) return fail(VAL_ERR_NO_MEMORY, "hipMalloc(staging)", e);
    *cap = sz;
    return VAL_OK;
}

// Host pointer -> region state (used by the scalar hooks).
val_status_t region_host(const void *data, size_t len, uint32_t state_in, uint32_t *state_out)
{
    val_status_t st = bind_thread();
    if (st != VAL_OK) return st;
    std::lock_guard<std::recursive_mutex> lk(g_ctx.mu);
    if ((st = grow(&g_ctx.d_stage, &g_ctx.d_stage_cap, len ? len : 1)) != VAL_OK) return st;
    if ((st = grow(&g_ctx.d_small, &g_ctx.d_small_cap, 64)) != VAL_OK) return st;
    hipStream_t s = g_ctx.stream;
    if (len) VCRC_HIP(hipMemcpyAsync(g_ctx.d_stage, data, len, hipMemcpyHostToDevice, s), "H2D");
    uint32_t *d_out = reinterpret_cast<uint32_t *>(g_ctx.d_small);
    if ((st = region_dev(g_ctx.d_stage, len, state_in, d_out, s)) != VAL_OK) return st;
    VCRC_HIP(hipMemcpyAsync(state_out, d_out, 4, hipMemcpyDeviceToHost, s), "D2H");
    VCRC_HIP(hipStreamSynchronize(s), "hipStreamSynchronize");
    return VAL_OK;
}

[[noreturn]] void die(const char *fn)
{
    fprintf(stderr, "val_crc32_gpu: %s failed on the GPU path: %s (no CPU fallback by design)\n", fn, t_err.c_str());
    abort();
}

uint32_t scalar_state(const char *fn, uint32_t state, const void *data, size_t len)
{
    uint32_t out = 0;
    if (len && !data) die(fn);
    if (region_host(data, len, state, &out) != VAL_OK) die(fn);
    return out;
}

val_status_t frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off, const uint32_t *len,
                         uint64_t stride, uint32_t flen, uint32_t n, int verify, uint32_t *crc, uint32_t *hdr,
                         uint8_t *ok, uint32_t *nbad)
{
    if (!base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    if ((off == nullptr) != (len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    const uint64_t tail = verify ? 4u : 0u;
    uint64_t span = 0, len_sum = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t o = off ? off[i] : (uint64_t)i * stride;
        const uint64_t l = len ? len[i] : flen;
        if (o > base_len || l + tail > base_len - o) return fail(VAL_ERR_INVALID_ARG, "frame overruns the buffer");
        span = std::max(span, o + l + tail);
        len_sum += l;
    }
    val_status_t st = bind_thread();
    if (st != VAL_OK) return st;
    std::lock_guard<std::recursive_mutex> lk(g_ctx.mu);
    const size_t desc_bytes = off ? (size_t)n * 12u : 0u;
    const size_t out_bytes = (size_t)n * 9u + 16u;
    if ((st = grow(&g_ctx.d_stage, &g_ctx.d_stage_cap, span ? span : 1)) != VAL_OK) return st;
    if ((st = grow(&g_ctx.d_small, &g_ctx.d_small_cap, desc_bytes + out_bytes + 64)) != VAL_OK) return st;
    hipStream_t s = g_ctx.stream;
    uint8_t *sm = g_ctx.d_small;
    uint64_t *d_off = off ? reinterpret_cast<uint64_t *>(sm) : nullptr;
    uint32_t *d_len = off ? reinterpret_cast<uint32_t *>(sm + (size_t)n * 8u) : nullptr;
    uint32_t *d_crc = reinterpret_cast<uint32_t *>(sm + desc_bytes);
    uint32_t *d_hdr = d_crc + n;
    uint32_t *d_nbad = d_hdr + n;
    uint8_t *d_ok = reinterpret_cast<uint8_t *>(d_nbad + 4);
    if (span) VCRC_HIP(hipMemcpyAsync(g_ctx.d_stage, base, span, hipMemcpyHostToDevice, s), "H2D frames");
    if (off) {
        VCRC_HIP(hipMemcpyAsync(d_off, off, (size_t)n * 8u, hipMemcpyHostToDevice, s), "H2D off");
        VCRC_HIP(hipMemcpyAsync(d_len, len, (size_t)n * 4u, hipMemcpyHostToDevice, s), "H2D len");
    }
    VCRC_HIP(hipMemsetAsync(d_nbad, 0, 4, s), "memset");
    FrameParams p{};
    p.base = g_ctx.d_stage;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.flen = flen;
    p.last_len = flen;
    p.n = n;
    p.seed0 = p.seed_rest = 0xFFFFFFFFu;
    p.xorout = 0xFFFFFFFFu;
    p.out_crc = crc ? d_crc : nullptr;
    p.out_hdr = hdr ? d_hdr : nullptr;
    p.verify = verify ? 1u : 0u;
    p.out_ok = ok ? d_ok : nullptr;
    p.nbad = d_nbad;
    const uint32_t typical = n ? (uint32_t)std::min<uint64_t>(len_sum / n, 0xFFFFFFFFu) : 0u;
    if ((st = launch_frames(p, typical, s)) != VAL_OK) return st;
    if (crc) VCRC_HIP(hipMemcpyAsync(crc, d_crc, (size_t)n * 4u, hipMemcpyDeviceToHost, s), "D2H crc");
    if (hdr) VCRC_HIP(hipMemcpyAsync(hdr, d_hdr, (size_t)n * 4u, hipMemcpyDeviceToHost, s), "D2H hdr");
    if (ok) VCRC_HIP(hipMemcpyAsync(ok, d_ok, (size_t)n, hipMemcpyDeviceToHost, s), "D2H ok");
    uint32_t bad = 0;
    VCRC_HIP(hipMemcpyAsync(&bad, d_nbad, 4, hipMemcpyDeviceToHost, s), "D2H nbad");
    VCRC_HIP(hipStreamSynchronize(s), "hipStreamSynchronize");
    if (nbad) *nbad = bad;
    return VAL_OK;
}

}  // namespace vcrc

using namespace vcrc;

extern "C" {

val_status_t val_gpu_init(int device)
{
    t_err.clear();
    return ensure_init(device);
}

void val_gpu_shutdown(void)
{
    std::lock_guard<std::recursive_mutex> lk(g_ctx.mu);
    if (!g_ctx.ready) return;
    (void)hipSetDevice(g_ctx.device);
    if (g_ctx.stream) (void)hipStreamSynchronize(g_ctx.stream);
    if (g_ctx.d_stage) (void)hipFree(g_ctx.d_stage);
    if (g_ctx.d_small) (void)hipFree(g_ctx.d_small);
    if (g_ctx.stream) (void)hipStreamDestroy(g_ctx.stream);
    g_ctx.d_stage = g_ctx.d_small = nullptr;
    g_ctx.d_stage_cap = g_ctx.d_small_cap = 0;
    g_ctx.stream = nullptr;
    g_ctx.ready = false;
    g_ctx.device = -1;
}

int val_gpu_device_count(void)
{
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

uint32_t val_gpu_abi_version(void) { return VAL_GPU_ABI_VERSION; }

const char *val_gpu_last_error(void) { return t_err.c_str(); }

uint32_t val_gpu_lanes_per_frame(uint32_t typical_len) { return lanes_per_frame(typical_len); }

val_status_t val_gpu_set_lanes_per_frame(uint32_t lanes)
{
    if (lanes != 0 && !valid_lanes(lanes)) return fail(VAL_ERR_INVALID_ARG, "lanes must be 0 or a power of two <= 64");
    g_forced_lanes.store(lanes, std::memory_order_relaxed);
    return VAL_OK;
}

uint32_t val_gpu_chains_per_lane(uint32_t typical_len) { return chains_per_lane(typical_len); }

val_status_t val_gpu_set_unit_bytes(uint32_t unit)
{
    if (unit != 0 && !valid_unit(unit)) return fail(VAL_ERR_INVALID_ARG, "unit must be 0, 64 or 128");
    g_forced_unit.store(unit, std::memory_order_relaxed);
    return VAL_OK;
}

val_status_t val_gpu_set_prefetch(int on)
{
    g_forced_prefetch.store(on < 0 ? -1 : (on ? 1 : 0), std::memory_order_relaxed);
    return VAL_OK;
}

val_status_t val_gpu_set_chains_per_lane(uint32_t chains)
{
    if (chains != 0 && !valid_chains(chains)) return fail(VAL_ERR_INVALID_ARG, "chains must be 0, 1 or 2");
    g_forced_chains.store(chains, std::memory_order_relaxed);
    return VAL_OK;
}

uint32_t val_crc32_shift(uint32_t state, uint64_t nbytes) { return gf2_mul(gf2_x8n(nbytes), state); }

uint32_t val_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    return gf2_mul(gf2_x8n(len_b), crc_a) ^ crc_b;
}

uint32_t val_crc32_init_state(void) { return 0xFFFFFFFFu; }

uint32_t val_crc32_finalize_state(uint32_t state) { return state ^ 0xFFFFFFFFu; }

uint32_t val_crc32_update_state(uint32_t state, const void *data, size_t length)
{
    return scalar_state("val_crc32_update_state", state, data, length);
}

uint32_t val_crc32(const void *data, size_t length)
{
    return scalar_state("val_crc32", 0xFFFFFFFFu, data, length) ^ 0xFFFFFFFFu;
}

uint32_t val_gpu_crc32_provider(uint32_t seed, const void *buf, size_t len)
{
    return scalar_state("val_gpu_crc32_provider", seed, buf, len) ^ 0xFFFFFFFFu;
}

val_status_t val_crc32_frames_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len, uint64_t stride,
                                  uint32_t flen, uint32_t n, uint32_t len_hint, uint32_t *d_crc, uint32_t *d_hdr,
                                  void *stream)
{
    t_err.clear();
    if ((d_off == nullptr) != (d_len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    if (!d_base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    val_status_t st = bind_thread();
    if (st != VAL_OK) return st;
    FrameParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.flen = flen;
    p.last_len = flen;
    p.n = n;
    p.seed0 = p.seed_rest = 0xFFFFFFFFu;
    p.xorout = 0xFFFFFFFFu;
    p.out_crc = d_crc;
    p.out_hdr = d_hdr;
    const uint32_t typical = d_off ? (len_hint ? len_hint : 16384u) : flen;
    return launch_frames(p, typical, pick_stream(stream));
}

val_status_t val_crc32_verify_frames_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                                         uint64_t stride, uint32_t flen, uint32_t n, uint32_t len_hint, uint8_t *d_ok,
                                         uint32_t *d_nbad, uint32_t *d_crc, uint32_t *d_hdr, void *stream)
{
    t_err.clear();
    if ((d_off == nullptr) != (d_len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    if (!d_base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    val_status_t st = bind_thread();
    if (st != VAL_OK) return st;
    FrameParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.flen = flen;
    p.last_len = flen;
    p.n = n;
    p.seed0 = p.seed_rest = 0xFFFFFFFFu;
    p.xorout = 0xFFFFFFFFu;
    p.out_crc = d_crc;
    p.out_hdr = d_hdr;
    p.verify = 1;
    p.out_ok = d_ok;
    p.nbad = d_nbad;
    const uint32_t typical = d_off ? (len_hint ? len_hint : 16384u) : flen;
    return launch_frames(p, typical, pick_stream(stream));
}

val_status_t val_crc32_region_dev(const uint8_t *d_ptr, uint64_t len, uint32_t state_in, uint32_t *d_state_out,
                                  void *stream)
{
    t_err.clear();
    if (!d_state_out || (!d_ptr && len)) return fail(VAL_ERR_INVALID_ARG, "NULL pointer");
    val_status_t st = bind_thread();
    if (st != VAL_OK) return st;
    return region_dev(d_ptr, len, state_in, d_state_out, pick_stream(stream));
}

uint64_t val_crc32_region_scratch_bytes(uint64_t len)
{
    uint64_t clen;
    uint32_t n;
    region_geometry(len, &clen, &n);
    return n > 1 ? (uint64_t)n * 4u : 0u;
}

val_status_t val_crc32_frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off, const uint32_t *len,
                                   uint64_t stride, uint32_t flen, uint32_t n, uint32_t *crc, uint32_t *hdr)
{
    t_err.clear();
    return frames_host(base, base_len, off, len, stride, flen, n, 0, crc, hdr, nullptr, nullptr);
}

val_status_t val_crc32_verify_frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                          const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n, uint8_t *ok,
                                          uint32_t *nbad)
{
    t_err.clear();
    uint32_t bad = 0;
    val_status_t st = frames_host(base, base_len, off, len, stride, flen, n, 1, nullptr, nullptr, ok, &bad);
    if (nbad) *nbad = bad;
    if (st == VAL_OK && bad) return VAL_ERR_CRC;
    return st;
}

}  // extern "C"
