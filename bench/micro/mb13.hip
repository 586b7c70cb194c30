// Microbenchmark 13 (not product code): the read pattern of short frames,
// XOR only. k_frames at 1,100-B frames runs within 4% of its own loads without
// the table work (profiles/r03_ab_short_nohash.log), at about 5.15 TB/s, so
// the question for a next design is what other read patterns of the same
// buffer reach. 2,917,776 frames of 1,100 B at a 1,104-B stride (3.2 GB, the
// u1100d batch), one 1024-thread workgroup per CU, waves grid-stride over
// groups of 16 frames (17,664 B):
//   frames     the product's shape at G = 4: each round a frame's 4 lanes read
//              its next 256 B (64 B per lane, units anchored at the frame end,
//              unit 0 from the frame's first line), next round in flight
//   contig64   each round the wave reads the next 4 KiB of its group, 64 B per
//              lane (lane l at +64 l, the lanes' units ignore frame edges)
//   contig16   the same 4 KiB, but instruction q reads 1 KiB contiguously
//              (lane l at +1024 q + 16 l)
//   stream     plain read of the whole buffer, 4 KiB per wave per round
//   +desc, +st, +sh  the frames pattern with the product's per-frame work
//              added step by step (descriptors, output store, shuffles)
//   rtL        (round 4) the frame length from a kernel argument: "frames"
//              with the constant length had hipcc unroll the five rounds and
//              issue them all at the group start; rtL keeps one round in
//              flight, as the product does
//   ilv16      (round 4) the frames pattern read as a 16-B interleave:
//              instruction q covers G x 16 contiguous bytes of each frame
//   bidir      (round 4) odd frames read their rounds last first
// Frames start 512 B into the buffer: round 0's span starts before its
// frame (the 16-B interleave reads it whole).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef const uint8_t __attribute__((address_space(1))) gu8;
typedef const u32x4u __attribute__((address_space(1))) gu32x4u;

constexpr uint32_t kL = 1100, kStride = 1104, kG = 4, kGPW = 64 / kG;
constexpr uint64_t kN = (3ull << 30) / kStride;
constexpr uint64_t kGroups = (kN + kGPW - 1) / kGPW, kGroupBytes = (uint64_t)kGPW * kStride;

__global__ void k_fill(u32x4 *p, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z ^= z >> 29;
        p[i] = u32x4{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)(z * 3), (uint32_t)i};
    }
}

__device__ __forceinline__ void ld64(u32x4u (&v)[4], gu8 *p)
{
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = *(gu32x4u *)(p + 16 * q);
}
__device__ __forceinline__ void ld64i(u32x4u (&v)[4], gu8 *p)  // 16-B interleave: instruction q at +16 G q
{
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = *(gu32x4u *)(p + 16 * kG * q);
}
__device__ __forceinline__ uint32_t xr(const u32x4u (&v)[4])
{
    uint32_t a = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) a ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    return a;
}

// MODE 0 frames, 1 contig64, 2 contig16, 3 stream
template <int MODE>
__global__ __launch_bounds__(1024) void k_pat(const uint8_t *base, uint64_t bytes, uint32_t *out, const uint64_t *doff,
                                              const uint32_t *dlen, uint32_t *outf, uint32_t rtL)
{
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * 1024 + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * 1024) >> 6;
    uint32_t acc = 0;
    if (MODE == 3) {
        const uint64_t chunks = bytes / 4096;
        for (uint64_t c = wave; c < chunks; c += nw) {
            u32x4u v[4];
#pragma unroll
            for (int q = 0; q < 4; q++) v[q] = *(gu32x4u *)((gu8 *)base + c * 4096 + q * 1024 + lane * 16);
            acc ^= xr(v);
        }
    } else if ((MODE & 7) == 0) {
        // MODE bits above 0..2 add the product's per-frame work to the frames
        // pattern, XOR standing in for the table lookups: 8 = lengths and
        // offsets from descriptor arrays (R and the unit grid per lane at run
        // time), 16 = one 4-B output store per frame, 32 = the wave-wide
        // min-reduction of round 0's first word and a log2(G) shuffle merge
        // 64 = the length from a kernel argument (run-time geometry, as the
        // product: no unrolled, hoisted rounds); 128 = the 16-B interleave
        // (round span read as four instructions of G x 16 contiguous bytes
        // per frame, lane g at 16 g; mb14)
        // 256 (with 128) = bidirectional: odd frames read their rounds last
        // first, so both sides of every frame boundary are read in the same
        // round (the boundary line is otherwise fetched twice, R - 1 rounds
        // apart: 1.12x traffic on 1,100-B frames)
        constexpr bool DESC = MODE & 8, ST = MODE & 16, SH = MODE & 32, RTL = MODE & 64, ILV = MODE & 128,
                       BIDIR = MODE & 256;
        const int g = lane % kG;
        uint32_t nL = 0;  // DESC: the next group's descriptors, fetched while this group is read (as k_frames does)
        uint64_t noff = 0;
        if (DESC) {
            const uint64_t f = wave * kGPW + lane / kG;
            nL = f < kN ? dlen[f] : 0u;
            noff = f < kN ? doff[f] : 0u;
        }
        for (uint64_t grp = wave; grp < kGroups; grp += nw) {
            const uint64_t f = grp * kGPW + lane / kG;
            uint32_t L = RTL ? rtL : kL;
            uint64_t off = f * kStride;
            if (DESC) {
                L = nL;
                off = noff;
                const uint64_t fn = f + nw * kGPW;
                nL = fn < kN ? dlen[fn] : 0u;
                noff = fn < kN ? doff[fn] : 0u;
            } else if (f >= kN) {
                continue;
            }
            const uint32_t U = (L + 63) / 64, R = L ? (U + kG - 1) / kG : 0u, pad = U * 64 - L;
            gu8 *fp = (gu8 *)base + off;
            const int u0 = (int)U - (int)(kG * R) + g;
            u32x4u w0[4], nx[4];
            // round r's span starts at fp + 64 (U - G R + G r) - pad; lane g at 16 g + 16 G q
            gu8 *sp0 = fp + (int64_t)((int)U - (int)(kG * R)) * 64 - pad + 16 * g;
            const bool back = BIDIR && (f & 1);
            auto span = [&](uint32_t r) { return sp0 + (int64_t)(back ? R - 1 - r : r) * kG * 64; };
            if (ILV) {
                if (R > 0) ld64i(w0, span(0));
                if (R > 1) ld64i(nx, span(1));
            } else {
                if (R > 0 && u0 >= 0) {
                    const uint32_t inl = (uint32_t)((uintptr_t)fp & 127u);
                    const uint32_t skip = (u0 == 0 && pad > inl) ? pad - inl : 0u;
                    ld64(w0, fp + (int64_t)u0 * 64 - pad + skip);
                }
                if (R > 1) ld64(nx, fp + (int64_t)(u0 + kG) * 64 - pad);
            }
            gu8 *up = ILV ? fp + (int64_t)((int)U - (int)(kG * R) + kG) * 64 - pad + 16 * g
                          : fp + (int64_t)(u0 + kG) * 64 - pad;
            uint32_t a = 0;
            if (SH) {
                int first = (R == 0 || u0 < 0) ? 16 : (u0 == 0 ? (int)(pad >> 2) : 0);
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) first = min(first, __shfl_xor(first, o));
                a = (uint32_t)__builtin_amdgcn_readfirstlane(first);
            }
            if (R > 0 && (ILV || u0 >= 0)) a ^= xr(w0);
            for (uint32_t r = 1; r < R; r++) {
                u32x4u cur[4];
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = nx[q];
                if (r + 1 < R) {
                    if (ILV) ld64i(nx, span(r + 1));
                    else ld64(nx, up + (uint64_t)r * kG * 64);
                }
                a = (a << 1 | a >> 31) ^ xr(cur);
            }
            if (SH) {
#pragma unroll
                for (int j = 0; j < 2; j++) a ^= __shfl_xor(a, 1 << j);
            }
            if (ST && g == kG - 1 && f < kN) outf[f] = a;
            acc ^= a;
        }
    } else {
        constexpr uint32_t R = (uint32_t)((kGroupBytes + 4095) / 4096);
        for (uint64_t grp = wave; grp < kGroups; grp += nw) {
            gu8 *gp = (gu8 *)base + grp * kGroupBytes;
            auto addr = [&](uint32_t r, int q) {
                const uint64_t o = (uint64_t)r * 4096 + (MODE == 1 ? (uint64_t)lane * 64 + 16 * q : (uint64_t)q * 1024 + lane * 16);
                return o + 16 <= kGroupBytes ? gp + o : gp;  // a group's last round is partial
            };
            u32x4u nx[4];
#pragma unroll
            for (int q = 0; q < 4; q++) nx[q] = *(gu32x4u *)addr(0, q);
            for (uint32_t r = 0; r < R; r++) {
                u32x4u cur[4];
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = nx[q];
                if (r + 1 < R)
#pragma unroll
                    for (int q = 0; q < 4; q++) nx[q] = *(gu32x4u *)addr(r + 1, q);
                acc ^= xr(cur);
            }
        }
    }
    if (acc == 0x9u) out[0] = acc;
}

template <typename F> float timeit(F f, int reps = 9)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
        CHECK(hipEventRecord(a));
        f();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CHECK(hipGetLastError());
    return t[t.size() / 2];
}

int main()
{
    hipDeviceProp_t pr;
    CHECK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    const size_t bytes = (size_t)kGroups * kGroupBytes;
    uint8_t *d;
    uint32_t *out;
    CHECK(hipMalloc(&d, bytes + 8192));
    CHECK(hipMalloc(&out, 64));
    std::vector<uint64_t> hoff(kN);
    std::vector<uint32_t> hlen(kN, kL);
    for (uint64_t i = 0; i < kN; i++) hoff[i] = i * kStride;
    uint64_t *doff;
    uint32_t *dlen, *outf;
    CHECK(hipMalloc(&doff, kN * 8));
    CHECK(hipMalloc(&dlen, kN * 4));
    CHECK(hipMalloc(&outf, kN * 4));
    CHECK(hipMemcpy(doff, hoff.data(), kN * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dlen, hlen.data(), kN * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (u32x4 *)d, (bytes + 8192) / 16);
    CHECK(hipDeviceSynchronize());
    const double crc_bytes = (double)kN * kL;
#define RUN(M, name)                                                                                                 \
    {                                                                                                                \
        const float ms = timeit([&] { hipLaunchKernelGGL((k_pat<M>), dim3(cus), dim3(1024), 0, 0, d + 512, bytes, out, doff, dlen, outf, kL); }); \
        printf("%-9s %.4f ms  %7.1f GB/s of CRC input (%llu x %u B)  %7.1f GB/s of buffer\n", name, ms,                \
               crc_bytes / ms / 1e6, (unsigned long long)kN, kL, (double)bytes / ms / 1e6);                            \
        fflush(stdout);                                                                                              \
    }
    for (int rep = 0; rep < 2; rep++) {
        RUN(64, "frames rtL")
        RUN(64 + 128, "ilv16 rtL")
        RUN(64 + 128 + 256, "ilv16 rtL bidir")
        RUN(128, "ilv16")
        RUN(128 + 256, "ilv16 bidir")
        RUN(0, "frames")
        RUN(8, "+desc")
        RUN(24, "+desc+st")
        RUN(56, "+desc+st+sh")
        RUN(1, "contig64")
        RUN(2, "contig16")
        RUN(3, "stream")
    }
    printf("done\n");
    return 0;
}
