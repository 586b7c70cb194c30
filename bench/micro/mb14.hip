// Microbenchmark 14 (not product code): the short-frame read shape with
// run-time geometry. mb13's "frames" row (6.05 TB/s on 1,100-B frames) had
// the frame length as a compile-time constant: hipcc unrolled the five rounds
// of a group and issued all of them at the group's start, so that row was
// "every round in flight", not the product's one-round prefetch; its "+desc"
// row changed the geometry to run time as well as adding the descriptors.
// Here the length is a kernel argument in every variant, and the table work
// is the product's own (slice-by-4 over the LDS tables, a gap step per unit):
//   shape 0  the product's: lane g of a frame's G lanes reads a contiguous
//            64-B unit per round (units anchored at the frame end), so one
//            dwordx4 instruction touches 32 B of each of 32 lines
//   shape 1  16-B interleave: a round's G x 64 B span is read by four
//            instructions, instruction q covering [q 16G, (q + 1) 16G) with
//            lane g at 16 g (one instruction reads 16G contiguous bytes per
//            frame); a lane then hashes four 16-B pieces per round with a gap
//            step of (G - 1) x 16 B after each (4 maps per round, not 1)
//   PF       rounds issued ahead of the one hashed: 1, the product's (two
//            named round buffers; a first version that copied a buffer before
//            refilling it compiled to a full vmcnt(0) wait before every refill)
//   ST       one 4-B store per frame (lane G - 1), as the product
// 1,100-B frames at a 1,104-B stride (3.2 GB, the u1100d batch), G = 4, one
// 1024-thread workgroup per CU, waves grid-stride over groups of 16 frames.
// The CRCs are not the product's (no merge, no tail bytes): timing only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "crc_device.hpp"

using namespace vcrc;

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);           \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kG = 4, kGPW = 64 / kG;

__global__ void k_fill(u32x4 *p, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z ^= z >> 29;
        p[i] = u32x4{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)(z * 3), (uint32_t)i};
    }
}

struct Args {
    const uint8_t *base;  // frame 0 at base (512 B of slack in front: round 0 starts before its frame)
    uint64_t n;
    uint32_t L, stride;
    const uint32_t *consts;
    uint32_t *out;
};

template <int SHAPE>
__device__ __forceinline__ void issue(uint32_t (&w)[16], gu8 *fp, int64_t span, int g)
{
    if (SHAPE == 0) {
        // unit: 64 contiguous bytes at span + 64 g
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4u v = *reinterpret_cast<gu32x4u *>(fp + span + 64 * g + 16 * q);
            w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const u32x4u v = *reinterpret_cast<gu32x4u *>(fp + span + 16 * kG * q + 16 * g);
            w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
        }
    }
}

template <int SHAPE>
__device__ __forceinline__ uint32_t hash_round(uint32_t acc, const uint32_t (&w)[16], const SliceBases &sb, uint32_t gmap,
                                               uint32_t gmap16)
{
    if (SHAPE == 0) {
        acc = map_apply(acc, gmap);
#pragma unroll
        for (int i = 0; i < 16; i++) acc = s4_step(acc, w[i], sb);
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            acc = map_apply(acc, gmap16);
#pragma unroll
            for (int i = 0; i < 4; i++) acc = s4_step(acc, w[4 * q + i], sb);
        }
    }
    return acc;
}

// Two named round buffers, hashed alternately; a buffer is refilled with the
// round two ahead right after it is hashed, so one round is always in flight
// behind the one being hashed (the product's PF = 1) and no register copy
// makes the compiler wait for the prefetched round early.
template <int SHAPE, int PF, bool ST>
__global__ __launch_bounds__(1024) void k_pat(const Args a)
{
    static_assert(PF == 1, "double-buffered rounds");
    build_lds_tables(a.consts);
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane % kG;
    const SliceBases sb = slice_bases((uint32_t)(lane & 31) << 2);
    const uint64_t wave = ((uint64_t)blockIdx.x * 1024 + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * 1024) >> 6;
    const uint64_t groups = (a.n + kGPW - 1) / kGPW;
    const uint32_t gmap = gap_map(ilog2(kG));  // (G - 1) x 64 B
    const uint32_t gmap16 = pow_map(0);        // stand-in map for the 16-B interleave's (G - 1) x 16 B step
    uint32_t acc_all = 0;
    for (uint64_t grp = wave; grp < groups; grp += nw) {
        const uint64_t f = grp * kGPW + lane / kG;
        const bool act = f < a.n;
        const uint32_t L = act ? a.L : 0u;
        const uint32_t span = 64u * kG;
        const uint32_t R = (L + span - 1) / span;
        gu8 *fp = gptr(a.base) + f * a.stride;
        const int64_t s0 = (int64_t)L - (int64_t)R * span;  // round 0's span start (may be < 0: front padding)
        uint32_t A[16], B[16];
        if (R > 0) issue<SHAPE>(A, fp, s0, g);
        if (R > 1) issue<SHAPE>(B, fp, s0 + span, g);
        uint32_t acc = 0;
        for (uint32_t r = 0; r < R; r += 2) {
            acc = hash_round<SHAPE>(acc, A, sb, gmap, gmap16);
            if (r + 2 < R) issue<SHAPE>(A, fp, s0 + (int64_t)(r + 2) * span, g);
            if (r + 1 < R) {
                acc = hash_round<SHAPE>(acc, B, sb, gmap, gmap16);
                if (r + 3 < R) issue<SHAPE>(B, fp, s0 + (int64_t)(r + 3) * span, g);
            }
        }
        acc ^= __shfl_xor(acc, 1);
        acc ^= __shfl_xor(acc, 2);
        if (ST && act && g == kG - 1) a.out[f] = acc;
        acc_all ^= acc;
    }
    if (acc_all == 0x9u) a.out[0] = acc_all;
}

template <typename F>
float timeit(F f, int reps = 9)
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

int main(int argc, char **argv)
{
    const uint32_t L = argc > 1 ? (uint32_t)atoi(argv[1]) : 1100u;
    const uint32_t stride = L + 4;
    const uint64_t n = (3ull << 30) / stride;
    hipDeviceProp_t pr;
    CHECK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    // round 0's span starts up to 64 G - 1 = 255 B before a frame: 512 B of slack in front
    const size_t bytes = (size_t)n * stride + 1024;
    uint8_t *d;
    uint32_t *out, *consts;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&out, n * 4 + 64));
    std::vector<uint32_t> blob(kConstWords);
    fill_const_blob(blob.data());
    CHECK(hipMalloc(&consts, blob.size() * 4));
    CHECK(hipMemcpy(consts, blob.data(), blob.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (u32x4 *)d, bytes / 16);
    CHECK(hipDeviceSynchronize());
    Args a{d + 512, n, L, stride, consts, out};
    const double crc_bytes = (double)n * L;
#define RUN(S, P, T, name)                                                                                     \
    {                                                                                                          \
        const float ms = timeit([&] { hipLaunchKernelGGL((k_pat<S, P, T>), dim3(cus), dim3(1024), 0, 0, a); }); \
        printf("L=%u %-16s %.4f ms  %7.1f GB/s of CRC input\n", L, name, ms, crc_bytes / ms / 1e6);             \
        fflush(stdout);                                                                                        \
    }
    for (int rep = 0; rep < 2; rep++) {
        RUN(0, 1, false, "unit64 pf1")
        RUN(0, 1, true, "unit64 pf1 st")
        RUN(1, 1, false, "ilv16 pf1")
        RUN(1, 1, true, "ilv16 pf1 st")
    }
    printf("done\n");
    return 0;
}
