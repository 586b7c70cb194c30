// Microbenchmark 15 (not product code): cost ladder of a stream-sliced
// short-frame kernel. Each wave owns a contiguous region of the
// packed frame stream and walks it 4 KiB per round: four dwordx4 instructions
// that each read 1 KiB contiguously (16 B per lane), the read shape that
// streamed at 6.11 TB/s in mb13. A quad transpose gives every lane one 64-B
// stream unit (lane 4k + j holds unit 16 j + k). Steps, each adding to the last:
//   0  read only (XOR of the words)
//   1  + the transpose and the slice-by-4 chain over the unit (16 steps)
//   2  + a frame boundary inside the unit cuts the chain (register saved,
//        chain restarted: two selects per step; boundary from the frame stride)
//   3  + a segmented scan over the wave's 64 units in stream order (6 levels:
//        shuffle, LDS map "advance 64 2^j", segment flags) and the carry of the
//        open frame into the next round ("advance 4 KiB")
//   4  + each frame's end: the saved prefix joined to the scan value of the
//        units before it, advanced over the cut (<= 63 B: one LDS map per set
//        bit), and a 4-B store per frame
// 1,100-B frames at a 1,104-B stride (3.2 GB, as u1100d), one 1024-thread
// workgroup per CU. The CRCs are not exact (the words around a cut are not
// split at the byte, region edges are not joined): timing only.
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

__global__ void k_fill(u32x4 *p, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z ^= z >> 29;
        p[i] = u32x4{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)(z * 3), (uint32_t)i};
    }
}

struct Args {
    const uint8_t *base;
    uint64_t region;  // bytes per wave (multiple of 4 KiB)
    uint32_t stride;  // frame stride (boundaries at multiples of it)
    const uint32_t *consts;
    uint32_t *out;
};

template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

// 4 x 4 transpose of 16-B chunks across a quad (as crc_kernels.hpp ilv_to_units<4>):
// lane j's register q holds chunk j of unit q; afterwards lane j holds unit j
__device__ __forceinline__ void ilv_quad(uint32_t (&w)[16], int g)
{
    const bool o1 = g & 1, o2 = g & 2;
#pragma unroll
    for (int q = 0; q < 4; q += 2)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t r = qperm<0xB1>(o1 ? w[4 * q + i] : w[4 * (q + 1) + i]);
            if (o1) w[4 * q + i] = r;
            else w[4 * (q + 1) + i] = r;
        }
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t r = qperm<0x4E>(o2 ? w[4 * q + i] : w[4 * (q + 2) + i]);
            if (o2) w[4 * q + i] = r;
            else w[4 * (q + 2) + i] = r;
        }
}

__device__ __forceinline__ void load_chunk(uint32_t (&w)[16], gu8 *chunk, int lane)
{
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const u32x4u v = *reinterpret_cast<gu32x4u *>(chunk + 1024 * q + 16 * lane);
        w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
    }
}

template <int STEP>
__device__ __forceinline__ uint32_t round_work(uint32_t (&w)[16], uint64_t chunk_off, int lane, uint32_t stride,
                                               const SliceBases &sb, uint32_t &carry, uint32_t *out, uint32_t &sink)
{
    if (STEP == 0) {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) x ^= w[i];
        return x;
    }
    ilv_quad(w, lane & 3);
    const uint32_t u = 16u * (uint32_t)(lane & 3) + (uint32_t)(lane >> 2);  // this lane's unit in the chunk
    const uint64_t uo = chunk_off + 64u * u;                                  // its stream offset
    // first frame boundary at or after the unit start, in words (16 = none in this unit)
    const uint32_t to_b = stride - (uint32_t)(uo % stride);
    const int cut = to_b < 64u ? (int)(to_b >> 2) : 16;
    uint32_t c = 0, pre = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        if (STEP >= 2) {
            pre = (i == cut) ? c : pre;
            c = (i == cut) ? 0u : c;
        }
        c = s4_step(c, w[i], sb);
    }
    if (STEP < 2) return c;
    if (STEP == 2) return c ^ pre;
    // segmented inclusive scan in unit order: unit u - d is lane - 4 d (d < 16)
    // or lane - d / 16 (d = 16, 32); a segment head (a cut) stops the carry in
    const bool head = cut < 16;
    uint32_t v = c;
    bool f = head;
#pragma unroll
    for (int j = 0; j < 6; j++) {
        const int d = 1 << j;
        const int src = j < 4 ? lane - 4 * d : lane - (d >> 4);
        const bool ok = j < 4 ? (lane >> 2) >= d : (lane & 3) >= (d >> 4);
        const uint32_t pv = __shfl(v, src < 0 ? 0 : src);
        const bool pf = __shfl((int)f, src < 0 ? 0 : src) != 0;
        const uint32_t adv = map_apply(pv, tree_map(j));
        v = (ok && !f) ? (v ^ adv) : v;
        f = f || (ok && pf);
    }
    // carry of the open frame from the previous round into units before the
    // first head of this round (no head at or before this unit)
    if (!f) v ^= map_apply(carry, pow_map(0));  // stand-in map for "advance 64 (u + 1) bytes"
    // next round's carry: unit 63 (lane 63's u = 16 * 3 + 15)
    const uint32_t last = __shfl(v, 63);
    carry = map_apply(last, pow_map(12));  // "advance 4 KiB"
    if (STEP == 3) return v ^ pre;
    // frame end in this unit: scan value of the units before it (unit u - 1),
    // advanced over the cut's 4 cut bytes, joined to the prefix
    const int srcm = (u == 0) ? 63 : (int)(4 * ((u - 1) & 15) + ((u - 1) >> 4));
    uint32_t before = __shfl(v, srcm);
    if (head) {
        const uint32_t nb = 4u * (uint32_t)cut;
#pragma unroll
        for (int k = 0; k < 6; k++)
            if ((nb >> k) & 1u) before = map_apply(before, pow_map(k));
        const uint32_t crc = before ^ pre;
        out[(uo + to_b) / stride] = crc;
    }
    return v;
}

template <int STEP>
__global__ __launch_bounds__(1024) void k_stream(const Args a)
{
    build_lds_tables(a.consts);
    lds_pow_maps(a.consts, 0);
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const SliceBases sb = slice_bases((uint32_t)(lane & 31) << 2);
    const uint64_t wave = ((uint64_t)blockIdx.x * 1024 + threadIdx.x) >> 6;
    const uint64_t r0 = wave * a.region, rounds = a.region >> 12;
    gu8 *b = gptr(a.base);
    uint32_t A[16], B[16], acc = 0, carry = 0, sink = 0;
    load_chunk(A, b + r0, lane);
    if (rounds > 1) load_chunk(B, b + r0 + 4096, lane);
    for (uint64_t r = 0; r < rounds; r += 2) {
        acc ^= round_work<STEP>(A, r0 + r * 4096, lane, a.stride, sb, carry, a.out, sink);
        if (r + 2 < rounds) load_chunk(A, b + r0 + (r + 2) * 4096, lane);
        if (r + 1 < rounds) {
            acc ^= round_work<STEP>(B, r0 + (r + 1) * 4096, lane, a.stride, sb, carry, a.out, sink);
            if (r + 3 < rounds) load_chunk(B, b + r0 + (r + 3) * 4096, lane);
        }
    }
    if ((acc ^ sink) == 0x9u) a.out[0] = acc;
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
    hipDeviceProp_t pr;
    CHECK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    const uint64_t waves = (uint64_t)cus * 16;
    const uint64_t region = ((3ull << 30) / waves) & ~4095ull;
    const uint64_t bytes = region * waves;
    const uint64_t n = bytes / stride + 1;
    uint8_t *d;
    uint32_t *out, *consts;
    CHECK(hipMalloc(&d, bytes + 4096));
    CHECK(hipMalloc(&out, n * 4 + 64));
    std::vector<uint32_t> blob(kConstWords);
    fill_const_blob(blob.data());
    CHECK(hipMalloc(&consts, blob.size() * 4));
    CHECK(hipMemcpy(consts, blob.data(), blob.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (u32x4 *)d, (bytes + 4096) / 16);
    CHECK(hipDeviceSynchronize());
    Args a{d, region, stride, consts, out};
    const double crc_bytes = (double)bytes * L / stride;  // the frames' share of the stream
#define RUN(S, name)                                                                                          \
    {                                                                                                         \
        const float ms = timeit([&] { hipLaunchKernelGGL((k_stream<S>), dim3(cus), dim3(1024), 0, 0, a); }); \
        printf("L=%u %-34s %.4f ms  %7.1f GB/s stream  %7.1f GB/s of CRC input\n", L, name, ms,              \
               (double)bytes / ms / 1e6, crc_bytes / ms / 1e6);                                               \
        fflush(stdout);                                                                                       \
    }
    for (int rep = 0; rep < 2; rep++) {
        RUN(0, "0 read only")
        RUN(1, "1 + transpose + chain")
        RUN(2, "2 + cut selects")
        RUN(3, "3 + segmented scan + carry")
        RUN(4, "4 + frame ends + store")
    }
    printf("done\n");
    return 0;
}
