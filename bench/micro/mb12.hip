// Microbenchmark 12 (not product code): where do cfg3's last 4% go? On one
// box mb2's frames_read (G = 8, 16,384 B read from each frame's start, no
// prefetch) ran at 2.681 ms while k_frames<8,1> took 2.787 ms for the 16,400 B
// of CRC input per frame (3.8% slower per byte). The product's load pattern
// is rebuilt here step by step, XOR only (k_frames measured no faster without
// its table work), 1 M frames at a 16,404-B stride, G = 8 lanes per frame:
//   start16384  mb2: units at fp + 64u, u < 256, loop: 4 loads, wait, XOR
//   end16400    units anchored at the frame end (fp + 16 + 64u) plus unit 0 =
//               the first 16 B as 4 dword loads by lane 7, issued with round 1
//   end16400pf  the same with the next round issued before the current one is
//               consumed (k_frames PF = 1)
//   end16400hdr end16400pf + the header's 2 dwords + one output store per frame
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
typedef const uint32_t __attribute__((address_space(1))) gu32;

constexpr uint32_t kN = 1u << 20, kStride = 16404, kL = 16400, kG = 8;

__global__ void k_fill(u32x4 *p, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z ^= z >> 29;
        p[i] = u32x4{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)(z * 3), (uint32_t)i};
    }
}

__device__ __forceinline__ uint32_t x4(gu8 *up)
{
    uint32_t a = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const u32x4u v = *(gu32x4u *)(up + 16 * q);
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    return a;
}

// MODE 0 start16384, 1 end16400, 2 end16400pf, 3 end16400hdr
template <int MODE>
__global__ __launch_bounds__(1024) void k_pat(const uint8_t *base, uint32_t *out)
{
    const int lane = threadIdx.x & 63, g = lane % kG, grp = lane / kG;
    constexpr int GPW = 64 / kG;
    const uint64_t wave = ((uint64_t)blockIdx.x * 1024 + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * 1024) >> 6;
    uint32_t acc = 0;
    for (uint64_t fb = wave * GPW; fb < kN; fb += nw * GPW) {
        const uint64_t f = fb + grp;
        gu8 *fp = (gu8 *)base + f * kStride;
        if (MODE == 0) {
            for (uint32_t u = g; u < 256; u += kG) acc ^= x4(fp + (uint64_t)u * 64);
            continue;
        }
        gu8 *up = fp + 16 + (uint64_t)g * 64;  // unit 1 + g (units 1..256 are full)
        uint32_t u0 = 0, h0 = 0, h1 = 0;
        if (g == kG - 1) {
#pragma unroll
            for (int i = 0; i < 4; i++) u0 ^= *(gu32 *)(fp + 4 * i);
            if (MODE == 3) {
                h0 = *(gu32 *)fp;
                h1 = *(gu32 *)(fp + 4);
            }
        }
        if (MODE == 1) {
            for (uint32_t r = 0; r < 32; r++) acc ^= x4(up + (uint64_t)r * kG * 64);
        } else {
            u32x4u nx[4];
#pragma unroll
            for (int q = 0; q < 4; q++) nx[q] = *(gu32x4u *)(up + 16 * q);
            for (uint32_t r = 0; r < 32; r++) {
                u32x4u cur[4];
#pragma unroll
                for (int q = 0; q < 4; q++) cur[q] = nx[q];
                if (r + 1 < 32)
#pragma unroll
                    for (int q = 0; q < 4; q++) nx[q] = *(gu32x4u *)(up + (uint64_t)(r + 1) * kG * 64 + 16 * q);
#pragma unroll
                for (int q = 0; q < 4; q++) acc ^= cur[q].x ^ cur[q].y ^ cur[q].z ^ cur[q].w;
            }
        }
        acc ^= u0;
        if (MODE == 3) {
            acc ^= h0 + h1;
            if (g == kG - 1) out[16 + f] = acc;
        }
    }
    if (acc == 0x9u) out[0] = acc;
}

template <typename F> float timeit(F f, int reps = 7)
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
    const size_t bytes = (size_t)kN * kStride;
    uint8_t *d;
    uint32_t *out;
    CHECK(hipMalloc(&d, bytes + 4096));
    CHECK(hipMalloc(&out, (16 + kN) * 4));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (u32x4 *)d, (bytes + 4096) / 16);
    CHECK(hipDeviceSynchronize());
#define RUN(M, name, per)                                                                                              \
    {                                                                                                                  \
        const float ms = timeit([&] { hipLaunchKernelGGL((k_pat<M>), dim3(cus), dim3(1024), 0, 0, d, out); });        \
        printf("%-14s %.3f ms  %7.1f GB/s of %u B per frame; time per 16,400 B: %.3f ms\n", name, ms,                 \
               (double)kN * per / ms / 1e6, per, ms * 16400.0 / per);                                                \
        fflush(stdout);                                                                                                \
    }
    for (int rep = 0; rep < 2; rep++) {
        RUN(0, "start16384", 16384u)
        RUN(1, "end16400", 16400u)
        RUN(2, "end16400pf", 16400u)
        RUN(3, "end16400hdr", 16400u)
    }
    printf("done\n");
    return 0;
}
