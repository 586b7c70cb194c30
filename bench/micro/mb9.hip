// Microbenchmark 9: LDS-DMA on the cfg3 frame layout with the DMA lanes
// remapped (not product code). mb8 fed each lane's own unit through DMA, so an
// instruction covered G x 16 B of a frame (128 B at G = 8) and the stream fell
// to 5.5 TB/s. Here the DMA lanes are decoupled from the hashing lanes: at
// G = 16 one instruction loads one frame's whole round (1 KiB contiguous), at
// G = 8 two frames' 512-B rounds; inside each 64-B unit the four 16-B pieces
// are rotated by (reader lane / 2) so the ds_read_b128 read-back of a unit is
// bank-conflict free. Frames: 1 M x 16,404-B stride; the 256 full units after
// the 16-B prefix are hashed (slice-by-2 with 32 bank replicas, 64 KiB, so
// 16 waves x 4 KiB of staging fit beside it), gap step between a lane's
// units, a log2(G) merge tree. Variants checked against each other (XOR of
// the merged frame registers).
//   plain<G>     global_load_dwordx4 into VGPRs, next round prefetched
//   dma<G,AUX,H> DMA round r+1 while hashing round r (H=0: XOR only = stream roof)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));
#define LDSP(x) ((__attribute__((address_space(3))) void *)(x))

constexpr uint32_t kN = 1u << 20, kStride = 16404, kUnits = 256;
__shared__ uint32_t s_lds[160 * 256];
__device__ __forceinline__ uint32_t lr(uint32_t a) { return *(const uint32_t *)((const char *)s_lds + a); }
__device__ __forceinline__ uint32_t perm(uint32_t y, uint32_t base, int k) { return __builtin_amdgcn_perm(y, base, 0x0C020400u + ((uint32_t)k << 8)); }
// slice-by-2, 32 replicas: T1 (advance 2 bytes) at [0, 32K), T0 at [32K, 64K); row = byte * 128 B
__device__ __forceinline__ uint32_t step2(uint32_t c, uint32_t w, uint32_t lo)
{
    uint32_t y = c ^ w;
    uint32_t t = lr(perm(y, lo, 0)) ^ lr(perm(y, 32768u + lo, 1)) ^ (y >> 16);
    return lr(perm(t, lo, 0)) ^ lr(perm(t, 32768u + lo, 1)) ^ (t >> 16);
}
constexpr uint32_t kMaps = 65536;                       // 8 nibble maps x 512 B (gap + merge levels)
constexpr uint32_t kStage = kMaps + 8 * 512;            // 16 waves x 4 KiB
__device__ __forceinline__ uint32_t mapply(uint32_t a, uint32_t m)
{
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= lr(m + k * 64u + ((a >> (4 * k)) & 15u) * 4u);
    return r;
}
__device__ void build()
{
    // synthetic tables (speed only): word i of the table area = hash(i)
    for (uint32_t i = threadIdx.x; i < kStage / 4; i += blockDim.x) s_lds[i] = i * 0x9E3779B1u ^ (i >> 7);
    __syncthreads();
}
__global__ void k_fill(u32x4 *p, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z ^= z >> 29;
        p[i] = u32x4{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)(z * 3), (uint32_t)i};
    }
}
template <int G>
__device__ __forceinline__ uint32_t merge(uint32_t acc, int g)
{
#pragma unroll
    for (int j = 0; (1 << j) < G; j++) {
        const uint32_t other = __shfl_xor(acc, 1 << j);
        const bool right = (g >> j) & 1;
        acc = mapply(right ? other : acc, kMaps + (1 + j) * 512u) ^ (right ? acc : other);
    }
    return acc;
}

template <int G>
__global__ __launch_bounds__(1024) void k_plain(const uint8_t *p, uint32_t *out)
{
    build();
    const int lane = threadIdx.x & 63, g = lane % G;
    const uint32_t lo = (uint32_t)(lane & 31) << 2;
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    constexpr uint32_t F = 64 / G, R = kUnits / G;
    uint32_t x = 0;
    for (uint32_t fg = w * F; fg < kN; fg += nw * F) {
        const uint8_t *fp = p + (size_t)(fg + lane / G) * kStride + 16 + g * 64;
        u32x4 nx[4], cur[4];
#pragma unroll
        for (int q = 0; q < 4; q++) nx[q] = *(const u32x4u *)(fp + 16 * q);
        uint32_t acc = 0;
        for (uint32_t r = 0; r < R; r++) {
#pragma unroll
            for (int q = 0; q < 4; q++) cur[q] = nx[q];
            if (r + 1 < R) {
#pragma unroll
                for (int q = 0; q < 4; q++) nx[q] = *(const u32x4u *)(fp + (r + 1) * G * 64 + 16 * q);
            }
            acc = mapply(acc, kMaps);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                acc = step2(acc, cur[q].x, lo);
                acc = step2(acc, cur[q].y, lo);
                acc = step2(acc, cur[q].z, lo);
                acc = step2(acc, cur[q].w, lo);
            }
        }
        acc = merge<G>(acc, g);
        if (g == G - 1) x ^= acc;
    }
    atomicXor(out, x);
}

// DMA: the wave's round = 64 units (F frames x G units); instruction q loads
// units [16q, 16q + 16) = frame (16q / G)'s units, 1 KiB (G = 16) or 2 x 512 B
// (G = 8) contiguous. Unit m sits at slot + 64 m; its piece k at position
// (k + m / 2) % 4.
template <int G, int AUX, int H>
__global__ __launch_bounds__(1024) void k_dma(const uint8_t *p, uint32_t *out)
{
    build();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane % G;
    const uint32_t lo = (uint32_t)(lane & 31) << 2;
    const uint32_t slot = kStage + (uint32_t)wid * 4096u;
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = (gridDim.x * blockDim.x) >> 6;
    constexpr uint32_t F = 64 / G, R = kUnits / G;
    // DMA lane `lane` of instruction q writes slot + q*1024 + lane*16: unit m = 16q + lane/4, position lane%4
    // -> it must load piece k = (pos - m/2) mod 4 of unit m (frame m / G, unit-in-round m % G)
    uint32_t src[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t m = 16u * q + (uint32_t)lane / 4u, pos = (uint32_t)lane & 3u;
        const uint32_t k = (pos - m / 2u) & 3u;
        src[q] = (m / G) * kStride + 16u + (m % G) * 64u + 16u * k;  // + frame-group base + round offset
    }
    uint32_t x = 0, xs = 0;
    const uint32_t rd = slot + (uint32_t)lane * 64u;
    for (uint32_t fg = w * F; fg < kN; fg += nw * F) {
        const uint8_t *gb = p + (size_t)fg * kStride;
#pragma unroll
        for (int q = 0; q < 4; q++)
            __builtin_amdgcn_global_load_lds((const void *)(gb + src[q]), LDSP((char *)s_lds + slot + q * 1024), 16, 0, AUX);
        uint32_t acc = 0;
        for (uint32_t r = 0; r < R; r++) {
            __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): round r landed
            u32x4 cur[4];
#pragma unroll
            for (int k = 0; k < 4; k++) cur[k] = *(const u32x4 *)((const char *)s_lds + rd + 16u * ((k + lane / 2) & 3));
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): slot free
            if (r + 1 < R) {
#pragma unroll
                for (int q = 0; q < 4; q++)
                    __builtin_amdgcn_global_load_lds((const void *)(gb + src[q] + (r + 1) * G * 64u),
                                                     LDSP((char *)s_lds + slot + q * 1024), 16, 0, AUX);
            }
            if (H) {
                acc = mapply(acc, kMaps);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    acc = step2(acc, cur[k].x, lo);
                    acc = step2(acc, cur[k].y, lo);
                    acc = step2(acc, cur[k].z, lo);
                    acc = step2(acc, cur[k].w, lo);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++) xs ^= cur[k].x ^ cur[k].y ^ cur[k].z ^ cur[k].w;
            }
        }
        if (H) {
            acc = merge<G>(acc, g);
            if (g == G - 1) x ^= acc;
        }
    }
    atomicXor(out, H ? x : xs);
}

template <typename F> float timeit(F f, int reps = 5)
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
    CHECK(hipMalloc(&d, bytes + 64));
    uint32_t *out;
    CHECK(hipMalloc(&out, 64));
    k_fill<<<4096, 256>>>((u32x4 *)d, (bytes + 63) / 16);
    CHECK(hipDeviceSynchronize());
    const double hashed = (double)kN * kUnits * 64;  // bytes hashed per launch
    uint32_t h[16], ref8 = 0, ref16 = 0;
#define RUN(name, G, ...)                                                                                        \
    {                                                                                                            \
        CHECK(hipMemset(out, 0, 64));                                                                            \
        { __VA_ARGS__; }                                                                                         \
        CHECK(hipDeviceSynchronize());                                                                           \
        CHECK(hipMemcpy(h, out, 64, hipMemcpyDeviceToHost));                                                     \
        uint32_t &ref = (G == 8) ? ref8 : ref16;                                                                 \
        const char *ok = "";                                                                                     \
        if (strstr(name, "stream") == nullptr) { if (!ref) ref = h[0]; ok = (h[0] == ref) ? "same" : "MISMATCH"; } \
        float ms = timeit([&] { __VA_ARGS__; });                                                                 \
        printf("%-22s %.3f ms %7.1f GB/s hashed  %s\n", name, ms, hashed / ms / 1e6, ok);                          \
        fflush(stdout);                                                                                          \
    }
    RUN("plain G8", 8, (k_plain<8><<<cus, 1024>>>(d, out)))
    RUN("plain G16", 16, (k_plain<16><<<cus, 1024>>>(d, out)))
    RUN("dma stream G16 aux2", 16, (k_dma<16, 2, 0><<<cus, 1024>>>(d, out)))
    RUN("dma stream G8 aux2", 8, (k_dma<8, 2, 0><<<cus, 1024>>>(d, out)))
    RUN("dma G16 aux2", 16, (k_dma<16, 2, 1><<<cus, 1024>>>(d, out)))
    RUN("dma G8 aux2", 8, (k_dma<8, 2, 1><<<cus, 1024>>>(d, out)))
    RUN("dma G16 aux0", 16, (k_dma<16, 0, 1><<<cus, 1024>>>(d, out)))
    RUN("plain G8 (again)", 8, (k_plain<8><<<cus, 1024>>>(d, out)))
    RUN("dma G16 aux2 (again)", 16, (k_dma<16, 2, 1><<<cus, 1024>>>(d, out)))
    printf("done\n");
    return 0;
}
