// Microbenchmark 6: workgroup dispatch ramp. Each wave stamps
// s_memrealtime (100 MHz) at entry; the spread of first-instruction times over
// the grid is the dispatch ramp. Variants: block size, LDS per block, VGPRs
// (a kernel that keeps many registers live), code size. Not product code.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);}}while(0)

__device__ uint64_t g_t[65536];

template <int LDS_KB>
__global__ void k_stamp(uint32_t *out)
{
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) g_t[w] = t;
    if (LDS_KB > 0) {
        __shared__ uint32_t lds[LDS_KB > 0 ? LDS_KB * 256 : 1];
        lds[threadIdx.x] = threadIdx.x;
        __syncthreads();
        if (lds[(threadIdx.x + 1) % blockDim.x] == 7777u) out[0] = 1;
    }
}

// many live VGPRs: 96 values carried through a loop the compiler cannot fold
__global__ __launch_bounds__(1024) void k_stamp_vgpr(uint32_t *out, int iters)
{
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) g_t[w] = t;
    __shared__ uint32_t lds[160 * 256 - 64];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint32_t v[96];
#pragma unroll
    for (int i = 0; i < 96; i++) v[i] = lds[(threadIdx.x + i) & 1023];
    for (int k = 0; k < iters; k++) {
#pragma unroll
        for (int i = 0; i < 96; i++) v[i] = v[i] * 3u + v[(i + 1) % 96];
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 96; i++) x ^= v[i];
    if (x == 7777u) out[0] = x;
}

static void report(const char *name, int nwaves)
{
    std::vector<uint64_t> t(nwaves);
    CHECK(hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_t), nwaves * 8));
    const uint64_t t0 = *std::min_element(t.begin(), t.end());
    std::vector<double> us(nwaves);
    for (int i = 0; i < nwaves; i++) us[i] = (t[i] - t0) / 100.0;
    std::sort(us.begin(), us.end());
    printf("%-34s waves=%5d start spread p50 %5.2f p90 %5.2f max %5.2f us\n", name, nwaves, us[nwaves / 2], us[nwaves * 9 / 10],
           us[nwaves - 1]);
}

int main()
{
    hipDeviceProp_t pr;
    CHECK(hipGetDeviceProperties(&pr, 0));
    const int cus = pr.multiProcessorCount;
    uint32_t *out;
    CHECK(hipMalloc(&out, 64));
#define RUN(name, launch, nw)                                     \
    for (int r = 0; r < 3; r++) { launch; CHECK(hipDeviceSynchronize()); } \
    report(name, nw);
    RUN("1024 thr, no LDS, 256 blk", (k_stamp<0><<<cus, 1024>>>(out)), cus * 16)
    RUN("1024 thr, 64 KiB LDS, 256 blk", (k_stamp<64><<<cus, 1024>>>(out)), cus * 16)
    RUN("1024 thr, 150 KiB LDS, 256 blk", (k_stamp<150><<<cus, 1024>>>(out)), cus * 16)
    RUN("256 thr, no LDS, 1024 blk", (k_stamp<0><<<cus * 4, 256>>>(out)), cus * 16)
    RUN("256 thr, 32 KiB LDS, 1024 blk", (k_stamp<32><<<cus * 4, 256>>>(out)), cus * 16)
    RUN("512 thr, 64 KiB LDS, 512 blk", (k_stamp<64><<<cus * 2, 512>>>(out)), cus * 16)
    RUN("1024 thr, 160 KiB LDS, ~100 VGPR", (k_stamp_vgpr<<<cus, 1024>>>(out, 1)), cus * 16)
    printf("done\n");
    return 0;
}
