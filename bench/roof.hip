// Same-box achievable read roof for bench.py (measurement only, not the
// product): a plain read-only stream over the bench's own frame buffer, the
// shape that read fastest with plain loads in bench/micro (mb1/mb2 "slice128":
// one 1024-thread workgroup per CU, each lane reading 128 contiguous bytes per
// step with eight dwordx4 loads, grid-strided). SURVEY 8(d): "also measure a
// plain read-only streaming kernel as the achievable peak". The XOR of
// everything read goes to *sink so nothing is optimised away.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(1024) void k_read_roof(const u32x4 *p, uint64_t n128, uint32_t *sink)
{
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, lanes = (uint64_t)gridDim.x * blockDim.x;
    u32x4 acc = {0, 0, 0, 0};
    for (uint64_t i = lane; i < n128; i += lanes) {
        const u32x4 *q = p + i * 8;
        u32x4 v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = q[j];
#pragma unroll
        for (int j = 0; j < 8; j++) acc ^= v[j];
    }
    const uint32_t x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9E3779B9u) *sink = x;  // practically never taken: keeps the loads live
}

extern "C" int val_bench_read_roof(const void *buf, uint64_t bytes, uint32_t *sink, void *stream)
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_read_roof, dim3(cus), dim3(1024), 0, (hipStream_t)stream, (const u32x4 *)buf, bytes / 128, sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
