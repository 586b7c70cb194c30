// Minimal reproducer for the round-1 hazards behind DESIGN.md "Correctness
// hazards" (diagnostic, not product code). Each iteration:
//   mode 0: fill a reused PAGEABLE host buffer with pattern(it), hipMemcpyAsync
//           it H2D on a non-blocking stream, launch a checker kernel on the
//           same stream, hipStreamSynchronize;
//   mode 1: the same from PINNED memory (the product's path);
//   mode 2: pinned copy into a fresh hipMallocAsync block per iteration, freed
//           with hipFreeAsync after the checker (the old per-call scratch).
// The checker counts words that differ from pattern(it): any count > 0 means
// the kernel saw bytes the stream order says it cannot see.
// usage: repro_pageable MODE BYTES ITERS
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } } while (0)

__host__ __device__ inline uint32_t pattern(uint32_t it, uint32_t i) { return (it * 0x9E3779B1u) ^ (i * 0x85EBCA6Bu); }

__global__ void k_check(const uint32_t *d, uint32_t n, uint32_t it, uint32_t *bad)
{
    uint32_t local = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) local += d[i] != pattern(it, i);
    if (local) atomicAdd(bad, local);
}

int main(int argc, char **argv)
{
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const size_t bytes = argc > 2 ? strtoull(argv[2], nullptr, 0) : (70u << 10);
    const int iters = argc > 3 ? atoi(argv[3]) : 3000;
    const uint32_t n = (uint32_t)(bytes / 4);
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    uint32_t *h = nullptr, *d = nullptr, *bad = nullptr;
    if (mode == 0) h = (uint32_t *)malloc(bytes);
    else CHECK(hipHostMalloc((void **)&h, bytes, hipHostMallocDefault));
    if (mode != 2) CHECK(hipMalloc((void **)&d, bytes));
    CHECK(hipHostMalloc((void **)&bad, 4, hipHostMallocDefault));
    *bad = 0;
    int bad_iters = 0;
    for (int it = 0; it < iters; it++) {
        for (uint32_t i = 0; i < n; i++) h[i] = pattern((uint32_t)it, i);
        uint32_t *dst = d;
        if (mode == 2) CHECK(hipMallocAsync((void **)&dst, bytes, s));
        CHECK(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, s));
        const uint32_t before = *bad;
        hipLaunchKernelGGL(k_check, dim3(64), dim3(256), 0, s, dst, n, (uint32_t)it, bad);
        CHECK(hipGetLastError());
        if (mode == 2) CHECK(hipFreeAsync(dst, s));
        CHECK(hipStreamSynchronize(s));
        bad_iters += *bad != before;
    }
    printf("repro_pageable mode=%d bytes=%zu iters=%d bad_iterations=%d bad_words=%u\n", mode, bytes, iters, bad_iters, *bad);
    return 0;
}
