// Microbenchmark 2: read-roof probes for the frames kernel's access pattern
// (no CRC math): G lanes per frame, 64-B units per lane, frames at a 16,404-B
// stride, plus plain streaming and LDS-DMA streaming references. Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);}}while(0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

__global__ void k_fill(u32x4* p, size_t n){ size_t i=(size_t)blockIdx.x*blockDim.x+threadIdx.x, st=(size_t)gridDim.x*blockDim.x;
  for(; i<n; i+=st){ uint64_t z=i*0x9E3779B97F4A7C15ull; z^=z>>29; p[i]=u32x4{(uint32_t)z,(uint32_t)(z>>32),(uint32_t)(z*3),(uint32_t)i}; } }

template<bool NT> __device__ __forceinline__ u32x4 ld(const uint8_t* p){
  if (NT) { const u32x4* q=(const u32x4*)p; return __builtin_nontemporal_load(q); }
  return *(const u32x4u*)p; }

// frames pattern: wave = 64/G frames; lane g of a frame reads unit u = g + G*k (64 B) each round
template<int G, bool NT> __global__ __launch_bounds__(1024) void k_frames_read(const uint8_t* base, uint64_t stride, uint32_t flen, uint32_t n, uint32_t* out){
  const int lane=threadIdx.x&63, g=lane%G, grp=lane/G; constexpr int GPW=64/G;
  uint64_t wave=((uint64_t)blockIdx.x*1024+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*1024)>>6;
  uint32_t acc=0; const uint32_t U=flen/64;
  for(uint64_t fb=wave*GPW; fb<n; fb+=nw*GPW){ uint64_t f=fb+grp; if(f>=n) continue; const uint8_t* fp=base+f*stride;
    for(uint32_t u=g; u<U; u+=G){ const uint8_t* up=fp+(uint64_t)u*64; u32x4 a=ld<NT>(up),b=ld<NT>(up+16),c=ld<NT>(up+32),d=ld<NT>(up+48);
      acc^=a.x^a.y^a.z^a.w^b.x^b.y^b.z^b.w^c.x^c.y^c.z^c.w^d.x^d.y^d.z^d.w; } }
  if(acc==0x9u) out[0]=acc; }

// contiguous slices (probe best): wave covers 64*SL bytes per iteration
template<int SL, bool NT> __global__ __launch_bounds__(1024) void k_slice(const uint8_t* p, size_t bytes, uint32_t* out){
  const int lane=threadIdx.x&63; uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/(64*SL); uint32_t acc=0;
  for(size_t c=w;c<nch;c+=nw){ const uint8_t* q=p+c*64*SL+(size_t)lane*SL;
#pragma unroll
    for(int j=0;j<SL/16;j++){ u32x4 a=ld<NT>(q+16*j); acc^=a.x^a.y^a.z^a.w; } }
  if(acc==0x9u) out[0]=acc; }

// LDS-DMA stream: each wave moves 1 KiB per instruction into its LDS slot, 4 in flight, then reads it back
template<int INFLIGHT> __global__ __launch_bounds__(1024) void k_ldsdma(const uint8_t* p, size_t bytes, uint32_t* out){
  __shared__ __attribute__((aligned(16))) uint8_t lds[16*INFLIGHT*1024];
  const int lane=threadIdx.x&63, wid=threadIdx.x>>6; uint8_t* mine=lds+wid*INFLIGHT*1024;
  uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/(INFLIGHT*1024); uint32_t acc=0;
  for(size_t c=w;c<nch;c+=nw){ const uint8_t* q=p+c*INFLIGHT*1024;
#pragma unroll
    for(int j=0;j<INFLIGHT;j++) __builtin_amdgcn_global_load_lds((const void*)(q+j*1024+lane*16), (__attribute__((address_space(3))) void*)(mine+j*1024), 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0)
#pragma unroll
    for(int j=0;j<INFLIGHT;j++){ u32x4 a=*(u32x4*)(mine+j*1024+lane*16); acc^=a.x^a.y^a.z^a.w; } }
  if(acc==0x9u) out[0]=acc; }

template<typename F> float timeit(F f, int reps=7){ hipEvent_t a,b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); f(); CHECK(hipDeviceSynchronize());
  std::vector<float> t; for(int r=0;r<reps;r++){ CHECK(hipEventRecord(a)); f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms,a,b)); t.push_back(ms);}
  std::sort(t.begin(),t.end()); CHECK(hipGetLastError()); return t[t.size()/2]; }

int main(){
  hipDeviceProp_t pr; CHECK(hipGetDeviceProperties(&pr,0)); int cus=pr.multiProcessorCount;
  const uint32_t n=1u<<20, flen=16384+16, stride=flen+4; size_t bytes=(size_t)n*stride;
  uint8_t* d; CHECK(hipMalloc(&d, bytes+4096)); uint32_t* out; CHECK(hipMalloc(&out, 64));
  k_fill<<<4096,256>>>((u32x4*)d,(bytes+4096)/16); CHECK(hipDeviceSynchronize());
  const uint32_t flen64 = 16384; // read 16 KiB of each frame (64-B units) -> algorithmic bytes
  #define FR(G,NT) { float ms=timeit([&]{ k_frames_read<G,NT><<<cus,1024>>>(d,stride,flen64,n,out); }); printf("frames_read G=%d nt=%d: %.3f ms %.1f GB/s\n",G,NT,ms,(double)n*flen64/ms/1e6); }
  FR(4,false) FR(8,false) FR(16,false) FR(8,true) FR(16,true)
  #define SLC(S,NT,B) { float ms=timeit([&]{ k_slice<S,NT><<<cus*B,1024>>>(d,bytes,out); }); printf("slice%d nt=%d blocks/CU=%d: %.3f ms %.1f GB/s\n",S,NT,B,ms,bytes/ms/1e6); }
  SLC(64,false,1) SLC(128,false,1) SLC(128,false,2) SLC(64,true,1) SLC(128,true,1) SLC(128,true,2)
  #define DMA(I) { float ms=timeit([&]{ k_ldsdma<I><<<cus,1024>>>(d,bytes,out); }); printf("ldsdma inflight=%d: %.3f ms %.1f GB/s\n",I,ms,bytes/ms/1e6); }
  DMA(2) DMA(4) DMA(8)
  printf("done\n"); return 0; }
