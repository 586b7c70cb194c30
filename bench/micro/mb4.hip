// Microbenchmark 4: steady-state CRC loop (gap step + table steps per unit)
// over a contiguous 16 GiB stream, to choose table layout x load path before
// restructuring the frames kernel. Each wave streams rounds of 64 lanes x UNIT
// bytes; lane l owns unit l of every round (the frames kernel at G = 64).
//   TAB 0: slice-by-4, 32 bank replicas (128 KiB)   -- current product layout
//   TAB 1: slice-by-4, 16 bank replicas (64 KiB)    -- 2 lanes per bank per half-wave
//   TAB 2: slice-by-2, 32 bank replicas (64 KiB)    -- two dependent lookups per word
//   LOAD 0: global_load_dwordx4 to VGPRs, next round prefetched (current product)
//   LOAD 1: LDS-DMA nt, single buffer: issue round, wait, ds_read_b128, hash
//   LOAD 2: LDS-DMA nt, double buffer: issue round k+1, wait round k, hash k
// Results are not CRCs of anything (tables are synthetic); only time matters.
// Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);}}while(0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(u32x4* p, size_t n){ size_t i=(size_t)blockIdx.x*blockDim.x+threadIdx.x, st=(size_t)gridDim.x*blockDim.x;
  for(; i<n; i+=st){ uint64_t z=i*0x9E3779B97F4A7C15ull; z^=z>>29; p[i]=u32x4{(uint32_t)z,(uint32_t)(z>>32),(uint32_t)(z*3),(uint32_t)i}; } }

__shared__ uint32_t s_lds[160 * 256];
__device__ __forceinline__ uint32_t lr(uint32_t a){ return *(const uint32_t*)((const char*)s_lds + a); }
__device__ __forceinline__ uint32_t perm(uint32_t y, uint32_t base, int k){ return __builtin_amdgcn_perm(y, base, 0x0C020400u + ((uint32_t)k << 8)); }

// table geometry: TAB 0: row 256 B (two tables x 32 reps), pairs at 0 / 64K
//                 TAB 1: row 256 B holds four tables x 16 reps (64 B each)
//                 TAB 2: row 256 B holds two tables x 32 reps
template<int TAB> struct Tab {
  static constexpr uint32_t bytes = TAB == 0 ? 131072u : 65536u;
  uint32_t b0, b1, b2, b3;
  __device__ Tab(int lane){
    if (TAB == 0){ uint32_t lo=(lane&31)<<2; b0=lo; b1=128+lo; b2=65536+lo; b3=65536+128+lo; }
    else if (TAB == 1){ uint32_t lo=(lane&15)<<2; b0=lo; b1=64+lo; b2=128+lo; b3=192+lo; }
    else { uint32_t lo=(lane&31)<<2; b0=lo; b1=128+lo; b2=b0; b3=b1; }
  }
  __device__ __forceinline__ uint32_t step(uint32_t c, uint32_t w) const {
    uint32_t y=c^w;
    if (TAB == 2){
      uint32_t t=lr(perm(y,b0,0))^lr(perm(y,b1,1))^(y>>16);
      return lr(perm(t,b0,0))^lr(perm(t,b1,1))^(t>>16);
    }
    return lr(perm(y,b0,0))^lr(perm(y,b1,1))^lr(perm(y,b2,2))^lr(perm(y,b3,3));
  }
};
// gap map: 8 nibble tables x 16 rows x 16 reps (8 KiB) at gbase
__device__ __forceinline__ uint32_t gap(uint32_t a, uint32_t gbase, uint32_t lo){
  uint32_t r=0;
#pragma unroll
  for(int k=0;k<8;k++) r^=lr(gbase+k*1024u+((a>>(4*k))&15u)*64u+lo);
  return r; }

template<int TAB> __device__ void build(uint32_t gbase){
  for(uint32_t i=threadIdx.x;i<Tab<TAB>::bytes/4;i+=blockDim.x) s_lds[i]=i*0x9E3779B1u;
  for(uint32_t i=threadIdx.x;i<2048;i+=blockDim.x) s_lds[gbase/4+i]=i*0x85EBCA6Bu;
  __syncthreads(); }

template<int TAB, int LOAD, int UNIT, int AUX=2>
__global__ __launch_bounds__(1024) void k_crc(const uint8_t* p, size_t bytes, uint32_t* out){
  constexpr uint32_t W=UNIT/4, Q=UNIT/16;            // words / DMA instructions per round
  constexpr uint32_t gbase=Tab<TAB>::bytes;
  constexpr uint32_t sbase=gbase+8192;                 // staging
  build<TAB>(gbase);
  const int lane=threadIdx.x&63, wid=threadIdx.x>>6;
  Tab<TAB> tb(lane);
  const uint32_t glo=(lane&15)<<2;
  const uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  const size_t rb=64*UNIT;                             // bytes per wave-round
  const size_t nr=bytes/rb;
  uint32_t acc=0;
  if (LOAD==0){
    u32x4 nx[Q];
    size_t r=w;
    if(r<nr){
#pragma unroll
      for(int q=0;q<(int)Q;q++) nx[q]=*(const u32x4*)(p+r*rb+lane*UNIT+16*q);
    }
    for(;r<nr;r+=nw){
      u32x4 cur[Q];
#pragma unroll
      for(int q=0;q<(int)Q;q++) cur[q]=nx[q];
      if(r+nw<nr){
#pragma unroll
        for(int q=0;q<(int)Q;q++) nx[q]=*(const u32x4*)(p+(r+nw)*rb+lane*UNIT+16*q);
      }
      acc=gap(acc,gbase,glo);
#pragma unroll
      for(int q=0;q<(int)Q;q++){ acc=tb.step(acc,cur[q].x); acc=tb.step(acc,cur[q].y); acc=tb.step(acc,cur[q].z); acc=tb.step(acc,cur[q].w); }
    }
  } else if (LOAD==1){
    // single buffer: Q DMA instructions per round; instruction q loads piece q of every lane's unit
    const uint32_t mine=sbase+wid*Q*1024;
    for(size_t r=w;r<nr;r+=nw){
#pragma unroll
      for(int q=0;q<(int)Q;q++) __builtin_amdgcn_global_load_lds((const void*)(p+r*rb+lane*UNIT+16*q), (__attribute__((address_space(3))) void*)((char*)s_lds+mine+q*1024), 16, 0, AUX);
      __builtin_amdgcn_s_waitcnt(0x0f70);
      acc=gap(acc,gbase,glo);
#pragma unroll
      for(int q=0;q<(int)Q;q++){ u32x4 v=*(const u32x4*)((const char*)s_lds+mine+q*1024+lane*16);
        acc=tb.step(acc,v.x); acc=tb.step(acc,v.y); acc=tb.step(acc,v.z); acc=tb.step(acc,v.w); }
    }
  } else if (LOAD==3){
    // triple buffer: rounds k+1 and k+2 in flight while k hashes
    const uint32_t mine=sbase+wid*3*Q*1024;
    size_t r=w; int slot=0;
#pragma unroll
    for(int a=0;a<2;a++){ const size_t ra=r+a*nw; if(ra<nr){
#pragma unroll
      for(int q=0;q<(int)Q;q++) __builtin_amdgcn_global_load_lds((const void*)(p+ra*rb+lane*UNIT+16*q), (__attribute__((address_space(3))) void*)((char*)s_lds+mine+a*Q*1024+q*1024), 16, 0, AUX); } }
    for(;r<nr;r+=nw){
      const uint32_t cur=mine+slot*Q*1024;
      const int s2=slot==0?2:slot-1;
      if(r+2*nw<nr){
#pragma unroll
        for(int q=0;q<(int)Q;q++) __builtin_amdgcn_global_load_lds((const void*)(p+(r+2*nw)*rb+lane*UNIT+16*q), (__attribute__((address_space(3))) void*)((char*)s_lds+mine+s2*Q*1024+q*1024), 16, 0, AUX);
        __builtin_amdgcn_s_waitcnt(0x0f70 | (2*Q));
      } else if(r+nw<nr) __builtin_amdgcn_s_waitcnt(0x0f70 | Q); else __builtin_amdgcn_s_waitcnt(0x0f70);
      acc=gap(acc,gbase,glo);
#pragma unroll
      for(int q=0;q<(int)Q;q++){ u32x4 v=*(const u32x4*)((const char*)s_lds+cur+q*1024+lane*16);
        acc=tb.step(acc,v.x); acc=tb.step(acc,v.y); acc=tb.step(acc,v.z); acc=tb.step(acc,v.w); }
      slot=slot==2?0:slot+1;
    }
  } else {
    const uint32_t mine=sbase+wid*2*Q*1024;
    size_t r=w; int slot=0;
    if(r<nr){
#pragma unroll
      for(int q=0;q<(int)Q;q++) __builtin_amdgcn_global_load_lds((const void*)(p+r*rb+lane*UNIT+16*q), (__attribute__((address_space(3))) void*)((char*)s_lds+mine+q*1024), 16, 0, AUX);
    }
    for(;r<nr;r+=nw){
      const uint32_t cur=mine+slot*Q*1024, nxs=mine+(slot^1)*Q*1024;
      if(r+nw<nr){
#pragma unroll
        for(int q=0;q<(int)Q;q++) __builtin_amdgcn_global_load_lds((const void*)(p+(r+nw)*rb+lane*UNIT+16*q), (__attribute__((address_space(3))) void*)((char*)s_lds+nxs+q*1024), 16, 0, AUX);
        if(Q==2) __builtin_amdgcn_s_waitcnt(0x0f72); else __builtin_amdgcn_s_waitcnt(0x0f74);
      } else __builtin_amdgcn_s_waitcnt(0x0f70);
      acc=gap(acc,gbase,glo);
#pragma unroll
      for(int q=0;q<(int)Q;q++){ u32x4 v=*(const u32x4*)((const char*)s_lds+cur+q*1024+lane*16);
        acc=tb.step(acc,v.x); acc=tb.step(acc,v.y); acc=tb.step(acc,v.z); acc=tb.step(acc,v.w); }
      slot^=1;
    }
  }
  if(acc==0x12345u) out[0]=acc; }

template<typename F> float timeit(F f, int reps=5){ hipEvent_t a,b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); f(); CHECK(hipDeviceSynchronize());
  std::vector<float> t; for(int r=0;r<reps;r++){ CHECK(hipEventRecord(a)); f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms,a,b)); t.push_back(ms);}
  std::sort(t.begin(),t.end()); CHECK(hipGetLastError()); return t[t.size()/2]; }

int main(){
  hipDeviceProp_t pr; CHECK(hipGetDeviceProperties(&pr,0)); int cus=pr.multiProcessorCount;
  const size_t bytes=(size_t)16<<30;
  uint8_t* d; CHECK(hipMalloc(&d, bytes)); uint32_t* out; CHECK(hipMalloc(&out, 64));
  k_fill<<<4096,256>>>((u32x4*)d,bytes/16); CHECK(hipDeviceSynchronize());
  #define RUN(T,L,U,A,B) { float ms=timeit([&]{ k_crc<T,L,U,A><<<cus,B>>>(d,bytes,out); }); printf("tab=%d load=%d unit=%d aux=%d block=%d: %.3f ms %7.1f GB/s\n",T,L,U,A,B,ms,bytes/ms/1e6); fflush(stdout); }
  RUN(0,0,64,0,1024) RUN(2,0,64,0,1024)
  RUN(2,2,32,2,1024) RUN(2,2,32,0,1024) RUN(2,2,32,2,768) RUN(2,2,32,2,512)
  RUN(2,3,32,2,768) RUN(2,3,32,0,768) RUN(2,3,32,2,512) RUN(2,3,16,2,1024)
  RUN(2,2,16,2,1024) RUN(2,1,16,2,1024)
  printf("done\n"); return 0; }
