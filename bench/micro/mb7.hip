// Microbenchmark 7: LDS-DMA with full-line instructions beside the CRC loop.
// mb4's DMA variants let instruction q read 16 B of every lane's unit
// (lane*UNIT + 16q), so each instruction touched 16 lines by halves. Here a
// round is 64 lanes x 64 B = 4 KiB and instruction q reads the contiguous
// 1 KiB [q*1024, q*1024+1024) of it: lane l = 16k + j loads piece 4j + k of
// that KiB, i.e. the 16-B piece k of unit 16q + j. The LDS image is then the
// transpose that makes each ds_read_b128 lane group (16 lanes, every value
// of m % 16 once) hit 16 distinct slots of the 256-B bank row.
//   plain     : global_load_dwordx4 into VGPRs, next round prefetched (mb4 LOAD 0)
//   dma<AUX>  : wait round r, ds_read_b128 x4, issue round r+1's DMA into the
//               same slot, hash round r from VGPRs (4 KiB in flight per wave)
//   dmas<AUX> : the same schedule with the hash replaced by an XOR (roof)
//   TAB 1: slice-by-4, 16 bank replicas; TAB 2: slice-by-2, 32 replicas (64 KiB)
// The result check compares the XOR of everything each variant read.
// Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);}}while(0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define LDSP(x) ((__attribute__((address_space(3))) void*)(x))

__global__ void k_fill(u32x4* p, size_t n){ size_t i=(size_t)blockIdx.x*blockDim.x+threadIdx.x, st=(size_t)gridDim.x*blockDim.x;
  for(; i<n; i+=st){ uint64_t z=i*0x9E3779B97F4A7C15ull; z^=z>>29; p[i]=u32x4{(uint32_t)z,(uint32_t)(z>>32),(uint32_t)(z*3),(uint32_t)i}; } }

__shared__ uint32_t s_lds[160 * 256];
__device__ __forceinline__ uint32_t lr(uint32_t a){ return *(const uint32_t*)((const char*)s_lds + a); }
__device__ __forceinline__ uint32_t perm(uint32_t y, uint32_t base, int k){ return __builtin_amdgcn_perm(y, base, 0x0C020400u + ((uint32_t)k << 8)); }

template<int TAB> struct Tab {
  uint32_t b0, b1, b2, b3;
  __device__ Tab(int lane){
    if (TAB == 1){ uint32_t lo=(lane&15)<<2; b0=lo; b1=64+lo; b2=128+lo; b3=192+lo; }
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
__device__ __forceinline__ uint32_t gap(uint32_t a, uint32_t gbase, uint32_t lo){
  uint32_t r=0;
#pragma unroll
  for(int k=0;k<8;k++) r^=lr(gbase+k*1024u+((a>>(4*k))&15u)*64u+lo);
  return r; }

constexpr uint32_t kTabBytes=65536, kGap=kTabBytes, kStage=kGap+8192;  // 16 waves x 4 KiB staging

__device__ void build(){
  for(uint32_t i=threadIdx.x;i<kTabBytes/4;i+=blockDim.x) s_lds[i]=i*0x9E3779B1u;
  for(uint32_t i=threadIdx.x;i<2048;i+=blockDim.x) s_lds[kGap/4+i]=i*0x85EBCA6Bu;
  __syncthreads(); }

template<int TAB> __global__ __launch_bounds__(1024) void k_plain(const uint8_t* p, size_t bytes, uint32_t* out){
  build();
  const int lane=threadIdx.x&63; Tab<TAB> tb(lane); const uint32_t glo=(lane&15)<<2;
  const uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  const size_t nr=bytes/4096; uint32_t acc=0, x=0; u32x4 nx[4];
  size_t r=w;
  if(r<nr){
#pragma unroll
    for(int q=0;q<4;q++) nx[q]=*(const u32x4*)(p+r*4096+lane*64+16*q);
  }
  for(;r<nr;r+=nw){
    u32x4 cur[4];
#pragma unroll
    for(int q=0;q<4;q++) cur[q]=nx[q];
    if(r+nw<nr){
#pragma unroll
      for(int q=0;q<4;q++) nx[q]=*(const u32x4*)(p+(r+nw)*4096+lane*64+16*q);
    }
    acc=gap(acc,kGap,glo);
#pragma unroll
    for(int q=0;q<4;q++){ x^=cur[q].x^cur[q].y^cur[q].z^cur[q].w; acc=tb.step(acc,cur[q].x); acc=tb.step(acc,cur[q].y); acc=tb.step(acc,cur[q].z); acc=tb.step(acc,cur[q].w); }
  }
  if(acc==0x12345u) out[1]=acc;
  atomicXor(out, x); }

// HASH 0: XOR only (stream roof of this schedule); HASH 1: gap + table steps
template<int TAB, int AUX, int HASH> __global__ __launch_bounds__(1024) void k_dma(const uint8_t* p, size_t bytes, uint32_t* out){
  build();
  const int lane=threadIdx.x&63, wid=threadIdx.x>>6; Tab<TAB> tb(lane); const uint32_t glo=(lane&15)<<2;
  const uint32_t slot=kStage+wid*4096;
  const uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  const size_t nr=bytes/4096; uint32_t acc=0, x=0;
  const uint32_t src=(uint32_t)((lane&15)*64+(lane>>4)*16);            // within each KiB
  const uint32_t rd=slot+(uint32_t)(((lane>>4)*64+(lane&15))*16);        // + k*256
  size_t r=w;
  if(r<nr){
#pragma unroll
    for(int q=0;q<4;q++) __builtin_amdgcn_global_load_lds((const void*)(p+r*4096+q*1024+src), LDSP((char*)s_lds+slot+q*1024), 16, 0, AUX);
  }
  for(;r<nr;r+=nw){
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): this wave's round r landed
    u32x4 cur[4];
#pragma unroll
    for(int k=0;k<4;k++) cur[k]=*(const u32x4*)&s_lds[(rd+k*256)/4];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): slot free again
    if(r+nw<nr){
#pragma unroll
      for(int q=0;q<4;q++) __builtin_amdgcn_global_load_lds((const void*)(p+(r+nw)*4096+q*1024+src), LDSP((char*)s_lds+slot+q*1024), 16, 0, AUX);
    }
#pragma unroll
    for(int k=0;k<4;k++) x^=cur[k].x^cur[k].y^cur[k].z^cur[k].w;
    if(HASH){
      acc=gap(acc,kGap,glo);
#pragma unroll
      for(int k=0;k<4;k++){ acc=tb.step(acc,cur[k].x); acc=tb.step(acc,cur[k].y); acc=tb.step(acc,cur[k].z); acc=tb.step(acc,cur[k].w); }
    }
  }
  if(acc==0x12345u) out[1]=acc;
  atomicXor(out, x); }

// alignment probe: DMA 16 B from a dword-aligned (not 16-B aligned) address
__global__ void k_align(const uint8_t* p, uint32_t* out){
  __shared__ __attribute__((aligned(16))) uint32_t buf[256];
  const int lane=threadIdx.x;
  __builtin_amdgcn_global_load_lds((const void*)(p+4+lane*16), LDSP(buf), 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0x0f70);
  const uint32_t* g=(const uint32_t*)(p+4+lane*16);
  uint32_t bad=0;
  for(int k=0;k<4;k++) bad|=buf[lane*4+k]^g[k];
  if(bad) atomicAdd(out, 1u); }

template<typename F> float timeit(F f, int reps=5){ hipEvent_t a,b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); f(); CHECK(hipDeviceSynchronize());
  std::vector<float> t; for(int r=0;r<reps;r++){ CHECK(hipEventRecord(a)); f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms,a,b)); t.push_back(ms);}
  std::sort(t.begin(),t.end()); CHECK(hipGetLastError()); return t[t.size()/2]; }

int main(){
  hipDeviceProp_t pr; CHECK(hipGetDeviceProperties(&pr,0)); int cus=pr.multiProcessorCount;
  const size_t bytes=(size_t)16<<30;
  uint8_t* d; CHECK(hipMalloc(&d, bytes)); uint32_t* out; CHECK(hipMalloc(&out, 64));
  k_fill<<<4096,256>>>((u32x4*)d,bytes/16); CHECK(hipDeviceSynchronize());
  CHECK(hipMemset(out,0,64)); k_align<<<1,64>>>(d,out); uint32_t h[16]; CHECK(hipMemcpy(h,out,64,hipMemcpyDeviceToHost));
  printf("unaligned 16-B DMA: %u lanes wrong\n", h[0]);
  uint32_t ref=0;
  #define RUN(name, ...) { CHECK(hipMemset(out,0,64)); { __VA_ARGS__; } CHECK(hipDeviceSynchronize()); CHECK(hipMemcpy(h,out,64,hipMemcpyDeviceToHost)); \
    if(!ref) ref=h[0]; const char* ok=(h[0]==ref)?"ok":"MISMATCH"; float ms=timeit([&]{ __VA_ARGS__; }); \
    printf("%-18s %.3f ms %7.1f GB/s  xor %s\n", name, ms, bytes/ms/1e6, ok); fflush(stdout); }
  RUN("plain tab2", (k_plain<2><<<cus,1024>>>(d,bytes,out)))
  RUN("plain tab1", (k_plain<1><<<cus,1024>>>(d,bytes,out)))
  RUN("dmas aux0", (k_dma<2,0,0><<<cus,1024>>>(d,bytes,out)))
  RUN("dmas aux2", (k_dma<2,2,0><<<cus,1024>>>(d,bytes,out)))
  RUN("dma tab2 aux0", (k_dma<2,0,1><<<cus,1024>>>(d,bytes,out)))
  RUN("dma tab2 aux2", (k_dma<2,2,1><<<cus,1024>>>(d,bytes,out)))
  RUN("dma tab1 aux2", (k_dma<1,2,1><<<cus,1024>>>(d,bytes,out)))
  RUN("plain tab2 (again)", (k_plain<2><<<cus,1024>>>(d,bytes,out)))
  printf("done\n"); return 0; }
