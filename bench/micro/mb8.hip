// Microbenchmark 8: mb7's full-line LDS-DMA on the cfg3 frame layout.
// 1 M frames at stride 16,404 B (dword-aligned, 16-B alignment cycles 0/4/8/12);
// the first 16,384 B of each frame are hashed by G lanes per frame, 64/G frames
// per wave, lane g owning units g, g+G, ... (the product's lane assignment).
// A wave-round covers 64/G frame spans of G x 64 B. DMA instruction q loads
// G contiguous pieces (G x 16 B) of every span; the reader lane (f, g) finds
// piece k of its unit in instruction q = g / (G/4) at slot
// ((k + q) % 4) * (G/4) + g % (G/4) of its frame's G slots, which keeps each
// ds_read_b128 lane group on 16 distinct 16-B slots for G = 8, 16, 64.
//   plain<TAB>     : global_load_dwordx4, next round prefetched (product shape)
//   dma<TAB,AUX,H> : mb7's schedule (wait, ds_read_b128 x4, issue next round,
//                    hash); H = 0 replaces the hash by an XOR
//   TAB 0: slice-by-4, 32 replicas (128 KiB, the product's); TAB 2: slice-by-2, 32 replicas
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

constexpr uint64_t kStride = 16404, kHashed = 16384;
constexpr uint32_t kFrames = 1u << 20;

__global__ void k_fill(u32x4* p, size_t n){ size_t i=(size_t)blockIdx.x*blockDim.x+threadIdx.x, st=(size_t)gridDim.x*blockDim.x;
  for(; i<n; i+=st){ uint64_t z=i*0x9E3779B97F4A7C15ull; z^=z>>29; p[i]=u32x4{(uint32_t)z,(uint32_t)(z>>32),(uint32_t)(z*3),(uint32_t)i}; } }

__shared__ uint32_t s_lds[160 * 256];
__device__ __forceinline__ uint32_t lr(uint32_t a){ return *(const uint32_t*)((const char*)s_lds + a); }
__device__ __forceinline__ uint32_t perm(uint32_t y, uint32_t base, int k){ return __builtin_amdgcn_perm(y, base, 0x0C020400u + ((uint32_t)k << 8)); }

template<int TAB> struct Tab {
  static constexpr uint32_t bytes = TAB == 0 ? 131072u : 65536u;
  uint32_t b0, b1, b2, b3;
  __device__ Tab(int lane){
    uint32_t lo=(lane&31)<<2;
    if (TAB == 0){ b0=lo; b1=128+lo; b2=65536+lo; b3=65536+128+lo; }
    else { b0=lo; b1=128+lo; b2=b0; b3=b1; }
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
// gap map as in the product: 8 nibble tables x 16 words, one copy (512 B)
__device__ __forceinline__ uint32_t gap(uint32_t a, uint32_t gbase){
  uint32_t r=0;
#pragma unroll
  for(int k=0;k<8;k++) r^=lr(gbase+k*64u+((a>>(4*k))&15u)*4u);
  return r; }

template<int TAB> __device__ void build(){
  for(uint32_t i=threadIdx.x;i<Tab<TAB>::bytes/4;i+=blockDim.x) s_lds[i]=i*0x9E3779B1u;
  for(uint32_t i=threadIdx.x;i<128;i+=blockDim.x) s_lds[Tab<TAB>::bytes/4+i]=i*0x85EBCA6Bu;
  __syncthreads(); }

template<int TAB, int G> __global__ __launch_bounds__(1024) void k_plain(const uint8_t* p, uint32_t* out){
  build<TAB>();
  constexpr uint32_t FPW=64/G, R=kHashed/(64*G);
  const uint32_t gbase=Tab<TAB>::bytes;
  const int lane=threadIdx.x&63, f=lane/G, g=lane%G; Tab<TAB> tb(lane);
  const uint32_t w=(blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=(gridDim.x*blockDim.x)>>6;
  const uint32_t groups=kFrames/FPW;
  uint32_t acc=0, x=0;
  for(uint32_t grp=w; grp<groups; grp+=nw){
    const uint8_t* fb=p+(uint64_t)(grp*FPW+f)*kStride+g*64;
    u32x4 nx[4];
#pragma unroll
    for(int q=0;q<4;q++) nx[q]=*(const u32x4*)(fb+16*q);
    for(uint32_t r=0;r<R;r++){
      u32x4 cur[4];
#pragma unroll
      for(int q=0;q<4;q++) cur[q]=nx[q];
      if(r+1<R){
#pragma unroll
        for(int q=0;q<4;q++) nx[q]=*(const u32x4*)(fb+(r+1)*G*64+16*q);
      }
      acc=gap(acc,gbase);
#pragma unroll
      for(int q=0;q<4;q++){ x^=cur[q].x^cur[q].y^cur[q].z^cur[q].w; acc=tb.step(acc,cur[q].x); acc=tb.step(acc,cur[q].y); acc=tb.step(acc,cur[q].z); acc=tb.step(acc,cur[q].w); }
    }
  }
  if(acc==0x12345u) out[1]=acc;
  atomicXor(out, x); }

template<int TAB, int G, int AUX, int HASH> __global__ __launch_bounds__(1024) void k_dma(const uint8_t* p, uint32_t* out){
  build<TAB>();
  constexpr uint32_t FPW=64/G, R=kHashed/(64*G), GQ=G/4;
  const uint32_t gbase=Tab<TAB>::bytes, slot=gbase+512+(threadIdx.x>>6)*4096;
  const int lane=threadIdx.x&63, f=lane/G, g=lane%G; Tab<TAB> tb(lane);
  // writer: instruction q, lane (f, i) loads piece 4*gw + kw of frame f's span
  uint32_t wsrc[4];
#pragma unroll
  for(int q=0;q<4;q++){ const int i=g, kw=((i/GQ)-q+4)%4, gw=q*GQ+i%GQ; wsrc[q]=(uint32_t)(4*gw+kw)*16; }
  // reader: piece k of lane (f, g)
  uint32_t rd[4];
#pragma unroll
  for(int k=0;k<4;k++){ const int q=g/GQ, i=((k+q)%4)*GQ+g%GQ; rd[k]=slot+q*1024+(f*G+i)*16; }
  const uint32_t w=(blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=(gridDim.x*blockDim.x)>>6;
  const uint32_t groups=kFrames/FPW;
  uint32_t acc=0, x=0;
  uint32_t grp=w, r=0;
  if(grp<groups){
    const uint8_t* fb=p+(uint64_t)(grp*FPW+f)*kStride;
#pragma unroll
    for(int q=0;q<4;q++) __builtin_amdgcn_global_load_lds((const void*)(fb+wsrc[q]), LDSP((char*)s_lds+slot+q*1024), 16, 0, AUX);
  }
  while(grp<groups){
    __builtin_amdgcn_s_waitcnt(0x0f70);
    u32x4 cur[4];
#pragma unroll
    for(int k=0;k<4;k++) cur[k]=*(const u32x4*)&s_lds[rd[k]/4];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    uint32_t ng=grp, nr=r+1;
    if(nr==R){ nr=0; ng=grp+nw; }
    if(ng<groups){
      const uint8_t* fb=p+(uint64_t)(ng*FPW+f)*kStride+nr*G*64;
#pragma unroll
      for(int q=0;q<4;q++) __builtin_amdgcn_global_load_lds((const void*)(fb+wsrc[q]), LDSP((char*)s_lds+slot+q*1024), 16, 0, AUX);
    }
#pragma unroll
    for(int k=0;k<4;k++) x^=cur[k].x^cur[k].y^cur[k].z^cur[k].w;
    if(HASH){
      acc=gap(acc,gbase);
#pragma unroll
      for(int k=0;k<4;k++){ acc=tb.step(acc,cur[k].x); acc=tb.step(acc,cur[k].y); acc=tb.step(acc,cur[k].z); acc=tb.step(acc,cur[k].w); }
    }
    grp=ng; r=nr;
  }
  if(acc==0x12345u) out[1]=acc;
  atomicXor(out, x); }

template<typename F> float timeit(F f, int reps=5){ hipEvent_t a,b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); f(); CHECK(hipDeviceSynchronize());
  std::vector<float> t; for(int r=0;r<reps;r++){ CHECK(hipEventRecord(a)); f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms,a,b)); t.push_back(ms);}
  std::sort(t.begin(),t.end()); CHECK(hipGetLastError()); return t[t.size()/2]; }

int main(){
  hipDeviceProp_t pr; CHECK(hipGetDeviceProperties(&pr,0)); int cus=pr.multiProcessorCount;
  const size_t span=(size_t)kFrames*kStride, hashed=(size_t)kFrames*kHashed;
  uint8_t* d; CHECK(hipMalloc(&d, span+64)); uint32_t* out; CHECK(hipMalloc(&out, 64));
  k_fill<<<4096,256>>>((u32x4*)d,(span+64)/16); CHECK(hipDeviceSynchronize());
  uint32_t h[16], ref=0;
  #define RUN(name, ...) { CHECK(hipMemset(out,0,64)); { __VA_ARGS__; } CHECK(hipDeviceSynchronize()); CHECK(hipMemcpy(h,out,64,hipMemcpyDeviceToHost)); \
    if(!ref) ref=h[0]; const char* ok=(h[0]==ref)?"ok":"MISMATCH"; float ms=timeit([&]{ __VA_ARGS__; }); \
    printf("%-26s %.3f ms %7.1f GB/s  xor %s\n", name, ms, hashed/ms/1e6, ok); fflush(stdout); }
  RUN("plain tab0 G8", (k_plain<0,8><<<cus,1024>>>(d,out)))
  RUN("plain tab0 G16", (k_plain<0,16><<<cus,1024>>>(d,out)))
  RUN("plain tab0 G64", (k_plain<0,64><<<cus,1024>>>(d,out)))
  RUN("dma tab2 G8 aux0", (k_dma<2,8,0,1><<<cus,1024>>>(d,out)))
  RUN("dma tab2 G32 aux0", (k_dma<2,32,0,1><<<cus,1024>>>(d,out)))
  RUN("dma tab2 G32 aux2", (k_dma<2,32,2,1><<<cus,1024>>>(d,out)))
  RUN("dma tab2 G64 aux0", (k_dma<2,64,0,1><<<cus,1024>>>(d,out)))
  RUN("dma tab2 G64 aux2", (k_dma<2,64,2,1><<<cus,1024>>>(d,out)))
  RUN("dma stream G64 aux2", (k_dma<2,64,2,0><<<cus,1024>>>(d,out)))
  RUN("plain tab0 G8 (again)", (k_plain<0,8><<<cus,1024>>>(d,out)))
  RUN("dma tab2 G64 aux2 (again)", (k_dma<2,64,2,1><<<cus,1024>>>(d,out)))
  printf("done\n"); return 0; }
