// Microbenchmark 3: cache-policy probes for the streaming read (no CRC math).
// Contiguous 16 GiB buffer, 1 workgroup of 1024 threads per CU, each wave
// streams whole chunks. Variants:
//   buf<AUX>        raw_buffer_load_b128 with cache-policy bits AUX
//                   (gfx950 CPol: 1 = sc0, 2 = nt, 16 = sc1)
//   ldsdma<I, AUX>  global_load_lds_dwordx4, I KiB in flight per wave, AUX policy
//   glob            plain global_load_dwordx4 (reference)
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

// chunk = 4 KiB per wave per iteration (64 lanes x 64 B)
template<int AUX> __global__ __launch_bounds__(1024) void k_buf(const uint8_t* p, size_t bytes, uint32_t* out){
  const int lane=threadIdx.x&63; uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/4096; u32x4 acc={0,0,0,0};
  for(size_t c=w;c<nch;c+=nw){
    const uint8_t* q=p+c*4096;
    __amdgpu_buffer_rsrc_t r=__builtin_amdgcn_make_buffer_rsrc((void*)q,(short)0,4096,0x00020000);
#pragma unroll
    for(int j=0;j<4;j++){ u32x4 a=__builtin_amdgcn_raw_buffer_load_b128(r, lane*16+j*1024, 0, AUX); acc^=a; } }
  if((acc.x^acc.y^acc.z^acc.w)==0x9u) out[0]=1; }

__global__ __launch_bounds__(1024) void k_glob(const uint8_t* p, size_t bytes, uint32_t* out){
  const int lane=threadIdx.x&63; uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/4096; u32x4 acc={0,0,0,0};
  for(size_t c=w;c<nch;c+=nw){ const u32x4* q=(const u32x4*)(p+c*4096)+lane;
#pragma unroll
    for(int j=0;j<4;j++){ acc^=q[j*64]; } }
  if((acc.x^acc.y^acc.z^acc.w)==0x9u) out[0]=1; }

// LDS-DMA: wave moves I KiB per iteration into its own LDS slots, waits, reads back.
template<int I, int AUX> __global__ __launch_bounds__(1024) void k_ldsdma(const uint8_t* p, size_t bytes, uint32_t* out){
  __shared__ __attribute__((aligned(16))) uint8_t lds[16*I*1024];
  const int lane=threadIdx.x&63, wid=threadIdx.x>>6; uint8_t* mine=lds+wid*I*1024;
  uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/(I*1024); uint32_t acc=0;
  for(size_t c=w;c<nch;c+=nw){ const uint8_t* q=p+c*I*1024;
#pragma unroll
    for(int j=0;j<I;j++) __builtin_amdgcn_global_load_lds((const void*)(q+j*1024+lane*16), (__attribute__((address_space(3))) void*)(mine+j*1024), 16, 0, AUX);
    __builtin_amdgcn_s_waitcnt(0x0f70); // vmcnt(0)
#pragma unroll
    for(int j=0;j<I;j++){ u32x4 a=*(u32x4*)(mine+j*1024+lane*16); acc^=a.x^a.y^a.z^a.w; } }
  if(acc==0x9u) out[0]=acc; }

// LDS-DMA double-buffered: I KiB slots x 2, wait for the older slot only.
template<int I, int AUX> __global__ __launch_bounds__(1024) void k_ldsdma2(const uint8_t* p, size_t bytes, uint32_t* out){
  __shared__ __attribute__((aligned(16))) uint8_t lds[16*2*I*1024];
  const int lane=threadIdx.x&63, wid=threadIdx.x>>6; uint8_t* mine=lds+wid*2*I*1024;
  uint64_t w=((uint64_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((uint64_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/(I*1024); uint32_t acc=0; int slot=0;
  size_t c=w;
  if(c<nch){
#pragma unroll
    for(int j=0;j<I;j++) __builtin_amdgcn_global_load_lds((const void*)(p+c*I*1024+j*1024+lane*16), (__attribute__((address_space(3))) void*)(mine+j*1024), 16, 0, AUX);
  }
  for(;c<nch;c+=nw){
    const size_t cn=c+nw;
    uint8_t* cur=mine+slot*I*1024; uint8_t* nx=mine+(slot^1)*I*1024;
    if(cn<nch){
#pragma unroll
      for(int j=0;j<I;j++) __builtin_amdgcn_global_load_lds((const void*)(p+cn*I*1024+j*1024+lane*16), (__attribute__((address_space(3))) void*)(nx+j*1024), 16, 0, AUX);
      if(I==1) __builtin_amdgcn_s_waitcnt(0x0f71); else if(I==2) __builtin_amdgcn_s_waitcnt(0x0f72); else __builtin_amdgcn_s_waitcnt(0x0f74);
    } else __builtin_amdgcn_s_waitcnt(0x0f70);
#pragma unroll
    for(int j=0;j<I;j++){ u32x4 a=*(u32x4*)(cur+j*1024+lane*16); acc^=a.x^a.y^a.z^a.w; }
    slot^=1; }
  if(acc==0x9u) out[0]=acc; }

template<typename F> float timeit(F f, int reps=7){ hipEvent_t a,b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); f(); CHECK(hipDeviceSynchronize());
  std::vector<float> t; for(int r=0;r<reps;r++){ CHECK(hipEventRecord(a)); f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms,a,b)); t.push_back(ms);}
  std::sort(t.begin(),t.end()); CHECK(hipGetLastError()); return t[t.size()/2]; }

int main(){
  hipDeviceProp_t pr; CHECK(hipGetDeviceProperties(&pr,0)); int cus=pr.multiProcessorCount;
  const size_t bytes=(size_t)16<<30;
  uint8_t* d; CHECK(hipMalloc(&d, bytes)); uint32_t* out; CHECK(hipMalloc(&out, 64));
  k_fill<<<4096,256>>>((u32x4*)d,bytes/16); CHECK(hipDeviceSynchronize());
  #define RUN(name, ...) { float ms=timeit([&]{ __VA_ARGS__; }); printf("%-22s %.3f ms %7.1f GB/s\n", name, ms, bytes/ms/1e6); fflush(stdout); }
  RUN("glob", (k_glob<<<cus,1024>>>(d,bytes,out)))
  RUN("buf aux=0", (k_buf<0><<<cus,1024>>>(d,bytes,out)))
  RUN("buf aux=2 (nt)", (k_buf<2><<<cus,1024>>>(d,bytes,out)))
  RUN("buf aux=16 (sc1)", (k_buf<16><<<cus,1024>>>(d,bytes,out)))
  RUN("buf aux=1 (sc0)", (k_buf<1><<<cus,1024>>>(d,bytes,out)))
  RUN("buf aux=3 (sc0 nt)", (k_buf<3><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma I=1 aux=0", (k_ldsdma<1,0><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma I=1 aux=2", (k_ldsdma<1,2><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma I=2 aux=0", (k_ldsdma<2,0><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma I=2 aux=2", (k_ldsdma<2,2><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma I=4 aux=2", (k_ldsdma<4,2><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma2 I=1 aux=0", (k_ldsdma2<1,0><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma2 I=1 aux=2", (k_ldsdma2<1,2><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma2 I=2 aux=2", (k_ldsdma2<2,2><<<cus,1024>>>(d,bytes,out)))
  RUN("ldsdma2 I=4 aux=2", (k_ldsdma2<4,2><<<cus,1024>>>(d,bytes,out)))
  printf("done\n"); return 0; }
