// Microbenchmark 1: memory-pattern and LDS-table CRC throughput probes on gfx950.
// Not product code. Measures which load pattern / table layout can reach the HBM roof.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do{hipError_t e_=(x); if(e_!=hipSuccess){printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);}}while(0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

__device__ __forceinline__ uint32_t tab_entry(uint32_t i){ uint32_t c=i; for(int j=0;j<8;j++) c=(c&1u)?(0xEDB88320u^(c>>1)):(c>>1); return c; }

__global__ void k_fill(u32x4* p, size_t n, uint64_t seed){
  size_t i = (size_t)blockIdx.x*blockDim.x+threadIdx.x, st=(size_t)gridDim.x*blockDim.x;
  for(; i<n; i+=st){ uint64_t z=seed+i*0x9E3779B97F4A7C15ull; z=(z^(z>>30))*0xBF58476D1CE4E5B9ull; z=(z^(z>>27))*0x94D049BB133111EBull; z^=z>>31;
    uint64_t y=z*0x9E3779B97F4A7C15ull+i; y^=y>>29; p[i]=u32x4{(uint32_t)z,(uint32_t)(z>>32),(uint32_t)y,(uint32_t)(y>>32)}; }
}
__global__ void k_iota(uint32_t* p, size_t n){ size_t i=(size_t)blockIdx.x*blockDim.x+threadIdx.x; if(i<n) p[i]=(uint32_t)i; }

// unaligned dwordx4 correctness probe: out[i] = 1 if load at byte offset off+16i returned the right bytes
__global__ void k_unaligned_check(const uint8_t* p, uint32_t* bad, int off, size_t n){
  size_t i=(size_t)blockIdx.x*blockDim.x+threadIdx.x; if(i>=n) return;
  const uint8_t* a = p + off + 16*i; u32x4u v = *(const u32x4u*)a;
  uint32_t e[4]; for(int k=0;k<4;k++){ uint32_t w=0; for(int b=0;b<4;b++){ size_t bi=(size_t)(a-p)+4*k+b; uint32_t word=(uint32_t)(bi/4); w |= ((word>>(8*(bi%4)))&0xffu)<<(8*b);} e[k]=w; }
  if(v.x!=e[0]||v.y!=e[1]||v.z!=e[2]||v.w!=e[3]) atomicAdd(bad,1u);
}

// 1) coalesced stream read, 4 loads in flight per lane
__global__ void k_stream(const uint8_t* base, int off, size_t n16, uint32_t* out){
  const u32x4u* p=(const u32x4u*)(base+off);
  size_t i=(size_t)blockIdx.x*blockDim.x+threadIdx.x, st=(size_t)gridDim.x*blockDim.x; uint32_t acc=0;
  for(; i+3*st<n16; i+=4*st){ u32x4 a=p[i],b=p[i+st],c=p[i+2*st],d=p[i+3*st]; acc^=a.x^a.y^a.z^a.w^b.x^b.y^b.z^b.w^c.x^c.y^c.z^c.w^d.x^d.y^d.z^d.w; }
  for(; i<n16; i+=st){ u32x4 a=p[i]; acc^=a.x^a.y^a.z^a.w; }
  if(acc==0x9u) out[0]=acc;
}
// 2) per-lane contiguous slices of SLICE bytes (wave chunk = 64*SLICE)
template<int SLICE> __global__ void k_slice(const u32x4* p, size_t bytes, uint32_t* out){
  const int lane=threadIdx.x&63; size_t w=((size_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((size_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/(64*SLICE); uint32_t acc=0;
  for(size_t c=w;c<nch;c+=nw){ const u32x4* q=p+(c*64*SLICE+(size_t)lane*SLICE)/16;
#pragma unroll
    for(int j=0;j<SLICE/16;j++){ u32x4 a=q[j]; acc^=a.x^a.y^a.z^a.w; } }
  if(acc==0x9u) out[0]=acc;
}

// CRC step variants with 32x-replicated tables in LDS: T[idx*32 + (lane&31)]
__device__ __forceinline__ uint32_t bw_word(uint32_t c, uint32_t w, const uint32_t* T, uint32_t lo){
  uint32_t y=c^w;
#pragma unroll
  for(int k=0;k<4;k++){ y = T[((y&0xffu)<<5)|lo] ^ (y>>8); }
  return y;
}
__device__ __forceinline__ uint32_t s4_word(uint32_t c, uint32_t w, const uint32_t* T, uint32_t lo){
  uint32_t y=c^w; // T + k*8192 = table k (k=0 standard); lowest byte uses table 3
  return T[3*8192+(((y)&0xffu)<<5|lo)] ^ T[2*8192+(((y>>8)&0xffu)<<5|lo)] ^ T[1*8192+(((y>>16)&0xffu)<<5|lo)] ^ T[((y>>24)<<5)|lo];
}
__device__ void fill_tables(uint32_t* T, int ntab){
  for(int e=threadIdx.x; e<256*32*ntab; e+=blockDim.x){ int k=e/8192, idx=(e%8192)>>5; uint32_t v=tab_entry(idx); for(int s=0;s<k;s++) v=(v>>8)^tab_entry(v&0xffu); T[e]=v; }
  __syncthreads();
}

// 3) byte-wise CRC, CH chains per lane (lane slice split into CH sub-slices), direct loads
template<int SLICE,int CH> __global__ __launch_bounds__(256) void k_crc_bw(const u32x4* p, size_t bytes, uint32_t* out){
  __shared__ uint32_t T[8192]; fill_tables(T,1);
  const int lane=threadIdx.x&63; const uint32_t lo=lane&31; size_t w=((size_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((size_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/(64*SLICE); uint32_t acc=0;
  for(size_t c=w;c<nch;c+=nw){ const u32x4* q=p+(c*64*SLICE+(size_t)lane*SLICE)/16; uint32_t cr[CH];
#pragma unroll
    for(int h=0;h<CH;h++) cr[h]=0;
#pragma unroll
    for(int j=0;j<SLICE/16/CH;j++){
#pragma unroll
      for(int h=0;h<CH;h++){ u32x4 a=q[h*(SLICE/16/CH)+j]; cr[h]=bw_word(cr[h],a.x,T,lo); cr[h]=bw_word(cr[h],a.y,T,lo); cr[h]=bw_word(cr[h],a.z,T,lo); cr[h]=bw_word(cr[h],a.w,T,lo);} }
#pragma unroll
    for(int h=0;h<CH;h++) acc^=cr[h]; }
  if(acc==0x9u) out[0]=acc;
}
// 4) slice-by-4 CRC, 4 replicated tables (128 KiB), 1024-thread blocks
template<int SLICE,int CH> __global__ __launch_bounds__(1024) void k_crc_s4(const u32x4* p, size_t bytes, uint32_t* out){
  __shared__ uint32_t T[4*8192]; fill_tables(T,4);
  const int lane=threadIdx.x&63; const uint32_t lo=lane&31; size_t w=((size_t)blockIdx.x*blockDim.x+threadIdx.x)>>6, nw=((size_t)gridDim.x*blockDim.x)>>6;
  size_t nch=bytes/(64*SLICE); uint32_t acc=0;
  for(size_t c=w;c<nch;c+=nw){ const u32x4* q=p+(c*64*SLICE+(size_t)lane*SLICE)/16; uint32_t cr[CH];
#pragma unroll
    for(int h=0;h<CH;h++) cr[h]=0;
#pragma unroll
    for(int j=0;j<SLICE/16/CH;j++){
#pragma unroll
      for(int h=0;h<CH;h++){ u32x4 a=q[h*(SLICE/16/CH)+j]; cr[h]=s4_word(cr[h],a.x,T,lo); cr[h]=s4_word(cr[h],a.y,T,lo); cr[h]=s4_word(cr[h],a.z,T,lo); cr[h]=s4_word(cr[h],a.w,T,lo);} }
#pragma unroll
    for(int h=0;h<CH;h++) acc^=cr[h]; }
  if(acc==0x9u) out[0]=acc;
}
// 5) compute-only byte-wise (no global loads): ITER words per lane, CH chains
template<int CH> __global__ __launch_bounds__(256) void k_crc_bw_compute(int iters, uint32_t* out){
  __shared__ uint32_t T[8192]; fill_tables(T,1);
  const uint32_t lo=threadIdx.x&31; uint32_t cr[CH];
#pragma unroll
  for(int h=0;h<CH;h++) cr[h]=threadIdx.x*7+h;
  for(int i=0;i<iters;i++){
#pragma unroll
    for(int h=0;h<CH;h++) cr[h]=bw_word(cr[h],(uint32_t)i*0x9E3779B9u+h,T,lo); }
  uint32_t acc=0;
#pragma unroll
  for(int h=0;h<CH;h++) acc^=cr[h];
  if(acc==0x9u) out[0]=acc;
}
template<int CH> __global__ __launch_bounds__(1024) void k_crc_s4_compute(int iters, uint32_t* out){
  __shared__ uint32_t T[4*8192]; fill_tables(T,4);
  const uint32_t lo=threadIdx.x&31; uint32_t cr[CH];
#pragma unroll
  for(int h=0;h<CH;h++) cr[h]=threadIdx.x*7+h;
  for(int i=0;i<iters;i++){
#pragma unroll
    for(int h=0;h<CH;h++) cr[h]=s4_word(cr[h],(uint32_t)i*0x9E3779B9u+h,T,lo); }
  uint32_t acc=0;
#pragma unroll
  for(int h=0;h<CH;h++) acc^=cr[h];
  if(acc==0x9u) out[0]=acc;
}

template<typename F> float timeit(F f, int reps=5){ hipEvent_t a,b; CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); f(); CHECK(hipDeviceSynchronize());
  std::vector<float> t; for(int r=0;r<reps;r++){ CHECK(hipEventRecord(a)); f(); CHECK(hipEventRecord(b)); CHECK(hipEventSynchronize(b)); float ms; CHECK(hipEventElapsedTime(&ms,a,b)); t.push_back(ms);} 
  std::sort(t.begin(),t.end()); CHECK(hipGetLastError()); return t[0]; }

int main(int argc,char**argv){
  size_t bytes = (argc>1? strtoull(argv[1],0,0) : (16ull<<30));
  hipDeviceProp_t pr; CHECK(hipGetDeviceProperties(&pr,0)); printf("device %s CUs %d clock %d kHz\n", pr.gcnArchName, pr.multiProcessorCount, pr.clockRate);
  uint8_t* d; CHECK(hipMalloc(&d, bytes+4096)); uint32_t* out; CHECK(hipMalloc(&out, 4096));
  // unaligned correctness
  { size_t n=1<<20; k_iota<<<(n+255)/256,256>>>((uint32_t*)d,n); CHECK(hipDeviceSynchronize());
    for(int off: {0,1,2,3,4,5,7,8,13,15}){ CHECK(hipMemset(out,0,4)); k_unaligned_check<<<(n/4-2+255)/256,256>>>(d,out,off,n/4-2); uint32_t bad; CHECK(hipMemcpy(&bad,out,4,hipMemcpyDeviceToHost)); printf("unaligned dwordx4 off=%d bad=%u\n",off,bad);} }
  k_fill<<<4096,256>>>((u32x4*)d, (bytes+4096)/16, 12345); CHECK(hipDeviceSynchronize());
  const double GB=1e9; int cus=pr.multiProcessorCount;
  for(int off: {0,4,1}) for(int bpc: {4,8,16}){ size_t n16=bytes/16-1; float ms=timeit([&]{ k_stream<<<cus*bpc,256>>>(d,off,n16,out); }); printf("stream off=%d blocks/CU=%d: %.3f ms %.1f GB/s\n",off,bpc,ms,n16*16/ms/1e6); }
  #define SL(S) for(int bpc: {4,8}){ float ms=timeit([&]{ k_slice<S><<<cus*bpc,256>>>((const u32x4*)d,bytes,out); }); printf("slice%d blocks/CU=%d: %.3f ms %.1f GB/s\n",S,bpc,ms,bytes/ms/1e6); }
  SL(64) SL(128) SL(256) SL(512)
  #define BW(S,C) for(int bpc: {2,4,5}){ float ms=timeit([&]{ k_crc_bw<S,C><<<cus*bpc,256>>>((const u32x4*)d,bytes,out); }); printf("crc_bw slice%d ch%d blocks/CU=%d: %.3f ms %.1f GB/s\n",S,C,bpc,ms,bytes/ms/1e6); }
  BW(64,1) BW(128,1) BW(128,2) BW(256,1) BW(256,2) BW(256,4)
  #define S4(S,C) { float ms=timeit([&]{ k_crc_s4<S,C><<<cus,1024>>>((const u32x4*)d,bytes,out); }); printf("crc_s4 slice%d ch%d: %.3f ms %.1f GB/s\n",S,C,ms,bytes/ms/1e6); }
  S4(64,1) S4(128,1) S4(256,1) S4(256,2)
  { int it=4096; for(int bpc:{2,4,5}){ float ms=timeit([&]{ k_crc_bw_compute<1><<<cus*bpc,256>>>(it,out); }); double b=(double)cus*bpc*256*it*4; printf("bw_compute ch1 b/CU=%d: %.1f GB/s-equiv\n",bpc,b/ms/1e6);} 
    for(int bpc:{2,4,5}){ float ms=timeit([&]{ k_crc_bw_compute<2><<<cus*bpc,256>>>(it,out); }); double b=(double)cus*bpc*256*it*8; printf("bw_compute ch2 b/CU=%d: %.1f GB/s-equiv\n",bpc,b/ms/1e6);} 
    { float ms=timeit([&]{ k_crc_s4_compute<1><<<cus,1024>>>(it,out); }); double b=(double)cus*1024*it*4; printf("s4_compute ch1: %.1f GB/s-equiv\n",b/ms/1e6);} 
    { float ms=timeit([&]{ k_crc_s4_compute<2><<<cus,1024>>>(it,out); }); double b=(double)cus*1024*it*8; printf("s4_compute ch2: %.1f GB/s-equiv\n",b/ms/1e6);} }
  printf("done\n"); return 0;
}
