// Atomic request cost model on MI355X: k lanes of a wave-instruction add into one span of k
// consecutive floats (span aligned to k*4 B, random span), k = 1..64; plus "all k lanes add to the
// SAME address"; plus "2 lanes, 8-B pair at a random 8-B-aligned offset within a 64-B line".
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__device__ __forceinline__ uint32_t hash32(uint32_t x){x^=x>>16;x*=0x7feb352d;x^=x>>15;x*=0x846ca68b;x^=x>>16;return x;}
__global__ void span(float* buf, uint32_t n, int iters, int k, int same){
  const uint32_t t = blockIdx.x*blockDim.x+threadIdx.x;
  const uint32_t grp = t / k, sub = t % k;
  for(int i=0;i<iters;++i){
    uint32_t sp = hash32(grp*977u + i*7919u) % (n / k);
    uint32_t j = same ? sp*k : sp*k + sub;
    __hip_atomic_fetch_add(buf+j, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
int main(){
  const uint32_t n = 42u*1024*1024/4; float* buf; (void)hipMalloc(&buf, (size_t)n*4); (void)hipMemset(buf,0,(size_t)n*4);
  hipEvent_t a,b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int blocks=8192, threads=256, iters=16;
  for(int same=0; same<2; ++same) for(int k=1;k<=64;k*=2){
    float best=1e9;
    for(int rep=0;rep<3;++rep){ (void)hipEventRecord(a); span<<<blocks,threads>>>(buf,n,iters,k,same); (void)hipEventRecord(b);
      (void)hipEventSynchronize(b); float ms; (void)hipEventElapsedTime(&ms,a,b); if(ms<best) best=ms; }
    double lanes=(double)blocks*threads*iters, groups=lanes/k;
    printf("%s k=%2d  %7.3f ms  %7.2f G lane-adds/s  %7.2f G spans/s\n", same?"same-addr":"span     ", k, best, lanes/best/1e6, groups/best/1e6);
  }
  return 0;
}
