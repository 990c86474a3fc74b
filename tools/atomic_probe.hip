// Microbenchmark: random float atomic scatter into a 42 MB table (the fine hash levels' gradient),
// one lane = one 4-B add to a random line.  Variants: agent scope, workgroup scope into a per-XCD
// private copy (XCC_ID), and plain stores for comparison.  Prints G adds/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__device__ __forceinline__ uint32_t hash32(uint32_t x){x^=x>>16;x*=0x7feb352d;x^=x>>15;x*=0x846ca68b;x^=x>>16;return x;}
__device__ __forceinline__ int xcc_id(){ return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7; }
template<int MODE>
__global__ void k(float* buf, uint32_t n_floats, int iters, uint32_t salt){
  const uint32_t t = blockIdx.x*blockDim.x+threadIdx.x;
  float* base = buf;
  if (MODE==2) base = buf + (size_t)xcc_id()*n_floats;
  for(int i=0;i<iters;++i){
    uint32_t idx = hash32(t*977u + i*7919u + salt) % n_floats;
    if (MODE==0) __hip_atomic_fetch_add(base+idx, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (MODE==1) __hip_atomic_fetch_add(base+idx, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (MODE==2) __hip_atomic_fetch_add(base+idx, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else if (MODE==3) base[idx] = 1.0f;
    else if (MODE==4) { // 4 lanes share a 16-B span (line-paired), agent scope
      uint32_t j = (hash32((t>>2)*977u + i*7919u + salt) % (n_floats/4))*4 + (t&3);
      __hip_atomic_fetch_add(base+j, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
int main(){
  const uint32_t n = 42u*1024*1024/4; float* buf; hipMalloc(&buf, (size_t)n*4*8); hipMemset(buf,0,(size_t)n*4*8);
  hipEvent_t a,b; hipEventCreate(&a); hipEventCreate(&b);
  const int blocks=8192, threads=256, iters=32;
  const char* names[]={"agent random","workgroup random (shared buf)","workgroup per-XCD copy","plain store random","agent 4-lane 16B spans"};
  for(int mode=0;mode<5;++mode){ for(int rep=0;rep<3;++rep){
    hipEventRecord(a);
    switch(mode){case 0:k<0><<<blocks,threads>>>(buf,n,iters,rep);break;case 1:k<1><<<blocks,threads>>>(buf,n,iters,rep);break;
      case 2:k<2><<<blocks,threads>>>(buf,n,iters,rep);break;case 3:k<3><<<blocks,threads>>>(buf,n,iters,rep);break;
      case 4:k<4><<<blocks,threads>>>(buf,n,iters,rep);break;}
    hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms,a,b);
    double adds=(double)blocks*threads*iters;
    if(rep==2) printf("%-32s %8.3f ms  %7.2f G lane-ops/s\n", names[mode], ms, adds/ms/1e6);
  }}
  float h[4]; hipMemcpy(h, buf, 16, hipMemcpyDeviceToHost); printf("check %f\n", h[0]);
  return 0;
}
