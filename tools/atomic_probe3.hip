// Where do integer atomics execute on MI355X?  Same access shape as grid_bw's fine levels (each
// group of 4 lanes adds into one random 16-B span of a 42 MB buffer), for
//   f32 add (global_atomic_add_f32), u32 add (global_atomic_add), u64 add (global_atomic_add_x2),
// with agent and workgroup scope.  If integer atomics run in the XCD's L2 while float atomics go
// to the memory side, fixed-point accumulation of the table gradient escapes the float ceiling.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__device__ __forceinline__ uint32_t hash32(uint32_t x){x^=x>>16;x*=0x7feb352d;x^=x>>15;x*=0x846ca68b;x^=x>>16;return x;}
template <typename T, int SCOPE>
__global__ void add16(T* buf, uint32_t n_spans, int iters, uint32_t per_xcd) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t grp = t / 4, sub = t % 4;
  constexpr int PER = 16 / sizeof(T);  // elements per 16-B span
  // per_xcd != 0: block group b % 8 only touches its own 1/8 of the buffer (XCD-private region)
  const uint32_t region = per_xcd ? (blockIdx.x & 7) * (n_spans / 8) : 0;
  const uint32_t span_n = per_xcd ? n_spans / 8 : n_spans;
  for (int i = 0; i < iters; ++i) {
    const uint32_t sp = region + hash32(grp * 977u + i * 7919u) % span_n;
    if (sub < PER) {
      T* p = buf + (size_t)sp * PER + sub;
      if (SCOPE == 0) __hip_atomic_fetch_add(p, (T)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else __hip_atomic_fetch_add(p, (T)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}
template <typename T, int SCOPE>
void run(const char* name, void* buf, uint32_t bytes, uint32_t per_xcd) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int blocks = 8192, threads = 256, iters = 16;
  const uint32_t n_spans = bytes / 16;
  float best = 1e9;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(a);
    add16<T, SCOPE><<<blocks, threads>>>((T*)buf, n_spans, iters, per_xcd);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
  }
  const double spans = (double)blocks * threads / 4 * iters;
  printf("%-28s xcd-private=%u  %7.3f ms  %7.2f G spans/s\n", name, per_xcd, best, spans / best / 1e6);
}
int main() {
  const uint32_t bytes = 42u << 20;
  void* buf; (void)hipMalloc(&buf, bytes); (void)hipMemset(buf, 0, bytes);
  for (uint32_t px = 0; px < 2; ++px) {
    run<float, 0>("f32 agent", buf, bytes, px);
    run<float, 1>("f32 workgroup", buf, bytes, px);
    run<uint32_t, 0>("u32 agent", buf, bytes, px);
    run<uint32_t, 1>("u32 workgroup", buf, bytes, px);
    run<unsigned long long, 0>("u64 agent", buf, bytes, px);
    run<unsigned long long, 1>("u64 workgroup", buf, bytes, px);
  }
  (void)hipFree(buf);
  return 0;
}
