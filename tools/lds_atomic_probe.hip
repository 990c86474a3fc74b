// LDS atomic-add throughput probe (gfx950): every lane adds to pseudo-random words of a
// LDS_WORDS-word LDS array, ITERS times; one workgroup per CU (the array takes most of the LDS).
// Prints chip-wide LDS adds/s for ds_add_u32, ds_add_f32 and a plain (racy) ds read+write RMW,
// for 256 / 512 / 1024-thread workgroups.  Build: hipcc --offload-arch=gfx950 -O3 lds_atomic_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int LDS_WORDS = 32768;  // 128 KiB
constexpr int ITERS = 4096;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ void probe(uint32_t* out, uint32_t seed) {
    __shared__ uint32_t s[LDS_WORDS];
    for (int i = threadIdx.x; i < LDS_WORDS; i += blockDim.x) s[i] = 0;
    __syncthreads();
    uint32_t h = mix(seed ^ (blockIdx.x * 4096u + threadIdx.x));
    for (int it = 0; it < ITERS; ++it) {
        h = h * 1664525u + 1013904223u;
        const uint32_t a = (h >> 8) & (LDS_WORDS - 1);
        if (MODE == 0) atomicAdd(&s[a], 1u);
        else if (MODE == 1) atomicAdd(reinterpret_cast<float*>(&s[a]), 1.0f);
        else s[a] += 1u;
    }
    __syncthreads();
    uint32_t acc = 0;
    for (int i = threadIdx.x; i < LDS_WORDS; i += blockDim.x) acc += s[i];
    atomicAdd(out, acc);
}

template <int MODE>
void run(const char* name, int threads, int blocks, uint32_t* d) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<MODE>, dim3(blocks), dim3(threads), 0, 0, d, r + 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double adds = 5.0 * blocks * threads * (double)ITERS;
    printf("%-10s threads %4d blocks %4d: %.3f ms/launch, %.1f G adds/s chip, %.2f adds/clk/CU @2.4GHz\n", name,
           threads, blocks, ms / 5, adds / (ms * 1e-3) / 1e9, adds / (ms * 1e-3) / 256 / 2.4e9);
}

int main() {
    uint32_t* d;
    hipMalloc(&d, 4);
    for (int t : {256, 512, 1024}) {
        run<0>("ds_add_u32", t, 256, d);
        run<1>("ds_add_f32", t, 256, d);
        run<2>("plain_rmw", t, 256, d);
    }
    hipFree(d);
    return 0;
}
