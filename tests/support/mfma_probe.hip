// Test support (not part of the product library): one v_mfma_f32_32x32x16_f16 with A (32x16) and
// B (16x32) f16 row-major -> D (32x32) f32, through the lane maps field.hip assumes (A: row = lane&31,
// k = 8*(lane>>5) + j; B: col = lane&31, same k; D: row = (i&3) + 8*(i>>2) + 4*(lane>>5)).
// Built by tests/support/Makefile into libmfnerf_probe.so; loaded by tests/test_gpu_field.py.
#include <hip/hip_runtime.h>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void mfma_probe_kernel(const _Float16* A, const _Float16* B, float* D) {
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    half8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = A[r * 16 + 8 * h + j]; b[j] = B[(8 * h + j) * 32 + r]; }
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 16; ++i) D[((i & 3) + 8 * (i >> 2) + 4 * h) * 32 + r] = c[i];
}

extern "C" int mfnerf_probe_mfma(const void* A, const void* B, float* D, hipStream_t stream) {
    hipLaunchKernelGGL(mfma_probe_kernel, dim3(1), dim3(64), 0, stream, (const _Float16*)A, (const _Float16*)B, D);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
