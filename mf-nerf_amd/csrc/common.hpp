// common.hpp -- shared device helpers for the gfx950 kernels of libmfnerf_hip.
//
// Floating-point contract (shared bit-for-bit with oracle/vren_oracle.c): the whole
// library is compiled with -ffp-contract=off; every multiply-add the reference's nvcc
// build contracts is an explicit fmaf() here, every other op is one IEEE fp32 op.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/mfnerf.h"

#define MFN_SQRT3 1.73205080757f

namespace mfn {

__device__ __forceinline__ float clampf(float f, float a, float b) { return fmaxf(a, fminf(f, b)); }
__device__ __forceinline__ float signf(float x) { return copysignf(1.0f, x); }

// raymarching.cu:11-13
__device__ __forceinline__ float calc_dt(float t, float exp_step_factor, int max_samples, int grid_size, float scale) {
    return clampf(t * exp_step_factor, MFN_SQRT3 / (float)max_samples, MFN_SQRT3 * 2 * scale / (float)grid_size);
}

// raymarching.cu:19-23 -- frexpf exponent of the largest |coordinate|
__device__ __forceinline__ int mip_from_pos(float x, float y, float z, int cascades) {
    const float mx = fmaxf(fabsf(x), fmaxf(fabsf(y), fabsf(z)));
    int e; frexpf(mx, &e);
    return min(cascades - 1, max(0, e + 1));
}

// raymarching.cu:29-32
__device__ __forceinline__ int mip_from_dt(float dt, int grid_size, int cascades) {
    int e; frexpf(dt * (float)grid_size, &e);
    return min(cascades - 1, max(0, e));
}

// raymarching.cu:35-60 -- 3 x 10-bit Morton interleave and its inverse
__host__ __device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
__host__ __device__ __forceinline__ uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
__host__ __device__ __forceinline__ uint32_t morton3_invert(uint32_t x) {
    x = x & 0x49249249u;
    x = (x | (x >> 2)) & 0xc30c30c3u;
    x = (x | (x >> 4)) & 0x0f00f00fu;
    x = (x | (x >> 8)) & 0xff0000ffu;
    x = (x | (x >> 16)) & 0x0000ffffu;
    return x;
}

// One occupancy lookup (raymarching.cu:205-220).  Returns the occupancy bit and the cell.
struct Cell { int nx, ny, nz; float mip_bound; bool occ; };

__device__ __forceinline__ Cell lookup_cell(float x, float y, float z, float dt, int cascades, int grid_size,
                                            float scale, const uint8_t* __restrict__ bitfield) {
    const uint32_t g3 = (uint32_t)grid_size * grid_size * grid_size;
    const int mip = max(mip_from_pos(x, y, z, cascades), mip_from_dt(dt, grid_size, cascades));
    Cell c;
    c.mip_bound = fminf(scalbnf(1.0f, mip - 1), scale);
    const float inv = 1 / c.mip_bound;
    const float gs = (float)grid_size, gm1 = (float)grid_size - 1.0f;
    c.nx = (int)clampf(0.5f * fmaf(x, inv, 1.0f) * gs, 0.0f, gm1);
    c.ny = (int)clampf(0.5f * fmaf(y, inv, 1.0f) * gs, 0.0f, gm1);
    c.nz = (int)clampf(0.5f * fmaf(z, inv, 1.0f) * gs, 0.0f, gm1);
    const uint32_t idx = (uint32_t)mip * g3 + morton3((uint32_t)c.nx, (uint32_t)c.ny, (uint32_t)c.nz);
    c.occ = (bitfield[idx >> 3] >> (idx & 7)) & 1u;
    return c;
}

// DDA skip target (raymarching.cu:225-229)
__device__ __forceinline__ float skip_target(float t, const Cell& c, float x, float y, float z, float dx, float dy,
                                             float dz, float dxi, float dyi, float dzi, float gsi) {
    const float tx = fmaf(fmaf(fmaf(0.5f, signf(dx), (float)c.nx + 0.5f) * gsi, 2.0f, -1.0f), c.mip_bound, -x) * dxi;
    const float ty = fmaf(fmaf(fmaf(0.5f, signf(dy), (float)c.ny + 0.5f) * gsi, 2.0f, -1.0f), c.mip_bound, -y) * dyi;
    const float tz = fmaf(fmaf(fmaf(0.5f, signf(dz), (float)c.nz + 0.5f) * gsi, 2.0f, -1.0f), c.mip_bound, -z) * dzi;
    return t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
}

__device__ __forceinline__ float fast_exp(float x) { return __expf(x); }

template <typename T>
__host__ __device__ __forceinline__ T div_up(T a, T b) { return (a + b - 1) / b; }

// One Adam update (apex multi_tensor_adam ADAM_MODE, weight decay 0: m/(1-b1^t), v/(1-b2^t),
// p -= lr*m_hat/(sqrt(v_hat)+eps)); g already scaled.  bc1/bc2 = 1 - beta^t.
// a float4 streamed once (optimizer state): non-temporal, so it does not evict the working sets
typedef float mfn_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_load4(const float* p) {
    const mfn_f4v x = __builtin_nontemporal_load(reinterpret_cast<const mfn_f4v*>(p));
    return make_float4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void nt_store4(float* p, float4 v) {
    __builtin_nontemporal_store(mfn_f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<mfn_f4v*>(p));
}

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float b1, float b2, float eps,
                                          float lr, float bc1, float bc2) {
    m = b1 * m + (1.0f - b1) * g;
    v = b2 * v + (1.0f - b2) * g * g;
    const float denom = sqrtf(v / bc2) + eps;
    p = p - lr * ((m / bc1) / denom);
}

// The end of an optimizer step, once per launch (torch GradScaler.step + update as PL precision=16
// drives it, train.py:287; apex FusedAdam's step count): a skipped step (amp->nonfinite) counts in
// amp->skipped and backs the loss scale off; a clean step advances Adam's t and, after
// growth_interval clean steps in a row, grows the scale.  The flag is cleared and `zero` (nz floats,
// a per-step accumulator) zeroed for the next step.
__device__ __forceinline__ void amp_step_end(int32_t* step_dev, mfnerf_amp_state* amp, float* zero, int nz) {
    if (amp) {
        const bool bad = amp->nonfinite != 0;
        if (bad) amp->skipped += 1;
        else if (step_dev) *step_dev += 1;
        if (amp->growth_interval > 0) {  // dynamic loss scale (_amp_update_scale_)
            if (bad) {
                amp->scale *= amp->backoff_factor;
                amp->growth_tracker = 0;
            } else if (amp->growth_tracker + 1 >= amp->growth_interval) {
                const float grown = amp->scale * amp->growth_factor;
                if (isfinite(grown)) amp->scale = grown;
                amp->growth_tracker = 0;
            } else {
                amp->growth_tracker += 1;
            }
        }
        amp->nonfinite = 0;
    } else if (step_dev) {
        *step_dev += 1;
    }
    for (int k = 0; k < nz; ++k) zero[k] = 0.0f;
}

// Last-workgroup ticket: call from EVERY thread of every workgroup after the workgroup's last read of
// the state amp_step_end changes; the workgroup that arrives last runs it (and re-arms the ticket), so
// the step's bookkeeping needs no separate one-thread launch.
__device__ __forceinline__ void amp_step_end_last_block(int32_t* step_dev, mfnerf_amp_state* amp, float* zero,
                                                        int nz) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned total = gridDim.x * gridDim.y * gridDim.z;
        const int prev = __hip_atomic_fetch_add(&amp->ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)prev == total - 1) {
            amp_step_end(step_dev, amp, zero, nz);
            __hip_atomic_store(&amp->ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace mfn

// Error plumbing shared by every C-ABI entry point.
void mfn_set_error(const char* fmt, ...);
int mfn_check_launch(const char* what);
// zero `bytes` (a multiple of 4) with a kernel launch: safe inside a captured graph (capi.cpp)
void mfn_zero_async(void* p, int64_t bytes, hipStream_t stream);
