// adam.hip -- fused Adam step (apex FusedAdam semantics as used at train.py:136: adam_w_mode
// off, weight_decay 0, eps 1e-15) over the flat fp32 master params, optionally refreshing the
// fp16 compute copy of the hash table in the same pass (one read of p/g/m/v, one write of
// p/m/v/p16: 4+4+4+4 read + 4+4+4+2 write bytes per param, float4-vectorised).
#include "common.hpp"
#include "../../include/mfnerf.h"

namespace {

__global__ void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, __half* __restrict__ p16, int64_t n, float lr, float b1, float b2,
                            float eps, float gscale, int step, int32_t* __restrict__ step_dev,
                            const float* __restrict__ lr_dev, mfnerf_amp_state* __restrict__ amp, int zero_grads,
                            const float* __restrict__ flag_src, float* __restrict__ zero, int nz) {
    const int64_t n4 = n / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // step_dev counts completed steps; this update is number *step_dev + 1 (the last workgroup
    // advances it after every workgroup has read it)
    // GradScaler: no update on a non-finite gradient.  flag_src: the exchanged shard's first value
    // carries every rank's flag (mfnerf_flag_to_shards) -- read here instead of a flag_from_shard launch
    const bool flag_bad = flag_src && !isfinite(flag_src[0]);
    const bool skipped = amp && (flag_src ? flag_bad : amp->nonfinite != 0);
    const int st = step_dev ? *step_dev + 1 : step;
    if (lr_dev) lr = *lr_dev;
    if (skipped) {
        if (zero_grads) {
            for (int64_t i = t0; i < n4; i += stride) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int64_t i = n4 * 4 + t0; i < n; i += stride) g[i] = 0.0f;
        }
    } else {
        // apex multi_tensor_adam (ADAM_MODE, decay 0): m/(1-b1^t), v/(1-b2^t), p -= lr*m_hat/(sqrt(v_hat)+eps)
        const float bc1 = 1.0f - powf(b1, (float)st);
        const float bc2 = 1.0f - powf(b2, (float)st);
        for (int64_t i = t0; i < n4; i += stride) {
            float4 pp = mfn::nt_load4(p + 4 * i);
            const float4 gg = reinterpret_cast<const float4*>(g)[i];
            float4 mm = mfn::nt_load4(m + 4 * i);
            float4 vv = mfn::nt_load4(v + 4 * i);
            float* pa = &pp.x; const float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
            for (int k = 0; k < 4; ++k) mfn::adam_elem(pa[k], ma[k], va[k], ga[k] * gscale, b1, b2, eps, lr, bc1, bc2);
            mfn::nt_store4(p + 4 * i, pp);
            mfn::nt_store4(m + 4 * i, mm);
            mfn::nt_store4(v + 4 * i, vv);
            if (zero_grads) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (p16) {
                __half2 a = __floats2half2_rn(pp.x, pp.y), b = __floats2half2_rn(pp.z, pp.w);
                uint2 u; u.x = *reinterpret_cast<uint32_t*>(&a); u.y = *reinterpret_cast<uint32_t*>(&b);
                reinterpret_cast<uint2*>(p16)[i] = u;
            }
        }
        // tail
        for (int64_t i = n4 * 4 + t0; i < n; i += stride) {
            mfn::adam_elem(p[i], m[i], v[i], g[i] * gscale, b1, b2, eps, lr, bc1, bc2);
            if (zero_grads) g[i] = 0.0f;
            if (p16) p16[i] = __float2half_rn(p[i]);
        }
    }
    if (amp) {
        if (flag_src) {  // the bookkeeping's workgroup (the last) sets the flag it reads from the shard
            __syncthreads();
            if (threadIdx.x == 0) {
                const unsigned total = gridDim.x;
                const int prev = __hip_atomic_fetch_add(&amp->ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((unsigned)prev == total - 1) {
                    amp->nonfinite = flag_bad ? 1 : 0;
                    mfn::amp_step_end(step_dev, amp, zero, nz);
                    __hip_atomic_store(&amp->ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        } else {
            mfn::amp_step_end_last_block(step_dev, amp, zero, nz);
        }
    }
}

}  // namespace

// the step's bookkeeping as its own one-thread launch (callers without an amp state)
__global__ void mfn_bump_step_kernel(int32_t* s, mfnerf_amp_state* amp, float* zero, int nz) {
    mfn::amp_step_end(s, amp, zero, nz);
}

namespace {

// status[0] = 1 if any x is inf/nan (status[0] must be 0 on entry); one atomic per offending wave
__global__ void finite_kernel(const float* __restrict__ x, int64_t n, int32_t* __restrict__ status) {
    bool bad = false;
    const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const float4 v = reinterpret_cast<const float4*>(x)[i];
        bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) bad |= !isfinite(x[i]);
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(status, 1);
}


// Sharded data parallel: carry every rank's non-finite flag through the gradient reduce-scatter
// itself instead of a separate all-reduce.  Before: a flagged rank writes NaN into the first
// element of every shard; after: a shard whose first element is not finite flags the step (a NaN
// survives the sum), so all ranks take the same decision without another collective.
__global__ void flag_to_shards_kernel(float* g, int64_t world, int64_t shard_len, const int32_t* flag) {
    if (*flag && (int64_t)threadIdx.x < world) g[(int64_t)threadIdx.x * shard_len] = __int_as_float(0x7fc00000);
}
__global__ void flag_from_shard_kernel(const float* g_shard, int32_t* flag) {
    *flag = isfinite(g_shard[0]) ? 0 : 1;
}

}  // namespace

extern "C" int mfnerf_flag_to_shards(float* grads, int64_t world, int64_t shard_len, const int32_t* flag,
                                     mfnerf_stream_t stream) {
    if (!grads || !flag || world < 1 || world > 1024 || shard_len < 1) {
        mfn_set_error("flag_to_shards: bad arguments"); return MFN_ERR_INVALID;
    }
    hipLaunchKernelGGL(flag_to_shards_kernel, dim3(1), dim3(1024), 0, stream, grads, world, shard_len, flag);
    return mfn_check_launch("flag_to_shards");
}

extern "C" int mfnerf_flag_from_shard(const float* g_shard, int32_t* flag, mfnerf_stream_t stream) {
    if (!g_shard || !flag) { mfn_set_error("flag_from_shard: null pointer"); return MFN_ERR_INVALID; }
    hipLaunchKernelGGL(flag_from_shard_kernel, dim3(1), dim3(1), 0, stream, g_shard, flag);
    return mfn_check_launch("flag_from_shard");
}

extern "C" int mfnerf_adam_step(float* params, float* grads, float* m, float* v, void* p_f16, int64_t n,
                                float lr, float beta1, float beta2, float eps, float grad_scale, int step,
                                int32_t* step_dev, const float* lr_dev, mfnerf_amp_state* amp, int zero_grads,
                                mfnerf_stream_t stream) {
    if (n < 0) { mfn_set_error("adam_step: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!params || !grads || !m || !v) { mfn_set_error("adam_step: null pointer"); return MFN_ERR_INVALID; }
    if ((((uintptr_t)params) | ((uintptr_t)grads) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) {
        mfn_set_error("adam_step: buffers must be 16-byte aligned"); return MFN_ERR_INVALID;
    }
    if (p_f16 && (((uintptr_t)p_f16) & 7)) { mfn_set_error("adam_step: fp16 copy must be 8-byte aligned"); return MFN_ERR_INVALID; }
    if (!step_dev && step < 1) { mfn_set_error("adam_step: step must be >= 1"); return MFN_ERR_INVALID; }
    const int threads = 256;
    const int64_t want = mfn::div_up<int64_t>(mfn::div_up<int64_t>(n, 4), threads);
    // 1024 workgroups at most: each takes the last-workgroup ticket (one serialised memory-side
    // atomic on one address), grid-stride does the rest at the same bandwidth (grid.hip adam_fixed)
    const unsigned blocks = (unsigned)(want < 1024 ? (want < 1 ? 1 : want) : 1024);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(threads), 0, stream, params, grads, m, v, (__half*)p_f16, n, lr,
                       beta1, beta2, eps, grad_scale, step, step_dev, lr_dev, amp, zero_grads, (const float*)nullptr,
                       (float*)nullptr, 0);
    // with amp the last workgroup did the bookkeeping; without it only the step count remains
    if (step_dev && !amp)
        hipLaunchKernelGGL(mfn_bump_step_kernel, dim3(1), dim3(1), 0, stream, step_dev, (mfnerf_amp_state*)nullptr,
                           (float*)nullptr, 0);
    return mfn_check_launch("adam_step");
}

extern "C" int mfnerf_adam_step_shard(float* params, const float* g_shard, float* m, float* v, void* p_f16, int64_t n,
                                      float lr, float beta1, float beta2, float eps, float grad_scale,
                                      int32_t* step_dev, const float* lr_dev, mfnerf_amp_state* amp, float* zero, int nz,
                                      mfnerf_stream_t stream) {
    if (n < 1 || nz < 0 || nz > 64) { mfn_set_error("adam_step_shard: bad size"); return MFN_ERR_INVALID; }
    if (!params || !g_shard || !m || !v || !step_dev || !amp || (nz && !zero)) {
        mfn_set_error("adam_step_shard: null pointer"); return MFN_ERR_INVALID;
    }
    if ((((uintptr_t)params) | ((uintptr_t)g_shard) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) {
        mfn_set_error("adam_step_shard: buffers must be 16-byte aligned"); return MFN_ERR_INVALID;
    }
    if (p_f16 && (((uintptr_t)p_f16) & 7)) { mfn_set_error("adam_step_shard: fp16 copy must be 8-byte aligned"); return MFN_ERR_INVALID; }
    const int threads = 256;
    const int64_t want = mfn::div_up<int64_t>(mfn::div_up<int64_t>(n, 4), threads);
    const unsigned blocks = (unsigned)(want < 1024 ? want : 1024);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(threads), 0, stream, params, const_cast<float*>(g_shard), m, v,
                       (__half*)p_f16, n, lr, beta1, beta2, eps, grad_scale, 0, step_dev, lr_dev, amp, 0, g_shard,
                       zero, nz);
    return mfn_check_launch("adam_step_shard");
}

extern "C" int mfnerf_check_finite(const float* x, int64_t n, int32_t* status, mfnerf_stream_t stream) {
    if (n < 0 || !status || (n > 0 && !x)) { mfn_set_error("check_finite: bad arguments"); return MFN_ERR_INVALID; }
    if (((uintptr_t)x) & 15) { mfn_set_error("check_finite: x must be 16-byte aligned"); return MFN_ERR_INVALID; }
    mfn_zero_async(status, sizeof(int32_t), stream);
    if (n > 0) {
        const int64_t want = mfn::div_up<int64_t>(mfn::div_up<int64_t>(n, 4), 256);
        hipLaunchKernelGGL(finite_kernel, dim3((unsigned)(want < 2048 ? (want < 1 ? 1 : want) : 2048)), dim3(256), 0,
                           stream, x, n, status);
    }
    return mfn_check_launch("check_finite");
}
