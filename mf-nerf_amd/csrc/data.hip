// data.hip -- the training batch, sampled on the device from GPU-resident images: the
// reference's DataLoader step (datasets/base.py:22-35, 'all_images' / 'same_image' ray sampling)
// plus train.py:93-105 get_rays (datasets/ray_utils.py:50-70) fused into one launch, so a step's
// data never touches the host and the sampling sits inside the step's HIP graph.
//
// Random draws: np.random.choice(n, k) (uniform with replacement) is replaced by a counter-based
// hash of (seed, call, ray, stream) -- same distribution, not NumPy's stream.  `call` is read from
// a device counter that the launch's last workgroup advances (call[1] is its arrival ticket), so
// graph replays draw fresh batches without a separate one-thread launch.
#include "common.hpp"
#include "../../include/mfnerf.h"

using namespace mfn;

namespace {

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}
// per-launch key: the call index goes through a full avalanche (not added linearly to the
// counter, which would make draw (call c, k) equal draw (call c+1, k-1))
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ uint32_t below(uint64_t key, uint64_t ctr, uint32_t n) {
    return (uint32_t)(((uint64_t)mix32(key + ctr * 0x9E3779B97F4A7C15ull) * n) >> 32);
}

// optional march prologue outputs of mfnerf_sample_rays_prep
struct MarchPrep {
    const float* center;
    const float* half_size;
    float near;
    float* hits_t;  // (n_rays, 2), null: no prologue
    float* noise;   // (n_rays)
};

// one ray of the batch: image + pixel draw, rays, rgb, and optionally the march prologue
__device__ __forceinline__ void draw_ray(int64_t r, const float* __restrict__ images, const float* __restrict__ poses,
                                         const float* __restrict__ directions, int64_t n_img, int64_t hw,
                                         int64_t n_rays, int same_image, uint64_t seed,
                                         const uint64_t* __restrict__ call, float* __restrict__ out,
                                         int32_t* __restrict__ img_idx, int32_t* __restrict__ pix_idx,
                                         const MarchPrep& prep) {
    const uint64_t key = splitmix64(splitmix64(seed ^ 0xD1B54A32D192ED03ull) ^ (call ? *call : 0ull));
    const uint32_t im = below(key, same_image ? 0u : 2u * (uint64_t)r + 1u, (uint32_t)n_img);
    const uint32_t px = below(key, 2u * (uint64_t)r + 2u, (uint32_t)hw);
    const float* c2w = poses + 12 * (int64_t)im;  // (3,4) row-major
    const float* d = directions + 3 * (int64_t)px;
    const float dx = d[0], dy = d[1], dz = d[2];
    float* o = out;
    float* dd = out + 3 * n_rays;
    float* rgb = out + 6 * n_rays;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        // rays_d = directions @ c2w[:, :3].T ; rays_o = c2w[:, 3]
        dd[3 * r + a] = fmaf(dz, c2w[4 * a + 2], fmaf(dy, c2w[4 * a + 1], dx * c2w[4 * a]));
        o[3 * r + a] = c2w[4 * a + 3];
    }
    const float* px_rgb = images + ((int64_t)im * hw + px) * 3;
    rgb[3 * r] = px_rgb[0];
    rgb[3 * r + 1] = px_rgb[1];
    rgb[3 * r + 2] = px_rgb[2];
    if (img_idx) img_idx[r] = (int32_t)im;
    if (pix_idx) pix_idx[r] = (int32_t)px;
    if (prep.hits_t) {
        // the march's prologue for this ray: ray_aabb_intersect against the one scene box with
        // max_hits = 1 (intersection.cu:5-56, = ray_aabb_kernel for that case), the near clamp of
        // rendering.py:29 and the perturbation noise of custom_functions.py:83
        float t1 = -1.0f, t2 = -1.0f;
        const float ox = c2w[3], oy = c2w[7], oz = c2w[11];
        const float ix = 1.0f / dd[3 * r], iy = 1.0f / dd[3 * r + 1], iz = 1.0f / dd[3 * r + 2];
        const float cx = prep.center[0], cy = prep.center[1], cz = prep.center[2];
        const float hx = prep.half_size[0], hy = prep.half_size[1], hz = prep.half_size[2];
        const float tminx = (cx - hx - ox) * ix, tminy = (cy - hy - oy) * iy, tminz = (cz - hz - oz) * iz;
        const float tmaxx = (cx + hx - ox) * ix, tmaxy = (cy + hy - oy) * iy, tmaxz = (cz + hz - oz) * iz;
        float a = fmaxf(fmaxf(fminf(tminx, tmaxx), fminf(tminy, tmaxy)), fminf(tminz, tmaxz));
        float b = fminf(fminf(fmaxf(tminx, tmaxx), fmaxf(tminy, tmaxy)), fmaxf(tminz, tmaxz));
        if (a > b) { a = -1.0f; b = -1.0f; }
        if (b > 0) { t1 = fmaxf(a, 0.0f); t2 = b; }
        if (t1 >= 0.0f && t1 < prep.near) t1 = prep.near;
        prep.hits_t[2 * r] = t1;
        prep.hits_t[2 * r + 1] = t2;
        // U[0,1) with 24 random bits, from a key independent of the (image, pixel) draws
        const uint64_t nkey = splitmix64(splitmix64(seed ^ 0x8CB92BA72F3D8DD7ull) ^ (call ? *call : 0ull));
        prep.noise[r] = (float)(mix32(nkey + (uint64_t)r * 0x9E3779B97F4A7C15ull) >> 8) * (1.0f / 16777216.0f);
    }
}


// out: (3, n_rays, 3) f32 = rays_o | rays_d | rgb
__global__ void sample_rays_kernel(const float* __restrict__ images, const float* __restrict__ poses,
                                   const float* __restrict__ directions, int64_t n_img, int64_t hw, int64_t n_rays,
                                   int same_image, uint64_t seed, uint64_t* __restrict__ call,
                                   float* __restrict__ out, int32_t* __restrict__ img_idx,
                                   int32_t* __restrict__ pix_idx, const MarchPrep prep) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n_rays) draw_ray(r, images, poses, directions, n_img, hw, n_rays, same_image, seed, call, out, img_idx,
                             pix_idx, prep);
    if (call) {
        // every thread of the block has read *call above; the last block to arrive advances it
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint64_t prev = __hip_atomic_fetch_add(call + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (prev == (uint64_t)gridDim.x - 1) {
                call[0] += 1;
                __hip_atomic_store(call + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

}  // namespace

extern "C" int mfnerf_sample_rays(const float* images, const float* poses, const float* directions, int64_t n_img,
                                  int64_t hw, int64_t n_rays, int same_image, uint64_t seed, uint64_t* call,
                                  float* out, int32_t* img_idx, int32_t* pix_idx, mfnerf_stream_t stream) {
    if (n_img <= 0 || hw <= 0 || n_rays < 0 || n_img > 0x7fffffff || hw > 0x7fffffff) {
        mfn_set_error("sample_rays: bad sizes");
        return MFN_ERR_INVALID;
    }
    if (n_rays == 0) return MFN_OK;
    if (!images || !poses || !directions || !out) { mfn_set_error("sample_rays: null pointer"); return MFN_ERR_INVALID; }
    const MarchPrep none{nullptr, nullptr, 0.0f, nullptr, nullptr};
    hipLaunchKernelGGL(sample_rays_kernel, dim3((unsigned)div_up<int64_t>(n_rays, 256)), dim3(256), 0, stream, images,
                       poses, directions, n_img, hw, n_rays, same_image, seed, call, out, img_idx, pix_idx, none);
    return mfn_check_launch("sample_rays");
}

extern "C" int mfnerf_sample_rays_prep(const float* images, const float* poses, const float* directions, int64_t n_img,
                                       int64_t hw, int64_t n_rays, int same_image, uint64_t seed, uint64_t* call,
                                       float* out, const float* center, const float* half_size, float near,
                                       float* hits_t, float* noise, mfnerf_stream_t stream) {
    if (n_img <= 0 || hw <= 0 || n_rays < 0 || n_img > 0x7fffffff || hw > 0x7fffffff) {
        mfn_set_error("sample_rays_prep: bad sizes");
        return MFN_ERR_INVALID;
    }
    if (n_rays == 0) return MFN_OK;
    if (!images || !poses || !directions || !out || !center || !half_size || !hits_t || !noise) {
        mfn_set_error("sample_rays_prep: null pointer");
        return MFN_ERR_INVALID;
    }
    const MarchPrep prep{center, half_size, near, hits_t, noise};
    hipLaunchKernelGGL(sample_rays_kernel, dim3((unsigned)div_up<int64_t>(n_rays, 256)), dim3(256), 0, stream, images,
                       poses, directions, n_img, hw, n_rays, same_image, seed, call, out, (int32_t*)nullptr,
                       (int32_t*)nullptr, prep);
    return mfn_check_launch("sample_rays_prep");
}
