// grid.hip -- multiresolution grid encoding (tiny-cuda-nn HashGrid semantics, plus this repo's
// MixedFeature shared-table variant) forward and backward on gfx950.
//
// Forward: 4 lanes per point, each lane owns 4 consecutive levels (8 f16 features = one 16-B
// store), so the 4 lanes of a point write its 64-B output row with one coalesced 64-B burst and
// every lane keeps 32 independent 4-B corner gathers in flight.  Accumulation is fp32 (tcnn
// accumulates in half; the difference is inside the fp16 output rounding).
// Backward: see grid_bw_kernel (request-shaped float atomics with in-wave run merging).
#include <cstdlib>

#include "common.hpp"
#include "../../include/mfnerf.h"

using namespace mfn;

__global__ void mfn_bump_step_kernel(int32_t* s, mfnerf_amp_state* amp, float* zero, int nz);  // adam.hip

namespace {

constexpr uint32_t PRIME1 = 2654435761u, PRIME2 = 805459861u;

struct LevelGeo {
    uint32_t g[3];  // floor(pos)
    float w[3];     // pos - floor(pos)
};

// tcnn pos_fract (grid.h): pos = fmaf(scale, x, 0.5f); g = floor(pos); w = pos - g  (Linear)
__device__ __forceinline__ LevelGeo level_geo(float scale, float x, float y, float z) {
    LevelGeo L;
    const float px = fmaf(scale, x, 0.5f), py = fmaf(scale, y, 0.5f), pz = fmaf(scale, z, 0.5f);
    const float fx = floorf(px), fy = floorf(py), fz = floorf(pz);
    L.g[0] = (uint32_t)(int)fx; L.g[1] = (uint32_t)(int)fy; L.g[2] = (uint32_t)(int)fz;
    L.w[0] = px - fx; L.w[1] = py - fy; L.w[2] = pz - fz;
    return L;
}

// tcnn grid_index: dense strides while res^3 <= size, else the coherent prime hash; `% size`.
// MixedFeature shared tables hash the point's coordinates on the canonical grid.
__device__ __forceinline__ uint32_t corner_index(const mfnerf_grid_desc& D, int l, uint32_t x, uint32_t y,
                                                 uint32_t z) {
    const uint32_t res = D.res[l], size = D.size[l];
    uint32_t idx;
    if (D.table_kind[l] == 1) {
        const uint32_t rc = (uint32_t)D.canon_res;
        x = (uint32_t)(((uint64_t)x * rc) / res);
        y = (uint32_t)(((uint64_t)y * rc) / res);
        z = (uint32_t)(((uint64_t)z * rc) / res);
        idx = (x * 1u) ^ (y * PRIME1) ^ (z * PRIME2);
    } else if ((uint64_t)res * res * res <= size) {
        idx = x + y * res + z * res * res;
    } else {
        idx = (x * 1u) ^ (y * PRIME1) ^ (z * PRIME2);
    }
    if ((size & (size - 1)) == 0) return idx & (size - 1);
    return idx < size ? idx : idx % size;
}

__device__ __forceinline__ float corner_weight(const LevelGeo& L, int c) {
    float w = 1.0f;
    w *= (c & 1) ? L.w[0] : (1.0f - L.w[0]);
    w *= (c & 2) ? L.w[1] : (1.0f - L.w[1]);
    w *= (c & 4) ? L.w[2] : (1.0f - L.w[2]);
    return w;
}

constexpr int ENC_BLOCK = 256;
constexpr int LEVELS_PER_LANE = 4;

// out row = 32 halfs (L=16, F=2); requires n_levels % 4 == 0 and F == 2.
__global__ __launch_bounds__(ENC_BLOCK) void grid_fw_kernel(const float* __restrict__ X, int64_t n,
                                                             const int32_t* __restrict__ n_dev, float x_min,
                                                             float x_range, const mfnerf_grid_desc D,
                                                             const __half2* __restrict__ table,
                                                             __half* __restrict__ out) {
    const int groups = D.n_levels / LEVELS_PER_LANE;
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t total = nn * groups;
    for (int64_t t = (int64_t)blockIdx.x * ENC_BLOCK + threadIdx.x; t < total; t += (int64_t)gridDim.x * ENC_BLOCK) {
    const int64_t i = t / groups;
    const int grp = (int)(t - i * groups);
    const float x = (X[3 * i] - x_min) / x_range;
    const float y = (X[3 * i + 1] - x_min) / x_range;
    const float z = (X[3 * i + 2] - x_min) / x_range;
    float acc[2 * LEVELS_PER_LANE];
#pragma unroll
    for (int k = 0; k < LEVELS_PER_LANE; ++k) {
        const int l = grp * LEVELS_PER_LANE + k;
        const LevelGeo L = level_geo(D.scale[l], x, y, z);
        const __half2* tab = table + D.offset[l];
        __half2 v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
            v[c] = tab[corner_index(D, l, L.g[0] + (c & 1), L.g[1] + ((c >> 1) & 1), L.g[2] + ((c >> 2) & 1))];
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const float w = corner_weight(L, c);
            const float2 f = __half22float2(v[c]);
            a0 = fmaf(w, f.x, a0);
            a1 = fmaf(w, f.y, a1);
        }
        acc[2 * k] = a0; acc[2 * k + 1] = a1;
    }
    __half2 h[LEVELS_PER_LANE];
#pragma unroll
    for (int k = 0; k < LEVELS_PER_LANE; ++k) h[k] = __floats2half2_rn(acc[2 * k], acc[2 * k + 1]);
    uint4 pk;
    pk.x = *reinterpret_cast<uint32_t*>(&h[0]); pk.y = *reinterpret_cast<uint32_t*>(&h[1]);
    pk.z = *reinterpret_cast<uint32_t*>(&h[2]); pk.w = *reinterpret_cast<uint32_t*>(&h[3]);
    reinterpret_cast<uint4*>(out + i * (2 * D.n_levels))[grp] = pk;
    }
}

// Planar (level-major) forward, XCD-partitioned: blocks b and b+8 share an XCD (round-robin
// dispatch), so block group b % 8 owns the levels {l : snake(l % 16) == b % 8} (levels p and 15-p
// for L = 16) for every sample.  Each XCD's L2 then holds only its levels' tables (<= 4 MB of
// fp16 features), instead of every XCD streaming the whole 23 MB table through its 4 MB L2.
// out: n_levels planes of plane_stride half2 (features of level l of sample i at out[l*stride+i]),
// so each group's stores are contiguous.  Placement only affects speed, never the result.
__device__ __forceinline__ int level_group(int l) {
    const int q = l & 15;
    return q < 8 ? q : 15 - q;
}

// one (sample, level) of the planar forward
__device__ __forceinline__ void planar_level(const mfnerf_grid_desc& D, const __half2* __restrict__ table,
                                             __half2* __restrict__ out, int64_t plane_stride, int64_t i, int l,
                                             float x, float y, float z) {
    const LevelGeo L = level_geo(D.scale[l], x, y, z);
    const __half2* tab = table + D.offset[l];
    const uint32_t size = D.size[l], res = D.res[l];
    const bool dense = D.table_kind[l] == 0 && (uint64_t)res * res * res <= size;
    const bool pow2 = (size & (size - 1)) == 0;
    __half2 v[8];
    // The two x-corners of a (y,z) row are adjacent entries -- dense levels: idx+1 (one
    // unaligned 8-B load unless it wraps past the table end); hashed power-of-two levels
    // with even x: idx^1 (one aligned 8-B load) -- so each row costs one gather lane
    // instead of two (the kernel is bound by per-lane gather addresses).
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t gy = L.g[1] + (yz & 1), gz = L.g[2] + (yz >> 1);
        const uint32_t i0 = corner_index(D, l, L.g[0], gy, gz);
        if (dense && i0 + 1 < size) {
            const uint2 u = *reinterpret_cast<const uint2*>(tab + i0);
            v[2 * yz] = *reinterpret_cast<const __half2*>(&u.x);
            v[2 * yz + 1] = *reinterpret_cast<const __half2*>(&u.y);
        } else if (!dense && pow2 && D.table_kind[l] == 0 && (L.g[0] & 1) == 0) {
            const uint2 u = *reinterpret_cast<const uint2*>(tab + (i0 & ~1u));
            const bool lo = (i0 & 1) == 0;
            v[2 * yz] = *reinterpret_cast<const __half2*>(lo ? &u.x : &u.y);
            v[2 * yz + 1] = *reinterpret_cast<const __half2*>(lo ? &u.y : &u.x);
        } else {
            v[2 * yz] = tab[i0];
            v[2 * yz + 1] = tab[corner_index(D, l, L.g[0] + 1, gy, gz)];
        }
    }
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float w = corner_weight(L, c);
        const float2 f = __half22float2(v[c]);
        a0 = fmaf(w, f.x, a0);
        a1 = fmaf(w, f.y, a1);
    }
    out[(int64_t)l * plane_stride + i] = __floats2half2_rn(a0, a1);
}

__global__ __launch_bounds__(ENC_BLOCK) void grid_fw_planar_kernel(const float* __restrict__ X, int64_t n,
                                                                    const int32_t* __restrict__ n_dev, float x_min,
                                                                    float x_range, const mfnerf_grid_desc D,
                                                                    const __half2* __restrict__ table,
                                                                    __half2* __restrict__ out, int64_t plane_stride) {
    const int grp = blockIdx.x & 7;
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int nj = 2 * ((D.n_levels + 15) >> 4);
    const int64_t stride = (int64_t)(gridDim.x >> 3) * ENC_BLOCK;
    for (int64_t i = (int64_t)(blockIdx.x >> 3) * ENC_BLOCK + threadIdx.x; i < nn; i += stride) {
        const float x = (X[3 * i] - x_min) / x_range;
        const float y = (X[3 * i + 1] - x_min) / x_range;
        const float z = (X[3 * i + 2] - x_min) / x_range;
        // this group's levels, visited directly: 16m + grp and 16m + 15 - grp
        for (int j = 0; j < nj; ++j) {
            const int l = 16 * (j >> 1) + ((j & 1) ? 15 - grp : grp);
            if (l >= D.n_levels) continue;
            planar_level(D, table, out, plane_stride, i, l, x, y, z);
        }
    }
}

// Backward.  The table gradient is a scatter-add; on MI355X a float atomic executes at the memory
// side and costs one request per distinct 64-B line of a wave-instruction -- lanes of one line are
// free, lanes on the SAME address are not coalesced (tools/atomic_probe2.hip) -- so the kernel is
// shaped to minimise requests, not bytes:
//   * one wave = 16 consecutive samples, walking all levels; lane = (xb, f, s) with the sample s
//     fastest: per (y,z) corner pair the 4 lanes of a sample add to entries idx(x), idx(x+1) x
//     features f0,f1 -- one 16-B span, i.e. one line for dense levels and, for hashed levels,
//     whenever x->x+1 leaves the hash's low bits alone (7/8 of the time);
//   * consecutive samples lie along a ray, so coarse levels repeat a corner for many samples: a
//     4-step segmented suffix scan (DPP row shifts inside each 16-lane row = one (xb,f) stream)
//     merges such runs and only run heads issue the atomic;
//   * the dense coarse levels (a few hundred to a few thousand hot lines) add into GRAD_COPIES
//     private copies, picked per wave, folded back by fold_copies_kernel.
constexpr int GRAD_COPIES = 8;

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
#define DPP_ROW_SHL(d) (0x100 | (d))
#define DPP_ROW_SHR(d) (0x110 | (d))

// ABLATE: 0 = product; debug builds: 1 plain stores, 2 levels 0-5 only, 3 levels 10-15 only.
// MAXL: level-count bound (16 or 32) sizing the LDS tile and the prefetch registers.
// FIX: fixed-point accumulation -- per level l, each (run-merged) contribution v is added as the
// int32 rint(v * scale_l) with global_atomic_add (integer atomics run ~28% faster than float ones
// at the memory side, tools/atomic_probe3.hip), scale_l = fixed_scale(level_l1[l]); the buffers
// then hold int32 bit patterns until fold_convert_kernel turns them back into floats.
__device__ __forceinline__ float fixed_scale(float l1) {
    // |entry sum| <= sum over samples of |dL/dy| of the level = l1 < 2^e, so scale 2^(30-e) keeps
    // every entry (and every private copy of one) within 2^30: no int32 overflow is possible
    if (!(l1 > 0.0f)) return 0.0f;
    int e;
    frexpf(l1, &e);
    return ldexpf(1.0f, 30 - e);
}

// The scale of the table level l adds into.  A MixedFeature table shared by several levels takes
// the sum of their L1 bounds, so every level adding into it uses the table's one scale and the
// bound still holds for each entry.
__device__ __forceinline__ float table_fixed_scale(const mfnerf_grid_desc& D, const float* __restrict__ level_l1,
                                                   int l) {
    float l1 = 0.0f;
    for (int k = 0; k < D.n_levels; ++k)
        if (D.offset[k] == D.offset[l]) l1 += level_l1[k];
    return fixed_scale(l1);
}

template <int ABLATE, int MAXL, bool FIX>
__global__ __launch_bounds__(ENC_BLOCK) void grid_bw_kernel(const float* __restrict__ X, int64_t n,
                                                             const int32_t* __restrict__ n_dev, float x_min,
                                                             float x_range, const mfnerf_grid_desc D,
                                                             const float* __restrict__ dy, float* __restrict__ grad,
                                                             float* __restrict__ priv, int64_t dense_entries,
                                                             const float* __restrict__ level_l1) {
    // dL/dy of the wave's chunk (16 samples x 2L floats) is staged in LDS (rows padded by one
    // float: conflict-free column reads) and the NEXT chunk is prefetched into registers before
    // this chunk's atomics are issued.  On gfx9 no-return atomics count in vmcnt, so a global load
    // between atomics would make the wave wait for every earlier atomic's round trip; with the
    // loads hoisted there is at most one such wait per chunk (64 atomics) instead of per level.
    __shared__ float sdy_all[ENC_BLOCK / 64][16 * (2 * MAXL + 1)];
    const int L_ = D.n_levels;
    const int lane = threadIdx.x & 63, s = lane & 15, f = (lane >> 4) & 1, xb = lane >> 5;
    const int row = 2 * L_, rs = 2 * L_ + 1, per_chunk = 16 * row;
    float* sdy = sdy_all[threadIdx.x >> 6];
    __shared__ float fs_s[MAXL];  // fixed-point scale per level (its table's)
    if (FIX) {
        if ((int)threadIdx.x < L_) fs_s[threadIdx.x] = table_fixed_scale(D, level_l1, threadIdx.x);
        __syncthreads();
    }
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t chunks = div_up<int64_t>(nn, 16);
    const int64_t wave0 = ((int64_t)blockIdx.x * ENC_BLOCK + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * ENC_BLOCK) >> 6;
    const int64_t n_vals = nn * row;

    float pf[MAXL / 2];  // this lane's share of a chunk's dL/dy
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    auto fetch = [&](int64_t ch) {
        const int64_t base = ch * per_chunk;
#pragma unroll
        for (int k = 0; k < MAXL / 2; ++k) {
            const int idx = lane + 64 * k;
            pf[k] = (idx < per_chunk && base + idx < n_vals) ? dy[base + idx] : 0.0f;
        }
        const int64_t i = ch * 16 + s;
        if (i < nn) { px = X[3 * i]; py = X[3 * i + 1]; pz = X[3 * i + 2]; }
    };
    if (wave0 < chunks) fetch(wave0);
    for (int64_t chunk = wave0; chunk < chunks; chunk += n_waves) {
        const int64_t i = chunk * 16 + s;
        const bool valid = i < nn;
#pragma unroll
        for (int k = 0; k < MAXL / 2; ++k) {
            const int idx = lane + 64 * k;
            if (idx < per_chunk) sdy[(idx / row) * rs + idx % row] = pf[k];
        }
        const float x = valid ? (px - x_min) / x_range : 0.0f;
        const float y = valid ? (py - x_min) / x_range : 0.0f;
        const float z = valid ? (pz - x_min) / x_range : 0.0f;
        if (chunk + n_waves < chunks) fetch(chunk + n_waves);  // in flight during this chunk's atomics
        const float* srow = sdy + s * rs + f;
        for (int l = 0; l < L_; ++l) {
            if (ABLATE == 2 && l > 5) continue;
            if (ABLATE == 3 && l < 10) continue;
            const float g = srow[2 * l];
            const float fs = FIX ? fs_s[l] : 0.0f;
            const LevelGeo Lg = level_geo(D.scale[l], x, y, z);
            const bool spread = priv && (int64_t)D.offset[l] + D.size[l] <= dense_entries;
            float* gt = spread ? priv + 2 * ((chunk & (GRAD_COPIES - 1)) * dense_entries + (int64_t)D.offset[l])
                               : grad + 2 * (int64_t)D.offset[l];
#pragma unroll
            for (int yz = 0; yz < 4; ++yz) {
                const int c = xb | (yz << 1);
                const uint32_t idx =
                    corner_index(D, l, Lg.g[0] + (c & 1), Lg.g[1] + ((c >> 1) & 1), Lg.g[2] + ((c >> 2) & 1));
                const int key = valid ? (int)idx : -1;
                float v = corner_weight(Lg, c) * g;
                const int kn = dpp_i<DPP_ROW_SHL(1)>(key), kp = dpp_i<DPP_ROW_SHR(1)>(key);
                const bool head = (s == 0) || kp != key;
                int stop = (s == 15) || kn != key;  // this lane ends its run
                // segmented suffix sum within the 16-lane row: run heads end up with the run total
                { const float vp = dpp_f<DPP_ROW_SHL(1)>(v); const int sp = dpp_i<DPP_ROW_SHL(1)>(stop); if (!stop) { v += vp; stop = sp; } }
                { const float vp = dpp_f<DPP_ROW_SHL(2)>(v); const int sp = dpp_i<DPP_ROW_SHL(2)>(stop); if (!stop) { v += vp; stop = sp; } }
                { const float vp = dpp_f<DPP_ROW_SHL(4)>(v); const int sp = dpp_i<DPP_ROW_SHL(4)>(stop); if (!stop) { v += vp; stop = sp; } }
                { const float vp = dpp_f<DPP_ROW_SHL(8)>(v); const int sp = dpp_i<DPP_ROW_SHL(8)>(stop); if (!stop) { v += vp; stop = sp; } }
                if (FIX) {
                    const int q = (int)rintf(v * fs);
                    if (head && valid && q != 0)
                        __hip_atomic_fetch_add(reinterpret_cast<int*>(gt) + 2 * idx + f, q, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                } else if (head && valid && v != 0.0f) {
                    if (ABLATE == 1) gt[2 * idx + f] = v;
                    else __hip_atomic_fetch_add(gt + 2 * idx + f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
}

// fp16 variant (experiment / tcnn's grad_t = __half for F = 2): one lane adds BOTH features of a
// corner with global_atomic_pk_add_f16, lanes = (sample s, x-corner xb, yz-half), so a level takes
// 2 wave-instructions instead of 4.  Values are multiplied by gscale before rounding to fp16.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));

template <int MAXL>
__global__ __launch_bounds__(ENC_BLOCK) void grid_bw_h2_kernel(const float* __restrict__ X, int64_t n,
                                                                const int32_t* __restrict__ n_dev, float x_min,
                                                                float x_range, const mfnerf_grid_desc D,
                                                                const float* __restrict__ dy, h2v* __restrict__ grad,
                                                                h2v* __restrict__ priv, int64_t dense_entries,
                                                                float gscale) {
    __shared__ float sdy_all[ENC_BLOCK / 64][16 * (2 * MAXL + 1)];
    const int L_ = D.n_levels;
    const int lane = threadIdx.x & 63, s = lane & 15, xb = (lane >> 4) & 1, yzh = lane >> 5;
    const int row = 2 * L_, rs = 2 * L_ + 1, per_chunk = 16 * row;
    float* sdy = sdy_all[threadIdx.x >> 6];
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t chunks = div_up<int64_t>(nn, 16);
    const int64_t wave0 = ((int64_t)blockIdx.x * ENC_BLOCK + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)gridDim.x * ENC_BLOCK) >> 6;
    const int64_t n_vals = nn * row;
    float pf[MAXL / 2];
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    auto fetch = [&](int64_t ch) {
        const int64_t base = ch * per_chunk;
#pragma unroll
        for (int k = 0; k < MAXL / 2; ++k) {
            const int idx = lane + 64 * k;
            pf[k] = (idx < per_chunk && base + idx < n_vals) ? dy[base + idx] : 0.0f;
        }
        const int64_t i = ch * 16 + s;
        if (i < nn) { px = X[3 * i]; py = X[3 * i + 1]; pz = X[3 * i + 2]; }
    };
    if (wave0 < chunks) fetch(wave0);
    for (int64_t chunk = wave0; chunk < chunks; chunk += n_waves) {
        const int64_t i = chunk * 16 + s;
        const bool valid = i < nn;
#pragma unroll
        for (int k = 0; k < MAXL / 2; ++k) {
            const int idx = lane + 64 * k;
            if (idx < per_chunk) sdy[(idx / row) * rs + idx % row] = pf[k];
        }
        const float x = valid ? (px - x_min) / x_range : 0.0f;
        const float y = valid ? (py - x_min) / x_range : 0.0f;
        const float z = valid ? (pz - x_min) / x_range : 0.0f;
        if (chunk + n_waves < chunks) fetch(chunk + n_waves);
        const float* srow = sdy + s * rs;
        for (int l = 0; l < L_; ++l) {
            const float g0 = srow[2 * l] * gscale, g1 = srow[2 * l + 1] * gscale;
            const LevelGeo Lg = level_geo(D.scale[l], x, y, z);
            const bool spread = priv && (int64_t)D.offset[l] + D.size[l] <= dense_entries;
            h2v* gt = spread ? priv + ((chunk & (GRAD_COPIES - 1)) * dense_entries + (int64_t)D.offset[l])
                             : grad + (int64_t)D.offset[l];
#pragma unroll
            for (int yp = 0; yp < 2; ++yp) {
                const int c = xb | ((2 * yzh + yp) << 1);
                const uint32_t idx =
                    corner_index(D, l, Lg.g[0] + (c & 1), Lg.g[1] + ((c >> 1) & 1), Lg.g[2] + ((c >> 2) & 1));
                const int key = valid ? (int)idx : -1;
                const float w = corner_weight(Lg, c);
                float v0 = w * g0, v1 = w * g1;
                const int kn = dpp_i<DPP_ROW_SHL(1)>(key), kp = dpp_i<DPP_ROW_SHR(1)>(key);
                const bool head = (s == 0) || kp != key;
                int stop = (s == 15) || kn != key;
#define H2_STEP(d) { const float a = dpp_f<DPP_ROW_SHL(d)>(v0), b = dpp_f<DPP_ROW_SHL(d)>(v1); \
                     const int sp = dpp_i<DPP_ROW_SHL(d)>(stop); if (!stop) { v0 += a; v1 += b; stop = sp; } }
                H2_STEP(1) H2_STEP(2) H2_STEP(4) H2_STEP(8)
#undef H2_STEP
                if (head && valid && (v0 != 0.0f || v1 != 0.0f)) {
                    const h2v hv = {(_Float16)v0, (_Float16)v1};
                    __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2v*)(gt + idx), hv);
                }
            }
        }
    }
}

// Fixed-point gradient regions (shared memory, built by the whole block): the tables in address
// order -- a level's own table, or a shared MixedFeature table counted once (the levels sharing it
// have its offset) -- each with its table's 1/scale; lo_v[r] = first value index of region r.
struct TableRegions {
    float lvl_inv[MFN_MAX_LEVELS], inv_s[MFN_MAX_LEVELS];
    int64_t lo_v[MFN_MAX_LEVELS + 1];
    int n_reg;
    __device__ void build(const mfnerf_grid_desc& D, const float* __restrict__ level_l1, int64_t total_vals) {
        if (threadIdx.x < D.n_levels) {
            const float sc = table_fixed_scale(D, level_l1, threadIdx.x);
            lvl_inv[threadIdx.x] = sc > 0.0f ? 1.0f / sc : 0.0f;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int nr = 0;
            int64_t last = -1;
            for (int k = 0; k < D.n_levels; ++k) {
                if ((int64_t)D.offset[k] <= last) continue;
                last = D.offset[k];
                inv_s[nr] = lvl_inv[k];
                lo_v[nr++] = 2 * (int64_t)D.offset[k];
            }
            lo_v[nr] = total_vals;
            n_reg = nr;
        }
        __syncthreads();
    }
};

// grad[p] += sum_k priv[k][p]; priv[k][p] = 0 (ready for the next backward)
__global__ __launch_bounds__(256) void fold_copies_kernel(float* __restrict__ priv, int64_t n, float* __restrict__ grad) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 4; i += stride) {
        float4 acc = reinterpret_cast<float4*>(grad)[i];
#pragma unroll
        for (int k = 0; k < GRAD_COPIES; ++k) {
            float4* q = reinterpret_cast<float4*>(priv + k * n) + i;
            const float4 v = *q;
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            *q = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        reinterpret_cast<float4*>(grad)[i] = acc;
    }
}

// Fixed-point path: grad[p] (float) = sum_k priv[k][p] / scale for the dense prefix (copies zeroed),
// grad[p] = int(grad[p]) / scale for the rest; scale per level from the same level_l1 as grid_bw.
__global__ __launch_bounds__(256) void fold_convert_kernel(float* __restrict__ grad, int* __restrict__ priv,
                                                           int64_t dense_vals, int64_t total_vals,
                                                           const mfnerf_grid_desc D,
                                                           const float* __restrict__ level_l1) {
    // table regions in address order -- a level's own table, or a shared MixedFeature table counted
    // once (the levels sharing it have its offset) -- each with its table's scale
    __shared__ TableRegions R;
    R.build(D, level_l1, total_vals);
    const float* inv_s = R.inv_s;
    const int64_t* lo_v = R.lo_v;
    const int n_reg = R.n_reg;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int l = 0;  // region of value i (i increases per thread: walk forward)
    for (int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * i4 < total_vals; i4 += stride) {
        const int64_t i = 4 * i4;  // region boundaries are multiples of 16 values
        while (l + 1 < n_reg && i >= lo_v[l + 1]) ++l;
        const float is = inv_s[l];
        int4 acc;
        if (i < dense_vals) {
            acc = make_int4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < GRAD_COPIES; ++k) {
                int4* q = reinterpret_cast<int4*>(priv + k * dense_vals + i);
                const int4 v = *q;
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
                *q = make_int4(0, 0, 0, 0);
            }
            // the dense prefix's own entries in grad received no contributions (all went to copies)
        } else {
            acc = *reinterpret_cast<const int4*>(grad + i);
        }
        *reinterpret_cast<float4*>(grad + i) =
            make_float4((float)acc.x * is, (float)acc.y * is, (float)acc.z * is, (float)acc.w * is);
    }
}

// fold_convert + Adam in one pass (the unsharded, collective-free step): g[0, off) are float
// gradients (the MLPs), g[off, off + total_vals) the table's int32 fixed-point sums (the dense
// prefix's in GRAD_COPIES private copies); each value is converted exactly as fold_convert_kernel
// does, fed to the same Adam update as adam_kernel, and its gradient word (and copies) zeroed for
// the next step -- one pass over the gradient instead of a convert pass + a read in Adam.
__global__ __launch_bounds__(256) void adam_fixed_kernel(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         __half* __restrict__ p16, int64_t n, int64_t off,
                                                         int* __restrict__ priv, int64_t dense_vals,
                                                         int64_t total_vals, const mfnerf_grid_desc D,
                                                         float* __restrict__ level_l1, float lr, float b1,
                                                         float b2, float eps, int32_t* __restrict__ step_dev,
                                                         const float* __restrict__ lr_dev,
                                                         mfnerf_amp_state* __restrict__ amp, int n_levels) {
    __shared__ TableRegions R;
    R.build(D, level_l1, total_vals);
    const bool skipped = amp && amp->nonfinite;  // GradScaler: no update on a non-finite gradient, only the zeroing
    const int st = *step_dev + 1;
    if (lr_dev) lr = *lr_dev;
    const float bc1 = 1.0f - powf(b1, (float)st);
    const float bc2 = 1.0f - powf(b2, (float)st);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int l = 0;
    for (int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * i4 < n; i4 += stride) {
        const int64_t i = 4 * i4, j = i - off;  // off, dense_vals, region bounds: multiples of 4
        float4 gg;
        if (j < 0 || j >= total_vals) {
            gg = reinterpret_cast<const float4*>(g)[i4];
        } else {
            while (l + 1 < R.n_reg && j >= R.lo_v[l + 1]) ++l;
            const float is = R.inv_s[l];
            int4 acc;
            if (j < dense_vals) {
                acc = make_int4(0, 0, 0, 0);
#pragma unroll
                for (int k = 0; k < GRAD_COPIES; ++k) {
                    int4* q = reinterpret_cast<int4*>(priv + k * dense_vals + j);
                    const int4 c = *q;
                    acc.x += c.x; acc.y += c.y; acc.z += c.z; acc.w += c.w;
                    *q = make_int4(0, 0, 0, 0);
                }
            } else {
                acc = reinterpret_cast<const int4*>(g)[i4];
            }
            gg = make_float4((float)acc.x * is, (float)acc.y * is, (float)acc.z * is, (float)acc.w * is);
        }
        reinterpret_cast<float4*>(g)[i4] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (skipped) continue;
        float4 pp = reinterpret_cast<float4*>(p)[i4];
        float4 mm = reinterpret_cast<float4*>(m)[i4];
        float4 vv = reinterpret_cast<float4*>(v)[i4];
        mfn::adam_elem(pp.x, mm.x, vv.x, gg.x, b1, b2, eps, lr, bc1, bc2);
        mfn::adam_elem(pp.y, mm.y, vv.y, gg.y, b1, b2, eps, lr, bc1, bc2);
        mfn::adam_elem(pp.z, mm.z, vv.z, gg.z, b1, b2, eps, lr, bc1, bc2);
        mfn::adam_elem(pp.w, mm.w, vv.w, gg.w, b1, b2, eps, lr, bc1, bc2);
        reinterpret_cast<float4*>(p)[i4] = pp;
        reinterpret_cast<float4*>(m)[i4] = mm;
        reinterpret_cast<float4*>(v)[i4] = vv;
        if (p16) {
            __half2 a = __floats2half2_rn(pp.x, pp.y), b = __floats2half2_rn(pp.z, pp.w);
            uint2 u; u.x = *reinterpret_cast<uint32_t*>(&a); u.y = *reinterpret_cast<uint32_t*>(&b);
            reinterpret_cast<uint2*>(p16)[i4] = u;
        }
    }
    // step count / skip count / loss scale, and level_l1 zeroed for the next step's field_bw, by the
    // last workgroup (every workgroup has read level_l1, step_dev and the flag by now)
    if (amp) mfn::amp_step_end_last_block(step_dev, amp, level_l1, n_levels);
}

int64_t dense_entries_of(const mfnerf_grid_desc* d) {
    int64_t e = 0;  // dense own-table levels are laid out first (res grows with the level)
    for (int l = 0; l < d->n_levels; ++l) {
        const uint64_t r = d->res[l];
        if (d->table_kind[l] != 0 || r * r * r > d->size[l] || (int64_t)d->offset[l] != e) break;
        e += d->size[l];
    }
    return e;
}

// grid_bw's workgroup count cap (grid-stride beyond it).  MFNERF_GRID_BW_BLOCKS overrides the
// default for tuning experiments (tools/); read once.
int64_t grid_bw_block_cap() {
    static const int64_t cap = [] {
        const char* e = getenv("MFNERF_GRID_BW_BLOCKS");
        const long v = e ? atol(e) : 0;
        return (int64_t)(v > 0 ? v : 4096);
    }();
    return cap;
}

int check_desc(const mfnerf_grid_desc* d, const char* what) {
    if (!d) { mfn_set_error("%s: null grid desc", what); return MFN_ERR_INVALID; }
    if (d->n_features != 2 || d->n_levels <= 0 || d->n_levels > MFN_MAX_LEVELS || d->n_levels % 4 != 0) {
        mfn_set_error("%s: unsupported grid (n_features=%d must be 2, n_levels=%d must be a multiple of 4 <= %d)",
                      what, d->n_features, d->n_levels, MFN_MAX_LEVELS);
        return MFN_ERR_INVALID;
    }
    for (int l = 0; l < d->n_levels; ++l)
        if (d->size[l] == 0 || d->res[l] == 0 || d->table_kind[l] < 0 || d->table_kind[l] > 1) {
            mfn_set_error("%s: bad level %d", what, l); return MFN_ERR_INVALID;
        }
    return MFN_OK;
}

}  // namespace

extern "C" {

int mfnerf_grid_encode_fw(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                          const mfnerf_grid_desc* desc, const void* table_f16, void* out_f16,
                          mfnerf_stream_t stream) {
    int st = check_desc(desc, "grid_encode_fw");
    if (st) return st;
    if (n < 0) { mfn_set_error("grid_encode_fw: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!x || !table_f16 || !out_f16) { mfn_set_error("grid_encode_fw: null pointer"); return MFN_ERR_INVALID; }
    const int64_t want = div_up<int64_t>(n * (desc->n_levels / LEVELS_PER_LANE), ENC_BLOCK);
    const int64_t blocks = want < 8192 ? want : 8192;
    hipLaunchKernelGGL(grid_fw_kernel, dim3((unsigned)blocks), dim3(ENC_BLOCK), 0,
                       stream, x, n, n_dev, x_min, x_range, *desc, (const __half2*)table_f16, (__half*)out_f16);
    return mfn_check_launch("grid_encode_fw");
}

int mfnerf_grid_encode_fw_planar(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                 const mfnerf_grid_desc* desc, const void* table_f16, void* out_planes,
                                 int64_t plane_stride, mfnerf_stream_t stream) {
    int st = check_desc(desc, "grid_encode_fw_planar");
    if (st) return st;
    if (n < 0 || plane_stride < n) { mfn_set_error("grid_encode_fw_planar: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!x || !table_f16 || !out_planes) { mfn_set_error("grid_encode_fw_planar: null pointer"); return MFN_ERR_INVALID; }
    const int64_t want = div_up<int64_t>(n, ENC_BLOCK);
    const int64_t per_group = want < 2048 ? want : 2048;
    hipLaunchKernelGGL(grid_fw_planar_kernel, dim3((unsigned)(8 * per_group)), dim3(ENC_BLOCK), 0, stream, x, n, n_dev,
                       x_min, x_range, *desc, (const __half2*)table_f16, (__half2*)out_planes, plane_stride);
    return mfn_check_launch("grid_encode_fw_planar");
}

int64_t mfnerf_grid_encode_bw_workspace(const mfnerf_grid_desc* desc) {
    if (check_desc(desc, "grid_encode_bw_workspace")) return -1;
    return (int64_t)GRAD_COPIES * dense_entries_of(desc) * 2 * (int64_t)sizeof(float);
}

int mfnerf_grid_encode_bw_scatter(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                  const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                  void* workspace, const float* level_l1, mfnerf_stream_t stream) {
    int st = check_desc(desc, "grid_encode_bw");
    if (st) return st;
    if (n < 0) { mfn_set_error("grid_encode_bw: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!x || !dL_dout || !grad_table) { mfn_set_error("grid_encode_bw: null pointer"); return MFN_ERR_INVALID; }
    const int64_t want = div_up<int64_t>(div_up<int64_t>(n, 16), ENC_BLOCK / 64);
    const int64_t cap = grid_bw_block_cap();
    const int64_t blocks = want < cap ? want : cap;
    const int64_t dense = workspace ? dense_entries_of(desc) : 0;
    const bool big = desc->n_levels > 16;
    if (level_l1) {
        auto kern = big ? grid_bw_kernel<0, MFN_MAX_LEVELS, true> : grid_bw_kernel<0, 16, true>;
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(ENC_BLOCK), 0, stream, x, n, n_dev, x_min, x_range,
                           *desc, dL_dout, grad_table, (float*)workspace, dense, level_l1);
    } else {
        auto kern = big ? grid_bw_kernel<0, MFN_MAX_LEVELS, false> : grid_bw_kernel<0, 16, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(ENC_BLOCK), 0, stream, x, n, n_dev, x_min, x_range,
                           *desc, dL_dout, grad_table, (float*)workspace, dense, (const float*)nullptr);
    }
    return mfn_check_launch("grid_encode_bw_scatter");
}

int mfnerf_grid_encode_bw_finish(const mfnerf_grid_desc* desc, float* grad_table, void* workspace,
                                 const float* level_l1, mfnerf_stream_t stream) {
    int st = check_desc(desc, "grid_encode_bw_finish");
    if (st) return st;
    if (!grad_table) { mfn_set_error("grid_encode_bw_finish: null pointer"); return MFN_ERR_INVALID; }
    const int64_t dense = workspace ? dense_entries_of(desc) : 0;
    if (level_l1) {
        int64_t total = 0;
        for (int l = 0; l < desc->n_levels; ++l) {
            const int64_t e = 2 * ((int64_t)desc->offset[l] + desc->size[l]);
            total = e > total ? e : total;
        }
        const int64_t fb = div_up<int64_t>(total / 4, 256);
        hipLaunchKernelGGL(fold_convert_kernel, dim3((unsigned)(fb < 4096 ? fb : 4096)), dim3(256), 0, stream,
                           grad_table, (int*)workspace, 2 * dense, total, *desc, level_l1);
    } else if (dense > 0) {
        const int64_t nf = 2 * dense;  // multiple of 16 (level sizes are multiples of 8)
        const int64_t fb = div_up<int64_t>(nf / 4, 256);
        hipLaunchKernelGGL(fold_copies_kernel, dim3((unsigned)(fb < 2048 ? fb : 2048)), dim3(256), 0, stream,
                           (float*)workspace, nf, grad_table);
    }
    return mfn_check_launch("grid_encode_bw_finish");
}

int mfnerf_adam_step_fixed(float* params, float* grads, float* m, float* v, void* p_f16, int64_t n,
                           int64_t table_offset, const mfnerf_grid_desc* desc, void* workspace,
                           float* level_l1, float lr, float beta1, float beta2, float eps,
                           int32_t* step_dev, const float* lr_dev, mfnerf_amp_state* amp, mfnerf_stream_t stream) {
    int st = check_desc(desc, "adam_step_fixed");
    if (st) return st;
    if (!params || !grads || !m || !v || !step_dev || !level_l1) {
        mfn_set_error("adam_step_fixed: null pointer"); return MFN_ERR_INVALID;
    }
    if ((((uintptr_t)params) | ((uintptr_t)grads) | ((uintptr_t)m) | ((uintptr_t)v)) & 15 ||
        (p_f16 && (((uintptr_t)p_f16) & 7))) {
        mfn_set_error("adam_step_fixed: misaligned buffer"); return MFN_ERR_INVALID;
    }
    int64_t total = 0;
    for (int l = 0; l < desc->n_levels; ++l) {
        const int64_t e = 2 * ((int64_t)desc->offset[l] + desc->size[l]);
        total = e > total ? e : total;
    }
    const int64_t dense = workspace ? dense_entries_of(desc) : 0;
    if (n % 4 || table_offset % 4 || table_offset < 0 || table_offset + total > n) {
        mfn_set_error("adam_step_fixed: n (%lld) and table_offset (%lld) must be multiples of 4 holding the table",
                      (long long)n, (long long)table_offset);
        return MFN_ERR_INVALID;
    }
    const int64_t want = div_up<int64_t>(n / 4, 256);
    hipLaunchKernelGGL(adam_fixed_kernel, dim3((unsigned)(want < 4096 ? (want < 1 ? 1 : want) : 4096)), dim3(256), 0,
                       stream, params, grads, m, v, (__half*)p_f16, n, table_offset, (int*)workspace, 2 * dense,
                       total, *desc, level_l1, lr, beta1, beta2, eps, step_dev, lr_dev, amp, desc->n_levels);
    if (!amp)  // else the kernel's last workgroup did it
        hipLaunchKernelGGL(mfn_bump_step_kernel, dim3(1), dim3(1), 0, stream, step_dev, amp, level_l1, desc->n_levels);
    return mfn_check_launch("adam_step_fixed");
}

int mfnerf_grid_encode_bw(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                          const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table, void* workspace,
                          const float* level_l1, mfnerf_stream_t stream) {
    if (n == 0 && n >= 0) return MFN_OK;
    int st = mfnerf_grid_encode_bw_scatter(x, n, n_dev, x_min, x_range, desc, dL_dout, grad_table, workspace,
                                           level_l1, stream);
    if (st) return st;
    return mfnerf_grid_encode_bw_finish(desc, grad_table, workspace, level_l1, stream);
}

// Per-level L1 norm of dL/dout (n, L*F) f32: out[l] += sum_i |dy[i][2l]| + |dy[i][2l+1]| (the bound
// the fixed-point backward sizes its scales with, when the producer does not supply it).
__global__ __launch_bounds__(256) void level_l1_kernel(const float* __restrict__ dy, int64_t n,
                                                       const int32_t* __restrict__ n_dev, int L,
                                                       float* __restrict__ out) {
    __shared__ float part[MFN_MAX_LEVELS];
    if (threadIdx.x < L) part[threadIdx.x] = 0.0f;
    __syncthreads();
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int row = 2 * L;
    // flat (row, level) pairs f = t + k*S over the grid's first S = floor(threads / L) * L threads:
    // S is a multiple of L, so thread t always sees level l = t % L (any L, not only divisors of 64)
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t S = ((int64_t)gridDim.x * blockDim.x / L) * L;
    const int l = (int)(gt % L);
    float acc = 0.0f;
    if (gt < S)
        for (int64_t f = gt; f < nn * L; f += S) {
            const float2 v = *reinterpret_cast<const float2*>(dy + (f / L) * row + 2 * l);
            acc += fabsf(v.x) + fabsf(v.y);
        }
    if (64 % L == 0 && (blockDim.x % L) == 0) {
        // L divides the wave and the block: lanes l, l+L, ... of a wave share level l (block-local
        // lane index = global index mod L); reduce inside the wave first
        for (int off = 32; off >= L; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if ((threadIdx.x & 63) < L) atomicAdd(&part[l], acc);
    } else if (gt < S) {
        atomicAdd(&part[l], acc);
    }
    __syncthreads();
    if (threadIdx.x < L) atomicAdd(out + threadIdx.x, part[threadIdx.x]);
}

int mfnerf_debug_grid_bw_half(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                              const mfnerf_grid_desc* desc, const float* dL_dout, void* grad_h2, void* priv_h2,
                              float gscale, mfnerf_stream_t stream) {
    if (desc->n_levels > 16) { mfn_set_error("grid_bw_half: n_levels <= 16 only"); return MFN_ERR_INVALID; }
    const int64_t want = div_up<int64_t>(div_up<int64_t>(n, 16), ENC_BLOCK / 64);
    const int64_t cap = grid_bw_block_cap();
    const int64_t blocks = want < cap ? want : cap;
    const int64_t dense = priv_h2 ? dense_entries_of(desc) : 0;
    hipLaunchKernelGGL(grid_bw_h2_kernel<16>, dim3((unsigned)blocks), dim3(ENC_BLOCK), 0, stream, x, n, n_dev, x_min,
                       x_range, *desc, dL_dout, (h2v*)grad_h2, (h2v*)priv_h2, dense, gscale);
    return mfn_check_launch("grid_bw_half");
}

int mfnerf_grid_level_l1(const float* dL_dout, int64_t n, const int32_t* n_dev, int n_levels, float* out,
                         mfnerf_stream_t stream) {
    if (n < 0 || n_levels <= 0 || n_levels > MFN_MAX_LEVELS || !out || (n > 0 && !dL_dout)) {
        mfn_set_error("grid_level_l1: bad arguments"); return MFN_ERR_INVALID;
    }
    if (n == 0) return MFN_OK;
    // one workgroup per CU at most: the 16 per-level sums are atomics on 16 addresses, which
    // serialise at the memory side -- 2048 workgroups made this 36 us, most of it in that tail
    const int64_t want = div_up<int64_t>(n * n_levels, 256 * 16);
    hipLaunchKernelGGL(level_l1_kernel, dim3((unsigned)(want < 256 ? (want < 1 ? 1 : want) : 256)), dim3(256), 0,
                       stream, dL_dout, n, n_dev, n_levels, out);
    return mfn_check_launch("grid_level_l1");
}

// Debug (not part of the training path): the same launch with an ablated kernel body.
int mfnerf_debug_grid_bw_ablate(int mode, const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                mfnerf_stream_t stream) {
    const int64_t want = div_up<int64_t>(div_up<int64_t>(n, 16), ENC_BLOCK / 64);
    const int64_t blocks = want < 4096 ? want : 4096;
    if (desc->n_levels > 16) { mfn_set_error("grid_bw_ablate: n_levels <= 16 only"); return MFN_ERR_INVALID; }
    auto k = mode == 1   ? grid_bw_kernel<1, 16, false>
             : mode == 2 ? grid_bw_kernel<2, 16, false>
             : mode == 3 ? grid_bw_kernel<3, 16, false>
                         : grid_bw_kernel<0, 16, false>;
    hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(ENC_BLOCK), 0, stream, x, n, n_dev, x_min, x_range, *desc,
                       dL_dout, grad_table, nullptr, (int64_t)0, (const float*)nullptr);
    return mfn_check_launch("grid_bw_ablate");
}

}  // extern "C"
