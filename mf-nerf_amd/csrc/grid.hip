// grid.hip -- multiresolution grid encoding (tiny-cuda-nn HashGrid semantics, plus this repo's
// MixedFeature shared-table variant) forward and backward on gfx950.
//
// Forward: 4 lanes per point, each lane owns 4 consecutive levels (8 f16 features = one 16-B
// store), so the 4 lanes of a point write its 64-B output row with one coalesced 64-B burst and
// every lane keeps 32 independent 4-B corner gathers in flight.  Accumulation is fp32 (tcnn
// accumulates in half; the difference is inside the fp16 output rounding).
// Backward: see grid_bw_kernel (request-shaped float atomics with in-wave run merging).
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "field_pack.hpp"
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
// floor(x * rc / res) exactly, for x * rc < 2^31 (check_desc): the float quotient is within one of
// it (relative error ~2^-22 on a quotient <= 2^16), one integer correction each way.  A 64-bit
// division here (24 of them per sample-level, inlined) made the scatter kernels' code outgrow the
// instruction cache.
__device__ __forceinline__ uint32_t canon_coord(uint32_t x, uint32_t rc, uint32_t res, float inv) {
    const uint32_t n = x * rc;
    uint32_t q = (uint32_t)((float)n * inv);
    if (q * res > n) --q;
    else if ((q + 1) * res <= n) ++q;
    return q;
}

__device__ __forceinline__ uint32_t corner_index(const mfnerf_grid_desc& D, int l, uint32_t x, uint32_t y,
                                                 uint32_t z) {
    const uint32_t res = D.res[l], size = D.size[l];
    uint32_t idx;
    if (D.table_kind[l] == 1) {
        const uint32_t rc = (uint32_t)D.canon_res;
        const float inv = 1.0f / (float)res;  // one per level after CSE over the corners
        x = canon_coord(x, rc, res, inv);
        y = canon_coord(y, rc, res, inv);
        z = canon_coord(z, rc, res, inv);
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

// One (sample, level) of the planar forward in two phases: the gathers (issued for both of the
// lane's levels before any is used) and the interpolation.  Per (y,z) row every lane loads the 8 B
// holding its x-corner -- at idx (dense levels: idx+1 is the x+1 corner unless the index wraps) or
// at idx & ~1 (hashed power-of-two levels: the x+1 corner is idx ^ 1 when x is even), clamped into
// the table -- and loads the x+1 corner singly only where those 8 B miss it, so most rows cost one
// gather lane instead of two (the kernel is bound by per-lane gather addresses).  No branch chooses
// a load shape: round 4 did, per row, and used the row's values inside the branch, so each row's
// gather was waited for before the next one issued -- 8 dependent L2 round trips per lane and
// sample, 0.05 VMEM instructions in flight per wave (PMC r05_v22); and any merge of two shapes'
// results into one register (the compiler's phi copies) waits for the pending load as well.
struct PlanarGather {
    LevelGeo L;
    uint2 u[4];      // row yz: the 8 B holding the x-corner's half2
    uint32_t s[4];   // the x+1 corner's half2 where u misses it
    uint32_t f;      // row yz, bits 3 yz + {0: x-corner is u.y, 1: x+1 corner is in u, 2: ... as u.y}
};

__device__ __forceinline__ PlanarGather planar_gather(const mfnerf_grid_desc& D, const __half2* __restrict__ table,
                                                      int l, float x, float y, float z) {
    PlanarGather G;
    G.L = level_geo(D.scale[l], x, y, z);
    const uint32_t* __restrict__ tab = reinterpret_cast<const uint32_t*>(table + D.offset[l]);
    const uint32_t size = D.size[l], res = D.res[l];
    const bool dense = D.table_kind[l] == 0 && (uint64_t)res * res * res <= size;
    G.f = 0u;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t gy = G.L.g[1] + (yz & 1), gz = G.L.g[2] + (yz >> 1);
        const uint32_t i0 = corner_index(D, l, G.L.g[0], gy, gz);
        const uint32_t i1 = corner_index(D, l, G.L.g[0] + 1, gy, gz);
        const uint32_t a = min(dense ? i0 : (i0 & ~1u), size - 2u);  // i0 is a or a + 1
        G.u[yz] = *reinterpret_cast<const uint2*>(tab + a);
        const bool in_u = i1 - a < 2u;
        G.s[yz] = 0u;
        if (!in_u) G.s[yz] = tab[i1];
        G.f |= ((i0 != a ? 1u : 0u) | (in_u ? 2u : 0u) | (i1 != a ? 4u : 0u)) << (3 * yz);
    }
    return G;
}

__device__ __forceinline__ __half2 planar_interp(const PlanarGather& G) {
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        // integer masks, not selects, on the loaded words (a select between two of the struct's
        // loaded values may become a load from a selected address, the struct then in scratch)
        const uint32_t f = G.f >> (3 * yz);
        const uint32_t m0 = 0u - (f & 1u), m1 = 0u - ((f >> 1) & 1u), m2 = 0u - ((f >> 2) & 1u);
        const uint32_t lo = (G.u[yz].x & ~m0) | (G.u[yz].y & m0);
        const uint32_t hu = (G.u[yz].x & ~m2) | (G.u[yz].y & m2);
        const uint32_t hi = (hu & m1) | (G.s[yz] & ~m1);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float w = corner_weight(G.L, 2 * yz + c);
            const float2 v = __half22float2(__builtin_bit_cast(__half2, c ? hi : lo));
            a0 = fmaf(w, v.x, a0);
            a1 = fmaf(w, v.y, a1);
        }
    }
    return __floats2half2_rn(a0, a1);
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
        // this group's levels, visited directly: 16m + grp and 16m + 15 - grp (la < lb)
        for (int j = 0; j < nj; j += 2) {
            const int la = 16 * (j >> 1) + grp, lb = 16 * (j >> 1) + 15 - grp;
            if (la >= D.n_levels) continue;
            const bool has_b = lb < D.n_levels;  // (else level la is gathered twice, stored once)
            const PlanarGather Ga = planar_gather(D, table, la, x, y, z);
            const PlanarGather Gb = planar_gather(D, table, has_b ? lb : la, x, y, z);
            out[(int64_t)la * plane_stride + i] = planar_interp(Ga);
            if (has_b) out[(int64_t)lb * plane_stride + i] = planar_interp(Gb);
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
// power of two (8-64 copies measured the same; 1: grid_bw 0.300 -> 0.315 ms, 2: 0.306).  Round 6, the
// current dense kernel: 16 / 32 copies ran 0.538 / 0.638 vs 0.506 ms/step at Lego, 1.220 / 1.350 vs
// 1.184 at config 3's field (r6o: profiles/r06_v7_ab_dense_window.txt)
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

// the scatter as workgroup `bid` of `nblk` (a launch of its own, or a share of a fused launch)
template <int MAXL, bool FIX>
__device__ __forceinline__ void grid_bw_body(int bid, int nblk, const float* __restrict__ X, int64_t n,
                                             const int32_t* __restrict__ n_dev, float x_min, float x_range,
                                             const mfnerf_grid_desc& D, const float* __restrict__ dy,
                                             float* __restrict__ grad, float* __restrict__ priv,
                                             int64_t dense_entries, const float* __restrict__ level_l1, int l_end) {
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
    const int64_t wave0 = ((int64_t)bid * ENC_BLOCK + threadIdx.x) >> 6;
    const int64_t n_waves = ((int64_t)nblk * ENC_BLOCK) >> 6;
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
        for (int l = l_end >> 8; l < (l_end & 255); ++l) {  // levels [l_end >> 8, l_end & 255)
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
                if (FIX && spread) {  // private copies: both features as one packed 64-bit add
                    const int q = (int)rintf(v * fs);
                    const int q1 = __shfl_down(q, 16, 64);  // the f = 1 lane of this (sample, corner)
                    const long long pq = (long long)((uint64_t)(uint32_t)q1 << 32) + (long long)q;
                    if (f == 0 && head && valid && pq != 0)
                        __hip_atomic_fetch_add(reinterpret_cast<long long*>(gt) + idx, pq, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                } else if (FIX) {
                    const int q = (int)rintf(v * fs);
                    if (head && valid && q != 0)
                        __hip_atomic_fetch_add(reinterpret_cast<int*>(gt) + 2 * idx + f, q, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                } else if (head && valid && v != 0.0f) {
                    __hip_atomic_fetch_add(gt + 2 * idx + f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
    }
}

template <int MAXL, bool FIX>
__global__ __launch_bounds__(ENC_BLOCK) void grid_bw_kernel(const float* __restrict__ X, int64_t n,
                                                             const int32_t* __restrict__ n_dev, float x_min,
                                                             float x_range, const mfnerf_grid_desc D,
                                                             const float* __restrict__ dy, float* __restrict__ grad,
                                                             float* __restrict__ priv, int64_t dense_entries,
                                                             const float* __restrict__ level_l1, int l_end,
                                                             int32_t* __restrict__ zero_flag) {
    // zero_flag: a flag the NEXT launches on the stream start from zero (the binned scatter's slot
    // overflow), cleared here instead of by a memset launch of its own
    if (zero_flag && blockIdx.x == 0 && threadIdx.x == 0) *zero_flag = 0;
    grid_bw_body<MAXL, FIX>(blockIdx.x, gridDim.x, X, n, n_dev, x_min, x_range, D, dy, grad, priv,
                                    dense_entries, level_l1, l_end);
}

// Dense own-table levels [0, l_hi) into the private copies, one SAMPLE per lane.  grid_bw_body
// gives each sample 4 lanes (x-corner x feature) and merges runs with float segmented scans: it is
// VALU-bound (PMC: ~58 VALU wave-instructions per 16-sample row step; the same time with its
// atomics compiled out).  Here a lane holds its sample's whole cell (4 (y,z) rows x 2 x-corners x
// 2 features = 16 values) and a wave covers 64 consecutive samples (~ a ray):
//   * each value is rounded to the table's int32 fixed-point unit first (one rounding per sample
//     contribution); the run sums then come from an UNSEGMENTED integer prefix scan over the wave
//     (DPP row_shr 1/2/4/8 + row_bcast:15/:31 -- one v_add per step and value) as
//     P(tail) - P_excl(head): exact and order-free in two's complement;
//   * a run = consecutive samples in one cell (the 4 rows' keys change together), so one head/tail
//     structure serves all 16 values; heads and tails write their prefixes into a per-wave LDS
//     list, one entry per run;
//   * the list is issued 8 lanes per run -- (row, x-corner) -- each one 64-bit atomic carrying BOTH
//     features as the packed integer f1 * 2^32 + f0 (the fold decodes f0 = int32(low word),
//     f1 = int32(high word) + (f0 < 0); |sums| < 2^31 by the scale bound): a run costs 4 requests
//     (one 16-B span per row), 8 runs per instruction.
// Requires every level < l_hi to be a dense own table inside the private copies.

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ int dppz_i(int v) {  // lanes without a source (or outside ROW_MASK) read 0
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xF, false);
}

// a wave's window: consecutive chunks of 64 samples; the run open at a chunk's end is carried into
// the next chunk (per level, in LDS) instead of being issued twice.  Round 3 A/B (kbench, Lego step):
// 4 chunks 85 us; the smaller windows tried measured 95-101 us.  Round 6: the window is sized on the
// device from the live sample count so that ~DENSE_WAVES waves run, one window each -- the fixed
// 4-chunk window's optimum at the Lego step (~490 k samples: 1.9 k waves); at twice the samples
// (config 3's field, 16384 rays) 8 chunks ran 1.148 vs 1.184 ms/step, where the Lego step at 8
// chunks (960 waves) ran 0.526 vs 0.506 (r6o: profiles/r06_v7_ab_dense_window.txt).
#ifndef MFN_DENSE_WAVES
#define MFN_DENSE_WAVES 2048
#endif
constexpr int DENSE_WAVES = MFN_DENSE_WAVES;

struct DenseIn {
    float px, py, pz;
    bool valid;
};

template <int NG>  // float4 groups of dL/dy held per lane: levels < 2 NG
__global__ __launch_bounds__(ENC_BLOCK) void grid_bw_dense_kernel(const float* __restrict__ X, int64_t n,
                                                                  const int32_t* __restrict__ n_dev, float x_min,
                                                                  float x_range, const mfnerf_grid_desc D,
                                                                  const float* __restrict__ dy,
                                                                  float* __restrict__ priv, int64_t dense_entries,
                                                                  const float* __restrict__ level_l1, int l_hi,
                                                                  int32_t* __restrict__ zero_flag,
                                                                  int32_t* __restrict__ gate) {
    if (zero_flag && blockIdx.x == 0 && threadIdx.x == 0) *zero_flag = 0;
    // gate (gate.hip's {signals, waits, ticket}): opened as the table-gradient launches begin, so the
    // side stream's next march starts beside them with no one-thread signal kernel of its own on
    // the step's critical path
    if (gate && blockIdx.x == 0 && threadIdx.x == 0)  // relaxed: placement only (gate.hip)
        __hip_atomic_fetch_add(gate, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __shared__ float fs_s[MFN_MAX_LEVELS];
    // per wave, one entry per run: the 4 rows' (x0, x1) keys and the inclusive prefix at the run's
    // tail of the 16 values as 4 int4 (row r: x0f0, x0f1, x1f0, x1f1).  The runs tile the chunk's
    // valid lanes in order, so run r's exclusive prefix at its head is run r-1's tail prefix (0 for
    // r = 0): no head list (round 3: 45 -> 28 KB of LDS per block, 3 -> 4 blocks per CU)
    __shared__ int2 lkey[ENC_BLOCK / 64][64][4];
    __shared__ int4 ltail[ENC_BLOCK / 64][64][4];
    // per wave and level: the run left open at the previous chunk's end (sums, keys, on/off)
    __shared__ int4 csum[ENC_BLOCK / 64][2 * NG][4];
    __shared__ int2 ckey[ENC_BLOCK / 64][2 * NG][4];
    __shared__ int con[ENC_BLOCK / 64][2 * NG];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if ((int)threadIdx.x < D.n_levels) fs_s[threadIdx.x] = table_fixed_scale(D, level_l1, threadIdx.x);
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t n_waves = ((int64_t)gridDim.x * ENC_BLOCK) >> 6;
    const int row = 2 * D.n_levels;
    __syncthreads();  // fs_s
    auto load = [&](int64_t i, DenseIn& in, float4* gq) {
        in.valid = i < nn;
        in.px = in.valid ? (X[3 * i] - x_min) / x_range : 0.0f;
        in.py = in.valid ? (X[3 * i + 1] - x_min) / x_range : 0.0f;
        in.pz = in.valid ? (X[3 * i + 2] - x_min) / x_range : 0.0f;
        const float4* src = reinterpret_cast<const float4*>(dy + (in.valid ? i : 0) * row);
        const int ng = (2 * l_hi + 3) >> 2;
#pragma unroll
        for (int j = 0; j < NG; ++j) gq[j] = (in.valid && j < ng) ? src[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    const int64_t win = max<int64_t>(1, (nn + 64 * DENSE_WAVES - 1) / (64 * DENSE_WAVES));  // chunks (uniform)
    for (int64_t w = ((int64_t)blockIdx.x * ENC_BLOCK + threadIdx.x) >> 6; w * 64 * win < nn; w += n_waves) {
        const int64_t i0 = w * 64 * win;
        for (int l = lane; l < l_hi; l += 64) con[wv][l] = 0;
        DenseIn in, nx;
        float4 gq[NG], gn[NG];
        load(i0 + lane, in, gq);
        for (int k = 0; k < win && i0 + 64 * k < nn; ++k) {
            const bool more = k + 1 < win && i0 + 64 * (k + 1) < nn;
            if (more) load(i0 + 64 * (k + 1) + lane, nx, gn);  // in flight during this chunk's atomics
            const bool valid = in.valid;
            for (int l = 0; l < l_hi; ++l) {
                float g0 = 0.f, g1 = 0.f;
#pragma unroll
                for (int j = 0; j < NG; ++j) {  // uniform-index select of level l's pair
                    if (2 * j == l) { g0 = gq[j].x; g1 = gq[j].y; }
                    if (2 * j + 1 == l) { g0 = gq[j].z; g1 = gq[j].w; }
                }
                const float fs = fs_s[l];
                const LevelGeo Lg = level_geo(D.scale[l], in.px, in.py, in.pz);
                // dense index x + y res + z res^2 with corner_index's `% size`: corners of points in
                // [0,1]^3 stay below 2 size, where one conditional subtraction is that modulo
                const uint32_t res = D.res[l], size = D.size[l];
                int key[4], key1[4];
                bool far = false;
#pragma unroll
                for (int yz = 0; yz < 4; ++yz) {
                    const uint32_t gy = Lg.g[1] + (yz & 1), gz = Lg.g[2] + (yz >> 1);
                    const uint32_t k0 = Lg.g[0] + (gy + gz * res) * res, k1 = k0 + 1;
                    far |= valid && (k1 >= 2 * size || k1 < k0);
                    key[yz] = (int)(k0 >= size ? k0 - size : k0);
                    key1[yz] = (int)(k1 >= size ? k1 - size : k1);
                }
                if (__builtin_expect(__ballot(far) != 0, 0)) {  // points far outside the unit cube
#pragma unroll
                    for (int yz = 0; yz < 4; ++yz) {
                        const uint32_t gy = Lg.g[1] + (yz & 1), gz = Lg.g[2] + (yz >> 1);
                        key[yz] = (int)corner_index(D, l, Lg.g[0], gy, gz);
                        key1[yz] = (int)corner_index(D, l, Lg.g[0] + 1, gy, gz);
                    }
                }
                // the 16 contributions, each rounded once to the fixed-point unit
                int q[4][4];
                {
                    const float a0 = g0 * fs, a1 = g1 * fs;
                    const float w1 = Lg.w[0], w0 = 1.0f - Lg.w[0];
#pragma unroll
                    for (int yz = 0; yz < 4; ++yz) {
                        const float wy = (yz & 1) ? Lg.w[1] : 1.0f - Lg.w[1];
                        const float wz = (yz >> 1) ? Lg.w[2] : 1.0f - Lg.w[2];
                        const float wyz = wy * wz;
                        const float c0 = w0 * wyz, c1 = w1 * wyz;
                        q[yz][0] = valid ? (int)rintf(c0 * a0) : 0;
                        q[yz][1] = valid ? (int)rintf(c0 * a1) : 0;
                        q[yz][2] = valid ? (int)rintf(c1 * a0) : 0;
                        q[yz][3] = valid ? (int)rintf(c1 * a1) : 0;
                    }
                }
                // runs: consecutive samples in one cell (row 0's key identifies the cell)
                const int cell = valid ? key[0] : -1;
                // the run left open by the previous chunk: lane 0 continues it (its sums join lane
                // 0's values before the scan), or it is flushed as one more list entry
                const bool carried = con[wv][l] != 0;
                const bool cont = carried && lane == 0 && cell == ckey[wv][l][0].x;
                if (cont) {
#pragma unroll
                    for (int yz = 0; yz < 4; ++yz) {
                        const int4 c = csum[wv][l][yz];
                        q[yz][0] += c.x; q[yz][1] += c.y; q[yz][2] += c.z; q[yz][3] += c.w;
                    }
                }
                const bool flush = carried && !__shfl(cont ? 1 : 0, 0, 64);
                const int cp = __builtin_amdgcn_update_dpp(-2, cell, 0x138, 0xF, 0xF, false);  // wave_shr:1
                const int cn = __builtin_amdgcn_update_dpp(-2, cell, 0x130, 0xF, 0xF, false);  // wave_shl:1
                const bool head = valid && (lane == 0 || cp != cell);
                const bool tail = valid && (lane == 63 || cn != cell);
                // inclusive prefix sums over the wave (wraparound int32: differences are exact)
                int P[4][4];
#pragma unroll
                for (int yz = 0; yz < 4; ++yz)
#pragma unroll
                    for (int c = 0; c < 4; ++c) P[yz][c] = q[yz][c];
#define MFN_PSTEP(CTRL, RM)                                                                   \
    _Pragma("unroll") for (int yz = 0; yz < 4; ++yz)                                          \
        _Pragma("unroll") for (int c = 0; c < 4; ++c) P[yz][c] += dppz_i<CTRL, RM>(P[yz][c]);
                MFN_PSTEP(0x111, 0xF) MFN_PSTEP(0x112, 0xF) MFN_PSTEP(0x114, 0xF) MFN_PSTEP(0x118, 0xF)
                MFN_PSTEP(0x142, 0xA) MFN_PSTEP(0x143, 0xC)
#undef MFN_PSTEP
                // run index of each lane = heads at or before it - 1; tails write the inclusive
                // prefix and the keys
                const uint64_t hb = __ballot(head);
                const int nruns = __popcll(hb);
                const int run = __builtin_amdgcn_mbcnt_hi((uint32_t)(hb >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)hb, 0u)) + (head ? 0 : -1);
                if (tail) {
#pragma unroll
                    for (int yz = 0; yz < 4; ++yz) {
                        ltail[wv][run][yz] = make_int4(P[yz][0], P[yz][1], P[yz][2], P[yz][3]);
                        lkey[wv][run][yz] = make_int2(key[yz], key1[yz]);
                    }
                }
                long long* gt = reinterpret_cast<long long*>(priv) +
                                ((w & (GRAD_COPIES - 1)) * dense_entries + (int64_t)D.offset[l]);
                // one run's 16 sums, 8 lanes = (row, x-corner), both features packed in one 64-bit add
                auto issue = [&](int4 t, int2 kp, int c) {
                    const int f0 = c ? t.z : t.x, f1 = c ? t.w : t.y;
                    const long long pq = (long long)((uint64_t)(uint32_t)f1 << 32) + (long long)f0;
                    if (pq != 0)
                        __hip_atomic_fetch_add(gt + (c ? kp.y : kp.x), pq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                };
                // the run carried from the previous chunk that lane 0 did not continue: issued on its own
                if (flush && lane < 8) issue(csum[wv][l][(lane >> 1) & 3], ckey[wv][l][(lane >> 1) & 3], lane & 1);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                __builtin_amdgcn_wave_barrier();
                int nl = nruns;
                // the run at lane 63 stays open when the window's next chunk follows: carried (its
                // sums = its tail prefix minus the previous run's), and left out of this list
                con[wv][l] = 0;
                if (more && nruns > 0 && __shfl(tail ? 1 : 0, 63, 64)) {
                    const int r = nruns - 1;
                    if (lane < 4) {
                        const int4 t = ltail[wv][r][lane];
                        const int4 h = r > 0 ? ltail[wv][r - 1][lane] : make_int4(0, 0, 0, 0);
                        csum[wv][l][lane] = make_int4(t.x - h.x, t.y - h.y, t.z - h.z, t.w - h.w);
                        ckey[wv][l][lane] = lkey[wv][r][lane];
                    }
                    con[wv][l] = 1;
                    nl -= 1;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
                for (int b = 0; b < nl; b += 8) {
                    const int r = b + (lane >> 3), yz = (lane >> 1) & 3;
                    if (r < nl) {
                        const int4 t = ltail[wv][r][yz];
                        const int4 h = r > 0 ? ltail[wv][r - 1][yz] : make_int4(0, 0, 0, 0);
                        issue(make_int4(t.x - h.x, t.y - h.y, t.z - h.z, t.w - h.w), lkey[wv][r][yz], lane & 1);
                    }
                }
                __builtin_amdgcn_wave_barrier();  // the list is rewritten by the next level
            }
            if (more) {
                in = nx;
#pragma unroll
                for (int j = 0; j < NG; ++j) gq[j] = gn[j];
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
// The private copies of the fixed-point path hold each entry's two features as ONE packed integer
// f1 * 2^32 + f0 (64-bit atomics carry both; grid_bw_dense_kernel, grid_bw_body): the sum of the
// copies is exact in int64, and f0 = int32(low word), f1 = int32(high word) + (f0 < 0) undoes the
// borrow of a negative f0.  Values i .. i+3 (entries i/2, i/2+1); the copies are zeroed.
__device__ __forceinline__ int4 fold_packed_copies(int* __restrict__ priv, int64_t dense_vals, int64_t i) {
    // every copy's load issued before the first zeroing store (a load-store pair per copy in turn
    // made the fold one memory round trip per copy: ~55 us of fixed cost in the optimizer pass)
    longlong2 c[GRAD_COPIES];
#pragma unroll
    for (int k = 0; k < GRAD_COPIES; ++k) c[k] = *reinterpret_cast<const longlong2*>(priv + k * dense_vals + i);
    long long a = 0, b = 0;
#pragma unroll
    for (int k = 0; k < GRAD_COPIES; ++k) {
        a += c[k].x;
        b += c[k].y;
        *reinterpret_cast<longlong2*>(priv + k * dense_vals + i) = make_longlong2(0, 0);
    }
    const int a0 = (int)(uint32_t)(unsigned long long)a, b0 = (int)(uint32_t)(unsigned long long)b;
    return make_int4(a0, (int)(a >> 32) + (a0 < 0), b0, (int)(b >> 32) + (b0 < 0));
}

// ShardFlag (the data-parallel step): the step's non-finite flag into the first value of every
// exchange shard (NaN; mfnerf_flag_to_shards's job, without its launch) -- values this pass writes
// get it as they are written, the others (written by earlier launches) from workgroup 0.
struct ShardFlag {
    const int32_t* flag;  // NULL: none
    int64_t world, shard_len, table_off;  // grad[i] is flat value table_off + i
};

__global__ __launch_bounds__(256) void fold_convert_kernel(float* __restrict__ grad, int* __restrict__ priv,
                                                           int64_t dense_vals, int64_t total_vals,
                                                           const mfnerf_grid_desc D,
                                                           const float* __restrict__ level_l1,
                                                           const ShardFlag SF = ShardFlag{}) {
    // table regions in address order -- a level's own table, or a shared MixedFeature table counted
    // once (the levels sharing it have its offset) -- each with its table's scale
    __shared__ TableRegions R;
    R.build(D, level_l1, total_vals);
    const float* inv_s = R.inv_s;
    const int64_t* lo_v = R.lo_v;
    const int n_reg = R.n_reg;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const bool raise = SF.flag && *SF.flag;
    if (raise && blockIdx.x == 0 && (int64_t)threadIdx.x < SF.world) {
        const int64_t f = (int64_t)threadIdx.x * SF.shard_len - SF.table_off;  // relative to grad
        if (f < 0 || f >= total_vals) grad[f] = __int_as_float(0x7fc00000);
    }
    int l = 0;  // region of value i (i increases per thread: walk forward)
    for (int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * i4 < total_vals; i4 += stride) {
        const int64_t i = 4 * i4;  // region boundaries are multiples of 16 values
        while (l + 1 < n_reg && i >= lo_v[l + 1]) ++l;
        const float is = inv_s[l];
        int4 acc;
        if (i < dense_vals) {
            acc = fold_packed_copies(priv, dense_vals, i);
            // the dense prefix's own entries in grad received no contributions (all went to copies)
        } else {
            acc = *reinterpret_cast<const int4*>(grad + i);
        }
        float4 o = make_float4((float)acc.x * is, (float)acc.y * is, (float)acc.z * is, (float)acc.w * is);
        if (raise) {
            float* oc = &o.x;
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if ((SF.table_off + i + c) % SF.shard_len == 0 && (SF.table_off + i + c) / SF.shard_len < SF.world)
                    oc[c] = __int_as_float(0x7fc00000);
        }
        *reinterpret_cast<float4*>(grad + i) = o;
    }
}

// fold_convert + Adam in one pass (the unsharded, collective-free step): g[0, off) are float
// gradients (the MLPs), g[off, off + total_vals) the table's int32 fixed-point sums (the dense
// prefix's in GRAD_COPIES private copies); each value is converted exactly as fold_convert_kernel
// does, fed to the same Adam update as adam_kernel, and its gradient word (and copies) zeroed for
// the next step -- one pass over the gradient instead of a convert pass + a read in Adam.
// The float4 groups [i4_first, i4_end) step `stride` (a grid-stride loop over the caller's threads).
__device__ __forceinline__ void adam_fixed_body(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                float* __restrict__ v, __half* __restrict__ p16, int64_t off,
                                                int* __restrict__ priv, int64_t dense_vals, int64_t total_vals,
                                                const TableRegions& R, float lr, float b1, float b2, float eps,
                                                float bc1, float bc2, bool skipped, int64_t i4_first,
                                                int64_t i4_end, int64_t stride) {
    int l = 0;
    for (int64_t i4 = i4_first; i4 < i4_end; i4 += stride) {
        const int64_t i = 4 * i4, j = i - off;  // off, dense_vals, region bounds: multiples of 4
        float4 gg;
        if (j < 0 || j >= total_vals) {
            gg = reinterpret_cast<const float4*>(g)[i4];
        } else {
            while (l + 1 < R.n_reg && j >= R.lo_v[l + 1]) ++l;
            const float is = R.inv_s[l];
            int4 acc;
            if (j < dense_vals) {
                acc = fold_packed_copies(priv, dense_vals, j);
            } else {
                acc = reinterpret_cast<const int4*>(g)[i4];
            }
            gg = make_float4((float)acc.x * is, (float)acc.y * is, (float)acc.z * is, (float)acc.w * is);
        }
        reinterpret_cast<float4*>(g)[i4] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (skipped) continue;
        float4 pp = mfn::nt_load4(p + 4 * i4);
        float4 mm = mfn::nt_load4(m + 4 * i4);
        float4 vv = mfn::nt_load4(v + 4 * i4);
        mfn::adam_elem(pp.x, mm.x, vv.x, gg.x, b1, b2, eps, lr, bc1, bc2);
        mfn::adam_elem(pp.y, mm.y, vv.y, gg.y, b1, b2, eps, lr, bc1, bc2);
        mfn::adam_elem(pp.z, mm.z, vv.z, gg.z, b1, b2, eps, lr, bc1, bc2);
        mfn::adam_elem(pp.w, mm.w, vv.w, gg.w, b1, b2, eps, lr, bc1, bc2);
        mfn::nt_store4(p + 4 * i4, pp);
        mfn::nt_store4(m + 4 * i4, mm);
        mfn::nt_store4(v + 4 * i4, vv);
        if (p16) {
            __half2 a = __floats2half2_rn(pp.x, pp.y), b = __floats2half2_rn(pp.z, pp.w);
            uint2 u; u.x = *reinterpret_cast<uint32_t*>(&a); u.y = *reinterpret_cast<uint32_t*>(&b);
            reinterpret_cast<uint2*>(p16)[i4] = u;
        }
    }
}

// the MLP weights' repack riding the optimizer's last pass (out = nullptr: none)
struct PackArgs {
    const _Float16* px;  // xyz MLP (fp16 compute copy)
    const _Float16* pr;  // rgb MLP
    _Float16* out;       // the field head's fragment blob (mfnerf_field_pack_weights_f16's layout)
    int width;           // rgb width, 64 or 128
};

// tail_mode 0: values [0, n), or [0, fused_from) when the fused partitioned accumulate updated the
// rest (fused_ovf given; overflowed records included -- the accumulate adds them).  tail_mode 1
// (mfnerf_grid_encode_bw_binned_adam_all, whose accumulate launch updated every value): nothing but
// the MLP repack and the step's bookkeeping.
__global__ __launch_bounds__(256) void adam_fixed_kernel(float* __restrict__ p, float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         __half* __restrict__ p16, int64_t n, int64_t off,
                                                         int* __restrict__ priv, int64_t dense_vals,
                                                         int64_t total_vals, const mfnerf_grid_desc D,
                                                         float* __restrict__ level_l1, float lr, float b1,
                                                         float b2, float eps, int32_t* __restrict__ step_dev,
                                                         const float* __restrict__ lr_dev,
                                                         mfnerf_amp_state* __restrict__ amp, int n_levels,
                                                         int64_t fused_from, const int32_t* __restrict__ fused_ovf,
                                                         int tail_mode, const PackArgs pk) {
    __shared__ TableRegions R;
    int64_t lo = 0;
    if (tail_mode == 1) n = 0;                 // the accumulate launch updated every value
    else if (fused_ovf) n = fused_from;        // values >= fused_from: updated by the accumulate
    if (n > lo) {  // (uniform)
        R.build(D, level_l1, total_vals);
        const bool skipped = amp && amp->nonfinite;  // GradScaler: no update on a non-finite gradient, only the zeroing
        const int st = *step_dev + 1;
        if (lr_dev) lr = *lr_dev;
        const float bc1 = 1.0f - powf(b1, (float)st);
        const float bc2 = 1.0f - powf(b2, (float)st);
        const int64_t stride = (int64_t)gridDim.x * blockDim.x;
        adam_fixed_body(p, g, m, v, p16, off, priv, dense_vals, total_vals, R, lr, b1, b2, eps, bc1, bc2, skipped,
                        lo / 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x, n / 4, stride);
    }
    // tail_mode 1: the MLP weights' repack (their p16 was written by the accumulate launch)
    if (pk.out) {
        const int total = (pk.width == 64 ? mfn_field::Geo<64>::N : mfn_field::Geo<128>::N) * mfn_field::FRAG_HALFS;
        for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
            if (pk.width == 64) mfn_field::pack_elem<_Float16, 64>(t, pk.px, pk.pr, pk.out);
            else mfn_field::pack_elem<_Float16, 128>(t, pk.px, pk.pr, pk.out);
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

// grid_bw's workgroup count cap (grid-stride beyond it; 4096 / 1024 / 512 / 256 / 128 measured
// 832 / 860 / 855 / 869 / 1166 us for the round-1 float scatter)
int64_t grid_bw_block_cap() { return 4096; }

int check_desc(const mfnerf_grid_desc* d, const char* what) {
    if (!d) { mfn_set_error("%s: null grid desc", what); return MFN_ERR_INVALID; }
    if (d->n_features != 2 || d->n_levels <= 0 || d->n_levels > MFN_MAX_LEVELS || d->n_levels % 4 != 0) {
        mfn_set_error("%s: unsupported grid (n_features=%d must be 2, n_levels=%d must be a multiple of 4 <= %d)",
                      what, d->n_features, d->n_levels, MFN_MAX_LEVELS);
        return MFN_ERR_INVALID;
    }
    for (int l = 0; l < d->n_levels; ++l)
        if (d->size[l] == 0 || d->res[l] == 0 || d->table_kind[l] < 0 || d->table_kind[l] > 1 ||
            // the canonical-grid map computes (coord + 1) * canon_res in 32 bits (canon_coord)
            (d->table_kind[l] == 1 && ((uint64_t)d->res[l] + 2) * (uint64_t)d->canon_res >= (1ull << 31))) {
            mfn_set_error("%s: bad level %d", what, l); return MFN_ERR_INVALID;
        }
    return MFN_OK;
}

// ------------------------------------------------------------------------------------------------
// Partitioned table-gradient scatter ("binned").  The hashed levels' tables are small (2^19 entries
// = 4 MB of int32 pairs per level at the Lego config) and uniformly hit: every 64-B line receives
// ~30 adds per step from unrelated rays, so no ordering of the samples lets memory-side atomics
// merge them (tools/sim_scatter_requests.py: >= 3 requests per sample per fine level in any window
// of a Morton-sorted batch, 0.13 distinct lines per sample over the whole batch).  Instead each
// table is cut into 2^shift-entry partitions, every (sample, level, (y,z) corner row) becomes an
// 8-B record (entry, x weight, both features' values in fp16: the algorithmic fp16 scatter's own
// payload; 12 B with f32 values until round 3) routed to its partition by a counting sort, and one workgroup per partition sums its
// records into an LDS image with integer LDS atomics (ds_add_u32: ~4 T adds/s chip-wide at random
// addresses, tools/lds_atomic_probe.hip -- 20x ds_add_f32), then stores the image once.  The image
// holds one 64-bit word per entry: both features' sums in the table's int32 fixed-point unit,
// packed f1 * 2^32 + f0 (exact in two's complement, order-free: bit-reproducible), each weighted
// contribution rounded once to the unit -- 2 LDS atomics per pair record (an int64 image per
// feature at 2^32 x the unit, 4 atomics and a float -> int64 conversion per record, measured 349 vs
// 316 us for the whole scatter in round 2).  Passes: scatter (records into fixed per-(partition,
// unit) slots) -> accumulate (one workgroup per partition).
// partitions of 2^shift entries, shift in [MIN_BIN_SHIFT, MAX_BIN_SHIFT] chosen per layout so that
// there are >= ~1024 partitions (4 workgroups per CU); 2^11 entries = 16 KB of packed int32 pairs
constexpr int MIN_BIN_SHIFT = 8, MAX_BIN_SHIFT = 11, MAX_BIN_ENTRIES = 1 << MAX_BIN_SHIFT;
// partitions over all binned tables: the first LDS_CURSOR keep the scatter unit's running counts in
// LDS, the rest (own tables of 2^20-2^21 entries: --T 20/21, opt.py:78) in the unit's column of the
// slot counts in global memory, read and written by the one scanning wave (LDS for all 5120 of the
// T 2^20 layout measured the same: 0.654 vs 0.654 ms/step, r05_v27)
constexpr int LDS_CURSOR = 4096, MAX_BINS = 16384;

struct BinPlan {
    int n_binned;                    // levels routed through the bins
    int n_bins;                      // partitions over all their tables
    int n_tables;
    int shift;                       // partition = 2^shift entries of one table
    int pair_ok;                     // no x-pair can straddle two partitions (one record per row)
    int level[MFN_MAX_LEVELS];       // binned level list
    int pairable[MFN_MAX_LEVELS];    // per level: x+1's entry = x's entry ^ (x ^ (x+1)) (own power-of-two hash)
    int merge[MFN_MAX_LEVELS];       // per level: never a pair record -> runs merged (merged_level_records)
    int table_of[MFN_MAX_LEVELS];    // per level: its table
    uint32_t t_offset[MFN_MAX_LEVELS], t_size[MFN_MAX_LEVELS];
    int t_bin0[MFN_MAX_LEVELS + 1];  // first bin of each table; t_bin0[n_tables] = n_bins
    int t_level[MFN_MAX_LEVELS];     // a level of each table (its fixed-point scale)
};

__device__ __forceinline__ int bin_table(const BinPlan& P, int b) {
    int t = 0;
    while (t + 1 < P.n_tables && b >= P.t_bin0[t + 1]) ++t;
    return t;
}

// The records of one (sample, binned level j): up to 4 (y,z) rows x (1 or 2 records).  EMIT(bin,
// rec) is called per record; rec = {w0, a | b << 16} (8 B): a/b = wy*wz*dL/dy_f * scale * 2^-15 as
// fp16 (scale: the table's int32 fixed-point scale, so |wy*wz*dL/dy_f * scale| < 2^30 and the fp16
// value < 2^15 never overflows; rounded once to 11 significant bits -- the precision of the fp16
// operands field_bw computed dL/dy from, and of tcnn's own half-precision gradient, whose SUM is
// rounded to fp16 at every add) and
//   w0 = e0 (bits 0-10, entry in the bin) | t << 11 (4 bits) | single << 15 | sel << 16 | fx << 17,
// fx = the x weight as 15-bit unorm (exact for the fine levels, whose positions carry <= 13
// fraction bits).  A pair record adds (1-fx)(a,b) to e0 and fx(a,b) to e1 = e0 ^ ((2^(t+1) - 1) << s),
// s = bit 16 (sel has no meaning in a pair record): an own power-of-two hash table has idx(x+1) =
// idx(x) ^ (x ^ (x+1)), t = trailing ones of x, s = 0, and the two share a bin unless the carry
// reaches bit `shift` (1 x in 2^shift).  A shared MixedFeature table hashes the canonical coordinates
// c(x): where c(x+1) = c(x) + 1 the same holds with t = trailing ones of c(x); where c(x+1) = c(x) + 2
// (the levels one or two steps below the canonical resolution), c ^ (c + 2) = (c' ^ (c' + 1)) << 1 for
// c' = c >> 1: t = trailing ones of c', s = 1 (round 5).  Otherwise (larger steps, straddles, other
// tables) each entry gets a single record with weight sel ? fx : 1-fx.
// a record's two values: fp16 of v * 2^-15, round to nearest even (v in the table's int32 units)
constexpr float REC_DOWN = 1.0f / 32768.0f, REC_UP = 32768.0f;
typedef unsigned short ushort2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t rec_values(float a, float b) {
    const _Float16 ha = (_Float16)(a * REC_DOWN), hb = (_Float16)(b * REC_DOWN);  // (exact scaling)
    return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}
// value k of a record (0: a, 1: b) times 2^-15 (scale it by 2^15 x the unit to use)
__device__ __forceinline__ float rec_value(uint32_t ab, int k) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(ab >> (16 * k)));
}

template <typename EMIT>
__device__ __forceinline__ void level_records_geo(const mfnerf_grid_desc& D, const BinPlan& P, int j,
                                                  const LevelGeo& Lg, float g0, float g1, float fs, EMIT&& emit) {
    const int l = P.level[j];
    const int t = P.table_of[l];
    const int bin0 = P.t_bin0[t];
    const uint32_t fxq = min(32767u, (uint32_t)rintf(Lg.w[0] * 32768.0f)) << 17;
    uint32_t ones = (uint32_t)__builtin_ctz(~Lg.g[0]);  // trailing ones of x
    uint32_t pflags = 0u;                               // s << 16
    bool pair_hash = P.pairable[l] && ones < 15;
    if (D.table_kind[l] == 1 && (D.size[l] & (D.size[l] - 1)) == 0) {
        // a shared MixedFeature table: the x-pair's canonical step (corner_index's canon_coord)
        const uint32_t rc = (uint32_t)D.canon_res, res = D.res[l];
        const float inv = 1.0f / (float)res;
        const uint32_t c0 = canon_coord(Lg.g[0], rc, res, inv), c1 = canon_coord(Lg.g[0] + 1, rc, res, inv);
        const uint32_t cs = c1 - c0 == 2u ? c0 >> 1 : c0;
        ones = (uint32_t)__builtin_ctz(~cs);
        pflags = c1 - c0 == 2u ? 1u << 16 : 0u;
        pair_hash = (c1 - c0 == 1u || c1 - c0 == 2u) && ones < 15;
    }
    // the accumulate decodes e1 = e0 ^ (((2^(t+1) - 1) << s): valid only if that mask lies inside the
    // table (corner_index masks both indices by size - 1; with a table of at most one partition, the
    // same-partition test below would pass for a mask reaching past it -- ADVICE r5)
    pair_hash = pair_hash && ((((2u << ones) - 1u) << (pflags >> 16)) < D.size[l]);
    const float s0 = g0 * fs, s1 = g1 * fs;  // in the table's int32 fixed-point units
    const uint32_t mask = (1u << P.shift) - 1;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t gy = Lg.g[1] + (yz & 1), gz = Lg.g[2] + (yz >> 1);
        const float wy = (yz & 1) ? Lg.w[1] : 1.0f - Lg.w[1];
        const float wz = (yz >> 1) ? Lg.w[2] : 1.0f - Lg.w[2];
        const float wyz = wy * wz;
        const uint32_t i0 = corner_index(D, l, Lg.g[0], gy, gz);
        const uint32_t i1 = corner_index(D, l, Lg.g[0] + 1, gy, gz);
        const int b0 = bin0 + (int)(i0 >> P.shift), b1 = bin0 + (int)(i1 >> P.shift);
        const uint32_t ab = rec_values(wyz * s0, wyz * s1);
        // static record slots 2 yz, 2 yz + 1, both always emitted (bin -1: no record), so the
        // caller's per-slot register arrays see constant indices on every path and stay registers
        const bool pair = pair_hash && b0 == b1;
        emit(2 * yz, b0, make_uint2((i0 & mask) | (pair ? (ones << 11) | pflags : (1u << 15)) | fxq, ab));
        emit(2 * yz + 1, pair ? -1 : b1, make_uint2((i1 & mask) | (1u << 15) | (1u << 16) | fxq, ab));
    }
}

// The PAIR layout's records (BinPlan::pair_ok: every binned level an own power-of-two hash table and
// every x + 1 below 2^shift, so the x-pair never straddles a partition): one record per (y,z) row,
// the hash written out (corner_index's prime hash masked to the table size, no layout branches), the
// partition from the index's high bits, and s0 / s1 already scaled by the table unit x 2^-15 (exact:
// a power of two), so rec_values' own scaling is gone.  The same records as level_records_geo but
// for the fp16 rounding of a value: the compiler folds wyz * s0 and its conversion into one v_fma_mix
// (the exact product rounded once to f16), where level_records_geo rounds the product to f32 first
// (its last, exact scaling folds instead) -- the two differ only where that f32 rounding crosses an
// f16 rounding boundary.  Still deterministic.  EMIT(row, partition in the table, record).
template <typename EMIT>
__device__ __forceinline__ void pair_level_records(const mfnerf_grid_desc& D, const BinPlan& P, int l, float x,
                                                   float y, float z, float s0, float s1, EMIT&& emit) {
    const LevelGeo Lg = level_geo(D.scale[l], x, y, z);
    const uint32_t mask = D.size[l] - 1u, emask = (1u << P.shift) - 1u;
    const uint32_t fxq = min(32767u, (uint32_t)rintf(Lg.w[0] * 32768.0f)) << 17;
    // trailing ones of x (< shift for every x + 1 < 2^shift, which pair_ok guarantees inside the grid;
    // the clamp keeps a point outside it from naming an x-pair beyond its partition), and fx
    const uint32_t ones = min((uint32_t)__builtin_ctz(~Lg.g[0]), (uint32_t)P.shift - 1u);
    const uint32_t flags = (ones << 11) | fxq;
    const uint32_t hy0 = Lg.g[1] * PRIME1, hz0 = Lg.g[2] * PRIME2;
    const float wy1 = Lg.w[1], wy0 = 1.0f - wy1, wz1 = Lg.w[2], wz0 = 1.0f - wz1;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
        const uint32_t hy = (yz & 1) ? hy0 + PRIME1 : hy0, hz = (yz >> 1) ? hz0 + PRIME2 : hz0;
        const uint32_t i0 = (Lg.g[0] ^ hy ^ hz) & mask;
        const float wyz = ((yz & 1) ? wy1 : wy0) * ((yz >> 1) ? wz1 : wz0);
        // both values rounded to f32, then packed to f16 pairs by one v_cvt_pk_f16_f32 (the
        // rounding of level_records_geo; one conversion instead of two fma_mix + the packing)
        const float2v v = {wyz * s0, wyz * s1};
        const uint32_t ab = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, half2v));
        emit(yz, (int)(i0 >> P.shift), make_uint2((i0 & emask) | flags, ab));
    }
}

// Runs of one cell inside a 16-lane DPP row (a 16-sample chunk: consecutive samples of a ray, the
// scatter's lane order).  A dead lane (no gradient or no sample) is a run of its own.  suffix_sums
// leaves each run's sums in its first lane: a segmented suffix sum over the row, 4 DPP steps, one
// fixed order (every lane of the wave must call it).  keep[k]: 1 if the lane adds the values 2^k
// lanes on at step k (its run goes on past them) -- the same for every value, so computed once.
struct RunRow {
    bool same_prev, same_next;
    float keep[4];
    __device__ __forceinline__ void suffix_sums(float* v) const {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = fmaf(dpp_f<DPP_ROW_SHL(1)>(v[k]), keep[0], v[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = fmaf(dpp_f<DPP_ROW_SHL(2)>(v[k]), keep[1], v[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = fmaf(dpp_f<DPP_ROW_SHL(4)>(v[k]), keep[2], v[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = fmaf(dpp_f<DPP_ROW_SHL(8)>(v[k]), keep[3], v[k]);
    }
};
__device__ __forceinline__ RunRow run_row(const LevelGeo& Lg, bool live) {
    // every DPP read is unconditional and combined with non-short-circuit operators: a DPP inside a
    // `&&` or `?:` runs under a narrowed EXEC, and a lane reading a disabled neighbour reads 0
    RunRow r;
    const int lr = (int)(threadIdx.x & 15);
    const int k0 = live ? (int)Lg.g[0] : -1, k1 = live ? (int)Lg.g[1] : -1, k2 = live ? (int)Lg.g[2] : -1;
    const int n0 = dpp_i<DPP_ROW_SHL(1)>(k0), n1 = dpp_i<DPP_ROW_SHL(1)>(k1), n2 = dpp_i<DPP_ROW_SHL(1)>(k2);
    const int p0 = dpp_i<DPP_ROW_SHR(1)>(k0), p1 = dpp_i<DPP_ROW_SHR(1)>(k1), p2 = dpp_i<DPP_ROW_SHR(1)>(k2);
    r.same_next = (lr < 15) & (n0 == k0) & (n1 == k1) & (n2 == k2);
    r.same_prev = (lr > 0) & (p0 == k0) & (p1 == k1) & (p2 == k2);
    int stop = r.same_next ? 0 : 1;  // this lane's run ends within the lanes summed so far
    int t;
    r.keep[0] = stop ? 0.0f : 1.0f;
    t = dpp_i<DPP_ROW_SHL(1)>(stop);
    stop |= t;
    r.keep[1] = stop ? 0.0f : 1.0f;
    t = dpp_i<DPP_ROW_SHL(2)>(stop);
    stop |= t;
    r.keep[2] = stop ? 0.0f : 1.0f;
    t = dpp_i<DPP_ROW_SHL(4)>(stop);
    stop |= t;
    r.keep[3] = stop ? 0.0f : 1.0f;
    return r;
}

template <typename EMIT>
__device__ __forceinline__ void level_records(const mfnerf_grid_desc& D, const BinPlan& P, int j, float x, float y,
                                              float z, float g0, float g1, float fs, EMIT&& emit) {
    level_records_geo(D, P, j, level_geo(D.scale[P.level[j]], x, y, z), g0, g1, fs, emit);
}

// Round 6: the records of a level that never forms a pair record (BinPlan::merge: a MixedFeature
// shared table whose canonical x-step is >= 3, an own table without the power-of-two hash), with the
// samples of one run merged.  A 16-lane DPP row holds a 16-sample chunk -- consecutive samples of a
// ray -- and at the coarse shared levels ~2-3 consecutive samples fall in one cell: same 8 corner
// entries, other weights.  Per (y,z) row each lane computes its 4 weighted values ({x, x+1} x 2
// features, the x weight applied: (1 - fx) wyz g and fx wyz g in table units), a segmented suffix
// sum over the row (RunRow, 4 DPP steps, a fixed order) leaves each run's sums in its first lane,
// and only that lane emits the run's 8 single records, weight 1 (fx = 0, sel = 0).  Every lane of
// the wave must call it (DPP reads its row neighbours); `live` false: no gradient / no sample.
// Measured (r6c, config 3's field): mf128 step 1.244 -> 1.204 ms, grid_bw 0.674 -> 0.637 ms.  The
// same merge for the Lego layout's coarse PAIR levels (runs of >= 2 as two single-record halves
// from the run's first two lanes) ran 0.5125 vs 0.4953 ms/step: with two samples per lane it
// spilled (62 VGPRs) and its records saved less -- a run of two is two records either way.
// The same entries and contributions as level_records_geo's singles; each value is now the run's
// fp32 sum rounded once to fp16 (the 2^-11 record bound holds for the sum), and the x weight exact
// instead of a 15-bit fx.
template <typename EMIT>
__device__ __forceinline__ void merged_level_records(const mfnerf_grid_desc& D, const BinPlan& P, int j, float x,
                                                     float y, float z, float g0, float g1, float fs, bool live,
                                                     EMIT&& emit) {
    const int l = P.level[j];
    const LevelGeo Lg = level_geo(D.scale[l], live ? x : 0.0f, live ? y : 0.0f, live ? z : 0.0f);
    const RunRow rr = run_row(Lg, live);
    const float s0 = live ? g0 * fs : 0.0f, s1 = live ? g1 * fs : 0.0f;  // table int32 units
    const float wx1 = Lg.w[0], wx0 = 1.0f - wx1, wy1 = Lg.w[1], wy0 = 1.0f - wy1, wz1 = Lg.w[2], wz0 = 1.0f - wz1;
    const bool head = live && !rr.same_prev;  // a run's first lane emits the run's records
    const int bin0 = P.t_bin0[P.table_of[l]];
    const uint32_t emask = (1u << P.shift) - 1u;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {  // row by row: 4 values in flight
        const float wyz = ((yz & 1) ? wy1 : wy0) * ((yz >> 1) ? wz1 : wz0);
        const float a = wyz * s0, b = wyz * s1;
        float v[4] = {wx0 * a, wx0 * b, wx1 * a, wx1 * b};
        rr.suffix_sums(v);
        if (head) {
            const uint32_t gy = Lg.g[1] + (yz & 1), gz = Lg.g[2] + (yz >> 1);
            const uint32_t i0 = corner_index(D, l, Lg.g[0], gy, gz);
            const uint32_t i1 = corner_index(D, l, Lg.g[0] + 1, gy, gz);
            emit(2 * yz, bin0 + (int)(i0 >> P.shift), make_uint2((i0 & emask) | (1u << 15), rec_values(v[0], v[1])));
            emit(2 * yz + 1, bin0 + (int)(i1 >> P.shift), make_uint2((i1 & emask) | (1u << 15), rec_values(v[2], v[3])));
        }
    }
}

// A sample staged in registers for all its binned levels: normalised position and dL/dy of the
// binned levels (contiguous), loaded once before the level loop -- a load inside the loop would
// wait behind the previous level's record stores (one in-order vmcnt), serialising the levels.
constexpr int MAX_BINNED = 16;
template <int MAXB>
struct StagedSample {
    float x, y, z;
    float g[2 * MAXB];
};

template <int MAXB>
__device__ __forceinline__ void stage_sample(const mfnerf_grid_desc& D, const BinPlan& P, const float* __restrict__ X,
                                             float x_min, float x_range, const float* __restrict__ dy, int64_t i,
                                             StagedSample<MAXB>& S) {
    S.x = (X[3 * i] - x_min) / x_range;
    S.y = (X[3 * i + 1] - x_min) / x_range;
    S.z = (X[3 * i + 2] - x_min) / x_range;
    const float2* src = reinterpret_cast<const float2*>(dy + i * (2 * D.n_levels) + 2 * P.level[0]);
#pragma unroll
    for (int j = 0; j < MAXB; ++j) {
        const float2 v = j < P.n_binned ? src[j] : make_float2(0.f, 0.f);
        S.g[2 * j] = v.x;
        S.g[2 * j + 1] = v.y;
    }
}

// one sample's dL/dy pair at binned level j, selected once for both record passes (count, place)
struct SampleLevel {
    float g0, g1;
    bool live;
};

template <int MAXB>
__device__ __forceinline__ SampleLevel sample_level(const mfnerf_grid_desc& D, const BinPlan& P,
                                                    const StagedSample<MAXB>& S, int j) {
    float g0 = 0.f, g1 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXB; ++k)  // register-indexed select (j is uniform: scalar compares)
        if (k == j) { g0 = S.g[2 * k]; g1 = S.g[2 * k + 1]; }
    SampleLevel r;
    r.g0 = g0;
    r.g1 = g1;
    r.live = !(r.g0 == 0.0f && r.g1 == 0.0f);  // terminated samples: nothing to add
    return r;
}

template <int MAXB, typename EMIT>
__device__ __forceinline__ void staged_records(const mfnerf_grid_desc& D, const BinPlan& P,
                                               const StagedSample<MAXB>& S, const SampleLevel& Q, const float* fs_s,
                                               int j, EMIT&& emit) {
    if (!Q.live) return;
    level_records(D, P, j, S.x, S.y, S.z, Q.g0, Q.g1, fs_s[P.level[j]], emit);
}

__device__ __forceinline__ void load_fixed_scales(const mfnerf_grid_desc& D, const float* __restrict__ level_l1,
                                                  float* fs_s) {
    if ((int)threadIdx.x < D.n_levels) fs_s[threadIdx.x] = table_fixed_scale(D, level_l1, threadIdx.x);
}

// exclusive scan over the block (one value per thread, blockDim <= 1024): wave scans by lane
// shuffles, then the wave totals; out[threadIdx.x] = this thread's offset.  Returns the total.
__device__ __forceinline__ int wave_block_scan(int v, int* out) {
    __shared__ int wsum[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    const int nw = (int)(blockDim.x + 63) >> 6;
    int before = 0, total = 0;
    for (int k = 0; k < nw; ++k) {
        const int t = wsum[k];
        before += k < w ? t : 0;
        total += t;
    }
    out[threadIdx.x] = before + x - v;
    __syncthreads();
    return total;
}

// Records live in fixed slots: unit u's records of bin b at rec[(b * UNITS + u) * slot + k],
// k < scnt[b * UNITS + u] -- no counting pass, no scan.  slot = 3 x the mean records per slot at this
// step's live count + 96, so the buffer (sized for the largest live count) holds them; the records
// of a slot that still overflows (a sample distribution far from uniform) go into the table by
// atomics (overflow_add), and `ovf` tells the accumulate to add them to its image.
constexpr int UNITS = 256;       // scatter workgroups, each owning a contiguous sample range
constexpr int SC_THREADS = 1024;
constexpr int MAX_TBINS = 1024;  // bins of one table
constexpr int SC_STAGE = SC_THREADS * 8;  // staged records per tile (8 per thread)

// records per (partition, unit) slot at live count nn; non-decreasing in nn, so the workspace sized
// with slot_size(n_max) (binned_workspace_layout) holds every slot of any nn <= n_max
__host__ __device__ __forceinline__ int64_t slot_size(int64_t nn, const BinPlan& P) {
    const int64_t recs = nn * P.n_binned * (P.pair_ok ? 4 : 8);
    const int64_t s = 3 * ((recs + (int64_t)P.n_bins * UNITS - 1) / ((int64_t)P.n_bins * UNITS)) + 96;
    return (s + 15) / 16 * 16;  // 16 records = 128 B: every slot starts on a 128-B line
}

// A record past its slot's capacity (a sample distribution far from uniform over the partitions):
// added by 64-bit packed integer atomics (f1 * 2^32 + f0 per entry, each contribution rounded once
// to the table's int32 unit) into the workspace's overflow words (one per partitioned entry, zero
// between steps: the accumulate zeroes what it reads), and the accumulate adds the partition's words
// to its image (bin_scatter raises ovf).  Exact integer sums: the order of the two paths does not
// matter.  The words are not the gradient's own, so the gradient need not be zero before a scatter.
__device__ __forceinline__ void overflow_add(const BinPlan& P, int* __restrict__ ovw, int bin, uint2 r) {
    const int t = bin_table(P, bin);
    const int64_t base = (int64_t)(P.t_offset[t] - P.t_offset[0]) + ((int64_t)(bin - P.t_bin0[t]) << P.shift);
    const uint32_t w = r.x;
    const float a = rec_value(r.y, 0) * REC_UP, b = rec_value(r.y, 1) * REC_UP;
    const float fx = (float)(w >> 17) * (1.0f / 32768.0f);
    const int e0 = w & ((1 << P.shift) - 1);
    auto add = [&](int e, float wt) {
        const int q0 = (int)rintf(wt * a), q1 = (int)rintf(wt * b);
        const long long pq = (long long)((uint64_t)(uint32_t)q1 << 32) + (long long)q0;
        if (pq != 0)
            __hip_atomic_fetch_add(reinterpret_cast<long long*>(ovw) + base + e, pq, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    };
    if (w & (1u << 15)) {
        add(e0, (w & (1u << 16)) ? fx : 1.0f - fx);
    } else {
        add(e0, 1.0f - fx);
        add(e0 ^ (((2 << ((w >> 11) & 15)) - 1) << ((w >> 16) & 1)), fx);
    }
}

// pass 1: unit u (one 1024-thread workgroup) walks its samples, staged in registers, level by level
// in tiles of up to 2048 samples.  Per level, ONE pass computes the tile's records into registers
// (8 per thread: 2 samples x 4 pair rows, or 1 sample x 8 single records), each taking its rank in
// its bin from an LDS counter; one wave scans the bin counts; the records are placed sorted by bin
// into an LDS stage; the stage is stored as one contiguous run per bin into the unit's slot of the
// bin (~30 records per run at the Lego config: whole-line stores) while the NEXT level counts.  Three
// barriers per level (count | scan | place), the store overlapping the next count.
struct BinRec {
    uint2 r;
    uint32_t meta;  // bin in the table (bits 0-15) | rank in the bin's run (bits 16-31); ~0u: none
};

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>)
template <typename F, int... J>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

#ifdef MFN_SCATTER_PROBE
// a timing probe build (tools/build_variant.sh with EXTRA=-DMFN_SCATTER_PROBE): bin_scatter's phase
// cycles (s_memtime, which also waits for the wave's LDS operations -- perturbed, for proportions only)
__device__ unsigned long long g_scatter_probe[16 + MAX_BINNED];  // [16 + j]: wave 8's count of level j
// bin_accum's phases (wave 0, lane 0): [0] setup (counts, state loads issued, image zeroed, prefix),
// [1] record copies issued, [2] their wait, [3] the adds, [4] the last barrier, [5] the Adam update;
// [7] partition workgroups
__device__ unsigned long long g_accum_probe[8];
extern "C" int mfnerf_accum_probe_read(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_accum_probe), sizeof(g_accum_probe)) == hipSuccess ? 0 : -1;
}
extern "C" int mfnerf_scatter_probe_read(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_scatter_probe), sizeof(g_scatter_probe)) == hipSuccess ? 0 : -1;
}
#endif

template <int MAXB, bool PAIR>
__global__ __launch_bounds__(SC_THREADS) void bin_scatter_kernel(const float* __restrict__ X, int64_t n,
                                                                 const int32_t* __restrict__ n_dev, float x_min,
                                                                 float x_range, const mfnerf_grid_desc D,
                                                                 const BinPlan P, const float* __restrict__ dy,
                                                                 const float* __restrict__ level_l1,
                                                                 uint2* __restrict__ rec, int32_t* __restrict__ scnt,
                                                                 uint32_t* __restrict__ smax,
                                                                 int32_t* __restrict__ ovf, int64_t n_slots,
                                                                 int* __restrict__ ovw) {
    constexpr int SPT = PAIR ? 2 : 1;  // samples per thread per tile
    constexpr int TH = SC_THREADS, STG = SC_STAGE, LCUR = LDS_CURSOR;
    const int u = blockIdx.x;
    __shared__ int cursor[LCUR];  // the unit's running count per bin
    // per-level bin counts, double-buffered by level parity (a level's counts are read by the scan
    // and cleared during its placement, while the next level counts into the other buffer)
    __shared__ int hist2[2][MAX_TBINS], toff[MAX_TBINS];
    // per bin of the staged level: {index of the stage's first record of the bin in rec[] minus its
    // stage offset, the stage index its slot ends at} (one 8-B LDS read per stored record)
    __shared__ int2 gdst[2][MAX_TBINS];
    __shared__ uint2 stage[STG];
    __shared__ uint16_t sbin[STG];
    __shared__ float fs_s[MFN_MAX_LEVELS];
    __shared__ int s_total[2];
    uint32_t rmax2 = 0u;  // largest |a| (low half), |b| (high half) of this thread's records, fp16 bits
    load_fixed_scales(D, level_l1, fs_s);
    for (int b = threadIdx.x; b < min(P.n_bins, LCUR); b += blockDim.x) cursor[b] = 0;
    // the running counts of the bins past LCUR live in scnt: zeroed by the scanning wave, the only
    // one that touches them (program order within the wave)
    if (threadIdx.x < 64)
        for (int b = LCUR + (int)threadIdx.x; b < P.n_bins; b += 64) scnt[(int64_t)b * UNITS + u] = 0;
    for (int b = threadIdx.x; b < 2 * MAX_TBINS; b += blockDim.x) hist2[b >> 10][b & (MAX_TBINS - 1)] = 0;
    if (threadIdx.x < 2) s_total[threadIdx.x] = 0;
    __syncthreads();
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    // slots sized for at most the workspace's count: beyond it a slot may overflow (-> atomics)
    const int64_t slot = slot_size(min(nn, n_slots), P);
    // unit u owns the 16-sample chunks u, u + UNITS, u + 2 UNITS, ...: a ray's samples (which repeat
    // the coarse levels' rows) spread over many units, so every slot fills close to the mean
    const int64_t n_chunks = (nn + 15) / 16;
    const int64_t m = n_chunks > u ? ((n_chunks - 1 - u) / UNITS + 1) * 16 : 0;  // this unit's sample slots
    // Round 5: two barriers per level instead of three.  Phase A places level j's ranked records into
    // the stage and then counts level j + 1 (the next tile's first level after the last); phase B
    // stores level j's stage into the slots and scans level j + 1's bin counts.  Each LDS buffer is
    // written and read in different phases: the stage (A: place, B: store), toff (B: scan, A: place),
    // hist2 / gdst / s_total by level parity (count and scan of j + 1 beside place and store of j).
    int par = 0;  // parity of the level whose records R holds (its hist2 / gdst / s_total buffers)
    BinRec R[8];
    StagedSample<MAXB> S[SPT];
    bool live[SPT];
    auto stage_tile = [&](int64_t base) {
#pragma unroll
        for (int q = 0; q < SPT; ++q) {
            const int64_t k = base + (int64_t)q * TH + threadIdx.x;
            const int64_t i = ((k >> 4) * UNITS + u) * 16 + (k & 15);  // chunk k/16 of the unit
            live[q] = k < m && i < nn;
            if (live[q]) stage_sample(D, P, X, x_min, x_range, dy, i, S[q]);
        }
    };
    // count: level j's records computed once each, ranked in their bin by the LDS counter of parity cp;
    // G(q) = sample q's dL/dy pair at level j
    auto count = [&](int j, int cp, auto G) __attribute__((always_inline)) {
        const int b0 = P.t_bin0[P.table_of[P.level[j]]];
#pragma unroll
        for (int k = 0; k < 8; ++k) R[k].meta = ~0u;
#pragma unroll
        for (int q = 0; q < SPT; ++q) {
            const SampleLevel Q = G(q);
            // the record's |a|, |b| maxima as two packed u16 (fp16 bits order like the values)
            auto rank = [&](int k, int lb, uint2 r) {
                R[k].r = r;
                R[k].meta = (uint32_t)lb | ((uint32_t)atomicAdd(&hist2[cp][lb], 1) << 16);
                rmax2 = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(
                    __builtin_bit_cast(ushort2v, rmax2), __builtin_bit_cast(ushort2v, r.y & 0x7fff7fffu)));
            };
            if constexpr (!PAIR) {
                if (P.merge[P.level[j]]) {  // (uniform) every lane takes part: DPP over the row
                    merged_level_records(D, P, j, S[q].x, S[q].y, S[q].z, Q.g0, Q.g1, fs_s[P.level[j]],
                                         live[q] && Q.live, [&](int sl, int bin, uint2 r) { rank(sl, bin - b0, r); });
                    continue;
                }
            }
            if (!(live[q] && Q.live)) continue;
            if constexpr (PAIR) {
                const int l = P.level[j];
                const float fs = fs_s[l] * REC_DOWN;
                pair_level_records(D, P, l, S[q].x, S[q].y, S[q].z, Q.g0 * fs, Q.g1 * fs,
                                   [&](int yz, int lb, uint2 r) { rank(4 * q + yz, lb, r); });
            } else {
                level_records(D, P, j, S[q].x, S[q].y, S[q].z, Q.g0, Q.g1, fs_s[P.level[j]],
                              [&](int sl, int bin, uint2 r) {
                                  if (bin >= 0) rank(sl, bin - b0, r);
                              });
            }
        }
    };
    // scan: level j's bins -> sorted tile offsets (toff) and slot places (gdst[cp]); a run's k-th
    // record goes to slot position gdst + k.  Chunk q of 64 bins (consecutive lanes on consecutive LDS
    // words: no bank conflicts) is scanned by wave q % 16 with an integer DPP wave scan; its carry (the
    // bins of the chunks before it) is each lane's column sum over those chunks
    auto scan = [&](int j, int cp) {
        static_assert(MAX_TBINS == 1024, "hist2 indexing");
        const int t = P.table_of[P.level[j]];
        const int b0 = P.t_bin0[t], tb = P.t_bin0[t + 1] - b0;
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        const int per = (tb + 63) >> 6;
        const int* hs = hist2[cp];
        constexpr int nw = SC_THREADS / 64;
        for (int q = wv; q < per; q += nw) {
            int col = 0;  // chunks before q are whole (q < per - 1 ... < tb)
            for (int q2 = 0; q2 < q; ++q2) col += hs[q2 * 64 + lane];
            col += dppz_i<0x111, 0xF>(col); col += dppz_i<0x112, 0xF>(col);
            col += dppz_i<0x114, 0xF>(col); col += dppz_i<0x118, 0xF>(col);
            col += dppz_i<0x142, 0xA>(col); col += dppz_i<0x143, 0xC>(col);
            const int carry = __builtin_amdgcn_readlane(col, 63);
            const int lb = q * 64 + lane;
            const int c = lb < tb ? hs[lb] : 0;
            int x = c;
            x += dppz_i<0x111, 0xF>(x); x += dppz_i<0x112, 0xF>(x);
            x += dppz_i<0x114, 0xF>(x); x += dppz_i<0x118, 0xF>(x);
            x += dppz_i<0x142, 0xA>(x); x += dppz_i<0x143, 0xC>(x);
            const int run = carry + x - c;
            if (lb < tb) {
                toff[lb] = run;
                const int gb = b0 + lb, cl = gb;
                int32_t* gc = scnt + (int64_t)gb * UNITS + u;  // (bins past LCUR)
                const int cu = cl < LCUR ? cursor[cl] : *gc;
                // record k of the sorted stage is position cu - run + k of the slot
                gdst[cp][lb] = make_int2((int)((uint32_t)(b0 + lb) * UNITS + u) * (int)slot + cu - run,
                                         run + (int)slot - cu);
                if (cl < LCUR) cursor[cl] = cu + c;
                else *gc = cu + c;
            }
            if (q == per - 1 && lane == 63) s_total[cp] = carry + x;
        }
    };
    // place: level j's records (R, parity par) sorted by bin into the stage; its counts cleared for the
    // level after next, which counts into the same buffer
    auto place = [&](int j) {
        const int t = P.table_of[P.level[j]];
        const int tb = P.t_bin0[t + 1] - P.t_bin0[t];
        for (int b = threadIdx.x; b < tb; b += TH) hist2[par][b] = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (R[k].meta == ~0u) continue;
            const int lb = R[k].meta & 0xffff;
            const int p = toff[lb] + (int)(R[k].meta >> 16);
            stage[p] = R[k].r;
            sbin[p] = (uint16_t)lb;
        }
    };
    // store: level j's sorted stage as one contiguous run per bin into the unit's slot of the bin
    auto store = [&](int j) {
        const int b0 = P.t_bin0[P.table_of[P.level[j]]];
        const int total = s_total[par];
        const int2* gd = gdst[par];
        // SU records per thread in flight: their stage / bin reads, then their slot places, then the
        // stores -- two LDS round trips per SU records (round 6: one record per iteration waited three
        // times; tools/scatter_probe.py puts ~1/3 of the Lego scatter's time in this phase).  Measured
        // (r6ab / r6ac, profiles/r06_v9_scatter_phase_probe.txt): the Lego scatter alone 0.2425 ->
        // 0.238 ms at SU = 2, the step within noise (0.4881 vs 0.4892); SU = 4 made the Lego kernel
        // 124 VGPRs -- no room left beside it for the side stream's march -- and the step 4 us slower;
        // reading place()'s eight offsets before its writes gained nothing
        constexpr int SU = PAIR ? (MAXB <= 12 ? 2 : 1) : 4;
        for (int k0 = threadIdx.x; k0 < total; k0 += SU * TH) {
            int lb[SU];
            uint2 r[SU];
            int2 g[SU];
#pragma unroll
            for (int q = 0; q < SU; ++q) {
                const int k = k0 + q * TH, kc = k < total ? k : 0;
                lb[q] = sbin[kc];
                r[q] = stage[kc];
            }
#pragma unroll
            for (int q = 0; q < SU; ++q) g[q] = gd[lb[q]];
#pragma unroll
            for (int q = 0; q < SU; ++q) {
                const int k = k0 + q * TH;
                if (k >= total) break;
                if (k < g[q].y) {  // inside the unit's slot of the bin
                    // a plain store (round 5, r5c: the nontemporal store this was made the scatter 92 instead
                    // of 82.5 us and the step 3 us slower; the accumulate reads them the same either way)
                    rec[(uint32_t)(g[q].x + k)] = r[q];
                } else {
                    overflow_add(P, ovw, b0 + lb[q], r[q]);  // a full slot: into the overflow words
                }
            }
        }
    };
    // one level step: phase A (place j, count the next level), phase B (store j, scan the next level)
#ifdef MFN_SCATTER_PROBE
    uint64_t pt[6] = {0, 0, 0, 0, 0, 0};
    auto clk = [&]() { return __builtin_amdgcn_s_memtime(); };
#define MFN_TICK(k)                 \
    {                               \
        const uint64_t t_ = clk();  \
        pt[k] += t_ - tl;           \
        tl = t_;                    \
    }
#else
#define MFN_TICK(k)
#endif
    auto step = [&](int j, int64_t base, auto count_next) __attribute__((always_inline)) {
#ifdef MFN_SCATTER_PROBE
        uint64_t tl = clk();
#endif
        place(j);
        MFN_TICK(0)
        int jn = j + 1;
        bool next = true;
        if (jn == P.n_binned) {  // the next tile's first level
            jn = 0;
            next = base + (int64_t)SPT * TH < m;
            // (the single-record layout stages it below, a step earlier)
            if (next && (PAIR || P.n_binned < 2)) stage_tile(base + (int64_t)SPT * TH);
        }
        if (next) count_next(jn, par ^ 1);
#ifdef MFN_SCATTER_PROBE
        if (threadIdx.x == 512) atomicAdd(&g_scatter_probe[16 + jn], (unsigned long long)(clk() - tl));
#endif
        MFN_TICK(1)
        __syncthreads();
        MFN_TICK(2)
        // single-record layout (MixedFeature): the next tile's samples, loaded as soon as this tile's
        // last level is counted (phase A above) and ahead of this phase's record stores -- on gfx9 a
        // load's wait counts the stores issued before it too, and staged right before its first
        // count the load waited for the previous phase's stores and then its own round trip
        // (profiles/r06_v9_scatter_phase_probe.txt: that count 3x the others; config 3's step 1.151
        // -> 1.138 ms, r6v).  The PAIR kernels keep the late staging: the Lego layout's units hold
        // one tile, and the early form's code alone made its scatter 7 us slower (r6v)
        if constexpr (!PAIR)
            if (j == P.n_binned - 2 && base + (int64_t)SPT * TH < m) stage_tile(base + (int64_t)SPT * TH);
        store(j);
        MFN_TICK(3)
        if (next) scan(jn, par ^ 1);
        MFN_TICK(4)
        __syncthreads();
        MFN_TICK(5)
        par ^= 1;
    };
#undef MFN_TICK
    auto level_g = [&](int j) {  // runtime-level dL/dy pair (sample_level's register select)
        return [&, j](int q) { return sample_level(D, P, S[q], j); };
    };
    if (m > 0) {  // the first tile's first level: count, scan
        stage_tile(0);
        count(0, 0, level_g(0));
        __syncthreads();
        scan(0, 0);
        __syncthreads();
    }
    for (int64_t base = 0; base < m; base += (int64_t)SPT * TH) {
        if constexpr (PAIR && MAXB <= 10) {
            // the level loop written out: j a constant in every copy, so the staged pair is a plain
            // register (sample_level's select costs 2 MAXB v_cndmask per sample and level).  The
            // single-record layout (MixedFeature) written out the same way: 331 vs 325 us, code
            // 91 vs 24 KB (r05_v25)
            auto count_c = [&](int jn, int cp) __attribute__((always_inline)) {
                auto each = [&](auto jc) __attribute__((always_inline)) {
                    constexpr int jj = decltype(jc)::value;
                    if (jj == jn)
                        count(jj, cp, [&](int q) {
                            SampleLevel r;
                            r.g0 = S[q].g[2 * jj];
                            r.g1 = S[q].g[2 * jj + 1];
                            r.live = !(r.g0 == 0.0f && r.g1 == 0.0f);
                            return r;
                        });
                };
                static_for<MAXB>(each);
            };
            for (int j = 0; j < P.n_binned; ++j) step(j, base, count_c);
        } else {
            for (int j = 0; j < P.n_binned; ++j)
                step(j, base, [&](int jn, int cp) { count(jn, cp, level_g(jn)); });
        }
    }
#ifdef MFN_SCATTER_PROBE
    // phase cycles of waves 0 and 8 (lane 0), summed over units and launches; [15]: unit launches
    if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) % 8 == 0) {
        const int o = (threadIdx.x >> 6) == 0 ? 0 : 6;
        for (int k = 0; k < 6; ++k) atomicAdd(&g_scatter_probe[o + k], (unsigned long long)pt[k]);
        if (threadIdx.x == 0) atomicAdd(&g_scatter_probe[15], 1ull);
    }
#endif
    // the unit's largest contribution (one word per unit: the accumulate's per-partition bound is
    // sum over units of count x this max)
    {
        __shared__ uint32_t wmax[TH / 64];
        uint32_t rmax = max(rmax2 & 0xffffu, rmax2 >> 16);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) rmax = max(rmax, (uint32_t)__shfl_xor((int)rmax, off, 64));
        if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = rmax;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t mx = 0u;
            for (int k = 0; k < TH / 64; ++k) mx = max(mx, wmax[k]);
            smax[u] = __float_as_uint(rec_value(mx, 0) * REC_UP);  // as a float in table units
        }
    }
    // ovf[0]: this step's overflowed records (the accumulate adds the gradient words when non-zero;
    // zeroed by the next step's first scatter launch); ovf[1]: their running total (never reset by
    // the kernels: mfnerf_grid_encode_bw_binned_flag_offset + 4 bytes, read by the training tools)
    int over = 0;
    for (int b = threadIdx.x; b < min(P.n_bins, LCUR); b += blockDim.x) {
        const int c = cursor[b];
        over += c > slot ? (int)(c - slot) : 0;
        scnt[(int64_t)b * UNITS + u] = c;
    }
    if (threadIdx.x < 64)  // the counts past LCUR: already in scnt, read back by the wave that wrote them
        for (int b = LCUR + (int)threadIdx.x; b < P.n_bins; b += 64) {
            const int c = scnt[(int64_t)b * UNITS + u];
            over += c > slot ? (int)(c - slot) : 0;
        }
    if (over) {
        atomicAdd(ovf, over);
        atomicAdd(ovf + 1, over);
    }
}

// pass 2: one workgroup per partition sums the partition's records (every unit's slot) into an LDS
// image of its entries and stores it (or feeds it to the fused Adam update).
//
// The image holds one 64-bit word per entry: both features' int32 sums packed as f1 * 2^32 + f0
// (exact in two's complement; decoded f0 = lo, f1 = hi + (f0 < 0)), 2 LDS atomics per pair record.
// The sums run at the PARTITION's own finer unit 2^-k of the table's: k is the largest with
// (sum over units of the unit's record count in the partition x the unit's largest |a|, |b|) * 2^k
// <= 2^30 -- a bound on every entry's sum, from bin_scatter's counts and maxima -- so the int32
// fields cannot overflow, and the stored table-unit value is rounded once per entry.
// The partition's LDS image: both features' int32 sums of an entry as one packed 64-bit word
// (f1 * 2^32 + f0, one ds_add_u64 per entry; decoded f0 = lo, f1 = hi + (f0 < 0)).  Round 6 measured
// the two-plane form (one ds_add_u32 per feature, the review's suggestion): bank conflicts 49 -> 54 %
// of the LDS-active cycles (a 32-bit add's 32-lane group on 32 banks conflicts as randomly as a
// 64-bit add's 16-lane group on 16 bank pairs, and there are twice as many adds), LDS cycles per
// instruction 6.4 -> 5.4, the step unchanged (0.5017 / 0.5007 vs 0.5003 / 0.4995 ms,
// profiles/r06_v1_pmc_sq_grid_bw*.txt).
struct AccImage {
    unsigned long long w[MAX_BIN_ENTRIES];
    __device__ __forceinline__ void add(int e, int q0, int q1) {
        atomicAdd(&w[e], ((unsigned long long)(uint32_t)q1 << 32) + (unsigned long long)(long long)q0);
    }
    __device__ __forceinline__ int2 get(int i) const {
        const unsigned long long v = w[i];
        const int lo = (int)(uint32_t)v;
        return make_int2(lo, (int)(uint32_t)(v >> 32) + (lo < 0));
    }
    __device__ __forceinline__ void set(int i, int2 v) {
        w[i] = ((unsigned long long)(uint32_t)v.y << 32) + (unsigned long long)(long long)v.x;
    }
};
__device__ __forceinline__ void accum_record(AccImage& img, int mask, uint2 r, float k2) {
    const uint32_t w = r.x;
    const float a = rec_value(r.y, 0) * k2, b = rec_value(r.y, 1) * k2;  // exact: k2 a power of two
    if (a == 0.0f && b == 0.0f) return;
    const float fx = (float)(w >> 17) * (1.0f / 32768.0f);
    const int e0 = w & mask;
    if (w & (1u << 15)) {  // single entry, weight sel ? fx : 1 - fx
        const float wt = (w & (1u << 16)) ? fx : 1.0f - fx;
        img.add(e0, (int)rintf(wt * a), (int)rintf(wt * b));
    } else {
        const int e1 = e0 ^ (((2 << ((w >> 11) & 15)) - 1) << ((w >> 16) & 1));
        const float w0 = 1.0f - fx;
        img.add(e0, (int)rintf(w0 * a), (int)rintf(w0 * b));
        img.add(e1, (int)rintf(fx * a), (int)rintf(fx * b));
    }
}

constexpr int ACC_THREADS = 512;
static_assert(MAX_BIN_ENTRIES % ACC_THREADS == 0, "the fused Adam's per-thread entries");

struct AdamRest {
    float* g;            // the flat gradient (MLP floats, then the table's int32 sums)
    int* priv;           // the dense levels' private copies
    int64_t dense_vals, total_vals, end4;
    int n_blocks;        // 0: none
    int first;           // 1: the grid's first n_blocks workgroups (dispatched early), 0: its last
    int32_t* gate;       // opened as the dense-level launch starts (NULL: none)
};

// Round 5: the partition's records are routed through an LDS stage by LDS-DMA
// (global_load_lds_dword), so that a workgroup has ALL its record loads in flight at once.  The
// round-4 form loaded 8 slots' first 32 records per half-wave into registers, waited, added, then
// loaded the slots' records 32-63, then the next 8 slots: ~5 dependent memory round trips per
// workgroup at 0.11 VMEM reads in flight per wave (PMC r04_final: waiting 50 % of the wave cycles).
// Now: (1) the 256 slot counts (and the fused Adam's optimizer state of this thread's entries) are
// loaded; (2) an exclusive prefix of the counts gives every slot's place in a compacted stage; (3)
// wave w copies slots w, w + 8, ... into the stage, 32 records (64 lanes x 4 B) per DMA instruction,
// with no register destination -- one round trip for the whole partition; (4) the adds read the
// stage in a strided order (record 37 t mod 512 of each 512-record block for thread t) so one LDS
// instruction's lanes hold records ~37 apart -- different slots, i.e. different rays -- instead of a
// ray's run of consecutive samples in one cell (same-address atomics).  A partition holding more
// records than the stage is done in chunks of ACC_RB records.  Same records, same integer adds:
// bit-identical sums.  LDS: 16 KB image + 32 KB stage -> three workgroups per CU.
// records per stage chunk.  Round 5: 3840 (30 KB), three workgroups per CU (r05_v21: the unfused accumulate 91.2 -> 88.3 us,
// grid_bw by events 0.239 -> 0.2366 ms; with the Adam fused 142.9 vs 142.5 us; 2560 records: slower)
// Round 6 (r6ai, profiles/r06_v10_accum_probe.txt): 4096 records (32 KB, still three workgroups per
// CU) 0.4885 vs 0.4924 ms/step at Lego, whose partitions hold ~7.7 k records -- two chunks more often
// than at 3840; 4608 (36 KB) left room for only two workgroups per CU: 0.500
constexpr int ACC_RB = 4096;
struct AccumStage {
    AccImage img;
    uint2 recs[ACC_RB];
    int pre[UNITS + 1];  // exclusive prefix of the slots' record counts; pre[UNITS] = the partition's
    float wsum[ACC_THREADS / 64];
    int wtot[ACC_THREADS / 64];
};
union AccumShared {  // ONE __shared__ object (a second one beside an LDS-DMA stage can cost waits)
    AccumStage a;
    TableRegions tr;
};
static_assert(sizeof(AccumShared) <= 163840 / 3, "three accumulate workgroups per CU");

template <bool FUSED>  // FUSED: the Adam update from the finished sums (A.params != NULL)
__global__ __launch_bounds__(ACC_THREADS) void bin_accum_kernel(const BinPlan P, int64_t n,
                                                                const int32_t* __restrict__ n_dev,
                                                                const uint2* __restrict__ rec,
                                                                const int32_t* __restrict__ scnt,
                                                                const uint32_t* __restrict__ smax,
                                                                const int32_t* __restrict__ ovf,
                                                                int* __restrict__ ovw,
                                                                int* __restrict__ grad, int64_t n_slots,
                                                                const mfnerf_grid_desc D,
                                                                const float* __restrict__ level_l1,
                                                                const mfnerf_adam_fused A, const AdamRest X,
                                                                int float_out) {
    __shared__ AccumShared S;
    const int rest_b = X.first ? (int)blockIdx.x : (int)blockIdx.x - P.n_bins;
    if (rest_b >= 0 && rest_b < X.n_blocks) {
        // independent of the slot-overflow flag: these values never go through the partitions
        TableRegions& TR = S.tr;
        TR.build(D, level_l1, X.total_vals);
        const bool skipped = A.amp && A.amp->nonfinite;
        const int stp = *A.step_dev + 1;
        const float lr = A.lr_dev ? *A.lr_dev : A.lr;
        const float bc1 = 1.0f - powf(A.beta1, (float)stp);
        const float bc2 = 1.0f - powf(A.beta2, (float)stp);
        adam_fixed_body(A.params, X.g, A.m, A.v, reinterpret_cast<__half*>(A.p16), A.table_offset, X.priv,
                        X.dense_vals, X.total_vals, TR, lr, A.beta1, A.beta2, A.eps, bc1, bc2, skipped,
                        (int64_t)rest_b * blockDim.x + threadIdx.x, X.end4, (int64_t)X.n_blocks * blockDim.x);
        return;
    }
#ifdef MFN_SCATTER_PROBE
    uint64_t at[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t al = __builtin_amdgcn_s_memtime();
#define MFN_ATICK(k)                                          \
    {                                                         \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
        at[k] += t_ - al;                                     \
        al = t_;                                              \
    }
#else
#define MFN_ATICK(k)
#endif
    const bool add_words = *ovf != 0;  // a slot overflowed: its records are in the gradient words
    AccImage& img = S.a.img;
    const int bin = (int)blockIdx.x - (X.first ? X.n_blocks : 0);
    const int n_ent = 1 << P.shift, mask = n_ent - 1;
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t slot = slot_size(min(nn, n_slots), P);  // = bin_scatter_kernel's
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    constexpr int NW = ACC_THREADS / 64;
    const int32_t* cnt = scnt + (int64_t)bin * UNITS;
    const uint2* base = rec + (int64_t)bin * UNITS * slot;
    const int t = bin_table(P, bin);
    const int64_t e_lo = (int64_t)(bin - P.t_bin0[t]) << P.shift;
    const int n_e = (int)min<int64_t>(n_ent, (int64_t)P.t_size[t] - e_lo);
    // (1) the slot counts, each slot's largest contribution ...
    int c = 0;
    float term = 0.0f;
    bool full = false;  // a slot of this partition overflowed (its extra records: overflow_add)
    if (tid < UNITS) {
        const int c0 = cnt[tid];
        c = min(c0, (int32_t)slot);  // (slot is even: a 16-record multiple)
        full = c0 > slot;
        term = (float)c * __uint_as_float(smax[tid]);
    }
    // ... (fused) this thread's entries' optimizer state is loaded after the last chunk's records
    // (below): in flight through that chunk's adds
    constexpr int IT = MAX_BIN_ENTRIES / ACC_THREADS;
    float2 p[IT], m[IT], v[IT];
    const int64_t base_v = A.table_offset + 2 * ((int64_t)P.t_offset[t] + e_lo);
    float2* __restrict__ pp = reinterpret_cast<float2*>(A.params + base_v);
    float2* __restrict__ mm = reinterpret_cast<float2*>(A.m + base_v);
    float2* __restrict__ vv = reinterpret_cast<float2*>(A.v + base_v);
    for (int i = tid; i < n_ent; i += ACC_THREADS) img.set(i, make_int2(0, 0));
    // (2) exclusive prefix of the counts rounded up to even (waves 0-3 hold them): every slot's run
    // starts on a 16-B record pair in the stage; and the partition's bound (sum over units of count x
    // max, summed in a fixed order) -> its unit 2^-k
    const int c2 = (c + 1) & ~1;
    int x = c2;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) term += __shfl_xor(term, off, 64);
    if (lane == 63) S.a.wtot[wv] = x;
    if (lane == 0) S.a.wsum[wv] = term;
    full = __syncthreads_or(full);
    {
        int before = 0, total = 0;
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int s = S.a.wtot[k];
            before += k < wv ? s : 0;
            total += s;
        }
        if (tid < UNITS) S.a.pre[tid] = before + x - c2;
        if (tid == 0) S.a.pre[UNITS] = total;
    }
    float bound = 0.0f;
#pragma unroll
    for (int k = 0; k < NW; ++k) bound += S.a.wsum[k];
    int kbits = 0;
    // a partition with an overflowed slot sums at the table's own unit: every contribution, in the
    // image or added by overflow_add, is then rounded alike, so the sum does not depend on which of
    // them (an LDS-atomic arrival order) went past the slot -- bit-reproducible
    if (bound > 0.0f && !full) {
        int e;
        frexpf(bound * 1.0001f, &e);  // bound (with margin for its own rounding) < 2^e
        kbits = max(0, min(30, 30 - e));
    }
    const float k2 = ldexpf(1.0f, kbits + 15);  // the records' values are 2^-15 x table units
    __syncthreads();
    const int T = S.a.pre[UNITS];
    // lane j < 32 of wave wv: the run bounds of slot wv + NW j (read by the wave one slot at a time)
    const int my_u = wv + NW * (lane & 31);
    const int my_lo = my_u < UNITS ? S.a.pre[my_u] : T, my_hi = my_u < UNITS ? S.a.pre[my_u + 1] : T;
    static_assert(ACC_RB % 2 == 0, "chunks of whole record pairs");
    MFN_ATICK(0)
    auto copy_chunk = [&](int c0, int c1) __attribute__((always_inline)) {
        // (3) wave wv copies the part of its slots' runs inside [c0, c1): 16 B (a record pair) per lane,
        // 128 records per instruction (4-B lanes measured TA-bound: 48 us of the accumulate's 92).
        // (A gather -- instruction i of the chunk on wave i mod 8, each lane's pair found in its slot
        // by a binary search of the prefix: ~4x fewer instructions, all lanes busy -- measured 96.5
        // vs 94.3 us: the instruction count is not what bounds the copy, profiles/r05_v6_*.)
        // only the wave's slots with records inside the chunk (a ballot of its 32 slot lanes): the
        // chunks cover the slots in order, so most of a wave's slots lie in other chunks.  (Round 6
        // again measured the gather -- a pair -> slot byte map per chunk, every lane busy: Lego
        // within noise, config 3's field 1.143 vs 1.113 ms, its 8 chunks per partition each paying
        // the map; profiles/r06_v10_accum_probe.txt)
        uint64_t todo = __ballot((lane < 32) & (my_lo < c1) & (my_hi > c0) & (my_lo < my_hi));
        while (todo) {
            const int j = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int lo = max(__builtin_amdgcn_readlane(my_lo, j), c0);
            const int hi = min(__builtin_amdgcn_readlane(my_hi, j), c1);
            const int r0 = __builtin_amdgcn_readlane(my_lo, j);  // the slot's first record's place
            const uint4* src = reinterpret_cast<const uint4*>(base + (uint32_t)(NW * j + wv) * (uint32_t)slot);
            for (int q = lo; q < hi; q += 128) {
                const int k = q + 2 * lane;  // records k, k + 1 of the compacted partition (k even)
                if (k < hi)
                    __builtin_amdgcn_global_load_lds(src + ((k - r0) >> 1), &S.a.recs[q - c0], 16, 0, 2);  // nt: read once
            }
        }
        MFN_ATICK(1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // an odd slot's pad record (the slot's next, stale record) becomes a zero record (no adds)
        if (tid < UNITS && (c & 1)) {
            const int k = S.a.pre[tid] + c;
            if (k >= c0 && k < c1) S.a.recs[k - c0] = make_uint2(0u, 0u);
        }
        __syncthreads();
        MFN_ATICK(2)
    };
    auto add_chunk = [&](int c0, int c1) __attribute__((always_inline)) {
        // (4) the adds, in a strided order over the stage
        const int len = c1 - c0;
        const int perm = (tid * 37) & (ACC_THREADS - 1);
        constexpr int UR = 4;  // stage reads in flight per thread before the first add
        for (int i0 = 0; i0 < len; i0 += UR * ACC_THREADS) {
            uint2 r[UR];
#pragma unroll
            for (int q = 0; q < UR; ++q) r[q] = S.a.recs[min(i0 + q * ACC_THREADS + perm, ACC_RB - 1)];
#pragma unroll
            for (int q = 0; q < UR; ++q)
                if (i0 + q * ACC_THREADS + perm < len) accum_record(img, mask, r[q], k2);
        }
        MFN_ATICK(3)
    };
    int c0 = 0;
    for (; T - c0 > ACC_RB; c0 += ACC_RB) {
        if (c0 > 0) __syncthreads();  // the previous chunk's adds are done with the stage
        copy_chunk(c0, c0 + ACC_RB);
        add_chunk(c0, c0 + ACC_RB);
    }
    if (c0 > 0) __syncthreads();
    copy_chunk(c0, T);  // the last chunk (T == 0: no records, its barriers only)
    if constexpr (FUSED) {
        // the optimizer state, loaded now: its loads then overlap the last chunk's adds instead of
        // delaying the partition's start.  Round 6: loaded first and guarded by `i < n_e`, each
        // entry's three loads were waited for inside their branch (a register copy out of the
        // loaded pair), four round trips in a row before the record copies began -- 27 % of a
        // partition workgroup's cycles (tools/scatter_probe.py, profiles/r06_v10_accum_probe.txt).
        // Unconditional here (a clamped index: the values past n_e are never used), no branch
        // and no copy; issued after the copy's wait, so the stage reads below need no vmcnt wait.
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int i = min(tid + k * ACC_THREADS, n_e - 1);  // (streamed once per step: non-temporal)
            const float2v a = __builtin_nontemporal_load(reinterpret_cast<const float2v*>(pp + i));
            const float2v b = __builtin_nontemporal_load(reinterpret_cast<const float2v*>(mm + i));
            const float2v c3 = __builtin_nontemporal_load(reinterpret_cast<const float2v*>(vv + i));
            p[k] = make_float2(a.x, a.y);
            m[k] = make_float2(b.x, b.y);
            v[k] = make_float2(c3.x, c3.y);
        }
    }
    add_chunk(c0, T);
    __syncthreads();
    MFN_ATICK(4)
    int* dst = grad + 2 * ((int64_t)P.t_offset[t] + e_lo);
    int2* ow = reinterpret_cast<int2*>(ovw) + ((int64_t)(P.t_offset[t] - P.t_offset[0]) + e_lo);  // overflow words
    const int rnd = kbits > 0 ? 1 << (kbits - 1) : 0;
    if constexpr (FUSED) {
        // fused optimizer (mfnerf_adam_step_fixed_partial): the entry's finished int32 sums, converted
        // with the table's scale exactly as adam_fixed_kernel converts them, feed the same Adam update;
        // the gradient words are left alone (zero)
        const float sc = table_fixed_scale(D, level_l1, P.t_level[t]);
        const float is = sc > 0.0f ? 1.0f / sc : 0.0f;
        if (add_words) {  // the overflowed records' sums join the image; the words are zeroed
            for (int i = threadIdx.x; i < n_e; i += blockDim.x) {
                const int2 g = ow[i];  // overflow_add's packed word
                const int2 v = img.get(i);
                const int o0 = ((v.x + rnd) >> kbits) + g.x, o1 = ((v.y + rnd) >> kbits) + g.y + (g.x < 0);
                img.set(i, make_int2(o0, o1));
                ow[i] = make_int2(0, 0);
            }
            __syncthreads();
        }
        if (A.amp && A.amp->nonfinite) return;  // GradScaler skip: no update (gradient words stay zero)
        const int kb = add_words ? 0 : kbits, rd = add_words ? 0 : rnd;  // (image now in table units)
        const int stp = *A.step_dev + 1;
        const float lr = A.lr_dev ? *A.lr_dev : A.lr;
        const float bc1 = 1.0f - powf(A.beta1, (float)stp);
        const float bc2 = 1.0f - powf(A.beta2, (float)stp);
        __half2* __restrict__ hh = reinterpret_cast<__half2*>(reinterpret_cast<__half*>(A.p16) + base_v);
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int i = tid + k * ACC_THREADS;
            if (i >= n_e) break;
            const int2 vv2 = img.get(i);
            const float g0 = (float)((vv2.x + rd) >> kb) * is, g1 = (float)((vv2.y + rd) >> kb) * is;
            mfn::adam_elem(p[k].x, m[k].x, v[k].x, g0, A.beta1, A.beta2, A.eps, lr, bc1, bc2);
            mfn::adam_elem(p[k].y, m[k].y, v[k].y, g1, A.beta1, A.beta2, A.eps, lr, bc1, bc2);
            __builtin_nontemporal_store(float2v{p[k].x, p[k].y}, reinterpret_cast<float2v*>(pp + i));
            __builtin_nontemporal_store(float2v{m[k].x, m[k].y}, reinterpret_cast<float2v*>(mm + i));
            __builtin_nontemporal_store(float2v{v[k].x, v[k].y}, reinterpret_cast<float2v*>(vv + i));
            if (A.p16) hh[i] = __floats2half2_rn(p[k].x, p[k].y);
        }
        MFN_ATICK(5)
#ifdef MFN_SCATTER_PROBE
        if (threadIdx.x == 0) {
            for (int k = 0; k < 6; ++k) atomicAdd(&g_accum_probe[k], (unsigned long long)at[k]);
            atomicAdd(&g_accum_probe[7], 1ull);
        }
#endif
        return;
    }
#undef MFN_ATICK
    // float_out: the finished sums as float gradients (the int32 value times 1 / the table's scale,
    // exactly what fold_convert_kernel computes), else the int32 sums for the finish pass
    const float sc = float_out ? table_fixed_scale(D, level_l1, P.t_level[t]) : 0.0f;
    const float is = sc > 0.0f ? 1.0f / sc : 0.0f;
    for (int i = threadIdx.x; i < n_e; i += blockDim.x) {
        const int2 v = img.get(i);
        // back to the table's unit, rounded once (|fields| <= 2^30: no overflow adding rnd)
        int2 o = make_int2((v.x + rnd) >> kbits, (v.y + rnd) >> kbits);
        if (add_words) {
            const int2 g = ow[i];  // overflow_add's packed f1 * 2^32 + f0
            o.x += g.x;
            o.y += g.y + (g.x < 0);
            ow[i] = make_int2(0, 0);
        }
        if (float_out) reinterpret_cast<float2*>(dst)[i] = make_float2((float)o.x * is, (float)o.y * is);
        else reinterpret_cast<int2*>(dst)[i] = o;
    }
}

// The plan for a desc: binned levels = every level that is not a dense own table; tables in address
// order.  Returns the number of bins (0: nothing to bin), or -1 if over MAX_BINS.
int first_binned_level(const mfnerf_grid_desc* d);

int bin_plan(const mfnerf_grid_desc* d, BinPlan* P) {
    *P = BinPlan{};
    const int l_first = first_binned_level(d);
    P->pair_ok = 1;
    uint64_t entries = 0, max_x = 0;
    for (int l = 0; l < d->n_levels; ++l) {
        const uint64_t r = d->res[l];
        (void)r;
        if (l < l_first) continue;  // dense levels, and the coarse hashed ones: atomics
        int t = 0;
        while (t < P->n_tables && P->t_offset[t] != d->offset[l]) ++t;
        if (t == P->n_tables) {
            P->t_offset[t] = d->offset[l];
            P->t_size[t] = d->size[l];
            P->t_level[t] = l;
            P->n_tables++;
            entries += d->size[l];
        }
        P->table_of[l] = t;
        P->pairable[l] = d->table_kind[l] == 0 && (d->size[l] & (d->size[l] - 1)) == 0;
        // never a pair record: a shared table whose canonical x-step floor(canon_res / res) >= 3, or an
        // own table without the power-of-two hash -> runs merged (merged_level_records)
        P->merge[l] = d->table_kind[l] == 1 ? (uint64_t)d->canon_res >= 3 * (uint64_t)d->res[l] : !P->pairable[l];
        P->level[P->n_binned++] = l;
        max_x = max(max_x, (uint64_t)(d->table_kind[l] == 1 ? (uint32_t)d->canon_res : d->res[l]));
    }
    // the largest partition (fewest records to route, least LDS per entry) leaving >= 1024 of them
    // (round 6, config 3's field -- 2^20 binned entries, 1024 partitions of 2^10 here: at least 512 /
    // 2048 / 4096 partitions ran 1.158 / 1.167 / 1.211 vs 1.149 ms/step, and the Lego step at 5120
    // partitions of 2^10 0.624 vs 0.506; profiles/r06_v8_ab_partition_count.txt)
    P->shift = MAX_BIN_SHIFT;
    while (P->shift > MIN_BIN_SHIFT && (entries >> P->shift) < 1024) --P->shift;
    int nb = 0;
    for (int t = 0; t < P->n_tables; ++t) {
        P->t_bin0[t] = nb;
        nb += (int)((P->t_size[t] + (1u << P->shift) - 1) >> P->shift);
        // x-corner indices differ below the top bit of x ^ (x+1), x + 1 <= max_x, in an own power-of-two
        // hash table: one record per row; otherwise up to two
        if ((P->t_size[t] & (P->t_size[t] - 1)) || max_x >= (1ull << P->shift)) P->pair_ok = 0;
    }
    for (int j = 0; j < P->n_binned; ++j) {
        if (!P->pairable[P->level[j]]) P->pair_ok = 0;
    }
    P->t_bin0[P->n_tables] = nb;
    P->n_bins = nb;
    if (P->n_binned > MAX_BINNED) return -1;
    for (int j = 1; j < P->n_binned; ++j)  // the binned levels are contiguous (staged dL/dy rows)
        if (P->level[j] != P->level[0] + j) return -1;
    for (int t = 0; t < P->n_tables; ++t)
        if (P->t_bin0[t + 1] - P->t_bin0[t] > MAX_TBINS) return -1;
    return nb > MAX_BINS ? -1 : nb;
}

// first level routed through the bins (the dense levels before it use grid_bw_dense_kernel): every
// hashed level (binning only the last 6 measured 392 vs 365 us for the scatter in round 2) --
// extended down to every level that shares a table with them (MixedFeature), since a partition is
// stored whole.
int first_binned_level(const mfnerf_grid_desc* d) {
    int first_hashed = d->n_levels;
    for (int l = 0; l < d->n_levels; ++l) {
        const uint64_t r = d->res[l];
        if (!(d->table_kind[l] == 0 && r * r * r <= d->size[l])) { first_hashed = l; break; }
    }
    int l0 = first_hashed;
    for (bool moved = true; moved;) {
        moved = false;
        for (int a = first_hashed; a < l0 && !moved; ++a)
            for (int b = l0; b < d->n_levels; ++b)
                if (d->offset[a] == d->offset[b]) { l0 = a; moved = true; break; }
    }
    // (round 6: also partitioning a MixedFeature layout's finest dense levels -- res >= 60 or >= 80,
    // as merged single records instead of run-merged atomics -- measured the same: mf128 1.197-1.200
    // vs 1.199-1.202 ms/step, r6e)
    return l0;
}

int binned_impl(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table, void* workspace,
                int64_t n_slots, const float* level_l1, int parts, const mfnerf_adam_fused* adam,
                mfnerf_stream_t stream, const AdamRest* rest = nullptr);

struct BinWorkspace {
    float* priv;
    int32_t *scnt, *ovf;
    int* ovw;  // overflow words: one packed int64 per partitioned entry (zero between steps)
    uint32_t* smax;
    uint2* rec;
};

int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }

// workspace = [private copies of the dense levels | overflow words | slot counts | overflow flag |
// record slots]
int64_t binned_workspace_layout(const mfnerf_grid_desc* d, int64_t n_max, char* base, BinWorkspace* W) {
    BinPlan P;
    if (bin_plan(d, &P) < 0) return -1;
    int64_t off = align256((int64_t)GRAD_COPIES * dense_entries_of(d) * 2 * (int64_t)sizeof(float));
    if (W) W->priv = reinterpret_cast<float*>(base);
    int64_t part_entries = 0;
    for (int t = 0; t < P.n_tables; ++t) part_entries += P.t_size[t];
    if (W) W->ovw = reinterpret_cast<int*>(base + off);
    off += align256(part_entries * 8);
    const int64_t nb = P.n_bins > 0 ? P.n_bins : 1;
    if (W) W->scnt = reinterpret_cast<int32_t*>(base + off);
    off += align256(nb * UNITS * 4);
    if (W) W->smax = reinterpret_cast<uint32_t*>(base + off);
    off += align256(UNITS * 4);
    if (W) W->ovf = reinterpret_cast<int32_t*>(base + off);
    off += 256;
    if (W) W->rec = reinterpret_cast<uint2*>(base + off);
    // every slot at the largest live count (the same function the kernels size them with); the
    // scatter addresses records with 32-bit indices
    if (nb * UNITS * slot_size(n_max, P) >= (int64_t)1 << 31) return -1;
    off += align256(nb * UNITS * slot_size(n_max, P) * (int64_t)sizeof(uint2));
    return off;
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
        auto kern = big ? grid_bw_kernel<MFN_MAX_LEVELS, true> : grid_bw_kernel<16, true>;
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(ENC_BLOCK), 0, stream, x, n, n_dev, x_min, x_range,
                           *desc, dL_dout, grad_table, (float*)workspace, dense, level_l1, desc->n_levels,
                           (int32_t*)nullptr);
    } else {
        auto kern = big ? grid_bw_kernel<MFN_MAX_LEVELS, false> : grid_bw_kernel<16, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(ENC_BLOCK), 0, stream, x, n, n_dev, x_min, x_range,
                           *desc, dL_dout, grad_table, (float*)workspace, dense, (const float*)nullptr,
                           desc->n_levels, (int32_t*)nullptr);
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
    return mfnerf_adam_step_fixed_partial(params, grads, m, v, p_f16, n, table_offset, desc, workspace, level_l1, lr,
                                          beta1, beta2, eps, step_dev, lr_dev, amp, n, nullptr, stream);
}

int mfnerf_adam_step_fixed_partial(float* params, float* grads, float* m, float* v, void* p_f16, int64_t n,
                                   int64_t table_offset, const mfnerf_grid_desc* desc, void* workspace,
                                   float* level_l1, float lr, float beta1, float beta2, float eps,
                                   int32_t* step_dev, const float* lr_dev, mfnerf_amp_state* amp, int64_t fused_from,
                                   const int32_t* fused_ovf, mfnerf_stream_t stream) {
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
    if (fused_from < 0 || fused_from > n || fused_from % 4) {
        mfn_set_error("adam_step_fixed_partial: fused_from (%lld) must be a multiple of 4 in [0, n]",
                      (long long)fused_from);
        return MFN_ERR_INVALID;
    }
    if (n % 4 || table_offset % 4 || table_offset < 0 || table_offset + total > n) {
        mfn_set_error("adam_step_fixed: n (%lld) and table_offset (%lld) must be multiples of 4 holding the table",
                      (long long)n, (long long)table_offset);
        return MFN_ERR_INVALID;
    }
    // sized for the range normally updated: every workgroup takes the last-workgroup ticket (one
    // memory-side atomic on ONE address each, serialised: ~13 ns apiece), so an idle workgroup is
    // not free (4096 of them cost ~55 us in the fused_from case); grid-stride covers the rest
    const int64_t want = div_up<int64_t>((fused_ovf ? fused_from : n) / 4, 256);
    // measured: 4096 -> 1024 workgroups 88 -> 78 us (fewer tickets, same bandwidth)
    constexpr int64_t ADAM_BLOCKS = 1024;
    hipLaunchKernelGGL(adam_fixed_kernel,
                       dim3((unsigned)(want < ADAM_BLOCKS ? (want < 1 ? 1 : want) : ADAM_BLOCKS)), dim3(256), 0,
                       stream, params, grads, m, v, (__half*)p_f16, n, table_offset, (int*)workspace, 2 * dense,
                       total, *desc, level_l1, lr, beta1, beta2, eps, step_dev, lr_dev, amp, desc->n_levels,
                       fused_from, fused_ovf, 0, PackArgs{nullptr, nullptr, nullptr, 0});
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

// Partitioned (binned) fixed-point table-gradient scatter: the dense levels through grid_bw_body's
// private copies (parts & 1), the hashed / shared tables through scatter -> LDS accumulate (parts & 2).
int64_t mfnerf_grid_encode_bw_binned_workspace(const mfnerf_grid_desc* desc, int64_t n_max) {
    if (check_desc(desc, "grid_encode_bw_binned_workspace") || n_max < 0) return -1;
    return binned_workspace_layout(desc, n_max, nullptr, nullptr);
}

int mfnerf_grid_encode_bw_binned(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                 const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                 void* workspace, int64_t n_slots, const float* level_l1, int parts,
                                 mfnerf_stream_t stream) {
    return binned_impl(x, n, n_dev, x_min, x_range, desc, dL_dout, grad_table, workspace, n_slots, level_l1, parts,
                       nullptr, stream);
}

int mfnerf_grid_encode_bw_binned_float(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                       const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                       void* workspace, int64_t n_slots, const float* level_l1, int32_t* gate,
                                       const int32_t* flag, int64_t flag_world, int64_t flag_shard_len,
                                       int64_t table_offset, mfnerf_stream_t stream) {
    if (flag && (flag_world < 1 || flag_world > 256 || flag_shard_len < 1 || table_offset < 0)) {
        mfn_set_error("grid_encode_bw_binned_float: bad shard-flag arguments");
        return MFN_ERR_INVALID;
    }
    BinPlan P;
    if (check_desc(desc, "grid_encode_bw_binned_float") || bin_plan(desc, &P) <= 0) {
        mfn_set_error("grid_encode_bw_binned_float: bad desc or nothing partitioned");
        return MFN_ERR_INVALID;
    }
    AdamRest X{};  // no optimizer blocks; only the gate (opened as the dense-level launch starts)
    X.gate = gate;
    int st = binned_impl(x, n, n_dev, x_min, x_range, desc, dL_dout, grad_table, workspace, n_slots, level_l1, 7,
                         nullptr, stream, gate ? &X : nullptr);
    if (st || n == 0) return st;
    // the values before the partitioned tables: the dense levels' copies folded, any other level's
    // int32 sums converted (the accumulate wrote the partitioned tables' floats)
    const int64_t head = 2 * (int64_t)P.t_offset[0];
    const ShardFlag SF{flag, flag_world, flag_shard_len, table_offset};
    if (head > 0) {
        const int64_t fb = div_up<int64_t>(head / 4, 256);
        hipLaunchKernelGGL(fold_convert_kernel, dim3((unsigned)(fb < 4096 ? fb : 4096)), dim3(256), 0, stream,
                           grad_table, (int*)workspace, 2 * dense_entries_of(desc), head, *desc, level_l1, SF);
    } else if (flag) {
        mfn_set_error("grid_encode_bw_binned_float: a shard flag needs a table prefix to ride");
        return MFN_ERR_INVALID;
    }
    return mfn_check_launch("grid_encode_bw_binned_float");
}

int mfnerf_grid_encode_bw_binned_adam(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                      const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table,
                                      void* workspace, int64_t n_slots, const float* level_l1,
                                      const mfnerf_adam_fused* adam, mfnerf_stream_t stream) {
    if (!adam || !adam->params || !adam->m || !adam->v || !adam->step_dev ||
        (((uintptr_t)adam->params | (uintptr_t)adam->m | (uintptr_t)adam->v) & 7) || (adam->table_offset & 1)) {
        mfn_set_error("grid_encode_bw_binned_adam: bad Adam arguments (null or misaligned vectors, odd table_offset)");
        return MFN_ERR_INVALID;
    }
    return binned_impl(x, n, n_dev, x_min, x_range, desc, dL_dout, grad_table, workspace, n_slots, level_l1, 3,
                       adam, stream);
}

}  // extern "C"

namespace {
int adam_all_impl(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                  const mfnerf_grid_desc* desc, const float* dL_dout, float* grads, int64_t n_params,
                  void* workspace, int64_t n_slots, float* level_l1, const mfnerf_adam_fused* adam,
                  int32_t* step_dev, mfnerf_amp_state* amp, void* packed, int rgb_width, int32_t* gate,
                  mfnerf_stream_t stream) {
    if (packed && ((rgb_width != 64 && rgb_width != 128) || !adam || !adam->p16)) {
        mfn_set_error("grid_encode_bw_binned_adam_all: the repack needs rgb_width 64 or 128 and adam->p16");
        return MFN_ERR_INVALID;
    }
    if (!adam || !adam->params || !adam->m || !adam->v || !grads || !step_dev || adam->step_dev != step_dev ||
        adam->amp != amp || (((uintptr_t)adam->params | (uintptr_t)adam->m | (uintptr_t)adam->v |
                              (uintptr_t)grads) & 15) || (adam->p16 && ((uintptr_t)adam->p16 & 7)) ||
        adam->table_offset % 4 || n_params % 4 || adam->table_offset < 0) {
        mfn_set_error("grid_encode_bw_binned_adam_all: bad Adam arguments (null or misaligned vectors, "
                      "table_offset / n_params not multiples of 4, step_dev / amp differing from adam's)");
        return MFN_ERR_INVALID;
    }
    int st = check_desc(desc, "grid_encode_bw_binned_adam_all");
    if (st) return st;
    int64_t total = 0;
    for (int l = 0; l < desc->n_levels; ++l) {
        const int64_t e = 2 * ((int64_t)desc->offset[l] + desc->size[l]);
        total = e > total ? e : total;
    }
    BinPlan P;
    if (bin_plan(desc, &P) <= 0 || adam->table_offset + total > n_params) {
        mfn_set_error("grid_encode_bw_binned_adam_all: nothing partitioned, or the table outside [table_offset, n_params)");
        return MFN_ERR_INVALID;
    }
    const int64_t fused_from = adam->table_offset + 2 * (int64_t)P.t_offset[0];  // the partitioned tables' first value
    if (fused_from % 4) { mfn_set_error("grid_encode_bw_binned_adam_all: partitions not float4-aligned"); return MFN_ERR_INVALID; }
    BinWorkspace W;
    if (binned_workspace_layout(desc, n_slots <= 0 || n_slots > n ? n : n_slots, (char*)workspace, &W) < 0) {
        mfn_set_error("grid_encode_bw_binned_adam_all: the record slots overflow 32-bit record indices");
        return MFN_ERR_INVALID;
    }
    // [0, fused_from) by the accumulate launch's leading workgroups (one float4 per thread, <= 256 of
    // them)
    AdamRest X{grads, (int*)workspace, 2 * dense_entries_of(desc), total, fused_from / 4, 0, 1, gate};
    // <= 256 workgroups, the grid's first (256 vs 64 of them 0.655 vs 0.657 ms/step; first vs last
    // in the grid within noise)
    const int64_t want = div_up<int64_t>(fused_from / 4, ACC_THREADS);
    X.n_blocks = (int)(want < 1 ? 1 : (want < 256 ? want : 256));
    X.first = 1;
    st = binned_impl(x, n, n_dev, x_min, x_range, desc, dL_dout, grads + adam->table_offset, workspace, n_slots,
                     level_l1, 3, adam, stream, &X);
    if (st) return st;
    // the MLP repack and the step's bookkeeping (step count, loss scale, level_l1 zeroed) by the last
    // workgroup -- after every workgroup of the accumulate has read them
    hipLaunchKernelGGL(adam_fixed_kernel, dim3(64), dim3(256), 0, stream, adam->params, grads, adam->m, adam->v,
                       (__half*)adam->p16, n_params, adam->table_offset, (int*)workspace, 2 * dense_entries_of(desc),
                       total, *desc, level_l1, adam->lr, adam->beta1, adam->beta2, adam->eps, step_dev, adam->lr_dev,
                       amp, desc->n_levels, fused_from, (const int32_t*)W.ovf, 1,
                       PackArgs{(const _Float16*)adam->p16, (const _Float16*)adam->p16 + mfn_field::N_XYZ_PARAMS,
                                (_Float16*)packed, rgb_width});
    if (!amp)
        hipLaunchKernelGGL(mfn_bump_step_kernel, dim3(1), dim3(1), 0, stream, step_dev, amp, level_l1, desc->n_levels);
    return mfn_check_launch("grid_encode_bw_binned_adam_all");
}
}  // namespace

extern "C" {

int mfnerf_grid_encode_bw_binned_adam_all(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                                          const mfnerf_grid_desc* desc, const float* dL_dout, float* grads,
                                          int64_t n_params, void* workspace, int64_t n_slots, float* level_l1,
                                          const mfnerf_adam_fused* adam, int32_t* step_dev, mfnerf_amp_state* amp,
                                          void* packed, int rgb_width, int32_t* gate, mfnerf_stream_t stream) {
    return adam_all_impl(x, n, n_dev, x_min, x_range, desc, dL_dout, grads, n_params, workspace, n_slots, level_l1,
                         adam, step_dev, amp, packed, rgb_width, gate, stream);
}

int64_t mfnerf_grid_binned_first_value(const mfnerf_grid_desc* desc) {
    if (check_desc(desc, "grid_binned_first_value")) return -1;
    BinPlan P;
    if (bin_plan(desc, &P) <= 0) return -1;
    return 2 * (int64_t)P.t_offset[0];
}

int64_t mfnerf_grid_dense_values(const mfnerf_grid_desc* desc) {
    if (check_desc(desc, "grid_dense_values")) return -1;
    return 2 * dense_entries_of(desc);
}

int64_t mfnerf_grid_encode_bw_binned_flag_offset(const mfnerf_grid_desc* desc, int64_t n_slots) {
    if (check_desc(desc, "grid_encode_bw_binned_flag_offset") || n_slots <= 0) return -1;
    BinWorkspace W;
    if (binned_workspace_layout(desc, n_slots, nullptr, &W) < 0) return -1;
    return (int64_t)reinterpret_cast<uintptr_t>(W.ovf);
}

}  // extern "C"

namespace {
int binned_impl(const float* x, int64_t n, const int32_t* n_dev, float x_min, float x_range,
                const mfnerf_grid_desc* desc, const float* dL_dout, float* grad_table, void* workspace,
                int64_t n_slots, const float* level_l1, int parts, const mfnerf_adam_fused* adam,
                mfnerf_stream_t stream, const AdamRest* rest) {
    int st = check_desc(desc, "grid_encode_bw_binned");
    if (st) return st;
    if (n_slots <= 0 || n_slots > n) n_slots = n;
    if (n < 0 || parts < 1 || parts > 7 || (parts & 4 && adam)) {
        mfn_set_error("grid_encode_bw_binned: bad size or parts");
        return MFN_ERR_INVALID;
    }
    if (n == 0) return MFN_OK;
    if (!x || !dL_dout || !grad_table || !workspace || !level_l1) {
        mfn_set_error("grid_encode_bw_binned: null pointer (workspace and level_l1 are required)");
        return MFN_ERR_INVALID;
    }
    BinPlan P;
    if (bin_plan(desc, &P) < 0) {
        mfn_set_error("grid_encode_bw_binned: unsupported layout (> %d partitions, > %d bins per table, or binned "
                      "levels not the contiguous last %d)", MAX_BINS, MAX_TBINS, MAX_BINNED);
        return MFN_ERR_INVALID;
    }
    BinWorkspace W;
    if (binned_workspace_layout(desc, n_slots, (char*)workspace, &W) < 0) {
        mfn_set_error("grid_encode_bw_binned: %lld record slots per partition and unit overflow 32-bit record "
                      "indices (size the slots for fewer samples, n_slots)", (long long)n_slots);
        return MFN_ERR_INVALID;
    }
    const int l_first = first_binned_level(desc);
    const int64_t want = div_up<int64_t>(div_up<int64_t>(n, 16), ENC_BLOCK / 64);
    const int64_t cap = grid_bw_block_cap();
    const int64_t atomic_blocks = want < cap ? want : cap;
    const bool big = desc->n_levels > 16;
    int n_dense_levels = 0;  // leading levels that are dense own tables inside the private copies
    {
        const int64_t de = dense_entries_of(desc);
        while (n_dense_levels < desc->n_levels && desc->table_kind[n_dense_levels] == 0 &&
               (int64_t)desc->offset[n_dense_levels] + desc->size[n_dense_levels] <= de)
            ++n_dense_levels;
    }
    if ((parts & 1) && l_first > 0 && l_first <= n_dense_levels) {
        // levels [0, l_first) all dense: one sample per lane, packed 64-bit adds into the copies
        // DENSE_WAVES waves at most (the kernel's window spreads any sample count over them)
        const int64_t wb = std::min<int64_t>(div_up<int64_t>(n, (int64_t)64 * (ENC_BLOCK / 64)),
                                        div_up<int64_t>(DENSE_WAVES, ENC_BLOCK / 64));
        auto dk = l_first <= 8 ? grid_bw_dense_kernel<4> : l_first <= 16 ? grid_bw_dense_kernel<8> : grid_bw_dense_kernel<16>;
        hipLaunchKernelGGL(dk, dim3((unsigned)(wb < cap ? wb : cap)), dim3(ENC_BLOCK), 0, stream,
                           x, n, n_dev, x_min, x_range, *desc, dL_dout, W.priv, dense_entries_of(desc), level_l1,
                           l_first, (parts & 2) ? W.ovf : (int32_t*)nullptr, rest ? rest->gate : (int32_t*)nullptr);
    } else if ((parts & 1) && l_first > 0) {  // dense levels [0, l_first): request-shaped atomics, private copies
        auto kern = big ? grid_bw_kernel<MFN_MAX_LEVELS, true> : grid_bw_kernel<16, true>;
        hipLaunchKernelGGL(kern, dim3((unsigned)atomic_blocks), dim3(ENC_BLOCK), 0, stream, x, n, n_dev, x_min,
                           x_range, *desc, dL_dout, grad_table, W.priv, dense_entries_of(desc), level_l1, l_first,
                           (parts & 2) ? W.ovf : (int32_t*)nullptr);
    }
    // the gate opens here whichever dense path ran (only grid_bw_dense_kernel opens it itself)
    if (rest && rest->gate && !((parts & 1) && l_first > 0 && l_first <= n_dense_levels))
        mfnerf_gate_signal(rest->gate, stream);  // (after the request-shaped atomics, or first)
    if ((parts & 2) && P.n_bins > 0) {
        if (!((parts & 1) && l_first > 0)) mfn_zero_async(W.ovf, sizeof(int32_t), stream);
        // the staged dL/dy rows sized for the binned levels (10 at the Lego layout; MixedFeature's
        // shared tables bin more): the smallest staging that holds them leaves room on each CU for
        // the side stream's march kernels
        auto sk = P.pair_ok ? (P.n_binned <= 8    ? bin_scatter_kernel<8, true>
                               : P.n_binned <= 10 ? bin_scatter_kernel<10, true>
                               : P.n_binned <= 12 ? bin_scatter_kernel<12, true>
                                                  : bin_scatter_kernel<MAX_BINNED, true>)
                            : (P.n_binned <= 8    ? bin_scatter_kernel<8, false>
                               : P.n_binned <= 12 ? bin_scatter_kernel<12, false>
                                                  : bin_scatter_kernel<MAX_BINNED, false>);
        hipLaunchKernelGGL(sk, dim3(UNITS), dim3(SC_THREADS), 0, stream, x, n, n_dev, x_min, x_range,
                           *desc, P, dL_dout, level_l1, W.rec, W.scnt, W.smax, W.ovf, n_slots, W.ovw);

        mfnerf_adam_fused A{};
        if (adam) A = *adam;
        AdamRest X{};
        if (rest) X = *rest;
        hipLaunchKernelGGL(A.params ? bin_accum_kernel<true> : bin_accum_kernel<false>, dim3(P.n_bins + X.n_blocks),
                           dim3(ACC_THREADS), 0, stream, P, n, n_dev,
                           W.rec, W.scnt, W.smax, W.ovf, W.ovw, (int*)grad_table, n_slots, *desc, level_l1, A, X,
                           (parts & 4) ? 1 : 0);
    }
    return mfn_check_launch("grid_encode_bw_binned");
}
}  // namespace
