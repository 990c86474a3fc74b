// occupancy.hip -- the occupancy-grid refresh of models/networks.py:157-271 (train.py:165-168,
// every 16 steps) as device-only kernels: no torch.nonzero / .item() host synchronisation.
//
//   mfnerf_occupancy_cells   : cells to probe -> jittered world points + flat cell index
//       warm-up: every cell of every cascade (get_all_cells, networks.py:157-166);
//       otherwise per cascade M uniform cells + M cells drawn uniformly from the cells whose
//       density > threshold (sample_uniform_and_occupied_cells, networks.py:168-192).  The
//       occupied list is built by an order-preserving compaction (ascending morton index,
//       exactly torch.nonzero's order), so index r of the list is the reference's indices2[r].
//   (caller runs mfnerf_grid_encode_fw + mfnerf_field_fw(density_only) on the points)
//   mfnerf_occupancy_update  : tmp[cell] = sigma; grid = where(grid<0, grid, max(grid*decay, tmp));
//       thr = min(mean(grid[grid>0]), threshold); packbits(grid, thr)  (networks.py:242-271).
//
// Randomness: torch.randint / torch.rand are replaced by a counter-based hash (seed, call, point,
// coordinate) -- the same distributions, not torch's streams.
#include "common.hpp"
#include "../../include/mfnerf.h"

using namespace mfn;

namespace {

constexpr int OCC_BLOCK = 256;
constexpr int OCC_PER_THREAD = 16;
constexpr int OCC_CELLS_PER_BLOCK = OCC_BLOCK * OCC_PER_THREAD;  // 4096

__device__ __forceinline__ uint32_t mix64to32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return (uint32_t)x;
}
// per-call key: the call index goes through a full avalanche (added linearly to the counter it
// would make draw (call c, k) equal draw (call c+1, k-1))
__host__ __device__ __forceinline__ uint64_t splitmix64_host(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
constexpr uint64_t OCC_SEED_MIX = 0x5851F42D4C957F2Dull;
__device__ __forceinline__ uint32_t rnd32(uint64_t key, uint64_t ctr) {
    return mix64to32(key + ctr * 0x9E3779B97F4A7C15ull);
}
__device__ __forceinline__ uint32_t rnd_below(uint64_t key, uint64_t ctr, uint32_t n) {
    return (uint32_t)(((uint64_t)rnd32(key, ctr) * n) >> 32);
}
__device__ __forceinline__ float rnd_unit(uint64_t key, uint64_t ctr) {  // [0,1), 24 bits like torch.rand
    return (float)(rnd32(key, ctr) >> 8) * (1.0f / 16777216.0f);
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* lds) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds[w] = v;
    __syncthreads();
    T s = 0;
    for (int i = 0; i < OCC_BLOCK / 64; ++i) s += lds[i];
    return s;
}

// per block: number of cells with density > thr
__global__ __launch_bounds__(OCC_BLOCK) void occ_count_kernel(const float* __restrict__ grid, int64_t cells,
                                                              float thr, int32_t* __restrict__ block_counts) {
    __shared__ int lds[OCC_BLOCK / 64];
    const int c = blockIdx.y, nblk = gridDim.x;
    const int64_t base = (int64_t)c * cells + (int64_t)blockIdx.x * OCC_CELLS_PER_BLOCK + threadIdx.x * OCC_PER_THREAD;
    const int64_t end = (int64_t)c * cells + cells;
    int k = 0;
#pragma unroll
    for (int i = 0; i < OCC_PER_THREAD; ++i) k += (base + i < end && grid[base + i] > thr) ? 1 : 0;
    k = block_sum(k, lds);
    if (threadIdx.x == 0) block_counts[c * nblk + blockIdx.x] = k;
}

// order-preserving compaction of the occupied cells of each cascade
__global__ __launch_bounds__(OCC_BLOCK) void occ_compact_kernel(const float* __restrict__ grid, int64_t cells,
                                                                float thr, const int32_t* __restrict__ block_counts,
                                                                int32_t* __restrict__ list, int32_t* __restrict__ counts) {
    __shared__ int lds[OCC_BLOCK / 64];
    __shared__ int wave_tot[OCC_BLOCK / 64];
    const int c = blockIdx.y, nblk = gridDim.x, b = blockIdx.x;
    int pre = 0;
    for (int i = threadIdx.x; i < b; i += OCC_BLOCK) pre += block_counts[c * nblk + i];
    pre = block_sum(pre, lds);
    const int64_t j0 = (int64_t)b * OCC_CELLS_PER_BLOCK + threadIdx.x * OCC_PER_THREAD;
    const float* g = grid + (int64_t)c * cells;
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < OCC_PER_THREAD; ++i) mask |= (j0 + i < cells && g[j0 + i] > thr) ? (1u << i) : 0u;
    const int mine = __popc(mask);
    // exclusive scan of `mine` over the block (thread order == cell order)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wave_tot[w] = incl;
    __syncthreads();
    int wpre = 0;
    for (int i = 0; i < w; ++i) wpre += wave_tot[i];
    int pos = pre + wpre + incl - mine;
    int32_t* out = list + (int64_t)c * cells;
    while (mask) {
        const int i = __ffs(mask) - 1;
        mask &= mask - 1;
        out[pos++] = (int32_t)(j0 + i);
    }
    if (b == nblk - 1 && threadIdx.x == OCC_BLOCK - 1) counts[c] = pos;
}

struct PointsArgs {
    int cascades, G;
    int64_t cells, per_cascade, n_uniform;
    int warmup;
    float scale;
    uint64_t key;
    uint64_t seed;
    const uint64_t* call_dev;  // non-null: key from the device-resident call index (graph replays)
    uint64_t call_lag;         // the index was already advanced by this much (the probe kernel reads it
                               // after the marked-cell compaction advanced it)
};

// draw p's cell: cascade c, morton m; ok = false for an occupied draw from an empty set
__device__ __forceinline__ void draw_cell(const PointsArgs& a, const int32_t* __restrict__ list,
                                          const int32_t* __restrict__ counts, int64_t p, int& c, uint32_t& m,
                                          bool& ok) {
    c = (int)(p / a.per_cascade);
    const int64_t j = p - (int64_t)c * a.per_cascade;
    ok = true;
    if (a.warmup) {
        m = (uint32_t)j;
    } else if (j < a.n_uniform) {
        const uint32_t cx = rnd_below(a.key, 8 * (uint64_t)p + 0, a.G);
        const uint32_t cy = rnd_below(a.key, 8 * (uint64_t)p + 1, a.G);
        const uint32_t cz = rnd_below(a.key, 8 * (uint64_t)p + 2, a.G);
        m = morton3(cx, cy, cz);
    } else {
        const int cnt = counts[c];
        ok = cnt > 0;  // empty occupied set: the reference draws no such cells
        m = ok ? (uint32_t)list[(int64_t)c * a.cells + rnd_below(a.key, 8 * (uint64_t)p + 3, (uint32_t)cnt)] : 0u;
    }
}

// networks.py:253-258: s = min(2^(c-1), scale); x = (coords/(G-1)*2-1)*(s - s/G) + (2u-1)*(s/G);
// u from counters ctr + k of `key`
__device__ __forceinline__ void cell_point(const PointsArgs& a, int c, uint32_t m, uint64_t key, uint64_t ctr,
                                           float* __restrict__ out) {
    const float s = fminf(ldexpf(1.0f, c - 1), a.scale);
    const float hgs = s / (float)a.G;
    const float span = s - hgs;
    const float inv = (float)(a.G - 1);
    const uint32_t q[3] = {morton3_invert(m), morton3_invert(m >> 1), morton3_invert(m >> 2)};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float base = ((float)q[k] / inv * 2.0f - 1.0f) * span;
        const float u = rnd_unit(key, ctr + k);
        out[k] = base + (u * 2.0f - 1.0f) * hgs;
    }
}

__global__ __launch_bounds__(OCC_BLOCK) void occ_points_kernel(PointsArgs a, const int32_t* __restrict__ list,
                                                               const int32_t* __restrict__ counts,
                                                               float* __restrict__ xyzs, int32_t* __restrict__ cell) {
    const int64_t n = (int64_t)a.cascades * a.per_cascade;
    if (a.call_dev) a.key = splitmix64_host(splitmix64_host(a.seed ^ OCC_SEED_MIX) ^ (*a.call_dev - a.call_lag));
    for (int64_t p = (int64_t)blockIdx.x * OCC_BLOCK + threadIdx.x; p < n; p += (int64_t)gridDim.x * OCC_BLOCK) {
        int c;
        uint32_t m;
        bool ok;
        draw_cell(a, list, counts, p, c, m, ok);
        cell_point(a, c, m, a.key, 8 * (uint64_t)p + 4, xyzs + 3 * p);
        cell[p] = ok ? (int32_t)((int64_t)c * a.cells + m) : -1;
    }
}

// The byte map of the de-duplicated draw is indexed in ROW-MAJOR order within a cascade (x fastest),
// so the probe points reach the encode x-neighbour after x-neighbour: the hashed levels' index is
// x ^ (y p1) ^ (z p2), so x-adjacent probes read adjacent table entries (shared lines) where the
// morton order put y/z neighbours -- a different line per lane -- next to each other.
__device__ __forceinline__ uint32_t row_major(int G, uint32_t m) {
    return morton3_invert(m) + (uint32_t)G * (morton3_invert(m >> 1) + (uint32_t)G * morton3_invert(m >> 2));
}
__device__ __forceinline__ uint32_t morton_of_row_major(int G, uint32_t r) {
    const uint32_t x = r % (uint32_t)G, yz = r / (uint32_t)G;
    return morton3(x, yz % (uint32_t)G, yz / (uint32_t)G);
}

// ---- the de-duplicated draw (mfnerf_occupancy_cells_unique*): the reference probes every draw and
// keeps one sigma per cell (`density_grid_tmp[c, indices] = sigmas`, an index_put whose duplicate
// writes land in no defined order), so only one jittered point per DISTINCT drawn cell can reach the
// grid.  The draws only mark their cells in a byte map (idempotent plain stores, no atomics); the map
// is compacted in ascending row-major cell order within a cascade (x-neighbours adjacent, below) and
// each marked cell gets one uniform jitter keyed by (call, morton cell).  Same distribution as
// the reference's update -- the set of drawn cells, one uniform point per cell -- with ~60 % of the
// points at a trained scene's occupancy, and deterministic (no write race on duplicates).
__global__ __launch_bounds__(OCC_BLOCK) void occ_mark_kernel(PointsArgs a, const int32_t* __restrict__ list,
                                                             const int32_t* __restrict__ counts,
                                                             uint8_t* __restrict__ mark) {
    const int64_t n = (int64_t)a.cascades * a.per_cascade;
    if (a.call_dev) a.key = splitmix64_host(splitmix64_host(a.seed ^ OCC_SEED_MIX) ^ (*a.call_dev - a.call_lag));
    for (int64_t p = (int64_t)blockIdx.x * OCC_BLOCK + threadIdx.x; p < n; p += (int64_t)gridDim.x * OCC_BLOCK) {
        int c;
        uint32_t m;
        bool ok;
        draw_cell(a, list, counts, p, c, m, ok);
        if (ok) mark[(int64_t)c * a.cells + row_major(a.G, m)] = 1;
    }
}

// marked cells per 4096-cell block (16 bytes of the map per thread)
__global__ __launch_bounds__(OCC_BLOCK) void occ_mark_count_kernel(const uint8_t* __restrict__ mark, int64_t total,
                                                                   int32_t* __restrict__ block_counts) {
    __shared__ int lds[OCC_BLOCK / 64];
    const int64_t i0 = (int64_t)blockIdx.x * OCC_CELLS_PER_BLOCK + threadIdx.x * OCC_PER_THREAD;  // total % 16 == 0
    int k = 0;
    if (i0 < total) {
        const uint4 v = *reinterpret_cast<const uint4*>(mark + i0);  // marks are 0 / 1
        k = __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
    }
    k = block_sum(k, lds);
    if (threadIdx.x == 0) block_counts[blockIdx.x] = k;
}

// the marked cells in ascending order into list (their count into *count), the map zeroed behind
__global__ __launch_bounds__(OCC_BLOCK) void occ_mark_compact_kernel(uint8_t* __restrict__ mark, int64_t total,
                                                                     const int32_t* __restrict__ block_counts,
                                                                     int32_t* __restrict__ list,
                                                                     int32_t* __restrict__ count,
                                                                     uint64_t* __restrict__ call_dev) {
    // the draws' device call index advanced here: every read of it for these draws (the mark
    // kernel) is done, and the probe kernel after this reads it with call_lag 1 -- no launch of its own
    if (call_dev && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_fetch_add(call_dev, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __shared__ int lds[OCC_BLOCK / 64];
    __shared__ int wave_tot[OCC_BLOCK / 64];
    const int b = blockIdx.x, nblk = gridDim.x;
    int pre = 0;
    for (int i = threadIdx.x; i < b; i += OCC_BLOCK) pre += block_counts[i];
    pre = block_sum(pre, lds);
    const int64_t i0 = (int64_t)b * OCC_CELLS_PER_BLOCK + threadIdx.x * OCC_PER_THREAD;
    uint32_t bits = 0;
    if (i0 < total) {
        uint4* src = reinterpret_cast<uint4*>(mark + i0);
        const uint4 v = *src;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) bits |= ((w[k >> 2] >> (8 * (k & 3))) & 1u) << k;
        if (bits) *src = make_uint4(0u, 0u, 0u, 0u);
    }
    const int mine = __popc(bits);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(incl, o);
        if (lane >= o) incl += t;
    }
    if (lane == 63) wave_tot[w] = incl;
    __syncthreads();
    int wpre = 0;
    for (int i = 0; i < w; ++i) wpre += wave_tot[i];
    int pos = pre + wpre + incl - mine;
    while (bits) {
        const int k = __ffs(bits) - 1;
        bits &= bits - 1;
        list[pos++] = (int32_t)(i0 + k);
    }
    if (b == nblk - 1 && threadIdx.x == OCC_BLOCK - 1) *count = pos;
}

// one jittered point per listed cell: counters 4..6 of the cell's own stream (key mixed apart from
// the draws' key, so a cell's jitter is independent of which draws chose it)
constexpr uint64_t OCC_JITTER_MIX = 0x632BE59BD9B4E019ull;
__global__ __launch_bounds__(OCC_BLOCK) void occ_unique_points_kernel(PointsArgs a, const int32_t* __restrict__ list,
                                                                      const int32_t* __restrict__ count,
                                                                      float* __restrict__ xyzs,
                                                                      int32_t* __restrict__ cell) {
    if (a.call_dev) a.key = splitmix64_host(splitmix64_host(a.seed ^ OCC_SEED_MIX) ^ (*a.call_dev - a.call_lag));
    const uint64_t jkey = splitmix64_host(a.key ^ OCC_JITTER_MIX);
    const int64_t n = *count;
    for (int64_t i = (int64_t)blockIdx.x * OCC_BLOCK + threadIdx.x; i < n; i += (int64_t)gridDim.x * OCC_BLOCK) {
        const int32_t r = list[i];  // (row-major within the cascade)
        const int c = (int)(r / a.cells);
        const uint32_t m = morton_of_row_major(a.G, (uint32_t)(r - (int64_t)c * a.cells));
        const int64_t f = (int64_t)c * a.cells + m;
        cell_point(a, c, m, jkey, 8 * (uint64_t)f + 4, xyzs + 3 * i);
        cell[i] = (int32_t)f;
    }
}

__global__ __launch_bounds__(OCC_BLOCK) void occ_scatter_kernel(const float* __restrict__ sigma,
                                                                const int32_t* __restrict__ cell, int64_t n,
                                                                const int32_t* __restrict__ n_dev,
                                                                float* __restrict__ tmp) {
    if (n_dev) n = min<int64_t>(n, (int64_t)*n_dev);
    for (int64_t p = (int64_t)blockIdx.x * OCC_BLOCK + threadIdx.x; p < n; p += (int64_t)gridDim.x * OCC_BLOCK) {
        const int32_t k = cell[p];
        if (k >= 0) tmp[k] = sigma[p];
    }
}

// The mean over positive cells: each decay workgroup writes its partial (sum, count); the
// threshold kernel adds the partials in workgroup order (deterministic; round 2 added them with two
// memory-side atomics per workgroup on one address each: 4096 serialised atomics, ~55 us).
constexpr int DECAY_BLOCKS = 1024;
struct OccStats {
    double sum[DECAY_BLOCKS];
    unsigned long long count[DECAY_BLOCKS];
    float thr;
};

__device__ __forceinline__ float decay_cell(float v, float t, const float* __restrict__ count_grid, int64_t i,
                                            float decay) {
    if (v < 0.0f) return v;
    float d = decay;
    if (count_grid) d = clampf(powf(decay, 1.0f / count_grid[i]), 0.1f, 0.95f);  // erode (networks.py:262)
    return fmaxf(v * d, t);
}

// four cells per thread per step (float4), every load of a thread's slice issued before the math
__global__ __launch_bounds__(OCC_BLOCK) void occ_decay_kernel(float* __restrict__ grid, float* __restrict__ tmp,
                                                              const float* __restrict__ count_grid, int64_t n,
                                                              float decay, OccStats* __restrict__ st, int zero_tmp) {
    __shared__ double lds_d[OCC_BLOCK / 64];
    __shared__ unsigned long long lds_u[OCC_BLOCK / 64];
    double s = 0.0;
    unsigned long long k = 0;
    float4* g4 = reinterpret_cast<float4*>(grid);
    float4* t4 = reinterpret_cast<float4*>(tmp);
    for (int64_t i = (int64_t)blockIdx.x * OCC_BLOCK + threadIdx.x; i < n / 4; i += (int64_t)gridDim.x * OCC_BLOCK) {
        float4 v = g4[i];
        const float4 t = t4[i];
        if (zero_tmp) t4[i] = make_float4(0.f, 0.f, 0.f, 0.f);  // left zero for the next refresh
        v.x = decay_cell(v.x, t.x, count_grid, 4 * i, decay);
        v.y = decay_cell(v.y, t.y, count_grid, 4 * i + 1, decay);
        v.z = decay_cell(v.z, t.z, count_grid, 4 * i + 2, decay);
        v.w = decay_cell(v.w, t.w, count_grid, 4 * i + 3, decay);
        g4[i] = v;
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (e[q] > 0.0f) {
                s += (double)e[q];
                ++k;
            }
    }
    s = block_sum(s, lds_d);
    k = block_sum(k, lds_u);
    if (threadIdx.x == 0) {
        st->sum[blockIdx.x] = s;
        st->count[blockIdx.x] = k;
    }
}

// thr = min(mean, threshold) with Python's min(): NaN mean (no positive cell) stays NaN.  One wave:
// the partials of nb <= DECAY_BLOCKS workgroups summed in a fixed lane / tree order.
// occ_thr_pack_kernel: thr + packbits in one launch (the refresh's form): every workgroup's first
// wave derives thr from the partials in that order, workgroup 0 also stores it, then the workgroup
// packs its bytes (the partials are 16 KB, L2-resident; <= 256 workgroups re-read them).
__global__ __launch_bounds__(256) void occ_thr_pack_kernel(OccStats* st, int nb, float threshold,
                                                           const float* __restrict__ grid, int64_t n_bytes,
                                                           uint8_t* __restrict__ bits) {
    __shared__ float thr_s;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        double s = 0.0;
        unsigned long long k = 0;
        for (int b = lane; b < nb; b += 64) { s += st->sum[b]; k += st->count[b]; }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            s += __shfl_xor(s, off, 64);
            k += __shfl_xor(k, off, 64);
        }
        if (lane == 0) {
            const float mean = k ? (float)(s / (double)k) : __builtin_nanf("");
            thr_s = (threshold < mean) ? threshold : mean;
            if (blockIdx.x == 0) st->thr = thr_s;
        }
    }
    __syncthreads();
    const float t = thr_s;
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < n_bytes; m += (int64_t)gridDim.x * blockDim.x) {
        const float4 a = reinterpret_cast<const float4*>(grid)[2 * m];
        const float4 b = reinterpret_cast<const float4*>(grid)[2 * m + 1];
        const uint32_t v = (a.x > t) | ((a.y > t) << 1) | ((a.z > t) << 2) | ((a.w > t) << 3) |
                           ((b.x > t) << 4) | ((b.y > t) << 5) | ((b.z > t) << 6) | ((b.w > t) << 7);
        bits[m] = (uint8_t)v;
    }
}

__global__ void occ_thr_kernel(OccStats* st, int nb, float threshold) {
    const int lane = threadIdx.x;
    double s = 0.0;
    unsigned long long k = 0;
    for (int b = lane; b < nb; b += 64) { s += st->sum[b]; k += st->count[b]; }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        s += __shfl_xor(s, off, 64);
        k += __shfl_xor(k, off, 64);
    }
    if (lane == 0) {
        const float mean = k ? (float)(s / (double)k) : __builtin_nanf("");
        st->thr = (threshold < mean) ? threshold : mean;
    }
}

int64_t blocks_for(int64_t n, int64_t cap = 8192) {
    const int64_t b = div_up<int64_t>(n, OCC_BLOCK);
    return b < 1 ? 1 : (b < cap ? b : cap);
}

struct Ws {
    int32_t* block_counts;
    int32_t* counts;
    int32_t* list;
    OccStats* stats;
    uint8_t* mark;        // the de-duplicated draw's byte map (zero between calls)
    int32_t* ulist;       // its distinct cells, ascending
    int32_t* ublock;      // marked cells per 4096-cell block
};
int64_t ws_layout(int cascades, int G, char* base, Ws* w) {
    const int64_t cells = (int64_t)G * G * G;
    const int64_t nblk = div_up<int64_t>(cells, OCC_CELLS_PER_BLOCK);
    int64_t off = 0;
    auto take = [&](int64_t bytes) { const int64_t o = off; off += (bytes + 255) / 256 * 256; return base + o; };
    char* bc = take(4 * cascades * nblk);
    char* ct = take(4 * cascades);
    char* ls = take(4 * cascades * cells);
    char* sp = take(sizeof(OccStats));
    char* mk = take(cascades * cells);
    char* ul = take(4 * cascades * cells);
    char* ub = take(4 * div_up<int64_t>(cascades * cells, OCC_CELLS_PER_BLOCK));
    if (w) {
        w->block_counts = (int32_t*)bc;
        w->counts = (int32_t*)ct;
        w->list = (int32_t*)ls;
        w->stats = (OccStats*)sp;
        w->mark = (uint8_t*)mk;
        w->ulist = (int32_t*)ul;
        w->ublock = (int32_t*)ub;
    }
    return off;
}

bool bad_grid(int cascades, int G) { return cascades < 1 || cascades > 16 || G < 1 || G > 1024 || ((int64_t)G * G * G) % 8; }

// the refresh's call index kept on the device (mfnerf_occupancy_cells_dev): one lane, a vector store
__global__ void occ_call_bump_kernel(uint64_t* call) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(call, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
int occupancy_cells_impl(const float* density_grid, int cascades, int grid_size, float scale, int64_t n_uniform,
                         int warmup, float density_threshold, uint64_t seed, uint64_t call_index, uint64_t* call_dev,
                         float* xyzs, int32_t* cell_idx, void* workspace, mfnerf_stream_t stream,
                         int32_t* unique_count = nullptr);

__global__ void occ_set_count_kernel(int32_t* count, int32_t v) {
    if (threadIdx.x == 0) *count = v;
}

}  // namespace

extern "C" {

int64_t mfnerf_occupancy_workspace(int cascades, int grid_size) {
    if (bad_grid(cascades, grid_size)) return -1;
    return ws_layout(cascades, grid_size, nullptr, nullptr);
}

int64_t mfnerf_occupancy_points(int cascades, int grid_size, int64_t n_uniform, int warmup) {
    if (bad_grid(cascades, grid_size) || n_uniform < 0) return -1;
    const int64_t cells = (int64_t)grid_size * grid_size * grid_size;
    return (int64_t)cascades * (warmup ? cells : 2 * n_uniform);
}

int mfnerf_occupancy_cells(const float* density_grid, int cascades, int grid_size, float scale, int64_t n_uniform,
                           int warmup, float density_threshold, uint64_t seed, uint64_t call_index, float* xyzs,
                           int32_t* cell_idx, void* workspace, mfnerf_stream_t stream) {
    return occupancy_cells_impl(density_grid, cascades, grid_size, scale, n_uniform, warmup, density_threshold, seed,
                                call_index, nullptr, xyzs, cell_idx, workspace, stream);
}

int64_t mfnerf_occupancy_points_unique(int cascades, int grid_size, int64_t n_uniform, int warmup) {
    const int64_t n = mfnerf_occupancy_points(cascades, grid_size, n_uniform, warmup);
    const int64_t cells = (int64_t)cascades * grid_size * grid_size * grid_size;
    return n < 0 ? -1 : (n < cells ? n : cells);
}

int mfnerf_occupancy_cells_unique(const float* density_grid, int cascades, int grid_size, float scale,
                                  int64_t n_uniform, int warmup, float density_threshold, uint64_t seed,
                                  uint64_t call_index, float* xyzs, int32_t* cell_idx, int32_t* count_dev,
                                  void* workspace, mfnerf_stream_t stream) {
    if (!count_dev) { mfn_set_error("occupancy_cells_unique: null count"); return MFN_ERR_INVALID; }
    return occupancy_cells_impl(density_grid, cascades, grid_size, scale, n_uniform, warmup, density_threshold, seed,
                                call_index, nullptr, xyzs, cell_idx, workspace, stream, count_dev);
}

int mfnerf_occupancy_cells_unique_dev(const float* density_grid, int cascades, int grid_size, float scale,
                                      int64_t n_uniform, int warmup, float density_threshold, uint64_t seed,
                                      uint64_t* call_index_dev, float* xyzs, int32_t* cell_idx, int32_t* count_dev,
                                      void* workspace, mfnerf_stream_t stream) {
    if (!call_index_dev || !count_dev) { mfn_set_error("occupancy_cells_unique_dev: null pointer"); return MFN_ERR_INVALID; }
    const int st = occupancy_cells_impl(density_grid, cascades, grid_size, scale, n_uniform, warmup, density_threshold,
                                        seed, 0, call_index_dev, xyzs, cell_idx, workspace, stream, count_dev);
    if (st) return st;
    if (warmup)  // (otherwise the marked-cell compaction advanced it)
        hipLaunchKernelGGL(occ_call_bump_kernel, dim3(1), dim3(64), 0, stream, call_index_dev);
    return mfn_check_launch("occupancy_cells_unique_dev");
}

int mfnerf_occupancy_cells_dev(const float* density_grid, int cascades, int grid_size, float scale, int64_t n_uniform,
                               int warmup, float density_threshold, uint64_t seed, uint64_t* call_index_dev,
                               float* xyzs, int32_t* cell_idx, void* workspace, mfnerf_stream_t stream) {
    if (!call_index_dev) { mfn_set_error("occupancy_cells_dev: null call index"); return MFN_ERR_INVALID; }
    const int st = occupancy_cells_impl(density_grid, cascades, grid_size, scale, n_uniform, warmup, density_threshold,
                                        seed, 0, call_index_dev, xyzs, cell_idx, workspace, stream);
    if (st) return st;
    hipLaunchKernelGGL(occ_call_bump_kernel, dim3(1), dim3(64), 0, stream, call_index_dev);
    return mfn_check_launch("occupancy_cells_dev");
}

}  // extern "C"

namespace {
int occupancy_cells_impl(const float* density_grid, int cascades, int grid_size, float scale, int64_t n_uniform,
                         int warmup, float density_threshold, uint64_t seed, uint64_t call_index, uint64_t* call_dev,
                         float* xyzs, int32_t* cell_idx, void* workspace, mfnerf_stream_t stream,
                         int32_t* unique_count) {
    if (bad_grid(cascades, grid_size)) { mfn_set_error("occupancy_cells: bad cascades/grid_size"); return MFN_ERR_INVALID; }
    if (n_uniform < 0 || (!warmup && n_uniform == 0)) { mfn_set_error("occupancy_cells: bad n_uniform"); return MFN_ERR_INVALID; }
    if (!density_grid || !xyzs || !cell_idx || !workspace) { mfn_set_error("occupancy_cells: null pointer"); return MFN_ERR_INVALID; }
    if (!(scale > 0.0f)) { mfn_set_error("occupancy_cells: scale must be > 0"); return MFN_ERR_INVALID; }
    Ws w;
    ws_layout(cascades, grid_size, (char*)workspace, &w);
    const int64_t cells = (int64_t)grid_size * grid_size * grid_size;
    const int64_t nblk = div_up<int64_t>(cells, OCC_CELLS_PER_BLOCK);
    if (!warmup) {
        hipLaunchKernelGGL(occ_count_kernel, dim3(nblk, cascades), dim3(OCC_BLOCK), 0, stream, density_grid, cells,
                           density_threshold, w.block_counts);
        hipLaunchKernelGGL(occ_compact_kernel, dim3(nblk, cascades), dim3(OCC_BLOCK), 0, stream, density_grid, cells,
                           density_threshold, w.block_counts, w.list, w.counts);
    }
    PointsArgs a;
    a.cascades = cascades;
    a.G = grid_size;
    a.cells = cells;
    a.per_cascade = warmup ? cells : 2 * n_uniform;
    a.n_uniform = warmup ? 0 : n_uniform;
    a.warmup = warmup ? 1 : 0;
    a.scale = scale;
    a.key = splitmix64_host(splitmix64_host(seed ^ OCC_SEED_MIX) ^ call_index);
    a.seed = seed;
    a.call_dev = call_dev;
    a.call_lag = 0;
    const int64_t n = (int64_t)cascades * a.per_cascade;
    if (unique_count && !warmup) {
        if (((int64_t)cascades * cells) % 16) {
            mfn_set_error("occupancy_cells_unique: cascades * grid_size^3 must be a multiple of 16");
            return MFN_ERR_INVALID;
        }
        // mark -> count -> compact (ascending, map re-zeroed) -> one point per distinct cell
        const int64_t total = (int64_t)cascades * cells, ub = div_up<int64_t>(total, OCC_CELLS_PER_BLOCK);
        hipLaunchKernelGGL(occ_mark_kernel, dim3(blocks_for(n)), dim3(OCC_BLOCK), 0, stream, a, w.list, w.counts, w.mark);
        hipLaunchKernelGGL(occ_mark_count_kernel, dim3(ub), dim3(OCC_BLOCK), 0, stream, w.mark, total, w.ublock);
        hipLaunchKernelGGL(occ_mark_compact_kernel, dim3(ub), dim3(OCC_BLOCK), 0, stream, w.mark, total, w.ublock, w.ulist,
                           unique_count, call_dev);
        if (call_dev) a.call_lag = 1;
        const int64_t cap = n < total ? n : total;
        hipLaunchKernelGGL(occ_unique_points_kernel, dim3(blocks_for(cap)), dim3(OCC_BLOCK), 0, stream, a, w.ulist,
                           unique_count, xyzs, cell_idx);
        return mfn_check_launch("occupancy_cells_unique");
    }
    hipLaunchKernelGGL(occ_points_kernel, dim3(blocks_for(n)), dim3(OCC_BLOCK), 0, stream, a, w.list, w.counts, xyzs,
                       cell_idx);
    if (unique_count)  // warm-up: every cell once already
        hipLaunchKernelGGL(occ_set_count_kernel, dim3(1), dim3(64), 0, stream, unique_count, (int32_t)n);
    return mfn_check_launch("occupancy_cells");
}
}  // namespace

extern "C" {

int mfnerf_occupancy_update(float* density_grid, const float* sigmas, const int32_t* cell_idx, int64_t n_points,
                            int cascades, int grid_size, float decay, const float* count_grid, float density_threshold,
                            float* tmp, uint8_t* bitfield, void* workspace, mfnerf_stream_t stream) {
    return mfnerf_occupancy_update_dev(density_grid, sigmas, cell_idx, n_points, nullptr, cascades, grid_size, decay,
                                       count_grid, density_threshold, tmp, 0, bitfield, workspace, stream);
}

int mfnerf_occupancy_update_dev(float* density_grid, const float* sigmas, const int32_t* cell_idx, int64_t n_points,
                                const int32_t* n_dev, int cascades, int grid_size, float decay, const float* count_grid,
                                float density_threshold, float* tmp, int tmp_zero, uint8_t* bitfield, void* workspace,
                                mfnerf_stream_t stream) {
    if (bad_grid(cascades, grid_size)) { mfn_set_error("occupancy_update: bad cascades/grid_size"); return MFN_ERR_INVALID; }
    if (n_points < 0) { mfn_set_error("occupancy_update: bad n_points"); return MFN_ERR_INVALID; }
    if (!density_grid || !tmp || !bitfield || !workspace || (n_points && (!sigmas || !cell_idx))) {
        mfn_set_error("occupancy_update: null pointer");
        return MFN_ERR_INVALID;
    }
    Ws w;
    ws_layout(cascades, grid_size, (char*)workspace, &w);
    const int64_t n = (int64_t)cascades * grid_size * grid_size * grid_size;
    if (((uintptr_t)density_grid) & 15) {
        mfn_set_error("occupancy_update: density grid must be 16-byte aligned");
        return MFN_ERR_INVALID;
    }
    if (!tmp_zero) mfn_zero_async(tmp, n * sizeof(float), stream);  // (tmp_zero: zero on entry already)
    if (n_points)
        hipLaunchKernelGGL(occ_scatter_kernel, dim3(blocks_for(n_points)), dim3(OCC_BLOCK), 0, stream, sigmas, cell_idx,
                           n_points, n_dev, tmp);
    const int nb = (int)blocks_for(n, DECAY_BLOCKS);  // every partial written (grid-stride beyond)
    hipLaunchKernelGGL(occ_decay_kernel, dim3(nb), dim3(OCC_BLOCK), 0, stream, density_grid, tmp, count_grid, n,
                       decay, w.stats, tmp_zero);
    const int64_t nbytes = n / 8, pb = blocks_for(nbytes, 256);
    hipLaunchKernelGGL(occ_thr_pack_kernel, dim3((unsigned)pb), dim3(256), 0, stream, w.stats, nb, density_threshold,
                       density_grid, nbytes, bitfield);
    return mfn_check_launch("occupancy_update");
}

}  // extern "C"
