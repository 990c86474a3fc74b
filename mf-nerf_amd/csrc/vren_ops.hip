// vren_ops.hip -- gfx950 kernels for the reference's `vren` op set (models/csrc/*.cu) and their
// C-ABI entry points (include/mfnerf.h).  Kernel arithmetic follows the reference statement by
// statement (see common.hpp for the fp contract); launch geometry and data flow are MI355X-first:
//   * ray-level kernels use 64-thread workgroups (one wave) so a 8192-ray batch spreads over 128
//     CUs instead of 32 workgroups of 256;
//   * raymarching_train is count -> one-workgroup prefix scan -> write, with the sample count kept
//     on the device (no host sync, graph-capturable) and rays_a in canonical ray order;
//   * compositing writes every sample of every ray exactly once (zeros after termination), so no
//     n_samples-sized memsets are needed; the backward's per-ray scan runs in registers.
#include "common.hpp"
#include "../../include/mfnerf.h"

using namespace mfn;

namespace {

constexpr int RAY_BLOCK = 64;

// ------------------------------------------------------------------ ray / AABB (intersection.cu:5-56)
__global__ void ray_aabb_kernel(const float* __restrict__ o, const float* __restrict__ d,
                                const float* __restrict__ centers, const float* __restrict__ half_sizes,
                                int64_t n_rays, int64_t n_vox, int max_hits, int32_t* __restrict__ hit_cnt,
                                float* __restrict__ hits_t, int64_t* __restrict__ hits_idx) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const float ox = o[3 * r], oy = o[3 * r + 1], oz = o[3 * r + 2];
    const float ix = 1.0f / d[3 * r], iy = 1.0f / d[3 * r + 1], iz = 1.0f / d[3 * r + 2];
    float* ht = hits_t + r * max_hits * 2;
    int64_t* hi = hits_idx + r * max_hits;
    for (int k = 0; k < max_hits; ++k) { ht[2 * k] = -1.0f; ht[2 * k + 1] = -1.0f; hi[k] = -1; }
    int cnt = 0;
    for (int64_t v = 0; v < n_vox; ++v) {
        const float cx = centers[3 * v], cy = centers[3 * v + 1], cz = centers[3 * v + 2];
        const float hx = half_sizes[3 * v], hy = half_sizes[3 * v + 1], hz = half_sizes[3 * v + 2];
        const float tminx = (cx - hx - ox) * ix, tminy = (cy - hy - oy) * iy, tminz = (cz - hz - oz) * iz;
        const float tmaxx = (cx + hx - ox) * ix, tmaxy = (cy + hy - oy) * iy, tmaxz = (cz + hz - oz) * iz;
        float t1 = fmaxf(fmaxf(fminf(tminx, tmaxx), fminf(tminy, tmaxy)), fminf(tminz, tmaxz));
        float t2 = fminf(fminf(fmaxf(tminx, tmaxx), fmaxf(tminy, tmaxy)), fmaxf(tminz, tmaxz));
        if (t1 > t2) { t1 = -1.0f; t2 = -1.0f; }
        if (t2 > 0) {
            if (cnt < max_hits) { ht[2 * cnt] = fmaxf(t1, 0.0f); ht[2 * cnt + 1] = t2; hi[cnt] = v; }
            cnt++;
        }
    }
    hit_cnt[r] = cnt;
    // the reference sorts all max_hits slots by t1 (intersection.cu:95-97): unfilled slots (t1=-1)
    // come first, then the real hits ascending.  Insertion sort of the k real hits, then shift right.
    const int k = min(cnt, max_hits);
    for (int i = 1; i < k; ++i) {
        const float a = ht[2 * i], b = ht[2 * i + 1]; const int64_t c = hi[i];
        int j = i - 1;
        while (j >= 0 && ht[2 * j] > a) { ht[2 * j + 2] = ht[2 * j]; ht[2 * j + 3] = ht[2 * j + 1]; hi[j + 1] = hi[j]; --j; }
        ht[2 * j + 2] = a; ht[2 * j + 3] = b; hi[j + 1] = c;
    }
    const int sh = max_hits - k;
    if (sh > 0 && k > 0) {
        for (int i = k - 1; i >= 0; --i) {
            ht[2 * (i + sh)] = ht[2 * i]; ht[2 * (i + sh) + 1] = ht[2 * i + 1]; hi[i + sh] = hi[i];
        }
        for (int i = 0; i < sh; ++i) { ht[2 * i] = -1.0f; ht[2 * i + 1] = -1.0f; hi[i] = -1; }
    }
}

// ------------------------------------------------------------------ morton / packbits (raymarching.cu:62-161)
__global__ void morton_kernel(const int32_t* __restrict__ c, int64_t n, int32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = (int32_t)morton3((uint32_t)c[3 * i], (uint32_t)c[3 * i + 1], (uint32_t)c[3 * i + 2]);
}

__global__ void morton_invert_kernel(const int32_t* __restrict__ idx, int64_t n, int32_t* __restrict__ c) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = (uint32_t)idx[i];
    c[3 * i] = (int32_t)morton3_invert(v);
    c[3 * i + 1] = (int32_t)morton3_invert(v >> 1);
    c[3 * i + 2] = (int32_t)morton3_invert(v >> 2);
}

// one thread per output byte: two 16-B loads of the 8 floats, one byte store
__global__ void packbits_kernel(const float* __restrict__ grid, int64_t n_bytes, float thr,
                                const float* __restrict__ thr_dev, uint8_t* __restrict__ bits) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_bytes) return;
    const float t = thr_dev ? *thr_dev : thr;
    const float4 a = reinterpret_cast<const float4*>(grid)[2 * n];
    const float4 b = reinterpret_cast<const float4*>(grid)[2 * n + 1];
    uint32_t v = (a.x > t) | ((a.y > t) << 1) | ((a.z > t) << 2) | ((a.w > t) << 3) |
                 ((b.x > t) << 4) | ((b.y > t) << 5) | ((b.z > t) << 6) | ((b.w > t) << 7);
    bits[n] = (uint8_t)v;
}

// ------------------------------------------------------------------ ray marching (raymarching.cu:166-454)
struct MarchParams {
    const float* o; const float* d; const float* hits_t; int64_t hits_stride;
    const uint8_t* bitfield; int cascades; float scale; float exp_step; const float* noise;
    int grid_size; int max_samples;
};

// Marches ray r (raymarching.cu:190-234 / :243-279).  WRITE=false counts (up to max_samples);
// WRITE=true re-marches and stores the first `limit` samples at `base`.
template <bool WRITE>
__device__ __forceinline__ int march_ray(const MarchParams& p, int64_t r, int limit, int64_t base,
                                         float* __restrict__ xyzs, float* __restrict__ dirs,
                                         float* __restrict__ deltas, float* __restrict__ ts) {
    const float gsi = 1.0f / (float)p.grid_size;
    const float ox = p.o[3 * r], oy = p.o[3 * r + 1], oz = p.o[3 * r + 2];
    const float dx = p.d[3 * r], dy = p.d[3 * r + 1], dz = p.d[3 * r + 2];
    const float dxi = 1.0f / dx, dyi = 1.0f / dy, dzi = 1.0f / dz;
    float t1 = p.hits_t[r * p.hits_stride], t2 = p.hits_t[r * p.hits_stride + 1];
    if (t1 >= 0) {
        const float dt = calc_dt(t1, p.exp_step, p.max_samples, p.grid_size, p.scale);
        t1 = fmaf(dt, p.noise[r], t1);
    }
    float t = t1; int n = 0;
    while (0 <= t && t < t2 && n < limit) {
        const float x = fmaf(t, dx, ox), y = fmaf(t, dy, oy), z = fmaf(t, dz, oz);
        const float dt = calc_dt(t, p.exp_step, p.max_samples, p.grid_size, p.scale);
        const Cell c = lookup_cell(x, y, z, dt, p.cascades, p.grid_size, p.scale, p.bitfield);
        if (c.occ) {
            if (WRITE) {
                const int64_t s = base + n;
                xyzs[3 * s] = x; xyzs[3 * s + 1] = y; xyzs[3 * s + 2] = z;
                dirs[3 * s] = dx; dirs[3 * s + 1] = dy; dirs[3 * s + 2] = dz;
                ts[s] = t; deltas[s] = dt;
            }
            t += dt; n++;
        } else {
            const float tt = skip_target(t, c, x, y, z, dx, dy, dz, dxi, dyi, dzi, gsi);
            do { t += calc_dt(t, p.exp_step, p.max_samples, p.grid_size, p.scale); } while (t < tt);
        }
    }
    return n;
}

__global__ void march_count_kernel(MarchParams p, int64_t n_rays, int32_t* __restrict__ counts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    counts[r] = march_ray<false>(p, r, p.max_samples, 0, nullptr, nullptr, nullptr, nullptr);
}

// One-workgroup exclusive scan of the per-ray counts -> rays_a rows and counter (device resident).
// It runs on the side stream beside the table-gradient scatter, whose 1024-thread workgroups hold 4
// waves x 112 VGPRs of every SIMD: 64 VGPRs per SIMD lane stay free, room for ONE more wave of <= 64
// registers per SIMD.  So 256 threads (one wave per SIMD) at <= 64 VGPRs: the 512-thread form (two
// waves per SIMD) found no CU until the scatter ended -- 84 us in the step timeline
// (profiles/r05_v5_march_estimate_timeline.txt) for a few microseconds of work.
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_K = 16;  // counts per thread loaded together
__global__ __launch_bounds__(SCAN_THREADS) __attribute__((amdgpu_waves_per_eu(8))) void march_scan_kernel(
    const int32_t* __restrict__ counts, int64_t n_rays, int64_t capacity, int64_t* __restrict__ rays_a,
    int32_t* __restrict__ counter) {
    __shared__ int64_t wave_tot[SCAN_THREADS / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int n = (int)n_rays;  // (<= 2^31: checked by the caller)
    const int chunk = (n + SCAN_THREADS - 1) / SCAN_THREADS;
    const int b = tid * chunk, e = min(n, b + chunk);
    // SCAN_K counts per thread in flight together: one memory round trip per SCAN_K instead of chunk
    // dependent ones (beside the scatter every load waits behind its traffic)
    int64_t local = 0;
    for (int b0 = b; b0 < e; b0 += SCAN_K) {
        int32_t cr[SCAN_K];
#pragma unroll
        for (int k = 0; k < SCAN_K; ++k) cr[k] = counts[b0 + k < e ? b0 + k : 0];
#pragma unroll
        for (int k = 0; k < SCAN_K; ++k) local += b0 + k < e ? cr[k] : 0;
    }
    // inclusive wave scan
    int64_t v = local;
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t u = __shfl_up(v, off, 64);
        if (lane >= off) v += u;
    }
    if (lane == 63) wave_tot[wid] = v;
    __syncthreads();
    if (wid == 0) {
        int64_t w = lane < SCAN_THREADS / 64 ? wave_tot[lane] : 0;
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t u = __shfl_up(w, off, 64);
            if (lane >= off) w += u;
        }
        if (lane < SCAN_THREADS / 64) wave_tot[lane] = w;  // inclusive per-wave totals
    }
    __syncthreads();
    int64_t run = (v - local) + (wid > 0 ? wave_tot[wid - 1] : 0);  // exclusive start of this chunk
    // the write pass re-reads the counts (cache hits now), SCAN_K at a time again, rather than keep
    // them live through the scan: the kernel must stay within 64 registers
    for (int b0 = b; b0 < e; b0 += SCAN_K) {
        int32_t cr[SCAN_K];
#pragma unroll
        for (int k = 0; k < SCAN_K; ++k) cr[k] = counts[b0 + k < e ? b0 + k : 0];
        for (int k = 0; k < SCAN_K && b0 + k < e; ++k) {
            const int64_t i = b0 + k, c = cr[k];
            rays_a[3 * i] = i;
            rays_a[3 * i + 1] = min(run, capacity);
            rays_a[3 * i + 2] = max<int64_t>(0, min(c, capacity - run));
            run += c;
        }
    }
    if (tid == SCAN_THREADS - 1) {
        counter[0] = (int32_t)min(run, capacity);
        counter[1] = (int32_t)n_rays;
    }
}

__global__ void march_write_kernel(MarchParams p, int64_t n_rays, const int64_t* __restrict__ rays_a,
                                   float* __restrict__ xyzs, float* __restrict__ dirs, float* __restrict__ deltas,
                                   float* __restrict__ ts) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rays) return;
    const int limit = (int)rays_a[3 * r + 2];
    if (limit == 0) return;
    march_ray<true>(p, r, limit, rays_a[3 * r + 1], xyzs, dirs, deltas, ts);
}

// ---- wave-per-ray marching for constant dt (exp_step_factor == 0: every synthetic scene).
// One wave marches one ray 64 chain points at a time.  The chain t_{k+1} = fl(t_k + dt) that both
// reference branches walk (raymarching.cu:223,230-232) is laid on the lanes in closed form,
// t_j = fmaf(j, delta, t_base) with delta = fl(t_base+dt) - t_base, and every lane checks
// fl(t_j + dt) == t_{j+1}: the chunk is truncated at the first mismatch (binade crossing, tie), so
// the lane values ARE the sequential chain.  Each live lane looks up its cell; a scalar walk over
// the lanes then replays the reference's control flow exactly (occupied: emit and step; empty:
// jump to the first chain point >= the DDA target), and the emitted lanes are compacted with a
// ballot prefix count.  Bit-identical to march_ray<> (and the oracle), ~64x more parallel.
// The march runs ONCE: it counts the ray's samples and keeps their t values at tbuf[r * max_samples
// + j]; after the scan, march_expand_kernel writes the compacted samples from them (x = fmaf(t, d, o)
// as here, the ray's direction, t, the constant dt).  Until round 3 a second march re-walked every
// ray to write (count + re-march ~250 us on the side stream, beside the table-gradient scatter).
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int ffs64(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }

// One chunk of the chain on the lanes: its points, where the successor chain breaks, the next chunk's
// base, and each live lane's cell with its bitfield byte requested (chunk_occ reads it later).
struct MarchChunk {
    float t_base, tl, x, y, z, next_base;
    int chain_end;
    bool live;
    Cell c;
    uint32_t bit;      // bit of the cell in its byte
    uint32_t byte;     // the bitfield byte (in flight until chunk_occ)
};

__device__ __forceinline__ MarchChunk march_chunk(const MarchParams& p, float t_base, float dt, float t2, float ox,
                                                  float oy, float oz, float dx, float dy, float dz, int lane,
                                                  float inv_scale) {
    MarchChunk k;
    k.t_base = t_base;
    const float delta = (t_base + dt) - t_base;
    k.tl = fmaf((float)lane, delta, t_base);
    const float succ = k.tl + dt;
    const float tl_next = __shfl_down(k.tl, 1, 64);
    const uint64_t bad = __ballot(lane < 63 && succ != tl_next);
    k.chain_end = bad ? ffs64(bad) + 1 : 64;
    k.next_base = readlane_f(succ, k.chain_end - 1);
    k.live = lane < k.chain_end && k.tl < t2;
    k.x = fmaf(k.tl, dx, ox); k.y = fmaf(k.tl, dy, oy); k.z = fmaf(k.tl, dz, oz);
    // lookup_cell's arithmetic on every lane (branch-free: a load under a lane condition makes the
    // compiler wait for every outstanding load where the paths join, i.e. for this prefetch), the
    // byte load issued here and used a chunk later; a lane past the chain reads byte 0
    const uint32_t g3 = (uint32_t)p.grid_size * p.grid_size * p.grid_size;
    const int mip = max(mip_from_pos(k.x, k.y, k.z, p.cascades), mip_from_dt(dt, p.grid_size, p.cascades));
    k.c.mip_bound = fminf(scalbnf(1.0f, mip - 1), p.scale);
    // lookup_cell's 1 / mip_bound without a per-lane IEEE division: 2^(1-mip) is exact, and 1/scale
    // is the same correctly rounded quotient computed once (inv_scale)
    const float inv = k.c.mip_bound == p.scale ? inv_scale : scalbnf(1.0f, 1 - mip);
    const float gs = (float)p.grid_size, gm1 = (float)p.grid_size - 1.0f;
    k.c.nx = (int)clampf(0.5f * fmaf(k.x, inv, 1.0f) * gs, 0.0f, gm1);
    k.c.ny = (int)clampf(0.5f * fmaf(k.y, inv, 1.0f) * gs, 0.0f, gm1);
    k.c.nz = (int)clampf(0.5f * fmaf(k.z, inv, 1.0f) * gs, 0.0f, gm1);
    const uint32_t idx = (uint32_t)mip * g3 + morton3((uint32_t)k.c.nx, (uint32_t)k.c.ny, (uint32_t)k.c.nz);
    k.bit = idx & 7;
    k.byte = p.bitfield[k.live ? idx >> 3 : 0u];
    return k;
}

__device__ __forceinline__ void march_wave_ray(const MarchParams& p, int64_t r, int32_t* __restrict__ counts,
                                               float* __restrict__ tbuf) {
    const int lane = threadIdx.x & 63;
    const int limit = p.max_samples;
    float* tr = tbuf + r * (int64_t)p.max_samples;
    const float gsi = 1.0f / (float)p.grid_size;
    const float ox = p.o[3 * r], oy = p.o[3 * r + 1], oz = p.o[3 * r + 2];
    const float dx = p.d[3 * r], dy = p.d[3 * r + 1], dz = p.d[3 * r + 2];
    const float dxi = 1.0f / dx, dyi = 1.0f / dy, dzi = 1.0f / dz;
    float t1 = p.hits_t[r * p.hits_stride];
    const float t2 = p.hits_t[r * p.hits_stride + 1];
    int n = 0;
    if (t1 >= 0) {
        const float dt = calc_dt(t1, p.exp_step, p.max_samples, p.grid_size, p.scale);  // constant
        t1 = fmaf(dt, p.noise[r], t1);
        float t_base = t1, pending = 0.0f;
        bool skip = false, done = false;
        // round 5: the next chunk's points are pure arithmetic (the chain does not depend on the
        // walk), so its bitfield bytes are requested before this chunk's walk -- one memory round trip
        // hidden per chunk (the march runs beside the table-gradient scatter, where every load waits
        // behind its traffic)
        const float inv_scale = 1 / p.scale;
        MarchChunk cur = march_chunk(p, t_base, dt, t2, ox, oy, oz, dx, dy, dz, lane, inv_scale);
        while (!done) {
            if (!(t_base < t2) || n >= limit) break;  // every later visited point fails the loop test
            const MarchChunk nxt = march_chunk(p, cur.next_base, dt, t2, ox, oy, oz, dx, dy, dz, lane, inv_scale);
            const float tl = cur.tl;
            const int chain_end = cur.chain_end;
            const bool live = cur.live;
            const bool occ = live && ((cur.byte >> cur.bit) & 1u);
            const float tt = live && !occ ? skip_target(tl, cur.c, cur.x, cur.y, cur.z, dx, dy, dz, dxi, dyi, dzi, gsi)
                                          : 0.0f;
            const uint64_t live_m = __ballot(live), occ_m = __ballot(occ);
            const uint64_t chain_m = chain_end == 64 ? ~0ull : ((1ull << chain_end) - 1);
            // Round 5: the empty cells' DDA jumps resolved on the lanes instead of one scalar walk step
            // per empty cell (PMC: 27.8 M SALU vs 12.6 M VALU instructions, issue-blocked 50 % -- the
            // march was bound by its scalar walk).  Empty live lane j jumps to J(j) = the first chain
            // lane k > j with tl_k >= tt_j (tl_k = fmaf(k, delta, t_base) is monotone in k: a binary
            // search over the closed form, no lookups), or OUT (64) past the chunk.  Pointer doubling
            // over those jumps (occupied and non-live lanes stop) gives every lane the lane the walk
            // lands on from it, and the lane whose jump leaves the chunk (its target becomes the next
            // chunk's pending skip).  The scalar walk then steps once per occupied run instead of once
            // per empty cell.  The visited set -- hence counts, samples, order -- is the walk's own.
            constexpr int OUT = 64;
            int P = lane, L = -1;
            if (live && !occ) {
                // first k in [0, chain_end) with tl_k >= tt (chain_end: none).  Inside the verified
                // chain tl_k = t_base + k delta exactly, so k = ceil((tt - t_base) / delta); the
                // estimate (approximate reciprocal: off by far less than a lane) is put right by one
                // exact comparison each way
                const float delta = (cur.t_base + dt) - cur.t_base;
                const float est = (tt - cur.t_base) * __builtin_amdgcn_rcpf(delta);
                int k = tt == tt ? (int)ceilf(fminf(fmaxf(est, 0.0f), (float)chain_end)) : chain_end;
                if (k > 0 && fmaf((float)(k - 1), delta, cur.t_base) >= tt) --k;
                if (k < chain_end && !(fmaf((float)k, delta, cur.t_base) >= tt)) ++k;
                const int J = max(k, lane + 1);
                P = J < chain_end ? J : OUT;
                L = J < chain_end ? -1 : lane;
            }
#pragma unroll
            for (int it = 0; it < 6; ++it) {
                const int q = min(P, 63);
                const int Pq = __shfl(P, q, 64), Lq = __shfl(L, q, 64);
                if (P < OUT) { P = Pq; L = Lq; }
            }
            uint64_t emit_m = 0;
            const int n0 = n;
            int c = 0;
            if (skip) {
                const uint64_t ge = __ballot(tl >= pending) & chain_m;
                if (ge) { c = ffs64(ge); skip = false; } else c = chain_end;
            }
            while (c < chain_end) {
                const int s = __builtin_amdgcn_readlane(P, c);  // (c itself when occupied or not live)
                if (s >= OUT) {
                    skip = true;
                    pending = readlane_f(tt, __builtin_amdgcn_readlane(L, c));
                    break;
                }
                c = s;
                if (!((live_m >> c) & 1) || n >= limit) { done = true; break; }
                const uint64_t rest = ~(occ_m >> c);  // (lane c is occupied)
                int len = rest ? ffs64(rest) : 64 - c;
                len = min(len, limit - n);
                emit_m |= (len >= 64 ? ~0ull : ((1ull << len) - 1)) << c;
                n += len; c += len;
            }
            if ((emit_m >> lane) & 1) tr[n0 + __popcll(emit_m & ((1ull << lane) - 1))] = tl;
            t_base = cur.next_base;
            cur = nxt;
        }
    }
    if (lane == 0) counts[r] = n;
}

// one ray per wave per trip; a wave takes rays w, w + W, ... (W = the grid's waves)
__global__ __launch_bounds__(256) void march_wave_kernel(MarchParams p, int64_t n_rays, int32_t* __restrict__ counts,
                                                         float* __restrict__ tbuf) {
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n_rays; r += nw)  // wave-uniform
        march_wave_ray(p, r, counts, tbuf);
}


// The compacted samples of ray r (one wave): its first rays_a[r].count t values from march_wave.
// <= 64 VGPRs (waves_per_eu(8)): the kernel follows the scan beside the scatter, which leaves 64
// registers per SIMD lane free (see march_scan_kernel); at 68 it waited for the scatter to end and ran
// beside the accumulate instead.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void march_expand_kernel(MarchParams p, int64_t n_rays,
                                                           const int64_t* __restrict__ rays_a,
                                                           const float* __restrict__ tbuf, float* __restrict__ xyzs,
                                                           float* __restrict__ dirs, float* __restrict__ deltas,
                                                           float* __restrict__ ts) {
    const int lane = threadIdx.x & 63;
    const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (r >= n_rays) return;  // wave-uniform
    const int cnt = (int)rays_a[3 * r + 2];
    if (cnt == 0) return;
    const int64_t base = rays_a[3 * r + 1];
    const float ox = p.o[3 * r], oy = p.o[3 * r + 1], oz = p.o[3 * r + 2];
    const float dx = p.d[3 * r], dy = p.d[3 * r + 1], dz = p.d[3 * r + 2];
    // march_wave's constant step, from the same un-perturbed entry point
    const float dt = calc_dt(p.hits_t[r * p.hits_stride], p.exp_step, p.max_samples, p.grid_size, p.scale);
    const float* tr = tbuf + r * (int64_t)p.max_samples;
    for (int j = lane; j < cnt; j += 64) {
        const float t = tr[j];
        const int64_t s = base + j;
        xyzs[3 * s] = fmaf(t, dx, ox); xyzs[3 * s + 1] = fmaf(t, dy, oy); xyzs[3 * s + 2] = fmaf(t, dz, oz);
        dirs[3 * s] = dx; dirs[3 * s + 1] = dy; dirs[3 * s + 2] = dz;
        ts[s] = t; deltas[s] = dt;
    }
}

// raymarching_test_kernel (raymarching.cu:335-404) with the calc_dt(..., cascades) quirk.
__global__ void march_test_kernel(MarchParams p, float* __restrict__ hits_t, const int64_t* __restrict__ alive,
                                  int64_t n_alive, int N_samples, float* __restrict__ xyzs, float* __restrict__ dirs,
                                  float* __restrict__ deltas, float* __restrict__ ts, int32_t* __restrict__ n_eff) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    const int64_t r = alive[n];
    const float gsi = 1.0f / (float)p.grid_size;
    const float qscale = (float)p.cascades;  // the reference's quirk: cascades passed as `scale`
    const float ox = p.o[3 * r], oy = p.o[3 * r + 1], oz = p.o[3 * r + 2];
    const float dx = p.d[3 * r], dy = p.d[3 * r + 1], dz = p.d[3 * r + 2];
    const float dxi = 1.0f / dx, dyi = 1.0f / dy, dzi = 1.0f / dz;
    float t = hits_t[r * p.hits_stride], t2 = hits_t[r * p.hits_stride + 1];
    const int64_t row = n * N_samples;
    int s = 0;
    while (t < t2 && s < N_samples) {
        const float x = fmaf(t, dx, ox), y = fmaf(t, dy, oy), z = fmaf(t, dz, oz);
        const float dt = calc_dt(t, p.exp_step, p.max_samples, p.grid_size, qscale);
        const Cell c = lookup_cell(x, y, z, dt, p.cascades, p.grid_size, p.scale, p.bitfield);
        if (c.occ) {
            const int64_t k = row + s;
            xyzs[3 * k] = x; xyzs[3 * k + 1] = y; xyzs[3 * k + 2] = z;
            dirs[3 * k] = dx; dirs[3 * k + 1] = dy; dirs[3 * k + 2] = dz;
            ts[k] = t; deltas[k] = dt;
            t += dt;
            hits_t[r * p.hits_stride] = t;
            s++;
        } else {
            const float tt = skip_target(t, c, x, y, z, dx, dy, dz, dxi, dyi, dzi, gsi);
            do { t += calc_dt(t, p.exp_step, p.max_samples, p.grid_size, qscale); } while (t < tt);
        }
    }
    for (int k = s; k < N_samples; ++k) {  // zero the unused tail of this row (the reference zero-fills)
        const int64_t q = row + k;
        xyzs[3 * q] = 0.f; xyzs[3 * q + 1] = 0.f; xyzs[3 * q + 2] = 0.f;
        dirs[3 * q] = 0.f; dirs[3 * q + 1] = 0.f; dirs[3 * q + 2] = 0.f;
        ts[q] = 0.f; deltas[q] = 0.f;
    }
    n_eff[n] = s;
}

// ------------------------------------------------------------------ compositing (volumerendering.cu)
// ---- wave-per-ray compositing (volumerendering.cu:6-45 / :87-151).  One wave per ray, lanes =
// samples (coalesced loads/stores, 64 samples per chunk).  The transmittance chain T *= 1-a is
// evaluated in the reference's sequential order by a uniform loop over the lanes (bit-identical
// T, hence identical termination and total_samples); the rgb/depth/opacity sums and the backward's
// prefix sums are wave reductions/scans (fp32 reassociation only, ~1e-7 relative).
// Wave scans and sums on the DPP network: row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry the row totals -- a few cycles per step, where each __shfl step
// is an LDS-routed ds_bpermute with ~100 cycles of latency (this path runs one wave per ray).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_src(float v) {
    // lanes outside ROW_MASK, or without a source lane, read 0
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ float wave_incl_scan(float v, int lane) {
    (void)lane;
    v += dpp_src<0x111, 0xF>(v);  // row_shr:1
    v += dpp_src<0x112, 0xF>(v);  // row_shr:2
    v += dpp_src<0x114, 0xF>(v);  // row_shr:4
    v += dpp_src<0x118, 0xF>(v);  // row_shr:8
    v += dpp_src<0x142, 0xA>(v);  // row_bcast:15 -> rows 1 and 3
    v += dpp_src<0x143, 0xC>(v);  // row_bcast:31 -> rows 2 and 3
    return v;
}
__device__ __forceinline__ float wave_sum(float v) { return readlane_f(wave_incl_scan(v, 0), 63); }

// Sequential T over the chunk: returns this lane's T before its sample; T_run is advanced; *stop is
// the first lane whose post-update T <= thr (64 if none).  The reference's order is kept exactly:
// T_j = fl(T_{j-1} * fl(1 - a_{j-1})), so T, termination and total_samples are bit-identical to its
// sequential loop.  The chain is propagated one lane per step with a whole-wave DPP shift
// (wave_shr:1): after k steps lanes 0..k hold their final T, so n_valid-1 steps of one shifted
// multiply replace n_valid serial readlane/multiply/compare/branch rounds -- the long rays' chains
// (hundreds of samples) were this kernel's critical path.
__device__ __forceinline__ float t_chain(float a, float& T_run, float thr, int lane, int n_valid, int* stop) {
    constexpr int WAVE_SHR1 = 0x138;
    const float b = 1.0f - a;  // lanes past n_valid: a = 0, b = 1
    // bs[j] = b[j-1], bs[0] = 1 (T_0 = T_run * 1 exactly)
    const float bs = __int_as_float(
        __builtin_amdgcn_update_dpp(__float_as_int(1.0f), __float_as_int(b), WAVE_SHR1, 0xF, 0xF, false));
    const int t0 = __float_as_int(T_run);
    float X = T_run;
    const int nv = __builtin_amdgcn_readfirstlane(n_valid);  // wave-uniform: a scalar loop
    for (int k = 1; k < nv; ++k)
        X = __int_as_float(__builtin_amdgcn_update_dpp(t0, __float_as_int(X), WAVE_SHR1, 0xF, 0xF, false)) * bs;
    const float Ta = X * b;  // T after this lane's sample
    const uint64_t hit = __ballot(lane < n_valid && Ta <= thr);
    const int st = hit ? (int)__builtin_ctzll(hit) : 64;
    T_run = readlane_f(Ta, st < 64 ? st : n_valid - 1);
    *stop = st;
    return X;
}

__global__ __launch_bounds__(256) void composite_fw_wave_kernel(
    const float* __restrict__ sigmas, const float* __restrict__ rgbs, const float* __restrict__ deltas,
    const float* __restrict__ ts, const int64_t* __restrict__ rays_a, int64_t n_rays, float T_thr,
    int64_t* __restrict__ total_samples, float* __restrict__ opacity, float* __restrict__ depth,
    float* __restrict__ rgb, float* __restrict__ ws) {
    const int lane = threadIdx.x & 63;
    const int64_t n = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (n >= n_rays) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    float T = 1.0f, R = 0.f, G = 0.f, B = 0.f, D = 0.f, O = 0.f;
    int total = N;
    bool ended = false;
    for (int k0 = 0; k0 < N; k0 += 64) {
        const int nv = min(64, N - k0);
        const int64_t s = start + k0 + lane;
        const bool valid = lane < nv;
        float w = 0.0f;
        if (!ended) {
            const float a = valid ? 1.0f - fast_exp(-sigmas[s] * deltas[s]) : 0.0f;
            int stop;
            const float myT = t_chain(a, T, T_thr, lane, nv, &stop);
            if (valid && lane <= stop) {
                w = a * myT;
                R = fmaf(w, rgbs[3 * s], R); G = fmaf(w, rgbs[3 * s + 1], G); B = fmaf(w, rgbs[3 * s + 2], B);
                D = fmaf(w, ts[s], D);
                O += w;
            }
            if (stop < 64) { ended = true; total = k0 + stop; }
        }
        if (valid) ws[s] = w;
    }
    R = wave_sum(R); G = wave_sum(G); B = wave_sum(B); D = wave_sum(D); O = wave_sum(O);
    if (lane == 0) {
        opacity[ray] = O; depth[ray] = D;
        rgb[3 * ray] = R; rgb[3 * ray + 1] = G; rgb[3 * ray + 2] = B;
        total_samples[ray] = total;
    }
}

__global__ __launch_bounds__(256) void composite_bw_wave_kernel(
    const float* __restrict__ dL_dopacity, const float* __restrict__ dL_ddepth, const float* __restrict__ dL_drgb,
    const float* __restrict__ dL_dws, const float* __restrict__ sigmas, const float* __restrict__ rgbs,
    const float* __restrict__ ws, const float* __restrict__ deltas, const float* __restrict__ ts,
    const int64_t* __restrict__ rays_a, const float* __restrict__ opacity, const float* __restrict__ depth,
    const float* __restrict__ rgb, int64_t n_rays, float T_thr, float* __restrict__ dL_dsigmas,
    float* __restrict__ dL_drgbs) {
    const int lane = threadIdx.x & 63;
    const int64_t n = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (n >= n_rays) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    if (N <= 0) return;
    // total of dL_dws*ws over the whole ray (the inclusive scan's last element)
    float wsum = 0.0f;
    for (int k0 = 0; k0 < N; k0 += 64) {
        const int64_t s = start + k0 + lane;
        if (k0 + lane < N) wsum += dL_dws[s] * ws[s];
    }
    wsum = wave_sum(wsum);
    const float Rt = rgb[3 * ray], Gt = rgb[3 * ray + 1], Bt = rgb[3 * ray + 2];
    const float O = opacity[ray], Dt = depth[ray];
    const float gr = dL_drgb[3 * ray], gg = dL_drgb[3 * ray + 1], gb = dL_drgb[3 * ray + 2];
    const float go = dL_dopacity[ray], gd = dL_ddepth[ray];
    float T = 1.0f, cr = 0.f, cg = 0.f, cb = 0.f, cd = 0.f, cs = 0.f;  // carries of the prefix sums
    bool ended = false;
    for (int k0 = 0; k0 < N; k0 += 64) {
        const int nv = min(64, N - k0);
        const int64_t s = start + k0 + lane;
        const bool valid = lane < nv;
        float dsig = 0.0f, d0 = 0.0f, d1 = 0.0f, d2 = 0.0f;
        if (!ended) {
            float sg = 0.f, dl = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, tv = 0.f, dw = 0.f, wv = 0.f;
            if (valid) {
                sg = sigmas[s]; dl = deltas[s]; tv = ts[s]; dw = dL_dws[s]; wv = ws[s];
                c0 = rgbs[3 * s]; c1 = rgbs[3 * s + 1]; c2 = rgbs[3 * s + 2];
            }
            const float a = valid ? 1.0f - fast_exp(-sg * dl) : 0.0f;
            int stop;
            const float myT = t_chain(a, T, T_thr, lane, nv, &stop);
            const bool act = valid && lane <= stop;
            const float w = act ? a * myT : 0.0f;
            const float Tn = myT * (1.0f - a);  // T after this sample (the reference's updated T)
            const float pr = wave_incl_scan(w * c0, lane) + cr, pg = wave_incl_scan(w * c1, lane) + cg;
            const float pb = wave_incl_scan(w * c2, lane) + cb, pd = wave_incl_scan(w * tv, lane) + cd;
            const float ps = wave_incl_scan(act ? dw * wv : 0.0f, lane) + cs;
            cr = readlane_f(pr, 63); cg = readlane_f(pg, 63); cb = readlane_f(pb, 63); cd = readlane_f(pd, 63);
            cs = readlane_f(ps, 63);
            if (act) {
                d0 = gr * w; d1 = gg * w; d2 = gb * w;
                float acc = gr * fmaf(c0, Tn, -(Rt - pr));
                acc = fmaf(gg, fmaf(c1, Tn, -(Gt - pg)), acc);
                acc = fmaf(gb, fmaf(c2, Tn, -(Bt - pb)), acc);
                acc = fmaf(go, 1 - O, acc);
                acc = fmaf(gd, fmaf(tv, Tn, -(Dt - pd)), acc);
                acc = fmaf(Tn, dw, acc);
                acc = acc - (wsum - ps);
                dsig = dl * acc;
            }
            if (stop < 64) ended = true;
        }
        if (valid) {
            dL_dsigmas[s] = dsig;
            dL_drgbs[3 * s] = d0; dL_drgbs[3 * s + 1] = d1; dL_drgbs[3 * s + 2] = d2;
        }
    }
}

// Fused training compositing for the default loss (no distortion term): composite_train_fw ->
// background blend + NeRFLoss and its gradient -> composite_train_bw with dL/ddepth = 0 and
// dL/dws = 0, one wave per ray, one launch.  Pass 1 is composite_fw_wave_kernel's loop and also
// stores each sample's post-sample transmittance into dL_dsigmas (as scratch); pass 2 reads w and
// T back (same lane, same address) instead of re-walking the transmittance chain, so the result is
// bit-identical to the three separate kernels (the dropped terms are exact zeros).  The loss value
// is written as one partial sum per workgroup of 4 rays (plain stores: no zeroing, no atomics).

__global__ __launch_bounds__(256) void composite_fused_wave_kernel(
    const float* __restrict__ sigmas, const float* __restrict__ rgbs, const float* __restrict__ deltas,
    const float* __restrict__ ts, const int64_t* __restrict__ rays_a, int64_t n_rays, float T_thr,
    const float* __restrict__ target, int64_t n_mean, float lambda_o, float bg0, float bg1, float bg2,
    int64_t* __restrict__ total_samples, float* __restrict__ opacity, float* __restrict__ depth,
    float* __restrict__ rgb, float* __restrict__ ws, float* __restrict__ dL_drgb, float* __restrict__ dL_dop,
    float* __restrict__ dL_dsigmas, float* __restrict__ dL_drgbs, float* __restrict__ loss_part) {
    __shared__ float lsum[4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t n = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    float l = 0.0f;
    if (n < n_rays) {
        const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
        const int N = (int)rays_a[3 * n + 2];
        const float tg[3] = {target[3 * ray], target[3 * ray + 1], target[3 * ray + 2]};
        // ---- pass 1: forward (composite_fw_wave_kernel)
        float T = 1.0f, R = 0.f, G = 0.f, B = 0.f, D = 0.f, O = 0.f;
        int total = N;
        bool ended = false;
        for (int k0 = 0; k0 < N; k0 += 64) {
            const int nv = min(64, N - k0);
            const int64_t s = start + k0 + lane;
            const bool valid = lane < nv;
            float w = 0.0f, tn = 0.0f;
            if (!ended) {
                // the chunk's loads are all issued before the serial chain, which hides them
                float sg = 0.f, dl = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, tv = 0.f;
                if (valid) {
                    sg = sigmas[s]; dl = deltas[s]; tv = ts[s];
                    c0 = rgbs[3 * s]; c1 = rgbs[3 * s + 1]; c2 = rgbs[3 * s + 2];
                }
                const float a = valid ? 1.0f - fast_exp(-sg * dl) : 0.0f;
                int stop;
                const float myT = t_chain(a, T, T_thr, lane, nv, &stop);
                if (valid && lane <= stop) {
                    w = a * myT;
                    tn = myT * (1.0f - a);
                    R = fmaf(w, c0, R); G = fmaf(w, c1, G); B = fmaf(w, c2, B);
                    D = fmaf(w, tv, D);
                    O += w;
                }
                if (stop < 64) { ended = true; total = k0 + stop; }
            }
            if (valid) { ws[s] = w; dL_dsigmas[s] = tn; }
        }
        R = wave_sum(R); G = wave_sum(G); B = wave_sum(B); D = wave_sum(D); O = wave_sum(O);
        // ---- loss (nerf_loss_kernel, same expression order), wave-uniform
        const float inv3n = 1.0f / (3.0f * (float)n_mean), invn = 1.0f / (float)n_mean;
        const float bg[3] = {bg0, bg1, bg2}, col[3] = {R, G, B};
        float gcol[3], dop = 0.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float e = col[c] + bg[c] * (1.0f - O) - tg[c];
            l += e * e * inv3n;
            gcol[c] = 2.0f * e * inv3n;
            dop -= bg[c] * gcol[c];
        }
        const float o = O + 1e-10f;
        l += lambda_o * (-o * logf(o)) * invn;
        const float go = dop + lambda_o * (-(logf(o) + 1.0f)) * invn;
        if (lane == 0) {
            opacity[ray] = O; depth[ray] = D;
            rgb[3 * ray] = R; rgb[3 * ray + 1] = G; rgb[3 * ray + 2] = B;
            total_samples[ray] = total;
            dL_drgb[3 * ray] = gcol[0]; dL_drgb[3 * ray + 1] = gcol[1]; dL_drgb[3 * ray + 2] = gcol[2];
            dL_dop[ray] = go;
        }
        // ---- pass 2: backward (composite_bw_wave_kernel with dL_ddepth = dL_dws = 0)
        const int last = ended ? total : N - 1;  // the last accumulated sample
        const float gr = gcol[0], gg = gcol[1], gb = gcol[2];
        float cr = 0.f, cg = 0.f, cb = 0.f;
        for (int k0 = 0; k0 < N; k0 += 64) {
            const int64_t s = start + k0 + lane;
            const bool valid = k0 + lane < N;
            const bool act = k0 + lane <= last;
            if (k0 > last) {  // after termination: zero gradients
                if (valid) {
                    dL_dsigmas[s] = 0.0f;
                    dL_drgbs[3 * s] = 0.0f; dL_drgbs[3 * s + 1] = 0.0f; dL_drgbs[3 * s + 2] = 0.0f;
                }
                continue;
            }
            float w = 0.f, tn = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f, dl = 0.f;
            if (act) {
                w = ws[s]; tn = dL_dsigmas[s]; dl = deltas[s];
                c0 = rgbs[3 * s]; c1 = rgbs[3 * s + 1]; c2 = rgbs[3 * s + 2];
            }
            const float pr = wave_incl_scan(w * c0, lane) + cr, pg = wave_incl_scan(w * c1, lane) + cg;
            const float pb = wave_incl_scan(w * c2, lane) + cb;
            cr = readlane_f(pr, 63); cg = readlane_f(pg, 63); cb = readlane_f(pb, 63);
            float dsig = 0.0f, d0 = 0.0f, d1 = 0.0f, d2 = 0.0f;
            if (act) {
                d0 = gr * w; d1 = gg * w; d2 = gb * w;
                float acc = gr * fmaf(c0, tn, -(R - pr));
                acc = fmaf(gg, fmaf(c1, tn, -(G - pg)), acc);
                acc = fmaf(gb, fmaf(c2, tn, -(B - pb)), acc);
                acc = fmaf(go, 1 - O, acc);
                dsig = dl * acc;
            }
            if (valid) {
                dL_dsigmas[s] = dsig;
                dL_drgbs[3 * s] = d0; dL_drgbs[3 * s + 1] = d1; dL_drgbs[3 * s + 2] = d2;
            }
        }
    }
    if (lane == 0) lsum[wid] = l;
    __syncthreads();
    if (threadIdx.x == 0 && loss_part) loss_part[blockIdx.x] = (lsum[0] + lsum[1]) + (lsum[2] + lsum[3]);
}

__global__ void composite_test_kernel(const float* __restrict__ sigmas, const float* __restrict__ rgbs,
                                      const float* __restrict__ deltas, const float* __restrict__ ts,
                                      int64_t* __restrict__ alive, int64_t n_alive, int N_samples, float T_thr,
                                      const int32_t* __restrict__ n_eff, float* __restrict__ opacity,
                                      float* __restrict__ depth, float* __restrict__ rgb) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    const int ne = n_eff[n];
    if (ne == 0) { alive[n] = -1; return; }
    const int64_t r = alive[n];
    float O = opacity[r], D = depth[r], R = rgb[3 * r], G = rgb[3 * r + 1], B = rgb[3 * r + 2];
    float T = 1 - O;
    for (int s = 0; s < ne; ++s) {
        const int64_t k = n * N_samples + s;
        const float a = 1.0f - fast_exp(-sigmas[k] * deltas[k]);
        const float w = a * T;
        R = fmaf(w, rgbs[3 * k], R); G = fmaf(w, rgbs[3 * k + 1], G); B = fmaf(w, rgbs[3 * k + 2], B);
        D = fmaf(w, ts[k], D);
        O += w;
        T *= 1.0f - a;
        if (T <= T_thr) { alive[n] = -1; break; }
    }
    opacity[r] = O; depth[r] = D; rgb[3 * r] = R; rgb[3 * r + 1] = G; rgb[3 * r + 2] = B;
}

// ------------------------------------------------------------------ distortion loss (losses.cu)
__global__ void distortion_fw_kernel(const float* __restrict__ ws, const float* __restrict__ deltas,
                                     const float* __restrict__ ts, const int64_t* __restrict__ rays_a,
                                     int64_t n_rays, float* __restrict__ loss, float* __restrict__ ws_incl,
                                     float* __restrict__ wts_incl) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_rays) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    const float third = 1.0f / 3;
    float a = 0.f, b = 0.f, sum = 0.f;
    for (int k = 0; k < N; ++k) {
        const int64_t s = start + k;
        const float wx = a, wtx = b;
        a += ws[s]; b += ws[s] * ts[s];
        ws_incl[s] = a; wts_incl[s] = b;
        sum += 2 * (b * wx - a * wtx) + third * ws[s] * ws[s] * deltas[s];
    }
    loss[ray] = sum;
}

__global__ void distortion_bw_kernel(const float* __restrict__ dL_dloss, const float* __restrict__ ws_incl,
                                     const float* __restrict__ wts_incl, const float* __restrict__ ws,
                                     const float* __restrict__ deltas, const float* __restrict__ ts,
                                     const int64_t* __restrict__ rays_a, int64_t n_rays, float* __restrict__ dL_dws) {
    const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_rays) return;
    const int64_t ray = rays_a[3 * n], start = rays_a[3 * n + 1];
    const int N = (int)rays_a[3 * n + 2];
    if (N <= 0) return;
    const int64_t end = start + N - 1;
    const float ws_sum = ws_incl[end], wts_sum = wts_incl[end], g = dL_dloss[ray];
    for (int64_t s = start; s <= end; ++s) {
        const float first = (s == start) ? 0.0f : fmaf(ts[s], ws_incl[s - 1], -wts_incl[s - 1]);
        const float second = fmaf(-ts[s], ws_sum - ws_incl[s], wts_sum - wts_incl[s]);
        float v = g * 2 * (first + second);
        dL_dws[s] = fmaf(g * (float)2 / 3 * ws[s], deltas[s], v);
    }
}


// ------------------------------------------------------------------ NeRF loss (losses.py:47-60, train.py:178)
// pred = rgb + bg*(1-opacity) (rendering.py:153-161); loss = mean((pred-gt)^2) + lambda*mean(-o ln o),
// o = opacity + 1e-10.  Writes dL/drgb, dL/dopacity of that scalar and accumulates it into loss_sum.
__global__ void nerf_loss_kernel(const float* __restrict__ rgb, const float* __restrict__ opacity,
                                 const float* __restrict__ gt, int64_t n_rays, int64_t n_mean, float lambda_o,
                                 float bg0, float bg1,
                                 float bg2, float* __restrict__ dL_drgb, float* __restrict__ dL_dop,
                                 float* __restrict__ loss_sum) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float l = 0.0f;
    if (r < n_rays) {
        const float op = opacity[r];
        const float inv3n = 1.0f / (3.0f * (float)n_mean), invn = 1.0f / (float)n_mean;
        const float bg[3] = {bg0, bg1, bg2};
        float dop = 0.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float e = rgb[3 * r + c] + bg[c] * (1.0f - op) - gt[3 * r + c];
            l += e * e * inv3n;
            const float g = 2.0f * e * inv3n;
            dL_drgb[3 * r + c] = g;
            dop -= bg[c] * g;
        }
        const float o = op + 1e-10f;
        l += lambda_o * (-o * logf(o)) * invn;
        dL_dop[r] = dop + lambda_o * (-(logf(o) + 1.0f)) * invn;
    }
    // wave reduction, one atomic per wave
    for (int off = 32; off > 0; off >>= 1) l += __shfl_down(l, off, 64);
    if ((threadIdx.x & 63) == 0 && loss_sum) atomicAdd(loss_sum, l);
}

inline unsigned blocks_for(int64_t n, int b) { return (unsigned)div_up<int64_t>(n, b); }

}  // namespace

// ================================================================== C ABI
extern "C" {

int mfnerf_ray_aabb_intersect(const float* rays_o, const float* rays_d, const float* centers,
                              const float* half_sizes, int64_t n_rays, int64_t n_voxels, int max_hits,
                              int32_t* hit_cnt, float* hits_t, int64_t* hits_voxel_idx, mfnerf_stream_t stream) {
    if (n_rays < 0 || n_voxels < 0 || max_hits <= 0) { mfn_set_error("ray_aabb_intersect: bad sizes"); return MFN_ERR_INVALID; }
    if (n_rays == 0) return MFN_OK;
    if (!rays_o || !rays_d || !centers || !half_sizes || !hit_cnt || !hits_t || !hits_voxel_idx) {
        mfn_set_error("ray_aabb_intersect: null pointer"); return MFN_ERR_INVALID;
    }
    hipLaunchKernelGGL(ray_aabb_kernel, dim3(blocks_for(n_rays, RAY_BLOCK)), dim3(RAY_BLOCK), 0, stream,
                       rays_o, rays_d, centers, half_sizes, n_rays, n_voxels, max_hits, hit_cnt, hits_t,
                       hits_voxel_idx);
    return mfn_check_launch("ray_aabb_intersect");
}

int mfnerf_morton3d(const int32_t* coords, int64_t n, int32_t* out, mfnerf_stream_t stream) {
    if (n < 0) { mfn_set_error("morton3D: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!coords || !out) { mfn_set_error("morton3D: null pointer"); return MFN_ERR_INVALID; }
    hipLaunchKernelGGL(morton_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, stream, coords, n, out);
    return mfn_check_launch("morton3D");
}

int mfnerf_morton3d_invert(const int32_t* idx, int64_t n, int32_t* coords, mfnerf_stream_t stream) {
    if (n < 0) { mfn_set_error("morton3D_invert: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!idx || !coords) { mfn_set_error("morton3D_invert: null pointer"); return MFN_ERR_INVALID; }
    hipLaunchKernelGGL(morton_invert_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, stream, idx, n, coords);
    return mfn_check_launch("morton3D_invert");
}

int mfnerf_packbits(const float* grid, int64_t n_bytes, float thr, const float* thr_dev, uint8_t* bitfield,
                    mfnerf_stream_t stream) {
    if (n_bytes < 0) { mfn_set_error("packbits: bad size"); return MFN_ERR_INVALID; }
    if (n_bytes == 0) return MFN_OK;
    if (!grid || !bitfield) { mfn_set_error("packbits: null pointer"); return MFN_ERR_INVALID; }
    if (((uintptr_t)grid) & 15) { mfn_set_error("packbits: density grid must be 16-byte aligned"); return MFN_ERR_INVALID; }
    hipLaunchKernelGGL(packbits_kernel, dim3(blocks_for(n_bytes, 256)), dim3(256), 0, stream, grid, n_bytes, thr,
                       thr_dev, bitfield);
    return mfn_check_launch("packbits");
}

// the per-ray counts, then (constant-dt scenes) the per-ray sample t values of march_wave
int64_t mfnerf_raymarching_train_workspace(int64_t n_rays, int max_samples) {
    const int64_t counts = ((n_rays * 4 + 255) / 256) * 256;
    return counts + (max_samples > 0 ? n_rays * (int64_t)max_samples * 4 : 0);
}

int mfnerf_raymarching_train(const float* rays_o, const float* rays_d, const float* hits_t, int64_t hits_stride,
                             const uint8_t* bitfield, int cascades, float scale, float exp_step_factor,
                             const float* noise, int grid_size, int max_samples, int64_t n_rays, int64_t capacity,
                             int64_t* rays_a, float* xyzs, float* dirs, float* deltas, float* ts, int32_t* counter,
                             void* workspace, mfnerf_stream_t stream) {
    if (n_rays < 0 || n_rays > INT32_MAX - SCAN_THREADS || capacity < 0 || cascades < 1 || grid_size < 1 ||
        grid_size > 1024 || max_samples < 1 || hits_stride < 2) {
        mfn_set_error("raymarching_train: bad arguments"); return MFN_ERR_INVALID;
    }
    if (!counter) { mfn_set_error("raymarching_train: null counter"); return MFN_ERR_INVALID; }
    if (n_rays == 0) { mfn_zero_async(counter, 8, stream); return mfn_check_launch("raymarching_train"); }
    if (!rays_o || !rays_d || !hits_t || !bitfield || !noise || !rays_a || !workspace ||
        (capacity > 0 && (!xyzs || !dirs || !deltas || !ts))) {
        mfn_set_error("raymarching_train: null pointer"); return MFN_ERR_INVALID;
    }
    MarchParams p{rays_o, rays_d, hits_t, hits_stride, bitfield, cascades, scale, exp_step_factor, noise,
                  grid_size, max_samples};
    int32_t* counts = (int32_t*)workspace;
    float* tbuf = reinterpret_cast<float*>((char*)workspace + ((n_rays * 4 + 255) / 256) * 256);
    const unsigned nb = blocks_for(n_rays, RAY_BLOCK);
    const bool wave = exp_step_factor == 0.0f;  // constant dt: the wave-per-ray marcher applies
    const unsigned nbw = (unsigned)div_up<int64_t>(n_rays, 4);
    if (wave)
        hipLaunchKernelGGL(march_wave_kernel, dim3(nbw), dim3(256), 0, stream, p, n_rays, counts, tbuf);
    else
        hipLaunchKernelGGL(march_count_kernel, dim3(nb), dim3(RAY_BLOCK), 0, stream, p, n_rays, counts);
    hipLaunchKernelGGL(march_scan_kernel, dim3(1), dim3(SCAN_THREADS), 0, stream, counts, n_rays, capacity, rays_a,
                       counter);
    if (wave)
        hipLaunchKernelGGL(march_expand_kernel, dim3(nbw), dim3(256), 0, stream, p, n_rays, rays_a, tbuf, xyzs,
                           dirs, deltas, ts);
    else
        hipLaunchKernelGGL(march_write_kernel, dim3(nb), dim3(RAY_BLOCK), 0, stream, p, n_rays, rays_a, xyzs, dirs,
                           deltas, ts);
    return mfn_check_launch("raymarching_train");
}

int mfnerf_raymarching_test(const float* rays_o, const float* rays_d, float* hits_t, int64_t hits_stride,
                            const int64_t* alive_indices, int64_t n_alive, const uint8_t* bitfield, int cascades,
                            float scale, float exp_step_factor, int grid_size, int max_samples, int N_samples,
                            float* xyzs, float* dirs, float* deltas, float* ts, int32_t* n_eff,
                            mfnerf_stream_t stream) {
    if (n_alive < 0 || N_samples < 0 || cascades < 1 || grid_size < 1 || grid_size > 1024 || max_samples < 1 ||
        hits_stride < 2) {
        mfn_set_error("raymarching_test: bad arguments"); return MFN_ERR_INVALID;
    }
    if (n_alive == 0) return MFN_OK;
    if (!rays_o || !rays_d || !hits_t || !alive_indices || !bitfield || !n_eff ||
        (N_samples > 0 && (!xyzs || !dirs || !deltas || !ts))) {
        mfn_set_error("raymarching_test: null pointer"); return MFN_ERR_INVALID;
    }
    MarchParams p{rays_o, rays_d, hits_t, hits_stride, bitfield, cascades, scale, exp_step_factor, nullptr,
                  grid_size, max_samples};
    hipLaunchKernelGGL(march_test_kernel, dim3(blocks_for(n_alive, RAY_BLOCK)), dim3(RAY_BLOCK), 0, stream, p,
                       hits_t, alive_indices, n_alive, N_samples, xyzs, dirs, deltas, ts, n_eff);
    return mfn_check_launch("raymarching_test");
}

int mfnerf_composite_train_fw(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                              const int64_t* rays_a, int64_t n_rays, int64_t n_samples, float T_threshold,
                              int64_t* total_samples, float* opacity, float* depth, float* rgb, float* ws,
                              mfnerf_stream_t stream) {
    if (n_rays < 0 || n_samples < 0) { mfn_set_error("composite_train_fw: bad sizes"); return MFN_ERR_INVALID; }
    if (n_rays == 0) return MFN_OK;
    if (!rays_a || !total_samples || !opacity || !depth || !rgb ||
        (n_samples > 0 && (!sigmas || !rgbs || !deltas || !ts || !ws))) {
        mfn_set_error("composite_train_fw: null pointer"); return MFN_ERR_INVALID;
    }
    hipLaunchKernelGGL(composite_fw_wave_kernel, dim3(blocks_for(n_rays, 4)), dim3(256), 0, stream, sigmas, rgbs, deltas,
                       ts, rays_a, n_rays, T_threshold, total_samples, opacity, depth, rgb, ws);
    return mfn_check_launch("composite_train_fw");
}

int mfnerf_composite_train_bw(const float* dL_dopacity, const float* dL_ddepth, const float* dL_drgb,
                              const float* dL_dws, const float* sigmas, const float* rgbs, const float* ws,
                              const float* deltas, const float* ts, const int64_t* rays_a, const float* opacity,
                              const float* depth, const float* rgb, int64_t n_rays, int64_t n_samples,
                              float T_threshold, float* dL_dsigmas, float* dL_drgbs, mfnerf_stream_t stream) {
    if (n_rays < 0 || n_samples < 0) { mfn_set_error("composite_train_bw: bad sizes"); return MFN_ERR_INVALID; }
    if (n_rays == 0) return MFN_OK;
    if (!dL_dopacity || !dL_ddepth || !dL_drgb || !rays_a || !opacity || !depth || !rgb ||
        (n_samples > 0 && (!dL_dws || !sigmas || !rgbs || !ws || !deltas || !ts || !dL_dsigmas || !dL_drgbs))) {
        mfn_set_error("composite_train_bw: null pointer"); return MFN_ERR_INVALID;
    }
    hipLaunchKernelGGL(composite_bw_wave_kernel, dim3(blocks_for(n_rays, 4)), dim3(256), 0, stream,
                       dL_dopacity, dL_ddepth, dL_drgb, dL_dws, sigmas, rgbs, ws, deltas, ts, rays_a, opacity,
                       depth, rgb, n_rays, T_threshold, dL_dsigmas, dL_drgbs);
    return mfn_check_launch("composite_train_bw");
}

int mfnerf_composite_train_fused(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                                 const int64_t* rays_a, int64_t n_rays, int64_t n_samples, float T_threshold,
                                 const float* target, int64_t n_mean, float lambda_opacity, float bg_r, float bg_g,
                                 float bg_b, int64_t* total_samples, float* opacity, float* depth, float* rgb,
                                 float* ws, float* dL_drgb, float* dL_dopacity, float* dL_dsigmas, float* dL_drgbs,
                                 float* loss_partials, mfnerf_stream_t stream) {
    if (n_rays < 0 || n_samples < 0 || n_mean < 0 || (n_mean > 0 && n_mean < n_rays)) {
        mfn_set_error("composite_train_fused: bad sizes"); return MFN_ERR_INVALID;
    }
    if (n_mean == 0) n_mean = n_rays;
    if (n_rays == 0) return MFN_OK;
    if (!rays_a || !target || !total_samples || !opacity || !depth || !rgb || !dL_drgb || !dL_dopacity ||
        (n_samples > 0 && (!sigmas || !rgbs || !deltas || !ts || !ws || !dL_dsigmas || !dL_drgbs))) {
        mfn_set_error("composite_train_fused: null pointer"); return MFN_ERR_INVALID;
    }
    hipLaunchKernelGGL(composite_fused_wave_kernel, dim3(blocks_for(n_rays, 4)), dim3(256), 0, stream, sigmas, rgbs,
                       deltas, ts, rays_a, n_rays, T_threshold, target, n_mean, lambda_opacity, bg_r, bg_g, bg_b,
                       total_samples, opacity, depth, rgb, ws, dL_drgb, dL_dopacity, dL_dsigmas, dL_drgbs,
                       loss_partials);
    return mfn_check_launch("composite_train_fused");
}

int mfnerf_composite_test_fw(const float* sigmas, const float* rgbs, const float* deltas, const float* ts,
                             int64_t* alive_indices, int64_t n_alive, int N_samples, float T_threshold,
                             const int32_t* n_eff, float* opacity, float* depth, float* rgb,
                             mfnerf_stream_t stream) {
    if (n_alive < 0 || N_samples < 0) { mfn_set_error("composite_test_fw: bad sizes"); return MFN_ERR_INVALID; }
    if (n_alive == 0) return MFN_OK;
    if (!alive_indices || !n_eff || !opacity || !depth || !rgb ||
        (N_samples > 0 && (!sigmas || !rgbs || !deltas || !ts))) {
        mfn_set_error("composite_test_fw: null pointer"); return MFN_ERR_INVALID;
    }
    hipLaunchKernelGGL(composite_test_kernel, dim3(blocks_for(n_alive, RAY_BLOCK)), dim3(RAY_BLOCK), 0, stream,
                       sigmas, rgbs, deltas, ts, alive_indices, n_alive, N_samples, T_threshold, n_eff, opacity,
                       depth, rgb);
    return mfn_check_launch("composite_test_fw");
}

int mfnerf_distortion_loss_fw(const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                              int64_t n_rays, int64_t n_samples, float* loss, float* ws_incl, float* wts_incl,
                              mfnerf_stream_t stream) {
    if (n_rays < 0 || n_samples < 0) { mfn_set_error("distortion_loss_fw: bad sizes"); return MFN_ERR_INVALID; }
    if (n_rays == 0) return MFN_OK;
    if (!rays_a || !loss || (n_samples > 0 && (!ws || !deltas || !ts || !ws_incl || !wts_incl))) {
        mfn_set_error("distortion_loss_fw: null pointer"); return MFN_ERR_INVALID;
    }
    mfn_zero_async(loss, n_rays * sizeof(float), stream);
    hipLaunchKernelGGL(distortion_fw_kernel, dim3(blocks_for(n_rays, RAY_BLOCK)), dim3(RAY_BLOCK), 0, stream, ws,
                       deltas, ts, rays_a, n_rays, loss, ws_incl, wts_incl);
    return mfn_check_launch("distortion_loss_fw");
}

int mfnerf_distortion_loss_bw(const float* dL_dloss, const float* ws_incl, const float* wts_incl,
                              const float* ws, const float* deltas, const float* ts, const int64_t* rays_a,
                              int64_t n_rays, int64_t n_samples, float* dL_dws, mfnerf_stream_t stream) {
    if (n_rays < 0 || n_samples < 0) { mfn_set_error("distortion_loss_bw: bad sizes"); return MFN_ERR_INVALID; }
    if (n_rays == 0) return MFN_OK;
    if (!dL_dloss || !rays_a || (n_samples > 0 && (!ws_incl || !wts_incl || !ws || !deltas || !ts || !dL_dws))) {
        mfn_set_error("distortion_loss_bw: null pointer"); return MFN_ERR_INVALID;
    }
    if (n_samples > 0) mfn_zero_async(dL_dws, n_samples * sizeof(float), stream);
    hipLaunchKernelGGL(distortion_bw_kernel, dim3(blocks_for(n_rays, RAY_BLOCK)), dim3(RAY_BLOCK), 0, stream,
                       dL_dloss, ws_incl, wts_incl, ws, deltas, ts, rays_a, n_rays, dL_dws);
    return mfn_check_launch("distortion_loss_bw");
}

int mfnerf_nerf_loss(const float* rgb, const float* opacity, const float* target, int64_t n_rays, int64_t n_mean,
                     float lambda_opacity, float bg_r, float bg_g, float bg_b, float* dL_drgb, float* dL_dopacity,
                     float* loss_sum, mfnerf_stream_t stream) {
    if (n_rays < 0 || n_mean < 0 || (n_mean > 0 && n_mean < n_rays)) { mfn_set_error("nerf_loss: bad size"); return MFN_ERR_INVALID; }
    if (n_mean == 0) n_mean = n_rays;
    if (n_rays == 0) return MFN_OK;
    if (!rgb || !opacity || !target || !dL_drgb || !dL_dopacity) { mfn_set_error("nerf_loss: null pointer"); return MFN_ERR_INVALID; }
    hipLaunchKernelGGL(nerf_loss_kernel, dim3(blocks_for(n_rays, 256)), dim3(256), 0, stream, rgb, opacity, target,
                       n_rays, n_mean, lambda_opacity, bg_r, bg_g, bg_b, dL_drgb, dL_dopacity, loss_sum);
    return mfn_check_launch("nerf_loss");
}

}  // extern "C"
