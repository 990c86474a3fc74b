// field.hip -- NGP field head on gfx950 MFMA: the two tiny-cuda-nn FullyFusedMLPs of
// models/networks.py:36-79 (xyz: 32->64->16; rgb: [SH4(16) | h(16)] -> W -> W -> 3 with
// W = rgb_channels in {64, 128} (opt.py:87; the MF benchmark scripts use 128), ReLU, bias-free,
// fp16 operands / fp32 accumulation), TruncExp on h[0] and the SH4 direction encoding, forward
// and backward.
//
// Layout (one wave = one tile of 32 samples, v_mfma_f32_32x32x16_f16):
//   activations are kept TRANSPOSED -- channel on the MFMA row, sample on the lane (col = lane&31)
//   -- so layer k's fp32 accumulator, ReLU'd and packed to f16, IS layer k+1's B operand with no
//   LDS round trip (cdna_hip_programming.md section 3, "An accumulator tile as the next MFMA's
//   operand").  The weights are the A operands, pre-permuted once per optimizer step by
//   mfnerf_field_pack_weights into 1-KiB lane-linear fragments (ds_read_b128, conflict-free).
//   Backward: see the comments above field_bw_coop_kernel (W = 64) and field_bw_coop128_kernel.
#include <cstdlib>

#include "common.hpp"
#include "mfma_pack.hpp"
#include "field_pack.hpp"
#include "../../include/mfnerf.h"

using namespace mfn;
using namespace mfn_field;

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int FIELD_BLOCK = 256;    // forward: 4 waves

// Backward: 4 waves per workgroup, each the forward + data-gradient chain of its own 32-sample tile,
// the weight-gradient tiles split over the waves (field_bw_coop_kernel, field_bw_coop128_kernel).
// Rounds 1-4 held every tile in each wave (one wave per SIMD; at W = 128 a second pass recomputed the
// forward for dWr2's 16 tiles: 0.46 vs 0.23 ms on the mf128 step, profiles/r05_v8_*).
// Measured and not kept (rounds 1-2): every tile in an LDS image with two waves per SIMD (ds_add_f32
// per sample tile; W = 128: 836 vs 171 us), dWr2 by LDS atomics beside the register tiles (3.4 ms
// per 983k samples), Wr2^T read from global memory, two sample tiles per loop trip (~560 registers:
// 80-147 spilled, 177 vs 122 us inside the step).
// The weight gradients' operands need the samples in the MFMA K dimension: the TRANSPOSE of the
// chain's T operands (channel on the row, sample on the lane).  Each T chunk goes to a per-wave LDS
// image of the tile, [sample][channel] in 64-B rows of eight 8-B chunks (4 channels), the chunk index
// XOR-swizzled with (row >> 1) & 7 (2-way bank conflicts on the writes, none on the reads), and comes
// back with ds_read_b64_tr_b16, which hands each 16-lane group a 4-sample x 16-channel block column by
// column (cdna_hip_programming.md T10).  The S operand's k order is the one the accumulator-as-operand
// packing has (element j of lane half h = sample 8(j>>2) + 4h + (j&3) of the k-step), so both operands
// of every dW product agree.  Exact.  (Rounds 1-2 transposed on the matrix core instead: D = T x I,
// 2 MFMAs + 8 packing instructions per tile, ~30 of the 98 MFMAs of a sample tile.)
constexpr int TILE_HALFS = 32 * 32;
constexpr size_t TILE_BYTES = TILE_HALFS * 2;
typedef short short4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int tix(int row, int chunk) { return row * 32 + 4 * (chunk ^ ((row >> 1) & 7)); }

// this lane's 8 channels of a T chunk (sample = lane & 31) into the tile image; cbase = first channel / 4;
// perm: element j is channel 4 cbase + 8(j>>2) + 4h + (j&3) (a packed accumulator), else 4 cbase + 8h + j
__device__ __forceinline__ void t_put(_Float16* slot, int lane, const half8& v, int cbase, bool perm) {
    const int r = lane & 31, h = lane >> 5;
    const int c0 = cbase + (perm ? h : 2 * h), c1 = cbase + (perm ? 2 + h : 2 * h + 1);
    H8 u;
    u.h = v;
    *reinterpret_cast<u32x2*>(slot + tix(r, c0)) = u32x2{u.w[0], u.w[1]};
    *reinterpret_cast<u32x2*>(slot + tix(r, c1)) = u32x2{u.w[2], u.w[3]};
}

__device__ __forceinline__ u32x2 tr_read(const _Float16* p) {
    typedef __attribute__((address_space(3))) short4v* lds_s4;
    return __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4)(p)));
}

struct SOp;
__device__ __forceinline__ SOp s_get(const _Float16* slot, int lane);

// tcnn SphericalHarmonics degree 4 as a module of its own (the tinycudann route's dir_encoder,
// networks.py:60-67): in = (d/|d| + 1)/2 (n, 3) f32 -> (n, 16) f16, the IEEE operations and their
// order of mfnerf/tcnn.py sh4_torch (no contraction), rounded to f16 once.  The fused field head
// evaluates the same polynomial in-kernel (sh4 above).
__global__ __launch_bounds__(256) void sh4_fw_kernel(const float* __restrict__ in, int64_t n,
                                                     __half* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = in[3 * i] * 2.0f - 1.0f, y = in[3 * i + 1] * 2.0f - 1.0f, z = in[3 * i + 2] * 2.0f - 1.0f;
    const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    float o[16];
    o[0] = 0.28209479177387814f;
    o[1] = -0.48860251190291987f * y;
    o[2] = 0.48860251190291987f * z;
    o[3] = -0.48860251190291987f * x;
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
    o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
    o[10] = 2.8906114426405538f * xy * z;
    o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
    o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
    o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
    o[14] = 1.4453057213202769f * z * (x2 - y2);
    o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
    // each value rounded to f32 first, as torch does: an opaque use keeps the compiler from folding a
    // product and its f16 conversion into one v_fma_mix (a single rounding of the exact product,
    // which differs from torch's double rounding on ~1 value in 10^6)
#pragma unroll
    for (int k = 0; k < 16; ++k) asm volatile("" : "+v"(o[k]));
    __half2* dst = reinterpret_cast<__half2*>(out + 16 * i);
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k] = __floats2half2_rn(o[2 * k], o[2 * k + 1]);
}

template <typename TP, int W>
__global__ void pack_kernel(const TP* __restrict__ px, const TP* __restrict__ pr, _Float16* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < Geo<W>::N * FRAG_HALFS) pack_elem<TP, W>(t, px, pr, out);
}

__device__ __forceinline__ f32x16 mfma(const half8& a, const half8& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ half8 lds_frag(const _Float16* lds, int f, int lane) {
    return *reinterpret_cast<const half8*>(lds + (f * 64 + lane) * 8);
}

// tcnn SphericalHarmonics degree 4 on in = (d/|d| + 1)/2, mapped back x = in*2-1 (networks.py:145-146)
__device__ __forceinline__ void sh4(float dx, float dy, float dz, float* o) {
    const float nrm = sqrtf(dx * dx + dy * dy + dz * dz);
    float x = dx / nrm, y = dy / nrm, z = dz / nrm;
    x = ((x + 1.0f) / 2.0f) * 2.0f - 1.0f;
    y = ((y + 1.0f) / 2.0f) * 2.0f - 1.0f;
    z = ((z + 1.0f) / 2.0f) * 2.0f - 1.0f;
    const float xy = x * y, xz = x * z, yz = y * z, x2 = x * x, y2 = y * y, z2 = z * z;
    o[0] = 0.28209479177387814f;
    o[1] = -0.48860251190291987f * y;
    o[2] = 0.48860251190291987f * z;
    o[3] = -0.48860251190291987f * x;
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.94617469575755997f * z2 - 0.31539156525251999f;
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.54627421529603959f * x2 - 0.54627421529603959f * y2;
    o[9] = 0.59004358992664352f * y * (-3.0f * x2 + y2);
    o[10] = 2.8906114426405538f * xy * z;
    o[11] = 0.45704579946446572f * y * (1.0f - 5.0f * z2);
    o[12] = 0.3731763325901154f * z * (5.0f * z2 - 3.0f);
    o[13] = 0.45704579946446572f * x * (1.0f - 5.0f * z2);
    o[14] = 1.4453057213202769f * z * (x2 - y2);
    o[15] = 0.59004358992664352f * x * (-x2 + 3.0f * y2);
}

// Forward state of one tile that the backward needs again.
template <int W>
struct FwdTile {
    half8 x[2];             // B operands of layer 1 (natural order, features 16q+8h+j)
    half8 y1[2][2];         // relu(Y1) as B operands [t][q]
    half8 hb;               // h (16 features, perm order) = rgb-input k-step 1
    half8 sh;               // SH (natural order 8h+j)    = rgb-input k-step 0
    half8 r1[W / 32][2];
    half8 r2[W / 32][2];
    float h0;               // h[0] (f16-rounded) on lanes h==0
    float rgb[3];           // sigmoid outputs on lanes h==0 (fp32)
};

// Loads of one tile's inputs (feature row halves for this lane, direction), used directly or as
// the next tile's prefetch.
struct TileIn {
    half8 x[2];
    float d[3];
};

// feat layouts: plane_stride == 0 -> row-major (n, 32) f16 (tcnn's encoding output); > 0 ->
// level-major planes (16, plane_stride) half2 (mfnerf_grid_encode_fw_planar).
__device__ __forceinline__ void load_tile_in(const _Float16* __restrict__ feat, int64_t plane_stride,
                                             const float* __restrict__ dirs, int64_t s, bool valid, int h,
                                             bool want_dirs, TileIn& I) {
    if (valid) {
        if (plane_stride > 0) {
            // x[0] element j = feature 8h+j = level 4h + j/2; x[1]: level 8 + 4h + j/2
            const uint32_t* P = reinterpret_cast<const uint32_t*>(feat);
            uint32_t u[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                u[k] = P[(int64_t)(4 * h + k) * plane_stride + s];
                u[4 + k] = P[(int64_t)(8 + 4 * h + k) * plane_stride + s];
            }
            I.x[0] = *reinterpret_cast<const half8*>(&u[0]);
            I.x[1] = *reinterpret_cast<const half8*>(&u[4]);
        } else {
            const half8* row = reinterpret_cast<const half8*>(feat + s * 32);
            I.x[0] = row[h];
            I.x[1] = row[2 + h];
        }
        if (want_dirs) { I.d[0] = dirs[3 * s]; I.d[1] = dirs[3 * s + 1]; I.d[2] = dirs[3 * s + 2]; }
    } else {
        I.x[0] = half8{}; I.x[1] = half8{};
        I.d[0] = I.d[1] = I.d[2] = 0.0f;
    }
}

// The forward of P independent tiles, stage by stage: each layer's MFMAs for every tile, then the
// next layer.  The scheduler keeps this source order at one wave per SIMD, so a tile's packing
// (VALU) overlaps the next tile's MFMAs, and one fragment read from LDS serves all P tiles.
template <int W, bool DENSITY_ONLY, int P, bool ONE_TILE_FRAGS = false>
__device__ __forceinline__ void forward_tiles(const _Float16* lds, int lane, const TileIn* I, const bool* valid,
                                              FwdTile<W>* T) {
    using G = Geo<W>;
    constexpr int MT = G::MT;
    const int h = lane >> 5;
    const f32x16 z = {};
    // xyz layer 1: Y1^T = W1 X^T
    {
        const half8 f0 = lds_frag(lds, G::F1 + 0, lane), f1 = lds_frag(lds, G::F1 + 1, lane);
        const half8 f2 = lds_frag(lds, G::F1 + 2, lane), f3 = lds_frag(lds, G::F1 + 3, lane);
        f32x16 y1a[P], y1b[P];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            T[q].x[0] = I[q].x[0];
            T[q].x[1] = I[q].x[1];
            y1a[q] = mfma(f0, T[q].x[0], z);
            y1a[q] = mfma(f1, T[q].x[1], y1a[q]);
            y1b[q] = mfma(f2, T[q].x[0], z);
            y1b[q] = mfma(f3, T[q].x[1], y1b[q]);
        }
#pragma unroll
        for (int q = 0; q < P; ++q) {
            T[q].y1[0][0] = pack8<0, true>(y1a[q]); T[q].y1[0][1] = pack8<8, true>(y1a[q]);
            T[q].y1[1][0] = pack8<0, true>(y1b[q]); T[q].y1[1][1] = pack8<8, true>(y1b[q]);
        }
    }
    // xyz layer 2: H^T = W2 relu(Y1)^T (rows 0..15 valid)
    {
        half8 f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = lds_frag(lds, G::F2 + i, lane);
        f32x16 ha[P];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            ha[q] = mfma(f[0], T[q].y1[0][0], z);
            ha[q] = mfma(f[1], T[q].y1[0][1], ha[q]);
            ha[q] = mfma(f[2], T[q].y1[1][0], ha[q]);
            ha[q] = mfma(f[3], T[q].y1[1][1], ha[q]);
        }
#pragma unroll
        for (int q = 0; q < P; ++q) {
            T[q].hb = pack8<0, false>(ha[q]);   // the fp16 network output of tcnn
            T[q].h0 = (float)T[q].hb[0];        // row 0 on lanes h==0
        }
    }
    if (DENSITY_ONLY) return;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        float shv[16];
        sh4(I[q].d[0], I[q].d[1], I[q].d[2], shv);  // (0/0 on invalid lanes, selected away: no branch)
#pragma unroll
        for (int i = 0; i < 16; ++i) shv[i] = valid[q] ? shv[i] : 0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            // select the loaded VALUES (a conditional of the two array lvalues is an lvalue: a load
            // through a selected pointer, which kept shv in scratch memory)
            const float lo = shv[j], hi = shv[8 + j];
            T[q].sh[j] = (_Float16)(h ? hi : lo);
        }
    }
    // rgb layer 1
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const half8 f0 = lds_frag(lds, G::F3 + 2 * mt, lane), f1 = lds_frag(lds, G::F3 + 2 * mt + 1, lane);
        f32x16 a[P];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            a[q] = mfma(f0, T[q].sh, z);
            a[q] = mfma(f1, T[q].hb, a[q]);
        }
#pragma unroll
        for (int q = 0; q < P; ++q) { T[q].r1[mt][0] = pack8<0, true>(a[q]); T[q].r1[mt][1] = pack8<8, true>(a[q]); }
    }
    // rgb layer 2
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        // the forward kernel: one output tile's fragments at a time -- the scheduler otherwise hoists
        // all of layer 2's fragment reads (W = 128: 32 of them, 332 registers, one wave per SIMD;
        // with the barrier 128 registers, four).  Not in the backward's recomputation, whose
        // workgroups hold a whole CU's LDS (one wave per SIMD either way) and which ran 44 us slower
        // with it at W = 128 (r6f)
        if constexpr (ONE_TILE_FRAGS) __builtin_amdgcn_sched_barrier(0);
        f32x16 a[P];
#pragma unroll
        for (int q = 0; q < P; ++q) a[q] = z;
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const half8 f = lds_frag(lds, G::F4 + mt * G::KC + t * 2 + k, lane);
#pragma unroll
                for (int q = 0; q < P; ++q) a[q] = mfma(f, T[q].r1[t][k], a[q]);
            }
#pragma unroll
        for (int q = 0; q < P; ++q) { T[q].r2[mt][0] = pack8<0, true>(a[q]); T[q].r2[mt][1] = pack8<8, true>(a[q]); }
    }
    // rgb layer 3 (rows 0..2 = rgb logits on lanes h==0)
    f32x16 o[P];
#pragma unroll
    for (int q = 0; q < P; ++q) o[q] = z;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const half8 f = lds_frag(lds, G::F5 + t * 2 + k, lane);
#pragma unroll
            for (int q = 0; q < P; ++q) o[q] = mfma(f, T[q].r2[t][k], o[q]);
        }
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int c = 0; c < 3; ++c) T[q].rgb[c] = 1.0f / (1.0f + __expf(-o[q][c]));
}

template <int W, bool DENSITY_ONLY>
__device__ __forceinline__ void forward_tile(const _Float16* lds, int lane, const TileIn& I, bool valid,
                                             FwdTile<W>& T) {
    forward_tiles<W, DENSITY_ONLY, 1>(lds, lane, &I, &valid, &T);
}

__device__ __forceinline__ void load_frags(_Float16* lds, const _Float16* __restrict__ packed, int n_frags) {
    const uint4* src = reinterpret_cast<const uint4*>(packed);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < n_frags * 64; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

template <int W, bool DENSITY_ONLY>
__global__ __launch_bounds__(FIELD_BLOCK) void field_fw_kernel(const _Float16* __restrict__ feat,
                                                                int64_t plane_stride,
                                                                const float* __restrict__ dirs, int64_t n,
                                                                const int32_t* __restrict__ n_dev,
                                                                const _Float16* __restrict__ packed,
                                                                float* __restrict__ sigma, float* __restrict__ rgb,
                                                                const int32_t* __restrict__ cell,
                                                                float* __restrict__ cell_out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    _Float16* lds = reinterpret_cast<_Float16*>(smem);
    load_frags(lds, packed, DENSITY_ONLY ? 8 : Geo<W>::N_FW);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t tiles = div_up<int64_t>(nn, 32);
    // P tiles per trip (tile, tile + stride, ...), stage by stage (forward_tiles).  P = 2 measured no
    // faster at W = 64 (28.7 vs 28 us: 204 registers, one wave per SIMD instead of two) and spills
    // at W = 128
    constexpr int P = 1;
    const int64_t stride = (int64_t)gridDim.x * 4;
    for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile < tiles; tile += P * stride) {
        TileIn I[P];
        bool valid[P];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const int64_t s = (tile + q * stride) * 32 + r;
            valid[q] = s < nn;
            load_tile_in(feat, plane_stride, dirs, s, valid[q], h, !DENSITY_ONLY, I[q]);
        }
        FwdTile<W> T[P];
        forward_tiles<W, DENSITY_ONLY, P, true>(lds, lane, I, valid, T);
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const int64_t s = (tile + q * stride) * 32 + r;
            if (valid[q] && h == 0) {
                const float sg = __expf(T[q].h0);  // TruncExp forward (custom_functions.py:166)
                sigma[s] = sg;
                if (DENSITY_ONLY && cell_out) {  // the occupancy refresh's density_grid_tmp[cell] = sigma
                    const int32_t k = cell[s];
                    if (k >= 0) cell_out[k] = sg;
                }
                if (!DENSITY_ONLY) {
                    // tcnn returns fp16 rgb; the reference casts it to fp32 for compositing
                    rgb[3 * s] = (float)(_Float16)T[q].rgb[0];
                    rgb[3 * s + 1] = (float)(_Float16)T[q].rgb[1];
                    rgb[3 * s + 2] = (float)(_Float16)T[q].rgb[2];
                }
            }
        }
    }
}

// ---------------------------------------------------------------- backward
//
// Data gradients chain through accumulators exactly like the forward ("T" orientation: channel on
// the MFMA row, sample on the lane).  Weight gradients dW = dY^T X reduce over SAMPLES, which must
// therefore sit in the MFMA K dimension, i.e. inside each lane's registers -- the transpose of the
// T operands, the "S" orientation (channel on the lane, samples in the registers): each T chunk is
// written to a per-wave LDS tile image and read back with the transposing ds_read_b64_tr_b16
// (t_put / s_get above; exact, no wave-level synchronisation).
//   dW[out][in] (32x32 tile) += S(dY)[out-tile] x S(X)[in-tile], K = the tile's 32 samples (2 MFMAs)
// The dW tiles accumulate across all sample tiles a wave processes (persistent grid) in registers
// or in the workgroup's LDS image (BwCfg), then one slab row per workgroup, summed in a fixed order
// by slab_reduce_kernel.

template <int W, int NW>
__device__ __forceinline__ void load_frags_bw(_Float16* lds, const _Float16* __restrict__ packed) {
    using G = Geo<W>;
    const uint4* src = reinterpret_cast<const uint4*>(packed);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < G::N * 64; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// S operands (K = samples 0..15 / 16..31 of the tile) of one 32-channel tile given as two T chunks
struct SOp { half8 k[2]; };

// the S operand of a tile image (t_put): lane 4q+p of 16-lane group g supplies row (sample)
// 16s + 4h + q (+8) at channels 16(g&1) + 4p; lane i of the group gets channel 16(g&1) + i
__device__ __forceinline__ SOp s_get(const _Float16* slot, int lane) {
    const int h = lane >> 5, q = (lane >> 2) & 3, c = 4 * ((lane >> 4) & 1) + (lane & 3);
    SOp o;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int r0 = 16 * s + 4 * h + q;
        const u32x2 a = tr_read(slot + tix(r0, c)), b = tr_read(slot + tix(r0 + 8, c));
        H8 u;
        u.w[0] = a[0]; u.w[1] = a[1]; u.w[2] = b[0]; u.w[3] = b[1];
        o.k[s] = u.h;
    }
    return o;
}

__device__ __forceinline__ void dw_acc(f32x16& acc, const SOp& dy, const SOp& x) {
    acc = mfma(dy.k[0], x.k[0], acc);
    acc = mfma(dy.k[1], x.k[1], acc);
}
// The same product into a PERSISTENT accumulator pinned to AGPRs: with MFMA results in VGPRs
// (-amdgpu-mfma-vgpr-form, which the data-gradient chain needs) the compiler otherwise moves each
// of the 12 accumulator tiles AGPR <-> VGPR around every update (~500 v_accvgpr moves per tile).
// The leading s_nop covers the VALU-write -> MFMA-read hazard on the packed operands (the compiler's
// hazard recognizer does not look into inline asm); back-to-back accumulation into the same
// registers needs none.  Readers of the accumulators wait with xdl_drain().
__device__ __forceinline__ void dw_acc_agpr(f32x16& acc, const SOp& dy, const SOp& x) {
    asm("s_nop 2\n\t"
        "v_mfma_f32_32x32x16_f16 %0, %1, %2, %0\n\t"
        "v_mfma_f32_32x32x16_f16 %0, %3, %4, %0"
        : "+a"(acc)
        : "v"(dy.k[0]), "v"(x.k[0]), "v"(dy.k[1]), "v"(x.k[1]));
}
__device__ __forceinline__ void xdl_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }

// add one 32x32 dW tile (row = out 32*ot + (i&3)+8(i>>2)+4h, col = in 32*it + lane&31) into a
// row-major fp32 LDS image of a (rows x cols) matrix; rows/cols are compile-time at every call, so
// the register rows that can never be in range are dropped statically
// A workgroup's slab row holds non-finite values: raise the step's flag now.  Every row finite
// bounds every slab sum: |row value| <= (samples of one workgroup) x 65504^2 (fp16 operands,
// f32 accumulation) ~ 1e13, 512 rows ~ 5e15, far below the f32 range -- so with the rows checked
// here the flag is final when field_bw returns, even with the fold deferred past the table's Adam
// (mfnerf_grid_encode_bw_binned_adam_all's slab tail).
__device__ __forceinline__ void slab_row_flag(int32_t* nonfinite, bool bad) {
    if (nonfinite && __any(bad) && (threadIdx.x & 63) == 0) atomicOr(nonfinite, 1);
}

__device__ __forceinline__ void dw_add32(float* img, const f32x16& a, int ot, int it, int rows, int cols, int lane,
                                         bool store = false) {
    const int col = 32 * it + (lane & 31), h = lane >> 5;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = 32 * ot + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (row < rows && col < cols) {
            if (store) img[row * cols + col] = a[i];  // the first wave of a fixed-order sum
            else atomicAdd(img + row * cols + col, a[i]);
        }
    }
}

// one dW tile += dY x X into its register accumulator
__device__ __forceinline__ void acc_tile(f32x16& reg, const SOp& dy, const SOp& x) { dw_acc_agpr(reg, dy, x); }

// ---------------------------------------------------------------- cooperative backward (W = 64)
// The round 1-3 per-wave backward held all 12 weight-gradient tiles in each wave (192 accumulator registers + ~170
// for the chain): one wave per SIMD, nothing hides the chain's dependencies (PMC: waiting 56 % of
// its cycles).  Here the 12 tiles are split over the workgroup's 4 waves -- 3 each, 48 accumulator
// registers -- so a wave fits 256 registers and TWO workgroups share a CU (76 KB of LDS each: the
// 44 fragments + 4 transpose images per wave), two waves per SIMD.  Each wave still runs the
// forward and the data-gradient chain of its own 32-sample tile; the weight-gradient operands (the
// transposed T chunks, t_put) are written stage by stage into the wave's 4 images, the workgroup
// synchronises, and each wave accumulates ITS tiles of that stage over all four waves' sample tiles
// (waves 0..3 in order: a fixed summation order, deterministic).  Tiles per wave:
//   wave 0: dWr3[0], dWr2[0][0], dW2[0]      wave 2: dWr1[0], dWr2[1][0], dW1[0]
//   wave 1: dWr3[1], dWr2[0][1], dW2[1]      wave 3: dWr1[1], dWr2[1][1], dW1[1]
// Stages (images per wave): S1 dO, R2 x2 | S2 dR2 x2, R1 x2 | S3 dR1 x2, [SH;h] | S4 dh, Y1 x2 |
// S5 dY1 x2, X; the chain's next MFMAs are issued between a stage's writes and its products.
constexpr int COOP_SLOTS = 4;      // transpose images per wave live at once (stage 2)
constexpr int COOP_BLOCKS = 512;   // two workgroups per CU (persistent)
constexpr size_t COOP_LDS = (size_t)Geo<64>::N * FRAG_HALFS * 2 + (size_t)4 * COOP_SLOTS * TILE_BYTES;
static_assert(COOP_LDS <= 80 * 1024, "two cooperative workgroups per CU");

template <bool PLANAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void field_bw_coop_kernel(
    const _Float16* __restrict__ feat, int64_t plane_stride, const float* __restrict__ dirs, int64_t n,
    const int32_t* __restrict__ n_dev, const _Float16* __restrict__ packed, const float* __restrict__ dL_dsigma,
    const float* __restrict__ dL_drgb, float grad_scale, const float* __restrict__ scale_dev,
    float* __restrict__ dL_dfeat, float* __restrict__ slab, int32_t* __restrict__ nonfinite, float* __restrict__ level_l1) {
    constexpr int W = 64;
    using G = Geo<W>;
    constexpr int MT = G::MT;
    constexpr int oR1 = N_XYZ_PARAMS, oR2 = oR1 + W * 32, oR3 = oR2 + W * W;
    constexpr size_t IMG_OFF = (size_t)G::N * FRAG_HALFS * 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    _Float16* lds_base = reinterpret_cast<_Float16*>(smem);
    load_frags_bw<W, 4>(lds_base, packed);
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform)
    const int r = lane & 31, h = lane >> 5;
    const float S = scale_dev ? *scale_dev : grad_scale, invS = 1.0f / S;
    const f32x16 z = {};
    f32x16 acc0 = z, acc1 = z, acc2 = z;  // this wave's three tiles (table above)
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t tiles = div_up<int64_t>(nn, 32);
    const int64_t groups = div_up<int64_t>(tiles, 4);  // group g = tiles 4g .. 4g+3, one per wave
    struct BwIn { TileIn I; float gs, g0, g1, g2; bool live; };
    BwIn nx;
    // branch-free: every lane loads (index clamped), the incoming gradients are zeroed where
    // the sample is out of range or on lanes h == 1 -- an idle wave's tile contributes exact zeros
    auto fetch = [&](int64_t tile, BwIn& o) {
        const int64_t s = tile * 32 + r;
        const bool v = s < nn && h == 0;
        const int64_t sc = max<int64_t>(0, min<int64_t>(s, nn - 1));
        if constexpr (PLANAR) {
            const uint32_t* Pp = reinterpret_cast<const uint32_t*>(feat);
            uint32_t u[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                u[k] = Pp[(int64_t)(4 * h + k) * plane_stride + sc];
                u[4 + k] = Pp[(int64_t)(8 + 4 * h + k) * plane_stride + sc];
            }
            o.I.x[0] = *reinterpret_cast<const half8*>(&u[0]);
            o.I.x[1] = *reinterpret_cast<const half8*>(&u[4]);
        } else {
            const half8* row = reinterpret_cast<const half8*>(feat + sc * 32);
            o.I.x[0] = row[h];
            o.I.x[1] = row[2 + h];
        }
        o.I.d[0] = dirs[3 * sc]; o.I.d[1] = dirs[3 * sc + 1]; o.I.d[2] = dirs[3 * sc + 2];
        o.gs = dL_dsigma[sc]; o.g0 = dL_drgb[3 * sc]; o.g1 = dL_drgb[3 * sc + 1]; o.g2 = dL_drgb[3 * sc + 2];
        o.live = v;
    };
    auto zero_grads = [&](BwIn& o) {
        o.gs = o.live ? o.gs : 0.0f;
        o.g0 = o.live ? o.g0 : 0.0f;
        o.g1 = o.live ? o.g1 : 0.0f;
        o.g2 = o.live ? o.g2 : 0.0f;
    };
    if ((int64_t)blockIdx.x < groups) fetch(4 * (int64_t)blockIdx.x + wid, nx);
    bool bad = false;
    float l1a[4] = {0.f, 0.f, 0.f, 0.f}, l1b[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t g = blockIdx.x; g < groups; g += gridDim.x) {
        int opaque = 0;
        asm volatile("" : "+s"(opaque));
        const _Float16* lds = lds_base + opaque;
        _Float16* area = lds_base + opaque + IMG_OFF / 2;
        auto slot = [&](int u, int k) { return area + (u * COOP_SLOTS + k) * TILE_HALFS; };
        auto put2 = [&](_Float16* sl, const half8* v) {  // a 32-channel tile as two perm chunks
            t_put(sl, lane, v[0], 0, true);
            t_put(sl, lane, v[1], 4, true);
        };
        // this wave's tile of the group; the next group's inputs are loaded while it computes
        const int64_t tile = 4 * g + wid;
        BwIn in = nx;
        zero_grads(in);
        fetch(4 * (g + (int64_t)gridDim.x) + wid, nx);  // (clamped past the end)
        const bool valid = tile * 32 + r < nn;
        FwdTile<W> T;
        forward_tiles<W, false, 1>(lds, lane, &in.I, &valid, &T);
        half8 dOb;
        {
            f32x16 dO = z;
            dO[0] = in.g0 * S * T.rgb[0] * (1.0f - T.rgb[0]);
            dO[1] = in.g1 * S * T.rgb[1] * (1.0f - T.rgb[1]);
            dO[2] = in.g2 * S * T.rgb[2] * (1.0f - T.rgb[2]);
            dOb = pack8<0, false>(dO);
        }
        //    dR2 = Wr3^T dO, masked by R2 > 0
        half8 dr2p[MT][2];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const f32x16 a = mfma(lds_frag(lds, G::B5 + mt, lane), dOb, z);
            dr2p[mt][0] = relu_mask8(pack8<0, false>(a), T.r2[mt][0]);
            dr2p[mt][1] = relu_mask8(pack8<8, false>(a), T.r2[mt][1]);
        }
        // ---- S1: dO, R2 -> dWr3 (waves 0, 1)
        t_put(slot(wid, 0), lane, dOb, 0, true);  // (channels 16..31 stale: rows 16..31 of dWr3, dropped)
        put2(slot(wid, 1), T.r2[0]);
        put2(slot(wid, 2), T.r2[1]);
        __syncthreads();
        if (wid < 2) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc_tile(acc0, s_get(slot(u, 0), lane), s_get(slot(u, 1 + wid), lane));
        }
        //    dR1 = Wr2^T dR2, masked by R1 > 0
        half8 dr1p[MT][2];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            f32x16 a = z;
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int k = 0; k < 2; ++k) a = mfma(lds_frag(lds, G::B4 + mt * G::KC + t * 2 + k, lane), dr2p[t][k], a);
            dr1p[mt][0] = relu_mask8(pack8<0, false>(a), T.r1[mt][0]);
            dr1p[mt][1] = relu_mask8(pack8<8, false>(a), T.r1[mt][1]);
        }
        __syncthreads();
        // ---- S2: dR2, R1 -> dWr2 (one tile per wave)
        put2(slot(wid, 0), dr2p[0]);
        put2(slot(wid, 1), dr2p[1]);
        put2(slot(wid, 2), T.r1[0]);
        put2(slot(wid, 3), T.r1[1]);
        //    d[SH;h] = Wr1^T dR1 (rows 16..31 = dh) + TruncExp backward into h[0]
        half8 dhb;
        {
            f32x16 dsh = z;
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int k = 0; k < 2; ++k) dsh = mfma(lds_frag(lds, G::B3 + t * 2 + k, lane), dr1p[t][k], dsh);
            const float dh0 = in.gs * S * __expf(fminf(fmaxf(T.h0, -15.0f), 15.0f));
            dsh[8] = h == 0 ? dsh[8] + dh0 : dsh[8];
            dhb = pack8<8, false>(dsh);
        }
        __syncthreads();
        {
            const int o = wid >> 1, i = wid & 1;
#pragma unroll
            for (int u = 0; u < 4; ++u) acc_tile(acc1, s_get(slot(u, o), lane), s_get(slot(u, 2 + i), lane));
        }
        //    dY1 = W2^T dh, masked by Y1 > 0; dX = W1^T dY1
        half8 dy1p[2][2];
        f32x16 dx = z;
        {
            const f32x16 a0 = mfma(lds_frag(lds, G::B2 + 0, lane), dhb, z);
            const f32x16 a1 = mfma(lds_frag(lds, G::B2 + 1, lane), dhb, z);
            dy1p[0][0] = relu_mask8(pack8<0, false>(a0), T.y1[0][0]);
            dy1p[0][1] = relu_mask8(pack8<8, false>(a0), T.y1[0][1]);
            dy1p[1][0] = relu_mask8(pack8<0, false>(a1), T.y1[1][0]);
            dy1p[1][1] = relu_mask8(pack8<8, false>(a1), T.y1[1][1]);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int k = 0; k < 2; ++k) dx = mfma(lds_frag(lds, G::B1 + t * 2 + k, lane), dy1p[t][k], dx);
        }
        __syncthreads();
        // ---- S3: dR1, [SH;h] -> dWr1 (waves 2, 3)
        put2(slot(wid, 0), dr1p[0]);
        put2(slot(wid, 1), dr1p[1]);
        t_put(slot(wid, 2), lane, T.sh, 0, false);
        t_put(slot(wid, 2), lane, T.hb, 4, true);
        __syncthreads();
        if (wid >= 2) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc_tile(acc0, s_get(slot(u, wid - 2), lane), s_get(slot(u, 2), lane));
        }
        // dX = W1^T dY1 -> global fp32 (features (i&3)+8(i>>2)+4h), this wave's own tile
        {
            const int64_t s = tile * 32 + r;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 o = make_float4(dx[4 * q] * invS, dx[4 * q + 1] * invS, dx[4 * q + 2] * invS, dx[4 * q + 3] * invS);
                bad |= !(isfinite(o.x) && isfinite(o.y) && isfinite(o.z) && isfinite(o.w));
                if (s < nn) reinterpret_cast<float4*>(dL_dfeat + s * 32)[2 * q + h] = o;
                l1a[q] += fabsf(o.x) + fabsf(o.y);
                l1b[q] += fabsf(o.z) + fabsf(o.w);
            }
        }
        __syncthreads();
        // ---- S4: dh, Y1 -> dW2 (waves 0, 1)
        t_put(slot(wid, 0), lane, dhb, 0, true);  // (channels 16..31 stale: rows of dW2 dropped)
        put2(slot(wid, 1), T.y1[0]);
        put2(slot(wid, 2), T.y1[1]);
        __syncthreads();
        if (wid < 2) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc_tile(acc2, s_get(slot(u, 0), lane), s_get(slot(u, 1 + wid), lane));
        }
        __syncthreads();
        // ---- S5: dY1, X -> dW1 (waves 2, 3)
        put2(slot(wid, 0), dy1p[0]);
        put2(slot(wid, 1), dy1p[1]);
        t_put(slot(wid, 2), lane, T.x[0], 0, false);
        t_put(slot(wid, 2), lane, T.x[1], 4, false);
        __syncthreads();
        if (wid >= 2) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc_tile(acc2, s_get(slot(u, wid - 2), lane), s_get(slot(u, 2), lane));
        }
        __syncthreads();  // the images are rewritten by the next group's S1
    }
    if (nonfinite && __any(bad) && lane == 0) atomicOr(nonfinite, 1);

    // ---- epilogue: each tile stored by its owner wave (disjoint) -> one slab row per workgroup
    float* row = slab + (int64_t)blockIdx.x * G::N_DW;
    {
        constexpr int N_IMG = G::N_DW;
        static_assert((size_t)N_IMG * 4 + 64 <= IMG_OFF, "reduction image must fit the fragment area");
        xdl_drain();
        __syncthreads();
        float* img = reinterpret_cast<float*>(smem);
        float* l1_part = img + N_IMG;
        if (threadIdx.x < 16) l1_part[threadIdx.x] = 0.0f;
        __syncthreads();
        if (level_l1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float a = l1a[q], b = l1b[q];
#pragma unroll
                for (int off = 16; off > 0; off >>= 1) { a += __shfl_xor(a, off, 64); b += __shfl_xor(b, off, 64); }
                if (r == 0) { atomicAdd(l1_part + 4 * q + 2 * h, a); atomicAdd(l1_part + 4 * q + 2 * h + 1, b); }
            }
        }
        if (wid == 0) {
            dw_add32(img + oR3, acc0, 0, 0, 16, W, lane, true);
            dw_add32(img + oR2, acc1, 0, 0, W, W, lane, true);
            dw_add32(img + 64 * 32, acc2, 0, 0, 16, 64, lane, true);
        } else if (wid == 1) {
            dw_add32(img + oR3, acc0, 0, 1, 16, W, lane, true);
            dw_add32(img + oR2, acc1, 0, 1, W, W, lane, true);
            dw_add32(img + 64 * 32, acc2, 0, 1, 16, 64, lane, true);
        } else if (wid == 2) {
            dw_add32(img + oR1, acc0, 0, 0, W, 32, lane, true);
            dw_add32(img + oR2, acc1, 1, 0, W, W, lane, true);
            dw_add32(img, acc2, 0, 0, 64, 32, lane, true);
        } else {
            dw_add32(img + oR1, acc0, 1, 0, W, 32, lane, true);
            dw_add32(img + oR2, acc1, 1, 1, W, W, lane, true);
            dw_add32(img, acc2, 1, 0, 64, 32, lane, true);
        }
        __syncthreads();
        bool rbad = false;  // a non-finite weight-gradient partial (see slab_row_flag)
        for (int i = threadIdx.x; i < G::N_DW; i += blockDim.x) {
            const float val = img[i] * invS;
            row[i] = val;
            rbad |= !isfinite(val);
        }
        slab_row_flag(nonfinite, rbad);
        if (level_l1 && threadIdx.x < 16) atomicAdd(level_l1 + threadIdx.x, l1_part[threadIdx.x]);
    }
}

// ---------------------------------------------------------------- cooperative backward (W = 128)
// Round 5: the width-128 field (configs 3/4, MF-NeRF's benchmark field) in ONE pass, the W = 64
// cooperative scheme scaled up.  The per-wave backward (removed) held all weight-gradient tiles but dWr2's
// 16 (one wave per SIMD, 448 accumulator registers do not fit), and a second pass recomputed the
// forward and dR2 for them: 0.46 ms of the 1.67 ms mf128 step (profiles/r04_final_bench_mf128.json).
// Here the 28 tiles are split over the workgroup's 4 waves -- 7 each, 112 accumulator registers
// pinned to AGPRs -- every wave runs the forward and the data-gradient chain of its own 32-sample
// tile, writes the weight-gradient operands (transposed T chunks) stage by stage into its images, and
// after a barrier accumulates ITS tiles of that stage over all four waves' tiles, waves 0..3 in order
// (a fixed summation order: deterministic).  Tiles per wave w:
//   dWr3[w] (16 x 32 block w of the 16 x 128), dWr2[w][0..3] (row block w), dWr1[w],
//   and dW2[w] (waves 0, 1) or dW1[w - 2] (waves 2, 3).
// All 106 fragments stay in LDS (106 KB) beside 6 images per wave (48 KB): one workgroup per CU.
// Stages (images per wave): S1 dO, R2 x4 | S2a dR2 x4, R1[0..1] | S2b R1[2..3] over R1[0..1] |
// S3 dR1 x4, [SH;h] | S4 dh, Y1 x2 | S5 dY1 x2, X.
constexpr int COOP128_SLOTS = 6;
constexpr size_t COOP128_LDS = (size_t)Geo<128>::N * FRAG_HALFS * 2 + (size_t)4 * COOP128_SLOTS * TILE_BYTES;
static_assert(COOP128_LDS <= 160 * 1024, "one cooperative W = 128 workgroup per CU");

template <bool PLANAR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1))) void field_bw_coop128_kernel(
    const _Float16* __restrict__ feat, int64_t plane_stride, const float* __restrict__ dirs, int64_t n,
    const int32_t* __restrict__ n_dev, const _Float16* __restrict__ packed, const float* __restrict__ dL_dsigma,
    const float* __restrict__ dL_drgb, float grad_scale, const float* __restrict__ scale_dev,
    float* __restrict__ dL_dfeat, float* __restrict__ slab, int32_t* __restrict__ nonfinite, float* __restrict__ level_l1) {
    constexpr int W = 128;
    using G = Geo<W>;
    constexpr int MT = G::MT;
    constexpr int oR1 = N_XYZ_PARAMS, oR2 = oR1 + W * 32, oR3 = oR2 + W * W;
    constexpr size_t IMG_OFF = (size_t)G::N * FRAG_HALFS * 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    _Float16* lds_base = reinterpret_cast<_Float16*>(smem);
    load_frags_bw<W, 4>(lds_base, packed);
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (uniform)
    const int r = lane & 31, h = lane >> 5;
    const float S = scale_dev ? *scale_dev : grad_scale, invS = 1.0f / S;
    const f32x16 z = {};
    f32x16 a_r3 = z, a_r1 = z, a_x = z, a_r2[MT];  // this wave's seven tiles (table above)
#pragma unroll
    for (int i = 0; i < MT; ++i) a_r2[i] = z;
    const int64_t nn = n_dev ? min<int64_t>(n, (int64_t)*n_dev) : n;
    const int64_t tiles = div_up<int64_t>(nn, 32);
    const int64_t groups = div_up<int64_t>(tiles, 4);  // group g = tiles 4g .. 4g+3, one per wave
    struct BwIn { TileIn I; float gs, g0, g1, g2; bool live; };
    BwIn nx;
    // as field_bw_coop_kernel: every lane loads (index clamped), the incoming gradients are zeroed
    // where the sample is out of range or on lanes h == 1 -- an idle wave's tile contributes zeros
    auto fetch = [&](int64_t tile, BwIn& o) {
        const int64_t s = tile * 32 + r;
        const bool v = s < nn && h == 0;
        const int64_t sc = max<int64_t>(0, min<int64_t>(s, nn - 1));
        if constexpr (PLANAR) {
            const uint32_t* Pp = reinterpret_cast<const uint32_t*>(feat);
            uint32_t u[8];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                u[k] = Pp[(int64_t)(4 * h + k) * plane_stride + sc];
                u[4 + k] = Pp[(int64_t)(8 + 4 * h + k) * plane_stride + sc];
            }
            o.I.x[0] = *reinterpret_cast<const half8*>(&u[0]);
            o.I.x[1] = *reinterpret_cast<const half8*>(&u[4]);
        } else {
            const half8* row = reinterpret_cast<const half8*>(feat + sc * 32);
            o.I.x[0] = row[h];
            o.I.x[1] = row[2 + h];
        }
        o.I.d[0] = dirs[3 * sc]; o.I.d[1] = dirs[3 * sc + 1]; o.I.d[2] = dirs[3 * sc + 2];
        o.gs = dL_dsigma[sc]; o.g0 = dL_drgb[3 * sc]; o.g1 = dL_drgb[3 * sc + 1]; o.g2 = dL_drgb[3 * sc + 2];
        o.live = v;
    };
    auto zero_grads = [&](BwIn& o) {
        o.gs = o.live ? o.gs : 0.0f;
        o.g0 = o.live ? o.g0 : 0.0f;
        o.g1 = o.live ? o.g1 : 0.0f;
        o.g2 = o.live ? o.g2 : 0.0f;
    };
    if ((int64_t)blockIdx.x < groups) fetch(4 * (int64_t)blockIdx.x + wid, nx);
    bool bad = false;
    float l1a[4] = {0.f, 0.f, 0.f, 0.f}, l1b[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t g = blockIdx.x; g < groups; g += gridDim.x) {
        int opaque = 0;
        asm volatile("" : "+s"(opaque));
        const _Float16* lds = lds_base + opaque;
        _Float16* area = lds_base + opaque + IMG_OFF / 2;
        auto slot = [&](int u, int k) { return area + (u * COOP128_SLOTS + k) * TILE_HALFS; };
        auto put2 = [&](_Float16* sl, const half8* v) {  // a 32-channel tile as two perm chunks
            t_put(sl, lane, v[0], 0, true);
            t_put(sl, lane, v[1], 4, true);
        };
        const int64_t tile = 4 * g + wid;
        BwIn in = nx;
        zero_grads(in);
        fetch(4 * (g + (int64_t)gridDim.x) + wid, nx);  // (clamped past the end)
        const bool valid = tile * 32 + r < nn;
        FwdTile<W> T;
        forward_tiles<W, false, 1>(lds, lane, &in.I, &valid, &T);
        half8 dOb;
        {
            f32x16 dO = z;
            dO[0] = in.g0 * S * T.rgb[0] * (1.0f - T.rgb[0]);
            dO[1] = in.g1 * S * T.rgb[1] * (1.0f - T.rgb[1]);
            dO[2] = in.g2 * S * T.rgb[2] * (1.0f - T.rgb[2]);
            dOb = pack8<0, false>(dO);
        }
        //    dR2 = Wr3^T dO, masked by R2 > 0
        half8 dr2p[MT][2];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const f32x16 a = mfma(lds_frag(lds, G::B5 + mt, lane), dOb, z);
            dr2p[mt][0] = relu_mask8(pack8<0, false>(a), T.r2[mt][0]);
            dr2p[mt][1] = relu_mask8(pack8<8, false>(a), T.r2[mt][1]);
        }
        // ---- S1: dO, R2 -> dWr3[w]
        t_put(slot(wid, 0), lane, dOb, 0, true);  // (channels 16..31 stale: rows 16..31 of dWr3, dropped)
#pragma unroll
        for (int i = 0; i < MT; ++i) put2(slot(wid, 1 + i), T.r2[i]);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) acc_tile(a_r3, s_get(slot(u, 0), lane), s_get(slot(u, 1 + wid), lane));
        //    dR1 = Wr2^T dR2, masked by R1 > 0
        half8 dr1p[MT][2];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            f32x16 a = z;
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int k = 0; k < 2; ++k) a = mfma(lds_frag(lds, G::B4 + mt * G::KC + t * 2 + k, lane), dr2p[t][k], a);
            dr1p[mt][0] = relu_mask8(pack8<0, false>(a), T.r1[mt][0]);
            dr1p[mt][1] = relu_mask8(pack8<8, false>(a), T.r1[mt][1]);
        }
        __syncthreads();
        // ---- S2a: dR2, R1[0..1] -> dWr2[w][0..1]
#pragma unroll
        for (int o = 0; o < MT; ++o) put2(slot(wid, o), dr2p[o]);
        put2(slot(wid, 4), T.r1[0]);
        put2(slot(wid, 5), T.r1[1]);
        //    d[SH;h] = Wr1^T dR1 (rows 16..31 = dh) + TruncExp backward into h[0]
        half8 dhb;
        {
            f32x16 dsh = z;
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int k = 0; k < 2; ++k) dsh = mfma(lds_frag(lds, G::B3 + t * 2 + k, lane), dr1p[t][k], dsh);
            const float dh0 = in.gs * S * __expf(fminf(fmaxf(T.h0, -15.0f), 15.0f));
            dsh[8] = h == 0 ? dsh[8] + dh0 : dsh[8];
            dhb = pack8<8, false>(dsh);
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const SOp d = s_get(slot(u, wid), lane);
            acc_tile(a_r2[0], d, s_get(slot(u, 4), lane));
            acc_tile(a_r2[1], d, s_get(slot(u, 5), lane));
        }
        //    dY1 = W2^T dh, masked by Y1 > 0; dX = W1^T dY1
        half8 dy1p[2][2];
        f32x16 dx = z;
        {
            const f32x16 a0 = mfma(lds_frag(lds, G::B2 + 0, lane), dhb, z);
            const f32x16 a1 = mfma(lds_frag(lds, G::B2 + 1, lane), dhb, z);
            dy1p[0][0] = relu_mask8(pack8<0, false>(a0), T.y1[0][0]);
            dy1p[0][1] = relu_mask8(pack8<8, false>(a0), T.y1[0][1]);
            dy1p[1][0] = relu_mask8(pack8<0, false>(a1), T.y1[1][0]);
            dy1p[1][1] = relu_mask8(pack8<8, false>(a1), T.y1[1][1]);
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int k = 0; k < 2; ++k) dx = mfma(lds_frag(lds, G::B1 + t * 2 + k, lane), dy1p[t][k], dx);
        }
        __syncthreads();
        // ---- S2b: R1[2..3] over R1[0..1] -> dWr2[w][2..3] (dR2 still in slots 0..3)
        put2(slot(wid, 4), T.r1[2]);
        put2(slot(wid, 5), T.r1[3]);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const SOp d = s_get(slot(u, wid), lane);
            acc_tile(a_r2[2], d, s_get(slot(u, 4), lane));
            acc_tile(a_r2[3], d, s_get(slot(u, 5), lane));
        }
        // dX = W1^T dY1 -> global fp32 (features (i&3)+8(i>>2)+4h), this wave's own tile
        {
            const int64_t s = tile * 32 + r;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 o = make_float4(dx[4 * q] * invS, dx[4 * q + 1] * invS, dx[4 * q + 2] * invS, dx[4 * q + 3] * invS);
                bad |= !(isfinite(o.x) && isfinite(o.y) && isfinite(o.z) && isfinite(o.w));
                if (s < nn) reinterpret_cast<float4*>(dL_dfeat + s * 32)[2 * q + h] = o;
                l1a[q] += fabsf(o.x) + fabsf(o.y);
                l1b[q] += fabsf(o.z) + fabsf(o.w);
            }
        }
        __syncthreads();
        // ---- S3: dR1, [SH;h] -> dWr1[w]
#pragma unroll
        for (int o = 0; o < MT; ++o) put2(slot(wid, o), dr1p[o]);
        t_put(slot(wid, 4), lane, T.sh, 0, false);
        t_put(slot(wid, 4), lane, T.hb, 4, true);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) acc_tile(a_r1, s_get(slot(u, wid), lane), s_get(slot(u, 4), lane));
        __syncthreads();
        // ---- S4: dh, Y1 -> dW2 (waves 0, 1)
        t_put(slot(wid, 0), lane, dhb, 0, true);  // (channels 16..31 stale: rows of dW2 dropped)
        put2(slot(wid, 1), T.y1[0]);
        put2(slot(wid, 2), T.y1[1]);
        __syncthreads();
        if (wid < 2) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc_tile(a_x, s_get(slot(u, 0), lane), s_get(slot(u, 1 + wid), lane));
        }
        __syncthreads();
        // ---- S5: dY1, X -> dW1 (waves 2, 3)
        put2(slot(wid, 0), dy1p[0]);
        put2(slot(wid, 1), dy1p[1]);
        t_put(slot(wid, 2), lane, T.x[0], 0, false);
        t_put(slot(wid, 2), lane, T.x[1], 4, false);
        __syncthreads();
        if (wid >= 2) {
#pragma unroll
            for (int u = 0; u < 4; ++u) acc_tile(a_x, s_get(slot(u, wid - 2), lane), s_get(slot(u, 2), lane));
        }
        __syncthreads();  // the images are rewritten by the next group's S1
    }
    if (nonfinite && __any(bad) && lane == 0) atomicOr(nonfinite, 1);

    // ---- epilogue: each tile stored by its owner wave (disjoint, every entry once) -> one slab row
    float* row = slab + (int64_t)blockIdx.x * G::N_DW;
    {
        constexpr int N_IMG = G::N_DW;
        static_assert((size_t)N_IMG * 4 + 64 <= IMG_OFF, "reduction image must fit the fragment area");
        xdl_drain();
        __syncthreads();
        float* img = reinterpret_cast<float*>(smem);
        float* l1_part = img + N_IMG;
        if (threadIdx.x < 16) l1_part[threadIdx.x] = 0.0f;
        __syncthreads();
        if (level_l1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float a = l1a[q], b = l1b[q];
#pragma unroll
                for (int off = 16; off > 0; off >>= 1) { a += __shfl_xor(a, off, 64); b += __shfl_xor(b, off, 64); }
                if (r == 0) { atomicAdd(l1_part + 4 * q + 2 * h, a); atomicAdd(l1_part + 4 * q + 2 * h + 1, b); }
            }
        }
        dw_add32(img + oR3, a_r3, 0, wid, 16, W, lane, true);
        dw_add32(img + oR1, a_r1, wid, 0, W, 32, lane, true);
#pragma unroll
        for (int i = 0; i < MT; ++i) dw_add32(img + oR2, a_r2[i], wid, i, W, W, lane, true);
        if (wid < 2) dw_add32(img + 64 * 32, a_x, 0, wid, 16, 64, lane, true);
        else dw_add32(img, a_x, wid - 2, 0, 64, 32, lane, true);
        __syncthreads();
        bool rbad = false;  // a non-finite weight-gradient partial (see slab_row_flag)
        for (int i = threadIdx.x; i < G::N_DW; i += blockDim.x) {
            const float val = img[i] * invS;
            row[i] = val;
            rbad |= !isfinite(val);
        }
        slab_row_flag(nonfinite, rbad);
        if (level_l1 && threadIdx.x < 16) atomicAdd(level_l1 + threadIdx.x, l1_part[threadIdx.x]);
    }
}

// grad[p] += sum over slab rows (fixed order: deterministic).  64 columns x 4 row groups per block.
template <int W>
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, int rows,
                                                          float* __restrict__ gx, float* __restrict__ gr,
                                                          int32_t* __restrict__ nonfinite, int store = 0) {
    // 64 parameters per block as 16 float4 columns x 16 row groups; each thread sums its rows
    // (rows/16, all loads in flight) and the 16 partials are added in a fixed tree order
    constexpr int N_DW = Geo<W>::N_DW;
    static_assert(N_DW % 4 == 0 && N_XYZ_PARAMS % 4 == 0, "float4 columns");
    __shared__ float4 part[16][16];
    const int c = threadIdx.x & 15, rg = threadIdx.x >> 4;
    const int p = blockIdx.x * 64 + 4 * c;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p < N_DW) {
        const float4* src = reinterpret_cast<const float4*>(slab + p);
        constexpr int RS = N_DW / 4;  // row stride in float4
        // 8 rows' loads issued before their adds (same order of adds): 512 slab rows (the coop
        // backward) are 4 round trips per thread instead of 32 -- measured 42 us beside the side
        // stream's march (r4e timeline), whose waves make every dependent round trip longer
        constexpr int U = 8;
        for (int b0 = rg; b0 < rows; b0 += 16 * U) {
            float4 v[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int b = b0 + 16 * k;
                v[k] = b < rows ? src[(int64_t)b * RS] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int k = 0; k < U; ++k)
                if (b0 + 16 * k < rows) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
        }
    }
    part[rg][c] = acc;
    __syncthreads();
    if (rg == 0 && p < N_DW) {
        float4 t[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) t[k] = part[k][c];
#pragma unroll
        for (int w = 8; w > 0; w >>= 1)
#pragma unroll
            for (int k = 0; k < w; ++k) {
                t[k].x += t[k + w].x; t[k].y += t[k + w].y; t[k].z += t[k + w].z; t[k].w += t[k + w].w;
            }
        const float v[4] = {t[0].x, t[0].y, t[0].z, t[0].w};
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = p + k;
            float* dst = q < N_XYZ_PARAMS ? gx + q : gr + (q - N_XYZ_PARAMS);
            *dst = store ? v[k] : *dst + v[k];
            bad |= !isfinite(v[k]);
        }
        if (nonfinite && bad) atomicOr(nonfinite, 1);
    }
}

constexpr int BW_BLOCKS = 256;  // one workgroup per CU (persistent)

// slab rows: W = 64 field_bw_coop_kernel (two workgroups per CU), W = 128 field_bw_coop128_kernel (one)
int bw_rows(int w) { return w == 64 ? COOP_BLOCKS : BW_BLOCKS; }

bool width_ok(int w) { return w == 64 || w == 128; }

int bad_width(int w) {
    mfn_set_error("field: rgb_width=%d unsupported (this build: 64 or 128)", w);
    return MFN_ERR_INVALID;
}

template <typename TP, int W>
void launch_pack(const TP* px, const TP* pr, void* packed, mfnerf_stream_t stream) {
    const int total = Geo<W>::N * FRAG_HALFS;
    hipLaunchKernelGGL((pack_kernel<TP, W>), dim3((total + 255) / 256), dim3(256), 0, stream, px, pr,
                       (_Float16*)packed);
}

template <int W>
void launch_fw(const void* feat, int64_t ps, const float* dirs, int64_t n, const int32_t* n_dev, const void* packed,
               int density_only, float* sigma, float* rgb, mfnerf_stream_t stream, const int32_t* cell = nullptr,
               float* cell_out = nullptr) {
    const int64_t tiles = div_up<int64_t>(n, 32);
    const int64_t want = div_up<int64_t>(tiles, 4);
    const unsigned blocks = (unsigned)(want < 2048 ? want : 2048);
    if (density_only)
        hipLaunchKernelGGL((field_fw_kernel<W, true>), dim3(blocks), dim3(FIELD_BLOCK), 8 * FRAG_HALFS * 2, stream,
                           (const _Float16*)feat, ps, dirs, n, n_dev, (const _Float16*)packed, sigma, rgb, cell,
                           cell_out);
    else
        hipLaunchKernelGGL((field_fw_kernel<W, false>), dim3(blocks), dim3(FIELD_BLOCK),
                           (size_t)Geo<W>::N_FW * FRAG_HALFS * 2, stream, (const _Float16*)feat, ps, dirs, n, n_dev,
                           (const _Float16*)packed, sigma, rgb, nullptr, nullptr);
}

// the cooperative backward of width W (its kernel pair, workgroups = slab rows, LDS), then the slab fold
// (unless deferred: grad_xyz null, mfnerf_field_bw_reduce folds the slab later)
template <int W>
int launch_bw(const void* feat, int64_t ps, const float* dirs, int64_t n, const int32_t* n_dev, const void* packed,
              const float* dL_dsigma, const float* dL_drgb, float grad_scale, const float* scale_dev, float* dL_dfeat,
              float* grad_xyz, float* grad_rgb, void* workspace, int32_t* nonfinite, float* level_l1,
              mfnerf_stream_t stream) {
    using K = decltype(&field_bw_coop_kernel<false>);
    constexpr K k0 = W == 64 ? field_bw_coop_kernel<false> : field_bw_coop128_kernel<false>;
    constexpr K k1 = W == 64 ? field_bw_coop_kernel<true> : field_bw_coop128_kernel<true>;
    constexpr size_t lds = W == 64 ? COOP_LDS : COOP128_LDS;
    const int rows = bw_rows(W);
    static const hipError_t attr = [] {
        const hipError_t a0 = hipFuncSetAttribute(reinterpret_cast<const void*>(k0),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(k1),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        return a0 != hipSuccess ? a0 : a1;
    }();
    if (attr != hipSuccess) {
        mfn_set_error("field_bw: cannot raise the LDS limit to %d bytes", (int)lds);
        return MFN_ERR_INVALID;
    }
    hipLaunchKernelGGL(ps > 0 ? k1 : k0, dim3(rows), dim3(256), lds, stream, (const _Float16*)feat, ps, dirs, n,
                       n_dev, (const _Float16*)packed, dL_dsigma, dL_drgb, grad_scale, scale_dev, dL_dfeat,
                       (float*)workspace, nonfinite, level_l1);
    if (grad_xyz)
        hipLaunchKernelGGL(slab_reduce_kernel<W>, dim3((Geo<W>::N_DW + 63) / 64), dim3(256), 0, stream,
                           (const float*)workspace, rows, grad_xyz, grad_rgb, nonfinite, 0);
    return MFN_OK;
}

}  // namespace

extern "C" {

int64_t mfnerf_field_packed_bytes(int rgb_width) {
    if (rgb_width == 64) return (int64_t)Geo<64>::N * FRAG_HALFS * 2;
    if (rgb_width == 128) return (int64_t)Geo<128>::N * FRAG_HALFS * 2;
    return -1;
}

int mfnerf_field_pack_weights(const float* params_xyz, const float* params_rgb, int rgb_width, void* packed,
                              mfnerf_stream_t stream) {
    if (!width_ok(rgb_width)) return bad_width(rgb_width);
    if (!params_xyz || !params_rgb || !packed) { mfn_set_error("field_pack_weights: null pointer"); return MFN_ERR_INVALID; }
    if (rgb_width == 64) launch_pack<float, 64>(params_xyz, params_rgb, packed, stream);
    else launch_pack<float, 128>(params_xyz, params_rgb, packed, stream);
    return mfn_check_launch("field_pack_weights");
}

int mfnerf_sh4_fw(const float* dirs01, int64_t n, void* out_f16, mfnerf_stream_t stream) {
    if (n < 0 || (n > 0 && (!dirs01 || !out_f16))) { mfn_set_error("sh4_fw: bad arguments"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    hipLaunchKernelGGL(sh4_fw_kernel, dim3((unsigned)div_up<int64_t>(n, 256)), dim3(256), 0, stream, dirs01, n,
                       (__half*)out_f16);
    return mfn_check_launch("sh4_fw");
}

int mfnerf_field_pack_weights_f16(const void* params_xyz_f16, const void* params_rgb_f16, int rgb_width, void* packed,
                                  mfnerf_stream_t stream) {
    if (!width_ok(rgb_width)) return bad_width(rgb_width);
    if (!params_xyz_f16 || !params_rgb_f16 || !packed) { mfn_set_error("field_pack_weights_f16: null pointer"); return MFN_ERR_INVALID; }
    const _Float16* px = (const _Float16*)params_xyz_f16;
    const _Float16* pr = (const _Float16*)params_rgb_f16;
    if (rgb_width == 64) launch_pack<_Float16, 64>(px, pr, packed, stream);
    else launch_pack<_Float16, 128>(px, pr, packed, stream);
    return mfn_check_launch("field_pack_weights_f16");
}

int mfnerf_field_fw(const void* feat_f16, int64_t feat_plane_stride, const float* dirs, int64_t n,
                    const int32_t* n_dev, const void* packed,
                    int rgb_width, int density_only, float* sigma, float* rgb, mfnerf_stream_t stream) {
    if (!width_ok(rgb_width)) return bad_width(rgb_width);
    if (n < 0 || (feat_plane_stride != 0 && feat_plane_stride < n)) { mfn_set_error("field_fw: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!feat_f16 || !packed || !sigma || (!density_only && (!dirs || !rgb))) {
        mfn_set_error("field_fw: null pointer"); return MFN_ERR_INVALID;
    }
    if (rgb_width == 64) launch_fw<64>(feat_f16, feat_plane_stride, dirs, n, n_dev, packed, density_only, sigma, rgb, stream);
    else launch_fw<128>(feat_f16, feat_plane_stride, dirs, n, n_dev, packed, density_only, sigma, rgb, stream);
    return mfn_check_launch("field_fw");
}

int mfnerf_field_fw_density_scatter(const void* feat_f16, int64_t feat_plane_stride, int64_t n, const int32_t* n_dev,
                                    const void* packed, int rgb_width, float* sigma, const int32_t* cell_idx,
                                    float* tmp, mfnerf_stream_t stream) {
    if (!width_ok(rgb_width)) return bad_width(rgb_width);
    if (n < 0 || (feat_plane_stride != 0 && feat_plane_stride < n)) {
        mfn_set_error("field_fw_density_scatter: bad size");
        return MFN_ERR_INVALID;
    }
    if (n == 0) return MFN_OK;
    if (!feat_f16 || !packed || !sigma || !cell_idx || !tmp) {
        mfn_set_error("field_fw_density_scatter: null pointer");
        return MFN_ERR_INVALID;
    }
    if (rgb_width == 64) launch_fw<64>(feat_f16, feat_plane_stride, nullptr, n, n_dev, packed, 1, sigma, nullptr, stream, cell_idx, tmp);
    else launch_fw<128>(feat_f16, feat_plane_stride, nullptr, n, n_dev, packed, 1, sigma, nullptr, stream, cell_idx, tmp);
    return mfn_check_launch("field_fw_density_scatter");
}

int mfnerf_field_bw_slab_rows(int rgb_width) {
    return rgb_width == 64 ? bw_rows(64) : rgb_width == 128 ? BW_BLOCKS : -1;
}

int64_t mfnerf_field_bw_workspace(int64_t n, int rgb_width) {
    (void)n;
    if (rgb_width == 64) return (int64_t)bw_rows(64) * Geo<64>::N_DW * 4;
    if (rgb_width == 128) return (int64_t)BW_BLOCKS * Geo<128>::N_DW * 4;
    return -1;
}

int mfnerf_field_bw(const void* feat_f16, int64_t feat_plane_stride, const float* dirs, int64_t n,
                    const int32_t* n_dev, const void* packed,
                    int rgb_width, const float* dL_dsigma, const float* dL_drgb, float grad_scale, float* dL_dfeat,
                    float* grad_xyz, float* grad_rgb, void* workspace, mfnerf_amp_state* amp, float* level_l1,
                    mfnerf_stream_t stream) {
    if (!width_ok(rgb_width)) return bad_width(rgb_width);
    if (n < 0 || !(grad_scale >= 0.0f) || (grad_scale == 0.0f && !amp) ||
        (feat_plane_stride != 0 && feat_plane_stride < n)) {
        mfn_set_error("field_bw: bad size, plane stride or grad_scale (0 = dynamic needs amp)"); return MFN_ERR_INVALID;
    }
    if (n == 0) return MFN_OK;
    if (!feat_f16 || !dirs || !packed || !dL_dsigma || !dL_drgb || !dL_dfeat || !workspace || (!grad_xyz != !grad_rgb)) {
        mfn_set_error("field_bw: null pointer"); return MFN_ERR_INVALID;
    }
    int32_t* nonfinite = amp ? &amp->nonfinite : nullptr;
    const float* scale_dev = grad_scale == 0.0f ? &amp->scale : nullptr;
    int st;
    if (rgb_width == 128)
        st = launch_bw<128>(feat_f16, feat_plane_stride, dirs, n, n_dev, packed, dL_dsigma, dL_drgb, grad_scale,
                               scale_dev, dL_dfeat, grad_xyz, grad_rgb, workspace, nonfinite, level_l1, stream);
    else
        st = launch_bw<64>(feat_f16, feat_plane_stride, dirs, n, n_dev, packed, dL_dsigma, dL_drgb, grad_scale,
                              scale_dev, dL_dfeat, grad_xyz, grad_rgb, workspace, nonfinite, level_l1, stream);
    if (st != MFN_OK) return st;
    return mfn_check_launch("field_bw");
}

static int field_bw_fold(int rgb_width, const void* workspace, float* grad_xyz, float* grad_rgb, int32_t* nonfinite,
                         int store, mfnerf_stream_t stream) {
    if (!width_ok(rgb_width)) return bad_width(rgb_width);
    if (!workspace || !grad_xyz || !grad_rgb) { mfn_set_error("field_bw_reduce: null pointer"); return MFN_ERR_INVALID; }
    if (rgb_width == 64)
        hipLaunchKernelGGL(slab_reduce_kernel<64>, dim3((Geo<64>::N_DW + 63) / 64), dim3(256), 0, stream,
                           (const float*)workspace, bw_rows(64), grad_xyz, grad_rgb, nonfinite, store);
    else
        hipLaunchKernelGGL(slab_reduce_kernel<128>, dim3((Geo<128>::N_DW + 63) / 64), dim3(256), 0, stream,
                           (const float*)workspace, BW_BLOCKS, grad_xyz, grad_rgb, nonfinite, store);
    return mfn_check_launch("field_bw_reduce");
}

int mfnerf_field_bw_reduce(int rgb_width, const void* workspace, float* grad_xyz, float* grad_rgb,
                           int32_t* nonfinite, mfnerf_stream_t stream) {
    return field_bw_fold(rgb_width, workspace, grad_xyz, grad_rgb, nonfinite, 0, stream);
}

int mfnerf_field_bw_reduce_store(int rgb_width, const void* workspace, float* grad_xyz, float* grad_rgb,
                                 int32_t* nonfinite, mfnerf_stream_t stream) {
    return field_bw_fold(rgb_width, workspace, grad_xyz, grad_rgb, nonfinite, 1, stream);
}


}  // extern "C"
