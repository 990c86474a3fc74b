// field_pack.hpp -- the MFMA weight-fragment layout of field.hip (and the repack that builds it),
// shared with grid.hip, whose optimizer tail repacks the MLP weights in its own launch.
#pragma once

#include <hip/hip_runtime.h>

namespace mfn_field {

constexpr int N_XYZ_PARAMS = 64 * 32 + 16 * 64;
constexpr int FRAG_HALFS = 64 * 8;  // one A fragment: 64 lanes x 8 f16 (1 KiB)

// Fragment table for rgb width W: MT = W/32 row tiles, KC = W/16 K chunks of a W-wide input.
template <int W>
struct Geo {
    static constexpr int MT = W / 32, KC = W / 16;
    static constexpr int F1 = 0;             // W1  (64x32)  [mt*2+q]  natural, kbase 16q
    static constexpr int F2 = 4;             // W2  (16x64)  [t*2+q]   perm, kbase 32t+16q
    static constexpr int F3 = 8;             // Wr1 (Wx32)   [mt*2+q]  q=0 natural kbase 0 (SH); q=1 perm kbase 16 (h)
    static constexpr int F4 = F3 + 2 * MT;   // Wr2 (WxW)    [mt*KC+c] perm, kbase 16c
    static constexpr int F5 = F4 + MT * KC;  // Wr3 (16xW)   [c]       perm
    static constexpr int B5 = F5 + KC;       // Wr3^T (Wx16) [mt]      perm kbase 0
    static constexpr int B4 = B5 + MT;       // Wr2^T        [mt*KC+c]
    static constexpr int B3 = B4 + MT * KC;  // Wr1^T (32xW) [c]
    static constexpr int B2 = B3 + KC;       // W2^T  (64x16) [mt]     perm kbase 0
    static constexpr int B1 = B2 + 2;        // W1^T  (32x64) [t*2+q]
    static constexpr int N = B1 + 4;         // 44 (W = 64), 106 (W = 128)
    static constexpr int N_FW = B5;          // the forward's fragments
    static constexpr int N_RGB = W * 32 + W * W + 16 * W;
    static constexpr int N_DW = N_XYZ_PARAMS + N_RGB;  // weight-gradient floats (one slab row)
};

struct FragSpec { int mat, trans, mtile, kbase, perm; };

template <int W>
__device__ FragSpec frag_spec(int f) {
    using G = Geo<W>;
    FragSpec s{0, 0, 0, 0, 1};
    if (f < G::F2) { s.mat = 0; s.mtile = f >> 1; s.kbase = 16 * (f & 1); s.perm = 0; }
    else if (f < G::F3) { int i = f - G::F2; s.mat = 1; s.kbase = 32 * (i >> 1) + 16 * (i & 1); }
    else if (f < G::F4) { int i = f - G::F3; s.mat = 2; s.mtile = i >> 1; s.kbase = 16 * (i & 1); s.perm = i & 1; }
    else if (f < G::F5) { int i = f - G::F4; s.mat = 3; s.mtile = i / G::KC; s.kbase = 16 * (i % G::KC); }
    else if (f < G::B5) { int i = f - G::F5; s.mat = 4; s.kbase = 16 * i; }
    else if (f < G::B4) { s.mat = 4; s.trans = 1; s.mtile = f - G::B5; s.kbase = 0; }
    else if (f < G::B3) { int i = f - G::B4; s.mat = 3; s.trans = 1; s.mtile = i / G::KC; s.kbase = 16 * (i % G::KC); }
    else if (f < G::B2) { int i = f - G::B3; s.mat = 2; s.trans = 1; s.kbase = 16 * i; }
    else if (f < G::B1) { s.mat = 1; s.trans = 1; s.mtile = f - G::B2; s.kbase = 0; }
    else { int i = f - G::B1; s.mat = 0; s.trans = 1; s.kbase = 16 * i; }
    return s;
}

// weight matrices, row-major (out, in) in the tcnn params vectors
template <int W, typename TP>
__device__ __forceinline__ void mat_info(int mat, const TP* px, const TP* pr, const TP** p, int* rows, int* cols) {
    switch (mat) {
        case 0: *p = px; *rows = 64; *cols = 32; break;
        case 1: *p = px + 64 * 32; *rows = 16; *cols = 64; break;
        case 2: *p = pr; *rows = W; *cols = 32; break;
        case 3: *p = pr + W * 32; *rows = W; *cols = W; break;
        default: *p = pr + W * 32 + W * W; *rows = 16; *cols = W; break;
    }
}

// k index carried by element j of lane half h (natural B order, or accumulator-as-operand order)
__device__ __forceinline__ int k_of(int j, int h, int perm) { return perm ? 8 * (j >> 2) + 4 * h + (j & 3) : 8 * h + j; }

// one element t of the packed blob (t < Geo<W>::N * FRAG_HALFS) from the row-major weights
template <typename TP, int W>
__device__ __forceinline__ void pack_elem(int t, const TP* __restrict__ px, const TP* __restrict__ pr,
                                          _Float16* __restrict__ out) {
    const int f = t / FRAG_HALFS, lane = (t / 8) & 63, j = t & 7;
    const FragSpec s = frag_spec<W>(f);
    const int r = lane & 31, h = lane >> 5;
    const int m = 32 * s.mtile + r, k = s.kbase + k_of(j, h, s.perm);
    const TP* p; int rows, cols;
    mat_info<W>(s.mat, px, pr, &p, &rows, &cols);
    float v = 0.0f;
    if (!s.trans) { if (m < rows && k < cols) v = (float)p[m * cols + k]; }
    else { if (k < rows && m < cols) v = (float)p[k * cols + m]; }
    out[t] = (_Float16)v;
}

}  // namespace mfn_field
