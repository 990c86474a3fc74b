// mlp.hip -- a standalone tiny-cuda-nn FullyFusedMLP (bias-free, ReLU hidden layers, output
// activation None or Sigmoid, fp16 operands / fp32 accumulation) on gfx950 MFMA, for the modules
// MF-NeRF builds one by one (models/networks.py:36-79: xyz_encoder's network 32 -> 64 -> 16 and
// rgb_net 32 -> W -> W -> 3), i.e. what tinycudann.Network / NetworkWithInputEncoding compute when
// the reference's own networks.py runs on this library (module swap).  The training
// step does not use these kernels: it runs both MLPs fused with the SH encoding and TruncExp in
// field.hip.  Same MFMA layout as field.hip (v_mfma_f32_32x32x16_f16; one wave = 32 samples;
// activations TRANSPOSED -- channel on the MFMA row, sample on the lane -- so a layer's
// accumulator, activated and packed, is the next layer's B operand):
//   forward : x (n, 32) f16 -> out (n, 16) f16 (tcnn pads the output width to 16);
//   backward: recompute, chain the data gradients through the transposed weights (A fragments
//             pre-permuted to the accumulator order), write dL/dx (n, 32) f32 and, per layer, the
//             layer input and the pre-activation gradient transposed (channel-major f16); the
//             weight gradients dW = dZ^T A then run as split-K MFMA GEMMs over sample chunks
//             (K = samples in both operands' registers, no transpose needed), partial tiles summed
//             over chunks in a fixed order: deterministic.
#include "common.hpp"
#include "mfma_pack.hpp"
#include "../../include/mfnerf.h"

using namespace mfn;

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int N_IN = 32, N_OUT = 16;  // the MF-NeRF networks' (padded) widths
constexpr int FRAG = 64 * 8;          // one A fragment: 64 lanes x 8 f16
constexpr int MLP_BLOCK = 256;

// Fragment table of a (W, NH) network: NH hidden layers of width W (layer 0: W x 32, layers
// 1..NH-1: W x W, layer NH: 16 x W).  Forward fragments (A = W_l), then backward (A = W_l^T).
template <int W, int NH>
struct MG {
    static constexpr int MT = W / 32, KC = W / 16;
    static constexpr int F0 = 0;                          // [mt][q]  natural k
    static constexpr int FH = F0 + 2 * MT;                // [(l-1)][mt][c] perm
    static constexpr int FO = FH + (NH - 1) * MT * KC;    // [c]      perm, rows 16..31 zero
    static constexpr int N_FW = FO + KC;
    static constexpr int BO = N_FW;                       // W_out^T [mt]       k = out (16), perm
    static constexpr int BH = BO + MT;                    // W_l^T   [(l-1)][mt][c]
    static constexpr int B0 = BH + (NH - 1) * MT * KC;    // W_0^T   [c]        rows = the 32 inputs
    static constexpr int N = B0 + KC;
    static constexpr int P_H = W * N_IN;                  // param offsets (floats)
    static constexpr int P_O = P_H + (NH - 1) * W * W;
    static constexpr int N_PARAMS = P_O + N_OUT * W;
    static constexpr int ACT_ROWS = N_IN + NH * W;        // transposed layer inputs per sample
    static constexpr int DZ_ROWS = NH * W + N_OUT;        // transposed pre-activation grads per sample
};

__device__ __forceinline__ int k_of(int j, int h, int perm) { return perm ? 8 * (j >> 2) + 4 * h + (j & 3) : 8 * h + j; }

// fragment f -> (matrix offset, rows, cols, transposed, row tile, k base, perm)
template <int W, int NH>
__device__ void frag_of(int f, int* off, int* rows, int* cols, int* tr, int* mt, int* kb, int* perm) {
    using G = MG<W, NH>;
    *tr = 0; *perm = 1; *mt = 0; *kb = 0;
    if (f < G::FH) { *off = 0; *rows = W; *cols = N_IN; *mt = f >> 1; *kb = 16 * (f & 1); *perm = 0; }
    else if (f < G::FO) {
        const int i = f - G::FH, l = i / (G::MT * G::KC), r = i % (G::MT * G::KC);
        *off = G::P_H + l * W * W; *rows = W; *cols = W; *mt = r / G::KC; *kb = 16 * (r % G::KC);
    } else if (f < G::BO) { *off = G::P_O; *rows = N_OUT; *cols = W; *kb = 16 * (f - G::FO); }
    else if (f < G::BH) { *off = G::P_O; *rows = N_OUT; *cols = W; *tr = 1; *mt = f - G::BO; }
    else if (f < G::B0) {
        const int i = f - G::BH, l = i / (G::MT * G::KC), r = i % (G::MT * G::KC);
        *off = G::P_H + l * W * W; *rows = W; *cols = W; *tr = 1; *mt = r / G::KC; *kb = 16 * (r % G::KC);
    } else { *off = 0; *rows = W; *cols = N_IN; *tr = 1; *kb = 16 * (f - G::B0); }
}

template <int W, int NH>
__global__ void mlp_pack_kernel(const float* __restrict__ params, _Float16* __restrict__ out) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= MG<W, NH>::N * FRAG) return;
    const int f = t / FRAG, lane = (t / 8) & 63, j = t & 7;
    int off, rows, cols, tr, mt, kb, perm;
    frag_of<W, NH>(f, &off, &rows, &cols, &tr, &mt, &kb, &perm);
    const int m = 32 * mt + (lane & 31), k = kb + k_of(j, lane >> 5, perm);
    float v = 0.0f;
    if (!tr) { if (m < rows && k < cols) v = params[off + m * cols + k]; }  // A = W: row out, k in
    else { if (k < rows && m < cols) v = params[off + k * cols + m]; }      // A = W^T: row in, k out
    out[t] = (_Float16)v;
}

__device__ __forceinline__ f32x16 mfma(const half8& a, const half8& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ half8 frag(const _Float16* lds, int f, int lane) {
    return *reinterpret_cast<const half8*>(lds + (f * 64 + lane) * 8);
}
// the forward of one 32-sample tile: the layer inputs as B operands (kept for the backward) and
// the output layer's accumulator (rows 0..15)
template <int W, int NH>
struct Fwd {
    half8 x[2];
    half8 a[NH][2 * (W / 32)];  // activated hidden layers, perm chunks
    f32x16 o;
};

template <int W, int NH>
__device__ __forceinline__ void forward(const _Float16* lds, int lane, Fwd<W, NH>& T) {
    using G = MG<W, NH>;
    const f32x16 z = {};
#pragma unroll
    for (int mt = 0; mt < G::MT; ++mt) {
        f32x16 a = mfma(frag(lds, G::F0 + 2 * mt, lane), T.x[0], z);
        a = mfma(frag(lds, G::F0 + 2 * mt + 1, lane), T.x[1], a);
        T.a[0][2 * mt] = pack8<0, true>(a);
        T.a[0][2 * mt + 1] = pack8<8, true>(a);
    }
#pragma unroll
    for (int l = 1; l < NH; ++l)
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) {
            f32x16 a = z;
#pragma unroll
            for (int c = 0; c < G::KC; ++c) a = mfma(frag(lds, G::FH + ((l - 1) * G::MT + mt) * G::KC + c, lane), T.a[l - 1][c], a);
            T.a[l][2 * mt] = pack8<0, true>(a);
            T.a[l][2 * mt + 1] = pack8<8, true>(a);
        }
    f32x16 o = z;
#pragma unroll
    for (int c = 0; c < G::KC; ++c) o = mfma(frag(lds, G::FO + c, lane), T.a[NH - 1][c], o);
    T.o = o;
}

__device__ __forceinline__ float out_act(float v, int oa) { return oa ? 1.0f / (1.0f + __expf(-v)) : v; }

__device__ __forceinline__ void load_frags(_Float16* lds, const _Float16* __restrict__ packed, int n) {
    const uint4* src = reinterpret_cast<const uint4*>(packed);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int i = threadIdx.x; i < n * 64; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

__device__ __forceinline__ void load_x(const _Float16* __restrict__ x, int64_t s, bool valid, int h, half8* xo) {
    const half8* row = reinterpret_cast<const half8*>(x + s * N_IN);
    xo[0] = valid ? row[h] : half8{};
    xo[1] = valid ? row[2 + h] : half8{};
}

template <int W, int NH, int OA>
__global__ __launch_bounds__(MLP_BLOCK) void mlp_fw_kernel(const _Float16* __restrict__ x, int64_t n,
                                                            const _Float16* __restrict__ packed,
                                                            _Float16* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    _Float16* lds = reinterpret_cast<_Float16*>(smem);
    load_frags(lds, packed, MG<W, NH>::N_FW);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5;
    const int64_t tiles = div_up<int64_t>(n, 32);
    for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile < tiles; tile += (int64_t)gridDim.x * 4) {
        const int64_t s = tile * 32 + (lane & 31);
        const bool valid = s < n;
        Fwd<W, NH> T;
        load_x(x, s, valid, h, T.x);
        forward<W, NH>(lds, lane, T);
        if (valid) {  // lane h holds rows 4h..4h+3 (elements 0..3) and 8+4h..11+4h (4..7)
            _Float16 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = (_Float16)out_act(T.o[i], OA);
            *reinterpret_cast<uint2*>(out + s * N_OUT + 4 * h) = *reinterpret_cast<const uint2*>(&v[0]);
            *reinterpret_cast<uint2*>(out + s * N_OUT + 8 + 4 * h) = *reinterpret_cast<const uint2*>(&v[4]);
        }
    }
}

// a perm-order B operand's element j of lane (s, h) is channel 16 c + k_of(j, h, 1): store it into
// a channel-major (rows, ld) f16 buffer
__device__ __forceinline__ void store_t(_Float16* __restrict__ buf, int64_t ld, int c, int h, int64_t s,
                                        const half8& v, int perm) {
#pragma unroll
    for (int j = 0; j < 8; ++j) buf[(int64_t)(16 * c + k_of(j, h, perm)) * ld + s] = v[j];
}

// backward of the data path; writes dL/dx and the transposed layer inputs (act: [x | a_0 .. a_NH-1])
// and pre-activation gradients (dz: [dz_0 .. dz_NH-1 | dz_out]) for the weight-gradient GEMMs.
// Rows beyond n (up to ld, a multiple of 32) are written as zeros.
template <int W, int NH, int OA>
__global__ __launch_bounds__(MLP_BLOCK) void mlp_bw_kernel(const _Float16* __restrict__ x, int64_t n, int64_t ld,
                                                            const _Float16* __restrict__ packed,
                                                            const _Float16* __restrict__ dout,
                                                            float* __restrict__ dx, _Float16* __restrict__ act,
                                                            _Float16* __restrict__ dz) {
    using G = MG<W, NH>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    _Float16* lds = reinterpret_cast<_Float16*>(smem);
    load_frags(lds, packed, G::N);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5;
    const f32x16 z = {};
    const int64_t tiles = ld / 32;
    for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile < tiles; tile += (int64_t)gridDim.x * 4) {
        const int64_t s = tile * 32 + (lane & 31);
        const bool valid = s < n;
        Fwd<W, NH> T;
        load_x(x, s, valid, h, T.x);
        forward<W, NH>(lds, lane, T);
        // dZ_out (perm order = the accumulator's rows): dL/dout x the output activation's derivative
        half8 d;
        {
            _Float16 g[8];
            if (valid) {
                *reinterpret_cast<uint2*>(&g[0]) = *reinterpret_cast<const uint2*>(dout + s * N_OUT + 4 * h);
                *reinterpret_cast<uint2*>(&g[4]) = *reinterpret_cast<const uint2*>(dout + s * N_OUT + 8 + 4 * h);
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v = valid ? (float)g[j] : 0.0f;
                if (OA) { const float y = out_act(T.o[j], 1); v *= y * (1.0f - y); }
                d[j] = (_Float16)v;
            }
        }
        // transposed layer inputs and the output layer's dZ
        _Float16* dzo = dz + (int64_t)NH * W * ld;
        store_t(dzo, ld, 0, h, s, d, 1);
#pragma unroll
        for (int q = 0; q < 2; ++q) store_t(act, ld, q, h, s, T.x[q], 0);
#pragma unroll
        for (int l = 0; l < NH; ++l)
#pragma unroll
            for (int c = 0; c < G::KC; ++c) store_t(act + (int64_t)(N_IN + l * W) * ld, ld, c, h, s, T.a[l][c], 1);
        // down the hidden layers: dZ_l = relu'(a_l) * (W_{l+1}^T dZ_{l+1})
        half8 dzc[2 * (W / 32)];
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt) {
            f32x16 a = mfma(frag(lds, G::BO + mt, lane), d, z);
            dzc[2 * mt] = relu_mask8(pack8<0, false>(a), T.a[NH - 1][2 * mt]);
            dzc[2 * mt + 1] = relu_mask8(pack8<8, false>(a), T.a[NH - 1][2 * mt + 1]);
        }
#pragma unroll
        for (int l = NH - 1; l >= 1; --l) {
#pragma unroll
            for (int c = 0; c < G::KC; ++c) store_t(dz + (int64_t)l * W * ld, ld, c, h, s, dzc[c], 1);
            half8 nx[2 * (W / 32)];
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt) {
                f32x16 a = z;
#pragma unroll
                for (int c = 0; c < G::KC; ++c) a = mfma(frag(lds, G::BH + ((l - 1) * G::MT + mt) * G::KC + c, lane), dzc[c], a);
                nx[2 * mt] = relu_mask8(pack8<0, false>(a), T.a[l - 1][2 * mt]);
                nx[2 * mt + 1] = relu_mask8(pack8<8, false>(a), T.a[l - 1][2 * mt + 1]);
            }
#pragma unroll
            for (int c = 0; c < G::KC; ++c) dzc[c] = nx[c];
        }
#pragma unroll
        for (int c = 0; c < G::KC; ++c) store_t(dz, ld, c, h, s, dzc[c], 1);
        // dL/dx = W_0^T dZ_0 (rows = the 32 inputs)
        f32x16 a = z;
#pragma unroll
        for (int c = 0; c < G::KC; ++c) a = mfma(frag(lds, G::B0 + c, lane), dzc[c], a);
        if (valid) {
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4)
                *reinterpret_cast<float4*>(dx + s * N_IN + 8 * g4 + 4 * h) =
                    make_float4(a[4 * g4], a[4 * g4 + 1], a[4 * g4 + 2], a[4 * g4 + 3]);
        }
    }
}

// weight-gradient GEMMs, split over sample chunks: workgroup k sums samples [k CH, (k+1) CH) of
// every layer's dW = dZ^T A into its slab row (n_params floats); both operands are channel-major,
// so a lane's 8 consecutive samples ARE its K elements (A: row = out channel, B: col = in channel)
constexpr int DW_CH = 1024;

template <int W, int NH>
__global__ __launch_bounds__(MLP_BLOCK) void mlp_dw_kernel(const _Float16* __restrict__ act,
                                                            const _Float16* __restrict__ dz, int64_t ld,
                                                            float* __restrict__ slab) {
    using G = MG<W, NH>;
    constexpr int T0 = G::MT, TH = G::MT * G::MT, TO = G::MT;  // 32x32 tiles per layer (in tile x out tile)
    constexpr int N_TILES = T0 + (NH - 1) * TH + TO;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, r = lane & 31;
    const int64_t s0 = (int64_t)blockIdx.x * DW_CH, s1 = min<int64_t>(s0 + DW_CH, ld);
    float* out = slab + (int64_t)blockIdx.x * G::N_PARAMS;
    for (int t = wid; t < N_TILES; t += MLP_BLOCK / 64) {
        int l, ot, it, rows, cols, poff;
        if (t < T0) { l = 0; ot = t; it = 0; rows = W; cols = N_IN; poff = 0; }
        else if (t < T0 + (NH - 1) * TH) {
            const int i = t - T0; l = 1 + i / TH; ot = (i % TH) / G::MT; it = i % G::MT; rows = W; cols = W;
            poff = G::P_H + (l - 1) * W * W;
        } else { l = NH; ot = 0; it = t - T0 - (NH - 1) * TH; rows = N_OUT; cols = W; poff = G::P_O; }
        const _Float16* dzr = dz + ((int64_t)l * W + 32 * ot + r) * ld;  // dZ_l row (out channel)
        const _Float16* arow = act + ((l == 0 ? 0 : N_IN + (int64_t)(l - 1) * W) + 32 * it + r) * ld;
        const bool rok = 32 * ot + r < rows;
        f32x16 acc = {};
        for (int64_t k = s0; k < s1; k += 16) {
            const half8 av = rok ? *reinterpret_cast<const half8*>(dzr + k + 8 * h) : half8{};
            const half8 bv = *reinterpret_cast<const half8*>(arow + k + 8 * h);
            acc = mfma(av, bv, acc);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = 32 * ot + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (row < rows) out[poff + row * cols + 32 * it + r] = acc[i];
        }
    }
}

// grad[p] += sum over chunks of slab[chunk][p], in chunk order
__global__ __launch_bounds__(256) void mlp_dw_reduce_kernel(const float* __restrict__ slab, int64_t chunks,
                                                            int n_params, float* __restrict__ grad) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_params) return;
    float s = 0.0f;
    for (int64_t c = 0; c < chunks; ++c) s += slab[c * n_params + p];
    grad[p] += s;
}

int mlp_check(int n_in, int width, int n_hidden, int n_out, const char* what) {
    if (n_in != N_IN || n_out < 1 || n_out > N_OUT || !(width == 64 || width == 128) || n_hidden < 1 || n_hidden > 2) {
        mfn_set_error("%s: unsupported network (n_in=%d must be 32, width=%d must be 64 or 128, n_hidden_layers=%d "
                      "must be 1 or 2, n_out=%d must be <= 16)", what, n_in, width, n_hidden, n_out);
        return MFN_ERR_INVALID;
    }
    return MFN_OK;
}

template <typename F>
auto mlp_dispatch(int width, int n_hidden, F&& f) -> decltype(f(MG<64, 1>{})) {
    if (width == 64 && n_hidden == 1) return f(MG<64, 1>{});
    if (width == 64 && n_hidden == 2) return f(MG<64, 2>{});
    if (width == 128 && n_hidden == 1) return f(MG<128, 1>{});
    return f(MG<128, 2>{});
}

template <int W, int NH>
constexpr int width_of(MG<W, NH>) { return W; }
template <int W, int NH>
constexpr int hidden_of(MG<W, NH>) { return NH; }

}  // namespace

extern "C" {

int64_t mfnerf_mlp_n_params(int n_in, int width, int n_hidden, int n_out) {
    if (mlp_check(n_in, width, n_hidden, n_out, "mlp_n_params")) return -1;
    return mlp_dispatch(width, n_hidden, [](auto g) { return (int64_t)decltype(g)::N_PARAMS; });
}

int64_t mfnerf_mlp_packed_bytes(int n_in, int width, int n_hidden, int n_out) {
    if (mlp_check(n_in, width, n_hidden, n_out, "mlp_packed_bytes")) return -1;
    return mlp_dispatch(width, n_hidden, [](auto g) { return (int64_t)decltype(g)::N; }) * FRAG * 2;
}

int mfnerf_mlp_pack(const float* params, int n_in, int width, int n_hidden, int n_out, void* packed,
                    mfnerf_stream_t stream) {
    int st = mlp_check(n_in, width, n_hidden, n_out, "mlp_pack");
    if (st) return st;
    if (!params || !packed) { mfn_set_error("mlp_pack: null pointer"); return MFN_ERR_INVALID; }
    return mlp_dispatch(width, n_hidden, [&](auto g) {
        using G = decltype(g);
        constexpr int W = width_of(G{}), NH = hidden_of(G{});
        const int total = G::N * FRAG;
        hipLaunchKernelGGL((mlp_pack_kernel<W, NH>), dim3((total + 255) / 256), dim3(256), 0, stream, params,
                           (_Float16*)packed);
        return mfn_check_launch("mlp_pack");
    });
}

int mfnerf_mlp_fw(const void* x_f16, int64_t n, const void* packed, int n_in, int width, int n_hidden, int n_out,
                  int output_sigmoid, void* out_f16, mfnerf_stream_t stream) {
    int st = mlp_check(n_in, width, n_hidden, n_out, "mlp_fw");
    if (st) return st;
    if (n < 0) { mfn_set_error("mlp_fw: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!x_f16 || !packed || !out_f16) { mfn_set_error("mlp_fw: null pointer"); return MFN_ERR_INVALID; }
    return mlp_dispatch(width, n_hidden, [&](auto g) {
        using G = decltype(g);
        constexpr int W = width_of(G{}), NH = hidden_of(G{});
        const int64_t want = div_up<int64_t>(n, 128), blocks = want < 4096 ? want : 4096;
        const size_t lds = (size_t)G::N_FW * FRAG * 2;
        auto k = output_sigmoid ? mlp_fw_kernel<W, NH, 1> : mlp_fw_kernel<W, NH, 0>;
        if (lds > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(MLP_BLOCK), lds, stream, (const _Float16*)x_f16, n,
                           (const _Float16*)packed, (_Float16*)out_f16);
        return mfn_check_launch("mlp_fw");
    });
}

int64_t mfnerf_mlp_bw_workspace(int64_t n, int n_in, int width, int n_hidden, int n_out) {
    if (mlp_check(n_in, width, n_hidden, n_out, "mlp_bw_workspace") || n < 0) return -1;
    return mlp_dispatch(width, n_hidden, [&](auto g) {
        using G = decltype(g);
        const int64_t ld = div_up<int64_t>(n > 0 ? n : 1, 32) * 32;
        const int64_t chunks = div_up<int64_t>(ld, DW_CH);
        return (int64_t)(G::ACT_ROWS + G::DZ_ROWS) * ld * 2 + chunks * (int64_t)G::N_PARAMS * 4;
    });
}

int mfnerf_mlp_bw(const void* x_f16, int64_t n, const void* packed, int n_in, int width, int n_hidden, int n_out,
                  int output_sigmoid, const void* dout_f16, float* dx, float* grad, void* workspace,
                  mfnerf_stream_t stream) {
    int st = mlp_check(n_in, width, n_hidden, n_out, "mlp_bw");
    if (st) return st;
    if (n < 0) { mfn_set_error("mlp_bw: bad size"); return MFN_ERR_INVALID; }
    if (n == 0) return MFN_OK;
    if (!x_f16 || !packed || !dout_f16 || !dx || !grad || !workspace) {
        mfn_set_error("mlp_bw: null pointer"); return MFN_ERR_INVALID;
    }
    if (((uintptr_t)dx | (uintptr_t)workspace) & 15) { mfn_set_error("mlp_bw: misaligned buffer"); return MFN_ERR_INVALID; }
    return mlp_dispatch(width, n_hidden, [&](auto g) {
        using G = decltype(g);
        constexpr int W = width_of(G{}), NH = hidden_of(G{});
        const int64_t ld = div_up<int64_t>(n, 32) * 32;
        const int64_t chunks = div_up<int64_t>(ld, DW_CH);
        _Float16* act = (_Float16*)workspace;
        _Float16* dz = act + (int64_t)G::ACT_ROWS * ld;
        float* slab = (float*)(dz + (int64_t)G::DZ_ROWS * ld);  // 16-B aligned: ld is a multiple of 32
        const int64_t want = div_up<int64_t>(ld, 128), blocks = want < 4096 ? want : 4096;
        const size_t lds = (size_t)G::N * FRAG * 2;
        auto k = output_sigmoid ? mlp_bw_kernel<W, NH, 1> : mlp_bw_kernel<W, NH, 0>;
        if (lds > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(MLP_BLOCK), lds, stream, (const _Float16*)x_f16, n, ld,
                           (const _Float16*)packed, (const _Float16*)dout_f16, dx, act, dz);
        hipLaunchKernelGGL((mlp_dw_kernel<W, NH>), dim3((unsigned)chunks), dim3(MLP_BLOCK), 0, stream,
                           (const _Float16*)act, (const _Float16*)dz, ld, slab);
        hipLaunchKernelGGL(mlp_dw_reduce_kernel, dim3((G::N_PARAMS + 255) / 256), dim3(256), 0, stream, slab, chunks,
                           (int)G::N_PARAMS, grad);
        return mfn_check_launch("mlp_bw");
    });
}

}  // extern "C"
