// mfma_pack.hpp -- fp32 MFMA accumulator halves -> f16 B operands, with the ReLU and the ReLU
// backward mask done on the packed halves (shared by field.hip and mlp.hip).
#pragma once
#include <cstdint>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace mfn {

typedef short short2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
union H8 { half8 h; half2v p[4]; short2v s[4]; uint32_t w[4]; };

// ReLU applied AFTER the round to f16, on the packed halves as int16 (v_pk_max_i16): an f16 and its
// bits order the same way for non-negative values and every negative f16 (-0 included) is a
// negative int16, so max(bits, 0) == f16(max(v, 0)) for every finite v -- 4 packed ops per 8 values
// instead of a canonicalising v_max_f32 pair per value (IEEE mode).  A NaN stays NaN here.
template <int BASE, bool RELU>
__device__ __forceinline__ half8 pack8(const f32x16& a) {
    H8 r;
#pragma unroll
    for (int w = 0; w < 4; ++w) {  // v_cvt_pk_f16_f32 (round to nearest even) per pair
        const float2v p = {a[BASE + 2 * w], a[BASE + 2 * w + 1]};
        r.p[w] = __builtin_convertvector(p, half2v);
    }
    if (RELU) {
        const short2v zero = {0, 0};
#pragma unroll
        for (int w = 0; w < 4; ++w) r.s[w] = __builtin_elementwise_max(r.s[w], zero);
    }
    return r.h;
}

// zero the packed dY halves where the forward activation y (f16, post-ReLU: +0 or positive, never
// negative) is not positive: dY * min(bits(y), 1) on the packed halves (v_pk_min_u16 +
// v_pk_mul_lo_u16), bit-identical to selecting on (float)y > 0 before the round to f16
__device__ __forceinline__ half8 relu_mask8(const half8& d, const half8& y) {
    H8 D, Y;
    D.h = d;
    Y.h = y;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t m;
        // the 1s come from a register: an inline constant of a packed op feeds only the low half
        asm("v_pk_min_u16 %0, %1, %3\n\tv_pk_mul_lo_u16 %0, %2, %0"
            : "=&v"(m)
            : "v"(Y.w[w]), "v"(D.w[w]), "v"(0x00010001u));
        D.w[w] = m;
    }
    return D.h;
}

}  // namespace mfn
