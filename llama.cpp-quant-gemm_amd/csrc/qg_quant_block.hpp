// qg_quant_block.hpp — one 32-element FP32 -> Q8_1 block, reference semantics (device side).
//
// Shared by the standalone quantizer (qg_quantize.hip) and the fused-activation GEMV prologue
// (qg_gemv_kernel.hpp, AIN != 0), so both produce the same bytes:
//   include/quantize.h:165-193 (variant 0): d = amax/127, id = 1/d, q = clamp(roundf(x*id), -128, 127),
//     s = sum(x) accumulated in element order, both stored as f16 (RNE, as __float2half);
//   tests/framework/test_framework.cuh:195-225 (variant 1): q clamped to +-127, s = d * sum(q).
// roundf is round-half-away-from-zero; the division and reciprocal are IEEE-correct (the library
// builds with -fhip-fp32-correctly-rounded-divide-sqrt).
//   kernels/gemm/gemm_fused.cuh:76-143 (the fused FP16 path, quantize_q8_1_block_fp16_fused): amax and
//     sum tree-reduced (halving 16, 8, 4, 2, then elements 0 + 1), id = 1 / f16(d), q clamped to +-127.
#pragma once
#include "qg_common.hpp"

namespace qg {

__device__ __forceinline__ uint32_t f2h_bits(float f) {
    // Materialise the fp32 value first: without this barrier the compiler folds a preceding fmul
    // into a mixed-precision v_fma_mix (one rounding straight to f16), which differs from the
    // reference's double rounding (f32 product, then __float2half RNE) at f16 ties.
    asm volatile("" : "+v"(f));
    return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f);  // RNE, as __float2half
}

// roundf(y) as (int)(y + copysign(0.49999997f, y)): the fp32 add rounds to nearest even, the conversion
// truncates (and saturates, as (int)roundf does here). Identical for every float in [0, 2^23] (checked
// exhaustively, tools/verify_quant_arith.py, tests/test_quantizer_round.py); above 2^23 every float is an
// integer and the add returns y; negative y mirror through copysign. 3 instructions instead of 7.
__device__ __forceinline__ int roundf_rc(float y) { return (int)(y + copysignf(0.49999997f, y)); }

// m / 127 correctly rounded for m >= 0 (m never NaN: it is an fmaxf over |x| from 0): q0 = m * R with
// R = RN(1/127), the residual fma(-q0, 127, m) and the correction fma(residual, R, q0) — identical to the
// IEEE division for every finite m >= 0 (all 2,139,095,040 checked, tools/verify_quant_arith.py,
// profiles/r05_tuning/quant/verify_quant_arith.txt), +inf passed through. 5 instructions instead of 11.
__device__ __forceinline__ float div127(float m) {
    const float R = __builtin_bit_cast(float, 0x3C010204u);  // RN(1/127)
    const float q0 = m * R;
    const float d = __builtin_fmaf(__builtin_fmaf(-q0, 127.0f, m), R, q0);
    return m == __builtin_inff() ? m : d;
}

// out[0] = f16(d) | f16(s) << 16; out[1..8] = qs (4 int8 per dword, element order).
template <int VARIANT>
__device__ __forceinline__ void quantize_q8_1_block(const float (&v)[32], uint32_t (&out)[9]) {
    float amax = 0.0f, sum = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        amax = fmaxf(amax, fabsf(v[j]));
        sum += v[j];
    }
    const float d = div127(amax);
    const float id = d > 0.0f ? 1.0f / d : 0.0f;
    uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int sq = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        int t = roundf_rc(v[j] * id);
        t = VARIANT == 1 ? max(-127, min(127, t)) : max(-128, min(127, t));
        sq += t;
        q[j / 4] |= ((uint32_t)t & 0xFFu) << (8 * (j & 3));
    }
    const float s = VARIANT == 1 ? (float)sq * d : sum;
    out[0] = f2h_bits(d) | (f2h_bits(s) << 16);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[1 + i] = q[i];
}

// The fused kernel's shared-memory quantizer, one thread per block (its 32 "threads" are the
// 32 array slots here, its halving reduction the same pairing).
__device__ __forceinline__ void quantize_q8_1_block_fp16_fused(const float (&v)[32], uint32_t (&out)[9]) {
    float mx[32], sm[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) {
        mx[t] = fabsf(v[t]);
        sm[t] = v[t];
    }
#pragma unroll
    for (int h = 16; h >= 2; h /= 2) {
#pragma unroll
        for (int t = 0; t < h; ++t) {
            mx[t] = fmaxf(mx[t], mx[t + h]);
            sm[t] += sm[t + h];
        }
    }
    const uint32_t dbits = f2h_bits(div127(fmaxf(mx[0], mx[1])));
    const float d = h2f(dbits);
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int t = max(-127, min(127, roundf_rc(v[j] * id)));
        q[j / 4] |= ((uint32_t)t & 0xFFu) << (8 * (j & 3));
    }
    out[0] = dbits | (f2h_bits(sm[0] + sm[1]) << 16);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[1 + i] = q[i];
}

}  // namespace qg
