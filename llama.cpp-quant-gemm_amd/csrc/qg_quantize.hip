// qg_quantize.hip — FP32 -> block quantizers and block -> FP32 dequantizers on gfx950.
//
// One thread per 32-element block, operation order and rounding exactly as the reference CPU
// quantizers so the bytes are identical (roundf = round-half-away-from-zero, NOT the RNE
// __float2int_rn of the reference's own GPU kernels, include/quantize.h:335; the division and the
// reciprocal are IEEE-correct: the library builds with -fhip-fp32-correctly-rounded-divide-sqrt):
//   Q8_1 (variant 0)  include/quantize.h:165-193  d = amax/127, s = sum(x) in element order
//   Q8_1 (variant 1)  tests/framework/test_framework.cuh:195-225  s = d * sum(q), q clamped to +-127
//   Q4_0              include/quantize.h:35-70     d = amax/7, q = clamp(roundf(x/d)+8, 0, 15)
//   Q8_0              include/quantize.h:111-135
//   Q4_1 / Q5_0 / Q5_1  tests/framework/test_framework.cuh:256-367 (the repo's only quantizers)
//   Q8_1 / Q4_0 (variant 2)  the Solution definitions schemas/definitions/quantization/quantize_q8_1.json:58
//     and quantize_q4_0.json:55 (torch reference): d = amax/127 (/7) in double, or 1.0 for an all-zero
//     block; q = round-half-EVEN(x / f32(d)) (+8 for Q4_0), clamped; the stored f16 d = f16(f32(d)),
//     which equals the one correct rounding of the definition's Python float (tests/test_oracle.py);
//     Q8_1 s = sum(x) in element order as variant 0 (the definition's torch.sum order is unspecified)
#include "qg_common.hpp"
#include "qg_kernels.hpp"
#include "qg_quant_block.hpp"

namespace qg {

template <bool VEC> __device__ __forceinline__ void load32(const float* __restrict__ x, float (&v)[32]) {
    if constexpr (VEC) {
        const float4* p = reinterpret_cast<const float4*>(x);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 t = p[i];
            v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = x[i];
    }
}

// Store `nbytes` (even) bytes held little-endian in dwords w[] as 16-bit stores (blocks are only
// 2-byte aligned inside AoS arrays).
template <int NB> __device__ __forceinline__ void store_u16(uint8_t* dst, const uint32_t (&w)[(NB + 3) / 4]) {
    uint16_t* p = reinterpret_cast<uint16_t*>(dst);
#pragma unroll
    for (int i = 0; i < NB / 2; ++i) p[i] = (uint16_t)(w[i / 2] >> (16 * (i & 1)));
}

// variant 2: the definitions' semantics (header). out as quantize_q8_1_block / the Q4_0 packing.
__device__ __forceinline__ void quantize_q8_1_block_def(const float (&v)[32], uint32_t (&out)[9]) {
    float amax = 0.0f, sum = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        amax = fmaxf(amax, fabsf(v[j]));
        sum += v[j];
    }
    const float d = amax > 0.0f ? amax / 127.0f : 1.0f;
    // f16(f32(amax / 127)) is also the single rounding of the exact quotient the definition's Python
    // float converts to: f32(amax / 127) is never an inexact f16 midpoint (tests/test_oracle.py)
    const uint32_t dh = f2h_bits(d);
    uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const float r = fminf(fmaxf(rintf(v[j] / d), -128.0f), 127.0f);
        q[j / 4] |= ((uint32_t)(int)r & 0xFFu) << (8 * (j & 3));
    }
    out[0] = dh | (f2h_bits(sum) << 16);
#pragma unroll
    for (int i = 0; i < 8; ++i) out[1 + i] = q[i];
}

template <int TYPE, int VARIANT, bool VEC>
__global__ __launch_bounds__(256) void quantize_kernel(const float* __restrict__ x, uint8_t* __restrict__ y, int64_t nblocks) {
    const int64_t ib = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ib >= nblocks) return;
    float v[32];
    load32<VEC>(x + ib * QK, v);

    if constexpr (TYPE == FMT_Q8_1) {
        uint32_t w[9];
        if constexpr (VARIANT == 2) quantize_q8_1_block_def(v, w);
        else quantize_q8_1_block<VARIANT>(v, w);
        uint32_t* dst = reinterpret_cast<uint32_t*>(y + ib * 36);  // 36-B blocks stay 4-B aligned
#pragma unroll
        for (int i = 0; i < 9; ++i) dst[i] = w[i];
    } else if constexpr (TYPE == FMT_Q8_0) {
        float amax = 0.0f;
#pragma unroll
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
        const float d = amax / 127.0f;
        const float id = d > 0.0f ? 1.0f / d : 0.0f;
        uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const int t = max(-128, min(127, (int)roundf(v[j] * id)));
            q[j / 4] |= ((uint32_t)t & 0xFFu) << (8 * (j & 3));
        }
        uint32_t w[9];
        w[0] = f2h_bits(d) | ((q[0] & 0xFFFFu) << 16);
#pragma unroll
        for (int i = 1; i < 8; ++i) w[i] = (q[i - 1] >> 16) | ((q[i] & 0xFFFFu) << 16);
        w[8] = q[7] >> 16;
        store_u16<34>(y + ib * 34, w);
    } else if constexpr (TYPE == FMT_Q4_0 || TYPE == FMT_Q5_0) {
        float amax = 0.0f;
#pragma unroll
        for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(v[j]));
        constexpr float DIV = TYPE == FMT_Q4_0 ? 7.0f : 15.0f;
        constexpr int OFF = TYPE == FMT_Q4_0 ? 8 : 16;
        constexpr int QMAX = TYPE == FMT_Q4_0 ? 15 : 31;
        const float d = VARIANT == 2 && amax == 0.0f ? 1.0f : amax / DIV;
        const float id = d > 0.0f ? 1.0f / d : 0.0f;
        uint8_t qs[16];
        uint32_t qh = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            int q0, q1;
            if constexpr (VARIANT == 2) {  // torch.round(x / d) + 8: ties to even, true division
                q0 = (int)rintf(v[j] / d) + OFF;
                q1 = (int)rintf(v[j + 16] / d) + OFF;
            } else {
                q0 = (int)roundf(v[j] * id) + OFF;
                q1 = (int)roundf(v[j + 16] * id) + OFF;
            }
            q0 = max(0, min(QMAX, q0));
            q1 = max(0, min(QMAX, q1));
            qs[j] = (uint8_t)((q0 & 0xF) | ((q1 & 0xF) << 4));
            qh |= (uint32_t)((q0 >> 4) & 1) << j;
            qh |= (uint32_t)((q1 >> 4) & 1) << (j + 16);
        }
        if constexpr (TYPE == FMT_Q4_0) {
            uint32_t w[5];
            w[0] = f2h_bits(d) | ((uint32_t)qs[0] << 16) | ((uint32_t)qs[1] << 24);
#pragma unroll
            for (int i = 1; i < 4; ++i)
                w[i] = (uint32_t)qs[4 * i - 2] | ((uint32_t)qs[4 * i - 1] << 8) | ((uint32_t)qs[4 * i] << 16) |
                       ((uint32_t)qs[4 * i + 1] << 24);
            w[4] = (uint32_t)qs[14] | ((uint32_t)qs[15] << 8);
            store_u16<18>(y + ib * 18, w);
        } else {
            uint32_t w[6];
            w[0] = f2h_bits(d) | ((qh & 0xFFFFu) << 16);
            w[1] = (qh >> 16) | ((uint32_t)qs[0] << 16) | ((uint32_t)qs[1] << 24);
#pragma unroll
            for (int i = 2; i < 5; ++i)
                w[i] = (uint32_t)qs[4 * i - 6] | ((uint32_t)qs[4 * i - 5] << 8) | ((uint32_t)qs[4 * i - 4] << 16) |
                       ((uint32_t)qs[4 * i - 3] << 24);
            w[5] = (uint32_t)qs[14] | ((uint32_t)qs[15] << 8);
            store_u16<22>(y + ib * 22, w);
        }
    } else {  // Q4_1 / Q5_1: min/max, sequential compare from element 0 as the reference loop
        float mn = v[0], mx = v[0];
#pragma unroll
        for (int j = 1; j < 32; ++j) {
            if (v[j] < mn) mn = v[j];
            if (v[j] > mx) mx = v[j];
        }
        constexpr float DIV = TYPE == FMT_Q4_1 ? 15.0f : 31.0f;
        constexpr int QMAX = TYPE == FMT_Q4_1 ? 15 : 31;
        const float d = (mx - mn) / DIV;
        const float id = d > 0.0f ? 1.0f / d : 0.0f;
        uint8_t qs[16];
        uint32_t qh = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            int q0 = (int)roundf((v[j] - mn) * id);
            int q1 = (int)roundf((v[j + 16] - mn) * id);
            q0 = max(0, min(QMAX, q0));
            q1 = max(0, min(QMAX, q1));
            qs[j] = (uint8_t)((q0 & 0xF) | ((q1 & 0xF) << 4));
            qh |= (uint32_t)((q0 >> 4) & 1) << j;
            qh |= (uint32_t)((q1 >> 4) & 1) << (j + 16);
        }
        const uint32_t dm = f2h_bits(d) | (f2h_bits(mn) << 16);
        if constexpr (TYPE == FMT_Q4_1) {
            uint32_t w[5];
            w[0] = dm;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                w[1 + i] = (uint32_t)qs[4 * i] | ((uint32_t)qs[4 * i + 1] << 8) | ((uint32_t)qs[4 * i + 2] << 16) |
                           ((uint32_t)qs[4 * i + 3] << 24);
            store_u16<20>(y + ib * 20, w);
        } else {
            uint32_t w[6];
            w[0] = dm;
            w[1] = qh;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                w[2 + i] = (uint32_t)qs[4 * i] | ((uint32_t)qs[4 * i + 1] << 8) | ((uint32_t)qs[4 * i + 2] << 16) |
                           ((uint32_t)qs[4 * i + 3] << 24);
            store_u16<24>(y + ib * 24, w);
        }
    }
}

// Q8_1, eight lanes per block (round 5): the one-thread-per-block kernel above ran a
// decode-size activation row (K = 4096: 128 blocks) as ONE workgroup whose 128 threads each walked 32
// elements through ~350 dependent VALU ops — 4.4-5.5 us for 16 KB (profiles/r04c_bench_kernel_trace*.md).
// Here lane j of a block's 8 lanes loads elements 4j..4j+3 (one 16-B load per lane, 1 KB contiguous per
// wave instruction), 64-thread workgroups (8 blocks each: 16 workgroups at K = 4096) spread the row over
// the CUs, and the per-lane work is 4 elements. Bytes identical to quantize_q8_1_block /
// quantize_q8_1_block_def:
//   amax: max over the 8 lanes' partial maxima (v_max_f32 is order-free on non-NaN values; every partial
//     starts at 0.0f as the sequential loop does, so NaN inputs are ignored the same way);
//   s = sum(x) in ELEMENT order: the partial sum walks the 8 lanes in turn (lane j adds its 4 elements to
//     what lane j - 1 handed over by DPP row_shr:1), the very sequence of fp32 adds of the reference loop.
//     Every lane runs every step (no select): after step t lane j holds the ordered sum of lanes j - t..j,
//     and lane 7's step-7 value reaches back only to lane 0's step-0 value 0 + x, so what a group's first
//     lane receives from the previous group (or a row edge) never enters lane 7's result;
//   variant 1: s = d * sum(q) (an integer sum, any order);
//   roundf and d = m / 127 through roundf_rc / div127 (qg_quant_block.hpp: same results, fewer instructions).
// Lane j stores qs dword j; lane 7 (which ends holding s) stores the d | s dword.
// One block's quantization by its 8 lanes (all 64 lanes of the wave take part in the DPP steps): lane j holds
// elements 4j..4j+3 in v; returns qs dword j, and in lane 7 the d | s dword in hdr.
template <int VARIANT> __device__ __forceinline__ uint32_t q8_1_lanes(const float4 v, int j, uint32_t& hdr) {
    float m = fmaxf(fmaxf(fmaxf(fmaxf(0.0f, fabsf(v.x)), fabsf(v.y)), fabsf(v.z)), fabsf(v.w));
    m = fmaxf(m, dpp_f<0xB1>(m));   // quad_perm [1,0,3,2]
    m = fmaxf(m, dpp_f<0x4E>(m));   // quad_perm [2,3,0,1]
    m = fmaxf(m, dpp_f<0x141>(m));  // row_half_mirror: the other quad of the 8 lanes
    const float xs[4] = {v.x, v.y, v.z, v.w};
    uint32_t qd = 0;
    int sq = 0;
    float d;
    if constexpr (VARIANT == 2) {
        d = m > 0.0f ? m / 127.0f : 1.0f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float r = fminf(fmaxf(rintf(xs[e] / d), -128.0f), 127.0f);
            qd |= ((uint32_t)(int)r & 0xFFu) << (8 * e);
        }
    } else {
        d = div127(m);
        const float id = d > 0.0f ? 1.0f / d : 0.0f;
        uint32_t t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int q = roundf_rc(xs[e] * id);  // |q| <= 127 unless d is subnormal (inexact): clamp kept
            const int c = VARIANT == 1 ? max(-127, min(127, q)) : max(-128, min(127, q));
            sq += c;
            t[e] = (uint32_t)c;
        }
        // low bytes of t[0..3] into one dword: two byte permutes and an or
        qd = __builtin_amdgcn_perm(t[1], t[0], 0x0c0c0400u) | __builtin_amdgcn_perm(t[3], t[2], 0x04000c0cu);
    }
    float s;
    if constexpr (VARIANT == 1) {
        sq += __builtin_amdgcn_update_dpp(0, sq, 0xB1, 0xF, 0xF, false);
        sq += __builtin_amdgcn_update_dpp(0, sq, 0x4E, 0xF, 0xF, false);
        sq += __builtin_amdgcn_update_dpp(0, sq, 0x141, 0xF, 0xF, false);
        s = (float)sq * d;
    } else {
        float p = (((0.0f + v.x) + v.y) + v.z) + v.w;
#pragma unroll
        for (int step = 1; step < 8; ++step) p = (((dpp_f<0x111>(p) + v.x) + v.y) + v.z) + v.w;  // row_shr:1
        s = p;  // complete in lane 7
    }
    hdr = f2h_bits(d) | (f2h_bits(s) << 16);
    return qd;
}

// I: the index type — uint32_t where every float4 index and output dword fits (the launcher's choice; fewer
// address instructions on the one-wave-per-workgroup critical path), int64_t otherwise.
// FULL: the grid covers exactly nblocks (nblocks % 8 == 0): no bounds predicate.
template <int VARIANT, typename I, bool FULL>
__global__ __launch_bounds__(64) void quantize_q8_1_lanes_kernel(const float4* __restrict__ x, uint32_t* __restrict__ y,
                                                                 I nblocks) {
    const I gi = (I)blockIdx.x * 64 + threadIdx.x;  // float4 index: block gi / 8, lane j = gi % 8
    const I ib = gi >> 3;
    const int j = threadIdx.x & 7;
    const bool ok = FULL || ib < nblocks;
    const float4 v = ok ? x[gi] : make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t hdr;
    const uint32_t qd = q8_1_lanes<VARIANT>(v, j, hdr);
    if (!ok) return;
    uint32_t* dst = y + (gi + ib);  // = block ib's dword j (9 ib + j): qs dword j at +1, the header at -j
    dst[1] = qd;
    if (j == 7) dst[-7] = hdr;
}

// Q8_1 straight into the tiled activation layout (LAY_TILED_ACT, qg_kernels.hpp): block b of token m lands in
// token tile m / 16, stage b / 4, at (m % 16) * 144 + (b % 4) * 36 of that (tile, stage)'s 2304-B run; tokens
// past M (to a multiple of 16) and blocks past K / 32 (to a multiple of 4) are zero blocks (d = s = 0, qs = 0:
// an exact +0 term against any weights). Same bytes per real block as quantize_q8_1_lanes_kernel.
__device__ __forceinline__ int64_t tiled_act_dword(int m, int b, int H) {
    return ((((int64_t)(m / ACT_TILE) * H + b / 4) * ACT_TILE + m % ACT_TILE) * 4 + b % 4) * 9;
}
__global__ __launch_bounds__(64) void quantize_q8_1_tiled_kernel(const float4* __restrict__ x, uint32_t* __restrict__ y, int M,
                                                                 int nb, int H, int64_t nblk) {
    const int64_t gi = (int64_t)blockIdx.x * 64 + threadIdx.x;
    const int64_t ib = gi >> 3;  // padded block index, token-major over 4 H blocks per token
    const int j = threadIdx.x & 7;
    const bool ok = ib < nblk;
    const int m = (int)(ib / (4 * H)), b = (int)(ib - (int64_t)m * 4 * H);
    const bool real = ok && m < M && b < nb;
    const float4 v = real ? x[((int64_t)m * nb + b) * 8 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t hdr;
    const uint32_t qd = q8_1_lanes<0>(v, j, hdr);
    if (!ok) return;
    uint32_t* dst = y + tiled_act_dword(m, b, H);
    dst[1 + j] = qd;
    if (j == 7) dst[0] = real ? hdr : 0u;
}

// Q8_1 rows [M][K/32] -> the tiled activation layout (one thread per destination dword)
__global__ __launch_bounds__(256) void tile_activations_kernel(const uint32_t* __restrict__ a, uint32_t* __restrict__ y, int M,
                                                               int nb, int H, int64_t ndw) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= ndw) return;
    const int64_t blk = i / 9;
    const int w = (int)(i - blk * 9);
    const int64_t st = blk / (ACT_TILE * 4);  // (tile, stage) run
    const int r = (int)(blk - st * ACT_TILE * 4), t = r / 4, bl = r % 4;
    const int tile = (int)(st / H), h = (int)(st - (int64_t)tile * H);
    const int m = tile * ACT_TILE + t, b = h * 4 + bl;
    y[i] = m < M && b < nb ? a[((int64_t)m * nb + b) * 9 + w] : 0u;
}

// FP16 -> Q8_1 with the fused kernel's semantics (kernels/gemm/gemm_fused.cuh:76-143), the
// workspace producer of qg_gemm_q4_0_fp16_fused_ws for token counts beyond the fused GEMV.
__global__ __launch_bounds__(256) void quantize_f16_fused_kernel(const uint16_t* __restrict__ x, uint8_t* __restrict__ y,
                                                                 int64_t nblocks) {
    const int64_t ib = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ib >= nblocks) return;
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = h2f(x[ib * QK + j]);
    uint32_t w[9];
    quantize_q8_1_block_fp16_fused(v, w);
    uint32_t* dst = reinterpret_cast<uint32_t*>(y + ib * 36);
#pragma unroll
    for (int i = 0; i < 9; ++i) dst[i] = w[i];
}

// Dequantize: x = (q - off) * d  or  q * d + m  (include/quantize.h:84-102, 140-150, 198-210).
template <int TYPE>
__global__ __launch_bounds__(256) void dequantize_kernel(const uint8_t* __restrict__ x, float* __restrict__ y, int64_t nblocks) {
    const int64_t ib = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ib >= nblocks) return;
    float* o = y + ib * QK;
    if constexpr (TYPE == FMT_Q8_0 || TYPE == FMT_Q8_1) {
        constexpr int BB = TYPE == FMT_Q8_0 ? 34 : 36;
        constexpr int QO = TYPE == FMT_Q8_0 ? 2 : 4;
        const uint8_t* b = x + ib * BB;
        const float d = h2f((uint32_t)b[0] | ((uint32_t)b[1] << 8));
#pragma unroll
        for (int j = 0; j < 32; ++j) o[j] = (float)(int8_t)b[QO + j] * d;
    } else {
        using T = wfmt<TYPE>;
        const uint8_t* b = x + ib * T::BB;
        const float d = h2f((uint32_t)b[0] | ((uint32_t)b[1] << 8));
        float m = 0.0f;
        if constexpr (T::MOFF >= 0) m = h2f((uint32_t)b[T::MOFF] | ((uint32_t)b[T::MOFF + 1] << 8));
        uint32_t qh = 0;
        if constexpr (T::QH >= 0)
            qh = (uint32_t)b[T::QH] | ((uint32_t)b[T::QH + 1] << 8) | ((uint32_t)b[T::QH + 2] << 16) |
                 ((uint32_t)b[T::QH + 3] << 24);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            int q0 = b[T::QS + j] & 0xF, q1 = b[T::QS + j] >> 4;
            if constexpr (T::QH >= 0) {
                q0 |= (int)((qh >> j) & 1u) << 4;
                q1 |= (int)((qh >> (j + 16)) & 1u) << 4;
            }
            if constexpr (TYPE == FMT_Q4_0) { o[j] = (float)(q0 - 8) * d; o[j + 16] = (float)(q1 - 8) * d; }
            else if constexpr (TYPE == FMT_Q5_0) { o[j] = (float)(q0 - 16) * d; o[j + 16] = (float)(q1 - 16) * d; }
            else { o[j] = (float)q0 * d + m; o[j + 16] = (float)q1 * d + m; }
        }
    }
}

// Q8_1 rows of K floats -> rows of nbp >= nb = K/32 blocks: the first nb exactly as quantize_kernel
// (include/quantize.h:165-193), then zero blocks (d = 0, s = 0) — the activation side of the padded
// layout of qg_repack_weights (qg_quantize_q8_1_padded, qg_gemm_w4a8_padded).
template <bool VEC>
__global__ __launch_bounds__(256) void quantize_q8_1_padded_kernel(const float* __restrict__ x, uint8_t* __restrict__ y,
                                                                   int64_t rows, int nb, int nbp) {
    const int64_t ib = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (ib >= rows * nbp) return;
    const int64_t r = ib / nbp;
    const int b = (int)(ib - r * nbp);
    uint32_t w[9] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    if (b < nb) {
        float v[32];
        load32<VEC>(x + (r * nb + b) * QK, v);
        quantize_q8_1_block<0>(v, w);
    }
    uint32_t* dst = reinterpret_cast<uint32_t*>(y + ib * 36);
#pragma unroll
    for (int i = 0; i < 9; ++i) dst[i] = w[i];
}

hipError_t launch_quantize_q8_1_padded(const float* x, void* y, int64_t rows, int nb, int nbp, hipStream_t st) {
    const int64_t n = rows * nbp;
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (((uintptr_t)x & 15) == 0)
        hipLaunchKernelGGL((quantize_q8_1_padded_kernel<true>), grid, dim3(256), 0, st, x, (uint8_t*)y, rows, nb, nbp);
    else
        hipLaunchKernelGGL((quantize_q8_1_padded_kernel<false>), grid, dim3(256), 0, st, x, (uint8_t*)y, rows, nb, nbp);
    return hipGetLastError();
}

namespace {
template <int TYPE, int VARIANT>
hipError_t lq(const float* x, void* y, int64_t nblocks, hipStream_t st) {
    if constexpr (TYPE == FMT_Q8_1) {
        if (((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 3) == 0 && (nblocks + 7) / 8 <= 0x7fffffffL) {
            const dim3 grid((unsigned)((nblocks + 7) / 8));
            if (nblocks <= (int64_t(1) << 26) && nblocks % 8 == 0)
                hipLaunchKernelGGL((quantize_q8_1_lanes_kernel<VARIANT, uint32_t, true>), grid, dim3(64), 0, st,
                                   (const float4*)x, (uint32_t*)y, (uint32_t)nblocks);
            else if (nblocks <= (int64_t(1) << 26))
                hipLaunchKernelGGL((quantize_q8_1_lanes_kernel<VARIANT, uint32_t, false>), grid, dim3(64), 0, st,
                                   (const float4*)x, (uint32_t*)y, (uint32_t)nblocks);
            else
                hipLaunchKernelGGL((quantize_q8_1_lanes_kernel<VARIANT, int64_t, false>), grid, dim3(64), 0, st,
                                   (const float4*)x, (uint32_t*)y, nblocks);
            return hipGetLastError();
        }
    }
    const dim3 grid((unsigned)((nblocks + 255) / 256));
    if (((uintptr_t)x & 15) == 0)
        hipLaunchKernelGGL((quantize_kernel<TYPE, VARIANT, true>), grid, dim3(256), 0, st, x, (uint8_t*)y, nblocks);
    else
        hipLaunchKernelGGL((quantize_kernel<TYPE, VARIANT, false>), grid, dim3(256), 0, st, x, (uint8_t*)y, nblocks);
    return hipGetLastError();
}
template <int TYPE> hipError_t ld(const void* x, float* y, int64_t nblocks, hipStream_t st) {
    hipLaunchKernelGGL((dequantize_kernel<TYPE>), dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, st,
                       (const uint8_t*)x, y, nblocks);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_quantize(int type, int variant, const float* x, void* y, int64_t nblocks, hipStream_t st) {
    if (nblocks == 0) return hipSuccess;
    switch (type) {
        case FMT_Q8_1:
            return variant == 1 ? lq<FMT_Q8_1, 1>(x, y, nblocks, st)
                 : variant == 2 ? lq<FMT_Q8_1, 2>(x, y, nblocks, st) : lq<FMT_Q8_1, 0>(x, y, nblocks, st);
        case FMT_Q8_0: return lq<FMT_Q8_0, 0>(x, y, nblocks, st);
        case FMT_Q4_0: return variant == 2 ? lq<FMT_Q4_0, 2>(x, y, nblocks, st) : lq<FMT_Q4_0, 0>(x, y, nblocks, st);
        case FMT_Q4_1: return lq<FMT_Q4_1, 0>(x, y, nblocks, st);
        case FMT_Q5_0: return lq<FMT_Q5_0, 0>(x, y, nblocks, st);
        case FMT_Q5_1: return lq<FMT_Q5_1, 0>(x, y, nblocks, st);
    }
    return hipErrorInvalidValue;
}

size_t tiled_act_bytes(int M, int K) {
    const int nb = K / QK, H = (nb + 3) / 4;
    return (size_t)((M + ACT_TILE - 1) / ACT_TILE) * (size_t)H * ACT_STG;
}

hipError_t launch_quantize_q8_1_tiled(const float* x, void* y, int M, int K, hipStream_t st) {
    const int nb = K / QK, H = (nb + 3) / 4;
    const int64_t nblk = (int64_t)((M + ACT_TILE - 1) / ACT_TILE) * ACT_TILE * 4 * H;
    hipLaunchKernelGGL(quantize_q8_1_tiled_kernel, dim3((unsigned)((nblk + 7) / 8)), dim3(64), 0, st, (const float4*)x,
                       (uint32_t*)y, M, nb, H, nblk);
    return hipGetLastError();
}

hipError_t launch_tile_activations(const void* a, void* y, int M, int K, hipStream_t st) {
    const int nb = K / QK, H = (nb + 3) / 4;
    const int64_t ndw = (int64_t)tiled_act_bytes(M, K) / 4;
    hipLaunchKernelGGL(tile_activations_kernel, dim3((unsigned)((ndw + 255) / 256)), dim3(256), 0, st, (const uint32_t*)a,
                       (uint32_t*)y, M, nb, H, ndw);
    return hipGetLastError();
}

hipError_t launch_quantize_f16_fused(const void* x, void* y, int64_t nblocks, hipStream_t st) {
    if (nblocks == 0) return hipSuccess;
    hipLaunchKernelGGL(quantize_f16_fused_kernel, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, st,
                       (const uint16_t*)x, (uint8_t*)y, nblocks);
    return hipGetLastError();
}

hipError_t launch_dequantize(int type, const void* x, float* y, int64_t nblocks, hipStream_t st) {
    if (nblocks == 0) return hipSuccess;
    switch (type) {
        case FMT_Q8_1: return ld<FMT_Q8_1>(x, y, nblocks, st);
        case FMT_Q8_0: return ld<FMT_Q8_0>(x, y, nblocks, st);
        case FMT_Q4_0: return ld<FMT_Q4_0>(x, y, nblocks, st);
        case FMT_Q4_1: return ld<FMT_Q4_1>(x, y, nblocks, st);
        case FMT_Q5_0: return ld<FMT_Q5_0>(x, y, nblocks, st);
        case FMT_Q5_1: return ld<FMT_Q5_1>(x, y, nblocks, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
