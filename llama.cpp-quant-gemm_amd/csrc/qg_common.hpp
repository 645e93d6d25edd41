// qg_common.hpp — device-side building blocks shared by every W4A8 kernel (gfx950 only).
//
// Block formats are the byte-exact llama.cpp ones (include/qg/blocks.h). Everything here works on
// raw dwords already in VGPRs: a block's fields are pulled out of a register-resident "super-block"
// (8 consecutive blocks = 256 elements, 144/160/176/192 B for Q4_0/Q4_1/Q5_0/Q5_1 — always a
// multiple of 16 B, so a lane can fetch it with global_load_dwordx4) with compile-time byte offsets,
// i.e. v_alignbyte_b32 / shifts, never LDS or byte loads.
//
// Per-block epilogues restate the reference formulas operation for operation (no contraction; the
// library is built with -ffp-contract=off) so a block's fp32 term is bit-identical to the CPU
// oracle's:
//   Q4_0  d_w * (d_a * sumi - 8 * s_a)        include/gemm_reference.h:216
//   Q5_0  d_w * (d_a * sumi - 16 * s_a)       kernels/gemm/gemm_quant_formats.cuh:207
//   Q4_1  d_w * d_a * sumi + m_w * s_a        flashinfer_trace/definitions/quant_gemm/w4_1a8_q4_1_q8_1_n4096_k4096.json:79
//   Q5_1  d_w * d_a * sumi + m_w * s_a        (the reference's /4 at gemm_quant_formats.cuh:148,266 is a
//                                              mis-port and is NOT reproduced; SURVEY.md §0 defect 2)
//   Q8_0  sumi * d_a * d_w                    include/gemm_reference.h:260 (W8A8, gemm_w8a8_reference)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include <utility>

namespace qg {

// ggml_type ids (compat/ggml_types.h:199-215)
enum : int { FMT_Q4_0 = 2, FMT_Q4_1 = 3, FMT_Q5_0 = 6, FMT_Q5_1 = 7, FMT_Q8_0 = 8, FMT_Q8_1 = 9 };

// Field byte offsets inside one weight block; -1 = field absent. Q8 = 32 signed bytes in element
// order (Q8_0) instead of 16 nibble pairs.
template <int F> struct wfmt;
template <> struct wfmt<FMT_Q4_0> { static constexpr int BB = 18, MOFF = -1, QH = -1, QS = 2; static constexpr bool Q8 = false; };
template <> struct wfmt<FMT_Q4_1> { static constexpr int BB = 20, MOFF = 2, QH = -1, QS = 4; static constexpr bool Q8 = false; };
template <> struct wfmt<FMT_Q5_0> { static constexpr int BB = 22, MOFF = -1, QH = 2, QS = 6; static constexpr bool Q8 = false; };
template <> struct wfmt<FMT_Q5_1> { static constexpr int BB = 24, MOFF = 2, QH = 4, QS = 8; static constexpr bool Q8 = false; };
template <> struct wfmt<FMT_Q8_0> { static constexpr int BB = 34, MOFF = -1, QH = -1, QS = 2; static constexpr bool Q8 = true; };

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int QK = 32;
constexpr int SB_BLOCKS = 8;        // blocks per super-block
constexpr int SB_ELEMS = 256;       // elements per super-block
constexpr int Q8_1_BYTES = 36;

__device__ __forceinline__ float h2f(uint32_t bits16) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
}

template <int N> using ic = std::integral_constant<int, N>;
template <int... Is, class Fn>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, Is...>, Fn&& fn) {
    (fn(ic<Is>{}), ...);
}
template <int N, class Fn> __device__ __forceinline__ void static_for(Fn&& fn) {
    static_for_impl(std::make_integer_sequence<int, N>{}, fn);
}

// 32 bits starting at compile-time byte offset OFF of a register-resident byte stream.
template <int OFF> __device__ __forceinline__ uint32_t ld32(const uint32_t* w) {
    if constexpr (OFF % 4 == 0) return w[OFF / 4];
    else return __builtin_amdgcn_alignbyte(w[OFF / 4 + 1], w[OFF / 4], OFF % 4);
}
// 16 bits at an even compile-time offset.
template <int OFF> __device__ __forceinline__ uint32_t ld16(const uint32_t* w) {
    static_assert(OFF % 2 == 0, "fp16 fields are 2-byte aligned");
    if constexpr (OFF % 4 == 0) return w[OFF / 4] & 0xFFFFu;
    else return w[OFF / 4] >> 16;
}

// c ? a : b on VALUES. Both operands are pinned in VGPRs first: a plain ternary over two elements
// of a register-resident array gets folded into a load through a selected pointer, which demotes
// the whole array to scratch memory.
__device__ __forceinline__ uint32_t vsel(bool c, uint32_t a, uint32_t b) {
    asm volatile("" : "+v"(a), "+v"(b));
    return c ? a : b;
}

// Spread 4 bits (x in [0,15]) to bit 4 of each byte: bit k -> bit 8k+4. v_mul_u32_u24 is full rate.
__device__ __forceinline__ uint32_t spread4_bit4(uint32_t x) {
    return ((uint32_t)__umul24(x, 0x00204081u) & 0x01010101u) << 4;
}

constexpr int TILE_ROWS = 32;  // weight rows per tile of LAY_TILED

// One (tile, stage) of LAY_TILED: 32 rows x 4 blocks = 128 * BB bytes, as planes
//   QS  [row tile i of 16 rows][half][lane = q * 16 + r][16 B]: dword q of the 4 blocks' qs of row
//       16 i + r (half 1, Q8_0 only: dword 4 + q) — exactly MFMA lane (r, q)'s k-slot of each block;
//   QH  [row][16 B]: the 4 blocks' qh dwords (Q5_0 / Q5_1);
//   SC  [row][SCB]: f16 d of blocks 0..3, then (Q4_1 / Q5_1) f16 m of blocks 0..3.
// Rows past N and blocks past K/32 are zero bytes (d = 0: an exact +0 term).
template <int F> struct tiled_fmt {
    using T = wfmt<F>;
    static constexpr int QSL = T::Q8 ? 32 : 16;       // qs bytes per lane and row tile
    static constexpr int QSB = 2 * 64 * QSL;          // QS plane bytes
    static constexpr int QHB = T::QH >= 0 ? 16 : 0;   // qh bytes per row
    static constexpr int SCB = T::MOFF >= 0 ? 16 : 8; // scale bytes per row
    static constexpr int OQH = QSB, OSC = QSB + TILE_ROWS * QHB;
    static constexpr int STG = OSC + TILE_ROWS * SCB;  // bytes per (tile, stage)
    static_assert(STG == TILE_ROWS * 4 * T::BB, "the planes hold exactly the stage's blocks");
};

// Decoded weight block: q[i] = elements 4i..4i+3 (i<4) / 16+4(i-4).. (i>=4), i.e. elements 4i..4i+3,
// exactly the stored values (no offset removed; unsigned nibbles, or Q8_0's signed bytes), plus its
// scale(s).
struct wblock {
    uint32_t q[8];
    float d, m;
};

// Decode block BI (0..7) of a register-resident super-block of format F.
template <int F, int BI> __device__ __forceinline__ wblock decode_block(const uint32_t* w) {
    using T = wfmt<F>;
    constexpr int base = BI * T::BB;
    wblock r;
    r.d = h2f(ld16<base>(w));
    if constexpr (T::MOFF >= 0) r.m = h2f(ld16<base + T::MOFF>(w));
    else r.m = 0.0f;
    if constexpr (T::Q8) {
        static_for<8>([&](auto I) { r.q[decltype(I)::value] = ld32<base + T::QS + 4 * decltype(I)::value>(w); });
        return r;
    }
    uint32_t qh = 0;
    if constexpr (T::QH >= 0) qh = ld32<base + T::QH>(w);
    static_for<4>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const uint32_t v = ld32<base + T::QS + 4 * i>(w);
        uint32_t lo = v & 0x0F0F0F0Fu;
        uint32_t hi = (v >> 4) & 0x0F0F0F0Fu;
        if constexpr (T::QH >= 0) {
            lo |= spread4_bit4((qh >> (4 * i)) & 0xFu);
            hi |= spread4_bit4((qh >> (16 + 4 * i)) & 0xFu);
        }
        r.q[i] = lo;
        r.q[4 + i] = hi;
    });
    return r;
}

// Integer dot of one decoded weight block with 8 activation dwords (elements 0..31 in order).
__device__ __forceinline__ int dot_block(const uint32_t* q, const uint32_t* a) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s = __builtin_amdgcn_sdot4((int)q[i], (int)a[i], s, false);
    return s;
}

// Sum of x over each aligned group of G lanes (G = 1..64, a power of two), delivered in the LAST
// lane of the group (other lanes hold partial sums). DPP row ops, no LDS round trips: xor-1 and
// xor-2 quad permutes, row_shr 4 and 8 inside each 16-lane row, then row_bcast 15 / 31 across rows
// (gfx9 DPP). The pairing order is fixed, so the result is deterministic.
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWMASK, 0xF, false));
}
template <int G> __device__ __forceinline__ float group_sum_last(float x) {
    static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "power-of-two group");
    if constexpr (G >= 2) x += dpp_f<0xB1>(x);        // quad_perm [1,0,3,2]
    if constexpr (G >= 4) x += dpp_f<0x4E>(x);        // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x += dpp_f<0x114>(x);       // row_shr:4
    if constexpr (G >= 16) x += dpp_f<0x118>(x);      // row_shr:8
    if constexpr (G >= 32) x += dpp_f<0x142, 0xA>(x); // row_bcast:15 into rows 1, 3
    if constexpr (G >= 64) x += dpp_f<0x143, 0xC>(x); // row_bcast:31 into rows 2, 3
    return x;
}

// XCD-aware tile order. Workgroups of a launch are placed round-robin over the 8 XCDs (linear
// workgroup b on XCD b % 8); for a grid of G tiles along x this gives XCD x the contiguous tile range
// [x*(G/8) + min(x, G%8), ...) (a bijection on 0..G-1), so neighbouring tiles — and the output lines
// they share — stay in one XCD's L2. Only for grids of one dispatch round: with many rounds the
// linear order streams better (qg_gemv_kernel.hpp).
__device__ __forceinline__ int xcd_tile(int b, int G) {
    const int g8 = G >> 3, r8 = G & 7, x = b & 7;
    return x * g8 + min(x, r8) + (b >> 3);
}

// Per-block fp32 term, operation order as in the reference (see header comment).
// fs = (float)sumi (exact: |sumi| < 2^24).
template <int F> __device__ __forceinline__ float block_term_f(float fs, float dw, float mw, float da, float sa) {
    if constexpr (F == FMT_Q4_0) return dw * (da * fs - 8.0f * sa);
    else if constexpr (F == FMT_Q5_0) return dw * (da * fs - 16.0f * sa);
    else if constexpr (F == FMT_Q8_0) return fs * da * dw;
    else return dw * da * fs + mw * sa;
}
template <int F> __device__ __forceinline__ float block_term(int sumi, float dw, float mw, float da, float sa) {
    return block_term_f<F>((float)sumi, dw, mw, da, sa);
}

}  // namespace qg
