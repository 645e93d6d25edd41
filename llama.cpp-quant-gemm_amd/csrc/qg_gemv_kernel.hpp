// qg_gemv_kernel.hpp — the W4A8 GEMV / small-batch kernels (M <= 8 activation rows).
//
// Included by qg_gemv.hip (the product's instantiations + dispatch) and by profiles/tools_archive/gemv_probe.hip
// (the tuning sweep). Computes, for the reference's activation-major contract
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222):
//   C[m*ldc_m + n*ldc_n] = sum_b term(A[m][b], B[n][b]).
//
// Work decomposition:
//  * A lane owns "units" of BPL consecutive Q-blocks of one weight row (BPL*BB bytes, e.g. Q4_0
//    BPL=4 -> 72 B; 4 x dwordx4 + 1 x dwordx2). LPR lanes share a row and stride over its units
//    (the next unit in flight while the current one computes); 64/LPR rows per wave, WGS/64 waves
//    per workgroup.
//  * The workgroup stages the M activation rows once into LDS, one 12-dword record per Q8_1 block
//    (one thread per block; unit stride 12*BPL+4 dwords = 4 x odd, so the 16 lanes of a
//    ds_read_b128 group hit distinct bank slots). The first block's loads are issued before the
//    weight stream, so the staging waits only on them.
//  * Integer dot, exact int32 sumi, two forms:
//      - nibble planes (Q4_0, Q4_1 weights): each activation byte a = 16*h + l with h = a >> 4
//        (signed 4-bit) and l = a & 15; the record holds the l and h nibbles of elements
//        (4i+k, 16+4i+k) interleaved exactly like the weight nibbles of qs dword i, so one raw
//        weight dword q feeds v_dot8_u32_u4(q, l) and, XORed with 0x88888888 (= signed q - 8),
//        v_dot8_i32_i4(q^0x8.., h): sumi = L + 16*H + 128*sum(h), the last term (activation only)
//        folded into the accumulator's initial value. 8 dot8 + 4 XOR per block, no nibble
//        unpacking;
//      - bytes (Q5_0, Q5_1, Q8_0): blocks decoded in registers with compile-time
//        alignbyte/shift/mask (qg_common.hpp), 8 v_dot4c_i32_i8 per block.
//    Both accumulate on top of the bit pattern of 1.5*2^23, so the int32 result read as f32 is
//    1.5*2^23 + sumi (|sumi| < 2^22): no int->float convert.
//  * Per-block epilogue in the reference's operation order, so each block's fp32 term is
//    bit-identical to the CPU oracle's: fma(d_a, cf, -1.5*2^23*d_a) = round(d_a*sumi) (the
//    constant is exact), c*s_a precomputed in the record (exact: c is 8, 16 or 1), d_w (and m_w)
//    taken straight from the f16 bits by v_fma_mix_f32 with a zero addend (= one rounding of the
//    f32 product, as the reference's d_w * (...)).
//  * Per-lane partials (unit order, block order) are reduced across the row's LPR lanes with DPP
//    row ops (group_sum_last); the row's last lane stores. Deterministic.
//  * AIN != 0 (fused activation quantization): A is FP32 (AIN_F32, quantized as
//    quantize_row_q8_1_ref) or FP16 (AIN_F16_FUSED, as kernels/gemm/gemm_fused.cuh:76-143) [M][K];
//    each thread quantizes whole 32-element blocks (qg_quant_block.hpp) and builds the same LDS
//    record, so every output is bit-identical to the two-step quantize + GEMV path.
//  * NT: the weight stream is loaded with the nontemporal hint (read once per launch).
// Tuning record (probes, per-wave timelines, rejected designs): profiles/r01_tuning/README.md.
#pragma once
#include "qg_common.hpp"
#include "qg_kernels.hpp"
#include "qg_quant_block.hpp"

namespace qg {

constexpr uint32_t ACC_BIAS = 0x4B400000u;  // bits of 12582912.0f = 1.5 * 2^23
constexpr float ACC_BIAS_F = 12582912.0f;

template <int F, int BPL> struct gemv_geom {
    static constexpr int BB = wfmt<F>::BB;
    static constexpr int UB = BPL * BB;          // unit bytes
    static constexpr int UDW = UB / 4;           // unit dwords (BB even, BPL even -> whole dwords)
    static constexpr int REC_DW = 12 * BPL + 4;  // LDS record dwords per (m, unit)
};

// Nibble-plane dot for Q4_0 / Q4_1 weights (see header).
template <int F> constexpr bool gemv_planes = F == FMT_Q4_0 || F == FMT_Q4_1;
// c in the record's c * s_a: Q4_0 -8 s_a, Q5_0 -16 s_a, Q4_1 / Q5_1 + m_w s_a, Q8_0 none.
template <int F> constexpr float gemv_cs = F == FMT_Q4_0 ? 8.0f : F == FMT_Q5_0 ? 16.0f : F == FMT_Q8_0 ? 0.0f : 1.0f;

// x * (f16 value in the low / high half of h), one rounding (v_fma_mix_f32 with a zero addend).
template <int HI> __device__ __forceinline__ float mixmul(uint32_t h, float x) {
    float r;
    if constexpr (HI) asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(x));
    else asm("v_fma_mix_f32 %0, %1, %2, 0 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(x));
    return r;
}
// f16 field at compile-time byte offset OFF of a register-resident byte stream, times x.
template <int OFF> __device__ __forceinline__ float mixmul_at(const uint32_t* w, float x) {
    static_assert(OFF % 2 == 0, "fp16 fields are 2-byte aligned");
    return mixmul<(OFF % 4) / 2>(w[OFF / 4], x);
}

// The 12-dword LDS record of one Q8_1 block (b[0] = f16 d | f16 s << 16, b[1..8] = qs):
//   planes: [0..3] l nibbles, [4..7] h nibbles (element pairs (4i+k, 16+4i+k) at nibbles 2k, 2k+1
//           of dword i), [11] initial accumulator bits 1.5*2^23 + 128*sum(h);
//   bytes:  [0..7] qs;
//   both:   [8] d_a, [9] c * s_a, [10] -1.5*2^23 * d_a (fp32).
template <int F> __device__ __forceinline__ void build_act_record(const uint32_t* b, uint32_t (&r)[12]) {
    const float d = h2f(b[0] & 0xFFFFu), s = h2f(b[0] >> 16);
    if constexpr (gemv_planes<F>) {
        int sh = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t a0 = b[1 + i], a1 = b[5 + i];
            r[i] = (a0 & 0x0F0F0F0Fu) | ((a1 << 4) & 0xF0F0F0F0u);
            r[4 + i] = ((a0 >> 4) & 0x0F0F0F0Fu) | (a1 & 0xF0F0F0F0u);
            sh = __builtin_amdgcn_sdot8((int)r[4 + i], 0x11111111, sh, false);
        }
        r[11] = ACC_BIAS + (uint32_t)(128 * sh);
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) r[i] = b[1 + i];
        r[11] = ACC_BIAS;
    }
    r[8] = __float_as_uint(d);
    r[9] = __float_as_uint(gemv_cs<F> * s);
    r[10] = __float_as_uint(-(d * ACC_BIAS_F));
}
template <int F> __device__ __forceinline__ void make_act_record(const uint32_t (&b)[9], uint32_t* rec) {
    uint32_t r[12];
    build_act_record<F>(b, r);
    *reinterpret_cast<uint4*>(rec) = make_uint4(r[0], r[1], r[2], r[3]);
    *reinterpret_cast<uint4*>(rec + 4) = make_uint4(r[4], r[5], r[6], r[7]);
    *reinterpret_cast<uint4*>(rec + 8) = make_uint4(r[8], r[9], r[10], r[11]);
}

// Biased int32 dot (bits of 1.5*2^23 + sumi) of block BI of a register-resident unit with its
// activation record.
template <int F, int BI> __device__ __forceinline__ uint32_t block_dot(const uint32_t* w, const uint4 (&a)[3]) {
    using T = wfmt<F>;
    constexpr int base = BI * T::BB;
    if constexpr (gemv_planes<F>) {
        const uint32_t l[4] = {a[0].x, a[0].y, a[0].z, a[0].w};
        const uint32_t h[4] = {a[1].x, a[1].y, a[1].z, a[1].w};
        uint32_t L = a[2].w;
        int H = 0;
        static_for<4>([&](auto I) {
            constexpr int i = decltype(I)::value;
            const uint32_t q = ld32<base + T::QS + 4 * i>(w);
            L = __builtin_amdgcn_udot8(q, l[i], L, false);
            H = __builtin_amdgcn_sdot8((int)(q ^ 0x88888888u), (int)h[i], H, false);
        });
        return L + ((uint32_t)H << 4);
    } else {
        const wblock wb = decode_block<F, BI>(w);
        const uint32_t av[8] = {a[0].x, a[0].y, a[0].z, a[0].w, a[1].x, a[1].y, a[1].z, a[1].w};
        int s = (int)ACC_BIAS;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = __builtin_amdgcn_sdot4((int)wb.q[i], (int)av[i], s, false);
        return (uint32_t)s;
    }
}

// The reference's per-block term from the biased dot (see header).
template <int F, int BI> __device__ __forceinline__ float block_term_rec(const uint32_t* w, uint32_t acc, const uint4& sc) {
    using T = wfmt<F>;
    constexpr int base = BI * T::BB;
    const float cf = __uint_as_float(acc);
    const float da = __uint_as_float(sc.x), cs = __uint_as_float(sc.y), nda = __uint_as_float(sc.z);
    if constexpr (F == FMT_Q4_0 || F == FMT_Q5_0) {
        const float t1 = __builtin_fmaf(da, cf, nda);  // d_a * sumi
        return mixmul_at<base>(w, t1 - cs);             // d_w * (d_a * sumi - c * s_a)
    } else if constexpr (F == FMT_Q8_0) {
        return mixmul_at<base>(w, __builtin_fmaf(da, cf, nda));  // (sumi * d_a) * d_w
    } else {
        const float fs = cf - ACC_BIAS_F;                             // exact: sumi
        const float t = mixmul_at<base>(w, da) * fs;                  // (d_w * d_a) * sumi
        return t + mixmul_at<base + T::MOFF>(w, cs);                  // + m_w * s_a
    }
}

// ------------------------------------------------------------------------------------------------
// Weight units on the tiled layout (LAY_TILED / LAY_TILED_ACT; tiled_fmt in qg_common.hpp), round 6: the
// decode GEMV of qg_gemvt.hip. A lane's unit is BPL = 4 blocks (one stage) of ONE weight row — the same bytes
// as a 4-block unit of the row layout, gathered from the stage run's planes: per k-slot q one 16-B piece of
// the row's QS plane entry (dword q of the 4 blocks), its qh dwords (Q5_x) and its f16 scales. In registers
// (UDW dwords, as the row layout's unit):
//   [b * QSD + i]  qs dword i of block b (QSD = 4; Q8_0 8: half 1 = dwords 4..7)
//   [OQH + b]      qh of block b (Q5_0 / Q5_1)
//   [OD + b / 2]   f16 d of blocks b (low half: even b)      [OM + b / 2] f16 m (Q4_1 / Q5_1)
// so every block's fields sit at compile-time register indices: no alignbyte, no address arithmetic.
template <int F, int BPL> struct gemvt_unit {
    using T = wfmt<F>;
    static constexpr int QSD = T::Q8 ? 8 : 4;
    static constexpr int OQH = BPL * QSD;
    static constexpr int OD = OQH + (T::QH >= 0 ? BPL : 0);
    static constexpr int OM = OD + BPL / 2;
    static constexpr int UDW = OM + (T::MOFF >= 0 ? BPL / 2 : 0);
    static_assert(UDW * 4 == BPL * T::BB, "the unit holds exactly its blocks' bytes");
};

template <int F, int BI, int BPL> __device__ __forceinline__ wblock decode_block_t(const uint32_t* w) {
    using T = wfmt<F>;
    using U = gemvt_unit<F, BPL>;
    wblock r;
    r.d = r.m = 0.0f;  // (the dot needs the codes only)
    if constexpr (T::Q8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) r.q[i] = w[BI * 8 + i];
        return r;
    }
    uint32_t qh = 0;
    if constexpr (T::QH >= 0) qh = w[U::OQH + BI];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t v = w[BI * 4 + i];
        uint32_t lo = v & 0x0F0F0F0Fu, hi = (v >> 4) & 0x0F0F0F0Fu;
        if constexpr (T::QH >= 0) {
            lo |= spread4_bit4((qh >> (4 * i)) & 0xFu);
            hi |= spread4_bit4((qh >> (16 + 4 * i)) & 0xFu);
        }
        r.q[i] = lo;
        r.q[4 + i] = hi;
    }
    return r;
}

// block_dot / block_term_rec of a tiled-layout unit (same arithmetic, same results bit for bit)
template <int F, int BI, int BPL> __device__ __forceinline__ uint32_t block_dot_t(const uint32_t* w, const uint4 (&a)[3]) {
    if constexpr (gemv_planes<F>) {
        const uint32_t l[4] = {a[0].x, a[0].y, a[0].z, a[0].w};
        const uint32_t h[4] = {a[1].x, a[1].y, a[1].z, a[1].w};
        uint32_t L = a[2].w;
        int H = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = w[BI * 4 + i];
            L = __builtin_amdgcn_udot8(q, l[i], L, false);
            H = __builtin_amdgcn_sdot8((int)(q ^ 0x88888888u), (int)h[i], H, false);
        }
        return L + ((uint32_t)H << 4);
    } else {
        const wblock wb = decode_block_t<F, BI, BPL>(w);
        const uint32_t av[8] = {a[0].x, a[0].y, a[0].z, a[0].w, a[1].x, a[1].y, a[1].z, a[1].w};
        int s = (int)ACC_BIAS;
#pragma unroll
        for (int i = 0; i < 8; ++i) s = __builtin_amdgcn_sdot4((int)wb.q[i], (int)av[i], s, false);
        return (uint32_t)s;
    }
}
template <int F, int BI, int BPL> __device__ __forceinline__ float block_term_t(const uint32_t* w, uint32_t acc, const uint4& sc) {
    using U = gemvt_unit<F, BPL>;
    const float cf = __uint_as_float(acc);
    const float da = __uint_as_float(sc.x), cs = __uint_as_float(sc.y), nda = __uint_as_float(sc.z);
    const uint32_t dw = w[U::OD + BI / 2];
    if constexpr (F == FMT_Q4_0 || F == FMT_Q5_0) {
        return mixmul<BI & 1>(dw, __builtin_fmaf(da, cf, nda) - cs);
    } else if constexpr (F == FMT_Q8_0) {
        return mixmul<BI & 1>(dw, __builtin_fmaf(da, cf, nda));
    } else {
        const float fs = cf - ACC_BIAS_F;
        const float t = mixmul<BI & 1>(dw, da) * fs;
        return t + mixmul<BI & 1>(w[U::OM + BI / 2], cs);
    }
}

// ------------------------------------------------------------------------------------------------
// Load the 32 activation values of block g (AIN_F32: 128 B, AIN_F16_FUSED: 64 B; 16-B aligned).
template <int AIN> __device__ __forceinline__ void load_act_block(const uint8_t* __restrict__ X, int g, float (&v)[32]) {
    if constexpr (AIN == AIN_F32) {
        const float4* p = reinterpret_cast<const float4*>(X) + (long)g * 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float4 t = p[i];
            v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
        }
    } else {
        const uint4* p = reinterpret_cast<const uint4*>(X) + (long)g * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 t = p[i];
            const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[8 * i + 2 * j] = h2f(w[j] & 0xFFFFu);
                v[8 * i + 2 * j + 1] = h2f(w[j] >> 16);
            }
        }
    }
}

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2_a4 __attribute__((ext_vector_type(2), aligned(4)));

// PRE: read the unit's LDS records into registers right after the staging barrier, before the
// first weight byte is used, so the LDS latency overlaps the weight stream and only VALU work
// remains once the weights land (MT <= 2: 12 * BPL * MT dwords of registers).
// ONEU > 1 (round 5): every lane owns at most ONEU units (K <= 32 * BPL * LPR * ONEU), all their weight loads
// issued before the activation staging, no unit loop: ONEU units of weights in flight per lane instead of the
// loop's two (the published K = 14336 decode shapes, VERDICT r04 missing #1).
// ONEU == 1: every lane owns at most one unit (K <= 32 * BPL * LPR): the kernel has no unit loop, so the
// waits for the weight loads sit at their first use, behind the record reads (with a loop in the
// kernel, hipcc's wait insertion falls back to vmcnt(0) before the first record read).
// Argument order: everything the first loads need (A, B, their batch strides, M, N, K) sits in the
// first 14 dwords, which the dispatch preloads into SGPRs (-amdgpu-kernarg-preload-count, Makefile);
// the rest (output pointer and strides, the sumi hook) is fetched by an s_load that is only waited
// for at the store, so no kernarg fetch sits in front of the weight stream.
// (The round-1..4 ablation bits and timeline stamps used to decompose this kernel live in
// profiles/tools_archive/qg_gemv_kernel_r04_knobs.hpp, not here.)
// The kernel body is shared by two entry points (below): the general one and the M = 1 one with the
// minimal argument list.
// TPW (tiles per workgroup, loop-free form only): the workgroup computes TPW consecutive row tiles of
// one product — the activations are staged and their records read ONCE for all of them, and every
// tile's weight unit is in flight before the staging barrier. Each row's arithmetic is unchanged, so
// outputs are bit-identical to TPW = 1 (used by the batched and grouped launches, whose grids have
// thousands of workgroups; the single launch keeps one tile per workgroup to fill the CUs).
// The largest M tile whose unit loop preloads the unit's records (0: per format — 4 for the byte-decode formats
// on their 512-thread workgroups, 2 for the nibble-plane ones: profiles/r06_tuning/r6l_ab_gemv_pre_mt4.txt, M = 4,
// K = 14336: Q5_0 19.18 -> 18.64 us, Q8_0 19.02 -> 18.27, but Q4_0 11.21 -> 12.32, Q4_1 12.00 -> 16.23)
#ifndef QG_GEMV_PRE_MT
#define QG_GEMV_PRE_MT 0
#endif
template <int F> constexpr int gemv_pre_mt = QG_GEMV_PRE_MT ? QG_GEMV_PRE_MT : (F == FMT_Q4_0 || F == FMT_Q4_1) ? 2 : 4;
#ifndef QG_GEMV_ACT2
#define QG_GEMV_ACT2 1  // (A/B builds) 0: M >= 2 loads each further activation block after the previous record
#endif
template <int F, int MT, int BPL, int LPR, int WGS, bool SUMI, int AIN, bool NT, bool PRE, int ONEU, int TPW = 1>
__device__ __forceinline__ void gemv_body(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, long sA, long sB,
                                          int M, int N, int K, float* __restrict__ C, long sC, long ldc_m, long ldc_n,
                                          int32_t* __restrict__ sumi_out, int tile_in = -1) {
    static_assert(TPW == 1 || ONEU == 1, "several tiles per workgroup: the one-unit form only");
    constexpr int NUN = ONEU > 1 ? ONEU : 1;  // weight units in registers per lane (loop-free forms)
    using G = gemv_geom<F, BPL>;
    A = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(A) + blockIdx.y * sA);
    B += blockIdx.y * sB;
    C += blockIdx.y * sC;
    constexpr int RPW = 64 / LPR;
    constexpr int RPB = (WGS / 64) * RPW;  // rows per workgroup
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];

    const int nb = K / QK;
    const int U = nb / BPL;  // units per row
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int lir = lane % LPR;
    // XCD-aware tile order for grids of one dispatch round (<= 512 workgroups): workgroups are placed
    // round-robin over the 8 XCDs (b -> XCD b % 8), and XCD x takes a contiguous range of row tiles,
    // so the 64-B output pieces of neighbouring workgroups dirty whole lines of ONE XCD's L2 (the
    // end-of-kernel write-back is the GEMV's largest fixed cost after the launch;
    // profiles/r02_tuning/ab_xcd.txt: M=1 3.33 -> 3.29 us, M=2 3.66 -> 3.58). Larger grids keep
    // the linear order (N=32000: 12.55 us linear, 13.28 remapped).
    // (a grouped launch passes the workgroup's tile within its item, tile_in >= 0)
    const int tile = tile_in >= 0 ? tile_in : gridDim.x <= 512 ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    int rows[TPW];
    bool rows_ok[TPW];
    const uint8_t* wrows[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        rows[t] = (tile * TPW + t) * RPB + (tid >> 6) * RPW + lane / LPR;
        rows_ok[t] = rows[t] < N;
        wrows[t] = B + (long)(rows_ok[t] ? rows[t] : 0) * ((long)U * G::UB);
    }
    const int row = rows[0];
    const bool row_ok = rows_ok[0];
    auto load_unit = [&](uint32_t (&dst)[G::UDW], int u, int t = 0) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(wrows[t] + (long)((rows_ok[t] && u < U) ? u : 0) * G::UB);
        if constexpr (NT) {
#pragma unroll
            for (int v = 0; v + 4 <= G::UDW; v += 4) {
                const u32x4_a4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4*>(p + v));
                dst[v] = t.x; dst[v + 1] = t.y; dst[v + 2] = t.z; dst[v + 3] = t.w;
            }
            if constexpr (G::UDW % 4 == 2) {
                const u32x2_a4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x2_a4*>(p + G::UDW - 2));
                dst[G::UDW - 2] = t.x; dst[G::UDW - 1] = t.y;
            }
        } else {
#pragma unroll
            for (int v = 0; v < G::UDW; ++v) dst[v] = p[v];
        }
    };
    // record of activation block blk = m * nb + b: unit (m * U + b / BPL) = blk / BPL, slot b % BPL
    auto rec_of = [&](int blk) { return (blk / BPL) * G::REC_DW + (blk % BPL) * 12; };
    uint32_t curs[NUN][G::UDW];
    uint32_t(&cur)[G::UDW] = curs[0];
    uint32_t more[TPW > 1 ? TPW - 1 : 1][G::UDW];  // tiles 1.. of the workgroup (TPW > 1)
    auto load_first = [&]() {
        load_unit(cur, lir);
#pragma unroll
        for (int j = 1; j < NUN; ++j) load_unit(curs[j], lir + j * LPR);
#pragma unroll
        for (int t = 1; t < TPW; ++t) load_unit(more[t - 1], lir, t);
    };

    // 1) activation block loads of this thread (one thread per block), the first before the
    //    weight stream; 2) the lane's first weight unit; 3) LDS records
    const int totb = M * nb;
    if constexpr (AIN == AIN_Q8_1) {
        // M >= 2: a thread's first TWO blocks are loaded before the weight stream (M = 4 at K = 14336 stages
        // 1792 blocks over 1024 threads: the second round no longer waits behind the first one's records)
        constexpr int NA = MT >= 2 && QG_GEMV_ACT2 ? 2 : 1;
        uint32_t ab[NA][9];
        auto load_ablk = [&](int g, uint32_t (&d)[9]) {
            const uint32_t* p = A + (long)g * 9;
#pragma unroll
            for (int i = 0; i < 9; ++i) d[i] = p[i];
        };
#pragma unroll
        for (int k = 0; k < NA; ++k)
            if (tid + k * WGS < totb) load_ablk(tid + k * WGS, ab[k]);
        load_first();
#pragma unroll
        for (int k = 0; k < NA; ++k)
            if (tid + k * WGS < totb) make_act_record<F>(ab[k], lds + rec_of(tid + k * WGS));
        for (int g = tid + NA * WGS; g < totb; g += WGS) {
            load_ablk(g, ab[0]);
            make_act_record<F>(ab[0], lds + rec_of(g));
        }
    } else {
        const uint8_t* X = reinterpret_cast<const uint8_t*>(A);
        float xv[32];
        if (tid < totb) load_act_block<AIN>(X, tid, xv);
        load_first();
        for (int g = tid; g < totb; g += WGS) {
            if (g != tid) load_act_block<AIN>(X, g, xv);
            uint32_t w[9];
            if constexpr (AIN == AIN_F32) quantize_q8_1_block<0>(xv, w);
            else quantize_q8_1_block_fp16_fused(xv, w);
            make_act_record<F>(w, lds + rec_of(g));
        }
    }
    __syncthreads();

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;

    // one unit of this lane: activation records preloaded (PRE) or read per block
    uint4 pre[PRE ? BPL : 1][PRE ? MT : 1][3];
    auto read_pre = [&](int u) {
        if constexpr (PRE) {
#pragma unroll
            for (int bi = 0; bi < BPL; ++bi)
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    const uint32_t* rec = lds + (min(m, M - 1) * U + u) * G::REC_DW + bi * 12;
#pragma unroll
                    for (int x = 0; x < 3; ++x) pre[bi][m][x] = *reinterpret_cast<const uint4*>(rec + 4 * x);
                }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto dot_unit = [&](const uint32_t (&cur)[G::UDW], int u, int row, bool row_ok) {
        static_for<BPL>([&](auto BI) {
            constexpr int bi = decltype(BI)::value;
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (m < M) {
                    uint4 a[3];
                    if constexpr (PRE) {
                        a[0] = pre[bi][m][0]; a[1] = pre[bi][m][1]; a[2] = pre[bi][m][2];
                    } else {
                        const uint32_t* rec = lds + (m * U + u) * G::REC_DW + bi * 12;
                        a[0] = *reinterpret_cast<const uint4*>(rec);
                        a[1] = *reinterpret_cast<const uint4*>(rec + 4);
                        a[2] = *reinterpret_cast<const uint4*>(rec + 8);
                    }
                    const uint32_t d = block_dot<F, bi>(cur, a);
                    if constexpr (SUMI) {
                        if (row_ok) sumi_out[((long)m * N + row) * nb + u * BPL + bi] = (int)(d - ACC_BIAS);
                    } else {
                        acc[m] += block_term_rec<F, bi>(cur, d, a[2]);
                    }
                }
            }
        });
    };
    auto do_unit = [&](int u) {
        read_pre(u);
        dot_unit(cur, u, row, row_ok);
    };
    const int iters = (U + LPR - 1) / LPR;
    if constexpr (TPW > 1) {
        // tiles 1.. after tile 0 (below): the records read once, each tile its own sum and store
        static_assert(!SUMI || TPW == 1, "parity hook: one tile per workgroup");
    }
    if constexpr (ONEU == 1) {
        if (lir < U) do_unit(lir);
    } else if constexpr (ONEU > 1) {
#pragma unroll
        for (int j = 0; j < NUN; ++j) {
            const int u = lir + j * LPR;
            if (u < U) {
                read_pre(u);
                dot_unit(curs[j], u, row, row_ok);
            }
        }
    } else {
        for (int j = 0; j < iters; ++j) {
            const int u = lir + j * LPR;
            uint32_t nxt[G::UDW];
            if (j + 1 < iters) load_unit(nxt, u + LPR);
            if (u < U) do_unit(u);
            if (j + 1 < iters) {
#pragma unroll
                for (int v = 0; v < G::UDW; ++v) cur[v] = nxt[v];
            }
        }
    }
    if constexpr (!SUMI) {
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = group_sum_last<LPR>(acc[m]);
        if (row_ok && lir == LPR - 1) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                if (m < M) C[m * ldc_m + row * ldc_n] = acc[m];
        }
    }
    if constexpr (TPW > 1 && !SUMI) {
#pragma unroll
        for (int t = 1; t < TPW; ++t) {
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
            if (lir < U) dot_unit(more[t - 1], lir, rows[t], rows_ok[t]);
#pragma unroll
            for (int m = 0; m < MT; ++m) acc[m] = group_sum_last<LPR>(acc[m]);
            if (rows_ok[t] && lir == LPR - 1) {
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    if (m < M) C[m * ldc_m + rows[t] * ldc_n] = acc[m];
            }
        }
    }
}

template <int F, int MT, int BPL, int LPR, int WGS, bool SUMI, int AIN = AIN_Q8_1, bool NT = false, bool PRE = (MT <= 2),
          int ONEU = 0, int TPW = 1>
__global__ __launch_bounds__(WGS) void gemv_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                   long sA, long sB, int M, int N, int K, float* __restrict__ C,
                                                   long sC, long ldc_m, long ldc_n, int32_t* __restrict__ sumi_out) {
    gemv_body<F, MT, BPL, LPR, WGS, SUMI, AIN, NT, PRE, ONEU, TPW>(A, B, sA, sB, M, N, K, C, sC, ldc_m, ldc_n, sumi_out);
}

// M = 2..8, one product: (A, B, M, N, K, out, ldc_m, ldc_n) with 32-bit output strides = 10 dwords
// (the general entry preloads 14 and s_loads the rest).
template <int F, int MT, int BPL, int LPR, int WGS, bool SUMI, int AIN = AIN_Q8_1, bool PRE = (MT <= 2), int ONEU = 0>
__global__ __launch_bounds__(WGS) void gemvs_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int M,
                                                    int N, int K, void* __restrict__ out, int ldc_m, int ldc_n) {
    gemv_body<F, MT, BPL, LPR, WGS, SUMI, AIN, false, PRE, ONEU>(A, B, 0, 0, M, N, K, SUMI ? nullptr : (float*)out, 0,
                                                                     ldc_m, ldc_n, SUMI ? (int32_t*)out : nullptr);
}

// M = 1, one product, out[n] (activation- and weight-major coincide at M = 1): the minimal argument
// list (A, B, N, K, out) = 8 dwords, all preloaded into SGPRs. Each preloaded kernel-argument dword
// costs every wave's launch: the single-launch M = 1 GEMV took 0.11 us longer with the general
// entry's 13 preloaded dwords than with these 8 (profiles/tools_archive/gemv_direct_probe.hip,
// profiles/r02_tuning/gemv_abl*.txt). SUMI: out is the parity hook's int32 buffer.
template <int F, int BPL, int LPR, int WGS, bool SUMI, int AIN = AIN_Q8_1, int ONEU = 0>
__global__ __launch_bounds__(WGS) void gemv1_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B, int N,
                                                    int K, void* __restrict__ out) {
    gemv_body<F, 1, BPL, LPR, WGS, SUMI, AIN, false, true, ONEU>(A, B, 0, 0, 1, N, K, SUMI ? nullptr : (float*)out, 0, 0,
                                                                     1, SUMI ? (int32_t*)out : nullptr);
}

// Grouped GEMV (qg_gemm_w4a8_grouped): up to GEMV_GROUP_MAX independent products with their own A,
// B, C and N (and output row stride), one M and K, in ONE launch — e.g. a decoder layer's Q / K / V
// or gate / up projections. The descriptor travels by value in the kernel arguments (GemvGroup in
// qg_kernels.hpp: no device allocation, capture-safe); blockIdx.y is the item, blockIdx.x its row
// tile, and workgroups past an item's rows exit at once (grid.x = the largest item's tiles). The
// item's pointers are ONE scalar load (32-B record); the outputs are bit-identical to the single
// launch (same body, same per-row summation). A first version located each workgroup's item in a
// tile prefix table (a lane-parallel vector load + ballot, or 64 scalar compares): 1.72 / 2.10 us per
// GEMV in a group of 64 vs 1.44 for the strided batch (the lookup sat in front of every workgroup's
// weight stream).
// Groups whose items all have the launch's row-tile count (grp.full) skip the early-exit test. (The
// round-4 item-per-XCD 1-D grid for uniform groups measured slower, 1.59 -> 1.64 us per GEMV; round 5:
// staging the activations of groups with one shared A from the preloaded header, before the item's
// descriptor returns, measured no gain — profiles/r05_tuning/r5b_ab_grouped.txt, 1.510 -> 1.516 us.)
// row tiles per workgroup of the loop-free launches (gemv_body TPW): grouped (QG_GEMVG_TPW) and strided
// batch (QG_GEMV_TPW). profiles/r04_tuning/r04d_bench_tpw*.json, 64 GEMVs (M = 1, N = K = 4096) per
// launch: grouped 1.606 -> 1.529 us per GEMV with 2 (one descriptor load and one activation staging per
// two tiles), strided batch 1.450 -> 1.452 (no descriptor to amortise: kept at 1)
#ifndef QG_GEMV_TPW
#define QG_GEMV_TPW 1
#endif
#ifndef QG_GEMVG_TPW
#define QG_GEMVG_TPW 2
#endif
// M >= 2 grouped / strided-batch launches whose items fit one round: 256-thread workgroups of two row
// tiles (profiles/r04_tuning/ab_mt_wgs_r4m.txt, 64 products per launch, N = K = 4096, vs the M = 1 rule:
// strided Q4_0 M = 2 1.72 -> 1.64 us, M = 4 2.78 -> 2.42, Q4_1 M = 3 3.54 -> 2.59; grouped Q4_0 M = 2
// 1.75 -> 1.61, M = 4 2.49 -> 2.41; Q5_x / Q8_0 within +-1 % except grouped Q8_0 M = 4 +2 %; one row tile
// per 256-thread workgroup is slower everywhere). 0: the M = 1 rule.
#ifndef QG_GEMV_MTGW
#define QG_GEMV_MTGW 256
#endif
#ifndef QG_GEMV_MTTPW
#define QG_GEMV_MTTPW 2
#endif
#ifndef QG_GEMVG_WDIV
#define QG_GEMVG_WDIV 2  // grouped launch workgroup size = the single launch's / QG_GEMVG_WDIV (below)
#endif
template <int F, int MT, int BPL, int LPR, int WGS, bool PRE, int ONEU, int TPW = 1>
__global__ __launch_bounds__(WGS) void gemvg_kernel(const GemvGroup grp) {
    constexpr int RPB = (WGS / 64) * (64 / LPR) * TPW;  // rows per workgroup
    const int item = blockIdx.y;
    // the single launch's XCD-aware tile order (gemv_body) within the item: with grid.x a multiple of 8 the
    // workgroup's XCD is blockIdx.x % 8, so each XCD takes a contiguous range of its tiles
    const int tile = gridDim.x <= 512 ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const GemvItemDesc d = grp.it[item];
    if (!grp.full && tile * RPB >= d.N) return;  // past this item's rows (uniform)
    gemv_body<F, MT, BPL, LPR, WGS, false, AIN_Q8_1, false, PRE, ONEU, TPW>(
        reinterpret_cast<const uint32_t*>(d.A), reinterpret_cast<const uint8_t*>(d.B), 0, 0, grp.M, d.N, grp.K,
        d.C, 0, d.ldc, 1, nullptr, tile);
}

// Loop-free multi-unit single launches (ONEU = 2 / 4, above): 1 = on, 0 = the unit loop (A/B builds).
#ifndef QG_GEMV_NU
#define QG_GEMV_NU 1
#endif
#ifndef QG_GEMV_NU_MT
#define QG_GEMV_NU_MT 1  // (A/B builds) the largest M tile that takes the multi-unit form
#endif

// Host side -------------------------------------------------------------------------------------

template <int F, int BPL> inline size_t gemv_lds_bytes(int M, int K) {
    return (size_t)M * (K / QK / BPL) * gemv_geom<F, BPL>::REC_DW * 4;
}

// Preconditions of the kernel for unit size BPL: whole units per row, 4-byte aligned operands
// (units and rows are then whole dwords), LDS records fit.
template <int F, int BPL>
inline bool gemv_shape_ok(const GemmArgs& g) {
    if (g.M < 1 || g.M > 8) return false;
    if (g.K % (QK * BPL) != 0) return false;
    const int aal = g.ain == AIN_Q8_1 ? 3 : 15;  // fused: 16-B vector loads of the FP32/FP16 rows
    if (((uintptr_t)g.B & 3) != 0 || ((uintptr_t)g.A & aal) != 0) return false;
    if (g.batch > 1 && ((g.sB & 3) != 0 || (g.sA & aal) != 0)) return false;
    if (g.sumi && g.ain != AIN_Q8_1) return false;
    if (g.M > 2 && gemv_lds_bytes<F, BPL>(g.M, g.K) > 96 * 1024) return false;
    return true;
}

template <int F, int MT, int BPL, int LPR, int WGS, bool SUMI, int AIN = AIN_Q8_1, bool NT = false, bool PRE = (MT <= 2)>
hipError_t gemv_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    const size_t lds = gemv_lds_bytes<F, BPL>(g.M, g.K);
    const int grid = (g.N + RPB - 1) / RPB;
    const bool one = g.K / QK / BPL <= LPR;
    // units per lane of the loop-free multi-unit form: Q4_0 M = 1 single launches only (0: the unit loop).
    // profiles/r05_tuning/r5zd_ab.txt, unit loop -> multi-unit: Q4_0 M = 1 K = 14336 7.69 -> 7.46 us, K = 11008
    // 6.32 -> 6.17, K = 8192 5.02 -> 4.78; slower for M = 2..4 (8.93 -> 9.45 at M = 2), Q4_1 (8.02 -> 9.50) and
    // Q8_0 (12.37 -> 12.53), which keep the loop
    constexpr bool NU_OK = QG_GEMV_NU && MT <= QG_GEMV_NU_MT && F == FMT_Q4_0;
    const int nu_all = (g.K / QK / BPL + LPR - 1) / LPR;
    const int nu = one ? 1 : !NU_OK ? 0 : nu_all <= 2 ? 2 : nu_all <= 4 ? 4 : 0;
    // M = 1, one product, unit output stride: the minimal-argument entry (gemv1_kernel)
    const bool m1 = MT == 1 && PRE && !NT && g.M == 1 && g.batch == 1 && g.ldc_n == 1;
    const bool shrt = !m1 && !NT && g.batch == 1 && g.ldc_m <= INT32_MAX && g.ldc_n <= INT32_MAX;
    // the ONEU the chosen entry launches: the short entry takes the multi-unit form only when
    // NU_OK && MT > 1, otherwise its loop (ONEU 0) or the one-unit form
    const int oneu = m1 ? nu : shrt ? ((nu > 1 && !(NU_OK && MT > 1)) ? 0 : nu) : (int)one;
    if (g.group && (SUMI || AIN != AIN_Q8_1 || NT || MT > 4)) return hipErrorInvalidValue;  // no grouped form here
    if (g.describe) {  // qg_debug_config: name the instantiation instead of launching it
        describe_kernel(g, "gemv F=%d MT=%d BPL=%d LPR=%d WGS=%d AIN=%d NT=%d PRE=%d ONEU=%d SIG=%s grid=%dx%d", F, MT, BPL,
                        LPR, WGS, AIN, (int)NT, (int)(one ? PRE : (PRE && MT <= (shrt && !oneu ? gemv_pre_mt<F> : 2))), oneu,
                        m1 ? "m1" : shrt ? "short" : "full",
                        grid, g.batch);
        return hipSuccess;
    }
    if constexpr (!SUMI && AIN == AIN_Q8_1 && !NT && MT <= 4) {  // (AUTO sends only M <= 4 to the GEMV)
        if (g.group) {  // grouped launch (qg_gemm_w4a8_grouped): blockIdx.y = item
            const GemvGroup& grp0 = *static_cast<const GemvGroup*>(g.group);
            auto go = [&](auto GWc, auto TPc) -> hipError_t {
                constexpr int GW = decltype(GWc)::value, TP = decltype(TPc)::value;
                GemvGroup grp = grp0;
                constexpr int RPBG = (GW / 64) * (64 / LPR);
                const int rpw = one ? RPBG * TP : RPBG;  // rows per workgroup
                int tiles = 0, tmin = INT32_MAX;
                for (int i = 0; i < grp.count; ++i) {
                    const int t = (grp.it[i].N + rpw - 1) / rpw;
                    tiles = std::max(tiles, t);
                    tmin = std::min(tmin, t);
                }
                auto kg = one ? gemvg_kernel<F, MT, BPL, LPR, GW, PRE, true, TP>
                              : gemvg_kernel<F, MT, BPL, LPR, GW, PRE && (MT <= 2), false>;
                if (lds > 64 * 1024) {
                    hipError_t e = hipFuncSetAttribute((const void*)kg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                    if (e != hipSuccess) return e;
                }
                if (tiles == 0 || grp.count == 0) return hipSuccess;
                grp.full = tiles == tmin ? 1 : 0;
                hipLaunchKernelGGL(kg, dim3(tiles, grp.count), dim3(GW), lds, st, grp);
                return hipGetLastError();
            };
            // workgroups of WGS / QG_GEMVG_WDIV threads while the largest item's rows fit one round of
            // full-size workgroups (<= 256): twice as many resident per CU, so one workgroup's descriptor
            // load and activation staging overlap another's weight stream (profiles/r04_tuning/
            // ab_grouped_wgs_r4g2.txt, 64 items per launch, N = K = 4096: Q4_0 M = 1 1.541 -> 1.509 us per
            // GEMV, M = 2 1.853 -> 1.688, M = 4 2.705 -> 2.494, Q8_0 2.885 -> 2.767; N = 11008 (344 tiles)
            // 3.92 -> 4.01 with them, so larger items keep full-size workgroups)
            constexpr bool MTW = QG_GEMV_MTGW > 0 && MT >= 2;
            constexpr int GWH = MTW ? (QG_GEMV_MTGW < WGS ? QG_GEMV_MTGW : WGS) : WGS / QG_GEMVG_WDIV;
            constexpr int TPH = MTW ? QG_GEMV_MTTPW : QG_GEMVG_TPW;
            if constexpr (GWH < WGS && GWH >= 64) {
                const int rpw_full = one ? RPB * QG_GEMVG_TPW : RPB;
                int nmax = 0;
                for (int i = 0; i < grp0.count; ++i) nmax = std::max(nmax, grp0.it[i].N);
                if ((nmax + rpw_full - 1) / rpw_full <= device_cus())
                    return go(std::integral_constant<int, GWH>{}, std::integral_constant<int, TPH>{});
            }
            return go(std::integral_constant<int, WGS>{}, std::integral_constant<int, QG_GEMVG_TPW>{});
        }
    }
    if (m1) {
        auto k1 = nu == 1 ? gemv1_kernel<F, BPL, LPR, WGS, SUMI, AIN, 1> : gemv1_kernel<F, BPL, LPR, WGS, SUMI, AIN, 0>;
        if constexpr (NU_OK) {
            if (nu == 2) k1 = gemv1_kernel<F, BPL, LPR, WGS, SUMI, AIN, 2>;
            if (nu == 4) k1 = gemv1_kernel<F, BPL, LPR, WGS, SUMI, AIN, 4>;
        }
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        void* out = SUMI ? (void*)g.sumi : (void*)g.C;
        hipLaunchKernelGGL(k1, dim3(grid), dim3(WGS), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.N, g.K, out);
        return hipGetLastError();
    }
    // one product with 32-bit output strides: the short-argument entry (gemvs_kernel)
    if (shrt) {
        auto ks = one ? gemvs_kernel<F, MT, BPL, LPR, WGS, SUMI, AIN, PRE, 1>
                      : gemvs_kernel<F, MT, BPL, LPR, WGS, SUMI, AIN, PRE && (MT <= gemv_pre_mt<F>), 0>;
        if constexpr (NU_OK && MT > 1) {
            if (nu == 2) ks = gemvs_kernel<F, MT, BPL, LPR, WGS, SUMI, AIN, PRE && (MT <= 2), 2>;
            if (nu == 4) ks = gemvs_kernel<F, MT, BPL, LPR, WGS, SUMI, AIN, PRE && (MT <= 2), 4>;
        }
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void*)ks, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        void* out = SUMI ? (void*)g.sumi : (void*)g.C;
        hipLaunchKernelGGL(ks, dim3(grid), dim3(WGS), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, out,
                           (int)g.ldc_m, (int)g.ldc_n);
        return hipGetLastError();
    }
    // PRE beyond MT = 2 only in the loop-free form (with the unit loop it spills at MT = 4); a strided
    // batch of loop-free GEMVs takes QG_GEMV_TPW row tiles per workgroup (same per-row arithmetic)
// A strided batch of loop-free GEMVs whose N fits one round of full-size workgroups runs half-size
// ones, as the grouped launch (profiles/r04_tuning/ab_batched_wgs_r4b.txt, 64 products per launch,
// N = K = 4096: Q4_0 M = 1 1.526 -> 1.478 us per GEMV, M = 2 1.772 -> 1.641, M = 4 3.32 -> 2.76,
// N = 1024 0.436 -> 0.421; Q5_0 / Q8_0 M = 1 within +-0.7 %)
#ifndef QG_GEMVB_WDIV
#define QG_GEMVB_WDIV 2
#endif
    constexpr bool MTB = QG_GEMV_MTGW > 0 && MT >= 2;
    constexpr int GWB = MTB ? (QG_GEMV_MTGW < WGS ? QG_GEMV_MTGW : WGS) : WGS / QG_GEMVB_WDIV;
    constexpr int TPB = MTB ? QG_GEMV_MTTPW : QG_GEMV_TPW;
    if constexpr (GWB < WGS && GWB >= 64 && !SUMI && !NT) {
        constexpr int GW = GWB, RPBB = (GW / 64) * (64 / LPR) * TPB;
        if (one && g.batch > 1 && grid <= device_cus()) {
            auto kb = gemv_kernel<F, MT, BPL, LPR, GW, SUMI, AIN, NT, PRE, true, TPB>;
            if (lds > 64 * 1024) {
                hipError_t e = hipFuncSetAttribute((const void*)kb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(kb, dim3((g.N + RPBB - 1) / RPBB, g.batch), dim3(GW), lds, st, (const uint32_t*)g.A,
                               (const uint8_t*)g.B, g.sA, g.sB, g.M, g.N, g.K, g.C, g.sC, g.ldc_m, g.ldc_n, g.sumi);
            return hipGetLastError();
        }
    }
    constexpr bool tpw_ok = !SUMI && !NT && QG_GEMV_TPW > 1;
    const bool multi = tpw_ok && one && g.batch > 1;
    auto kfn = multi ? gemv_kernel<F, MT, BPL, LPR, WGS, SUMI, AIN, NT, PRE, true, tpw_ok ? QG_GEMV_TPW : 1>
             : one   ? gemv_kernel<F, MT, BPL, LPR, WGS, SUMI, AIN, NT, PRE, true>
                     : gemv_kernel<F, MT, BPL, LPR, WGS, SUMI, AIN, NT, PRE && (MT <= 2), false>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const int gx = multi ? (g.N + RPB * QG_GEMV_TPW - 1) / (RPB * QG_GEMV_TPW) : grid;
    hipLaunchKernelGGL(kfn, dim3(gx, g.batch), dim3(WGS), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.sA,
                       g.sB, g.M, g.N, g.K, g.C, g.sC, g.ldc_m, g.ldc_n, g.sumi);
    return hipGetLastError();
}

}  // namespace qg
