// qg_w4a16.hip — W4A16 / W8A16: FP32 activations x Q4_0 / Q8_0 weights, fp32 arithmetic.
//
// C[M,N] = A_f32[M,K] . dequant(B_w[N,K])^T, activation-major, the device twin of
// gemm_w4a16_reference (include/gemm_reference.h:73-112; GPU: gemm_w4a16_{naive,tiled},
// include/gemm_cuda_naive.cuh:267-274, gemm_cuda_tiled.cuh:284-291; python/quant_gemm/csrc/
// gemm_ops.cu:431-466 gemm_q4_0_fp32) and of gemm_w8a16_naive (gemm_cuda_naive.cuh:276-283).
//
// The reference accumulates a[k] * ((q[k] - 8) * d) element by element into one fp32 sum. Here a
// block's 32 products a[k] * (q[k] - 8) (q - 8 exact in fp32) are fma-accumulated, then scaled
// by d once: the same real value, different rounding — the parity bar is the fp32
// summation-order bound over the K element terms (tests/test_gpu_w4a16.py).
//
// GEMV-shaped decomposition as the W4A8 GEMV (qg_gemv_kernel.hpp): lanes own units of BPL blocks
// of one weight row (register-resident decode), the activations are staged once per workgroup
// into LDS records [m][unit][BPL x 32 floats] (+4 dwords pad: the 16 lanes of a ds_read_b128 group
// read units at a stride of 4 x odd dwords, distinct bank slots), rows reduce with DPP. M > 8
// runs on the matrix cores instead (w16_mfma_kernel below; the GEMV's row chunks remain for
// activations that are not 16-B aligned).
#include "qg_common.hpp"
#include "qg_kernels.hpp"

#include <algorithm>

namespace qg {

template <int F, int BPL> struct w16_geom {
    static constexpr int BB = wfmt<F>::BB;
    static constexpr int UB = BPL * BB;
    static constexpr int UDW = UB / 4;
    static constexpr int REC_DW = 32 * BPL + 4;
    static_assert(UB % 4 == 0, "whole-dword units");
};

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// Exact float value of weight element j (0..3) of decoded dword x: q - 8 (Q4_0), q (Q8_0).
template <int F> __device__ __forceinline__ float w16_elem(uint32_t x, int j) {
    if constexpr (F == FMT_Q8_0) return (float)(int)(int8_t)(x >> (8 * j));
    else return (float)((x >> (8 * j)) & 0xFFu) - 8.0f;
}

// One block of a lane's unit against its activation records (registers or LDS): element pairs on
// the packed-f32 ALU — byte -> f32 (v_cvt_f32_ubyte*), minus the offset as one v_pk_add per pair
// (Q8_0: sign bit flipped first, offset 128), one v_pk_fma per pair into two pair accumulators;
// exact weight values.
template <int F> __device__ __forceinline__ float w16_block_dot(const wblock& wb, const float4* a4) {
    constexpr float OFF = F == FMT_Q8_0 ? -128.0f : -8.0f;
    f32x2 p0 = {0.0f, 0.0f}, p1 = {0.0f, 0.0f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t x = F == FMT_Q8_0 ? wb.q[i] ^ 0x80808080u : wb.q[i];
        const f32x2 w0 = f32x2{(float)(x & 0xFFu), (float)((x >> 8) & 0xFFu)} + f32x2{OFF, OFF};
        const f32x2 w1 = f32x2{(float)((x >> 16) & 0xFFu), (float)(x >> 24)} + f32x2{OFF, OFF};
        const float4 a = a4[i];
        p0 = __builtin_elementwise_fma(f32x2{a.x, a.y}, w0, p0);
        p1 = __builtin_elementwise_fma(f32x2{a.z, a.w}, w1, p1);
    }
    return (p0.x + p1.x) + (p0.y + p1.y);
}

// ONEU (MT == 1, K <= 32 * BPL * LPR): every lane owns at most one unit, so there is no unit loop;
// the lane's activation records are read into registers right after the staging barrier, before
// its weights land (as the W4A8 GEMV's PRE / ONEU, qg_gemv_kernel.hpp), leaving only VALU work
// once the weight bytes arrive.
// The body is shared by the general entry and the M = 1 one with the minimal argument list (below).
template <int F, int MT, int BPL, int LPR, int WGS, bool ONEU>
__device__ __forceinline__ void w16_gemv_body(const float* __restrict__ A, const uint8_t* __restrict__ B, long sA, int M,
                                              int N, int K, float* __restrict__ C, long sC, long ldc_m, long ldc_n) {
    using G = w16_geom<F, BPL>;
    // chunk of <= MT activation rows
    A += blockIdx.y * sA;
    C += blockIdx.y * sC;
    M = min(MT, M - (int)blockIdx.y * MT);
    constexpr int RPW = 64 / LPR;
    constexpr int RPB = (WGS / 64) * RPW;
    extern __shared__ __attribute__((aligned(16))) float lds_f[];

    const int nb = K / QK;
    const int U = nb / BPL;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int lir = lane % LPR;
const int row = blockIdx.x * RPB + (tid >> 6) * RPW + lane / LPR;
    const bool row_ok = row < N;

    // 1) first activation float4s in flight, 2) this lane's first weight unit, 3) stage to LDS
    const int tot4 = M * (K / 4);
    constexpr int NPRE = 4;
    float4 av[NPRE];
#pragma unroll
    for (int i = 0; i < NPRE; ++i) {
        const int g = tid + i * WGS;
        av[i] = g < tot4 ? reinterpret_cast<const float4*>(A)[g] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const uint8_t* wrow = B + (long)(row_ok ? row : 0) * ((long)U * G::UB);
    auto load_unit = [&](uint32_t (&dst)[G::UDW], int u) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(wrow + (long)((row_ok && u < U) ? u : 0) * G::UB);
#pragma unroll
        for (int v = 0; v < G::UDW; ++v) dst[v] = p[v];
    };
    uint32_t cur[G::UDW];
    load_unit(cur, lir);
    const int k4 = K / 4;
    auto stage = [&](int g, float4 v) {
        const int m = g / k4;
        const int e4 = g - m * k4;
        const int b = e4 >> 3;
        const int u = b / BPL;
        *reinterpret_cast<float4*>(lds_f + (m * U + u) * G::REC_DW + (b - u * BPL) * 32 + (e4 & 7) * 4) = v;
    };
#pragma unroll
    for (int i = 0; i < NPRE; ++i) {
        const int g = tid + i * WGS;
        if (g < tot4) stage(g, av[i]);
    }
    for (int g = tid + NPRE * WGS; g < tot4; g += WGS) stage(g, reinterpret_cast<const float4*>(A)[g]);
    __syncthreads();

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;

    auto block_dot = [&](const wblock& wb, const float4* a4) { return w16_block_dot<F>(wb, a4); };
    if constexpr (ONEU) {
        static_assert(MT == 1, "one activation row");
        const int u = lir;
        float4 pre[BPL][8];
        if (u < U) {
#pragma unroll
            for (int bi = 0; bi < BPL; ++bi)
#pragma unroll
                for (int i = 0; i < 8; ++i) pre[bi][i] = *reinterpret_cast<const float4*>(lds_f + u * G::REC_DW + bi * 32 + 4 * i);
            __builtin_amdgcn_sched_barrier(0);
            static_for<BPL>([&](auto BI) {
                const wblock wb = decode_block<F, decltype(BI)::value>(cur);
                acc[0] = __builtin_fmaf(wb.d, block_dot(wb, pre[decltype(BI)::value]), acc[0]);
            });
        }
    }
    const int iters = ONEU ? 0 : (U + LPR - 1) / LPR;
    for (int j = 0; j < iters; ++j) {
        const int u = lir + j * LPR;
        uint32_t nxt[G::UDW];
        if (j + 1 < iters) load_unit(nxt, u + LPR);
        if (u < U) {
            static_for<BPL>([&](auto BI) {
                constexpr int bi = decltype(BI)::value;
                const wblock wb = decode_block<F, bi>(cur);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < M) {
                        const float* rec = lds_f + (m * U + u) * G::REC_DW + bi * 32;
                        const float s = block_dot(wb, reinterpret_cast<const float4*>(rec));
                        acc[m] = __builtin_fmaf(wb.d, s, acc[m]);
                    }
                }
            });
        }
        if (j + 1 < iters) {
#pragma unroll
            for (int v = 0; v < G::UDW; ++v) cur[v] = nxt[v];
        }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = group_sum_last<LPR>(acc[m]);
    if (row_ok && lir == LPR - 1) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
            if (m < M) C[m * ldc_m + row * ldc_n] = acc[m];
    }
}

// (arguments the first loads need lead, within the 14 preloaded kernarg dwords: qg_gemv_kernel.hpp)
template <int F, int MT, int BPL, int LPR, int WGS, bool ONEU = false>
__global__ __launch_bounds__(WGS) void w16_gemv_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B,
                                                       long sA, int M, int N, int K, float* __restrict__ C,
                                                       long sC, long ldc_m, long ldc_n) {
    w16_gemv_body<F, MT, BPL, LPR, WGS, ONEU>(A, B, sA, M, N, K, C, sC, ldc_m, ldc_n);
}

// M = 1, unit output stride: (A, B, N, K, C) = 8 preloaded argument dwords (as the W4A8 GEMV's
// gemv1_kernel, qg_gemv_kernel.hpp: every preloaded dword costs each wave's launch)
template <int F, int BPL, int LPR, int WGS, bool ONEU = false>
__global__ __launch_bounds__(WGS) void w16_gemv1_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B, int N,
                                                        int K, float* __restrict__ C) {
    w16_gemv_body<F, 1, BPL, LPR, WGS, ONEU>(A, B, 0, 1, N, K, C, 0, 0, 1);
}

// M = 1, one 2-block unit per lane (K <= 4096), RPL weight rows per wave: the lane reads its 64
// activation floats from LDS once and uses them for RPL rows (rows w, w + W, ... of the workgroup's
// RPL * W), so the workgroup's LDS reads shrink RPL-fold (each row needs all K activations; with one
// row per wave a CU re-reads the 16 KB vector 16 times). Per row the same summation order as the
// one-row kernel: bit-identical outputs.
template <int F, int WGS, int RPL>
__global__ __launch_bounds__(WGS) void w16_gemv1r_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B, int N,
                                                         int K, float* __restrict__ C) {
    using G = w16_geom<F, 2>;
    constexpr int W = WGS / 64;
    extern __shared__ __attribute__((aligned(16))) float lds_f[];
    const int nb = K / QK, U = nb / 2;  // U <= 64
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int k4 = K / 4;
    constexpr int NPRE = 4;
    float4 av[NPRE];
#pragma unroll
    for (int i = 0; i < NPRE; ++i) {
        const int g = tid + i * WGS;
        av[i] = g < k4 ? reinterpret_cast<const float4*>(A)[g] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    uint32_t cur[RPL][G::UDW];
    const int u = lane < U ? lane : 0;
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
        const int row = blockIdx.x * (W * RPL) + j * W + wave;
        const uint32_t* p = reinterpret_cast<const uint32_t*>(B + (long)(row < N ? row : 0) * ((long)U * G::UB) + (long)u * G::UB);
#pragma unroll
        for (int v = 0; v < G::UDW; ++v) cur[j][v] = p[v];
    }
    auto stage = [&](int g, float4 v) {
        const int b = g >> 3, uu = b >> 1;
        *reinterpret_cast<float4*>(lds_f + uu * G::REC_DW + (b & 1) * 32 + (g & 7) * 4) = v;
    };
#pragma unroll
    for (int i = 0; i < NPRE; ++i) {
        const int g = tid + i * WGS;
        if (g < k4) stage(g, av[i]);
    }
    for (int g = tid + NPRE * WGS; g < k4; g += WGS) stage(g, reinterpret_cast<const float4*>(A)[g]);
    __syncthreads();
    float acc[RPL];
#pragma unroll
    for (int j = 0; j < RPL; ++j) acc[j] = 0.0f;
    if (lane < U) {
        float4 pre[2][8];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
            for (int i = 0; i < 8; ++i) pre[bi][i] = *reinterpret_cast<const float4*>(lds_f + lane * G::REC_DW + bi * 32 + 4 * i);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < RPL; ++j)
            static_for<2>([&](auto BI) {
                const wblock wb = decode_block<F, decltype(BI)::value>(cur[j]);
                acc[j] = __builtin_fmaf(wb.d, w16_block_dot<F>(wb, pre[decltype(BI)::value]), acc[j]);
            });
    }
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
        acc[j] = group_sum_last<64>(acc[j]);
        const int row = blockIdx.x * (W * RPL) + j * W + wave;
        if (lane == 63 && row < N) C[row] = acc[j];
    }
}

// Any K % 32 == 0 and alignment: one wave per output element, lanes stride over blocks.
template <int F>
__global__ __launch_bounds__(256) void w16_generic_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B,
                                                          float* __restrict__ C, int M, int N, int K, long ldc_m,
                                                          long ldc_n) {
    using T = wfmt<F>;
    const int nb = K / QK;
    const int lane = threadIdx.x & 63;
    const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int m = blockIdx.y;
    if (n >= N) return;  // wave-uniform
    float acc = 0.0f;
    for (int b = lane; b < nb; b += 64) {
        const uint8_t* wb = B + ((long)n * nb + b) * T::BB;
        const float* a = A + (long)m * K + b * QK;
        const float d = h2f((uint32_t)wb[0] | ((uint32_t)wb[1] << 8));
        float s = 0.0f;
        if constexpr (F == FMT_Q8_0) {
#pragma unroll
            for (int j = 0; j < 32; ++j) s = __builtin_fmaf(a[j], (float)(int8_t)wb[2 + j], s);
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                s = __builtin_fmaf(a[j], (float)(wb[2 + j] & 0xF) - 8.0f, s);
                s = __builtin_fmaf(a[j + 16], (float)(wb[2 + j] >> 4) - 8.0f, s);
            }
        }
        acc = __builtin_fmaf(d, s, acc);
    }
    acc = group_sum_last<64>(acc);
    if (lane == 63) C[m * ldc_m + n * ldc_n] = acc;
}

// ------------------------------------------------------------------------------------------------
// Prefill (M > 8): bf16 MFMA with exact operands. A Q4_0 / Q8_0 weight code minus its offset
// (q - 8, or the signed Q8_0 byte) is an exact bf16; an fp32 activation is split exactly into three
// bf16 parts, a = hi + mid + lo (each the truncated top 8 significant bits of what is left; 24 bits
// in all). Per block and 16 x 16 tile, three chained v_mfma_f32_16x16x32_bf16 (K = 32 = one block)
// accumulate sum_k w_k (hi_k + mid_k + lo_k) in fp32 — the block's exact-product dot — and the
// epilogue adds d_w * dot into the output accumulator. Operand maps (cdna_hip_programming.md §3):
// lane l holds A[row l&15][k = 8(l>>4) + j] and B[k][col l&15]; C col = l&15, row = 4(l>>4) + e.
// Here k = element index within the block, rows = weight rows, cols = tokens.
// A workgroup owns 16 RT rows x 16 TT tokens; its W waves split the blocks round-robin (the next
// block's loads in flight while the current one computes); partial tiles are summed in fixed wave
// order through LDS at the end.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x4a4_t __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ uint32_t hi16_pack(uint32_t lo_elem, uint32_t hi_elem) {
    return __builtin_amdgcn_perm(hi_elem, lo_elem, 0x07060302u);  // {lo_elem[31:16], hi_elem[31:16]}
}

// hi = RNE_bf16 of a clamped to the largest finite bf16 (0x7F7F): a finite |a| >= (2 - 2^-8) 2^127 would
// otherwise round hi to inf and make mid = a - hi = -inf, hi + mid = NaN. With the clamp
// hi stays finite, a - hi is still exact (same binade) and |a - hi - mid| <= 2^-17 |a|; an infinite a
// gives hi = max, mid = inf (the product is inf, as the reference's); NaN stays NaN.
// The truncated three-part split clamps the same way before each truncation (only an infinite a or
// residual is changed by it: |a| <= FLT_MAX truncates to a finite bf16), so an infinite a gives
// hi = mid = max and lo = inf, an infinite product instead of inf - inf = NaN.
__device__ __forceinline__ float bf16_clamp(float a) {
    constexpr float BFMAX = 0x1.fep127f;  // 0x7F7F0000
    return __builtin_amdgcn_fmed3f(a, -BFMAX, BFMAX);
}
__device__ __forceinline__ uint32_t bf16x2_rne_clamped(float a0, float a1) {
    const f32x2 c = {bf16_clamp(a0), bf16_clamp(a1)};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(c, bf16x2_t));
}

// 8 fp32 activations -> hi / mid / lo bf16 fragments with a = hi + mid + lo exactly
__device__ __forceinline__ void w16_afrag(const float4 x0, const float4 x1, u32x4_t& h, u32x4_t& m, u32x4_t& l) {
    const float a[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    uint32_t hb[8], mb[8], lb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        hb[j] = __float_as_uint(bf16_clamp(a[j])) & 0xFFFF0000u;
        const float r1 = a[j] - __uint_as_float(hb[j]);
        mb[j] = __float_as_uint(bf16_clamp(r1)) & 0xFFFF0000u;
        const float r2 = r1 - __uint_as_float(mb[j]);
        lb[j] = __float_as_uint(r2);  // <= 8 significant bits left: its top half is exact
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        h[p] = hi16_pack(hb[2 * p], hb[2 * p + 1]);
        m[p] = hi16_pack(mb[2 * p], mb[2 * p + 1]);
        l[p] = hi16_pack(lb[2 * p], lb[2 * p + 1]);
    }
}

// 8 fp32 activations -> two bf16 fragments, hi = RNE(a), mid = RNE(a - hi) (a - hi exact): a = hi + mid
// + r with |r| <= 2^-16 |a| (w16s_parts: from K = 1024 on, inside the K-term bound by a factor >= 8)
__device__ __forceinline__ void w16_afrag2(const float4 x0, const float4 x1, u32x4_t& h, u32x4_t& m) {
    const float a[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const f32x2 v = {a[2 * p], a[2 * p + 1]};
        const uint32_t h2 = bf16x2_rne_clamped(a[2 * p], a[2 * p + 1]);
        const f32x2 r = v - f32x2{__uint_as_float(h2 << 16), __uint_as_float(h2 & 0xFFFF0000u)};  // exact
        h[p] = h2;
        m[p] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2_t));
    }
}

template <int F, int RT, int TT, int W>
__global__ __launch_bounds__(W * 64) void w16_mfma_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B,
                                                          float* __restrict__ C, int M, int N, int K, long ldc_m,
                                                          long ldc_n) {
    using T = wfmt<F>;
    constexpr int NACC = RT * TT * 4;
    extern __shared__ __attribute__((aligned(16))) float red[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * 16 * RT, m0 = blockIdx.y * 16 * TT;
    const int nb = K / QK;
    const long RB = (long)nb * T::BB;

    const uint8_t* wrow[RT];
    const float* arow[TT];
#pragma unroll
    for (int i = 0; i < RT; ++i) wrow[i] = B + (long)min(n0 + 16 * i + r16, N - 1) * RB;
#pragma unroll
    for (int t = 0; t < TT; ++t) arow[t] = A + (long)min(m0 + 16 * t + r16, M - 1) * K + 8 * q;

    struct raw_t {
        uint32_t wq[RT][2];
        uint32_t wd[RT];
        float4 a[TT][2];
    };
    auto load = [&](raw_t& r, int b) {
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const uint8_t* blk = wrow[i] + (long)b * T::BB;
            __builtin_memcpy(r.wq[i], blk + 2 + (T::Q8 ? 8 * q : 8 * (q & 1)), 8);
            r.wd[i] = *reinterpret_cast<const uint16_t*>(blk);
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) {
            const float4* p = reinterpret_cast<const float4*>(arow[t] + b * QK);
            r.a[t][0] = p[0];
            r.a[t][1] = p[1];
        }
    };

    float acc[NACC];
#pragma unroll
    for (int x = 0; x < NACC; ++x) acc[x] = 0.0f;

    raw_t cur, nxt;
    if (wave < nb) load(cur, wave);
    for (int b = wave; b < nb; b += W) {
        if (b + W < nb) load(nxt, b + W);
        u32x4_t wf[RT], ah[TT], am[TT], al[TT];
        float dw[RT][4];
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            float v[8];
            if constexpr (T::Q8) {
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (float)(int)(int8_t)(cur.wq[i][j / 4] >> (8 * (j & 3)));
            } else {
                const int sh = (q >> 1) * 4;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (float)((cur.wq[i][j / 4] >> (8 * (j & 3) + sh)) & 0xFu) - 8.0f;
            }
#pragma unroll
            for (int p = 0; p < 4; ++p) wf[i][p] = hi16_pack(__float_as_uint(v[2 * p]), __float_as_uint(v[2 * p + 1]));
            const float d_own = h2f(cur.wd[i]);  // this lane's row r16
#pragma unroll
            for (int e = 0; e < 4; ++e) dw[i][e] = __shfl(d_own, 4 * q + e);  // rows 4q + e
        }
#pragma unroll
        for (int t = 0; t < TT; ++t) w16_afrag(cur.a[t][0], cur.a[t][1], ah[t], am[t], al[t]);
        f32x4_t c[RT][TT];
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t)
                c[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[i]),
                                                                  __builtin_bit_cast(bf16x8_t, ah[t]),
                                                                  f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t)
                c[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[i]),
                                                                  __builtin_bit_cast(bf16x8_t, am[t]), c[i][t], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t)
                c[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, wf[i]),
                                                                  __builtin_bit_cast(bf16x8_t, al[t]), c[i][t], 0, 0, 0);
        // MFMA results read by the VALU only behind an explicit wait (see qg_mmq_kernel.hpp)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float ce = c[i][t][e];
                    acc[(i * TT + t) * 4 + e] = __builtin_fmaf(dw[i][e], ce, acc[(i * TT + t) * 4 + e]);
                }
        if (b + W < nb) cur = nxt;
    }

    // fixed-order sum of the W partial tiles
#pragma unroll
    for (int x = 0; x < NACC; ++x) red[(wave * NACC + x) * 64 + lane] = acc[x];
    __syncthreads();
    for (int idx = threadIdx.x; idx < NACC * 64; idx += W * 64) {
        float v = red[idx];
#pragma unroll
        for (int ww = 1; ww < W; ++ww) v += red[ww * NACC * 64 + idx];
        const int x = idx >> 6, ln = idx & 63;
        const int e = x & 3, t = (x >> 2) % TT, i = (x >> 2) / TT;
        const int n = n0 + 16 * i + 4 * (ln >> 4) + e;
        const int m = m0 + 16 * t + (ln & 15);
        if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
    }
}

// Split-K prefill (M > 8; round-1 second design, replaces w16_mfma_kernel where it applies).
// w16_mfma_kernel re-reads and re-splits all M x K fp32 activations in every workgroup (512 KB per
// workgroup at M = 32, K = 4096: 26 us). Here a workgroup owns 16 RT weight rows x 16 TT tokens x
// one K slice (blockIdx.z): it splits each activation once into hi / mid / lo bf16 fragment images
// in LDS (lane-linear, one ds_read_b128 per operand), every wave owns one 16-row tile and takes its
// weights straight from HBM into registers (all KB blocks of a chunk in flight before the staging
// starts). Operands are swapped against w16_mfma_kernel — A = tokens, B = weight rows — so a
// lane's output column is its own weight row and the block scale d_w is a per-lane scalar. The
// KS slices' partial tiles meet through the workspace as in mmq_kernel (KS > 1): agent-scope
// stores, a per-tile counter, the last slice sums the partials in slice order and re-arms it.
// Weight k-slot q of a block: elements 8q..8q+7 = nibble plane q>>1 of qs[8(q&1)..] (Q4_0) or
// qs[8q..] (Q8_0); the activation fragments use the same element order.
template <int F> __device__ __forceinline__ u32x4_t w16_wfrag(uint32_t x, uint32_t y, int sh) {
    // bytes of x, y (nibbles at shift sh for Q4_0, sign-flipped bytes for Q8_0) -> exact bf16 of
    // q - 8 (Q4_0) or q (Q8_0): unsigned byte -> f32 (v_cvt_f32_ubyte*), minus the offset
    uint32_t u0, u1;
    float off;
    if constexpr (F == FMT_Q8_0) { u0 = x ^ 0x80808080u; u1 = y ^ 0x80808080u; off = -128.0f; }
    else { u0 = (x >> sh) & 0x0F0F0F0Fu; u1 = (y >> sh) & 0x0F0F0F0Fu; off = -8.0f; }
    const f32x2 o = {off, off};
    f32x2 v[4];
    v[0] = f32x2{(float)(u0 & 0xFFu), (float)((u0 >> 8) & 0xFFu)} + o;
    v[1] = f32x2{(float)((u0 >> 16) & 0xFFu), (float)(u0 >> 24)} + o;
    v[2] = f32x2{(float)(u1 & 0xFFu), (float)((u1 >> 8) & 0xFFu)} + o;
    v[3] = f32x2{(float)((u1 >> 16) & 0xFFu), (float)(u1 >> 24)} + o;
    u32x4_t r;
#pragma unroll
    for (int p = 0; p < 4; ++p) r[p] = hi16_pack(__float_as_uint(v[p].x), __float_as_uint(v[p].y));
    return r;
}

// ABL (tuning probe only; the product uses 0): 1 = each slice stores its partial tile and exits
// (no counter, no reduction: timing of the slice work alone).
template <int F, int RT, int TT, int KB, int ABL = 0, int NP = 3>
__global__ __launch_bounds__(RT * 64) void w16_sk_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B,
                                                         float* __restrict__ C, int M, int N, int K, long ldc_m,
                                                         long ldc_n, int kbs, float* __restrict__ part,
                                                         unsigned* __restrict__ cnt) {
    using T = wfmt<F>;
    static_assert(F == FMT_Q4_0 || F == FMT_Q8_0, "Q4_0 / Q8_0 weights");
    static_assert(KB % 4 == 0 && (TT * KB) % RT == 0, "whole block groups, whole staging rounds");
    constexpr int FR = 1024;             // bytes per fragment image: 64 lanes x 16 B
    constexpr int SJ = TT * KB / RT;     // staging items per thread per chunk
    constexpr int GB = TT >= 4 ? 2 : 4;  // blocks per compute group (operand registers)
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ int s_last;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, r16 = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * 16 * RT, m0 = blockIdx.y * 16 * TT;
    const int nb = K / QK;
    const long RB = (long)nb * T::BB;
    const int n = n0 + 16 * wave + r16;  // this lane's weight row (its output column)
    const uint8_t* wrow = B + (long)min(n, N - 1) * RB;
    const int qoff = T::QS + (T::Q8 ? 8 * q : 8 * (q & 1));  // its 8 bytes in a block (even: +2 mod 4)
    const int sh = T::Q8 ? 0 : 4 * (q >> 1);

    f32x4_t acc[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int c0 = 0; c0 < kbs; c0 += KB) {
        const int kb0 = blockIdx.z * kbs + c0;  // even (KB even, kbs a multiple of KB)
        // 1) the chunk's weight bytes in flight: rows are 4-B aligned (nb even), a block's 8 bytes
        //    start 2 bytes into a dword in even blocks (3 dwords) and on a dword in odd ones
        //    Q4_0: a block pair is 36 contiguous bytes (9 dwords, 4-B aligned) — 3 loads per pair
        //    (x4, x4, x1) instead of 4 per block; the lane's 8 bytes and d of each block are picked
        //    from them at compute time (PW). Q8_0: 4 loads per block.
        constexpr bool PW = F == FMT_Q4_0;
        uint32_t wx[KB], wy[KB], wz[KB], wd[KB];
        u32x4_t pa[PW ? KB / 2 : 1], pb[PW ? KB / 2 : 1];
        uint32_t pc[PW ? KB / 2 : 1];
        if constexpr (PW) {
#pragma unroll
            for (int pr = 0; pr < KB / 2; ++pr) {
                const uint32_t* p = reinterpret_cast<const uint32_t*>(wrow + (long)(kb0 + 2 * pr) * T::BB);
                pa[pr] = *reinterpret_cast<const u32x4a4_t*>(p);
                pb[pr] = *reinterpret_cast<const u32x4a4_t*>(p + 4);
                pc[pr] = p[8];
            }
        } else {
#pragma unroll
            for (int b = 0; b < KB; ++b) {
                const uint8_t* blk = wrow + (long)(kb0 + b) * T::BB;
                const uint32_t* p = reinterpret_cast<const uint32_t*>(blk + ((qoff + (b & 1) * 2) & ~3) - (b & 1) * 2);
                wx[b] = p[0];
                wy[b] = p[1];
                wz[b] = (b & 1) ? 0u : p[2];
                wd[b] = *reinterpret_cast<const uint16_t*>(blk);
            }
        }
        // 2) activation fragments: token 16 t + (lane & 15), elements 8 (lane >> 4) .. + 8 of block b
        float4 x[SJ][2];
#pragma unroll
        for (int j = 0; j < SJ; ++j) {
            const int it = threadIdx.x + j * RT * 64, ln = it & 63, tb = it >> 6;
            const int t = tb % TT, b = tb / TT;
            const int m = min(m0 + 16 * t + (ln & 15), M - 1);
            const float4* p = reinterpret_cast<const float4*>(A + (long)m * K + (long)(kb0 + b) * QK + 8 * (ln >> 4));
            x[j][0] = p[0];
            x[j][1] = p[1];
        }
#pragma unroll
        for (int j = 0; j < SJ; ++j) {
            const int it = threadIdx.x + j * RT * 64;
            u32x4_t h, mi, lo;
            if constexpr (NP == 2) w16_afrag2(x[j][0], x[j][1], h, mi);
            else w16_afrag(x[j][0], x[j][1], h, mi, lo);
            u32x4_t* dst = reinterpret_cast<u32x4_t*>(lds + (size_t)(it >> 6) * NP * FR) + (it & 63);
            dst[0] = h;
            dst[64] = mi;
            if constexpr (NP == 3) dst[128] = lo;
        }
        __syncthreads();
        // 3) GB blocks at a time: operand reads + weight decode, 3 GB TT MFMAs, then the d_w epilogue
        //    (MFMA results read behind an explicit wait, as in mmq_kernel)
#pragma unroll
        for (int g = 0; g < KB; g += GB) {
            u32x4_t wf[GB], af[GB][TT][NP];
            float dw[GB];
            f32x4_t c[GB][TT];
#pragma unroll
            for (int bb = 0; bb < GB; ++bb) {
                const int b = g + bb;
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const u32x4_t* fa = reinterpret_cast<const u32x4_t*>(lds + (size_t)(b * TT + t) * NP * FR) + lane;
#pragma unroll
                    for (int pl = 0; pl < NP; ++pl) af[bb][t][pl] = fa[64 * pl];
                }
                uint32_t xl, yl, wdb;
                if constexpr (PW) {
                    // pair dwords d0..d8; even block: d = d0.lo, bytes 2+8 q1 .. ; odd: d = d4.hi,
                    // bytes 20+8 q1 .. (q1 = q & 1)
                    const u32x4_t& A4 = pa[b >> 1];
                    const u32x4_t& B4 = pb[b >> 1];
                    const bool q1 = q & 1;
                    if ((b & 1) == 0) {
                        xl = q1 ? __builtin_amdgcn_alignbyte(A4[3], A4[2], 2) : __builtin_amdgcn_alignbyte(A4[1], A4[0], 2);
                        yl = q1 ? __builtin_amdgcn_alignbyte(B4[0], A4[3], 2) : __builtin_amdgcn_alignbyte(A4[2], A4[1], 2);
                        wdb = A4[0] & 0xFFFFu;
                    } else {
                        xl = q1 ? B4[3] : B4[1];
                        yl = q1 ? pc[b >> 1] : B4[2];
                        wdb = B4[0] >> 16;
                    }
                } else {
                    xl = (b & 1) ? wx[b] : __builtin_amdgcn_alignbyte(wy[b], wx[b], 2);
                    yl = (b & 1) ? wy[b] : __builtin_amdgcn_alignbyte(wz[b], wy[b], 2);
                    wdb = wd[b];
                }
                wf[bb] = w16_wfrag<F>(xl, yl, sh);
                dw[bb] = h2f(wdb);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int bb = 0; bb < GB; ++bb)
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const bf16x8_t wb = __builtin_bit_cast(bf16x8_t, wf[bb]);
                    f32x4_t r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[bb][t][0]), wb,
                                                                        f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                    if constexpr (NP == 3)
                        r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[bb][t][1]), wb, r, 0, 0, 0);
                    c[bb][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, af[bb][t][NP - 1]), wb, r, 0, 0, 0);
                }
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int bb = 0; bb < GB; ++bb)
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[t][e] = __builtin_fmaf(dw[bb], c[bb][t][e], acc[t][e]);
        }
        __syncthreads();  // every wave done with the fragments before the next chunk's staging
    }

    // lane: column n, rows (tokens) m0 + 16 t + 4 q + e
    auto store = [&](int t, int e, float v) {
        const int m = m0 + 16 * t + 4 * q + e;
        if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
    };
    if (gridDim.z == 1) {
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) store(t, e, acc[t][e]);
        return;
    }
    constexpr int TS = RT * TT * 4 * 64;  // floats per partial tile
    const int KS = gridDim.z;
    const long tile = (long)blockIdx.y * gridDim.x + blockIdx.x;
    float* pt = part + tile * KS * TS;
    auto pidx = [&](int t, int e) { return ((wave * TT + t) * 4 + e) * 64 + lane; };
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e)
            __hip_atomic_store(pt + blockIdx.z * TS + pidx(t, e), acc[t][e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (ABL == 1) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)KS - 1;
    __syncthreads();
    if (!s_last) return;
    // slice-order sum; each round's loads are all issued before its first add (atomic loads keep
    // program order, so a load-add chain would wait out one memory latency per slice)
    float v[TT][4];
    for (int s0 = 0; s0 < KS; s0 += 4) {
        float x[4][TT][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    x[j][t][e] = __hip_atomic_load(pt + min(s0 + j, KS - 1) * TS + pidx(t, e), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (s0 + j == 0) v[t][e] = x[j][t][e];
                    else if (s0 + j < KS) v[t][e] += x[j][t][e];
                }
    }
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) store(t, e, v[t][e]);
    if (threadIdx.x == 0) __hip_atomic_store(cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------
// W4A16 prefill, round-2 design (Q4_0, 8 < M <= 64, K % 256 == 0; w16s_kernel).
//
// w16_sk_kernel above loads every 8-block chunk into registers, splits it, writes it to LDS and only
// then computes it (profiles/r01_tuning/w16_sk_probe.txt: 14.3 us of slice work alone at M = 32).
// Here a workgroup (4 waves) owns 128 weight rows x 16 tokens x a K slice of ns 4-block stages
// streamed by LDS-DMA (global_load_lds, no VGPR staging) through a ring of R stage slots: per stage
// a 128 x 80-B weight image (each row's 72-B stage segment in a 16-B aligned window, as
// qg_mmq_kernel.hpp's P16 form) and a 16-token x 528-B image of the raw fp32 activations (512 B + a
// 16-B pad piece). Per stage: each wave waits for its own DMA (counted vmcnt), a barrier; the
// workgroup splits the stage's activations ONCE (wave w takes block w) into hi / mid / lo bf16
// operand planes (a = hi + mid + lo exactly, truncated parts) in LDS; a barrier; then every wave
// (32 rows = two 16-row tiles, all 16 tokens) computes the stage:
//   * k-slot q of a block = elements 4q..4q+3 and 16+4q..16+4q+3 (the W4A8 MMQ order), so a lane's
//     weights are ONE qs dword (low / high nibbles) -> 8 exact bf16 of q - 8 (v_cvt_f32_ubyteN,
//     -8, pack); its activation planes are three ds_read_b128;
//   * v_mfma_f32_16x16x32_bf16 with A = tokens, B = weight rows: the three planes chain into the
//     block's exact-product dot, then acc += d_w * dot (d_w a per-lane scalar: the lane's column is
//     its weight row).
// The VALU is the budget (a wave64 VALU op occupies its SIMD 4 cycles): sharing the split and the
// one-dword weight fragments took the stage from ~480 to ~200 VALU per wave (w16s_probe.txt).
// The K slices of a tile meet through the workspace: 16-B write-through (sc1) partial stores, a
// per-tile agent-scope counter, and the last slice to arrive sums the partials in slice order
// (deterministic) with sc1 loads and re-arms the counter (MI355X_MICROARCH.md hand-off table, row 1).
// TT: 16-token tiles per workgroup (1: 16 tokens; 2: 32 tokens, each weight fragment decoded once
// for both token tiles).
#ifndef QG_W16S_U128
#define QG_W16S_U128 0  // Q4_0 weight fragments as bf16 128 + q (w16s_wfrag_u128): measured M=16 +0.06,
                        // M=32 -0.29, M=64 +0.11 us (profiles/r02_tuning/ab_u128.txt) — the stage is not
                        // VALU-bound once the split is shared; off (exact q - 8 products kept)
#endif

template <int TT, int F = FMT_Q4_0, int NP = 3> struct w16s_geom {
    static constexpr int ROWS = 128;              // weight rows per workgroup (4 waves x 2 tiles of 16)
    static constexpr int TOK = 16 * TT;           // tokens per workgroup
    static constexpr int BB = wfmt<F>::BB;        // 18 (Q4_0) or 34 (Q8_0): 4 blocks = 8 mod 16 bytes
    static constexpr int RSB = 4 * BB;            // weight bytes per row per stage (4 blocks)
    static constexpr int RIMG = RSB + 8;          // 16-B aligned row window (80 / 144 B)
    static constexpr int PPR = RIMG / 16;         // 16-B pieces per row window
    static constexpr int WP = ROWS * PPR;         // weight pieces per stage (640 / 1152)
    static constexpr int ATS = 33;                // pieces per token image (32 data + 1 pad)
    static constexpr int AP = TOK * ATS;          // activation pieces per stage
    static constexpr int NI = ((WP + AP + 63) / 64 + 3) / 4 * 4;  // DMA instructions per stage (whole per wave)
    static constexpr int NIW = NI / 4;            // per wave
    static constexpr int SBYTES = NI * 1024;      // LDS bytes per stage
    static constexpr int AOFF = WP * 16;          // activation image offset in a stage
    static constexpr int PT = 4 * 2 * TT * 64 * 4;  // floats per partial tile (4 waves x 2 x TT tiles x 64 lanes x 4)
    static constexpr int PLB = NP * 4 * TT * 1024;  // activation planes of one stage ([plane][block][tt][lane] x 16 B)
    static_assert(WP + AP <= NI * 64, "stage pieces fit the DMA instructions");
};

__device__ __forceinline__ void w16_glds16(const uint8_t* g, uint8_t* l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
// s_waitcnt vmcnt(k * NIW): this wave's DMA of the oldest stage in flight landed, k later ones may fly
template <int NIW> __device__ __forceinline__ void w16s_wait(int k) {
    switch (k) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIW) : "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NIW) : "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NIW) : "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NIW) : "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * NIW) : "memory"); break;
        case 6: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * NIW) : "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(7 * NIW) : "memory"); break;
    }
}

// 16-B write-through store / L2-served load (the hand-off's sc1 accesses)
__device__ __forceinline__ void st_x4_sc1(float* p, f32x4_t v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ f32x4_t ld_x4_sc1(const float* p) {
    f32x4_t v;
    asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// byte N of x as f32 (v_cvt_f32_ubyteN; written out so the compiler cannot fold a mask into a bfe)
template <int N> __device__ __forceinline__ float cvt_ubyte(uint32_t x) {
    float r;
    if constexpr (N == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(r) : "v"(x));
    else if constexpr (N == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(r) : "v"(x));
    else if constexpr (N == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(r) : "v"(x));
    else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// k-slot q of a block (the W4A8 MMQ order, qg_mmq_kernel.hpp): elements 4q..4q+3 and 16+4q..16+4q+3,
// i.e. the low and high nibbles of qs dword q. One Q4_0 qs dword -> the 8 exact bf16 of q - 8.
__device__ __forceinline__ u32x4_t w16s_wfrag(uint32_t v) {
    const uint32_t lo = v & 0x0F0F0F0Fu, hi = (v >> 4) & 0x0F0F0F0Fu;
    const f32x2 o = {-8.0f, -8.0f};
    const f32x2 v0 = f32x2{cvt_ubyte<0>(lo), cvt_ubyte<1>(lo)} + o;
    const f32x2 v1 = f32x2{cvt_ubyte<2>(lo), cvt_ubyte<3>(lo)} + o;
    const f32x2 v2 = f32x2{cvt_ubyte<0>(hi), cvt_ubyte<1>(hi)} + o;
    const f32x2 v3 = f32x2{cvt_ubyte<2>(hi), cvt_ubyte<3>(hi)} + o;
    return u32x4_t{hi16_pack(__float_as_uint(v0.x), __float_as_uint(v0.y)), hi16_pack(__float_as_uint(v1.x), __float_as_uint(v1.y)),
                   hi16_pack(__float_as_uint(v2.x), __float_as_uint(v2.y)), hi16_pack(__float_as_uint(v3.x), __float_as_uint(v3.y))};
}

// The same k-slot as 8 exact bf16 of 128 + q (QG_W16S_U128): a nibble q under a 0x43 high byte is
// the bf16 0x430q = 128 + q, so one v_perm_b32 builds two elements (7 VALU per dword instead of 19);
// the stage subtracts 136 * (the block's activation dot with a constant-136 fragment) — the same
// MFMA chain on the same activation planes, so a row of zero weights (q = 8) cancels exactly.
__device__ __forceinline__ u32x4_t w16s_wfrag_u128(uint32_t v) {
    const uint32_t lo = v & 0x0F0F0F0Fu, hi = (v >> 4) & 0x0F0F0F0Fu, c = 0x43434343u;
    return u32x4_t{__builtin_amdgcn_perm(c, lo, 0x04010400u), __builtin_amdgcn_perm(c, lo, 0x04030402u),
                   __builtin_amdgcn_perm(c, hi, 0x04010400u), __builtin_amdgcn_perm(c, hi, 0x04030402u)};
}

// Q8_0: k-slot q = signed qs bytes 4q..4q+3 (dword v0) and 16+4q..16+4q+3 (v1) -> 8 exact bf16.
__device__ __forceinline__ u32x4_t w16s_wfrag_q8(uint32_t v0, uint32_t v1) {
    const uint32_t a = v0 ^ 0x80808080u, b = v1 ^ 0x80808080u;  // q + 128, unsigned
    const f32x2 o = {-128.0f, -128.0f};
    const f32x2 x0 = f32x2{cvt_ubyte<0>(a), cvt_ubyte<1>(a)} + o;
    const f32x2 x1 = f32x2{cvt_ubyte<2>(a), cvt_ubyte<3>(a)} + o;
    const f32x2 x2 = f32x2{cvt_ubyte<0>(b), cvt_ubyte<1>(b)} + o;
    const f32x2 x3 = f32x2{cvt_ubyte<2>(b), cvt_ubyte<3>(b)} + o;
    return u32x4_t{hi16_pack(__float_as_uint(x0.x), __float_as_uint(x0.y)), hi16_pack(__float_as_uint(x1.x), __float_as_uint(x1.y)),
                   hi16_pack(__float_as_uint(x2.x), __float_as_uint(x2.y)), hi16_pack(__float_as_uint(x3.x), __float_as_uint(x3.y))};
}

// ds_write_b128 the compiler does not see: an LDS store it sees makes it wait for every LDS-DMA in
// flight (vmcnt(0)), which would drain the stage ring (qg_mmq_kernel.hpp). Ordered by "memory"
// clobbers; completion waited for explicitly (lgkmcnt) before the barrier that publishes it.
__device__ __forceinline__ void ds_write_x4_asm(uint8_t* p, u32x4_t v) {
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)p;
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// The activation planes of one stage, split once per workgroup: wave w takes block w of the stage
// (for every token tile); lane (r16, q) reads its token's 8 fp32 of k-slot q (elements 4q.. and
// 16+4q.., two 16-B pieces of the raw image) and writes a = hi + mid + lo (truncated bf16 parts,
// exact) as three 16-B operand fragments, planes [plane][block][tt][lane] (1 KiB each).
template <int TT, int F, int NP>
__device__ __forceinline__ void w16s_split(const uint8_t* sb, uint8_t* planes, int wave, int lane) {
    using G = w16s_geom<TT, F, NP>;
    const int r16 = lane & 15, q = lane >> 4;
#pragma unroll
    for (int t = 0; t < TT; ++t) {
        const uint8_t* ar = sb + G::AOFF + (16 * t + r16) * (G::ATS * 16) + 128 * wave;
        const f32x4_t x0 = *reinterpret_cast<const f32x4_t*>(ar + 16 * q);
        const f32x4_t x1 = *reinterpret_cast<const f32x4_t*>(ar + 64 + 16 * q);
        const float a[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        uint8_t* d = planes + (size_t)(wave * TT + t) * 1024 + 16 * lane;
        if constexpr (NP == 2) {
            // a = hi + mid + r with hi = RNE_bf16(a), mid = RNE_bf16(a - hi) (a - hi exact in f32):
            // |r| <= 2^-16 |a| (v_cvt_pk_bf16_f32, two elements per op)
            u32x4_t ph, pm;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t h2 = bf16x2_rne_clamped(a[2 * k], a[2 * k + 1]);
                const f32x2 hf = {__uint_as_float(h2 << 16), __uint_as_float(h2 & 0xFFFF0000u)};
                const f32x2 r = f32x2{a[2 * k], a[2 * k + 1]} - hf;  // exact
                ph[k] = h2;
                pm[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2_t));
            }
            ds_write_x4_asm(d, ph);
            ds_write_x4_asm(d + 4 * TT * 1024, pm);
            continue;
        }
        uint32_t r1[8], r2[8];
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            const f32x2 x = {a[j], a[j + 1]};
            const f32x2 h = {__uint_as_float(__float_as_uint(bf16_clamp(a[j])) & 0xFFFF0000u),
                             __uint_as_float(__float_as_uint(bf16_clamp(a[j + 1])) & 0xFFFF0000u)};
            const f32x2 m1 = x - h;  // exact
            const f32x2 mh = {__uint_as_float(__float_as_uint(bf16_clamp(m1.x)) & 0xFFFF0000u),
                              __uint_as_float(__float_as_uint(bf16_clamp(m1.y)) & 0xFFFF0000u)};
            const f32x2 l2 = m1 - mh;  // exact, <= 8 significant bits
            r1[j] = __float_as_uint(m1.x); r1[j + 1] = __float_as_uint(m1.y);
            r2[j] = __float_as_uint(l2.x); r2[j + 1] = __float_as_uint(l2.y);
        }
        u32x4_t ph, pm, pl;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ph[k] = hi16_pack(__float_as_uint(a[2 * k]), __float_as_uint(a[2 * k + 1]));
            pm[k] = hi16_pack(r1[2 * k], r1[2 * k + 1]);
            pl[k] = hi16_pack(r2[2 * k], r2[2 * k + 1]);
        }
        ds_write_x4_asm(d, ph);
        ds_write_x4_asm(d + 4 * TT * 1024, pm);
        ds_write_x4_asm(d + 8 * TT * 1024, pl);
    }
}

// One 4-block stage of a wave (SH: the data's byte offset in the row windows, 0 on even stages, 8
// on odd ones). acc[i][t][e]: token 16 t + 4q + e, weight row 32 wave + 16 i + r16.
template <int TT, int F, int SH, int NP>
__device__ __forceinline__ void w16s_stage(const uint8_t* sb, const uint8_t* planes, int wave, int lane,
                                           f32x4_t (&acc)[2][TT]) {
    using G = w16s_geom<TT, F, NP>;
    constexpr bool U128 = QG_W16S_U128 && F == FMT_Q4_0;
    const int r16 = lane & 15, q = lane >> 4;
    u32x4_t ap[NP][4][TT];
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int t = 0; t < TT; ++t)
                ap[pl][b][t] = *reinterpret_cast<const u32x4_t*>(planes + ((pl * 4 + b) * TT + t) * 1024 + 16 * lane);
    u32x4_t wf[4][2];
    float dw[4][2];
    static_for<4>([&](auto BI) {
        constexpr int b = decltype(BI)::value;
        constexpr int X0 = SH + G::BB * b + 2;  // qs[0] of block b in the row window (+4q for k-slot q)
        constexpr int al = X0 % 4;
        constexpr int D = SH + G::BB * b;       // its f16 d
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint8_t* row = sb + (32 * wave + 16 * i + r16) * G::RIMG;
            const uint32_t* pw = reinterpret_cast<const uint32_t*>(row + (X0 & ~3) + 4 * q);
            uint32_t v = pw[0];
            if constexpr (al != 0) v = __builtin_amdgcn_alignbyte(pw[1], v, al);
            if constexpr (F == FMT_Q8_0) {
                uint32_t v1 = pw[4];  // qs[16 + 4q ..]
                if constexpr (al != 0) v1 = __builtin_amdgcn_alignbyte(pw[5], v1, al);
                wf[b][i] = w16s_wfrag_q8(v, v1);
            } else if constexpr (U128) {
                wf[b][i] = w16s_wfrag_u128(v);
            } else {
                wf[b][i] = w16s_wfrag(v);
            }
            dw[b][i] = h2f(*reinterpret_cast<const uint16_t*>(row + D));
        }
    });
    __builtin_amdgcn_sched_barrier(0);
    f32x4_t c[4][2][TT];
    f32x4_t z[4][TT];  // U128: 136 * the block's activation sum, per token (the same for every row)
    const u32x4_t k136 = {0x43084308u, 0x43084308u, 0x43084308u, 0x43084308u};  // bf16 136
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int t = 0; t < TT; ++t) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
                c[b][i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ap[0][b][t]),
                                                                     __builtin_bit_cast(bf16x8_t, wf[b][i]),
                                                                     f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            if constexpr (U128)
                z[b][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ap[0][b][t]),
                                                                  __builtin_bit_cast(bf16x8_t, k136),
                                                                  f32x4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
#pragma unroll
    for (int pl = 1; pl < NP; ++pl)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int t = 0; t < TT; ++t) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    c[b][i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ap[pl][b][t]),
                                                                         __builtin_bit_cast(bf16x8_t, wf[b][i]), c[b][i][t], 0, 0, 0);
                if constexpr (U128)
                    z[b][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ap[pl][b][t]),
                                                                      __builtin_bit_cast(bf16x8_t, k136), z[b][t], 0, 0, 0);
            }
    // MFMA results read by the VALU behind an explicit wait (8 states needed; qg_mmq_kernel.hpp)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if constexpr (U128) acc[i][t][e] = __builtin_fmaf(dw[b][i], c[b][i][t][e] - z[b][t][e], acc[i][t][e]);
                    else acc[i][t][e] = __builtin_fmaf(dw[b][i], c[b][i][t][e], acc[i][t][e]);
                }
}

// grid (ceil(N / 128), ceil(M / (16 TT)), ks); slice z = stages [z * ns, min(nst, (z + 1) * ns)) of
// the nst = K / 128 stages. ks == 1: direct stores, no workspace.
// R: LDS stage slots (a ring, R - 1 stages in flight ahead of the one being computed, a slot refilled
// right after the barrier that follows its last reader). After the raw activation planes of stage s
// have landed, the workgroup splits them once (w16s_split) into the planes buffer, a second barrier
// publishes it, and every wave computes the stage. ABL (tuning probes only): 1 = DMA and waits
// without split / compute, 2 = split + compute on whatever the LDS holds, no DMA, 3 = neither (the
// launch, barriers and the split-K hand-off alone).
template <int TT, int R, int ABL, int F = FMT_Q4_0, int NP = 3>
__global__ __launch_bounds__(256) void w16s_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B,
                                                   float* __restrict__ C, int M, int N, int K, long ldc_m, long ldc_n,
                                                   int ns, float* __restrict__ part, unsigned* __restrict__ cnt) {
    using G = w16s_geom<TT, F, NP>;
    static_assert(R >= 2 && R <= 7, "ring slots (w16s_wait counts up to 7 younger stages)");
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int n0 = blockIdx.x * G::ROWS, m0 = blockIdx.y * G::TOK;
    const int nst = K / 128;
    const int h0 = blockIdx.z * ns;
    const int nloc = min(ns, nst - h0);  // stages of this slice
    const long RB = (long)(K / QK) * G::BB;
    uint8_t* planes = lds + R * G::SBYTES;

    // this wave's DMA instructions i = wave + 4 k: piece p = 64 i + lane (clamped into the padding)
    const uint8_t* src[G::NIW];
    bool isw[G::NIW];
#pragma unroll
    for (int k = 0; k < G::NIW; ++k) {
        const int p = min(64 * (wave + 4 * k) + lane, G::WP + G::AP - 1);
        isw[k] = p < G::WP;
        if (isw[k]) {
            const int row = p / G::PPR, j = p - (p / G::PPR) * G::PPR;
            src[k] = B + (long)min(n0 + row, N - 1) * RB + 16 * j;
        } else {
            const int a = p - G::WP, tok = a / G::ATS, j = min(a - (a / G::ATS) * G::ATS, 31);
            src[k] = reinterpret_cast<const uint8_t*>(A + (long)min(m0 + tok, M - 1) * K) + 16 * j;
        }
    }
    auto slot = [&](int s) { return lds + (s % R) * G::SBYTES; };
    auto issue = [&](int s) {
        if constexpr (ABL >= 2) return;
        const int h = h0 + s;
        const long dw = (long)h * G::RSB - ((h & 1) ? 8 : 0), da = (long)h * 512;
        uint8_t* dst = slot(s) + 1024 * wave;
#pragma unroll
        for (int k = 0; k < G::NIW; ++k) w16_glds16(src[k] + (isw[k] ? dw : da), dst + 4096 * k);
    };
    constexpr int AHEAD = R - 1;  // stages in flight ahead of the one being computed
    for (int s = 0; s < min(nloc, AHEAD); ++s) issue(s);

    f32x4_t acc[2][TT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < TT; ++t) acc[i][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < nloc; ++s) {
        // stages issued so far: 0 .. min(nloc, s + AHEAD) - 1; wait for stage s
        if constexpr (ABL < 2) w16s_wait<G::NIW>(min(nloc, s + AHEAD) - 1 - s);
        __builtin_amdgcn_s_barrier();  // stage s landed everywhere; stage s - 1 and the planes are free
        asm volatile("" ::: "memory");
        if (s + AHEAD < nloc) issue(s + AHEAD);  // into the slot of stage s - 1
        if constexpr (ABL != 1 && ABL != 3) {
            w16s_split<TT, F, NP>(slot(s), planes, wave, lane);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();  // planes of stage s published
            asm volatile("" ::: "memory");
            if ((h0 + s) & 1) w16s_stage<TT, F, 8, NP>(slot(s), planes, wave, lane, acc);
            else w16s_stage<TT, F, 0, NP>(slot(s), planes, wave, lane, acc);
        }
    }

    // lane: weight rows n0 + 32 wave + 16 i + r16, tokens m0 + 16 t + 4 q + e
    const int r16 = lane & 15, q = lane >> 4;
    auto store = [&](int i, int t, const f32x4_t& v) {
        const int n = n0 + 32 * wave + 16 * i + r16;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int m = m0 + 16 * t + 4 * q + e;
            if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v[e];
        }
    };
    if (gridDim.z == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t) store(i, t, acc[i][t]);
        return;
    }
    const int KS = gridDim.z;
    const long tile = (long)blockIdx.y * gridDim.x + blockIdx.x;
    float* pt = part + tile * KS * G::PT;
    // 16 B per lane, whole lines per wave instruction
    auto pidx = [&](int i, int t) { return (((wave * 2 + i) * TT + t) * 64 + lane) * 4; };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < TT; ++t) st_x4_sc1(pt + blockIdx.z * G::PT + pidx(i, t), acc[i][t]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave's partial is at the coherence point
    __syncthreads();
    int* last = reinterpret_cast<int*>(lds);
    if (threadIdx.x == 0)
        *last = __hip_atomic_fetch_add(cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)KS - 1;
    __syncthreads();
    if (!*last) return;
    // slice-order sum, up to RS slices' loads in flight per round; this slice's own partial from registers
    constexpr int RS = TT == 1 ? 8 : 4;
    const int z = blockIdx.z;
    f32x4_t v[2][TT];
    for (int s0 = 0; s0 < KS; s0 += RS) {
        f32x4_t x[RS][2][TT];
#pragma unroll
        for (int j = 0; j < RS; ++j)
            if (s0 + j < KS && s0 + j != z) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t) x[j][i][t] = ld_x4_sc1(pt + (s0 + j) * G::PT + pidx(i, t));
            } else {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t) x[j][i][t] = acc[i][t];
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < RS; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t) asm volatile("" : "+v"(x[j][i][t]));  // uses stay behind the wait
#pragma unroll
        for (int j = 0; j < RS; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    if (s0 + j == 0) v[i][t] = x[j][i][t];
                    else if (s0 + j < KS) v[i][t] += x[j][i][t];
                }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < TT; ++t) store(i, t, v[i][t]);
    if (threadIdx.x == 0) __hip_atomic_store(cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Round-4 small-M prefill without split-K (the split-K hand-off of w16s_kernel
// — 8 KB partial slab per workgroup, counter, last-arriver sum — cost ~5 us and 9x the output in
// writes at M = 32). A workgroup owns 16 RT weight rows x 16 tokens and ALL of K; its W waves take
// the 2-block stages h = w, w + W, ... through wave-private LDS-DMA rings (NB slots, counted vmcnt,
// no barrier in the main loop, as qg_mmq_kernel.hpp): per stage the RT x 16-row weight windows (48 B
// each: the 36-B segment sits 0 / 4 / 8 / 12 B into a 16-B aligned window) and the 16 tokens' raw fp32
// activations (256 B per token + 32 B pad: the ds_read_b128 fragment reads of a lane group hit distinct
// banks). Each lane reads its token's k-slot (elements 4q.., 16+4q..) of a block as two ds_read_b128
// and splits it in registers (w16_afrag2 / w16_afrag: nothing written back to LDS, so no LDS store ever
// waits for the DMA), its weight row's qs dword q -> 8 exact bf16 of q - 8 (w16s_wfrag), NP chained
// v_mfma_f32_16x16x32_bf16 per (block, row tile), acc += d_w * dot. The W partial tiles are summed in
// fixed wave order through LDS at the end: deterministic, and the only global writes are the outputs.
#ifndef QG_W16D_NB
#define QG_W16D_NB 0  // (tuning knob) w16d_kernel stage slots per wave; 0: the most that fit, <= 3
#endif
// 32 bits at byte offset (compile-time OFF) of an LDS row, from aligned dword reads
template <int OFF> __device__ __forceinline__ uint32_t w16_lds32(const uint8_t* base) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(base + (OFF & ~3));
    if constexpr (OFF % 4 == 0) return p[0];
    else return __builtin_amdgcn_alignbyte(p[1], p[0], OFF % 4);
}

template <int F, int RT, int W, int NP, int SB_ = 2> struct w16d_geom {
    static constexpr int BB = wfmt<F>::BB;
    static constexpr int SB = SB_;                         // blocks per stage
    static constexpr int RSB = SB * BB;                    // 36 (Q4_0) / 68 (Q8_0) weight bytes per row
    // a stage's row segment starts (h * RSB) % 16 bytes into its 16-B aligned window: at most
    // SHMAX = 16 - gcd(RSB, 16); the window ends at the row's end for the last stage exactly when its
    // shift is SHMAX, i.e. RSB % 16 is 0 or gcd(RSB, 16) (36, 68, 72, 136 B: yes) — no read past a row
    static constexpr int G16 = (RSB & 15) == 0 ? 16 : (RSB & -RSB);
    static constexpr int SHMAX = 16 - G16;
    static constexpr int RIMG = RSB + SHMAX;
    static constexpr int RP = RIMG / 16;
    static constexpr int ROWS = 16 * RT;
    static constexpr int WP = ROWS * RP;                   // weight pieces per stage
    static constexpr int ATS = SB * 8 + 2;                 // pieces per token image (256 B + 32 B pad)
    static constexpr int AP = 16 * ATS;
    static constexpr int NI = (WP + AP + 63) / 64;         // DMA instructions per stage
    static constexpr int SBYTES = NI * 1024;
    static constexpr int AOFF = WP * 16;
    // stage slots per wave: QG_W16D_NB if set, else the most that fit, at most 3
    static constexpr int NBFIT = (160 * 1024) / (W * SBYTES);
    static constexpr int NB = QG_W16D_NB > 0 ? QG_W16D_NB : NBFIT >= 3 ? 3 : NBFIT >= 1 ? NBFIT : 1;
    static constexpr int NACC = RT * 4;
    static constexpr size_t LDS = (size_t)W * NB * SBYTES;
    static constexpr bool FITS = LDS <= 160 * 1024 && (size_t)W * NACC * 64 * 4 <= LDS;  // asserted by the kernel
    static_assert(NB >= 1 && NB <= 3 && (NB - 1) * NI <= 63, "vmcnt range");
    static_assert(RIMG % 16 == 0 && ((RSB & 15) == 0 || (RSB & 15) == G16), "windows end inside the row");
};

// ABL (tuning probes only; the product uses 0): 1 = DMA and waits without compute, 2 = compute without DMA.
template <int F, int RT, int W, int NP, int SB = 2, int ABL = 0>
__global__ __launch_bounds__(W * 64, 1) void w16d_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B,
                                                         float* __restrict__ C, int M, int N, int K, int ldc_m, int ldc_n) {
    using G = w16d_geom<F, RT, W, NP, SB>;
    using T = wfmt<F>;
    static_assert(G::FITS, "LDS per workgroup");
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15, q = lane >> 4;
    const int n0 = blockIdx.x * G::ROWS, m0 = blockIdx.y * 16;
    const int nst = K / (QK * G::SB);
    const long RB = (long)(K / QK) * G::BB;
    uint8_t* bufs = lds + wave * G::NB * G::SBYTES;

    // per-lane DMA offsets of a stage (32-bit, relative to stage 0 of the tile's first row / token; rows
    // / tokens past the edge re-read the last valid one, their results are dropped; pad pieces re-read
    // the image's last data piece). Instructions wholly inside the weight or the activation images
    // address from one wave-uniform 64-bit base (the saddr form: no per-lane 64-bit math per issue);
    // only the one instruction that straddles both selects per lane.
    const uint8_t* Bw = B + (long)n0 * RB;
    const uint8_t* Aw = reinterpret_cast<const uint8_t*>(A + (long)m0 * K);
    uint32_t off[G::NI];
    bool isw[G::NI];
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        const int p = min(64 * i + lane, G::WP + G::AP - 1);
        isw[i] = p < G::WP;
        if (isw[i]) {
            const int row = p / G::RP, j = p - row * G::RP;
            off[i] = (uint32_t)((long)(min(n0 + row, N - 1) - n0) * RB + 16 * j);
        } else {
            const int a = p - G::WP, tok = a / G::ATS, j = min(a - tok * G::ATS, G::SB * 8 - 1);
            off[i] = (uint32_t)((long)(min(m0 + tok, M - 1) - m0) * K * 4 + 16 * j);
        }
    }
    // buffer resources over the tile's weight rows / token rows (raw byte buffers: a load past
    // num_records returns zeros instead of faulting)
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
        (void*)Bw, (short)0, (int)min((long)(N - n0) * RB, 0x7FFFFFF0L), 0x00020000);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
        (void*)Aw, (short)0, (int)min((long)(M - m0) * K * 4, 0x7FFFFFF0L), 0x00020000);
    auto issue = [&](int h, uint8_t* buf) {
        if constexpr (ABL == 2) return;
        const int dw = h * G::RSB - ((h * G::RSB) & 15), da = h * (G::SB * QK * 4);
        static_for<G::NI>([&](auto I) {
            constexpr int i = decltype(I)::value;
            auto dst = (__attribute__((address_space(3))) void*)(buf + 1024 * i);
            if constexpr (64 * i + 63 < G::WP) __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, dst, 16, (int)off[i], dw, 0, 0);
            else if constexpr (64 * i >= G::WP) __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, dst, 16, (int)off[i], da, 0, 0);
            else w16_glds16((isw[i] ? Bw + dw : Aw + da) + off[i], buf + 1024 * i);
        });
    };

    f32x4_t acc[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int mine = wave < nst ? (nst - 1 - wave) / W + 1 : 0;
#pragma unroll
    for (int k = 0; k < G::NB; ++k)
        if (k < mine) issue(wave + k * W, bufs + k * G::SBYTES);
    for (int k = 0; k < mine; ++k) {
        const int h = wave + k * W;
        uint8_t* buf = bufs + (k % G::NB) * G::SBYTES;
        const int younger = ABL == 2 ? 0 : min(mine - 1 - k, G::NB - 1);
        if (younger <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::NI) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * G::NI) : "memory");
        // operands of the stage's SB blocks: every LDS read first, then the splits / decodes, MFMAs, epilogue
        const int sh = (h * G::RSB) & 15;
        f32x4_t xa[G::SB][2];
        uint32_t wv[G::SB][RT][2];
        uint32_t wd[G::SB][RT];
        static_for<G::SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            const uint8_t* ar = buf + G::AOFF + r16 * (G::ATS * 16) + b * (QK * 4) + 16 * q;
            xa[b][0] = *reinterpret_cast<const f32x4_t*>(ar);
            xa[b][1] = *reinterpret_cast<const f32x4_t*>(ar + 64);
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const uint8_t* row = buf + (16 * i + r16) * G::RIMG + sh;
                wv[b][i][0] = w16_lds32<b * G::BB + 2>(row + 4 * q);
                if constexpr (T::Q8) wv[b][i][1] = w16_lds32<b * G::BB + 2 + 16>(row + 4 * q);
                wd[b][i] = *reinterpret_cast<const uint16_t*>(row + b * G::BB);
            }
        });
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (ABL == 1) {
            if (k + G::NB < mine) issue(h + G::NB * W, buf);
            continue;
        }
        if (k + G::NB < mine) {  // every LDS read of this buffer has returned: refill it
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue(h + G::NB * W, buf);
        }
        // every split and decode first, then every MFMA (no VALU between the MFMAs: a VALU write into a
        // register an in-flight MFMA still reads as its accumulator is a hazard, tests/test_isa_hazards.py)
        u32x4_t ap[G::SB][NP], wf[G::SB][RT];
        static_for<G::SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            if constexpr (NP == 2) {
                w16_afrag2(__builtin_bit_cast(float4, xa[b][0]), __builtin_bit_cast(float4, xa[b][1]), ap[b][0], ap[b][1]);
            } else {
                u32x4_t lo;
                w16_afrag(__builtin_bit_cast(float4, xa[b][0]), __builtin_bit_cast(float4, xa[b][1]), ap[b][0], ap[b][1], lo);
                ap[b][NP - 1] = lo;
            }
#pragma unroll
            for (int i = 0; i < RT; ++i) wf[b][i] = T::Q8 ? w16s_wfrag_q8(wv[b][i][0], wv[b][i][1]) : w16s_wfrag(wv[b][i][0]);
        });
        __builtin_amdgcn_sched_barrier(0);
        f32x4_t c[G::SB][RT];
        static_for<G::SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int i = 0; i < RT; ++i)
                c[b][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ap[b][0]),
                                                                  __builtin_bit_cast(bf16x8_t, wf[b][i]), f32x4_t{0.f, 0.f, 0.f, 0.f},
                                                                  0, 0, 0);
        });
#pragma unroll
        for (int pl = 1; pl < NP; ++pl)
            static_for<G::SB>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
#pragma unroll
                for (int i = 0; i < RT; ++i)
                    c[b][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, ap[b][pl]),
                                                                      __builtin_bit_cast(bf16x8_t, wf[b][i]), c[b][i], 0, 0, 0);
            });
        // MFMA results read by the VALU behind an explicit wait (8 states needed; qg_mmq_kernel.hpp)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        static_for<G::SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const float d = h2f(wd[b][i]);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[i][e] = __builtin_fmaf(d, c[b][i][e], acc[i][e]);
            }
        });
    }

    // fixed-order sum of the W partial tiles (every DMA has landed: the last wait was vmcnt(0))
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[(wave * G::NACC + 4 * i + e) * 64 + lane] = acc[i][e];
    __syncthreads();
    for (int idx = threadIdx.x; idx < G::NACC * 64; idx += W * 64) {
        float v = red[idx];
#pragma unroll
        for (int ww = 1; ww < W; ++ww) v += red[ww * G::NACC * 64 + idx];
        const int x = idx >> 6, ln = idx & 63;
        const int e = x & 3, i = x >> 2;
        const int n = n0 + 16 * i + (ln & 15);      // lane's column: weight row r16
        const int m = m0 + 4 * (ln >> 4) + e;       // rows 4q + e: tokens
        if (n < N && m < M) C[(long)m * ldc_m + (long)n * ldc_n] = v;
    }
}

#ifndef QG_GEMV_SMALLK
#define QG_GEMV_SMALLK 1
#endif
#ifndef QG_W16_RPL
#define QG_W16_RPL 0  // weight rows per wave of the M = 1 W4A16 GEMV: 0 = by N (below), 1 = w16_gemv1_kernel
#endif
namespace {
constexpr int W16_MT = 8;
constexpr size_t W16_LDS_MAX = 160 * 1024;

template <int F, int BPL> size_t w16_lds(int mt, int K) { return (size_t)mt * (K / QK / BPL) * w16_geom<F, BPL>::REC_DW * 4; }

template <int F, int MT, int BPL, int LPR, int WGS, bool ONEU = false>
hipError_t w16_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    const int rows = g.M < MT ? g.M : MT;
    const size_t lds = w16_lds<F, BPL>(rows, g.K);
    const dim3 grid((g.N + RPB - 1) / RPB, (g.M + MT - 1) / MT);
    if constexpr (MT == 1) {
        if (g.M == 1 && g.ldc_n == 1) {
            auto k1 = w16_gemv1_kernel<F, BPL, LPR, WGS, ONEU>;
            if (lds > 64 * 1024) {
                hipError_t e = hipFuncSetAttribute((const void*)k1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(k1, dim3(grid.x), dim3(WGS), lds, st, (const float*)g.A, (const uint8_t*)g.B, g.N, g.K, g.C);
            return hipGetLastError();
        }
    }
    auto kfn = w16_gemv_kernel<F, MT, BPL, LPR, WGS, ONEU>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, grid, dim3(WGS), lds, st, (const float*)g.A, (const uint8_t*)g.B, (long)MT * g.K, g.M, g.N,
                       g.K, g.C, (long)MT * g.ldc_m, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}

template <int F, int MT> hipError_t w16_launch_mt(const GemmArgs& g, hipStream_t st) {
    const int nb = g.K / QK;
    // 2-block units, one row per wave, 1024-thread workgroups: half the per-wave work of the 4-block
    // shape (as the W4A8 GEMV, qg_gemv.hip)
    if (MT <= 4 && nb % 2 == 0 && nb / 2 >= 64 && w16_lds<F, 2>(g.M < MT ? g.M : MT, g.K) <= W16_LDS_MAX) {
        // K == 4096, Q4_0: one unit per lane (M=1 4.82 -> 4.61 us; Q8_0 measured no better)
        if constexpr (MT == 1 && F == FMT_Q4_0)
            if (nb / 2 <= 64) {
                // two weight rows per wave from N = 8192 on (profiles/r03_tuning/r03_ab_rpl.txt: N = 11008
                // 9.01 -> 7.73 us, N = 32000 21.3 -> 18.4; N = 4096 +1 %), bit-identical
                constexpr int RPL = QG_W16_RPL ? QG_W16_RPL : 2;
                if (RPL > 1 && (QG_W16_RPL || g.N >= 8192) && g.M == 1 && g.ldc_n == 1) {
                    constexpr int WG = 1024 / RPL, RPB = (WG / 64) * RPL;
                    const size_t lds = w16_lds<F, 2>(1, g.K);
                    hipLaunchKernelGGL((w16_gemv1r_kernel<F, WG, RPL>), dim3((g.N + RPB - 1) / RPB), dim3(WG), lds, st,
                                       (const float*)g.A, (const uint8_t*)g.B, g.N, g.K, g.C);
                    return hipGetLastError();
                }
                return w16_launch<F, 1, 2, 64, 1024, true>(g, st);
            }
        return w16_launch<F, MT, 2, 64, 1024>(g, st);
    }
    if (QG_GEMV_SMALLK && MT <= 4 && nb % 2 == 0 && nb / 2 >= 16 && w16_lds<F, 2>(g.M < MT ? g.M : MT, g.K) <= W16_LDS_MAX) {
        // K < 4096: 32 / 16 lanes per row, 16 rows per workgroup (as the W4A8 GEMV)
        if (nb / 2 >= 32) {
            if constexpr (MT == 1)
                if (nb / 2 == 32) return w16_launch<F, 1, 2, 32, 512, true>(g, st);
            return w16_launch<F, MT, 2, 32, 512>(g, st);
        }
        if constexpr (MT == 1)
            if (nb / 2 == 16) return w16_launch<F, 1, 2, 16, 256, true>(g, st);
        return w16_launch<F, MT, 2, 16, 256>(g, st);
    }
    if (nb % 4 == 0) {
        if (nb / 4 >= 32) return w16_launch<F, MT, 4, 32, 512>(g, st);
        return w16_launch<F, MT, 4, 4, 256>(g, st);
    }
    return w16_launch<F, MT, 2, 8, 256>(g, st);
}

// Rows per chunk: the next power of two >= M (at most 8), halved until the LDS records fit; 0 if
// the fast kernel does not apply (alignment, K not a multiple of 64).
template <int F> int w16_pick_mt(const GemmArgs& g) {
    const int nb = g.K / QK;
    const int bpl = nb % 4 == 0 ? 4 : 2;
    if (nb % bpl != 0) return 0;
    if (((uintptr_t)g.A & 15) != 0 || ((uintptr_t)g.B & 3) != 0) return 0;
    for (int mt = g.M <= 1 ? 1 : g.M <= 2 ? 2 : g.M <= 4 ? 4 : W16_MT; mt >= 1; mt /= 2) {
        const size_t lds = bpl == 4 ? w16_lds<F, 4>(mt, g.K) : w16_lds<F, 2>(mt, g.K);
        if (lds <= W16_LDS_MAX && (g.M + mt - 1) / mt <= 65535) return mt;
    }
    return 0;
}

template <int F, int RT, int TT, int W> hipError_t w16_mfma_launch(const GemmArgs& g, hipStream_t st) {
    const dim3 grid((g.N + 16 * RT - 1) / (16 * RT), (g.M + 16 * TT - 1) / (16 * TT));
    const size_t lds = (size_t)W * RT * TT * 4 * 64 * 4;
    hipLaunchKernelGGL((w16_mfma_kernel<F, RT, TT, W>), grid, dim3(W * 64), lds, st, (const float*)g.A,
                       (const uint8_t*)g.B, g.C, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}

// Split-K prefill plan: RT 16-row tiles (one per wave) x 16 TT tokens x ks slices of K, KB blocks
// per LDS chunk. ks: the fewest slices (a divisor of the chunk count) that give >= 256 workgroups.
struct w16_plan {
    int rt = 0, tt = 0, kb = 0, ks = 1;
    int ns = 0;  // > 0: the round-2 kernel (w16s_kernel) with ns stages per slice
    long gx = 0, gy = 0;
    size_t ws_bytes = 0;  // workspace for ks > 1: tile counters, then ks partial tiles per tile
};
// Workspace layout, the same for every shape: W16_CNT_BYTES of tile counters (split-K runs only
// while the grid has < 512 tiles), then the partial tiles. A fixed counter region keeps the
// counters zero across shapes: every launch re-arms its own counters, and no other shape's
// partial tiles ever overlap them (a shape-dependent offset let one shape's partials
// land in another shape's counters on a shared workspace).
constexpr size_t W16_CNT_BYTES = 4096;

w16_plan w16_make_plan(int M, int N, int K) {
    w16_plan p;
    const int nb = K / QK;
    if (M <= 8 || K % QK != 0) return p;
    // M <= 64: 64-row x 32-token tiles, 8-block chunks, K split until >= 512 workgroups (two per CU:
    // one's loads overlap the other's compute); tools/w16_sk_probe.hip, profiles/r01_tuning/
    // w16_sk_probe.txt: M=32 N=K=4096 16.7 us vs 18.8 for 128-row tiles, 16-block chunks, 256 WGs.
    // M > 64: 128-row (N >= 2048) or 64-row tiles x 64 tokens, >= 256 workgroups.
    int want = 256;
    if (M <= 64 && nb % 8 == 0) { p.tt = 2; p.kb = 8; p.rt = 4; want = 512; }
    else if (M > 64 && nb % 8 == 0) { p.tt = 4; p.kb = 8; p.rt = N >= 2048 ? 8 : 4; }
    else return p;
    p.gx = (N + 16 * p.rt - 1) / (16 * p.rt);
    p.gy = (M + 16 * p.tt - 1) / (16 * p.tt);
    const int chunks = nb / p.kb;
    if (p.gx * p.gy < want)
        for (int d = 2; d <= chunks && d <= 32; ++d) {
            if (chunks % d) continue;
            p.ks = d;
            if (p.gx * p.gy * d >= want) break;
        }
    static_assert(W16_CNT_BYTES / 4 >= 512, "counter region holds every split-K grid");
    if (p.ks > 1) p.ws_bytes = W16_CNT_BYTES + (size_t)p.gx * p.gy * p.ks * p.rt * p.tt * 4 * 64 * 4;
    return p;
}

// Round-2 plan (w16s_kernel; Q4_0, 8 < M <= 64, K % 256 == 0): 128-row x 16-token tiles, K split
// into ks slices of ns 4-block stages (see below for the count).
#ifndef QG_W16S
#define QG_W16S 1
#endif
#ifndef W16S_R
#define W16S_R 2  // LDS ring slots of w16s_kernel (2: one stage in flight ahead; 3-4 measured slower)
#endif
#ifndef QG_W16S_Q8
#define QG_W16S_Q8 1  // the round-2 prefill for W8A16 (Q8_0 weights) too
#endif
#ifndef W16S_TT2
#define W16S_TT2 2  // 32-token tiles: 0 never, 1 for every M > 16, 2 by the rule in w16s_make_plan
#endif
#ifndef W16S_MINWG
#define W16S_MINWG 512  // split K until the grid has this many workgroups (tuning knob)
#endif
#ifndef W16S_MINST
#define W16S_MINST 4  // ... keeping at least this many 4-block stages per slice (tuning knob)
#endif
#ifndef QG_W16S_NP2_MINK
#define QG_W16S_NP2_MINK 1024  // K from which w16s_kernel splits activations into TWO bf16 parts (0: never)
#endif
// Activation parts of the round-2 prefill. Three truncated parts represent every fp32 activation
// exactly; two round-to-nearest parts leave |r| <= 2^-16 |a| per element, i.e. at most
// 2^-16 sum_k |a_k w_k| = 256 u sum_k |a_k w_k| (u = 2^-24) on an output, against the fp32 K-term
// summation bound 2 (K + 2) u sum_k |a_k w_k| the parity tests hold the kernel to (oracle.w16_tol):
// from K = 1024 on the representation error stays below an eighth of that bound.
inline int w16s_parts(int K) { return QG_W16S_NP2_MINK > 0 && K >= QG_W16S_NP2_MINK ? 2 : 3; }
w16_plan w16s_make_plan(int M, int N, int K) {
    w16_plan p;
    if (!QG_W16S || M <= 8 || M > 64 || N < 1 || K % 256 != 0) return p;
    p.gx = (N + 127) / 128;
    // 32-token tiles decode each weight fragment once for two token tiles; they pay off only while the
    // grid keeps >= 64 tiles of 128 rows x 32 tokens with no idle token rows (profiles/r03_tuning/
    // r03_ab_w16_tt2.txt: M = 32 N = 11008 27.8 -> 23.6 us, M = 64 N = 4096 18.3 -> 17.9; slower at
    // N = 4096 M = 24 / 32 (12.7 -> 14.8: half the tiles) and M = 48 (idle rows))
    const bool tt2 = W16S_TT2 == 1 ? M > 16 : W16S_TT2 == 2 && M % 32 == 0 && p.gx * (M / 32) >= 64;
    p.tt = tt2 ? 2 : 1;
    p.gy = (M + 16 * p.tt - 1) / (16 * p.tt);
    const long tiles = p.gx * p.gy;
    const int nst = K / 128;
    // >= 512 workgroups (two per CU overlap each other's barriers and LDS latency) with >= 4 stages per
    // slice (tools/w16s_probe.hip, profiles/r02_tuning/w16s_probe.txt: M=32 N=K=4096 14.3 us at 8 x 4
    // stages vs 15.8 at 4 x 8, 16.8 for the round-1 kernel)
    int ks = (int)std::max<long>(1, std::min<long>(nst / W16S_MINST, (W16S_MINWG + tiles - 1) / tiles));
    p.ns = (nst + ks - 1) / ks;
    p.ks = (nst + p.ns - 1) / p.ns;
    if (p.ks > 1 && tiles > (long)(W16_CNT_BYTES / 4)) return w16_plan{};
    const size_t pt = p.tt == 2 ? w16s_geom<2>::PT : w16s_geom<1>::PT;
    if (p.ks > 1) p.ws_bytes = W16_CNT_BYTES + (size_t)tiles * p.ks * pt * 4;
    return p;
}

template <int F, int TT, int NP> hipError_t w16s_launch_tt(const GemmArgs& g, const w16_plan& p, void* ws, hipStream_t st) {
    using G = w16s_geom<TT, F, NP>;
    unsigned* cnt = (unsigned*)ws;
    float* part = ws ? (float*)((uint8_t*)ws + W16_CNT_BYTES) : nullptr;
    constexpr size_t lds = (size_t)W16S_R * G::SBYTES + G::PLB;
    static_assert(lds <= 160 * 1024, "LDS per workgroup");
    static std::atomic<unsigned long long> attr_done{0};
    {
        const hipError_t e = set_max_lds_once((const void*)w16s_kernel<TT, W16S_R, 0, F, NP>, (int)lds, attr_done);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((w16s_kernel<TT, W16S_R, 0, F, NP>), dim3(p.gx, p.gy, p.ks), dim3(256), lds, st, (const float*)g.A,
                       (const uint8_t*)g.B, g.C, g.M, g.N, g.K, g.ldc_m, g.ldc_n, p.ns, part, cnt);
    return hipGetLastError();
}
template <int F> hipError_t w16s_launch(const GemmArgs& g, const w16_plan& p, void* ws, hipStream_t st) {
    if (w16s_parts(g.K) == 2) return p.tt == 2 ? w16s_launch_tt<F, 2, 2>(g, p, ws, st) : w16s_launch_tt<F, 1, 2>(g, p, ws, st);
    return p.tt == 2 ? w16s_launch_tt<F, 2, 3>(g, p, ws, st) : w16s_launch_tt<F, 1, 3>(g, p, ws, st);
}

template <int F, int RT, int TT, int KB, int NP> hipError_t w16_sk_launch_np(const GemmArgs& g, const w16_plan& p, void* ws,
                                                                          hipStream_t st) {
    const int ks = ws ? p.ks : 1;
    unsigned* cnt = (unsigned*)ws;
    float* part = ws ? (float*)((uint8_t*)ws + W16_CNT_BYTES) : nullptr;
    constexpr size_t lds = (size_t)TT * KB * NP * 1024;
    auto kfn = w16_sk_kernel<F, RT, TT, KB, 0, NP>;
    if (lds > 64 * 1024) {
        static std::atomic<unsigned long long> attr_done{0};
        const hipError_t e = set_max_lds_once((const void*)kfn, (int)lds, attr_done);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, dim3(p.gx, p.gy, ks), dim3(RT * 64), lds, st, (const float*)g.A, (const uint8_t*)g.B, g.C,
                       g.M, g.N, g.K, g.ldc_m, g.ldc_n, g.K / QK / ks, part, cnt);
    return hipGetLastError();
}
template <int F, int RT, int TT, int KB> hipError_t w16_sk_launch(const GemmArgs& g, const w16_plan& p, void* ws, hipStream_t st) {
    if (w16s_parts(g.K) == 2) return w16_sk_launch_np<F, RT, TT, KB, 2>(g, p, ws, st);
    return w16_sk_launch_np<F, RT, TT, KB, 3>(g, p, ws, st);
}

#ifndef QG_W16D
#define QG_W16D 1  // the no-split-K small-M prefill (w16d_kernel) where w16d_ok holds
#endif
#ifndef QG_W16D_MAXK
#define QG_W16D_MAXK 8192  // beyond, the split-K kernel is faster (K = 14336: 30.4 vs 29.4 us, ab_w16d_v2.txt)
#endif
// 8 < M <= 32 tokens, K % 256 == 0 (16-B aligned weight rows), 16-B aligned operands, 32-bit strides.
// One dispatch round only (<= one workgroup per CU: device_cus(), 256 on a whole MI355X): with more, each
// CU runs several workgroups in turn
// (one fits at a time) and the split-K kernel is faster (M = 32, N = 11008: 29.6 vs 23.5 us,
// profiles/r04_tuning/ab_w16d_v1.txt).
inline bool w16d_ok(const GemmArgs& g) {
    if (!(QG_W16D && g.M > 8 && g.M <= 32 && g.N >= 1 && g.K % 256 == 0 && ((uintptr_t)g.A & 15) == 0 &&
          ((uintptr_t)g.B & 15) == 0 && g.ldc_m <= INT32_MAX && g.ldc_n <= INT32_MAX))
        return false;
    const long rows = (g.N + 15) / 16 * ((g.M + 15) / 16);  // 16-row tiles
    const long cus = device_cus();
    return (rows <= cus || (long)((g.N + 31) / 32) * ((g.M + 15) / 16) <= cus) && g.K <= QG_W16D_MAXK &&
           (long)g.M * g.K * 4 < 0x7FFFFFF0L && (long)g.N * (g.K / QK) * wfmt<FMT_Q8_0>::BB < 0x7FFFFFF0L;  // buffer ranges
}
#ifndef QG_W16D_W
// waves per workgroup (stage slots per wave: the most that fit): 16 waves with one slot each
// (profiles/r04_tuning/ab_waves_r4v.txt, W4A16 M = 32: 10.80 -> 10.15 us, M = 24 10.34 -> 9.52, M = 16
// 8.54 -> 8.40, K = 8192 18.47 -> 17.57 against 12 waves with two slots, which beat 8 waves with three:
// ab_w16d_waves.txt, 11.75 -> 10.78; that record's `wtype=8` row timed the W4A16 kernel, DESIGN.md §6, so
// the W8A16 (Q8_0) wave count is inherited from Q4_0, not separately tuned) — more waves per SIMD overlap one wave's DMA
// wait with another's VALU; the refill of a wave's slot is issued right after its LDS reads, before the
// stage's compute
#define QG_W16D_W 16
#endif
#ifndef QG_W16D_SB
#define QG_W16D_SB 2  // blocks per stage (tuning knob; Q4_0 from K = QG_W16D_SB4_MINK takes 4, w16d_launch)
#endif
#ifndef QG_W16D_ABL
#define QG_W16D_ABL 0  // (tuning probes only) w16d_kernel ablation
#endif
template <int F, int RT, int NP, int SB = QG_W16D_SB, int WREQ = QG_W16D_W>
hipError_t w16d_launch_np(const GemmArgs& g, hipStream_t st) {
    constexpr int W = w16d_geom<F, RT, WREQ, NP, SB>::FITS         ? WREQ
                      : w16d_geom<F, RT, WREQ - 1, NP, SB>::FITS ? WREQ - 1
                      : w16d_geom<F, RT, WREQ - 2, NP, SB>::FITS ? WREQ - 2
                                                                 : 8;
    using G = w16d_geom<F, RT, W, NP, SB>;
    auto k = w16d_kernel<F, RT, W, NP, SB, QG_W16D_ABL>;
    static std::atomic<unsigned long long> attr_done{0};
    const hipError_t e = set_max_lds_once((const void*)k, (int)G::LDS, attr_done);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3((g.N + G::ROWS - 1) / G::ROWS, (g.M + 15) / 16), dim3(W * 64), G::LDS, st, (const float*)g.A,
                       (const uint8_t*)g.B, g.C, g.M, g.N, g.K, (int)g.ldc_m, (int)g.ldc_n);
    return hipGetLastError();
}
// 16-row tiles while their grid fits one dispatch round (<= one workgroup per CU), else 32-row ones (w16d_ok)
inline bool w16d_rt2(const GemmArgs& g) { return (long)((g.N + 15) / 16) * ((g.M + 15) / 16) > device_cus(); }
// Q4_0 from K = 4096 (>= 32 four-block stages, so each of 12 waves takes two or three): 4-block stages
// with 12 waves (profiles/r04_tuning/ab_w16d_sb4*.txt: M = 32 10.12 -> 9.90 us, M = 16 8.38 -> 8.19,
// M = 12 8.20 -> 8.06, K = 8192 17.54 -> 17.25, M = 20 / 24 +0.8 / +1.3 %; K = 1024 +8 %: 8 stages for 12
// waves). The longer 72-B weight windows take fewer DMA requests per byte.
#ifndef QG_W16D_SB4_MINK
#define QG_W16D_SB4_MINK 4096
#endif
template <int F> hipError_t w16d_launch(const GemmArgs& g, hipStream_t st) {
    const bool rt2 = w16d_rt2(g);
    if constexpr (F == FMT_Q4_0 && QG_W16D_SB4_MINK > 0 && QG_W16D_SB == 2) {
        if (g.K >= QG_W16D_SB4_MINK) {
            if (w16s_parts(g.K) == 2) return rt2 ? w16d_launch_np<F, 2, 2, 4, 12>(g, st) : w16d_launch_np<F, 1, 2, 4, 12>(g, st);
            return rt2 ? w16d_launch_np<F, 2, 3, 4, 12>(g, st) : w16d_launch_np<F, 1, 3, 4, 12>(g, st);
        }
    }
    if (w16s_parts(g.K) == 2) return rt2 ? w16d_launch_np<F, 2, 2>(g, st) : w16d_launch_np<F, 1, 2>(g, st);
    return rt2 ? w16d_launch_np<F, 2, 3>(g, st) : w16d_launch_np<F, 1, 3>(g, st);
}

template <int F> hipError_t w16_dispatch(const GemmArgs& g, hipStream_t st) {
    if constexpr (F == FMT_Q4_0 || F == FMT_Q8_0)
        if (w16d_ok(g)) return w16d_launch<F>(g, st);
    if constexpr (F == FMT_Q4_0 || (F == FMT_Q8_0 && QG_W16S_Q8)) {
        // round-2 prefill: 16-B aligned activations and weights (rows are then 16-B multiples)
        if (((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 && (g.M + 15) / 16 <= 65535) {
            const w16_plan p = w16s_make_plan(g.M, g.N, g.K);
            if (p.ns) {
                // hold: the library buffer's lock stays taken until the kernel is enqueued, so another
                // host thread on this stream cannot grow (and free) it in between
                std::unique_lock<std::mutex> hold;
                void* ws = nullptr;
                if (p.ks > 1) {
                    if (g.ws) ws = g.ws_bytes >= p.ws_bytes && ((uintptr_t)g.ws & 255) == 0 ? g.ws : nullptr;
                    else ws = stream_workspace(st, p.ws_bytes, 0, &hold);
                }
                if (ws || p.ks == 1) return w16s_launch<F>(g, p, ws, st);
            }
        }
    }
    if (((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 3) == 0 && (g.M + 63) / 64 <= 65535) {
        const w16_plan p = w16_make_plan(g.M, g.N, g.K);
        if (p.rt) {
            // the caller's workspace (qg_gemm_w4a16_ws), else the library's one for this stream
            std::unique_lock<std::mutex> hold;
            void* ws = nullptr;
            if (p.ks > 1) {
                if (g.ws) ws = g.ws_bytes >= p.ws_bytes && ((uintptr_t)g.ws & 255) == 0 ? g.ws : nullptr;
                else ws = stream_workspace(st, p.ws_bytes, 0, &hold);
            }
            // without one, a grid this small would leave most CUs idle: the older kernel below
            if (ws || p.ks == 1 || p.gx * p.gy >= 128) {
                if (p.tt == 2) return w16_sk_launch<F, 4, 2, 8>(g, p, ws, st);
                return p.rt == 8 ? w16_sk_launch<F, 8, 4, 8>(g, p, ws, st) : w16_sk_launch<F, 4, 4, 8>(g, p, ws, st);
            }
        }
    }
    if (g.M > 8 && ((uintptr_t)g.A & 15) == 0 && (g.M + 31) / 32 <= 65535) {
        // one 16-row tile per workgroup while that leaves < 256 workgroups of 32 rows
        if ((long)((g.N + 31) / 32) * ((g.M + 31) / 32) < 256) return w16_mfma_launch<F, 1, 2, 16>(g, st);
        return w16_mfma_launch<F, 2, 2, 16>(g, st);
    }
    switch (w16_pick_mt<F>(g)) {
        case 1: return w16_launch_mt<F, 1>(g, st);
        case 2: return w16_launch_mt<F, 2>(g, st);
        case 4: return w16_launch_mt<F, 4>(g, st);
        case 8: return w16_launch_mt<F, 8>(g, st);
    }
    if (g.M > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(w16_generic_kernel<F>, dim3((g.N + 3) / 4, g.M), dim3(256), 0, st, (const float*)g.A,
                       (const uint8_t*)g.B, g.C, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}
}  // namespace

// one size for both weight types: the larger of the two plans' workspaces
size_t w16_workspace_bytes(int M, int N, int K) {
    return std::max(w16_make_plan(M, N, K).ws_bytes, w16s_make_plan(M, N, K).ws_bytes);
}

hipError_t launch_w16(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return w16_dispatch<FMT_Q4_0>(g, st);
        case FMT_Q8_0: return w16_dispatch<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
