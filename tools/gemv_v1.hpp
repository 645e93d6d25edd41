// gemv_v1.hpp — the round-1 product GEMV kernel (classic dot4 decode), kept as the A/B baseline of
// tools/gemv_probe.hip. Not part of the product.
// (the tuning sweep). Computes, for the reference's activation-major contract
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222):
//   C[m*ldc_m + n*ldc_n] = sum_b term(A[m][b], B[n][b]).
//
// Work decomposition:
//  * A lane owns "units" of BPL consecutive Q-blocks of one weight row (BPL*BB bytes, e.g. Q4_0
//    BPL=4 -> 72 B; the compiler issues them as 4 x dwordx4 + 1 x dwordx2). LPR lanes share a row
//    and stride over its units (the next unit in flight while the current one computes); 64/LPR
//    rows per wave, WGS/64 waves per workgroup.
//  * The workgroup stages the M Q8_1 rows once into LDS records (8 qs dwords, f32 d, f32 s, pad;
//    dword stride 12*BPL+4 per (m, unit) = 4 x odd, so the 16 lanes of a ds_read_b128 group hit
//    distinct bank slots). The activation loads are issued before the weight stream, so the
//    staging waits only on them.
//  * Blocks are decoded in registers with compile-time alignbyte/shift/mask (qg_common.hpp) and
//    dotted with v_dot4c_i32_i8: exact int32 sumi; the per-block epilogue is the reference's
//    operation order, no contraction -> block terms bit-identical to the CPU oracle.
//  * Per-lane partials (unit order, block order) are reduced across the row's LPR lanes with DPP
//    row ops (group_sum_last: no LDS round trips — the ds_bpermute chain it replaced was ~0.1 us of
//    a 4 us launch); the row's last lane stores. Deterministic.
//  * AIN != 0 (fused activation quantization): A is FP32 (AIN_F32, quantized as
//    quantize_row_q8_1_ref) or FP16 (AIN_F16_FUSED, as kernels/gemm/gemm_fused.cuh:76-143) [M][K];
//    each thread quantizes whole 32-element blocks straight into the LDS records
//    (qg_quant_block.hpp), so the records — and every output — are bit-identical to the two-step
//    quantize + GEMV path. The first block's loads are issued before the weight stream.
// Tuning record (probes, per-wave timelines, rejected designs): profiles/r01_tuning/README.md.
#pragma once
#include "qg_common.hpp"
#include "qg_kernels.hpp"
#include "qg_quant_block.hpp"

namespace qg {

template <int F, int BPL> struct gemv_v1_geom {
    static constexpr int BB = wfmt<F>::BB;
    static constexpr int UB = BPL * BB;          // unit bytes
    static constexpr int UDW = UB / 4;           // unit dwords (BB even, BPL even -> whole dwords)
    static constexpr int REC_DW = 12 * BPL + 4;  // LDS record dwords per (m, unit)
};

// ------------------------------------------------------------------------------------------------
// Load the 32 activation values of block g (AIN_F32: 128 B, AIN_F16_FUSED: 64 B; 16-B aligned).
template <int AIN> __device__ __forceinline__ void load_act_block_v1(const uint8_t* __restrict__ X, int g, float (&v)[32]) {
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

// NSTAGE: activation dwords per thread loaded before the weight stream (AIN_Q8_1).
template <int F, int MT, int BPL, int LPR, int WGS, int NSTAGE, bool SUMI, int AIN = AIN_Q8_1>
__global__ __launch_bounds__(WGS) void gemv_v1_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                   float* __restrict__ C, int32_t* __restrict__ sumi_out, int M,
                                                   int N, int K, long ldc_m, long ldc_n, long sA, long sB, long sC) {
    using G = gemv_v1_geom<F, BPL>;
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
    const int row = blockIdx.x * RPB + (tid >> 6) * RPW + lane / LPR;
    const bool row_ok = row < N;

    const uint8_t* wrow = B + (long)(row_ok ? row : 0) * ((long)U * G::UB);
    auto load_unit = [&](uint32_t (&dst)[G::UDW], int u) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(wrow + (long)((row_ok && u < U) ? u : 0) * G::UB);
#pragma unroll
        for (int v = 0; v < G::UDW; ++v) dst[v] = p[v];
    };
    auto rec_of = [&](int blk) {
        const int m = blk / nb;
        const int b = blk - m * nb;
        const int u = b / BPL;
        return (m * U + u) * G::REC_DW + (b - u * BPL) * 12;
    };
    uint32_t cur[G::UDW];

    if constexpr (AIN == AIN_Q8_1) {
        // 1) activation staging loads first
        const int tot = M * nb * 9;
        uint32_t av[NSTAGE];
#pragma unroll
        for (int i = 0; i < NSTAGE; ++i) {
            const int g = tid + i * WGS;
            av[i] = g < tot ? A[g] : 0u;
        }
        // 2) weight stream: first unit of this lane
        load_unit(cur, lir);
        // 3) activations -> LDS records (the first NSTAGE*WGS dwords were loaded above; a K too
        //    large for that chunk stages the remainder here, after the weight stream is in flight)
        auto stage = [&](int g, uint32_t v) {
            const int blk = g / 9;
            const int w = g - blk * 9;
            const int rec = rec_of(blk);
            if (w == 0) {
                lds[rec + 8] = __float_as_uint(h2f(v & 0xFFFFu));
                lds[rec + 9] = __float_as_uint(h2f(v >> 16));
            } else {
                lds[rec + w - 1] = v;
            }
        };
#pragma unroll
        for (int i = 0; i < NSTAGE; ++i) {
            const int g = tid + i * WGS;
            if (g < tot) stage(g, av[i]);
        }
        for (int g = tid + NSTAGE * WGS; g < tot; g += WGS) stage(g, A[g]);
    } else {
        // Fused quantization: one thread per 32-element block, first block's loads in flight
        // before the weight stream.
        const uint8_t* X = reinterpret_cast<const uint8_t*>(A);
        const int totb = M * nb;
        float xv[32];
        if (tid < totb) load_act_block_v1<AIN>(X, tid, xv);
        load_unit(cur, lir);
        for (int g = tid; g < totb; g += WGS) {
            if (g != tid) load_act_block_v1<AIN>(X, g, xv);
            uint32_t w[9];
            if constexpr (AIN == AIN_F32) quantize_q8_1_block<0>(xv, w);
            else quantize_q8_1_block_fp16_fused(xv, w);
            uint32_t* r = lds + rec_of(g);
            *reinterpret_cast<uint4*>(r) = make_uint4(w[1], w[2], w[3], w[4]);
            *reinterpret_cast<uint4*>(r + 4) = make_uint4(w[5], w[6], w[7], w[8]);
            *reinterpret_cast<float2*>(r + 8) = make_float2(h2f(w[0] & 0xFFFFu), h2f(w[0] >> 16));
        }
    }
    __syncthreads();

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;

    const int iters = (U + LPR - 1) / LPR;
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
                        const uint32_t* rec = lds + (m * U + u) * G::REC_DW + bi * 12;
                        const uint4 a0 = *reinterpret_cast<const uint4*>(rec);
                        const uint4 a1 = *reinterpret_cast<const uint4*>(rec + 4);
                        const float2 ds = *reinterpret_cast<const float2*>(rec + 8);
                        const uint32_t a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                        const int sumi = dot_block(wb.q, a);
                        if constexpr (SUMI) {
                            if (row_ok) sumi_out[((long)m * N + row) * nb + u * BPL + bi] = sumi;
                        } else {
                            acc[m] += block_term<F>(sumi, wb.d, wb.m, ds.x, ds.y);
                        }
                    }
                }
            });
        }
        if (j + 1 < iters) {
#pragma unroll
            for (int v = 0; v < G::UDW; ++v) cur[v] = nxt[v];
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
}

// Host side -------------------------------------------------------------------------------------

template <int F, int BPL> inline size_t gemv_v1_lds_bytes(int M, int K) {
    return (size_t)M * (K / QK / BPL) * gemv_v1_geom<F, BPL>::REC_DW * 4;
}

// Preconditions of both kernels for unit size BPL: whole units per row, 4-byte aligned operands
// (units and rows are then whole dwords), LDS records fit (staged kernel).
template <int F, int BPL>
inline bool gemv_v1_shape_ok(const GemmArgs& g) {
    if (g.M < 1 || g.M > 8) return false;
    if (g.K % (QK * BPL) != 0) return false;
    const int aal = g.ain == AIN_Q8_1 ? 3 : 15;  // fused: 16-B vector loads of the FP32/FP16 rows
    if (((uintptr_t)g.B & 3) != 0 || ((uintptr_t)g.A & aal) != 0) return false;
    if (g.batch > 1 && ((g.sB & 3) != 0 || (g.sA & aal) != 0)) return false;
    if (g.sumi && g.ain != AIN_Q8_1) return false;
    if (g.M > 2 && gemv_v1_lds_bytes<F, BPL>(g.M, g.K) > 96 * 1024) return false;
    return true;
}

template <int F, int MT, int BPL, int LPR, int WGS, int NSTAGE, bool SUMI, int AIN = AIN_Q8_1>
hipError_t gemv_v1_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    const size_t lds = gemv_v1_lds_bytes<F, BPL>(g.M, g.K);
    const int grid = (g.N + RPB - 1) / RPB;
    auto kfn = gemv_v1_kernel<F, MT, BPL, LPR, WGS, NSTAGE, SUMI, AIN>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, dim3(grid, g.batch), dim3(WGS), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.C,
                       g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n, g.sA, g.sB, g.sC);
    return hipGetLastError();
}

}  // namespace qg
