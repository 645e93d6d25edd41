// qg_gemv_kernel.hpp — the W4A8 GEMV / small-batch kernel template (M <= 8 activation rows).
//
// Included by qg_gemv.hip (the product's instantiations + dispatch) and by tools/gemv_probe.hip
// (the tuning sweep). Computes, for the reference's activation-major contract
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222):
//   C[m*ldc_m + n*ldc_n] = sum_b term(A[m][b], B[n][b]).
//
// Work decomposition:
//  * A lane owns "units" of BPL consecutive Q-blocks of one weight row. A unit is BPL*BB bytes
//    = NL loads of LW = 2*BPL bytes each (BB even), e.g. Q4_0: BPL=2 -> 9 x dword (36 B),
//    BPL=4 -> 9 x dwordx2 (72 B), BPL=8 -> 9 x dwordx4 (144 B). Unit starts are LW-aligned
//    because rows are K/32*BB bytes with (K/32) % BPL == 0. Smaller units -> more waves in
//    flight per CU and less serial decode per lane (the launch is latency-bound, §4).
//  * LPR lanes share a row and stride over its units; 64/LPR rows per wave, WGS/64 waves per
//    workgroup. Blocks are decoded in registers with compile-time alignbyte/shift/mask
//    (qg_common.hpp) and dotted with v_dot4c_i32_i8: exact int32 sumi.
//  * Q8_1 activations are staged once per workgroup into LDS records per (row m, unit): BPL
//    blocks x 48 B (32 B int8 qs, float d, float s, 8 B pad) + 16 B pad, i.e. a dword stride of
//    12*BPL + 4 = 4 x odd, so the 16 lanes of a ds_read_b128 group hit 16 distinct 4-bank slots.
//    Activation loads are issued before the weight stream so the ds_write waits only on them.
//  * Per-lane partials (unit order, block order) are tree-reduced across the row's LPR lanes
//    with __shfl_xor; lane 0 of the row stores. Deterministic.
#pragma once
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int LW> struct load_vec;
template <> struct load_vec<4> { typedef uint32_t type; };
template <> struct load_vec<8> { typedef u32x2 type; };
template <> struct load_vec<16> { typedef u32x4 type; };

template <int F, int BPL> struct gemv_geom {
    static constexpr int BB = wfmt<F>::BB;
    static constexpr int LW = 2 * BPL;           // bytes per load
    static constexpr int NL = BB / 2;            // loads per unit
    static constexpr int UB = BPL * BB;          // unit bytes
    static constexpr int UDW = UB / 4;           // unit dwords
    static constexpr int REC_DW = 12 * BPL + 4;  // LDS record dwords per (m, unit)
};

// ABL (tuning ablations, tools/gemv_probe.hip only; the product uses 0): 1 = skip the activation
// staging (LDS left uninitialised), 2 = skip decode/dot (fold the weight words), 3 = both.
// DMA: the workgroup's weight rows (one contiguous span) are copied HBM -> LDS with
// global_load_lds_dwordx4 (perfectly coalesced 1 KB per wave-instruction, no VGPRs), then each lane
// reads its units from LDS; otherwise lanes load their units straight into VGPRs.
template <int F, int MT, int BPL, int LPR, int WGS, int NSTAGE, bool NT, bool SUMI, int ABL = 0, bool DMA = false>
__global__ __launch_bounds__(WGS) void gemv_kernel(const uint32_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                   float* __restrict__ C, int32_t* __restrict__ sumi_out, int M,
                                                   int N, int K, long ldc_m, long ldc_n, long sA, long sB, long sC) {
    using G = gemv_geom<F, BPL>;
    // strided batch: blockIdx.y selects an independent GEMV (sA/sB in bytes, sC in floats)
    A = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(A) + blockIdx.y * sA);
    B += blockIdx.y * sB;
    C += blockIdx.y * sC;
    using LT = typename load_vec<G::LW>::type;
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

    // 1) activation staging loads first
    const int tot = (ABL & 1) ? 0 : M * nb * 9;
    uint32_t av[NSTAGE];
#pragma unroll
    for (int i = 0; i < NSTAGE; ++i) {
        const int g = tid + i * WGS;
        av[i] = g < tot ? A[g] : 0u;
    }

    // 2) weight stream: first unit of this lane
    const LT* wrow = reinterpret_cast<const LT*>(B + (long)(row_ok ? row : 0) * ((long)U * G::UB));
    auto load_unit = [&](LT (&dst)[G::NL], int u) {
        const LT* p = wrow + (long)((row_ok && u < U) ? u : 0) * G::NL;
#pragma unroll
        for (int v = 0; v < G::NL; ++v) {
            if constexpr (NT) dst[v] = __builtin_nontemporal_load(p + v);
            else dst[v] = p[v];
        }
    };
    // DMA: weight span of this workgroup at the front of LDS, activation records after it
    const int row0 = blockIdx.x * RPB;
    const long row_bytes = (long)U * G::UB;
    uint8_t* wlds = reinterpret_cast<uint8_t*>(lds);
    uint32_t* alds = lds;
    if constexpr (DMA) {
        const long span = (long)max(0, min(RPB, N - row0)) * row_bytes;
        alds = lds + (RPB * row_bytes + 15) / 16 * 4;
        const uint8_t* src = B + (long)row0 * row_bytes;
        const int nchunks = (int)((span + 1023) / 1024);
        for (int j = tid >> 6; j < nchunks; j += WGS / 64) {
            const long off = (long)j * 1024 + lane * 16;
            if (off < span)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + off),
                                                 (__attribute__((address_space(3))) void*)(wlds + (long)j * 1024),
                                                 16, 0, 0);
        }
    }
    auto lds_unit = [&](LT (&dst)[G::NL], int u) {
        const LT* p = reinterpret_cast<const LT*>(wlds + (long)(row - row0) * row_bytes + (long)(u < U ? u : 0) * G::UB);
#pragma unroll
        for (int v = 0; v < G::NL; ++v) dst[v] = p[v];
    };
    LT cur[G::NL];
    if constexpr (!DMA) load_unit(cur, lir);

    // 3) activations -> LDS records (the first NSTAGE*WGS dwords were loaded above; a K too
    //    large for that chunk stages the remainder here, after the weight stream is in flight)
    auto stage = [&](int g, uint32_t v) {
        const int blk = g / 9;
        const int w = g - blk * 9;
        const int m = blk / nb;
        const int b = blk - m * nb;
        const int u = b / BPL;
        const int rec = (m * U + u) * G::REC_DW + (b - u * BPL) * 12;
        if (w == 0) {
            alds[rec + 8] = __float_as_uint(h2f(v & 0xFFFFu));
            alds[rec + 9] = __float_as_uint(h2f(v >> 16));
        } else {
            alds[rec + w - 1] = v;
        }
    };
#pragma unroll
    for (int i = 0; i < NSTAGE; ++i) {
        const int g = tid + i * WGS;
        if (g < tot) stage(g, av[i]);
    }
    for (int g = tid + NSTAGE * WGS; g < tot; g += WGS) stage(g, A[g]);
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS-DMA is not tracked
    __syncthreads();
    if constexpr (DMA) {
        if (row_ok) lds_unit(cur, lir);
    }

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;

    const int iters = (U + LPR - 1) / LPR;
    for (int j = 0; j < iters; ++j) {
        const int u = lir + j * LPR;
        LT nxt[G::NL];
        if (j + 1 < iters) {
            if constexpr (DMA) {
                if (row_ok) lds_unit(nxt, u + LPR);
            } else {
                load_unit(nxt, u + LPR);
            }
        }
        if constexpr ((ABL & 2) != 0) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(cur);
            uint32_t x = 0;
#pragma unroll
            for (int i = 0; i < G::UDW; ++i) x ^= w[i];
            acc[0] += (float)(x & 0xFF);
        } else if (u < U) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(cur);
            static_for<BPL>([&](auto BI) {
                constexpr int bi = decltype(BI)::value;
                const wblock wb = decode_block<F, bi>(w);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < M) {
                        const uint32_t* rec = alds + (m * U + u) * G::REC_DW + bi * 12;
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
            for (int v = 0; v < G::NL; ++v) cur[v] = nxt[v];
        }
    }
    if constexpr (!SUMI) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
#pragma unroll
            for (int off = LPR / 2; off > 0; off >>= 1) acc[m] += __shfl_xor(acc[m], off);
        }
        if (row_ok && lir == 0) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                if (m < M) C[m * ldc_m + row * ldc_n] = acc[m];
        }
    }
}

// Host side -------------------------------------------------------------------------------------

template <int F, int BPL> inline size_t gemv_lds_bytes(int M, int K) {
    return (size_t)M * (K / QK / BPL) * gemv_geom<F, BPL>::REC_DW * 4;
}

template <int F, int MT, int BPL, int LPR, int WGS, int NSTAGE, bool NT, bool SUMI, int ABL = 0, bool DMA = false>
hipError_t gemv_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    size_t lds = gemv_lds_bytes<F, BPL>(g.M, g.K);
    if (DMA) lds += ((size_t)RPB * (g.K / QK) * wfmt<F>::BB + 15) / 16 * 16;
    const int grid = (g.N + RPB - 1) / RPB;
    auto kfn = gemv_kernel<F, MT, BPL, LPR, WGS, NSTAGE, NT, SUMI, ABL, DMA>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, dim3(grid, g.batch), dim3(WGS), lds, st, (const uint32_t*)g.A, (const uint8_t*)g.B, g.C,
                       g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n, g.sA, g.sB, g.sC);
    return hipGetLastError();
}

// Preconditions of gemv_kernel<F, *, BPL, *, WGS, NSTAGE>.
template <int F, int BPL>
inline bool gemv_shape_ok(const GemmArgs& g) {
    using G = gemv_geom<F, BPL>;
    if (g.M < 1 || g.M > 8) return false;
    if (g.K % (QK * BPL) != 0) return false;
    if (((uintptr_t)g.B % G::LW) != 0 || ((uintptr_t)g.A & 3) != 0) return false;
    if (gemv_lds_bytes<F, BPL>(g.M, g.K) > 96 * 1024) return false;
    return true;
}

}  // namespace qg
