// gemv_experiments.hpp — experimental GEMV variants (tuning probes only, not the product): cheaper activation staging and
// fewer/wider weight loads per lane. Not yet wired into the product dispatch.
#pragma once
#include "qg_gemv_kernel.hpp"  // -I ../llama.cpp-quant-gemm_amd/csrc
#include "qg_kernels.hpp"

namespace qg {

// QG_STAMPS diagnostics: see qg_gemv_kernel.hpp

typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef unsigned int u32x2b __attribute__((ext_vector_type(2)));

// Stage M Q8_1 rows (M*nb*36 bytes, 16-B aligned base) into LDS records of 12 dwords per block
// (8 qs dwords, f32 d, f32 s, 2 pad), using dwordx4 loads: piece p holds dwords 4p..4p+3.
// Returns nothing; caller issues the loads (ld) early and calls st() later.
template <int WGS, int NP>
struct act_stage {
    u32x4 v[NP];
    int tot16;  // 16-B pieces
    __device__ __forceinline__ void ld(const uint8_t* A, int bytes, int tid) {
        tot16 = (bytes + 15) >> 4;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int p = tid + i * WGS;
            v[i] = p < tot16 ? *reinterpret_cast<const u32x4*>(A + p * 16) : u32x4{0u, 0u, 0u, 0u};
        }
    }
    __device__ __forceinline__ static void put(uint32_t* rec_base, int dw, uint32_t val, int ndw) {
        if (dw >= ndw) return;
        const int blk = dw / 9;
        const int w = dw - blk * 9;
        if (w == 0) {
            rec_base[blk * 12 + 8] = __float_as_uint(h2f(val & 0xFFFFu));
            rec_base[blk * 12 + 9] = __float_as_uint(h2f(val >> 16));
        } else {
            rec_base[blk * 12 + w - 1] = val;
        }
    }
    __device__ __forceinline__ void st(uint32_t* recs, const uint8_t* A, int bytes, int tid) {
        const int ndw = bytes >> 2;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
            const int p = tid + i * WGS;
            if (p < tot16) {
                put(recs, 4 * p, v[i].x, ndw);
                put(recs, 4 * p + 1, v[i].y, ndw);
                put(recs, 4 * p + 2, v[i].z, ndw);
                put(recs, 4 * p + 3, v[i].w, ndw);
            }
        }
        for (int p = tid + NP * WGS; p < tot16; p += WGS) {
            const u32x4 x = *reinterpret_cast<const u32x4*>(A + p * 16);
            put(recs, 4 * p, x.x, ndw);
            put(recs, 4 * p + 1, x.y, ndw);
            put(recs, 4 * p + 2, x.z, ndw);
            put(recs, 4 * p + 3, x.w, ndw);
        }
    }
};

// ------------------------------------------------------------------------------------------------
// Design B/C: per-lane units of BPL blocks (as qg_gemv_kernel.hpp) with a chosen load shape.
//   LM 0: NL x (2*BPL)-byte loads (the product's shape)
//   LM 1: Q4_0 BPL=2: 3 x dwordx3 (36 B)
//   LM 2: Q4_0 BPL=4: 4 x dwordx4 + 1 x dwordx2 with lane-parity offsets (72 B)
// Rows per wave 64/LPR, WGS/64 waves; activation records: (m, unit) records of BPL x 12 dwords + 4.
template <int F, int MT, int BPL, int LPR, int WGS, int LM, int NPA>
__global__ __launch_bounds__(WGS) void gemv2_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                    float* __restrict__ C, int M, int N, int K, long ldc_m,
                                                    long ldc_n) {
    constexpr int BB = wfmt<F>::BB;
    constexpr int UB = BPL * BB;
    constexpr int UDW = UB / 4;
    constexpr int REC = 12 * BPL + 4;
    constexpr int RPW = 64 / LPR;
    constexpr int RPB = (WGS / 64) * RPW;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int nb = K / QK;
    const int U = nb / BPL;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int lir = lane % LPR;
    const int row = blockIdx.x * RPB + (tid >> 6) * RPW + lane / LPR;
    const bool row_ok = row < N;
    QG_STAMP(t0);
    QG_CLK(c0);

    act_stage<WGS, NPA> as;
    const int abytes = M * nb * 36;
    as.ld(A, abytes, tid);

    const uint8_t* wrow = B + (long)(row_ok ? row : 0) * ((long)U * UB);
    uint32_t w[UDW];
    auto load_unit = [&](int u) {
        const uint8_t* p = wrow + (long)((row_ok && u < U) ? u : 0) * UB;
        if constexpr (LM == 0) {
            constexpr int LW = 2 * BPL;
            constexpr int NL = UB / LW;
#pragma unroll
            for (int i = 0; i < NL; ++i) {
                if constexpr (LW == 4) w[i] = *reinterpret_cast<const uint32_t*>(p + 4 * i);
                else if constexpr (LW == 8) {
                    const u32x2b t = *reinterpret_cast<const u32x2b*>(p + 8 * i);
                    w[2 * i] = t.x; w[2 * i + 1] = t.y;
                } else {
                    const u32x4 t = *reinterpret_cast<const u32x4*>(p + 16 * i);
                    w[4 * i] = t.x; w[4 * i + 1] = t.y; w[4 * i + 2] = t.z; w[4 * i + 3] = t.w;
                }
            }
        } else if constexpr (LM == 1) {
            static_assert(UB == 36, "LM1: Q4_0, BPL=2");
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const u32x3 t = *reinterpret_cast<const u32x3*>(p + 12 * i);
                w[3 * i] = t.x; w[3 * i + 1] = t.y; w[3 * i + 2] = t.z;
            }
        } else {
            static_assert(UB == 72, "LM2: Q4_0, BPL=4");
            const bool odd = (reinterpret_cast<uintptr_t>(p) & 8) != 0;
            const int o2 = odd ? 0 : 64;
            const int o4 = odd ? 8 : 0;
            const u32x2b x2 = *reinterpret_cast<const u32x2b*>(p + o2);
            u32x4 x4[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) x4[i] = *reinterpret_cast<const u32x4*>(p + o4 + 16 * i);
            uint32_t s[16];
#pragma unroll
            for (int i = 0; i < 4; ++i) { s[4 * i] = x4[i].x; s[4 * i + 1] = x4[i].y; s[4 * i + 2] = x4[i].z; s[4 * i + 3] = x4[i].w; }
            // even: s[0..15], x2 -> w[16..17]; odd: x2 -> w[0..1], s[0..15] -> w[2..17]
            w[0] = vsel(odd, x2.x, s[0]);
            w[1] = vsel(odd, x2.y, s[1]);
#pragma unroll
            for (int i = 2; i < 16; ++i) w[i] = vsel(odd, s[i - 2], s[i]);
            w[16] = vsel(odd, s[14], x2.x);
            w[17] = vsel(odd, s[15], x2.y);
        }
    };
    load_unit(lir);

    // activation records
    {
        // records indexed (m*U + u)*REC + (b%BPL)*12: remap the flat block index blk = m*nb + b
        uint32_t* recs = lds;
        const int ndw = abytes >> 2;
        auto put = [&](int dw, uint32_t val) {
            if (dw >= ndw) return;
            const int blk = dw / 9;
            const int wd = dw - blk * 9;
            const int m = blk / nb;
            const int b = blk - m * nb;
            const int u = b / BPL;
            const int rec = (m * U + u) * REC + (b - u * BPL) * 12;
            if (wd == 0) {
                recs[rec + 8] = __float_as_uint(h2f(val & 0xFFFFu));
                recs[rec + 9] = __float_as_uint(h2f(val >> 16));
            } else {
                recs[rec + wd - 1] = val;
            }
        };
#pragma unroll
        for (int i = 0; i < NPA; ++i) {
            const int p = tid + i * WGS;
            if (p < as.tot16) { put(4 * p, as.v[i].x); put(4 * p + 1, as.v[i].y); put(4 * p + 2, as.v[i].z); put(4 * p + 3, as.v[i].w); }
        }
        for (int p = tid + NPA * WGS; p < as.tot16; p += WGS) {
            const u32x4 x = *reinterpret_cast<const u32x4*>(A + p * 16);
            put(4 * p, x.x); put(4 * p + 1, x.y); put(4 * p + 2, x.z); put(4 * p + 3, x.w);
        }
    }
    __syncthreads();
    QG_STAMP(tb);
    QG_WAIT_STAMP(t1);

    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
    const int iters = (U + LPR - 1) / LPR;
    for (int j = 0; j < iters; ++j) {
        const int u = lir + j * LPR;
        uint32_t cur[UDW];
#pragma unroll
        for (int i = 0; i < UDW; ++i) cur[i] = w[i];
        if (j + 1 < iters) load_unit(u + LPR);
        if (u < U) {
            static_for<BPL>([&](auto BI) {
                constexpr int bi = decltype(BI)::value;
                const wblock wb = decode_block<F, bi>(cur);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < M) {
                        const uint32_t* rec = lds + (m * U + u) * REC + bi * 12;
                        const uint4 a0 = *reinterpret_cast<const uint4*>(rec);
                        const uint4 a1 = *reinterpret_cast<const uint4*>(rec + 4);
                        const float2 ds = *reinterpret_cast<const float2*>(rec + 8);
                        const uint32_t a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                        acc[m] += block_term<F>(dot_block(wb.q, a), wb.d, wb.m, ds.x, ds.y);
                    }
                }
            });
        }
    }
    QG_STAMP(tc);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = group_sum_last<LPR>(acc[m]);
    if (row_ok && lir == LPR - 1) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
            if (m < M) C[m * ldc_m + row * ldc_n] = acc[m];
    }
    QG_STAMP(t2);
    QG_CLK(c2);
    QG_STAMP_STORE(t0, tb, t1, tc, t2, c0, c2);
}

template <int F, int MT, int BPL, int LPR, int WGS, int LM, int NPA>
hipError_t gemv2_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    const size_t lds = (size_t)g.M * (g.K / QK / BPL) * (12 * BPL + 4) * 4;
    const int grid = (g.N + RPB - 1) / RPB;
    auto kfn = gemv2_kernel<F, MT, BPL, LPR, WGS, LM, NPA>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(WGS), lds, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.C, g.M, g.N,
                       g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Design A: workgroup-cooperative, one block per thread (Q4_0/Q4_1/Q5_x), activation staging by
// dwordx4. WGS threads, RW rows; weight span pieces (tid + i*WGS) -> LDS (VGPR or DMA); compute
// thread t < RW*TPR takes blocks lt, lt+TPR, ... of row t/TPR (TPR a multiple of 64).
template <int F, int MT, int WGS, int RW, int TPR, int NLD, int NPA, bool DMA>
__global__ __launch_bounds__(WGS) void gemv_coop2_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                         float* __restrict__ C, int M, int N, int K, long ldc_m,
                                                         long ldc_n) {
    constexpr int BB = wfmt<F>::BB;
    constexpr int BDW = (BB + 2 + 3) / 4;
    static_assert(TPR % 64 == 0 && RW * TPR <= WGS, "compute threads");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int nb = K / QK;
    const long RB = (long)nb * BB;
    const int tid = threadIdx.x;
    const int row0 = blockIdx.x * RW;
    const int rows_here = min(RW, N - row0);
    const int span = (int)(rows_here * RB);
    uint8_t* wl = reinterpret_cast<uint8_t*>(lds);
    uint32_t* recs = lds + (RW * RB + 15) / 16 * 4;
    float* red = reinterpret_cast<float*>(recs + M * nb * 12);

    act_stage<WGS, NPA> as;
    const int abytes = M * nb * 36;
    as.ld(A, abytes, tid);

    const uint8_t* src = B + (long)row0 * RB;
    u32x4 v[DMA ? 1 : NLD];
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int off = (tid + i * WGS) * 16;
        if constexpr (DMA) {
            if (off < span)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(src + off),
                    (__attribute__((address_space(3))) void*)(wl + (i * WGS + (tid & ~63)) * 16), 16, 0, 0);
        } else {
            v[i] = off < span ? *reinterpret_cast<const u32x4*>(src + off) : u32x4{0u, 0u, 0u, 0u};
        }
    }
    as.st(recs, A, abytes, tid);
    if constexpr (!DMA) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int off = (tid + i * WGS) * 16;
            if (off < span) *reinterpret_cast<u32x4*>(wl + off) = v[i];
        }
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();

    const int r = tid / TPR;
    const int lt = tid - r * TPR;
    const int row = row0 + r;
    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
    if (r < rows_here) {
        for (int j = lt; j < nb; j += TPR) {
            const int off = (int)(r * RB) + j * BB;
            const uint32_t* p = reinterpret_cast<const uint32_t*>(wl + (off & ~3));
            uint32_t raw[BDW + 1], w[BDW];
#pragma unroll
            for (int i = 0; i < BDW; ++i) raw[i] = p[i];
            raw[BDW] = 0;
            const uint32_t sh = (uint32_t)(off & 3);
#pragma unroll
            for (int i = 0; i < BDW; ++i) w[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh);
            const wblock wb = decode_block<F, 0>(w);
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (m < M) {
                    const uint32_t* rec = recs + (m * nb + j) * 12;
                    const uint4 a0 = *reinterpret_cast<const uint4*>(rec);
                    const uint4 a1 = *reinterpret_cast<const uint4*>(rec + 4);
                    const float2 ds = *reinterpret_cast<const float2*>(rec + 8);
                    const uint32_t a[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
                    acc[m] += block_term<F>(dot_block(wb.q, a), wb.d, wb.m, ds.x, ds.y);
                }
            }
        }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc[m] += __shfl_xor(acc[m], o);
    }
    constexpr int WPR = TPR / 64;
    if constexpr (WPR == 1) {
        if (lt == 0 && r < rows_here) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                if (m < M) C[m * ldc_m + (long)row * ldc_n] = acc[m];
        }
    } else {
        if ((lt & 63) == 0 && r < RW) {
#pragma unroll
            for (int m = 0; m < MT; ++m) red[(r * MT + m) * WPR + (lt >> 6)] = acc[m];
        }
        __syncthreads();
        if (lt == 0 && r < rows_here) {
#pragma unroll
            for (int m = 0; m < MT; ++m) {
                if (m < M) {
                    float s = red[(r * MT + m) * WPR];
#pragma unroll
                    for (int q = 1; q < WPR; ++q) s += red[(r * MT + m) * WPR + q];
                    C[m * ldc_m + (long)row * ldc_n] = s;
                }
            }
        }
    }
}

template <int F, int MT, int WGS, int RW, int TPR, int NLD, int NPA, bool DMA>
hipError_t gemv_coop2_launch(const GemmArgs& g, hipStream_t st) {
    const long RB = (long)(g.K / QK) * wfmt<F>::BB;
    if ((RB * RW) % 16 != 0 || RB * RW > (long)NLD * WGS * 16 || g.N % RW != 0) return hipErrorInvalidValue;
    const size_t lds = (size_t)(RW * RB + 15) / 16 * 16 + (size_t)g.M * (g.K / QK) * 48 + (size_t)RW * MT * (TPR / 64) * 4;
    const int grid = (g.N + RW - 1) / RW;
    auto kfn = gemv_coop2_kernel<F, MT, WGS, RW, TPR, NLD, NPA, DMA>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(WGS), lds, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.C, g.M, g.N,
                       g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}

}  // namespace qg

// ------------------------------------------------------------------------------------------------
// Design D ("register activations", M = 1): no LDS, no barrier. Lane (row, unit u) loads its
// weight unit (BPL blocks) AND the matching BPL activation blocks (BPL*36 B, L2/L1-resident after
// the first touch) straight into VGPRs; the dot products read both from registers. Waves are fully
// independent; the per-row reduction is DPP.
namespace qg {
template <int F, int BPL, int LPR, int WGS>
__global__ __launch_bounds__(WGS) void gemv_rax_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                      float* __restrict__ C, int N, int K) {
    constexpr int BB = wfmt<F>::BB;
    constexpr int UB = BPL * BB;
    constexpr int UDW = UB / 4;
    constexpr int ADW = BPL * 9;  // activation dwords per unit
    constexpr int RPW = 64 / LPR;
    constexpr int RPB = (WGS / 64) * RPW;
    const int nb = K / QK;
    const int U = nb / BPL;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int lir = lane % LPR;
    const int row = blockIdx.x * RPB + (tid >> 6) * RPW + lane / LPR;
    const bool row_ok = row < N;
    QG_STAMP(t0);
    QG_CLK(c0);
    const uint8_t* wrow = B + (long)(row_ok ? row : 0) * ((long)U * UB);
    float acc = 0.0f;
    const int iters = (U + LPR - 1) / LPR;
    for (int j = 0; j < iters; ++j) {
        const int u = lir + j * LPR;
        const int uu = (row_ok && u < U) ? u : 0;
        uint32_t w[UDW], a[ADW];
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(wrow + (long)uu * UB);
        const uint32_t* ap = reinterpret_cast<const uint32_t*>(A + (long)uu * BPL * 36);
#pragma unroll
        for (int i = 0; i < UDW; ++i) w[i] = wp[i];
#pragma unroll
        for (int i = 0; i < ADW; ++i) a[i] = ap[i];
        QG_STAMP(tb);
        QG_WAIT_STAMP(t1);
        if (u < U) {
            static_for<BPL>([&](auto BI) {
                constexpr int bi = decltype(BI)::value;
                const wblock wb = decode_block<F, bi>(w);
                const float da = h2f(a[9 * bi] & 0xFFFFu);
                const float sa = h2f(a[9 * bi] >> 16);
                acc += block_term<F>(dot_block(wb.q, a + 9 * bi + 1), wb.d, wb.m, da, sa);
            });
        }
        if (j + 1 == iters) {
            QG_STAMP(tc);
            acc = group_sum_last<LPR>(acc);
            if (row_ok && lir == LPR - 1) C[row] = acc;
            QG_STAMP(t2);
            QG_CLK(c2);
            QG_STAMP_STORE(t0, tb, t1, tc, t2, c0, c2);
        }
    }
}

template <int F, int BPL, int LPR, int WGS>
hipError_t gemv_rax_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    if (g.M != 1 || (g.K / QK) % BPL != 0) return hipErrorInvalidValue;
    const int grid = (g.N + RPB - 1) / RPB;
    hipLaunchKernelGGL((gemv_rax_kernel<F, BPL, LPR, WGS>), dim3(grid), dim3(WGS), 0, st, (const uint8_t*)g.A,
                       (const uint8_t*)g.B, g.C, g.N, g.K);
    return hipGetLastError();
}
}  // namespace qg

// ------------------------------------------------------------------------------------------------
// Design D, generalised ("register activations", M <= 2, optional next-unit prefetch): measured
// equal to the staged product kernel at N=K=4096 and slower at N=32000 / other formats
// (profiles/r01_tuning/gemv_probe5.txt), so not dispatched.
namespace qg {
// ------------------------------------------------------------------------------------------------
template <int F, int MT, int BPL, int LPR, int WGS, bool PF, bool SUMI>
__global__ __launch_bounds__(WGS) void gemv_ra_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                      float* __restrict__ C, int32_t* __restrict__ sumi_out, int M,
                                                      int N, int K, long ldc_m, long ldc_n, long sA, long sB,
                                                      long sC) {
    using G = gemv_geom<F, BPL>;
    constexpr int ADWX = BPL * 9;
    static_assert(BPL % 2 == 0, "units must be whole dwords");
    A += blockIdx.y * sA;  // strided batch: blockIdx.y selects an independent product
    B += blockIdx.y * sB;
    C += blockIdx.y * sC;
    constexpr int RPW = 64 / LPR;
    constexpr int RPB = (WGS / 64) * RPW;
    const int nb = K / QK;
    const int U = nb / BPL;
    const int lane = threadIdx.x & 63;
    const int lir = lane % LPR;
    const int row = blockIdx.x * RPB + (threadIdx.x >> 6) * RPW + lane / LPR;
    const bool row_ok = row < N;
    const uint8_t* wrow = B + (long)(row_ok ? row : 0) * ((long)U * G::UB);
    const long arow = (long)nb * 36;

    // one unit's weight dwords + the matching activation dwords of every row m
    auto load = [&](uint32_t (&w)[G::UDW], uint32_t (&a)[MT][ADWX], int u) {
        const int uu = (row_ok && u < U) ? u : 0;
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(wrow + (long)uu * G::UB);
#pragma unroll
        for (int i = 0; i < G::UDW; ++i) w[i] = wp[i];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const uint32_t* ap = reinterpret_cast<const uint32_t*>(A + (m < M ? m : 0) * arow + (long)uu * BPL * 36);
#pragma unroll
            for (int i = 0; i < ADWX; ++i) a[m][i] = ap[i];
        }
    };
    float acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = 0.0f;
    const int iters = (U + LPR - 1) / LPR;
    uint32_t w[G::UDW], a[MT][ADWX];
    load(w, a, lir);
    for (int j = 0; j < iters; ++j) {
        const int u = lir + j * LPR;
        uint32_t w2[G::UDW], a2[MT][ADWX];
        if (PF && j + 1 < iters) load(w2, a2, u + LPR);  // next unit in flight during this one
        if (row_ok && u < U) {
            static_for<BPL>([&](auto BI) {
                constexpr int bi = decltype(BI)::value;
                const wblock wb = decode_block<F, bi>(w);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < M) {
                        const int s = dot_block(wb.q, &a[m][9 * bi + 1]);
                        if constexpr (SUMI) {
                            sumi_out[((long)m * N + row) * nb + u * BPL + bi] = s;
                        } else {
                            const float da = h2f(a[m][9 * bi] & 0xFFFFu);
                            const float sa = h2f(a[m][9 * bi] >> 16);
                            acc[m] += block_term<F>(s, wb.d, wb.m, da, sa);
                        }
                    }
                }
            });
        }
        if (j + 1 < iters) {
            if constexpr (PF) {
#pragma unroll
                for (int i = 0; i < G::UDW; ++i) w[i] = w2[i];
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int i = 0; i < ADWX; ++i) a[m][i] = a2[m][i];
            } else {
                load(w, a, u + LPR);
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
}

template <int F, int MT, int BPL, int LPR, int WGS, bool PF, bool SUMI>
hipError_t gemv_ra_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    const int grid = (g.N + RPB - 1) / RPB;
    hipLaunchKernelGGL((gemv_ra_kernel<F, MT, BPL, LPR, WGS, PF, SUMI>), dim3(grid, g.batch), dim3(WGS), 0, st,
                       (const uint8_t*)g.A, (const uint8_t*)g.B, g.C, g.sumi, g.M, g.N, g.K, g.ldc_m, g.ldc_n, g.sA,
                       g.sB, g.sC);
    return hipGetLastError();
}

}  // namespace qg
