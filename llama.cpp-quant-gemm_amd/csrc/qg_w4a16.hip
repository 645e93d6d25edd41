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
// runs as chunks of 8 activation rows on blockIdx.y (the weights are streamed once per chunk).
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {

template <int F, int BPL> struct w16_geom {
    static constexpr int BB = wfmt<F>::BB;
    static constexpr int UB = BPL * BB;
    static constexpr int UDW = UB / 4;
    static constexpr int REC_DW = 32 * BPL + 4;
    static_assert(UB % 4 == 0, "whole-dword units");
};

// Exact float value of weight element j (0..3) of decoded dword x: q - 8 (Q4_0), q (Q8_0).
template <int F> __device__ __forceinline__ float w16_elem(uint32_t x, int j) {
    if constexpr (F == FMT_Q8_0) return (float)(int)(int8_t)(x >> (8 * j));
    else return (float)((x >> (8 * j)) & 0xFFu) - 8.0f;
}

template <int F, int MT, int BPL, int LPR, int WGS>
__global__ __launch_bounds__(WGS) void w16_gemv_kernel(const float* __restrict__ A, const uint8_t* __restrict__ B,
                                                       float* __restrict__ C, int M, int N, int K, long ldc_m,
                                                       long ldc_n, long sA, long sC) {
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

    const int iters = (U + LPR - 1) / LPR;
    for (int j = 0; j < iters; ++j) {
        const int u = lir + j * LPR;
        uint32_t nxt[G::UDW];
        if (j + 1 < iters) load_unit(nxt, u + LPR);
        if (u < U) {
            static_for<BPL>([&](auto BI) {
                constexpr int bi = decltype(BI)::value;
                const wblock wb = decode_block<F, bi>(cur);
                float w[32];
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int e = 0; e < 4; ++e) w[4 * i + e] = w16_elem<F>(wb.q[i], e);
#pragma unroll
                for (int m = 0; m < MT; ++m) {
                    if (m < M) {
                        const float* rec = lds_f + (m * U + u) * G::REC_DW + bi * 32;
                        float s = 0.0f;
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const float4 a = *reinterpret_cast<const float4*>(rec + 4 * i);
                            s = __builtin_fmaf(a.x, w[4 * i], s);
                            s = __builtin_fmaf(a.y, w[4 * i + 1], s);
                            s = __builtin_fmaf(a.z, w[4 * i + 2], s);
                            s = __builtin_fmaf(a.w, w[4 * i + 3], s);
                        }
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

namespace {
constexpr int W16_MT = 8;
constexpr size_t W16_LDS_MAX = 128 * 1024;

template <int F, int BPL> size_t w16_lds(int mt, int K) { return (size_t)mt * (K / QK / BPL) * w16_geom<F, BPL>::REC_DW * 4; }

template <int F, int MT, int BPL, int LPR, int WGS>
hipError_t w16_launch(const GemmArgs& g, hipStream_t st) {
    constexpr int RPB = (WGS / 64) * (64 / LPR);
    const int rows = g.M < MT ? g.M : MT;
    const size_t lds = w16_lds<F, BPL>(rows, g.K);
    const dim3 grid((g.N + RPB - 1) / RPB, (g.M + MT - 1) / MT);
    auto kfn = w16_gemv_kernel<F, MT, BPL, LPR, WGS>;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kfn, grid, dim3(WGS), lds, st, (const float*)g.A, (const uint8_t*)g.B, g.C, g.M, g.N, g.K,
                       g.ldc_m, g.ldc_n, (long)MT * g.K, (long)MT * g.ldc_m);
    return hipGetLastError();
}

template <int F, int MT> hipError_t w16_launch_mt(const GemmArgs& g, hipStream_t st) {
    const int nb = g.K / QK;
    if (nb % 4 == 0) {
        if (nb / 4 >= 32) return w16_launch<F, MT, 4, 32, 512>(g, st);
        return w16_launch<F, MT, 4, 4, 256>(g, st);
    }
    return w16_launch<F, MT, 2, 8, 256>(g, st);
}

template <int F> bool w16_fast_ok(const GemmArgs& g) {
    const int nb = g.K / QK;
    const int bpl = nb % 4 == 0 ? 4 : 2;
    if (nb % bpl != 0) return false;
    if (((uintptr_t)g.A & 15) != 0 || ((uintptr_t)g.B & 3) != 0) return false;
    if ((g.M + W16_MT - 1) / W16_MT > 65535) return false;
    const int mt = g.M < W16_MT ? (g.M <= 1 ? 1 : g.M <= 2 ? 2 : g.M <= 4 ? 4 : W16_MT) : W16_MT;
    const size_t lds = bpl == 4 ? w16_lds<F, 4>(mt, g.K) : w16_lds<F, 2>(mt, g.K);
    return lds <= W16_LDS_MAX;
}

template <int F> hipError_t w16_dispatch(const GemmArgs& g, hipStream_t st) {
    if (w16_fast_ok<F>(g)) {
        if (g.M <= 1) return w16_launch_mt<F, 1>(g, st);
        if (g.M <= 2) return w16_launch_mt<F, 2>(g, st);
        if (g.M <= 4) return w16_launch_mt<F, 4>(g, st);
        return w16_launch_mt<F, W16_MT>(g, st);
    }
    if (g.M > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(w16_generic_kernel<F>, dim3((g.N + 3) / 4, g.M), dim3(256), 0, st, (const float*)g.A,
                       (const uint8_t*)g.B, g.C, g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_w16(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return w16_dispatch<FMT_Q4_0>(g, st);
        case FMT_Q8_0: return w16_dispatch<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
