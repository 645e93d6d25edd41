// mmq_direct_experiment.hpp — (probe only, not product) W4A8 small-batch prefill (M <= 32 activation rows), weights straight to VGPRs.
//
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222), activation-major; the same
// arithmetic as qg_mmq_kernel.hpp (one v_mfma_i32_16x16x32_i8 per Q-block = exact int32 sumi of
// 16 weight rows x 16 tokens; MFMA-assisted scale epilogue), with the data movement of the GEMV.
//
// Why (profiles/r02_tuning/ring_probe*.txt): the round-1 prefill DMAs weights
// AND activations into LDS. Its weight stream is the slow half — halving the weight bytes per CU
// (16-row x 32-token tiles) did not shorten the weight-only DMA — while LDS-DMA of bytes every CU
// shares (the activations: L2-resident) runs at ~150 GB/s per CU. The GEMV streams the same weight
// bytes from HBM at 5.4-6.4 TB/s with plain coalesced loads into registers. So here:
//  * a workgroup owns 16 weight rows x 16*TT tokens and all of K; its W waves split K into chunks of
//    BPC blocks (wave w: chunks w, w + W, ...);
//  * weights: lane (r, q) = (lane & 15, lane >> 4) loads row r's contiguous BPC/4 blocks
//    q*BPC/4 .. of the chunk (72 B for Q4_0 at BPC = 16: GEMV-like coalesced loads into VGPRs,
//    no LDS). The MFMA wants lane (r, q) to hold qs dword q of ONE block for all four q: a 4 x 4
//    transpose across the four 16-lane groups (v_permlane32_swap + v_permlane16_swap, 4 VALU ops
//    per 4 dwords) turns "4 blocks x 4 dwords per group" into "4 blocks x dword q" — the product
//    kernel's operand (qs dword q split into low / high nibbles);
//  * activations: each wave DMAs its own chunk slice of the 16*TT token rows into a wave-private
//    LDS image (global_load_lds, lane-linear, one pad piece per token against bank conflicts) and
//    reads the B fragments from it — the L2-resident stream;
//  * scale epilogue: per block one v_mfma_f32_16x16x16_f16 forms d_w (x) d_a in the accumulator
//    layout (only the lane group that loaded the block feeds its k-slot: no exchange); the
//    compensation sum_b X s_a (X = d_w, or m_w for Q4_1 / Q5_1) of all BPC blocks of a chunk is ONE
//    f16 MFMA (group q feeds its 4 blocks in k-slots 4q..4q+3);
//  * the W partial tiles are summed in fixed wave order through LDS: deterministic.
// A chunk's DMA and weight loads are all issued before its compute; with one chunk per wave
// (K = 32 * BPC * W, e.g. K = 4096 at BPC = 16, W = 8) the whole workgroup's bytes are in flight
// at once. With several chunks per wave the next chunk's DMA and loads go out before the current
// chunk's compute (two LDS images per wave).
#pragma once
#include "qg_mmq_kernel.hpp"

namespace qg {

#ifdef QG_DIRECT_STAMPS
// diagnostic build only (tools/ring_probe.hip): per wave s_memrealtime stamps (100 MHz) at entry,
// issue done, weights landed, activations landed, compute done, exit
__device__ unsigned long long g_direct_stamps[8 * 65536];
#define DSTAMP(k) dst[k] = __builtin_amdgcn_s_memrealtime()
#else
#define DSTAMP(k)
#endif

template <int F, int TT, int W, int BPC, int NBUF> struct direct_geom {
    using T = wfmt<F>;
    static_assert(BPC == 8 || BPC == 16, "chunks of 8 or 16 blocks (2 or 4 per lane group)");
    static_assert(TT == 1 || TT == 2, "16 or 32 tokens");
    static_assert(NBUF == 1 || NBUF == 2, "one or two LDS images per wave");
    static constexpr int BPG = BPC / 4;                   // blocks per lane group per chunk
    static constexpr int UB = BPG * T::BB;                // weight bytes per lane per chunk
    static constexpr int UDW = (UB + 3) / 4;              // ... as dwords (UB is even; Q4_0 BPG=2: 36 B)
    static constexpr int NTOK = 16 * TT;
    static constexpr int ASEG = BPC * Q8_1_BYTES;         // activation bytes per token per chunk
    static constexpr int APR = ASEG / 16;                 // 16-B pieces per token
    static constexpr int APRP = APR + 1;                  // + pad piece
    static constexpr int AIMG = APRP * 16;                // token image stride
    static constexpr int NP = NTOK * APRP;                // pieces per chunk image
    static constexpr int NI = (NP + 63) / 64;             // DMA instructions per chunk
    static constexpr int IMG = NI * 1024;                 // image bytes (whole instructions)
    static constexpr size_t WAVE_LDS = (size_t)NBUF * IMG;
    static constexpr size_t RED = (size_t)W * TT * 4 * 64 * 4;
    static constexpr size_t LDS = (size_t)W * WAVE_LDS > RED ? (size_t)W * WAVE_LDS : RED;
    static_assert(LDS <= 160 * 1024, "LDS per workgroup");
    static_assert(ASEG % 16 == 0, "16-B pieces");
};

// 4 x 4 transpose of dwords across the four 16-lane groups: group q holds x[0..3] = X[q][0..3] on
// entry and X[0..3][q] on exit.
__device__ __forceinline__ void xpose4(uint32_t (&x)[4]) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // lanes 32..63 of x[k] <-> lanes 0..31 of x[k + 2]
        const auto r = __builtin_amdgcn_permlane32_swap(x[k], x[k + 2], false, false);
        x[k] = r[0];
        x[k + 2] = r[1];
    }
#pragma unroll
    for (int k = 0; k < 4; k += 2) {  // odd 16-lane rows of x[k] <-> even rows of x[k + 1]
        const auto r = __builtin_amdgcn_permlane16_swap(x[k], x[k + 1], false, false);
        x[k] = r[0];
        x[k + 1] = r[1];
    }
}

template <int F, int TT, int W, int BPC, int NBUF, bool SUMI>
__global__ __launch_bounds__(W * 64, 1) void mmq_direct_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                               int M, int N, int K, float* __restrict__ C, long ldc_m,
                                                               long ldc_n, int32_t* __restrict__ sumi_out) {
    using G = direct_geom<F, TT, W, BPC, NBUF>;
    using T = wfmt<F>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

#ifdef QG_DIRECT_STAMPS
    unsigned long long dst[8] = {};
#endif
    DSTAMP(0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15;
    const int q = lane >> 4;
    const int n0 = blockIdx.x * 16;
    const int m0 = blockIdx.y * G::NTOK;
    const int nb = K / QK;
    const int nch = nb / BPC;                                   // chunks
    const int nmine = wave < nch ? (nch - 1 - wave) / W + 1 : 0;  // this wave's chunks
    const long RB = (long)nb * T::BB;
    const long AB = (long)nb * Q8_1_BYTES;
    uint8_t* img0 = smem + wave * G::WAVE_LDS;

    // weight unit of this lane: row n0 + r16 (clamped), blocks q * BPG .. of each chunk
    const uint8_t* wrow = B + (long)min(n0 + r16, N - 1) * RB + q * G::UB;
    // activation DMA: piece p of a chunk image -> token p / APRP (clamped to M - 1), piece p % APRP
    // (the pad piece re-fetches piece 0); lanes past the image fetch a clamped piece into the tail
    const uint8_t* Aw = A + (long)m0 * AB;
    auto issue = [&](int c, uint8_t* img, uint32_t (&wu)[G::UDW]) {  // weights (HBM) first, then the DMA
        const uint32_t* p = reinterpret_cast<const uint32_t*>(wrow + (long)c * BPC * T::BB);
#pragma unroll
        for (int v = 0; v < G::UDW; ++v) wu[v] = p[v];
        const uint8_t* asrc = Aw + (long)c * G::ASEG;
        int ln = lane;
        asm volatile("" : "+v"(ln));  // offsets recomputed per call, not held live across the compute
#pragma unroll
        for (int i = 0; i < G::NI; ++i) {
            const int pc = min(64 * i + ln, G::NP - 1);
            const int tok = pc / G::APRP, k = pc - tok * G::APRP;
            glds<16>(asrc + (min(m0 + tok, M - 1) - m0) * (int)AB + (k < G::APR ? k : 0) * 16, img + i * 1024);
        }
    };

    float acc[TT * 4];
#pragma unroll
    for (int i = 0; i < TT * 4; ++i) acc[i] = 0.0f;
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr bool HAS_M = T::MOFF >= 0;
    constexpr bool HAS_S = F != FMT_Q8_0;
    constexpr float CFAC = F == FMT_Q4_0 ? -8.0f : F == FMT_Q5_0 ? -16.0f : 1.0f;
    f32x4v c2[TT];
#pragma unroll
    for (int t = 0; t < TT; ++t) c2[t] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};
    const f32x4v z4 = {0.f, 0.f, 0.f, 0.f};
    auto h4 = [](unsigned long v) { return __builtin_bit_cast(f16x4, v); };

    // One chunk: weight unit wu (this lane's BPG blocks of row r16), activation image img.
    auto compute = [&](const uint32_t (&wu)[G::UDW], const uint8_t* img, int c) {
        // per block slot j: the 4 blocks i * BPG + j (i = lane group that loaded it)
        static_for<G::BPG>([&](auto J) {
            constexpr int j = decltype(J)::value;
            constexpr int o = j * T::BB;
            // A fragments: dword q of block i*BPG+j for i = 0..3 (transpose across groups)
            uint32_t lo[4], hi[4];
            if constexpr (T::Q8) {
                uint32_t x0[4], x1[4];
                static_for<4>([&](auto K4) {
                    constexpr int k = decltype(K4)::value;
                    x0[k] = ld32<o + T::QS + 4 * k>(wu);
                    x1[k] = ld32<o + T::QS + 16 + 4 * k>(wu);
                });
                xpose4(x0);
                xpose4(x1);
#pragma unroll
                for (int i = 0; i < 4; ++i) { lo[i] = x0[i]; hi[i] = x1[i]; }
            } else {
                uint32_t x[4];
                static_for<4>([&](auto K4) { x[decltype(K4)::value] = ld32<o + T::QS + 4 * decltype(K4)::value>(wu); });
                xpose4(x);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    lo[i] = x[i] & 0x0F0F0F0Fu;
                    hi[i] = (x[i] >> 4) & 0x0F0F0F0Fu;
                }
                if constexpr (T::QH >= 0) {
                    const uint32_t qh = ld32<o + T::QH>(wu);
                    uint32_t h[4] = {qh, qh, qh, qh};
                    xpose4(h);  // h[i] = qh of block i*BPG+j
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        lo[i] |= spread4_bit4((h[i] >> (4 * q)) & 0xFu);
                        hi[i] |= spread4_bit4((h[i] >> (16 + 4 * q)) & 0xFu);
                    }
                }
            }
            const uint32_t dw = ld16<o>(wu);  // d_w of this lane's block q*BPG+j (f16 bits)
            // phase 1: every LDS read of the 4 blocks (B fragments, d_a)
            long bf[4][TT];
            uint32_t da[4][TT];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const uint8_t* ar = img + (16 * t + r16) * G::AIMG + (i * G::BPG + j) * Q8_1_BYTES;
                    const uint32_t qa0 = *reinterpret_cast<const uint32_t*>(ar + 4 + 4 * q);
                    const uint32_t qa1 = *reinterpret_cast<const uint32_t*>(ar + 20 + 4 * q);
                    bf[i][t] = (long)(((unsigned long)qa1 << 32) | qa0);
                    da[i][t] = *reinterpret_cast<const uint16_t*>(ar);
                }
            // phase 2: the MFMAs (integer dots; d_w (x) d_a of block b = i*BPG+j, fed only by lane
            // group i, which loaded block b: no exchange)
            v4i cc[4][TT];
            f32x4v dd[4][TT];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const long af = (long)(((unsigned long)hi[i] << 32) | lo[i]);
#pragma unroll
                for (int t = 0; t < TT; ++t) cc[i][t] = __builtin_amdgcn_mfma_i32_16x16x32_i8(af, bf[i][t], bias, 0, 0, 0);
            }
            if constexpr (!SUMI) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const bool mine = q == i;
#pragma unroll
                    for (int t = 0; t < TT; ++t)
                        dd[i][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(h4(mine ? (unsigned long)dw : 0ul),
                                                                         h4(mine ? (unsigned long)da[i][t] : 0ul), z4, 0, 0, 0);
                }
            }
            // phase 3: epilogue (or the parity hook's per-block sumi)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    if constexpr (SUMI) {
                        const int b = i * G::BPG + j;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int n = n0 + 4 * q + e, m = m0 + 16 * t + r16;
                            if (n < N && m < M) sumi_out[((long)m * N + n) * nb + c * BPC + b] = cc[i][t][e] - MMQ_BIAS;
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; e += 2) {
                            const f32x2 sm = f32x2{__int_as_float(cc[i][t][e]), __int_as_float(cc[i][t][e + 1])} -
                                             f32x2{MMQ_BIAS_F, MMQ_BIAS_F};  // exact: sumi
                            float* a = &acc[t * 4 + e];
                            const f32x2 r = __builtin_elementwise_fma(f32x2{dd[i][t][e], dd[i][t][e + 1]}, sm, f32x2{a[0], a[1]});
                            a[0] = r.x;
                            a[1] = r.y;
                        }
                    }
                }
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (HAS_S && !SUMI) {
            // compensation over the chunk's BPC blocks in one MFMA per token tile: lane group q
            // feeds X of its blocks q*BPG + j (j < BPG <= 4) in k-slots 4q + j, and s_a of the same
            // blocks of its token
            uint32_t xs[4] = {0u, 0u, 0u, 0u};
            static_for<G::BPG>([&](auto J) {
                constexpr int o = decltype(J)::value * T::BB;
                xs[decltype(J)::value] = HAS_M ? ld16<o + (HAS_M ? T::MOFF : 0)>(wu) : ld16<o>(wu);
            });
            const unsigned long xa = ((unsigned long)((xs[3] << 16) | xs[2]) << 32) | ((xs[1] << 16) | xs[0]);
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                uint32_t sa[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                for (int j = 0; j < G::BPG; ++j)
                    sa[j] = *reinterpret_cast<const uint16_t*>(img + (16 * t + r16) * G::AIMG + (q * G::BPG + j) * Q8_1_BYTES + 2);
                const unsigned long sb = ((unsigned long)((sa[3] << 16) | sa[2]) << 32) | ((sa[1] << 16) | sa[0]);
                c2[t] = __builtin_amdgcn_mfma_f32_16x16x16f16(h4(xa), h4(sb), c2[t], 0, 0, 0);
            }
        }
    };

    if (nmine > 0) {
        uint32_t wu[NBUF][G::UDW];
        issue(wave, img0, wu[0]);
        for (int k = 0; k < nmine; ++k) {
            const int c = wave + k * W;
            if constexpr (NBUF == 2) {
                const int cur = k & 1;
                if (k + 1 < nmine) {
                    // next chunk in flight: its at least ceil(UB / 16) weight loads (at most 16 B
                    // each) and NI DMA instructions are younger than this chunk's DMA
                    if (cur == 0) issue(c + W, img0 + G::IMG, wu[1]);
                    else issue(c + W, img0, wu[0]);
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::NI + (G::UB + 15) / 16) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (cur == 0) compute(wu[0], img0, c);
                else compute(wu[1], img0 + G::IMG, c);
            } else {
#ifdef QG_DIRECT_STAMPS
                if (k == 0) {
                    DSTAMP(1);
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::NI) : "memory");
                    DSTAMP(2);
                }
#endif
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef QG_DIRECT_STAMPS
                if (k == 0) DSTAMP(3);
#endif
                compute(wu[0], img0, c);
#ifdef QG_DIRECT_STAMPS
                if (k == 0) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); DSTAMP(4); }
#endif
                if (k + 1 < nmine) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this image's reads retired
                    issue(c + W, img0, wu[0]);
                }
            }
        }
    }

    if constexpr (!SUMI) {
        if constexpr (HAS_S) {
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[t * 4 + e] = __builtin_fmaf(CFAC, c2[t][e], acc[t * 4 + e]);
        }
        float* red = reinterpret_cast<float*>(smem);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int i = 0; i < TT * 4; ++i) red[(wave * TT * 4 + i) * 64 + lane] = acc[i];
        __syncthreads();
        constexpr int TS = TT * 4 * 64;  // outputs per tile = 16 rows x 16*TT tokens
        const bool nfast = ldc_n == 1;
        for (int idx = threadIdx.x; idx < TS; idx += W * 64) {
            const int nl = nfast ? idx & 15 : idx / G::NTOK;
            const int ml = nfast ? idx >> 4 : idx % G::NTOK;
            const int qq = nl >> 2, e = nl & 3, t = ml >> 4, cl = ml & 15;
            const int src = (t * 4 + e) * 64 + qq * 16 + cl;
            float v = red[src];
#pragma unroll
            for (int ww = 1; ww < W; ++ww) v += red[ww * TS + src];
            const int n = n0 + nl, m = m0 + ml;
            if (n < N && m < M) C[m * ldc_m + n * ldc_n] = v;
        }
    }
#ifdef QG_DIRECT_STAMPS
    DSTAMP(5);
    if (lane == 0) {
        const int wv = (blockIdx.y * gridDim.x + blockIdx.x) * W + wave;
        for (int kk = 0; kk < 6; ++kk) g_direct_stamps[8 * wv + kk] = dst[kk];
    }
#endif
}

// Preconditions: K a multiple of 32 * BPC, 16-B aligned activation rows and base (DMA pieces),
// 4-B aligned weight units (B 4-B aligned; row and unit strides are even multiples of the block).
template <int F, int TT, int W, int BPC, int NBUF> inline bool direct_shape_ok(const GemmArgs& g) {
    if (g.M < 1 || g.N < 1 || g.K % (QK * BPC) != 0 || g.batch != 1) return false;
    if (g.M > 16 * TT * 65535) return false;
    const long RB = (long)(g.K / QK) * wfmt<F>::BB, AB = (long)(g.K / QK) * Q8_1_BYTES;
    if (((uintptr_t)g.A & 15) != 0 || AB % 16 != 0 || ((uintptr_t)g.B & 3) != 0 || RB % 4 != 0) return false;
    if (AB * 16 * TT >= (1L << 31)) return false;
    return true;
}

template <int F, int TT, int W, int BPC, int NBUF, bool SUMI> hipError_t direct_launch(const GemmArgs& g, hipStream_t st) {
    using G = direct_geom<F, TT, W, BPC, NBUF>;
    const dim3 grid((g.N + 15) / 16, (g.M + G::NTOK - 1) / G::NTOK);
    auto k = mmq_direct_kernel<F, TT, W, BPC, NBUF, SUMI>;
    if (g.describe) {  // qg_debug_config: name the instantiation instead of launching it
        describe_kernel(g, "mmq_direct F=%d TT=%d W=%d BPC=%d NBUF=%d grid=%ux%u", F, TT, W, BPC, NBUF, grid.x, grid.y);
        return hipSuccess;
    }
    if (G::LDS > 64 * 1024) {
        static bool attr_set = false;  // once per instantiation (not a stream op: capture-safe)
        if (!attr_set) {
            hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
            if (e != hipSuccess) return e;
            attr_set = true;
        }
    }
    hipLaunchKernelGGL(k, grid, dim3(W * 64), G::LDS, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, g.C,
                       g.ldc_m, g.ldc_n, g.sumi);
    return hipGetLastError();
}

}  // namespace qg
