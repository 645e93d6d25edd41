// mmq_tile_experiment.hpp — EXPERIMENT (tools only, not the product): W4A8 prefill GEMM for larger M where the waves of a workgroup split the OUTPUT tile
// and share every staged K slice (the classic GEMM structure), instead of splitting K as
// qg_mmq_kernel.hpp does.
//
// C[M,N] = A_q8_1[M,K] . B_w[N,K]^T (include/gemm_reference.h:175-222), activation-major.
//
// Why a second kernel: the K-split kernel keeps a whole 32-row x 16/32-token tile per wave, so its
// tiles stay small and every weight row is re-read from L2 once per 16-32 tokens; at M = 512 the
// loads alone took 34 of its 54 us (profiles/r01_tuning/mmq_probe_ablation.txt). Here a workgroup
// owns BNW = WR*RT*16 weight rows x BTW = WT*TT*16 tokens (128 x 64 at M >= 256): per K element it
// moves BNW*18/32 + BTW*36/32 bytes for BNW*BTW products, 3-4x fewer bytes per product.
//
// Per block (one v_mfma_i32_16x16x32_i8 per 16x16 sub-tile, exact int32 sumi) the arithmetic,
// operand k-order, C layout and epilogue are those of qg_mmq_kernel.hpp (biased accumulator,
// packed-f32 pairs, d_w / m_w as f16 through v_fma_mix_f32).
//
// Stages of 4 blocks (128 K) are fetched by LDS-DMA (global_load_lds_dwordx4) into NB shared
// buffers: every wave issues NIW of the stage's DMA instructions (weight pieces first, then
// activation pieces, one piece numbering), waits for its own (counted vmcnt), then one s_barrier
// makes the stage visible to all waves and frees the buffer consumed in the previous iteration,
// which is refilled NB-1 stages ahead. No LDS writes in the loop (hipcc would wait for every DMA in
// flight before one).
#pragma once
#include "qg_mmq_kernel.hpp"

namespace qg {

template <int F, int WR, int WT, int RT, int TT, int NB> struct mmq_tile_geom {
    using T = wfmt<F>;
    static constexpr int W = WR * WT;                          // waves
    static constexpr int BNW = WR * RT * 16;                   // weight rows per workgroup
    static constexpr int BTW = WT * TT * 16;                   // tokens per workgroup
    static constexpr int RSB = MMQ_SB * T::BB;                 // weight bytes per row per stage
    static constexpr int RIMG = RSB % 16 != 0 ? RSB + 8 : RSB; // 16-B aligned row window
    static constexpr int PPR = RIMG / 16;
    static constexpr int WPC = BNW * PPR;                      // weight pieces per stage
    static constexpr int APC = BTW * 9;                        // activation pieces per stage
    static constexpr int NIS = (WPC + APC + 63) / 64;          // DMA instructions per stage
    static constexpr int NIW = (NIS + W - 1) / W;              // ... per wave (padded)
    static constexpr int OFF_A = WPC * 16;
    static constexpr int BUF = NIW * W * 64 * 16;              // stage buffer bytes
    static constexpr size_t LDS = (size_t)NB * BUF;
    static_assert(LDS <= 160 * 1024, "LDS per workgroup");
    static_assert(NB >= 2 && NB <= 4 && NB * NIW <= 63, "stage ring / vmcnt range");
    static_assert(RSB % 8 == 0, "stage segments are 8-B multiples");
    __host__ __device__ static constexpr int shift(int h) { return (h * RSB) & 15; }
};

template <int F, int WR, int WT, int RT, int TT, int NB, bool SUMI>
__global__ __launch_bounds__(WR * WT * 64) void mmq_tile_kernel(const uint8_t* __restrict__ A,
                                                                const uint8_t* __restrict__ B,
                                                                float* __restrict__ C, int32_t* __restrict__ sumi_out,
                                                                int M, int N, int K, long ldc_m, long ldc_n) {
    using G = mmq_tile_geom<F, WR, WT, RT, TT, NB>;
    using T = wfmt<F>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15;
    const int q = lane >> 4;
    const int wr = wave % WR, wt = wave / WR;   // this wave's sub-tile
    const int n0 = blockIdx.x * G::BNW, m0 = blockIdx.y * G::BTW;
    const int rw = wr * RT * 16, tw = wt * TT * 16;
    const int nb = K / QK;
    const int H = nb / MMQ_SB;
    const long RB = (long)nb * T::BB;
    const long AB = (long)nb * Q8_1_BYTES;

    // this wave's DMA instructions j = wave + W * i of each stage: lane piece p = 64 j + lane
    int coff[G::NIW];
    bool cisw[G::NIW];
#pragma unroll
    for (int i = 0; i < G::NIW; ++i) {
        const int p = min(64 * (wave + G::W * i) + lane, G::WPC + G::APC - 1);
        cisw[i] = p < G::WPC;
        if (cisw[i]) {
            const int row = p / G::PPR;
            coff[i] = (int)((long)min(n0 + row, N - 1) * RB) + (p - row * G::PPR) * 16;
        } else {
            const int pa = p - G::WPC, tok = pa / 9;
            coff[i] = (int)((long)min(m0 + tok, M - 1) * AB) + (pa - tok * 9) * 16;
        }
    }
    // every lane issues every DMA instruction (see qg_mmq_kernel.hpp: no lane-predicated DMA)
    auto issue = [&](int h, uint8_t* buf) {
        const uint8_t* wsrc = B + (long)h * G::RSB - G::shift(h);
        const uint8_t* asrc = A + (long)h * 144;
#pragma unroll
        for (int i = 0; i < G::NIW; ++i)
            glds<16>((cisw[i] ? wsrc : asrc) + coff[i], buf + (wave + G::W * i) * 1024);
    };

    constexpr int NACC = RT * TT * 4;
    float acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = 0.0f;
    const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};
    constexpr float CS = F == FMT_Q4_0 ? 8.0f : F == FMT_Q5_0 ? 16.0f : F == FMT_Q8_0 ? 0.0f : -1.0f;
    constexpr bool HAS_M = T::MOFF >= 0;
    struct blk_t {
        v4i c[RT][TT];
        uint32_t dw[RT][4], mw[RT][4];
        f32x2 da[TT], nda[TT], ncs[TT];
    };
    auto u16 = [](const uint8_t* p) { return (uint32_t)*reinterpret_cast<const uint16_t*>(p); };
    auto epilogue = [&](const blk_t& p, int h, int b) {
#pragma unroll
        for (int t = 0; t < TT; ++t)
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                if constexpr (SUMI) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int n = n0 + rw + 16 * i + 4 * q + e, m = m0 + tw + 16 * t + r16;
                        if (n < N && m < M) sumi_out[((long)m * N + n) * nb + h * MMQ_SB + b] = p.c[i][t][e] - MMQ_BIAS;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 4; e += 2) {
                        const f32x2 cf = {__int_as_float(p.c[i][t][e]), __int_as_float(p.c[i][t][e + 1])};
                        float* a = &acc[(i * TT + t) * 4 + e];
                        if constexpr (!HAS_M) {
                            f32x2 t2 = __builtin_elementwise_fma(p.da[t], cf, p.nda[t]);  // d_a * sumi
                            if constexpr (CS != 0.0f) t2 = t2 + p.ncs[t];                   // - c * s_a
                            a[0] = fma_mix_lo(p.dw[i][e], t2.x, a[0]);
                            a[1] = fma_mix_lo(p.dw[i][e + 1], t2.y, a[1]);
                        } else {
                            const f32x2 x = cf - f32x2{MMQ_BIAS_F, MMQ_BIAS_F};            // exact: sumi
                            const f32x2 dd = {fma_mix_lo(p.dw[i][e], p.da[t].x, -0.0f),
                                              fma_mix_lo(p.dw[i][e + 1], p.da[t].x, -0.0f)};
                            const f32x2 t1 = dd * x;
                            a[0] += fma_mix_lo(p.mw[i][e], p.ncs[t].x, t1.x);              // + m_w * s_a
                            a[1] += fma_mix_lo(p.mw[i][e + 1], p.ncs[t].x, t1.y);
                        }
                    }
                }
            }
    };
    // one stage: every LDS read, then every MFMA, then every epilogue (qg_mmq_kernel.hpp)
    auto compute = [&](const uint8_t* buf, int h, int sh) {
        blk_t blk[MMQ_SB];
        long afrag[MMQ_SB][RT], bfrag[MMQ_SB][TT];
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            constexpr int o = b * T::BB;
#pragma unroll
            for (int i = 0; i < RT; ++i) {
                const uint8_t* wr_ = buf + (rw + 16 * i + r16) * G::RIMG + sh;
                uint32_t lo, hi;
                if constexpr (T::Q8) {
                    lo = lds32<o + T::QS>(wr_ + 4 * q);
                    hi = lds32<o + T::QS + 16>(wr_ + 4 * q);
                } else {
                    const uint32_t v = lds32<o + T::QS>(wr_ + 4 * q);
                    lo = v & 0x0F0F0F0Fu;
                    hi = (v >> 4) & 0x0F0F0F0Fu;
                }
                if constexpr (T::QH >= 0) {
                    const uint32_t qh = lds32<o + T::QH>(wr_);
                    lo |= spread4_bit4((qh >> (4 * q)) & 0xFu);
                    hi |= spread4_bit4((qh >> (16 + 4 * q)) & 0xFu);
                }
                afrag[b][i] = (long)(((unsigned long)hi << 32) | lo);
                const uint8_t* sr = buf + (rw + 16 * i + 4 * q) * G::RIMG + sh + o;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    blk[b].dw[i][e] = u16(sr + e * G::RIMG);
                    if constexpr (HAS_M) blk[b].mw[i][e] = u16(sr + e * G::RIMG + T::MOFF);
                }
            }
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const uint8_t* ar = buf + G::OFF_A + (tw + 16 * t + r16) * 144 + b * Q8_1_BYTES;
                const uint32_t qa0 = *reinterpret_cast<const uint32_t*>(ar + 4 + 4 * q);
                const uint32_t qa1 = *reinterpret_cast<const uint32_t*>(ar + 20 + 4 * q);
                bfrag[b][t] = (long)(((unsigned long)qa1 << 32) | qa0);
                const uint32_t dsh = *reinterpret_cast<const uint32_t*>(ar);
                const float da = h2f(dsh & 0xFFFFu), sa = h2f(dsh >> 16);
                const float nda = -(da * MMQ_BIAS_F), ncs = -(CS * sa);
                blk[b].da[t] = f32x2{da, da};
                blk[b].nda[t] = f32x2{nda, nda};
                blk[b].ncs[t] = f32x2{ncs, ncs};
            }
        });
        __builtin_amdgcn_sched_barrier(0);
        static_for<MMQ_SB>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int i = 0; i < RT; ++i)
                    blk[b].c[i][t] = __builtin_amdgcn_mfma_i32_16x16x32_i8(afrag[b][i], bfrag[b][t], bias, 0, 0, 0);
        });
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        static_for<MMQ_SB>([&](auto BI) { epilogue(blk[decltype(BI)::value], h, decltype(BI)::value); });
        __builtin_amdgcn_sched_barrier(0);
    };

    // stage ring: NB-1 stages in flight ahead of the one computed
#pragma unroll
    for (int s = 0; s < NB - 1; ++s)
        if (s < H) issue(s, smem + s * G::BUF);
    for (int h = 0; h < H; ++h) {
        wait_stage<G::NIW>(min(H - 1 - h, NB - 2));  // this wave's pieces of stage h landed
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();                // ... everyone's; everyone done with h - 1
        __builtin_amdgcn_sched_barrier(0);
        if (h + NB - 1 < H) issue(h + NB - 1, smem + ((h + NB - 1) % NB) * G::BUF);
        compute(smem + (h % NB) * G::BUF, h, G::shift(h));
    }

    if constexpr (!SUMI) {
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int n = n0 + rw + 16 * i + 4 * q + e, m = m0 + tw + 16 * t + r16;
                    if (n < N && m < M) C[m * ldc_m + n * ldc_n] = acc[(i * TT + t) * 4 + e];
                }
    }
}

// Preconditions: those of the P16 K-split kernel (16-B aligned A, B and rows; K % 128 == 0, and
// K % 256 == 0 when a stage's row segment is not a 16-B multiple), 32-bit byte offsets.
template <int F, int WR, int WT, int RT, int TT, int NB>
inline bool mmq_tile_shape_ok(const GemmArgs& g) {
    using G = mmq_tile_geom<F, WR, WT, RT, TT, NB>;
    if (g.M < 1 || g.N < 1 || g.K % (QK * MMQ_SB) != 0) return false;
    const long RB = (long)(g.K / QK) * wfmt<F>::BB, AB = (long)(g.K / QK) * Q8_1_BYTES;
    if (((uintptr_t)g.A & 15) != 0 || AB % 16 != 0) return false;
    if (G::RSB % 16 != 0 && g.K % 256 != 0) return false;
    if (((uintptr_t)g.B & 15) != 0 || RB % 16 != 0) return false;
    if (RB * g.N >= (1L << 31) || AB * g.M >= (1L << 31)) return false;
    if ((g.M + G::BTW - 1) / G::BTW > 65535) return false;
    return true;
}

template <int F, int WR, int WT, int RT, int TT, int NB, bool SUMI>
hipError_t mmq_tile_launch(const GemmArgs& g, hipStream_t st) {
    using G = mmq_tile_geom<F, WR, WT, RT, TT, NB>;
    const dim3 grid((g.N + G::BNW - 1) / G::BNW, (g.M + G::BTW - 1) / G::BTW);
    auto k = mmq_tile_kernel<F, WR, WT, RT, TT, NB, SUMI>;
    if (G::LDS > 64 * 1024) {
        static bool attr_set = false;  // once per instantiation (not a stream op: capture-safe)
        if (!attr_set) {
            hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::LDS);
            if (e != hipSuccess) return e;
            attr_set = true;
        }
    }
    hipLaunchKernelGGL(k, grid, dim3(G::W * 64), G::LDS, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.C, g.sumi,
                       g.M, g.N, g.K, g.ldc_m, g.ldc_n);
    return hipGetLastError();
}

}  // namespace qg
