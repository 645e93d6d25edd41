// mmqc_experiment.hpp (archived round-4 experiment, measured slower; not built into the product) — the small-M W4A8 prefill (M <= 32 tokens per token tile) with a
// workgroup-cooperative, chunked operand ingest (round 4).
//
// Same arithmetic as qg_mmq_kernel.hpp's EPI2 form (v_mfma_i32_16x16x32_i8: one MFMA = one Q-block's
// exact int32 sumi for 16 weight rows x 16 tokens, accumulator seeded with 1.5*2^23; the d_w (x) d_a
// outer product on v_mfma_f32_16x16x16_f16; the compensation sum_b X s_a over each wave's 4 blocks by
// one more MFMA per tile), so the per-element results obey the same reassociation bound and the
// parity hook (SUMI) covers the same fragment decode. What differs is how the operands reach LDS:
//
//  * The per-wave stages of the mmq kernel fetch 32 rows x 72 B (4 blocks) per DMA stage: 72-byte
//    row segments, ~26 cache lines per 1-KB wave-instruction. Measured DMA-only (tools/dma_probe2.hip,
//    profiles/r04_tuning/dma_probe2*.txt, M = 32, N = K = 4096): 72-B segments ~5.9 us, 144 B 5.0,
//    288 B 4.75, 576 B 4.33, linear 4.27 — the segment length, not the bytes, set the ingest time.
//  * Here a workgroup (BN = 32 rows x 16 tokens, W = 8 waves, all of K) moves K in chunks of
//    CB = 32 blocks: per chunk 32 row images of CB*BB bytes (576 B for Q4_0, one contiguous segment of
//    each row) and 16 token images of CB*36 = 1152 B, every wave issuing its share (NIW 1-KB
//    global_load_lds instructions) of every chunk. Images carry one 16-B pad piece (rows 592 B apart:
//    the fragment reads of 16 rows spread over the banks; the pad lanes re-fetch the row's previous
//    piece). R chunk slots (4 for Q4_0 / Q4_1 at 40 KB each) form a ring: at K = 4096 every byte is
//    requested at entry.
//  * Chunk c: each wave waits for ITS pieces of c (counted vmcnt), then one s_barrier — every wave's
//    pieces have landed, and every wave has finished reading chunk c - 1, whose slot then takes the
//    refill of chunk c + R - 1 — and each wave computes 4 of the chunk's 32 blocks for both row tiles.
//    One barrier per chunk (4 at K = 4096), no per-wave buffers.
//  * The W per-wave partial tiles are summed in fixed wave order through LDS at the end (as mmq), so
//    outputs are deterministic.
// Preconditions (mmqc_shape_ok): K % (32 * CB) == 0, 16-B aligned A, B and rows, 32-bit DMA offsets.
#pragma once
#include "qg_mmq_kernel.hpp"

namespace qg {

template <int F, int BN, int TT, int W, int CB> struct mmqc_geom {
    using T = wfmt<F>;
    static constexpr int NTOK = 16 * TT;
    static constexpr int RSEG = CB * T::BB;          // weight bytes of one row per chunk
    static constexpr int ASEG = CB * Q8_1_BYTES;     // activation bytes of one token per chunk
    static constexpr int RIMG = RSEG + 16;           // + one pad piece per image (bank spread)
    static constexpr int AIMG = ASEG + 16;
    static constexpr int RP = RIMG / 16, AP = AIMG / 16;  // 16-B pieces per row / token image
    static constexpr int WP = BN * RP, APC = NTOK * AP;
    static constexpr int NI = (WP + APC + 63) / 64;       // 1-KB DMA instructions per chunk
    static constexpr int NIW = (NI + W - 1) / W;          // ... per wave (the rest fetch a dummy piece)
    static constexpr int SLOT = NIW * W * 1024;
    static constexpr int WOFF = WP * 16;                  // token images follow the row images
    static constexpr int BPW = CB / W;                    // blocks per wave and chunk
    static constexpr int RT = BN / 16;
    static constexpr int NACC = RT * TT * 4;
    static constexpr int R0 = (160 * 1024) / SLOT;
    static constexpr int R = R0 > 4 ? 4 : R0;             // ring slots
    static constexpr size_t RED = (size_t)W * NACC * 64 * 4;  // end-of-kernel partial tiles
    static constexpr size_t LDS = (size_t)R * SLOT > RED ? (size_t)R * SLOT : RED;
    static_assert(RSEG % 16 == 0 && ASEG % 16 == 0, "chunk segments are whole 16-B pieces");
    static_assert(BPW == 4, "each wave computes one 4-block sub-stage per chunk");
    static_assert(R >= 2 && (R - 1) * NIW <= 63, "ring depth / vmcnt range");
    static_assert(LDS <= 160 * 1024, "LDS per workgroup");
    static_assert(BN % 16 == 0 && TT >= 1 && TT <= 2, "row tiles of 16, <= 32 tokens");
};

#ifdef QG_MMQC_STAMPS
// diagnostic build only (tools/mmqc_probe.hip): per wave 8 s_memrealtime stamps — entry, after the
// barrier of chunks 0..3, main loop done, exit
__device__ unsigned long long g_mmqc_stamps[8 * 65536];
#define MMQC_STAMP(k) stamps[k] = __builtin_amdgcn_s_memrealtime()
#else
#define MMQC_STAMP(k)
#endif

// s_waitcnt vmcnt(younger * NIW): this wave's pieces of the oldest chunk in flight have landed.
template <int NIW> __device__ __forceinline__ void mmqc_wait(int younger) {
    if (younger <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NIW) : "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NIW) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NIW) : "memory");
}

// SUMI: out is the parity hook's int32 [M][N][K/32] buffer, else fp32 C with (ldc_m, ldc_n) strides.
// ABL (tuning probes only; the product uses 0): 1 = DMA, waits and barriers without compute, 2 = compute
// without DMA (on whatever LDS holds).
template <int F, int BN, int TT, int W, int CB, bool SUMI, int ABL = 0>
__global__ __launch_bounds__(W * 64, 1) void mmqc_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B, int M,
                                                         int N, int K, void* __restrict__ out, int ldc_m, int ldc_n) {
    using G = mmqc_geom<F, BN, TT, W, CB>;
    using T = wfmt<F>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int r16 = lane & 15;
    const int q = lane >> 4;
    const int n0 = blockIdx.x * BN;
    const int m0 = blockIdx.y * G::NTOK;
    const int nb = K / QK;
    const int nch = nb / CB;
    const long RB = (long)nb * T::BB;
    const long AB = (long)nb * Q8_1_BYTES;
    const uint8_t* Bw = B + (long)n0 * RB;
    const uint8_t* Aw = A + (long)m0 * AB;
#ifdef QG_MMQC_STAMPS
    unsigned long long stamps[8] = {};
#endif
    MMQC_STAMP(0);

    // this lane's piece of each of the wave's NIW instructions per chunk (offsets relative to the
    // chunk's first byte of the tile's first row / token; rows / tokens past the edge re-read the last
    // valid one, their results are dropped; pad pieces re-read the image's previous piece)
    int off[G::NIW];
    bool isw[G::NIW];
#pragma unroll
    for (int i = 0; i < G::NIW; ++i) {
        const int p = (wave * G::NIW + i) * 64 + lane;
        if (p < G::WP) {
            const int r = p / G::RP, j = min(p - r * G::RP, G::RP - 2);
            off[i] = (min(n0 + r, N - 1) - n0) * (int)RB + j * 16;
            isw[i] = true;
        } else if (p < G::WP + G::APC) {
            const int pa = p - G::WP;
            const int t = pa / G::AP, j = min(pa - t * G::AP, G::AP - 2);
            off[i] = (min(m0 + t, M - 1) - m0) * (int)AB + j * 16;
            isw[i] = false;
        } else {  // past the slot's images: a dummy piece (the tile's first weight piece)
            off[i] = 0;
            isw[i] = true;
        }
    }
    // every lane issues every DMA instruction (a lane-predicated global_load_lds is miscompiled, see
    // qg_mmq_kernel.hpp); the LDS destination of instruction i is wave-uniform
    auto issue = [&](int c) {
        if constexpr (ABL == 2) return;
        uint8_t* slot = smem + (c % G::R) * G::SLOT;
        const uint8_t* ws = Bw + (long)c * G::RSEG;
        const uint8_t* as = Aw + (long)c * G::ASEG;
#pragma unroll
        for (int i = 0; i < G::NIW; ++i) glds<16>((isw[i] ? ws : as) + off[i], slot + (wave * G::NIW + i) * 1024);
    };

    float acc[G::NACC];
#pragma unroll
    for (int i = 0; i < G::NACC; ++i) acc[i] = 0.0f;
    typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
    typedef float f32x4v __attribute__((ext_vector_type(4)));
    constexpr bool HAS_M = T::MOFF >= 0;
    constexpr bool HAS_S = F != FMT_Q8_0;
    constexpr float CFAC = F == FMT_Q4_0 ? -8.0f : F == FMT_Q5_0 ? -16.0f : 1.0f;
    f32x4v c2[G::RT][TT];
#pragma unroll
    for (int i = 0; i < G::RT; ++i)
#pragma unroll
        for (int t = 0; t < TT; ++t) c2[i][t] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const v4i bias = {MMQ_BIAS, MMQ_BIAS, MMQ_BIAS, MMQ_BIAS};
    auto h4 = [](unsigned long v) { return __builtin_bit_cast(f16x4, v); };
    auto u16 = [](const uint8_t* p) { return (uint32_t)*reinterpret_cast<const uint16_t*>(p); };

    // k-slot q of the block at compile-time offset o of a row image (qg_mmq_kernel.hpp's wfrag)
    auto wfrag = [&](const uint8_t* wr, auto O) -> long {
        constexpr int o = decltype(O)::value;
        uint32_t lo, hi;
        if constexpr (T::Q8) {
            lo = lds32<o + T::QS>(wr + 4 * q);
            hi = lds32<o + T::QS + 16>(wr + 4 * q);
        } else {
            const uint32_t v = lds32<o + T::QS>(wr + 4 * q);
            lo = v & 0x0F0F0F0Fu;
            hi = (v >> 4) & 0x0F0F0F0Fu;
        }
        if constexpr (T::QH >= 0) {
            const uint32_t qh = lds32<o + T::QH>(wr);
            lo |= spread4_bit4((qh >> (4 * q)) & 0xFu);
            hi |= spread4_bit4((qh >> (16 + 4 * q)) & 0xFu);
        }
        return (long)(((unsigned long)hi << 32) | lo);
    };
    int32_t* sumi_out = SUMI ? reinterpret_cast<int32_t*>(out) : nullptr;
    auto store_sumi = [&](const v4i& cv, int i, int t, int blk) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int n = n0 + 16 * i + 4 * q + e, m = m0 + 16 * t + r16;
            if (n < N && m < M) sumi_out[((long)m * N + n) * nb + blk] = cv[e] - MMQ_BIAS;
        }
    };

    // this wave's 4 blocks (wave * 4 .. wave * 4 + 3) of chunk c, both row tiles, all token tiles;
    // the three phases of qg_mmq_kernel.hpp's compute4_e2 (all LDS reads, all MFMAs, the epilogue)
    auto compute = [&](int c) {
        const uint8_t* slot = smem + (c % G::R) * G::SLOT;
        const uint8_t* wbase = slot + wave * (4 * T::BB);                // 8-B aligned (4 * BB % 8 == 0)
        const uint8_t* abase = slot + G::WOFF + wave * (4 * Q8_1_BYTES);
        long afrag[4][G::RT], bfrag[4][TT];
        uint32_t wdb[4][G::RT], wmb[4][G::RT], adb[4][TT];
        const bool q0 = q == 0;
        static_for<4>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
            constexpr int o = b * T::BB;
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                const uint8_t* wr = wbase + (16 * i + r16) * G::RIMG;
                afrag[b][i] = wfrag(wr, ic<o>{});
                wdb[b][i] = u16(wr + o);
                if constexpr (HAS_M) wmb[b][i] = u16(wr + o + T::MOFF);
            }
#pragma unroll
            for (int t = 0; t < TT; ++t) {
                const uint8_t* ar = abase + (16 * t + r16) * G::AIMG + b * Q8_1_BYTES;
                const uint32_t qa0 = *reinterpret_cast<const uint32_t*>(ar + 4 + 4 * q);
                const uint32_t qa1 = *reinterpret_cast<const uint32_t*>(ar + 20 + 4 * q);
                bfrag[b][t] = (long)(((unsigned long)qa1 << 32) | qa0);
                adb[b][t] = *reinterpret_cast<const uint32_t*>(ar);  // f16 d_a | f16 s_a << 16
            }
        });
        __builtin_amdgcn_sched_barrier(0);
        f32x4v dd[4][G::RT][TT];
        v4i cc[4][G::RT][TT];
        const f32x4v z4 = {0.f, 0.f, 0.f, 0.f};
        if constexpr (!SUMI) {
            static_for<4>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t)
                        dd[b][i][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(
                            h4(q0 ? (unsigned long)(wdb[b][i] & 0xFFFFu) : 0ul),
                            h4(q0 ? (unsigned long)(adb[b][t] & 0xFFFFu) : 0ul), z4, 0, 0, 0);
            });
        }
        static_for<4>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int t = 0; t < TT; ++t)
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
                    cc[b][i][t] = __builtin_amdgcn_mfma_i32_16x16x32_i8(afrag[b][i], bfrag[b][t], bias, 0, 0, 0);
        });
        if constexpr (HAS_S && !SUMI) {
            // k-slots 0..3 = the wave's 4 blocks (lanes q = 0 only): sum_b X[n][b] s_a[m][b]
#pragma unroll
            for (int i = 0; i < G::RT; ++i) {
                uint32_t x01, x23;
                if constexpr (HAS_M) {
                    x01 = __builtin_amdgcn_perm(wmb[1][i], wmb[0][i], 0x05040100u);
                    x23 = __builtin_amdgcn_perm(wmb[3][i], wmb[2][i], 0x05040100u);
                } else {
                    x01 = __builtin_amdgcn_perm(wdb[1][i], wdb[0][i], 0x05040100u);
                    x23 = __builtin_amdgcn_perm(wdb[3][i], wdb[2][i], 0x05040100u);
                }
                const unsigned long xa = q0 ? (((unsigned long)x23 << 32) | x01) : 0ul;
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const uint32_t s01 = __builtin_amdgcn_perm(adb[1][t], adb[0][t], 0x07060302u);
                    const uint32_t s23 = __builtin_amdgcn_perm(adb[3][t], adb[2][t], 0x07060302u);
                    const unsigned long sb = q0 ? (((unsigned long)s23 << 32) | s01) : 0ul;
                    c2[i][t] = __builtin_amdgcn_mfma_f32_16x16x16f16(h4(xa), h4(sb), c2[i][t], 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // MFMA -> VALU margin (qg_mmq_kernel.hpp header)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SUMI) {
            static_for<4>([&](auto BI) {
                constexpr int b = decltype(BI)::value;
#pragma unroll
                for (int i = 0; i < G::RT; ++i)
#pragma unroll
                    for (int t = 0; t < TT; ++t) store_sumi(cc[b][i][t], i, t, c * CB + wave * 4 + b);
            });
            return;
        }
        static_for<4>([&](auto BI) {
            constexpr int b = decltype(BI)::value;
#pragma unroll
            for (int i = 0; i < G::RT; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int e = 0; e < 4; e += 2) {
                        const f32x2 sm = f32x2{__int_as_float(cc[b][i][t][e]), __int_as_float(cc[b][i][t][e + 1])} -
                                         f32x2{MMQ_BIAS_F, MMQ_BIAS_F};  // exact: sumi
                        float* a = &acc[(i * TT + t) * 4 + e];
                        const f32x2 r = __builtin_elementwise_fma(f32x2{dd[b][i][t][e], dd[b][i][t][e + 1]}, sm,
                                                                  f32x2{a[0], a[1]});
                        a[0] = r.x;
                        a[1] = r.y;
                    }
        });
        __builtin_amdgcn_sched_barrier(0);
    };

    const int pre = nch < G::R ? nch : G::R;
    for (int c = 0; c < pre; ++c) issue(c);
    int issued = pre;
    for (int c = 0; c < nch; ++c) {
        mmqc_wait<G::NIW>(issued - 1 - c);  // this wave's pieces of chunk c have landed
        // this wave's LDS reads of chunk c - 1 have returned (its slot is refilled below by any wave)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
#ifdef QG_MMQC_STAMPS
        if (c < 4) MMQC_STAMP(1 + c);
#endif
        if (c >= 1 && issued < nch) issue(issued++);  // into chunk c - 1's slot
        if constexpr (ABL != 1) compute(c);
    }
    MMQC_STAMP(5);
    if constexpr (!SUMI) {
        if constexpr (HAS_S) {
            asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");  // the last compensation MFMAs
#pragma unroll
            for (int i = 0; i < G::RT; ++i)
#pragma unroll
                for (int t = 0; t < TT; ++t)
#pragma unroll
                    for (int e = 0; e < 4; ++e) acc[(i * TT + t) * 4 + e] = __builtin_fmaf(CFAC, c2[i][t][e], acc[(i * TT + t) * 4 + e]);
        }
        // fixed-order sum of the W partial tiles through LDS (every DMA has landed: vmcnt(0) above)
        float* red = reinterpret_cast<float*>(smem);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int i = 0; i < G::NACC; ++i) red[(wave * G::NACC + i) * 64 + lane] = acc[i];
        __syncthreads();
        constexpr int TS = G::NACC * 64;
        float* C = reinterpret_cast<float*>(out);
        for (int idx = threadIdx.x; idx < TS; idx += W * 64) {
            float v = red[idx];
#pragma unroll
            for (int ww = 1; ww < W; ++ww) v += red[ww * TS + idx];
            const int a = idx >> 6, ln = idx & 63;
            const int e = a & 3, t = (a >> 2) % TT, i = (a >> 2) / TT;
            const int n = n0 + 16 * i + 4 * (ln >> 4) + e;
            const int m = m0 + 16 * t + (ln & 15);
            if (n < N && m < M) C[(long)m * ldc_m + (long)n * ldc_n] = v;
        }
    }
#ifdef QG_MMQC_STAMPS
    MMQC_STAMP(6);
    if (lane == 0) {
        const int wv = (blockIdx.y * gridDim.x + blockIdx.x) * W + wave;
        for (int kk = 0; kk < 7; ++kk) g_mmqc_stamps[8 * wv + kk] = stamps[kk];
    }
#endif
}

template <int F, int BN, int TT, int W, int CB> inline bool mmqc_shape_ok(const GemmArgs& g) {
    using G = mmqc_geom<F, BN, TT, W, CB>;
    if (g.M < 1 || g.N < 1 || g.K % (QK * CB) != 0) return false;
    const long RB = (long)(g.K / QK) * wfmt<F>::BB, AB = (long)(g.K / QK) * Q8_1_BYTES;
    if (((uintptr_t)g.A & 15) != 0 || ((uintptr_t)g.B & 15) != 0 || RB % 16 != 0 || AB % 16 != 0) return false;
    if (RB * BN >= (1L << 31) || AB * G::NTOK >= (1L << 31)) return false;  // 32-bit per-lane DMA offsets
    if (g.ldc_m > INT32_MAX || g.ldc_n > INT32_MAX) return false;
    return true;
}

template <int F, int BN, int TT, int W, int CB, bool SUMI> hipError_t mmqc_launch(const GemmArgs& g, hipStream_t st) {
    using G = mmqc_geom<F, BN, TT, W, CB>;
    const dim3 grid((g.N + BN - 1) / BN, (g.M + G::NTOK - 1) / G::NTOK);
    if (g.describe) {
        describe_kernel(g, "mmq F=%d BN=%d TT=%d W=%d FORM=chunked CB=%d R=%d NIW=%d EPI2=1 grid=%ux%u", F, BN, TT, W, CB, G::R,
                        G::NIW, grid.x, grid.y);
        return hipSuccess;
    }
    auto k = mmqc_kernel<F, BN, TT, W, CB, SUMI>;
    if (G::LDS > 64 * 1024) {
        static std::atomic<unsigned long long> attr_done{0};
        const hipError_t e = set_max_lds_once((const void*)k, 160 * 1024, attr_done);
        if (e != hipSuccess) return e;
    }
    void* o = SUMI ? (void*)g.sumi : (void*)g.C;
    hipLaunchKernelGGL(k, grid, dim3(W * 64), G::LDS, st, (const uint8_t*)g.A, (const uint8_t*)g.B, g.M, g.N, g.K, o,
                       (int)g.ldc_m, (int)g.ldc_n);
    return hipGetLastError();
}

}  // namespace qg
