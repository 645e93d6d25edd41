// qg_mmq_dispatch.hpp — tile configuration and dispatch of the prefill (M > 4) MFMA kernel
// (qg_mmq_kernel.hpp), instantiated once per weight format (qg_mmq_q*.hip) so the formats compile in
// parallel; qg_gemm_mfma.hip switches on the format.
//
// Tile configuration from the sweeps in profiles/tools_archive/mmq_probe.hip (profiles/r01_tuning/mmq_probe6.txt,
// mmq_probe_smallm.txt; cold weights, one MI355X):
//  * M <= 32: 16 tokens per workgroup, 8 waves splitting K; 32 weight rows when that still gives
//    >= 256 workgroups (one per CU; fewer re-reads of the activations), else 16
//    (M=32, N=4096: 32 rows x 2 token tiles = 256 WGs; M=8, N=4096: 16 rows = 256 WGs)
//  * M  > 32: 32 rows x 32 tokens; 8 waves splitting K while that grid has <= 256 workgroups, else
//    4 (two workgroups per CU under the kernel's register cap; mmq_probe_p4.txt, mmq_probe_mid.txt,
//    mmq_probe_lb.txt: M=64 10.1 us, M=128 15.2 us, M=512 47 us with the MFMA-assisted epilogue)
//  * round 4, measured and not adopted: the whole K of a 32 x 16 tile resident in LDS with every
//    operand byte requested at entry and a barrier per 32-block phase (profiles/tools_archive/
//    mmqr_resident_experiment.hpp; profiles/r04_tuning/ab_mmqr.txt: M = 32 6.91 -> 8.35 us, M = 24
//    6.72 -> 8.20, N = 11008 14.7 -> 21.3; parity green) — with everything in flight no phase completes
//    until most bytes have landed, so the compute no longer overlaps the ingest.
//  * round 4, measured and not adopted: a chunked, workgroup-cooperative ingest (576-B row segments
//    instead of 72 B, one barrier per 32-block chunk; profiles/tools_archive/mmqc_experiment.hpp,
//    profiles/r04_tuning/ab_mmqc_v1.txt: M = 32 6.91 -> 8.54 us, N = 11008 14.7 -> 22.3), early refill
//    of consumed stage buffers (ab_early.txt: M = 32 6.90 -> 7.14 us), raw fragment batches (ab_raw.txt),
//    dynamic stage hand-out (profiles/r02_tuning/ab_dyn.txt: M = 32 6.87 -> 7.25 us); their code is in
//    profiles/tools_archive/qg_mmq_kernel_r04_knobs.hpp.
// The same configurations serve every weight layout (LAY_ROWS, LAY_TILED) and the activation-window
// form (AW: odd K/32 against stage-padded weights).
#pragma once
#include "qg_mmql_kernel.hpp"

namespace qg {

namespace mmqd {
// The short-argument entry (mmq1_kernel) where measured faster: 16-row tiles (M <= 16: -0.08..-0.10
// us) and the 8-wave 32 x 32 tiles (M = 64 / 96: -0.2 us); the 32 x 16 8-wave tile (M = 32) and
// the 4-wave tiles keep the general entry (+0.05..+0.55 us with the short one; ab_sig3.txt).
template <int BN, int TT, int W> constexpr bool short_sig = (BN == 16 && W == 8) || (BN == 32 && TT == 2 && W == 8);
// Waves and stage slots per wave of the M <= 32, 32-row x 16-token tile when its grid is one dispatch
// round (<= 256 workgroups, one per CU): 12 waves with one stage each in flight beat 8 waves with two
// (profiles/r04_tuning/ab_waves_r4v.txt: M = 32 6.91 -> 6.50 us, M = 24 6.72 -> 6.12, Q4_1 7.00 -> 6.77,
// Q8_0 8.61 -> 8.43, M = 12 N = 8192 7.26 -> 6.98; more waves per SIMD overlap one wave's DMA wait with
// another's compute). Grids of several rounds keep 8 x 2 (N = 11008: 14.7 vs 15.6 us). Falls back to
// 8 x 2 where the rings would not fit the LDS.
// The same for the 16-row x 16-token tiles (M <= 16): 16 waves with one slot each where the grid is one
// round (profiles/r04_tuning/ab_waves_r4y.txt, N = K = 4096: Q4_0 M = 16 5.45 -> 5.28 us, M = 8
// 5.01 -> 4.82, M = 5 5.00 -> 4.77; Q4_1 M = 16 5.55 -> 5.36; Q5_0 M = 8 5.78 -> 5.34). Q8_0 keeps 8 x 2
// (M = 16 6.58 -> 7.15 with 16 waves: its 34-byte blocks double the per-stage ingest). The 8-wave
// 32 x 32 tiles (M > 32) keep 8 x 2: 12 or 16 waves exceed the VGPR budget of their accumulators
// (ab_waves_r4x.txt: M = 64 9.8 -> 24-55 us).
// The tiled layout's 32 x 16 tile (LAY_TILED): QG_MMQ_TILED_W waves x QG_MMQ_TILED_NB slots (a tuning
// choice only: every value computes the same bits — tests/test_gpu_tiled.py).
#ifndef QG_MMQ_TILED_W
#define QG_MMQ_TILED_W 12
#endif
#ifndef QG_MMQ_TILED_NB
#define QG_MMQ_TILED_NB 1
#endif
template <int F, int BN, int TT, int LAY>
constexpr int alt_w = BN == 32 && TT == 1 ? (LAY != LAY_ROWS ? QG_MMQ_TILED_W : 12) : BN == 16 ? (F != FMT_Q8_0 ? 16 : 8) : 8;
template <int F, int BN, int TT, int LAY>
constexpr int alt_nb = BN == 32 && TT == 1 ? (LAY != LAY_ROWS ? QG_MMQ_TILED_NB : 1) : BN == 16 ? (F != FMT_Q8_0 ? 1 : 2) : 2;

// grid of one dispatch round: at most one workgroup per CU (device_cus(): 256 on a whole MI355X)
inline bool one_round(const GemmArgs& g, int BN, int NTOK) {
    return (long)((g.N + BN - 1) / BN) * ((g.M + NTOK - 1) / NTOK) <= device_cus();
}

template <int F, int BN, int TT, int W, bool P16, int LAY, bool AW> hipError_t run_p(const GemmArgs& g, hipStream_t st) {
    constexpr bool S = short_sig<BN, TT, W> && LAY == LAY_ROWS && !AW;
    if constexpr (W == 8 && (alt_w<F, BN, TT, LAY> != 8 || alt_nb<F, BN, TT, LAY> != 2)) {
        constexpr int W2 = alt_w<F, BN, TT, LAY>, NB2 = alt_nb<F, BN, TT, LAY>;
        using G2 = mmq_geom<F, BN, TT, W2, P16, NB2, LAY, AW>;
        constexpr bool fits = (size_t)W2 * NB2 * G2::BUF <= 160 * 1024 && (size_t)W2 * G2::NACC * 256 <= 160 * 1024;
        if constexpr (fits) {
            if (one_round(g, BN, 16 * TT)) {
                if (g.sumi) return mmq_launch<F, BN, TT, W2, true, P16, NB2, LAY, AW, false>(g, st);
                return mmq_launch<F, BN, TT, W2, false, P16, NB2, LAY, AW, false>(g, st);
            }
        }
    }
    if (g.sumi) return mmq_launch<F, BN, TT, W, true, P16, 2, LAY, AW, S>(g, st);
    return mmq_launch<F, BN, TT, W, false, P16, 2, LAY, AW, S>(g, st);
}

// Variant of a tile configuration for the call's layout: LAY_ROWS with 16-B weight pieces when K % 256
// == 0 and B is 16-B aligned (else 4-B pieces), the activation-window form for the prepacked rows
// (g.nbw); LAY_TILED with or without activation windows.
template <int F, int BN, int TT, int W> int variant(const GemmArgs& g) {
    if (g.lay == LAY_TILED_ACT) return mmq_shape_ok<F, BN, TT, W, true, 2, LAY_TILED_ACT, false>(g) ? 6 : 0;
    if (g.lay == LAY_TILED) {
        if (mmq_shape_ok<F, BN, TT, W, true, 2, LAY_TILED, false>(g)) return 3;
        if (mmq_shape_ok<F, BN, TT, W, true, 2, LAY_TILED, true>(g)) return 4;
        return 0;
    }
    if (g.nbw > 0) return mmq_shape_ok<F, BN, TT, W, true, 2, LAY_ROWS, true>(g) ? 5 : 0;
    if (mmq_shape_ok<F, BN, TT, W, true>(g)) return 1;
    if (mmq_shape_ok<F, BN, TT, W, false>(g)) return 2;
    return 0;
}

// (a variant whose double-buffered rings exceed the LDS is never selected: mmq_shape_ok; nor compiled)
template <int F, int BN, int TT, int W, bool P16, int LAY, bool AW> hipError_t run_fit(const GemmArgs& g, hipStream_t st) {
    if constexpr (mmq_geom<F, BN, TT, W, P16, 2, LAY, AW>::FITS) return run_p<F, BN, TT, W, P16, LAY, AW>(g, st);
    return hipErrorInvalidValue;
}
template <int F, int BN, int TT, int W> hipError_t run_cfg(const GemmArgs& g, hipStream_t st) {
    switch (variant<F, BN, TT, W>(g)) {
        case 1: return run_fit<F, BN, TT, W, true, LAY_ROWS, false>(g, st);
        case 2: return run_fit<F, BN, TT, W, false, LAY_ROWS, false>(g, st);
        case 3: return run_fit<F, BN, TT, W, true, LAY_TILED, false>(g, st);
        case 4: return run_fit<F, BN, TT, W, true, LAY_TILED, true>(g, st);
        case 5: return run_fit<F, BN, TT, W, true, LAY_ROWS, true>(g, st);
        case 6: return run_fit<F, BN, TT, W, true, LAY_TILED_ACT, false>(g, st);
    }
    return hipErrorInvalidValue;
}

inline bool wide_rows(const GemmArgs& g) { return (long)((g.N + 31) / 32) * ((g.M + 15) / 16) >= device_cus(); }

// 8 waves per 32 x 32 tile only while that leaves <= 256 workgroups; beyond, 4-wave workgroups two
// per CU (profiles/r01_tuning/mmq_probe_mid.txt: M=96 16.5 -> 14.2 us, M=128 17.3 -> 15.5 us)
inline bool few_tiles(const GemmArgs& g) { return (long)((g.N + 31) / 32) * ((g.M + 31) / 32) <= device_cus(); }
}  // namespace mmqd

// Large M (qg_mmql_kernel.hpp): 64 rows x 64 tokens, 4 waves, two workgroups per CU, when that grid fills
// the CUs twice over (>= 2 device_cus() tiles; 64 x 128 tiles with 8 waves measured 2-9 % slower:
// profiles/r05_tuning/r5j_ab.txt, r5k_ab.txt); smaller grids keep the small tiles below. QG_MMQL=0 builds the round-4 dispatch
// (A/B variant builds only); QG_MMQL_NBUF: shared stage buffers (a tuning choice, same bits).
#ifndef QG_MMQL
#define QG_MMQL 1
#endif
#ifndef QG_MMQL_NBUF
#define QG_MMQL_NBUF 4
#endif
namespace mmqd {
template <int F, int WR, int WC> bool mmql_ok(const GemmArgs& g) {
    constexpr int NB = QG_MMQL_NBUF;
    if (!QG_MMQL) return false;
    // two workgroups per CU: at 1..1.5 per CU the small tiles are as fast or faster (r5l_ab.txt: M = 256
    // 30.8 vs 23.6 us, M = 384 33.3 vs 33.3; M = 512 35.7 vs 43.1, M = 1024 67.6 vs 82.2)
    if ((long)((g.N + 32 * WR - 1) / (32 * WR)) * ((g.M + 32 * WC - 1) / (32 * WC)) < 2L * device_cus()) return false;
    if (g.lay == LAY_TILED_ACT) return mmql_shape_ok<F, LAY_TILED_ACT, WR, WC, NB>(g);
    return g.lay == LAY_TILED ? mmql_shape_ok<F, LAY_TILED, WR, WC, NB>(g) : mmql_shape_ok<F, LAY_ROWS, WR, WC, NB>(g);
}
template <int F, int WR, int WC> hipError_t mmql_run(const GemmArgs& g, hipStream_t st) {
    constexpr int NB = QG_MMQL_NBUF;
    if (g.lay == LAY_TILED_ACT)
        return g.sumi ? mmql_launch<F, LAY_TILED_ACT, WR, WC, NB, true>(g, st) : mmql_launch<F, LAY_TILED_ACT, WR, WC, NB, false>(g, st);
    if (g.lay == LAY_TILED)
        return g.sumi ? mmql_launch<F, LAY_TILED, WR, WC, NB, true>(g, st) : mmql_launch<F, LAY_TILED, WR, WC, NB, false>(g, st);
    return g.sumi ? mmql_launch<F, LAY_ROWS, WR, WC, NB, true>(g, st) : mmql_launch<F, LAY_ROWS, WR, WC, NB, false>(g, st);
}
}  // namespace mmqd

// The configuration for the shape (above), or the 4-wave 32 x 32 tile where the preferred 8-wave one does
// not fit the LDS with this layout (Q8_0 with activation windows).
template <int F> int config(const GemmArgs& g) {
    using namespace mmqd;
    if (g.M > 32 && mmql_ok<F, 2, 2>(g)) return 5;
    if (g.M <= 32) return wide_rows(g) ? (variant<F, 32, 1, 8>(g) ? 1 : 0) : (variant<F, 16, 1, 8>(g) ? 2 : 0);
    if (few_tiles(g) && variant<F, 32, 2, 8>(g)) return 3;
    return variant<F, 32, 2, 4>(g) ? 4 : 0;
}

template <int F> bool mfma_eligible_f(const GemmArgs& g) { return config<F>(g) != 0; }

template <int F> hipError_t launch_mfma_f(const GemmArgs& g, hipStream_t st) {
    using namespace mmqd;
    switch (config<F>(g)) {
        case 1: return run_cfg<F, 32, 1, 8>(g, st);
        case 2: return run_cfg<F, 16, 1, 8>(g, st);
        case 3: return run_cfg<F, 32, 2, 8>(g, st);
        case 4: return run_cfg<F, 32, 2, 4>(g, st);
        case 5: return mmql_run<F, 2, 2>(g, st);
    }
    return hipErrorInvalidValue;
}

#define QG_MMQ_INSTANTIATE(F)                                                   \
    template bool mfma_eligible_f<F>(const GemmArgs& g);                        \
    template hipError_t launch_mfma_f<F>(const GemmArgs& g, hipStream_t st);

}  // namespace qg
