// qg_gemm_mfma.hip — product instantiations and dispatch of the prefill (M > 8) MFMA kernel
// (qg_mmq_kernel.hpp).
//
// Tile configuration from the sweeps in tools/archive/mmq_probe.hip (profiles/r01_tuning/mmq_probe6.txt,
// mmq_probe_smallm.txt; cold weights, one MI355X):
//  * M <= 32: 16 tokens per workgroup, 8 waves splitting K; 32 weight rows when that still gives
//    >= 256 workgroups (one per CU; fewer re-reads of the activations), else 16
//    (M=32, N=4096: 32 rows x 2 token tiles = 256 WGs; M=8, N=4096: 16 rows = 256 WGs)
//  * M  > 32: 32 rows x 32 tokens; 8 waves splitting K while that grid has <= 256 workgroups, else
//    4 (two workgroups per CU under the kernel's register cap; mmq_probe_p4.txt, mmq_probe_mid.txt,
//    mmq_probe_lb.txt: M=64 10.1 us, M=128 15.2 us, M=512 47 us with the MFMA-assisted epilogue)
//  * round 4, measured and not adopted: the whole K of a 32 x 16 tile resident in LDS with every
//    operand byte requested at entry and a barrier per 32-block phase (tools/archive/
//    mmqr_resident_experiment.hpp; profiles/r04_tuning/ab_mmqr.txt: M = 32 6.91 -> 8.35 us, M = 24
//    6.72 -> 8.20, N = 11008 14.7 -> 21.3; parity green) — with everything in flight no phase completes
//    until most bytes have landed, so the compute no longer overlaps the ingest.
//  * round 4, measured and not adopted: a chunked, workgroup-cooperative ingest (576-B row segments
//    instead of 72 B, one barrier per 32-block chunk; tools/archive/mmqc_experiment.hpp,
//    profiles/r04_tuning/ab_mmqc_v1.txt: M = 32 6.91 -> 8.54 us, N = 11008 14.7 -> 22.3). Its per-wave
//    timeline (mmqc_probe_v1.txt) shows why: the coalesced chunks all land together ~2.8 us after entry
//    (DMA + barriers alone 5.3 us per launch), and the lockstep compute then costs ~0.9-1.0 us per chunk
//    (the LDS reads, 16-cycle MFMAs and epilogue of 8 waves serialise), 4 chunks after the data.
#include "qg_mmq_kernel.hpp"

namespace qg {

namespace {
// 16-B weight DMA pieces when K % 256 == 0 and B is 16-B aligned, else 4-B pieces.
template <int F, int BN, int TT, int W> bool ok_cfg(const GemmArgs& g) {
    return mmq_shape_ok<F, BN, TT, W, true>(g) || mmq_shape_ok<F, BN, TT, W, false>(g);
}

// The MFMA-assisted epilogue (EPI2, qg_mmq_kernel.hpp) in every configuration:
// profiles/r01_tuning/mmq_probe_epi2.txt, mmq_probe_disp.txt, mmq_probe_lb.txt — M=8 5.56 -> 5.44
// us, M=32 7.61 -> 7.39, M=64 10.35 -> 10.19, M=256 29.2 -> 27.1, M=512 58.3 -> 50.9, M=1024
// 108.9 -> 96.5 (the 4-wave 32 x 32 tiles with the two-workgroups-per-CU register cap)
// The sumi parity hook runs the same instantiation with SUMI = true (the EPI2 form's own operand
// fragments and MFMAs; only the final accumulate becomes a store of each block's int32 dot).
// The short-argument entry (mmq1_kernel) where measured faster: 16-row tiles (M <= 16: -0.08..-0.10
// us) and the 8-wave 32 x 32 tiles (M = 64 / 96: -0.2 us); the 32 x 16 8-wave tile (M = 32) and
// the 4-wave tiles keep the general entry (+0.05..+0.55 us with the short one; ab_sig3.txt).
template <int BN, int TT, int W> constexpr bool short_sig = (BN == 16 && W == 8) || (BN == 32 && TT == 2 && W == 8);
// Dynamic stage hand-out (MMQ_DYN, qg_mmq_kernel.hpp) for the 32-row x 16-token 8-wave tiles: a
// tuning option, off in the product — measured slower (profiles/r02_tuning/ab_dyn.txt: M=32 6.87 ->
// 7.25 us, N=11008 14.6 -> 18.8 us: the per-stage partial slots take the LDS to 144 KB, one
// workgroup per CU, and the stage-order sum adds a tail; the waves' spread is not intra-workgroup).
#ifndef QG_MMQ_DYN
#define QG_MMQ_DYN 0
#endif
// Early refill of consumed stage buffers (MMQ_EARLY, qg_mmq_kernel.hpp): A/B knob, off — measured
// slower at the prefill sizes that matter (profiles/r04_tuning/ab_early.txt: M = 32 6.90 -> 7.14 us,
// M = 16 5.47 -> 5.54, N = 11008 14.55 -> 14.90, M = 64 9.69 -> 9.92; M = 8 -0.1 us, M = 512 -0.45);
// the refill must wait for the stage's LDS reads (lgkmcnt(0)), which takes the overlap away. Its first
// form, without that wait, was non-deterministic (profiles/r04_tuning/r04g_gpu_suite_fail_early_unwaited.txt).
#ifndef QG_MMQ_EARLY
#define QG_MMQ_EARLY 0
#endif
// Raw weight-fragment reads in one batch per stage (MMQ_RAW): A/B knob
#ifndef QG_MMQ_RAW
#define QG_MMQ_RAW 0
#endif
// Waves and stage slots per wave of the M <= 32, 32-row x 16-token tile when its grid is one dispatch
// round (<= 256 workgroups, one per CU): 12 waves with one stage each in flight beat 8 waves with two
// (profiles/r04_tuning/ab_waves_r4v.txt: M = 32 6.91 -> 6.50 us, M = 24 6.72 -> 6.12, Q4_1 7.00 -> 6.77,
// Q8_0 8.61 -> 8.43, M = 12 N = 8192 7.26 -> 6.98; more waves per SIMD overlap one wave's DMA wait with
// another's compute). Grids of several rounds keep 8 x 2 (N = 11008: 14.7 vs 15.6 us). Falls back to
// 8 x 2 where the rings would not fit the LDS.
#ifndef QG_MMQ_SMALL_W
#define QG_MMQ_SMALL_W 12
#endif
#ifndef QG_MMQ_SMALL_NB
#define QG_MMQ_SMALL_NB 1
#endif
// The same for the 16-row x 16-token tiles (M <= 16): 16 waves with one slot each where the grid is one
// round (profiles/r04_tuning/ab_waves_r4y.txt, N = K = 4096: Q4_0 M = 16 5.45 -> 5.28 us, M = 8
// 5.01 -> 4.82, M = 5 5.00 -> 4.77; Q4_1 M = 16 5.55 -> 5.36; Q5_0 M = 8 5.78 -> 5.34). Q8_0 keeps 8 x 2
// (M = 16 6.58 -> 7.15 with 16 waves: its 34-byte blocks double the per-stage ingest). The 8-wave
// 32 x 32 tiles (M > 32) keep 8 x 2: 12 or 16 waves exceed the VGPR budget of their accumulators
// (ab_waves_r4x.txt: M = 64 9.8 -> 24-55 us).
#ifndef QG_MMQ_S16_W
#define QG_MMQ_S16_W 16
#endif
#ifndef QG_MMQ_S16_NB
#define QG_MMQ_S16_NB 1
#endif
#ifndef QG_MMQ_L_W
#define QG_MMQ_L_W 8
#endif
#ifndef QG_MMQ_L_NB
#define QG_MMQ_L_NB 2
#endif
template <int F, int BN, int TT> constexpr bool alt_s16 = BN == 16 && F != FMT_Q8_0;
template <int F, int BN, int TT>
constexpr int alt_w = BN == 32 && TT == 1 ? QG_MMQ_SMALL_W : BN == 16 ? (alt_s16<F, BN, TT> ? QG_MMQ_S16_W : 8) : QG_MMQ_L_W;
template <int F, int BN, int TT>
constexpr int alt_nb = BN == 32 && TT == 1 ? QG_MMQ_SMALL_NB : BN == 16 ? (alt_s16<F, BN, TT> ? QG_MMQ_S16_NB : 2) : QG_MMQ_L_NB;
template <int F, int BN, int TT, int W, bool P16> hipError_t run_p(const GemmArgs& g, hipStream_t st) {
    constexpr bool S = short_sig<BN, TT, W>;
    if constexpr (W == 8 && (alt_w<F, BN, TT> != 8 || alt_nb<F, BN, TT> != 2)) {
        constexpr int W2 = alt_w<F, BN, TT>, NB2 = alt_nb<F, BN, TT>;
        constexpr bool fits = (size_t)W2 * NB2 * mmq_geom<F, BN, TT, W2, P16, NB2, 4>::BUF <= 160 * 1024 &&
                              (size_t)W2 * BN / 16 * TT * 4 * 256 <= 160 * 1024;
        if constexpr (fits) {
            if ((long)((g.N + BN - 1) / BN) * ((g.M + 16 * TT - 1) / (16 * TT)) <= 256) {
                if (g.sumi) return mmq_launch<F, BN, TT, W2, true, P16, NB2, 0, false, 4, 1, true, 0, false>(g, st);
                return mmq_launch<F, BN, TT, W2, false, P16, NB2, 0, false, 4, 1, true, 0, false>(g, st);
            }
        }
    }
    constexpr int E = (QG_MMQ_EARLY ? MMQ_EARLY : 0) | (QG_MMQ_RAW ? MMQ_RAW : 0);
    if constexpr (QG_MMQ_DYN && BN == 32 && TT == 1 && W == 8) {
        if (mmq_geom<F, BN, TT, W, P16, 2, 4, MMQ_DYN>::dyn_lds(g.K / QK / 4) <= 160 * 1024) {
            if (g.sumi) return mmq_launch<F, BN, TT, W, true, P16, 2, 0, false, 4, 1, true, MMQ_DYN, S>(g, st);
            return mmq_launch<F, BN, TT, W, false, P16, 2, 0, false, 4, 1, true, MMQ_DYN, S>(g, st);
        }
    }
    if (g.sumi) return mmq_launch<F, BN, TT, W, true, P16, 2, 0, false, 4, 1, true, E, S>(g, st);
    return mmq_launch<F, BN, TT, W, false, P16, 2, 0, false, 4, 1, true, E, S>(g, st);
}

template <int F, int BN, int TT, int W> hipError_t run_cfg(const GemmArgs& g, hipStream_t st) {
    return mmq_shape_ok<F, BN, TT, W, true>(g) ? run_p<F, BN, TT, W, true>(g, st) : run_p<F, BN, TT, W, false>(g, st);
}

inline bool wide_rows(const GemmArgs& g) { return (long)((g.N + 31) / 32) * ((g.M + 15) / 16) >= 256; }

// 8 waves per 32 x 32 tile only while that leaves <= 256 workgroups; beyond, 4-wave workgroups two
// per CU (profiles/r01_tuning/mmq_probe_mid.txt: M=96 16.5 -> 14.2 us, M=128 17.3 -> 15.5 us)
inline bool few_tiles(const GemmArgs& g) { return (long)((g.N + 31) / 32) * ((g.M + 31) / 32) <= 256; }

template <int F> bool ok_f(const GemmArgs& g) {
    if (g.M <= 32) return wide_rows(g) ? ok_cfg<F, 32, 1, 8>(g) : ok_cfg<F, 16, 1, 8>(g);
    return few_tiles(g) ? ok_cfg<F, 32, 2, 8>(g) : ok_cfg<F, 32, 2, 4>(g);
}

template <int F> hipError_t launch_f(const GemmArgs& g, hipStream_t st) {
    if (g.M <= 32) return wide_rows(g) ? run_cfg<F, 32, 1, 8>(g, st) : run_cfg<F, 16, 1, 8>(g, st);
    return few_tiles(g) ? run_cfg<F, 32, 2, 8>(g, st) : run_cfg<F, 32, 2, 4>(g, st);
}
}  // namespace

bool mfma_eligible(const GemmArgs& g) {
    if (g.M < 1 || g.N < 1 || (g.M + 15) / 16 > 65535) return false;
    switch (g.wtype) {
        case FMT_Q4_0: return ok_f<FMT_Q4_0>(g);
        case FMT_Q4_1: return ok_f<FMT_Q4_1>(g);
        case FMT_Q5_0: return ok_f<FMT_Q5_0>(g);
        case FMT_Q5_1: return ok_f<FMT_Q5_1>(g);
        case FMT_Q8_0: return ok_f<FMT_Q8_0>(g);
    }
    return false;
}

hipError_t launch_mfma(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return launch_f<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return launch_f<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return launch_f<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return launch_f<FMT_Q5_1>(g, st);
        case FMT_Q8_0: return launch_f<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
