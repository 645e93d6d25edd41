// qg_gemv_impl.hpp — the GEMV dispatch templates (configuration per shape), instantiated once per
// weight format in qg_gemv_<fmt>.hip so the formats compile in parallel; qg_gemv.hip holds the
// format switch (gemv_eligible, launch_gemv).
#pragma once
#include "qg_gemv_kernel.hpp"

// Workgroup size of the M = 1 loop-free GEMV (tuning knob for A/B builds; 1024 = product).
#ifndef QG_GEMV1_WGS
#define QG_GEMV1_WGS 1024
#endif
// tuning knobs (A/B builds): M = 2..4 workgroup size (0: per format, below); M = 1, N >= 16384
// workgroup size
#ifndef QG_GEMVM_WGS
#define QG_GEMVM_WGS 0
#endif
#ifndef QG_GEMV1L_WGS
#define QG_GEMV1L_WGS 0  // M = 1 with the unit loop (K > 4096); 0: per format, below
#endif
#ifndef QG_GEMV_SMALLK
#define QG_GEMV_SMALLK 1  // K < 4096 shapes on 16-row workgroups (0: the round-2 64-row form, A/B builds)
#endif
#ifndef QG_GEMVM_LPR
#define QG_GEMVM_LPR 64
#endif
#ifndef QG_GEMVBIG_WGS
#define QG_GEMVBIG_WGS 512
#endif

namespace qg {

// M = 2..4: 512-thread workgroups for the byte-decode formats (profiles/r03_tuning/r03_ab_m512.txt:
// Q5_0 M=2 4.41 -> 4.29 us, Q5_1 M=4 5.99 -> 5.75, Q8_0 M=4 5.87 -> 5.62), 1024 for the nibble-plane
// ones (Q4_1 M=2 3.78 -> 4.01 at 512; Q4_0 M=2 -0.06 but M=4 +0.02)
template <int F>
constexpr int gemvm_wgs = QG_GEMVM_WGS ? QG_GEMVM_WGS : (F == FMT_Q5_0 || F == FMT_Q5_1 || F == FMT_Q8_0) ? 512 : 1024;
// M = 1, K > 4096 (the unit loop): 512 for Q8_0 (r03_ab_l512.txt: K=11008 10.60 -> 9.72 us, K=14336
// 12.64 -> 12.36), 1024 for the rest (Q4_0 / Q4_1 +3 %, Q5_x equal at 512)
template <int F> constexpr int gemv1l_wgs = QG_GEMV1L_WGS ? QG_GEMV1L_WGS : F == FMT_Q8_0 ? 512 : 1024;

template <int F, int MT, bool SUMI, int AIN>
hipError_t launch_staged(const GemmArgs& g, hipStream_t st) {
    const int nb = g.K / QK;
    // 2-block units, one row per wave, 1024-thread workgroups (512 for a single row of activations
    // over N >= 16384 rows): profiles/r01_tuning/gemv_probe_focus.txt, gemv_probe_focus2.txt —
    // M=1 Q4_0 3.67 -> 3.60 us, Q5_0 / Q5_1 -6 %, M=2 -4 %, M=4 -11 % against 4-block units x 32
    // lanes x 512 threads; gemv_probe_v2b.txt: N=32000 -3.4 %, K=14336 -3.8 %
    // (a strided batch uses the same shape, so its outputs equal the single launches' bit for bit;
    // the fused-quantization prologue is repeated per workgroup, so it keeps 16 rows per workgroup,
    // with the same per-row summation order)
    if constexpr (MT <= 4) {
        if (nb % 2 == 0 && nb / 2 >= 64) {
            if (MT == 1 && AIN == AIN_Q8_1 && g.N >= 16384 && g.K < 8192)
                return gemv_launch<F, 1, 2, 64, QG_GEMVBIG_WGS, SUMI, AIN>(g, st);
            // activation records preloaded into registers for M <= 4 (profiles/tools_archive/gemv_pre_probe.hip,
            // profiles/r01_tuning/gemv_pre_probe.txt: M=3 4.76 -> 4.52 us, M=4 5.16 -> 5.04 us)
            // Q5_0 / Q5_1: 512-thread workgroups (profiles/r03_tuning/r03_ab_wgs.txt: M=1 3.82 -> 3.78 /
            // 3.93 -> 3.88 us; Q4_0 / Q8_0 are faster at 1024, Q4_1 equal)
            constexpr int W1 = (F == FMT_Q5_0 || F == FMT_Q5_1) ? 512 : QG_GEMV1_WGS;
            if constexpr (MT == 1) if (nb / 2 <= 64) return gemv_launch<F, MT, 2, 64, W1, SUMI, AIN, false, true>(g, st);
#if QG_GEMVM_LPR != 64  // (A/B builds) M >= 2: fewer lanes per row, the same rows per workgroup
            if constexpr (MT >= 2)
                return gemv_launch<F, MT, 2, QG_GEMVM_LPR, gemvm_wgs<F> * QG_GEMVM_LPR / 64, SUMI, AIN, false, true>(g, st);
#endif
            return gemv_launch<F, MT, 2, 64, MT == 1 ? gemv1l_wgs<F> : gemvm_wgs<F>, SUMI, AIN, false, true>(g, st);
        }
    }
    if constexpr (QG_GEMV_SMALLK && MT <= 4) {
        // K < 4096: 2-block units, 32 / 16 lanes per row, 16 rows per workgroup (256 workgroups at
        // N = 4096) instead of 64-row workgroups of 4-lane rows
        if (nb % 2 == 0 && nb / 2 >= 32) return gemv_launch<F, MT, 2, 32, 512, SUMI, AIN, false, true>(g, st);
        if (nb % 2 == 0 && nb / 2 >= 16) return gemv_launch<F, MT, 2, 16, 256, SUMI, AIN, false, true>(g, st);
    }
    if (nb % 4 == 0) {
        if (nb / 4 >= 32) return gemv_launch<F, MT, 4, 32, 512, SUMI, AIN>(g, st);
        return gemv_launch<F, MT, 4, 4, 256, SUMI, AIN>(g, st);
    }
    return gemv_launch<F, MT, 2, 8, 256, SUMI, AIN>(g, st);
}

// The sumi parity hook (SUMI = true) runs the very instantiation the product dispatch picks for
// this shape — same MT, unit size, lanes per row, workgroup size, PRE and loop-free form — and only
// replaces the final accumulate by a store of each block's int32 dot.
template <int F, bool SUMI, int AIN> hipError_t launch_m(const GemmArgs& g, hipStream_t st) {
    if (g.M <= 1) return launch_staged<F, 1, SUMI, AIN>(g, st);
    if (g.M <= 2) return launch_staged<F, 2, SUMI, AIN>(g, st);
    if (g.M <= 4) return launch_staged<F, 4, SUMI, AIN>(g, st);
    return launch_staged<F, 8, SUMI, AIN>(g, st);
}

template <int F> hipError_t launch_f(const GemmArgs& g, hipStream_t st) {
    if (g.sumi) return launch_m<F, true, AIN_Q8_1>(g, st);
    if (g.ain == AIN_F32) return launch_m<F, false, AIN_F32>(g, st);
    if (g.ain == AIN_F16_FUSED) return launch_m<F, false, AIN_F16_FUSED>(g, st);
    return launch_m<F, false, AIN_Q8_1>(g, st);
}

template <int F> bool ok_f(const GemmArgs& g) {
    return (g.K / QK) % 4 == 0 ? gemv_shape_ok<F, 4>(g) : gemv_shape_ok<F, 2>(g);
}

// one explicit specialization per format (qg_gemv_<fmt>.hip)
template <int F> hipError_t gemv_launch_fmt(const GemmArgs& g, hipStream_t st);
template <> hipError_t gemv_launch_fmt<FMT_Q4_0>(const GemmArgs& g, hipStream_t st);
template <> hipError_t gemv_launch_fmt<FMT_Q4_1>(const GemmArgs& g, hipStream_t st);
template <> hipError_t gemv_launch_fmt<FMT_Q5_0>(const GemmArgs& g, hipStream_t st);
template <> hipError_t gemv_launch_fmt<FMT_Q5_1>(const GemmArgs& g, hipStream_t st);
template <> hipError_t gemv_launch_fmt<FMT_Q8_0>(const GemmArgs& g, hipStream_t st);

}  // namespace qg
