// qg_gemv.hip — product instantiations and dispatch of the GEMV kernel (qg_gemv_kernel.hpp).
//
// Configuration from the tuning sweep (tools/gemv_probe.hip, profiles/r01_gemv_probe.txt): at
// K = 4096 the 4-block unit (72 B = 9 x dwordx2 per lane), 32 lanes per row, 512-thread workgroups
// and plain (not nt) loads were fastest cold and hot; nt loads cost 1.5-2.5x on this stream.
#include "qg_gemv_kernel.hpp"

namespace qg {

namespace {
template <int F, int MT, bool SUMI>
hipError_t launch_cfg(const GemmArgs& g, hipStream_t st) {
    const int nb = g.K / QK;
    if (nb % 4 == 0) {
        if (nb / 4 >= 32) return gemv_launch<F, MT, 4, 32, 512, 4 * MT, false, SUMI>(g, st);
        return gemv_launch<F, MT, 4, 4, 256, 8 * MT, false, SUMI>(g, st);
    }
    return gemv_launch<F, MT, 2, 8, 256, 8 * MT, false, SUMI>(g, st);
}

template <int F> hipError_t launch_f(const GemmArgs& g, hipStream_t st) {
    if (g.sumi) return launch_cfg<F, 8, true>(g, st);
    if (g.M <= 1) return launch_cfg<F, 1, false>(g, st);
    if (g.M <= 2) return launch_cfg<F, 2, false>(g, st);
    if (g.M <= 4) return launch_cfg<F, 4, false>(g, st);
    return launch_cfg<F, 8, false>(g, st);
}

template <int F> bool ok_f(const GemmArgs& g) {
    return (g.K / QK) % 4 == 0 ? gemv_shape_ok<F, 4>(g) : gemv_shape_ok<F, 2>(g);
}
}  // namespace

bool gemv_eligible(const GemmArgs& g) {
    switch (g.wtype) {
        case FMT_Q4_0: return ok_f<FMT_Q4_0>(g);
        case FMT_Q4_1: return ok_f<FMT_Q4_1>(g);
        case FMT_Q5_0: return ok_f<FMT_Q5_0>(g);
        case FMT_Q5_1: return ok_f<FMT_Q5_1>(g);
    }
    return false;
}

hipError_t launch_gemv(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return launch_f<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return launch_f<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return launch_f<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return launch_f<FMT_Q5_1>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
