// qg_gemv.hip — product instantiations and dispatch of the GEMV kernels (qg_gemv_kernel.hpp).
//
// Configuration from the tuning sweeps (profiles/tools_archive/gemv_probe.hip, profiles/r01_tuning/): M <= 4 with
// K >= 4096: 2-block units, 64 lanes (one wave) per row, 1024-thread workgroups (512 for M = 1 and
// N >= 16384); otherwise 4-block units (72 B for Q4_0), 32 lanes per row, 512-thread workgroups;
// short rows (K/32/4 < 32) 4 lanes per row; K/32 not a multiple of 4: 2-block units.
// The fused-quantization variants (AIN_F32 / AIN_F16_FUSED) share the configuration.
#include "qg_gemv_impl.hpp"

namespace qg {

bool gemv_eligible(const GemmArgs& g) {
    switch (g.wtype) {
        case FMT_Q4_0: return ok_f<FMT_Q4_0>(g);
        case FMT_Q4_1: return ok_f<FMT_Q4_1>(g);
        case FMT_Q5_0: return ok_f<FMT_Q5_0>(g);
        case FMT_Q5_1: return ok_f<FMT_Q5_1>(g);
        case FMT_Q8_0: return ok_f<FMT_Q8_0>(g);
    }
    return false;
}

hipError_t launch_gemv(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case FMT_Q4_0: return gemv_launch_fmt<FMT_Q4_0>(g, st);
        case FMT_Q4_1: return gemv_launch_fmt<FMT_Q4_1>(g, st);
        case FMT_Q5_0: return gemv_launch_fmt<FMT_Q5_0>(g, st);
        case FMT_Q5_1: return gemv_launch_fmt<FMT_Q5_1>(g, st);
        case FMT_Q8_0: return gemv_launch_fmt<FMT_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
