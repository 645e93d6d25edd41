// qg_gemm_mfma.hip — format switch of the prefill (M > 4) MFMA kernel; the tile configurations and
// their instantiations are in qg_mmq_dispatch.hpp / qg_mmq_q*.hip (one translation unit per format).
#include "qg_kernels.hpp"

namespace qg {

template <int F> bool mfma_eligible_f(const GemmArgs& g);
template <int F> hipError_t launch_mfma_f(const GemmArgs& g, hipStream_t st);
enum : int { F_Q4_0 = 2, F_Q4_1 = 3, F_Q5_0 = 6, F_Q5_1 = 7, F_Q8_0 = 8 };  // ggml_type ids (qg_common.hpp)

bool mfma_eligible(const GemmArgs& g) {
    if (g.M < 1 || g.N < 1 || (g.M + 15) / 16 > 65535) return false;
    switch (g.wtype) {
        case F_Q4_0: return mfma_eligible_f<F_Q4_0>(g);
        case F_Q4_1: return mfma_eligible_f<F_Q4_1>(g);
        case F_Q5_0: return mfma_eligible_f<F_Q5_0>(g);
        case F_Q5_1: return mfma_eligible_f<F_Q5_1>(g);
        case F_Q8_0: return mfma_eligible_f<F_Q8_0>(g);
    }
    return false;
}

hipError_t launch_mfma(const GemmArgs& g, hipStream_t st) {
    switch (g.wtype) {
        case F_Q4_0: return launch_mfma_f<F_Q4_0>(g, st);
        case F_Q4_1: return launch_mfma_f<F_Q4_1>(g, st);
        case F_Q5_0: return launch_mfma_f<F_Q5_0>(g, st);
        case F_Q5_1: return launch_mfma_f<F_Q5_1>(g, st);
        case F_Q8_0: return launch_mfma_f<F_Q8_0>(g, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace qg
