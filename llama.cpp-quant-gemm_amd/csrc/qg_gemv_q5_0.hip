// qg_gemv_q5_0.hip — the GEMV kernels for Q5_0 weights (qg_gemv_impl.hpp); one translation unit per
// weight format so the product library's largest template set compiles in parallel.
#include "qg_gemv_impl.hpp"

namespace qg {
template <> hipError_t gemv_launch_fmt<FMT_Q5_0>(const GemmArgs& g, hipStream_t st) { return launch_f<FMT_Q5_0>(g, st); }
}  // namespace qg
