// qg_gemm_mfma.hip — prefill path (M > 8). Placeholder until the MFMA kernel lands.
#include "qg_common.hpp"
#include "qg_kernels.hpp"

namespace qg {
bool mfma_eligible(const GemmArgs&) { return false; }
hipError_t launch_mfma(const GemmArgs&, hipStream_t) { return hipErrorInvalidValue; }
}  // namespace qg
