// qg_mmq_q5_0.hip — the prefill MFMA kernel's instantiations for q5_0 weights (qg_mmq_dispatch.hpp).
#include "qg_mmq_dispatch.hpp"

namespace qg {
QG_MMQ_INSTANTIATE(FMT_Q5_0)
}  // namespace qg
