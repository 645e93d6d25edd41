// qg_mmq_q4_0.hip — the prefill MFMA kernel's instantiations for q4_0 weights (qg_mmq_dispatch.hpp).
#include "qg_mmq_dispatch.hpp"

namespace qg {
QG_MMQ_INSTANTIATE(FMT_Q4_0)
}  // namespace qg
