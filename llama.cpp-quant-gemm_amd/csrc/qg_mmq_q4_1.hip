// qg_mmq_q4_1.hip — the prefill MFMA kernel's instantiations for q4_1 weights (qg_mmq_dispatch.hpp).
#include "qg_mmq_dispatch.hpp"

namespace qg {
QG_MMQ_INSTANTIATE(FMT_Q4_1)
}  // namespace qg
