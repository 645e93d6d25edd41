// qg_mmq_q8_0.hip — the prefill MFMA kernel's instantiations for q8_0 weights (qg_mmq_dispatch.hpp).
#include "qg_mmq_dispatch.hpp"

namespace qg {
QG_MMQ_INSTANTIATE(FMT_Q8_0)
}  // namespace qg
