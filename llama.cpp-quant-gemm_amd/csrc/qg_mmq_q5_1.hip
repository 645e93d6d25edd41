// qg_mmq_q5_1.hip — the prefill MFMA kernel's instantiations for q5_1 weights (qg_mmq_dispatch.hpp).
#include "qg_mmq_dispatch.hpp"

namespace qg {
QG_MMQ_INSTANTIATE(FMT_Q5_1)
}  // namespace qg
