// GEMV kernel instances with 32 lanes per weight row (see gemv_inst.h).
#include "gemv_inst.h"

namespace dl {
namespace hipk {
const void *gemvFnL32(bool q40, int B, int pro, int epi) {
    return q40 ? gemvFnB<32, true>(B, pro, epi) : gemvFnB<32, false>(B, pro, epi);
}
const void *gemvAttnFnL32(int epi, int hg, bool bf16) { return gemvAttnFnL<32>(epi, hg, bf16); }
}  // namespace hipk
}  // namespace dl
