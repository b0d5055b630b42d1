// GEMV kernel instances with 16 lanes per weight row (see gemv_inst.h).
#include "gemv_inst.h"

namespace dl {
namespace hipk {
const void *gemvFnL16(bool q40, int B, int pro, int epi) {
    return q40 ? gemvFnB<16, true>(B, pro, epi) : gemvFnB<16, false>(B, pro, epi);
}
const void *gemvAttnFnL16(int epi, int hg, bool bf16) { return gemvAttnFnL<16>(epi, hg, bf16); }
}  // namespace hipk
}  // namespace dl
