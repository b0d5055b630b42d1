// GEMV kernel instances with 64 lanes per weight row (see gemv_inst.h).
#include "gemv_inst.h"

namespace dl {
namespace hipk {
const void *gemvFnL64(bool q40, int B, int pro, int epi) {
    return q40 ? gemvFnB<64, true>(B, pro, epi) : gemvFnB<64, false>(B, pro, epi);
}
const void *gemvAttnFnL64(int epi, int hg, bool bf16) { return gemvAttnFnL<64>(epi, hg, bf16); }
}  // namespace hipk
}  // namespace dl
