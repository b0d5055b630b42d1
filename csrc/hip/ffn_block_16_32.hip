// Fused FFN block instance: w13 lanes 16, w2 lanes 32 (ffn_block_inst.h).
#include "ffn_block_inst.h"

namespace dl {
namespace hipk {
const void *ffnBlockFn_16_32(bool tp) { return ffnBlockFnT<16, 32>(tp); }
}  // namespace hipk
}  // namespace dl
