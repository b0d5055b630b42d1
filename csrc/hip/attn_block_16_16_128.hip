// Fused attention block instances: qkv 16 lanes per row, wo 16 (70B / 405B widths), head size 128 (attn_block_inst.h).
#include "attn_block_inst.h"

namespace dl {
namespace hipk {
const void *attnBlockFn_16_16_128(int hg, bool bf16, int md) { return attnBlockFnT<16, 16, 128>(hg, bf16, md); }
}  // namespace hipk
}  // namespace dl
