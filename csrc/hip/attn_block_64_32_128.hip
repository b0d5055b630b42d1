// Fused attention block instances: qkv 64 lanes per row, wo 32, head size 128 (attn_block_inst.h).
#include "attn_block_inst.h"

namespace dl {
namespace hipk {
const void *attnBlockFn_64_32_128(int hg, bool bf16, int md) { return attnBlockFnT<64, 32, 128>(hg, bf16, md); }
}  // namespace hipk
}  // namespace dl
