// Fused attention block instances: qkv 32 lanes per row, wo 64, head size 128 (attn_block_inst.h).
#include "attn_block_inst.h"

namespace dl {
namespace hipk {
const void *attnBlockFn_32_64_128(int hg, bool bf16, int md) { return attnBlockFnT<32, 64, 128>(hg, bf16, md); }
}  // namespace hipk
}  // namespace dl
