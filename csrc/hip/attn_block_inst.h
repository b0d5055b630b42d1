// Fused attention block kernel template (see kernels.h AttnBlockArgs): roles by workgroup index.
// Instances are compiled per (qkv lanes, wo lanes, head size) in attn_block_*.hip (parallel builds).
#pragma once
#include "decode_dev.h"

namespace dl {
namespace hipk {

template <int LQ, int LW, int HG, int HS, bool BF16, bool TP>
__global__ __launch_bounds__(kThreads) void attnBlockKernel(AttnBlockArgs ba) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nHG = ba.at.nHeads0 / HG;
    const int gq = (ba.qkv.rows + (kThreads / LQ) * 2 * ba.qkv.passes - 1) / ((kThreads / LQ) * 2 * ba.qkv.passes);
    const int ga = nHG * ba.at.splitGrid;
    BlockSync bs;
    bs.qkvCnt = ba.qkvCnt;
    bs.qkvExpect = ba.qkvExpect;
    bs.attnCnt = ba.attnCnt;
    bs.step = (*ba.epoch - 1u) * (unsigned)ba.nLayers + (unsigned)ba.layer + 1u;
    bs.attnTarget = bs.step * (unsigned)nHG;
    bs.error = ba.error;
    bs.timeoutTicks = ba.timeoutTicks;
    int x = blockIdx.x;
    if (x < gq) {  // producers first: dispatched ahead of the roles that wait on them
        gemvQ40Body<LQ, 1, PRO_RESNORM, EPI_QKV, GEMV_PRODUCER>(ba.qkv, x, smem, &bs);
        return;
    }
    x -= gq;
    if (x < ga) {
        if (attnTask<HG, HS, BF16, kThreads, true>(ba.at, 0, x % nHG, x / nHG, smem, &bs)) {
            blockDrain();  // this head group's final output is stored write-through: count it in
            if (threadIdx.x == 0) __hip_atomic_fetch_add(bs.attnCnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    x -= ga;
    gemvQ40Body<LW, 1, PRO_GLOBAL, TP ? EPI_STORE_TP : EPI_STORE, GEMV_CONSUMER>(ba.wo, x, smem, &bs);
}

template <int LQ, int LW, int HS>
static const void *attnBlockFnT(int hg, bool bf16, bool tp) {
#define DL_AB(G, F, T) \
    if (hg == G && bf16 == F && tp == T) return (const void *)attnBlockKernel<LQ, LW, G, HS, F, T>;
#define DL_AB4(G) DL_AB(G, true, false) DL_AB(G, true, true) DL_AB(G, false, false) DL_AB(G, false, true)
    DL_AB4(1) DL_AB4(2) DL_AB4(4) DL_AB4(8)
#undef DL_AB4
#undef DL_AB
    return nullptr;
}

}  // namespace hipk
}  // namespace dl
