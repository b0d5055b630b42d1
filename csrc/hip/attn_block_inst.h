// Fused attention block kernel template (see kernels.h AttnBlockArgs): roles by workgroup index.
// Instances are compiled per (qkv lanes, wo lanes, head size) in attn_block_*.hip (parallel builds).
#pragma once
#include "decode_dev.h"

namespace dl {
namespace hipk {

template <int LQ, int LW, int HG, int HS, bool BF16, int MD>
__global__ __launch_bounds__(kThreads) void attnBlockKernel(AttnBlockArgs ba) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nHG = ba.at.nHeads0 / HG;
    const int gq = (ba.qkv.rows + (kThreads / LQ) * 2 * ba.qkv.passes - 1) / ((kThreads / LQ) * 2 * ba.qkv.passes);
    const int ga = nHG * ba.at.splitGrid;
    BlockSync bs;
    bs.qkvCnt = ba.qkvCnt;
    bs.qkvExpect = ba.qkvExpect;
    bs.attnCnt = ba.attnCnt;
    bs.attnFlag = ba.attnFlag;
    bs.step = (*ba.epoch - 1u) * (unsigned)ba.nLayers + (unsigned)ba.layer + 1u;
    bs.attnTarget = bs.step * (unsigned)nHG;
    bs.nKv = ba.at.nHeads0 / ba.at.kvMul;
    bs.qkvAll = ba.attnFlag + 8 * kCntStride;   // layout: engine.cpp kBlockCntWords
    bs.qkvFlag = ba.attnFlag + 9 * kCntStride;
    bs.qkvAllTarget = bs.step * (unsigned)gq;
    bs.error = ba.error;
    bs.timeoutTicks = ba.timeoutTicks;
    int x = blockIdx.x;
    if (x < gq) {  // producers first: dispatched ahead of the roles that wait on them
        gemvQ40Body<LQ, 1, PRO_RESNORM, EPI_QKV, GEMV_PRODUCER>(ba.qkv, x, smem, &bs);
        return;
    }
    x -= gq;
    if (x < ga) {
        unsigned long long *tr = ba.trace ? ba.trace + 8 * (size_t)blockIdx.x : nullptr;
        const unsigned long long t0 = tr ? wall_clock64() : 0ull;
        const bool fin = attnTask<HG, HS, BF16, kThreads, true>(ba.at, 0, x % nHG, x / nHG, smem, &bs, tr);
        if (fin) {
            blockDrain();  // this head group's final output is stored write-through: count it in;
            // the last head group to arrive raises the step's per-XCD ready flags for the wo role
            if (threadIdx.x == 0 &&
                __hip_atomic_fetch_add(bs.attnCnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == bs.attnTarget) {
                raiseFlags(bs.attnFlag, bs.step);
            }
        }
        if (tr && threadIdx.x == 0) {
            tr[0] = t0;
            tr[3] = wall_clock64();
            tr[7] = 1u | (fin ? 16u : 0u);
        }
        return;
    }
    x -= ga;
    gemvQ40Body<LW, 1, PRO_GLOBAL, MD == 1 ? EPI_STORE_TP : EPI_STORE, GEMV_CONSUMER>(ba.wo, x, smem,
                                                                                                        &bs);
}

template <int LQ, int LW, int HS>
static const void *attnBlockFnT(int hg, bool bf16, int md) {
#define DL_AB(G, F, M) \
    if (hg == G && bf16 == F && md == M) return (const void *)attnBlockKernel<LQ, LW, G, HS, F, M>;
#define DL_AB4(G) DL_AB(G, true, 0) DL_AB(G, true, 1) DL_AB(G, false, 0) DL_AB(G, false, 1)
    DL_AB4(1) DL_AB4(2) DL_AB4(4) DL_AB4(8)
#undef DL_AB4
#undef DL_AB
    return nullptr;
}

}  // namespace hipk
}  // namespace dl
