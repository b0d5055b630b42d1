// Fused FFN block kernel template (kernels.h FfnBlockArgs): w13 producer rows, then w2 consumer
// rows. Instances are compiled per (w13 lanes, w2 lanes) in ffn_block_*.hip (parallel builds).
#pragma once
#include "decode_dev.h"

namespace dl {
namespace hipk {

template <int L13, int L2, bool TP>
__global__ __launch_bounds__(kThreads) void ffnBlockKernel(FfnBlockArgs fa) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int r13 = (kThreads / L13) * 2 * fa.w13.passes;
    const int g13 = (fa.w13.rows + r13 - 1) / r13;
    BlockSync bs;
    bs.step = (*fa.epoch - 1u) * (unsigned)fa.nLayers + (unsigned)fa.layer + 1u;
    bs.qkvAll = fa.cnt;
    bs.qkvAllTarget = bs.step * (unsigned)g13;
    bs.qkvFlag = fa.flag;   // ring start ...
    bs.attnFlag = fa.flag;  // ... and data ready: both "every w13 workgroup arrived"
    bs.error = fa.error;
    bs.timeoutTicks = fa.timeoutTicks;
    bs.codeBase = 10;
    bs.ringEarly = fa.ringEarly != 0;
    if (fa.sameWg) {
        const int r2 = (kThreads / L2) * 2 * fa.w2.passes;
        const int g2 = (fa.w2.rows + r2 - 1) / r2;
        if ((int)blockIdx.x < g13)
            gemvQ40Body<L13, 1, PRO_RESNORM, EPI_ACT_Q80, GEMV_PRODUCER>(fa.w13, blockIdx.x, smem, &bs);
        if ((int)blockIdx.x < g2) {
            __syncthreads();  // the w13 body's LDS is reused
            bs.ringEarly = true;
            gemvQ40Body<L2, 1, PRO_GLOBAL, TP ? EPI_STORE_TP : EPI_STORE, GEMV_CONSUMER>(fa.w2, blockIdx.x, smem, &bs);
        }
        return;
    }
    if ((int)blockIdx.x < g13) {  // producers first: dispatched ahead of the role that waits on them
        gemvQ40Body<L13, 1, PRO_RESNORM, EPI_ACT_Q80, GEMV_PRODUCER>(fa.w13, blockIdx.x, smem, &bs);
        return;
    }
    gemvQ40Body<L2, 1, PRO_GLOBAL, TP ? EPI_STORE_TP : EPI_STORE, GEMV_CONSUMER>(fa.w2, blockIdx.x - g13, smem, &bs);
}

template <int L13, int L2>
static const void *ffnBlockFnT(bool tp) {
    return tp ? (const void *)ffnBlockKernel<L13, L2, true> : (const void *)ffnBlockKernel<L13, L2, false>;
}

}  // namespace hipk
}  // namespace dl
