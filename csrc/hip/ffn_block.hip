// Fused FFN block of one decode row at a tensor-parallel rank (kernels.h FfnBlockArgs): the w13
// GEMV (pre-normalized Q80 input, SwiGLU epilogue) and the w2 GEMV (+ the exchange tail that applies
// the residual update and the next norm) in one launch, as two workgroup roles handing off through
// write-through stores and a monotonic arrival counter (gemv_dev.h BlockSync, the attention block's
// protocol). Reference op sequence: llm.cpp:316-391 (w1 / w3 matmuls, SiLU, mul, w2 matmul, the
// ZQ all-reduce and merge-add).
#include "decode_dev.h"
#include "device_comm.h"

namespace dl {
namespace hipk {

template <int L1, int L2, bool HQ>
__global__ __launch_bounds__(kThreads) void ffnBlockKernel(FfnBlockArgs fa) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int R1 = (kThreads / L1) * 2 * fa.w13.passes;
    const int g13 = (fa.w13.rows + R1 - 1) / R1;
    BlockSync bs;
    // steps are monotonic across layers and forwards (never reset): see BlockSync
    bs.step = (*fa.epoch - 1u) * (unsigned)fa.nLayers + (unsigned)fa.layer + 1u;
    bs.qkvAll = fa.cnt;                         // producer arrivals (the attention block's qkv phase count)
    bs.qkvAllTarget = bs.step * (unsigned)g13;
    bs.qkvFlag = fa.flag;
    bs.attnFlag = fa.flag;                      // the consumer's data wait: the whole w13 phase is done
    bs.ringEarly = true;                        // w2's weights stream while w13 runs
    bs.error = fa.error;
    bs.timeoutTicks = fa.timeoutTicks;
    bs.codeBase = 4;                            // wait codes 7 (data) / 8 (ring start, unused here)
    if ((int)blockIdx.x < g13) {  // producers first: dispatched ahead of the role that waits on them
        gemvQ40Body<L1, 1, PRO_PRENORM, HQ ? EPI_ACT_Q80 : EPI_ACT, GEMV_PRODUCER>(fa.w13, blockIdx.x, smem, &bs);
        return;
    }
    gemvQ40Body<L2, 1, HQ ? PRO_GLOBAL : PRO_RESNORM, EPI_RESQ_TP, GEMV_CONSUMER>(fa.w2, blockIdx.x - g13, smem, &bs);
}

template <int L1>
static const void *ffnBlockFnL1(int l2, bool hq) {
#define DL_FB(B2, H) \
    if (l2 == B2 && hq == H) return (const void *)ffnBlockKernel<L1, B2, H>;
    DL_FB(16, false) DL_FB(32, false) DL_FB(64, false) DL_FB(16, true) DL_FB(32, true) DL_FB(64, true)
#undef DL_FB
    return nullptr;
}

static const void *ffnBlockFn(int l1, int l2, bool hq) {
    if (l1 == 16) return ffnBlockFnL1<16>(l2, hq);
    if (l1 == 32) return ffnBlockFnL1<32>(l2, hq);
    if (l1 == 64) return ffnBlockFnL1<64>(l2, hq);
    return nullptr;
}

FfnBlockPlan ffnBlockPlan(const FfnBlockArgs &a) {
    FfnBlockPlan p;
    // the w2 role's f32 staging quantizes whole 32-element blocks; the exchange tail needs the
    // fused transport
    if (a.w13.lanes <= 0 || a.w2.lanes <= 0 || a.w2.n % 32 || !a.w2.tp.world) return p;
    p.fn = ffnBlockFn(a.w13.lanes, a.w2.lanes, a.hQ80 != 0);
    const int R1 = (kThreads / a.w13.lanes) * 2 * a.w13.passes, R2 = (kThreads / a.w2.lanes) * 2 * a.w2.passes;
    p.g13 = (a.w13.rows + R1 - 1) / R1;
    p.g2 = (a.w2.rows + R2 - 1) / R2;
    const size_t l1 = gemvLayout(a.w13.n, 1, true, R1, PRO_PRENORM).total;
    const GemvLds lay2 = gemvLayout(a.w2.n, 1, true, R2, PRO_RESNORM);
    size_t l2 = lay2.total;
    if (a.w2.tp.q80) l2 = std::max(l2, lay2.act + tpQ80Lds(R2, a.w2.tp.world));
    p.lds = std::max(l1, l2);
    return p;
}

GemvResidency ffnBlockResidency(const FfnBlockArgs &a) {
    GemvResidency r;
    const FfnBlockPlan p = ffnBlockPlan(a);
    if (!p.fn) return r;
    if (p.lds > 65536) allowLds(p.fn, p.lds);
    int dev = 0, cus = 0, perCu = 0;
    DL_HIP(hipGetDevice(&dev));
    DL_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, p.fn, kThreads, p.lds));
    // as attnBlockResidency: the query may over-report by one workgroup per CU
    r.grid = p.g13 + p.g2;
    r.maxResident = (perCu > 1 ? perCu - 1 : perCu) * cus;
    return r;
}

void launchFfnBlock(const FfnBlockArgs &a, hipStream_t s) {
    const FfnBlockPlan p = ffnBlockPlan(a);
    if (!p.fn) throw Error("launchFfnBlock: no kernel instance for this shape");
    if (!a.epoch || !a.cnt || !a.flag || !a.error) throw Error("launchFfnBlock: hand-off state missing");
    if (p.lds > 65536) allowLds(p.fn, p.lds);
    FfnBlockArgs args = a;
    void *kargs[] = {&args};
    DL_HIP(hipLaunchKernel(p.fn, dim3(p.g13 + p.g2), dim3(kThreads), kargs, p.lds, s));
}

}  // namespace hipk
}  // namespace dl
