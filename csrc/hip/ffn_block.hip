// Host side of the fused FFN block (kernels.h FfnBlockArgs): geometry, co-residency and the
// launch. The kernel is ffn_block_inst.h.
#include "decode_dev.h"
#include "device_comm.h"

#include <cstdlib>

namespace dl {
namespace hipk {

const void *ffnBlockFn_16_32(bool tp);
const void *ffnBlockFn_16_64(bool tp);
const void *ffnBlockFn_16_16(bool tp);
const void *ffnBlockFn_32_32(bool tp);
const void *ffnBlockFn_64_64(bool tp);

static const void *ffnBlockFn(int l13, int l2, bool tp) {
    if (l13 == 16 && l2 == 32) return ffnBlockFn_16_32(tp);
    if (l13 == 16 && l2 == 64) return ffnBlockFn_16_64(tp);
    if (l13 == 16 && l2 == 16) return ffnBlockFn_16_16(tp);
    if (l13 == 32 && l2 == 32) return ffnBlockFn_32_32(tp);
    if (l13 == 64 && l2 == 64) return ffnBlockFn_64_64(tp);
    return nullptr;
}

static int rowsPerWg(const GemvArgs &g) { return (kThreads / g.lanes) * 2 * g.passes; }

FfnBlockPlan ffnBlockPlan(const FfnBlockArgs &a, bool tp) {
    FfnBlockPlan p;
    p.fn = ffnBlockFn(a.w13.lanes, a.w2.lanes, tp);
    const int r13 = rowsPerWg(a.w13), r2 = rowsPerWg(a.w2);
    p.g13 = (a.w13.rows + r13 - 1) / r13;
    p.g2 = (a.w2.rows + r2 - 1) / r2;
    size_t l13 = gemvLayout(a.w13.n, 1, true, r13, PRO_RESNORM).total;
    size_t l2 = gemvLayout(a.w2.n, 1, true, r2, PRO_RESNORM).total;
    if (tp && a.w2.tp.q80) l2 = std::max(l2, gemvLayout(a.w2.n, 1, true, r2, PRO_RESNORM).act + tpQ80Lds(r2, a.w2.tp.world));
    p.lds = std::max(l13, l2);
    return p;
}

GemvResidency ffnBlockResidency(const FfnBlockArgs &a, bool tp) {
    GemvResidency r;
    const FfnBlockPlan p = ffnBlockPlan(a, tp);
    if (!p.fn) return r;
    if (p.lds > 65536) allowLds(p.fn, p.lds);
    int dev = 0, cus = 0, perCu = 0;
    DL_HIP(hipGetDevice(&dev));
    DL_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, p.fn, kThreads, p.lds));
    r.grid = a.sameWg ? std::max(p.g13, p.g2) : p.g13 + p.g2;
    // one workgroup per CU of margin, as the attention block (DL_FFN_MARGIN=0: none, diagnostics)
    static const int margin = [] {
        const char *e = std::getenv("DL_FFN_MARGIN");
        return e && *e ? std::atoi(e) : 1;
    }();
    r.maxResident = (perCu > margin ? perCu - margin : perCu) * cus;
    return r;
}

void launchFfnBlock(const FfnBlockArgs &a, bool tp, hipStream_t s) {
    const FfnBlockPlan p = ffnBlockPlan(a, tp);
    if (!p.fn) throw Error("launchFfnBlock: no kernel instance for this shape");
    if (p.lds > 65536) allowLds(p.fn, p.lds);
    FfnBlockArgs args = a;
    if (a.trace) {
        args.w13.trace = a.trace;
        args.w2.trace = a.trace + 8 * (size_t)p.g13;
    }
    void *kargs[] = {&args};
    DL_HIP(hipLaunchKernel(p.fn, dim3(a.sameWg ? std::max(p.g13, p.g2) : p.g13 + p.g2), dim3(kThreads), kargs, p.lds, s));
}

}  // namespace hipk
}  // namespace dl
