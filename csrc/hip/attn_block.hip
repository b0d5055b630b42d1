// Host side of the fused attention block (kernels.h AttnBlockArgs): geometry, expected arrival
// counts, co-residency and the launch. The kernel is attn_block_inst.h.
#include "decode_dev.h"
#include "device_comm.h"

namespace dl {
namespace hipk {

const void *attnBlockFn_16_16_128(int hg, bool bf16, int md);
const void *attnBlockFn_16_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_32_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_16_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_64_128(int hg, bool bf16, int md);
const void *attnBlockFn_32_64_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_64_64(int hg, bool bf16, int md);

static const void *attnBlockFn(int lq, int lw, int hs, int hg, bool bf16, int md) {
    if (lq == 16 && lw == 16 && hs == 128) return attnBlockFn_16_16_128(hg, bf16, md);
    if (lq == 16 && lw == 32 && hs == 128) return attnBlockFn_16_32_128(hg, bf16, md);
    if (lq == 32 && lw == 32 && hs == 128) return attnBlockFn_32_32_128(hg, bf16, md);
    if (lq == 64 && lw == 32 && hs == 128) return attnBlockFn_64_32_128(hg, bf16, md);
    if (lq == 64 && lw == 16 && hs == 128) return attnBlockFn_64_16_128(hg, bf16, md);
    if (lq == 64 && lw == 64 && hs == 128) return attnBlockFn_64_64_128(hg, bf16, md);
    if (lq == 32 && lw == 64 && hs == 128) return attnBlockFn_32_64_128(hg, bf16, md);
    if (lq == 64 && lw == 64 && hs == 64) return attnBlockFn_64_64_64(hg, bf16, md);
    return nullptr;
}

int attnBlockHG(const AttnArgs &a) {
    // as launchAttention: the fewest query heads per workgroup that keep the attention role within
    // 256 workgroups at the longest context (one row)
    const int hgMax = (a.kvMul & (a.kvMul - 1)) == 0 ? (a.kvMul < 8 ? a.kvMul : 8) : 1;
    int hg = 1;
    while (hg < hgMax && (long)(a.nHeads0 / hg) * a.splitGrid > 256) hg *= 2;
    return hg;
}

static int gemvGrid(const GemvArgs &g) {
    const int R = (kThreads / g.lanes) * 2 * g.passes;
    return (g.rows + R - 1) / R;
}

AttnBlockPlan attnBlockPlan(const AttnBlockArgs &a, bool tp) {
    AttnBlockPlan p;
    // md: 0 plain, 1 tensor-parallel wo exchange
    p.fn = attnBlockFn(a.qkv.lanes, a.wo.lanes, a.at.hs, a.hg, a.at.kvBf16 != 0, tp ? 1 : 0);
    p.gq = gemvGrid(a.qkv);
    p.ga = a.at.nHeads0 / a.hg * a.at.splitGrid;
    p.gw = gemvGrid(a.wo);
    const int Rq = (kThreads / a.qkv.lanes) * 2 * a.qkv.passes, Rw = (kThreads / a.wo.lanes) * 2 * a.wo.passes;
    size_t lq = gemvLayout(a.qkv.n, 1, true, Rq, PRO_RESNORM).total;
    size_t lw = gemvLayout(a.wo.n, 1, true, Rw, PRO_RESNORM).total;
    if (tp && a.wo.tp.q80) lw = std::max(lw, gemvLayout(a.wo.n, 1, true, Rw, PRO_RESNORM).act + tpQ80Lds(Rw, a.wo.tp.world));
    constexpr int NW = kThreads / 64;
    const size_t la = sizeof(float) * (2 * NW * a.hg + NW * a.hg * a.at.hs + a.hg * a.at.hs + 2 * a.hg) + 16;
    p.lds = std::max(lq, std::max(lw, la));
    return p;
}

void attnBlockExpect(const GemvArgs &q, int nKv, unsigned *out) {
    for (int g = 0; g < nKv; g++) out[g] = 0;
    const int R = (kThreads / q.lanes) * 2 * q.passes, grid = gemvGrid(q);
    for (int w = 0; w < grid; w++) {
        unsigned long long m = qkvGroupMask(w * R, std::min(w * R + R, q.rows), q.q0, q.kv0, q.hs, q.kvMul);
        for (int g = 0; g < nKv && g < 64; g++)
            if (m >> g & 1ull) out[g]++;
    }
}

GemvResidency attnBlockResidency(const AttnBlockArgs &a, bool tp) {
    GemvResidency r;
    const AttnBlockPlan p = attnBlockPlan(a, tp);
    if (!p.fn) return r;
    if (p.lds > 65536) allowLds(p.fn, p.lds);
    int dev = 0, cus = 0, perCu = 0;
    DL_HIP(hipGetDevice(&dev));
    DL_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, p.fn, kThreads, p.lds));
    // the query may over-report by one workgroup per CU for SGPR-heavy 256-thread kernels on ROCm
    // 7.2 (cdna_hip_programming.md §1): count one fewer
    r.grid = p.gq + p.ga + p.gw;
    r.maxResident = (perCu > 1 ? perCu - 1 : perCu) * cus;
    return r;
}

void launchAttnBlock(const AttnBlockArgs &a, bool tp, hipStream_t s) {
    const AttnBlockPlan p = attnBlockPlan(a, tp);
    if (!p.fn) throw Error("launchAttnBlock: no kernel instance for this shape");
    if (p.lds > 65536) allowLds(p.fn, p.lds);
    AttnBlockArgs args = a;
    if (a.trace) {  // per-role trace slots: qkv [0, gq), attention [gq, gq + ga), wo after them
        args.qkv.trace = a.trace;
        args.wo.trace = a.trace + 8 * (size_t)(p.gq + p.ga);
    }
    void *kargs[] = {&args};
    DL_HIP(hipLaunchKernel(p.fn, dim3(p.gq + p.ga + p.gw), dim3(kThreads), kargs, p.lds, s));
}

}  // namespace hipk
}  // namespace dl
