// Decode GEMV launches for gfx950 (kernels: gemv_inst.h, instances: gemv_l16/32/64.hip) and the
// co-residency query of a launch.
#include "decode_dev.h"
#include "device_comm.h"

namespace dl {
namespace hipk {

const void *gemvFnL16(bool q40, int B, int pro, int epi);
const void *gemvFnL32(bool q40, int B, int pro, int epi);
const void *gemvFnL64(bool q40, int B, int pro, int epi);
const void *gemvAttnFnL16(int epi, int hg, bool bf16);
const void *gemvAttnFnL32(int epi, int hg, bool bf16);
const void *gemvAttnFnL64(int epi, int hg, bool bf16);

// Launch geometry of one GEMV (shared by the launcher and the co-residency check).
struct GemvLaunch {
    const void *fn = nullptr;
    int grid = 0;
    size_t lds = 0;
};
static GemvLaunch gemvLaunchOf(const GemvArgs &a, int B, int pro, int epi, bool q40) {
    GemvLaunch g;
    const int L = a.lanes > 0 ? a.lanes : gemvLanesPerRow(a.n, a.rows, B, q40);
    const int R = (kThreads / L) * gemvRowGroup(B, q40) * a.passes;
    g.grid = (a.rows + R - 1) / R;
    g.lds = gemvLdsBytes(a.n, B, q40, R, pro);
    if (q40 && (epi == EPI_STORE_TP || epi == EPI_RESQ_TP) && a.tp.q80) {  // Q80 exchange staging reuses `act`
        const GemvLds lay = gemvLayout(a.n, B, true, R, PRO_RESNORM);
        g.lds = std::max(g.lds, lay.act + tpQ80Lds(B * R, a.tp.world));
    }
    g.fn = L == 16 ? gemvFnL16(q40, B, pro, epi) : L == 32 ? gemvFnL32(q40, B, pro, epi) : gemvFnL64(q40, B, pro, epi);
    return g;
}

void launchGemv(const GemvArgs &a, int B, int pro, int epi, bool q40, hipStream_t s) {
    const GemvLaunch g = gemvLaunchOf(a, B, pro, epi, q40);
    if (!g.fn) throw Error("launchGemv: unsupported prologue / epilogue / batch combination");
    if (g.lds > 65536) allowLds(g.fn, g.lds);
    GemvArgs args = a;
    void *kargs[] = {&args};
    DL_HIP(hipLaunchKernel(g.fn, dim3(g.grid), dim3(kThreads), kargs, g.lds, s));
}

// PRO_ATTN (the wo GEMV with the attention in its prologue): the GEMV's own geometry, plus the
// attention task's LDS after the GEMV layout
static GemvLaunch gemvAttnLaunchOf(const GemvArgs &a, const AttnArgs &at, int epi) {
    GemvLaunch g;
    if (at.hs != 128 || at.kvMul < 1 || at.kvMul > 8 || (at.kvMul & (at.kvMul - 1)) || at.nHeads0 % at.kvMul ||
        a.n != at.nHeads0 * 128 || (epi != EPI_STORE && epi != EPI_STORE_TP))
        return g;
    const int L = a.lanes > 0 ? a.lanes : gemvLanesPerRow(a.n, a.rows, 1, true);
    const int R = (kThreads / L) * gemvRowGroup(1, true) * a.passes;
    g.grid = (a.rows + R - 1) / R;
    const GemvLds lay = gemvLayout(a.n, 1, true, R, PRO_RESNORM);
    const int hg = at.kvMul;
    const size_t attn = sizeof(float) * (size_t)(2 * 4 * hg + 4 * hg * 128 + hg * 128 + 2 * hg) + 16;
    g.lds = alignUp(lay.total, 16) + attn;
    if (epi == EPI_STORE_TP && a.tp.q80) g.lds = std::max(g.lds, lay.act + tpQ80Lds(R, a.tp.world));
    g.fn = L == 16 ? gemvAttnFnL16(epi, hg, at.kvBf16 != 0) : L == 32 ? gemvAttnFnL32(epi, hg, at.kvBf16 != 0)
                                                             : gemvAttnFnL64(epi, hg, at.kvBf16 != 0);
    return g;
}

bool gemvAttnSupported(const GemvArgs &a, const AttnArgs &at, int epi) { return gemvAttnLaunchOf(a, at, epi).fn; }

void launchGemvAttn(const GemvArgs &a, const AttnArgs &at, int epi, hipStream_t s) {
    const GemvLaunch g = gemvAttnLaunchOf(a, at, epi);
    if (!g.fn) throw Error("launchGemvAttn: unsupported attention / GEMV shape");
    if (g.lds > 65536) allowLds(g.fn, g.lds);
    GemvArgs args = a;
    AttnArgs atArgs = at;
    void *kargs[] = {&args, &atArgs};
    DL_HIP(hipLaunchKernel(g.fn, dim3(g.grid), dim3(kThreads), kargs, g.lds, s));
}

GemvResidency gemvAttnResidency(const GemvArgs &a, const AttnArgs &at, int epi) {
    GemvResidency r;
    const GemvLaunch g = gemvAttnLaunchOf(a, at, epi);
    if (!g.fn) return r;
    if (g.lds > 65536) allowLds(g.fn, g.lds);
    int dev = 0, cus = 0, perCu = 0;
    DL_HIP(hipGetDevice(&dev));
    DL_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, g.fn, kThreads, g.lds));
    r.grid = g.grid;
    r.maxResident = perCu * cus;
    return r;
}

GemvResidency gemvResidency(const GemvArgs &a, int B, int pro, int epi, bool q40) {
    GemvResidency r;
    const GemvLaunch g = gemvLaunchOf(a, B, pro, epi, q40);
    if (!g.fn) return r;
    if (g.lds > 65536) allowLds(g.fn, g.lds);
    int dev = 0, cus = 0, perCu = 0;
    DL_HIP(hipGetDevice(&dev));
    DL_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DL_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, g.fn, kThreads, g.lds));
    r.grid = g.grid;
    r.maxResident = perCu * cus;
    return r;
}

}  // namespace hipk
}  // namespace dl
