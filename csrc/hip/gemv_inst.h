// GEMV kernel templates (Q40 ring, F32) and their per-(batch, prologue, epilogue) instance table,
// compiled once per lanes-per-row L in gemv_l16/32/64.hip (parallel builds).
#pragma once
#include "decode_dev.h"

namespace dl {
namespace hipk {

template <int L, int B, int PRO, int EPI>
__global__ __launch_bounds__(kThreads) void gemvQ40Kernel(GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    gemvQ40Body<L, B, PRO, EPI>(a, blockIdx.x, smem);
}

// The wo GEMV of one decode row with the layer's attention in its prologue (PRO_ATTN, kernels.h
// launchGemvAttn): HG query heads per KV head, bf16 or f32 cache, head size 128.
template <int L, int EPI, int HG, bool BF16>
__global__ __launch_bounds__(kThreads) void gemvAttnKernel(GemvArgs a, AttnArgs at) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    gemvQ40Body<L, 1, PRO_ATTN, EPI, GEMV_PLAIN, HG, BF16>(a, blockIdx.x, smem, nullptr, &at);
}

template <int L>
static const void *gemvAttnFnL(int epi, int hg, bool bf16) {
#define DL_GA(E, G, F) \
    if (epi == E && hg == G && bf16 == F) return (const void *)gemvAttnKernel<L, E, G, F>;
#define DL_GA4(E, F) DL_GA(E, 1, F) DL_GA(E, 2, F) DL_GA(E, 4, F) DL_GA(E, 8, F)
    DL_GA4(EPI_STORE_TP, true) DL_GA4(EPI_STORE_TP, false) DL_GA4(EPI_STORE, true) DL_GA4(EPI_STORE, false)
#undef DL_GA4
#undef DL_GA
    return nullptr;
}

// ------------------------------------------------------------------------------------------------
// F32-weight GEMV: out[b][row] = W[row,:] . act(in[b,:]), fused prologue/epilogue (Q40 weights use
// gemvQ40Kernel / gemmQ40Kernel).
// ------------------------------------------------------------------------------------------------
template <int L, int B, int PRO, int EPI, bool Q40>
__global__ __launch_bounds__(kThreads) void gemvKernel(GemvArgs a) {
    static_assert(!Q40, "Q40 weights go through gemvQ40Kernel");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int RG = gemvRowGroup(B, Q40);  // rows per lane group
    constexpr int RP = kThreads / L * RG;     // rows per pass
    const int n = a.n;
    const int R = RP * a.passes;
    const GemvLds lay = gemvLayout(n, B, Q40, R, PRO);
    float *scratch = reinterpret_cast<float *>(smem + lay.scratch);
    float *res = reinterpret_cast<float *>(smem + lay.res);
    float *hbuf = reinterpret_cast<float *>(smem + lay.hbuf);
    const int tid = threadIdx.x;
    const int gi = tid / L, li = tid % L;
    const int rowBase = blockIdx.x * R;

    // activation source: normalized copy in LDS or the caller's f32 rows
    const float *actF = PRO == PRO_RESNORM ? reinterpret_cast<const float *>(smem + lay.act) : a.in;

    auto rowOf = [&](int p, int r) { return rowBase + p * RP + gi * RG + r; };
    for (int p = 0; p < a.passes; p++) {
        float acc[RG][B];
#pragma unroll
        for (int r = 0; r < RG; r++)
#pragma unroll
            for (int b = 0; b < B; b++) acc[r][b] = 0.f;
        {
            if (PRO == PRO_RESNORM && p == 0) {
                resNormPrologue<B, false>(a, scratch, nullptr, nullptr, reinterpret_cast<float *>(smem + lay.act));
            }
            const int rowc = min(rowOf(p, 0), a.rows - 1);
            const f32x4 *wrow = reinterpret_cast<const f32x4 *>(a.wf + (size_t)rowc * n);
            const int n4 = n >> 2;
            const int ldx = PRO == PRO_RESNORM ? n : a.ldIn;
#pragma unroll 4
            for (int k = li; k < n4; k += L) {
                const f32x4 wv = __builtin_nontemporal_load(wrow + k);
#pragma unroll
                for (int b = 0; b < B; b++) {
                    const float4 xv = *reinterpret_cast<const float4 *>(actF + (size_t)b * ldx + k * 4);
                    acc[0][b] += wv.x * xv.x + wv.y * xv.y + wv.z * xv.z + wv.w * xv.w;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RG; r++)
#pragma unroll
            for (int b = 0; b < B; b++) acc[r][b] = groupSum<L>(acc[r][b]);
        if (li == 0) {
#pragma unroll
            for (int r = 0; r < RG; r++) {
                const int row = rowOf(p, r);
                if constexpr (EPI == EPI_STORE) {
                    if (row < a.rows) {
#pragma unroll
                        for (int b = 0; b < B; b++) a.out[(size_t)b * a.ldOut + row] = acc[r][b];
                    }
                } else {
#pragma unroll
                    for (int b = 0; b < B; b++) res[b * R + (row - rowBase)] = acc[r][b];
                }
            }
        }
    }
    if constexpr (EPI == EPI_STORE) return;
    __syncthreads();

    // ---- pair epilogues (rows 2k, 2k+1 of this workgroup) --------------------------------------
    const int halfR = R / 2;
    for (int i = tid; i < B * halfR; i += kThreads) {
        const int b = i / halfR, k = i % halfR;
        const int r0 = rowBase + 2 * k;
        const float v0 = res[b * R + 2 * k], v1 = res[b * R + 2 * k + 1];
        if constexpr (EPI == EPI_ACT || EPI == EPI_ACT_Q80) {
            // interleaved rows: 2i = gate (w1), 2i+1 = up (w3)
            const float g = gateAct(a, v0);
            if constexpr (EPI == EPI_ACT) {
                if (r0 < a.rows) a.out[(size_t)b * a.ldOut + (r0 >> 1)] = g * v1;
            } else {
                hbuf[b * halfR + k] = g * v1;
            }
        } else if constexpr (EPI == EPI_QKV) {
            if (r0 < a.rows) qkvPairStore(a, r0, v0, v1, a.rope + (size_t)a.pos[b] * (a.hs >> 1), a.pos[b], a.slot[b],
                                          a.out + (size_t)b * a.ldOut);
        }
    }
    if constexpr (EPI == EPI_ACT_Q80) {
        __syncthreads();
        storeHiddenQ80<B>(a, hbuf, halfR, rowBase >> 1);
    }
}


// Kernel instance of one GEMV launch configuration (null: unsupported combination).
template <int L, int B, bool Q40>
static const void *gemvFnPE(int pro, int epi) {
#define DL_GEMV_CASE(P, E)                                                     \
    if (pro == P && epi == E) {                                                \
        if constexpr (Q40) return (const void *)gemvQ40Kernel<L, B, P, E>;     \
        else return (const void *)gemvKernel<L, B, P, E, false>;               \
    }
    DL_GEMV_CASE(PRO_GLOBAL, EPI_STORE)
    DL_GEMV_CASE(PRO_RESNORM, EPI_STORE)
    DL_GEMV_CASE(PRO_RESNORM, EPI_QKV)
    DL_GEMV_CASE(PRO_RESNORM, EPI_ACT)
    if constexpr (Q40) {
        DL_GEMV_CASE(PRO_RESNORM, EPI_ACT_Q80)
        DL_GEMV_CASE(PRO_GLOBAL, EPI_STORE_TP)
        DL_GEMV_CASE(PRO_RESNORM, EPI_STORE_TP)
        if constexpr (B == 1) {
            DL_GEMV_CASE(PRO_RESNORM, EPI_ARGMAX)
            // pre-normalized hand-off (tensor-parallel single rows): producers and consumers
            DL_GEMV_CASE(PRO_GLOBAL, EPI_RESQ_TP)
            DL_GEMV_CASE(PRO_RESNORM, EPI_RESQ_TP)
            DL_GEMV_CASE(PRO_PRENORM, EPI_QKV)
            DL_GEMV_CASE(PRO_PRENORM, EPI_ACT)
            DL_GEMV_CASE(PRO_PRENORM, EPI_ACT_Q80)
            DL_GEMV_CASE(PRO_PRENORM, EPI_STORE)
            DL_GEMV_CASE(PRO_PRENORM, EPI_ARGMAX)
        }
    }
#undef DL_GEMV_CASE
    return nullptr;
}

template <int L, bool Q40>
static const void *gemvFnB(int B, int pro, int epi) {
    switch (B) {
        case 1: return gemvFnPE<L, 1, Q40>(pro, epi);
        case 2: return gemvFnPE<L, 2, Q40>(pro, epi);
        case 4: return gemvFnPE<L, 4, Q40>(pro, epi);
        default: return nullptr;
    }
}


}  // namespace hipk
}  // namespace dl
