// Wide batched Q40 GEMM on MFMA for prefill chunks and large serving batches (> 64 tokens per
// launch): 128-row x 128-token output tiles, so every weight and activation byte staged in LDS
// feeds 2 x 4 x 4 MFMAs per wave instead of the narrow kernel's 1 x MT (gemm.hip), and a launch
// covers all token tiles of a chunk (grid = row tiles x token tiles x K splits) instead of
// re-streaming the weights per 64-128 tokens.
//
// Reference roles: the batched Q80 x Q40 matmul of the CPU backend (src/nn/nn-cpu-ops.cpp:222-440,
// tinyBLAS src/nn/llamafile/sgemm.cpp:263-412 for its tile dispatch) and the chunked prefill of
// src/dllama.cpp:36-66.
//
// Workgroup: 256 threads = 4 waves in a 2 x 2 arrangement, wave (wr, wt) owning rows
// [64 wr, 64 wr + 64) x tokens [64 wt, 64 wt + 64) of the tile: 4 x 4 accumulators of
// v_mfma_f32_16x16x32_f16 (64 VGPRs). K advances two Q40 blocks (64) per pipeline stage; a stage
// holds the tile's 128 weight rows (2 x 16 B each), their f16 scales (u32 pairs) and the 128
// tokens' 64 f16 activations, copied HBM/L2 -> LDS by global_load_lds (6 wave-instructions per
// thread per stage, 3 stages = 2 in flight, ~43 KB per workgroup; one block per stage measured
// slower: twice the barriers). Per block a wave dequantizes its 4 weight fragments once (nibbles
// -> f16, gemm_dev.h) and reuses each for 4 token fragments. LDS images are bank-conflict free:
// a row's two 16-B units swap places for rows 8..15 of each 16 (ds_read_b64 of 16 rows x 2 halves
// covers all 64 banks), activation unit u of token t sits at position u ^ ((t >> 1) & 7).
// The grid is mapped XCD-aware: consecutive logical workgroups (the token tiles and K splits of one
// row tile, which share weights) are dispatched to the same XCD (its L2).
// Split-K (thin matrices: wo, w2, qkv) stores partials with write-through stores; the last arriving
// split sums them in split order (deterministic, gemm_dev.h splitArrive / splitCombine). The
// output tile goes through LDS (padded rows) into the shared fused epilogues (gemm_dev.h).
#include "gemm_dev.h"

#include <cstdlib>

namespace dl {
namespace hipk {

static constexpr int kWRows = 128, kWTok = 128, kWKB = 2, kWStages = 3, kWNld = 6;
static constexpr int kWStW = kWRows * kWKB * 16;   // [128 rows][2 blocks] x 16 B
static constexpr int kWStD = 2 * kWKB * 64 * 4;    // [2 blocks][64 row pairs] u32 scales + a dummy copy
static constexpr int kWStX = kWTok * kWKB * 64;    // [128 tokens][8 x 16 B], swizzled
static constexpr int kWStage = kWStW + kWStD + kWStX;
static constexpr int kWTileLd = kWRows + 4;  // padded f32 row stride of the output tile
static constexpr int kWMain = kWStages * kWStage > kWTok * kWTileLd * 4 ? kWStages * kWStage : kWTok * kWTileLd * 4;
static constexpr size_t kWLds = kWMain + 16 + (128 + 256) * 4;  // + flag + row scales / scratch

bool gemmWideOn() {
    static const bool v = [] {
        const char *e = std::getenv("DL_GEMM_WIDE");
        return !(e && std::atoi(e) == 0);
    }();
    return v;
}
int gemmWideMin() {  // below: narrow kernel (wide at 17-64 rows measured slower, r3); DL_GEMM_WIDE_MIN
    static const int v = [] {
        const char *e = std::getenv("DL_GEMM_WIDE_MIN");
        return e && std::atoi(e) > 0 ? std::atoi(e) : 65;
    }();
    return v;
}
bool gemmUsesWide(int M) { return gemmWideOn() && M >= gemmWideMin(); }

// K splits: grow while the grid stays under one workgroup per CU (256) and every split keeps >= 16
// blocks; at most 4 (the last arriver reads S x 64 KB).
int gemmWideSplits(int rows, int n, int M) {
    const int rowTiles = (rows + kWRows - 1) / kWRows, tokTiles = (M + kWTok - 1) / kWTok, nb = n / 32;
    int S = 1;
    while (S < 4 && rowTiles * tokTiles * S < 256 && nb % (4 * S) == 0 && nb / (2 * S) >= 16) S *= 2;
    return S;
}

size_t gemmWidePartFloats(int rows, int n, int maxTokens) {
    const int rowTiles = (rows + kWRows - 1) / kWRows;
    size_t best = 0;
    for (int tt = 1; tt <= (maxTokens + kWTok - 1) / kWTok; tt++) {
        const int S = gemmWideSplits(rows, n, tt * kWTok);
        if (S > 1) best = std::max(best, (size_t)S * rowTiles * tt * kWRows * kWTok);
    }
    return best;
}

int gemmWideCounters(int rows, int maxTokens) {
    return ((rows + kWRows - 1) / kWRows) * ((maxTokens + kWTok - 1) / kWTok);
}

template <int EPI>
__global__ __launch_bounds__(kThreads) void gemmWideKernel(GemmArgs ga, int rowTiles, int tokTiles) {
    const GemvArgs &a = ga.e;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int *flag = reinterpret_cast<int *>(smem + kWMain);
    float *rsL = reinterpret_cast<float *>(flag + 4);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int col = lane & 15, h = lane >> 4, wr = wave & 1, wt = wave >> 1;
    // XCD-aware order: dispatch sends workgroup id to XCD id % 8; logical tile L runs on XCD
    // L / (G / 8), so a row tile's token tiles and splits share one L2
    const int G = gridDim.x, id = blockIdx.x;
    const int L = (G & 7) == 0 ? (id & 7) * (G >> 3) + (id >> 3) : id;
    const int S = ga.splits, per = tokTiles * S;
    const int rt = L / per, rem = L - rt * per, tt = rem / S, sp = rem - tt * S;
    const int R0 = rt * kWRows, T0 = tt * kWTok;
    const int n = a.n, nb = n >> 5, Ln = a.lanes, NG = kThreads / Ln, KS = (nb + Ln - 1) / Ln;
    const int lgL = 31 - __builtin_clz(Ln);
    const int bps = nb / S, j0 = sp * bps;
    const uint8_t *qs = a.qs;
    const uint32_t *wd2 = reinterpret_cast<const uint32_t *>(a.wd);

    // global -> LDS copies of blocks j, j+1 into stage buffer b (6 wave-instructions per thread)
    auto issue = [&](int j, int b) {
        char *st = smem + b * kWStage;
        {  // weights: slot s = wave * 64 + lane -> row s / 2, position s & 1 holds block (s & 1) ^ ((row >> 3) & 1)
            const int sl = wave * 64 + lane, rl = sl >> 1, jb = j + ((sl & 1) ^ ((rl >> 3) & 1));
            const int row = min(R0 + rl, a.rows - 1);
            const int g = row / (2 * NG), rm = row % (2 * NG), gi = rm >> 1, rpar = rm & 1;
            const size_t unit = (((size_t)g * KS + (jb >> lgL)) * 2 + rpar) * kThreads + gi * Ln + (jb & (Ln - 1));
            glds16(qs + unit * 16, st + wave * 1024);
        }
        {  // scales of block j + (wave & 1): lane = row pair (waves 2, 3 repeat into a dummy copy)
            const int jb = j + (wave & 1), row = min(R0 + 2 * lane, a.rows - 1);
            const int g = row / (2 * NG), gi = (row % (2 * NG)) >> 1;
            glds4(wd2 + ((size_t)g * KS + (jb >> lgL)) * kThreads + gi * Ln + (jb & (Ln - 1)), st + kWStW + wave * 256);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {  // activations: 16 wave-instructions of 64 x 16 B
            const int k = wave + 4 * q, slot = k * 64 + lane, t = slot >> 3, u = (slot & 7) ^ ((t >> 1) & 7);
            glds16(ga.x + (size_t)(T0 + t) * n + (size_t)(j + (u >> 2)) * 32 + (u & 3) * 8,
                   st + kWStW + kWStD + k * 1024);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int f = 0; f < 4; f++)
#pragma unroll
        for (int t = 0; t < 4; t++) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int byteHalf = h & 1, nibHi = h >> 1;
    constexpr int PF = kWStages - 1;
    const int nch = bps / kWKB;
    for (int c = 0; c < PF && c < nch; c++) issue(j0 + kWKB * c, c);
    for (int c = 0; c < nch; c++) {
        if (c + PF < nch) issue(j0 + kWKB * (c + PF), (c + PF) % kWStages);
        // chunk c landed for this thread (the younger chunks may stay in flight), then for all
        switch (min(nch - 1, c + PF) - c) {
            case 2: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * kWNld) : "memory"); break;
            case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kWNld) : "memory"); break;
            default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        }
        __builtin_amdgcn_s_barrier();
        const char *st = smem + (c % kWStages) * kWStage;
#pragma unroll
        for (int kb = 0; kb < kWKB; kb++) {
            half8 b[4];
#pragma unroll
            for (int f = 0; f < 4; f++) {
                const int rl = wr * 64 + f * 16 + col;
                // opaque addresses: hipcc would otherwise pair the fragments (rows 16 apart) into
                // ds_read2st64_b64 / _b32, whose 32-bank rule makes the 32-B weight rows 2-way
                // conflicted (SQ_LDS_BANK_CONFLICT 27.6 % of LDS cycles); single ds_read_b64 follow
                // the 64-bank rule this image is conflict-free for
                uint32_t aw = (uint32_t)((rl * 2 + (kb ^ ((rl >> 3) & 1))) * 16 + byteHalf * 8);
                uint32_t ad = (uint32_t)(kWStW + (kb * 64 + (rl >> 1)) * 4);
                asm volatile("" : "+v"(aw), "+v"(ad));
                const u32x2 wv = *reinterpret_cast<const u32x2 *>(st + aw);
                const uint32_t dw = *reinterpret_cast<const uint32_t *>(st + ad);
                b[f] = dequantQ40x8(wv, nibHi, (rl & 1) ? dw >> 16 : dw & 0xFFFFu);
            }
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int tok = wt * 64 + t * 16 + col;
                const half8 av = *reinterpret_cast<const half8 *>(st + kWStW + kWStD +
                                                                 (tok * 8 + ((kb * 4 + h) ^ ((tok >> 1) & 7))) * 16);
#pragma unroll
                for (int f = 0; f < 4; f++) acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b[f], acc[f][t], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage c % kWStages is refilled at iteration c + 1
    }

    // C layout: acc[f][t][i] = out[token 64 wt + 16 t + 4 h + i][row 64 wr + 16 f + col]
    float *tile = reinterpret_cast<float *>(smem);  // [128 tokens][kWTileLd], the stages are free
    if (S == 1) {
#pragma unroll
        for (int f = 0; f < 4; f++)
#pragma unroll
            for (int t = 0; t < 4; t++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    tile[(wt * 64 + t * 16 + h * 4 + i) * kWTileLd + wr * 64 + f * 16 + col] = acc[f][t][i];
    } else {
        const int lt = rt * tokTiles + tt;
        const size_t tileF = (size_t)kWTok * kWRows, stride = (size_t)rowTiles * tokTiles * tileF;
        float *part = ga.part + sp * stride + lt * tileF;
#pragma unroll
        for (int f = 0; f < 4; f++)
#pragma unroll
            for (int t = 0; t < 4; t++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    wtStore(part + (wt * 64 + t * 16 + h * 4 + i) * kWRows + wr * 64 + f * 16 + col, acc[f][t][i]);
        if (!splitArrive(ga.counters + lt, S, flag)) return;
        splitCombine(ga.part + lt * tileF, stride, S, (int)(tileF / 4), reinterpret_cast<f32x4 *>(tile), kWRows / 4,
                     kWTileLd / 4);
    }
    __syncthreads();
    if (ga.ssIn) gemmRowScales(ga, T0, kWTok, rsL, rsL + 128);
    gemmEpilogue<EPI, kWRows / 2>(ga, tile, kWTileLd, 0, min(kWTok, ga.M - T0), T0, R0, rt * 2,
                                  ga.ssIn ? rsL : nullptr);
}

// preloadModules(): one kernel of this translation unit's code object
const void *gemmWideModuleKernel() { return (const void *)gemmWideKernel<EPI_STORE>; }

void launchGemmWide(const GemmArgs &ga, int epi, hipStream_t s) {
    const int rowTiles = (ga.e.rows + kWRows - 1) / kWRows, tokTiles = (ga.M + kWTok - 1) / kWTok;
    if (ga.e.n % 64 != 0 || (ga.e.n / 32) % (kWKB * ga.splits) != 0) throw Error("launchGemmWide: bad K split");
    if (ga.splits > 1 && (!ga.part || !ga.counters)) throw Error("launchGemmWide: split-K without buffers");
    const dim3 grid(rowTiles * tokTiles * ga.splits);
#define DL_GEMMW_CASE(E)                                                                              \
    if (epi == E) {                                                                                   \
        allowLds((const void *)gemmWideKernel<E>, kWLds);                                             \
        hipLaunchKernelGGL((gemmWideKernel<E>), grid, dim3(kThreads), kWLds, s, ga, rowTiles, tokTiles); \
        return;                                                                                       \
    }
    DL_GEMMW_CASE(EPI_STORE) DL_GEMMW_CASE(EPI_ACT) DL_GEMMW_CASE(EPI_ACT_Q80) DL_GEMMW_CASE(EPI_QKV)
    DL_GEMMW_CASE(EPI_ACT_F16) DL_GEMMW_CASE(EPI_RES)
#undef DL_GEMMW_CASE
    throw Error("launchGemmWide: unsupported epilogue");
}

}  // namespace hipk
}  // namespace dl
