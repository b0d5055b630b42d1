// Host-visible launchers for the gfx950 kernels (csrc/hip/kernels.hip).
//
// Kernel map vs the reference op inventory:
//   gemv<PRO_RESNORM, EPI_QKV>     OP_MERGE_ADD + OP_INV_RMS + OP_RMS_NORM + OP_CAST(Q80)
//                                  + 3x OP_MATMUL (q,k,v) + 2x OP_ROPE_LLAMA + 2x OP_SHIFT
//   attention                      OP_MULTIHEAD_ATT (flash-decoding split over the sequence, the
//                                  split combine done in-kernel by the last-arriving workgroup)
//                                  + OP_CAST(Q80) of its output
//   gemv<PRO_GLOBAL, EPI_STORE>    OP_MATMUL (wo, w2) on Q80 activations produced upstream
//   gemv<PRO_RESNORM, EPI_ACT_Q80> OP_MERGE_ADD + norm + OP_MATMUL (w1, w3) + OP_SILU/GELU + OP_MUL
//                                  + OP_CAST(Q80)
//   gemv<PRO_RESNORM, EPI_STORE>   final norm + OP_MATMUL (logits)
//   embedding                      OP_EMBEDDING
//   argmax                         greedy sampling on device (+ token feedback for decode chains)
#pragma once

#include <algorithm>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace dl {
namespace hipk {

// PRO_GLOBAL: activations are read straight from global memory in the main loop (Q80 blocks for
//             Q40 weights, f32 for F32 weights) - no prologue, no LDS, no barrier.
// PRO_RESNORM: (x + delta) -> RMS norm -> Q80 (or f32) staged once per workgroup in LDS
//             (normW == null: no norm, plain quantization of `in`).
// PRO_ATTN (Q40 ring GEMV, one row: the wo GEMV of a short-context decode step): the layer's
//             decode attention for every head of the rank is computed in the prologue of EVERY
//             workgroup (redundantly, from L2) and quantized to Q80 into LDS - no attention
//             launch and no hand-off (launchGemvAttn; the engine takes it for few heads per rank).
// PRO_PRENORM (Q40 ring GEMV, one row): the producer of this input (EPI_RESQ_TP, or the embedding)
//             already applied the residual update and the RMS norm's weights and quantized
//             x * normW to Q80 blocks (aq / as, unrounded block scale d' = amax / 127); the
//             workgroup only sums the producer's per-workgroup sums of squares (sspIn, nSsp, in
//             order) and folds 1 / rms into each block scale (d = f16(d' / rms)) while copying.
enum Prologue : int { PRO_GLOBAL = 0, PRO_RESNORM = 1, PRO_ATTN = 2, PRO_PRENORM = 3 };
// EPI_ACT_Q80: act(w1 x) * (w3 x), quantized to Q80 blocks for the next GEMV (32 hidden units/block).
// EPI_STORE_TP: EPI_STORE whose rows are first all-reduced over the tensor-parallel ranks (GemvArgs::tp).
// EPI_RES (batched GEMMs): residual update fused with the next RMS norm's elementwise half - see
// GemmArgs::resIn.
// EPI_ARGMAX (Q40 GEMV, one row, greedy logits): no logits are stored; the row's argmax (GemvArgs::am).
// EPI_RESQ_TP (Q40 GEMV, one row, 32-row workgroups): EPI_STORE_TP's rank-order sum, then the
// residual update and the NEXT RMS norm's elementwise half in the tail (GemvArgs::rq): x' = resIn +
// sum -> resOut, x' * resW quantized to Q80 blocks -> xq / xs, and this workgroup's sum of x'^2 ->
// ssp[workgroup] (the consumer, PRO_PRENORM, finishes the norm).
enum Epilogue : int { EPI_STORE = 0, EPI_ACT = 1, EPI_QKV = 2, EPI_ACT_Q80 = 3, EPI_ACT_F16 = 4, EPI_STORE_TP = 5, EPI_RES = 6,
                      EPI_ARGMAX = 7, EPI_RESQ_TP = 8 };

// Pre-normalized hand-off (EPI_RESQ_TP producer / embedding -> PRO_PRENORM consumer), one row.
struct PrenormOut {
    const float *resIn = nullptr;  // residual before this update (producer)
    float *resOut = nullptr;       // x' = residual after it
    const float *resW = nullptr;   // the next RMS norm's weights
    int8_t *xq = nullptr;          // [n] Q80 values of x' * resW
    float2 *xs = nullptr;          // [n / 32] (d' = amax / 127 unrounded, sum of q)
    float *ssp = nullptr;          // [workgroups] sums of x'^2
};

// Q40 weights live on the device TILED in the ring GEMV's consumption order, for a lanes-per-row
// count L fixed per matrix (NG = 256/L row pairs per workgroup pass, K = ceil(nb/L) steps):
//   chunk c = pass group g (2*NG consecutive rows) x step k (blocks j = li + k*L), c = g*K + k
//   qs: [c][r in {0,1}][256 threads] x 16 B    thread tid = gi*L + li -> row 2*(g*NG+gi) + r
//   d : [c][256 threads] x u32                 {lo: f16 scale of the even row, hi: odd row}
// so a workgroup streams one contiguous region (8 KB of nibbles + 1 KB of scales per step).
// Padding (rows past the end, j >= nb) is zero.
struct Q40Tiling {
    int L = 16, NG = 16, K = 0, groups = 0;
    size_t chunks = 0, qsBytes = 0, dBytes = 0;
};
Q40Tiling q40Tiling(int rows, int n, int L);
// Host repack of row-major SoA blocks (qs [rows][nb][16], d [rows][nb] f16) into the tiled layout.
void tileQ40(const uint8_t *qs, const uint16_t *d, int rows, int n, int L, uint8_t *qsOut, uint32_t *dOut);
// Same from the file's AoS blocks (BlockQ40: f16 scale + 16 nibble bytes): rowBlocks[r] points
// at row r's first block of the column slice being tiled.
void tileQ40AoS(const uint8_t *const *rowBlocks, int rows, int n, int L, uint8_t *qsOut, uint32_t *dOut);

// Paged KV cache: with a page table the cache rows of (slot, pos) live at row
// table[slot * pagesPerSlot + (pos >> pageShift)] * 2^pageShift + (pos & (2^pageShift - 1)) of a
// per-layer pool of pages, so slots hold only the pages their sequences reached; without one the
// cache is contiguous [slot][seqLen]. Pages are >= 32 positions (a 32-key attention tile never
// crosses a page).
struct KvMap {
    const int *table = nullptr;  // [slots][pagesPerSlot] page ids (null: contiguous)
    int pageShift = 0;
    int pagesPerSlot = 0;
};
// KV caches are head-major, so one KV head's keys are contiguous (a decode-attention workgroup
// streams one range instead of 2 * hs-byte slices kv0 apart): element offset of the head vector
// of (slot, pos, KV head kvh) in a layer's cache, contiguous [slot][nKv][seqLen][hs] or paged
// [page][nKv][pageSize][hs] (the page table maps a slot's position blocks to pool pages).
__host__ __device__ inline size_t kvPageOf(const KvMap &m, int slot, int pos) {
    return (size_t)m.table[slot * m.pagesPerSlot + (pos >> m.pageShift)];
}
__host__ __device__ inline size_t kvOffAt(const KvMap &m, int seqLen, int nKv, int hs, size_t block, int pos, int kvh) {
    // block = slot (contiguous) or pool page (paged)
    if (!m.table) return ((block * nKv + kvh) * seqLen + pos) * hs;
    return (((block * nKv + kvh) << m.pageShift) + (size_t)(pos & ((1 << m.pageShift) - 1))) * hs;
}
__host__ __device__ inline size_t kvOff(const KvMap &m, int seqLen, int nKv, int hs, int slot, int pos, int kvh) {
    return kvOffAt(m, seqLen, nKv, hs, m.table ? kvPageOf(m, slot, pos) : (size_t)slot, pos, kvh);
}

struct AttnArgs {
    const float *q = nullptr;   // [B][ldq], rotated queries
    int ldq = 0;
    const void *kcache = nullptr, *vcache = nullptr;  // layer base [slot][nKv][seqLen][hs] (or a page pool: kvOff)
    KvMap kvMap;
    const int *pos = nullptr, *slot = nullptr;
    int nHeads0 = 0, kvMul = 1, hs = 0, kv0 = 0, seqLen = 0;
    int splitGrid = 1;          // max sequence splits (grid.y)
    int chunkMax = 256;         // LDS capacity in positions per split
    int chunkMin = 256;         // fewest positions per split (attnChunkMin)
    int shortLen = 0;           // rows of <= shortLen keys split at kAttnShortChunk (single decode rows)
    float *partO = nullptr;     // [B][nHeads0][splitGrid][hs]
    float *partML = nullptr;    // [B][nHeads0][splitGrid][2]
    float *out = nullptr;       // [B][ldOut] f32 output (when outQ and outH are null)
    _Float16 *outH = nullptr;   // [B][ldOut] f16 output (batched path)
    int8_t *outQ = nullptr;     // [B][ldOut] Q80 output (+ outS [B][ldOut/32])
    float2 *outS = nullptr;
    int ldOut = 0;
    int kvBf16 = 1;
    int mfma = -1;              // decode kernel: 1 MFMA, 0 VALU, -1 by cache length (attnUsesMfma)
    int *counters = nullptr;    // [B][nHeads0/HG] arrival counters (zero-initialised, self-resetting)
    // diagnostics (MFMA decode kernel): 8 u64 s_memrealtime stamps per workgroup, index
    // (b * splitGrid + chunk) * headGroups + group: [0] entry, [1] DMA issued, [2] first tile
    // landed, [3] key loop done, [4] waves merged, [5] split hand-off / combine done, [6] 1 if
    // this workgroup combined the chunks (wave 0's view)
    unsigned long long *trace = nullptr;
};

// Tensor-parallel partial-sum exchange fused into the tail of the kernel that produces the partial
// (wo / w2 GEMV, argmax), replacing a separate all-reduce kernel per residual update (reference:
// cast to the ZQ pipe + SYNC_NODE_SLICES + merge-add, llm.cpp:308-314, nn-network.cpp:537-569).
// Every rank pushes its values straight into each peer's receive region as 8-byte words
// {payload u32, epoch u32} (one atomic store carries data and flag: no fence, no flag word, no
// remote read), then polls its own region until every peer's word carries the current epoch and
// sums all ranks' values in rank order, so every rank gets bitwise the same result. The regions
// live in uncached device memory (xgmi_comm.cpp), so a poll always reads HBM, never a stale line.
// Receive layout: recv[p] + (parity * world + sender) * stride + word; parity = epoch & 1.
// Epochs are per exchange element (per 32-element block in Q80 mode), counted on each rank in
// local memory: every rank runs the same exchange sequence, so the epochs agree.
constexpr int kTpMaxRanks = 16;
struct TpXchg {
    uint64_t *recv[kTpMaxRanks] = {};  // each rank's receive region (peer-mapped)
    unsigned *epochs = nullptr;         // local per-element (per-block) epoch counters, zeroed
    int *error = nullptr;               // local timeout flag (set when a peer never arrived)
    long long stride = 0;               // words per (parity, sender)
    long long timeoutTicks = 0;         // s_memrealtime ticks (100 MHz)
    int rank = 0, world = 1;
    int q80 = 0;                        // exchange Q80 blocks (the reference's ZQ wire format)
    // measured sync (ForwardStats::syncMs): when set, every wave that had to wait for a peer's
    // words raises this word to its waiting time in s_memrealtime ticks (10 ns), so the word holds
    // the longest wait of this exchange (tpWaitReport)
    unsigned *ticks = nullptr;
    // exchange span (DL_SYNC_MEASURE=2): the longest exchange tail of a workgroup of this exchange
    // (its first push to its last summed store), s_memrealtime ticks, atomic max
    unsigned *span = nullptr;
    // compute-only rank (makeComputeOnlyComm): nothing crosses a link, every peer contributes
    // zeros - a TP-N rank's kernels timed on one GPU without the exchange
    int loopback = 0;
};

// EPI_ARGMAX: each workgroup's (value, row) winner goes to partV / partI[workgroup]; the last to
// arrive (counter, reset by it) reduces them in workgroup order, trades the slice winner with the
// other ranks over GemvArgs::tp (world > 1: the argmax winners region, rows start at vocabStart)
// and writes ids[0] (CHAIN: also tokens[0], hist[pos[0]] and pos[0] += 1, as ArgmaxArgs).
struct ArgmaxTail {
    int *ids = nullptr, *tokens = nullptr, *pos = nullptr, *hist = nullptr;
    float *partV = nullptr;
    int *partI = nullptr, *counter = nullptr;
    int vocabStart = 0;
};

struct GemvArgs {
    // weights: Q40 tiled (see Q40Tiling; `lanes` must be the tiling's L) or F32 [rows][n]
    const uint8_t *qs = nullptr;
    const uint16_t *wd = nullptr;
    const float *wf = nullptr;
    int rows = 0, n = 0;
    int passes = 1;  // row passes per workgroup (rows per WG = passes * 256 / L)
    int lanes = 0;   // lanes per row (0 = auto from n)
    // PRO_GLOBAL, Q40 weights: Q80 activations [B][n] int8 + [B][n/32] (d, sum of q)
    const int8_t *aq = nullptr;
    const float2 *as = nullptr;
    // prologue / f32 input
    const float *in = nullptr;    // [B][ldIn]
    int ldIn = 0;
    const float *addIn = nullptr; // PRO_RESNORM: residual delta added to `in` (may be null)
    float *xNext = nullptr;       // PRO_RESNORM: receives in+addIn (written by workgroup 0)
    const float *normW = nullptr; // PRO_RESNORM: rms weights (null = no norm)
    float eps = 1e-5f;
    // epilogue
    float *out = nullptr;
    int ldOut = 0;
    int act = 1;                  // EPI_ACT: 0 = GELU, 1 = SiLU
    int8_t *oq = nullptr;         // EPI_ACT_Q80 outputs [B][ldOut] + [B][ldOut/32]
    float2 *os = nullptr;
    // EPI_QKV
    int q0 = 0, kv0 = 0, hs = 0, seqLen = 0;
    int kvMul = 1;                // query heads per KV head (fused attention block: KV groups of the rows)
    const float2 *rope = nullptr; // [seqLen][hs/2] (cos, sin)
    const int *pos = nullptr;     // per batch row
    const int *slot = nullptr;
    void *kcache = nullptr;       // layer base: [slot][nKv][seqLen][hs] (or a page pool: kvOff)
    void *vcache = nullptr;
    KvMap kvMap;
    int kvBf16 = 1;
    // EPI_STORE_TP (Q40 GEMV): the partial rows are all-reduced over the tensor-parallel ranks in
    // the kernel tail before `out` is written (exchange element = b * ldOut + row)
    TpXchg tp;
    ArgmaxTail am;  // EPI_ARGMAX
    PrenormOut rq;  // EPI_RESQ_TP
    const float *sspIn = nullptr;  // PRO_PRENORM: the producer's per-workgroup sums of squares
    int nSsp = 0;                  //   (<= 256) summed in order; aq / as hold its Q80 blocks
    // diagnostics (gemvQ40Kernel): when set, workgroup g writes 8 u64 at trace[8g..]: s_memrealtime
    // at entry, prologue done, exit, (HW_ID << 32 | XCC_ID), prologue loads landed (early path),
    // first ring slot consumed (thread 0's view)
    unsigned long long *trace = nullptr;
};

// Batched Q40 matmul on MFMA (1..64 tokens per launch): GemvArgs `e` carries the weights (tiled,
// `lanes` = tiling L) and the epilogue fields; activations are f16 [>= roundup(M,16)][n] (`x`,
// rows past M are read but their outputs dropped); split-K partials + per-tile counters
// (zero-initialised, reset by the kernel) when splits > 1. EPI_ACT_F16 writes SwiGLU as f16 to outH.
struct GemmArgs {
    GemvArgs e;
    const _Float16 *x = nullptr;
    _Float16 *outH = nullptr;
    int M = 0;
    int splits = 1;
    float *part = nullptr;
    size_t partFloats = 0;  // capacity of `part` (0: unchecked); launchers refuse a launch beyond it
    int *counters = nullptr;
    // EPI_RES (producer of the next norm's input, wo / w2 at TP1): x' = resIn + out -> resOut (f32,
    // [M][ldOut]), resX = x' * resW as f16 (the norm's per-column half) and per 64-row tile the
    // partial sum of squares ssOut[tile * ldSS + t]: the RMS reduction is left to the consumer.
    const float *resIn = nullptr;
    float *resOut = nullptr;
    const float *resW = nullptr;
    _Float16 *resX = nullptr;
    float *ssOut = nullptr;
    // consumer side (x = a producer's resX): ssIn != null -> each output row t is scaled by
    // 1 / sqrt(sum_j ssIn[j * ldSS + t] / n + eps) (ssTiles partials, summed in tile order)
    const float *ssIn = nullptr;
    int ssTiles = 0, ldSS = 0;
    // tensor parallel (narrow kernel, wo / w2): the final tile [M][64 rows] is all-reduced over the
    // ranks in the epilogue (e.tp: f32 or Q80 blocks, summed in rank order) before EPI_RES / STORE
    int tpx = 0;
    // batch-invariant launch: the narrow gemmQ40Kernel whatever M (no wide or 16-lane variant), so
    // a token row's reduction order does not depend on the launch's token count (splits: the caller's)
    int fixed = 0;
};
void launchGemmQ40(const GemmArgs &a, int epi, hipStream_t s);
// Same contract for F32 weights (`e.wf` [rows][n] row-major; EPI_ACT_Q80 not supported).
void launchGemmF32(const GemmArgs &a, int epi, hipStream_t s);
// Tile / split-K plan of one matrix (rt = 16-row tiles per wave: 64 * rt rows per workgroup).
struct GemmPlan {
    int rt = 1, tiles = 0, splits = 1;
};
constexpr int kGemmMaxTokens = 128;    // tokens per narrow Q40 GEMM launch (16, 32, 64 or 128 padded)
// Wide Q40 GEMM (gemm_wide.hip): launches of >= gemmWideMin() tokens (default 65; DL_GEMM_WIDE=0
// disables) run 128 x 128 tiles over every token tile of the launch; any token count per launch
// (activation operand padded to whole 128-token tiles).
bool gemmWideOn();
int gemmWideMin();
bool gemmUsesWide(int M);
int gemmWideSplits(int rows, int n, int M);
size_t gemmWidePartFloats(int rows, int n, int maxTokens);
int gemmWideCounters(int rows, int maxTokens);
void launchGemmWide(const GemmArgs &a, int epi, hipStream_t s);
// whether a narrow launch of M tokens can run the tensor-parallel tile exchange (GemmArgs::tpx)
bool gemmTpxFits(int M, int world, bool q80);
// split-K counter ints for any launch of up to maxTokens tokens on a matrix of `rows`
int gemmCounterInts(int rows, int maxTokens);
constexpr int kGemmF32MaxTokens = 64;  // tokens per F32 GEMM launch (16, 32 or 64 padded)
GemmPlan gemmPlan(int rows, int n, int M);
bool gemmSupported(int n);  // input width a multiple of 32 (whole Q40 blocks)
// K splits of a launch; lanes = the matrix's tiling L (16: the 16-block-chunk kernel's rule)
int gemmSplits(int rows, int n, int M, int lanes = 0);
// split-K partial floats for any launch of up to maxTokens tokens on this matrix
size_t gemmPartFloats(int rows, int n, int maxTokens);
// ... for the launches of a batch-invariant engine (GemmArgs::fixed: narrow, <= 128 tokens each)
size_t gemmPartFloatsFixed(int rows, int n);
// token rows one GEMM launch of M (1..128) tokens reads from its f16 activation operand (16/32/64/128)
int gemmTokenPad(int M);
// Residual add + RMS norm (normW may be null: no norm) of M rows -> f16:
// in/addIn/xNext [M][ldIn] f32 -> out [M][n] f16 (xNext = in + addIn when set).
void launchNormF16(const GemvArgs &a, _Float16 *out, int M, hipStream_t s);


// B = batch rows in this launch (1, 2 or 4); q40 = weight format.
void launchGemv(const GemvArgs &a, int B, int pro, int epi, bool q40, hipStream_t s);
// The wo GEMV of one decode row with the layer's attention in its prologue (PRO_ATTN): `at` is the
// row's attention (every head of the rank, one chunk over the whole context); epi EPI_STORE or
// EPI_STORE_TP. Supported: gemvAttnSupported (Q40, head size 128, query heads per KV head 1/2/4/8).
bool gemvAttnSupported(const GemvArgs &a, const AttnArgs &at, int epi);
void launchGemvAttn(const GemvArgs &a, const AttnArgs &at, int epi, hipStream_t s);
struct GemvResidency;
GemvResidency gemvAttnResidency(const GemvArgs &a, const AttnArgs &at, int epi);
// Co-residency of one GEMV launch on the current device: its grid and the most workgroups of that
// kernel (at its LDS size) the device holds at once (occupancy per CU x CUs). A kernel whose
// workgroups spin on peers (EPI_STORE_TP) is deadlock-free only if grid <= maxResident.
struct GemvResidency {
    int grid = 0, maxResident = 0;
};
GemvResidency gemvResidency(const GemvArgs &a, int B, int pro, int epi, bool q40);
// Rows handled by one lane group (2 at batch 1: the activation loads are shared by 2 rows).
__host__ __device__ constexpr int gemvRowGroup(int B, bool q40) { return q40 ? 2 : 1; }
// Lanes cooperating on one weight row for a given input width, row count and batch.
int gemvLanesPerRow(int n, int rows, int B, bool q40);
// Rows per workgroup and pass.
inline int gemvRowsPerPass(int n, int rows, int B, bool q40) {
    return 256 / gemvLanesPerRow(n, rows, B, q40) * gemvRowGroup(B, q40);
}
// Dynamic LDS bytes a gemv launch needs.
size_t gemvLdsBytes(int n, int B, bool q40, int rowsPerWg, int pro);
// Passes (row groups per lane group) for a launch: Q40 ring kernel -> enough that the whole grid is
// resident at once (DL_GEMV_RESIDENT workgroups, default 512); ACT_Q80 -> whole Q80 blocks per WG.
// lanes: the matrix's tiling L when known (0: the GEMV's own choice for this shape).
int gemvDefaultPasses(int n, int rows, int B, bool q40, int epi, int lanes = 0);

void launchAttention(const AttnArgs &a, int B, hipStream_t s);
// MFMA decode attention (attn_mfma.hip): bf16 cache, head size 128, kvMul 1/2/4/8; launchAttention
// takes it for caches of >= 1024 positions (DL_ATTN_MFMA=1: always, 0: never).
bool attnMfmaSupported(const AttnArgs &a);
bool attnUsesMfma(const AttnArgs &a);
void launchAttentionMfma(const AttnArgs &a, int B, hipStream_t s);
void launchAttentionValu(const AttnArgs &a, int B, hipStream_t s);  // the VALU kernel (attnTask)
// Prefill rows with LDS-DMA staged K / V (attn_mfma.hip; other shapes take the register-staged
// kernels.hip kernel): bf16 cache, head size 128, kvMul 1..16.
bool attnPrefillDmaSupported(const AttnArgs &a);
void launchAttentionPrefillDma(const AttnArgs &a, int nRows, hipStream_t s);

// Fused attention block of one decode row (B = 1): the qkv GEMV (norm prologue, RoPE + KV append),
// the decode attention and the wo GEMV in ONE launch, as three workgroup roles
//   [0, gq) qkv rows | [gq, gq + ga) attention tasks | [gq + ga, gq + ga + gw) wo rows,
// handing off in-launch through write-through stores and monotonic arrival counters (decode_dev.h
// BlockSync): attention tasks wait for their KV group's qkv workgroups, wo workgroups issue their
// weight ring first and then wait for every head group's output. Removes two kernel boundaries
// and the attention / wo start-up latency per layer. Requires the whole grid co-resident
// (attnBlockResidency) - every wait is bounded and raises `error` instead of hanging.
struct AttnBlockArgs {
    GemvArgs qkv;                 // PRO_RESNORM + EPI_QKV (lanes = the qkv tiling's L, kvMul set)
    AttnArgs at;                  // one row; outQ / outS = the wo input
    GemvArgs wo;                  // PRO_GLOBAL + EPI_STORE (or EPI_STORE_TP: wo.tp set)
    int hg = 1;                   // query heads per attention workgroup (attnBlockHG)
    int layer = 0, nLayers = 1;
    const unsigned *epoch = nullptr;  // per-forward epoch (1, 2, ...), incremented by launchEmbedding
    unsigned *qkvCnt = nullptr;       // [kv groups * 64] monotonic counters, one per 256-B line (zeroed once)
    const unsigned *qkvExpect = nullptr;  // [kv groups] qkv workgroups per group (attnBlockExpect)
    unsigned *attnCnt = nullptr;      // [1] monotonic counter (zeroed once)
    unsigned *attnFlag = nullptr;     // [8 * 64] per-XCD step-done flags (zeroed once)
    int *error = nullptr;             // wait timeout flag (zeroed once)
    long long timeoutTicks = 200LL * 1000 * 1000;  // 2 s of s_memrealtime (100 MHz)
    // diagnostics: 8 u64 per workgroup (qkv / wo: GemvArgs::trace layout + [6] wait done; attention:
    // [0] entry, [1] wait done, [2] compute done, [3] exit, [7] role 1 | 16 if it wrote the output)
    unsigned long long *trace = nullptr;
};
int attnBlockHG(const AttnArgs &a);  // query heads per attention workgroup (256 threads, one row)
// Launch geometry; fn == null when (qkv lanes, wo lanes, head size, HG) has no compiled instance.
struct AttnBlockPlan {
    const void *fn = nullptr;
    int gq = 0, ga = 0, gw = 0;
    size_t lds = 0;
};
AttnBlockPlan attnBlockPlan(const AttnBlockArgs &a, bool tp);
// qkv workgroups touching each KV group (host side of the counters' targets): out[g], g < nKv.
void attnBlockExpect(const GemvArgs &qkv, int nKv, unsigned *out);
GemvResidency attnBlockResidency(const AttnBlockArgs &a, bool tp);
void launchAttnBlock(const AttnBlockArgs &a, bool tp, hipStream_t s);

// Fused FFN block of one decode row at a tensor-parallel rank with the pre-normalized hand-off
// (ffn_block.hip): w13 (PRO_PRENORM, SwiGLU epilogue, hidden rows stored write-through as f32 or
// Q80) and w2 (EPI_RESQ_TP exchange tail) in ONE launch as two workgroup roles
//   [0, g13) w13 rows | [g13, g13 + g2) w2 rows.
// The w2 workgroups issue their weight ring at entry - it streams while w13 runs - then wait for
// every w13 workgroup (a monotonic counter, per-XCD "phase done" flags as the attention block's)
// and read the hidden rows write-through. Removes a kernel boundary and w2's start-up latency per
// layer. Requires the whole grid co-resident (ffnBlockResidency); waits are bounded (error word).
struct FfnBlockArgs {
    GemvArgs w13;                 // PRO_PRENORM + EPI_ACT (f32 hidden) or EPI_ACT_Q80 (hQ80)
    GemvArgs w2;                  // EPI_RESQ_TP: PRO_RESNORM (f32 hidden, no norm) or PRO_GLOBAL (Q80)
    int hQ80 = 0;
    int layer = 0, nLayers = 1;
    const unsigned *epoch = nullptr;  // per-forward epoch of the FFN block (incremented by launchEmbedding)
    unsigned *cnt = nullptr;          // [1] monotonic w13 arrivals (zeroed once)
    unsigned *flag = nullptr;         // [8 * 64] per-XCD "w13 phase done" step flags (zeroed once)
    int *error = nullptr;             // wait timeout flag (codes 7 data, 8 ring start)
    long long timeoutTicks = 200LL * 1000 * 1000;
};
struct FfnBlockPlan {
    const void *fn = nullptr;
    int g13 = 0, g2 = 0;
    size_t lds = 0;
};
FfnBlockPlan ffnBlockPlan(const FfnBlockArgs &a);
GemvResidency ffnBlockResidency(const FfnBlockArgs &a);
void launchFfnBlock(const FfnBlockArgs &a, hipStream_t s);

// Fused-exchange self-test (tp_check.hip): out[el] = sum over ranks of (val_rank + el % 1024) for
// el < n (n <= x.stride), through the transport of the fused exchange; every rank must call it.
void launchTpSelfTest(const TpXchg &x, float *out, int n, float val, hipStream_t s);

// Prefill rows on MFMA (bf16 caches): blocks of attnPrefillRowsPerBlock(kvMul) consecutive rows
// must share one slot (positions arbitrary, causal per row); counters >= blocks x KV heads.
void launchAttentionPrefill(const AttnArgs &a, int nRows, hipStream_t s);
int attnPrefillRowsPerBlock(int kvMul);
bool attnPrefillSupported(int hs, int kvMul, bool kvBf16);
int attnSplitGrid(int seqLen, bool shortChunks = false);
// single decode rows of at most kAttnShortLen keys split into chunks of kAttnShortChunk (attnSplit)
constexpr int kAttnShortLen = 512, kAttnShortChunk = 128;
// Fewest keys per attention split (DL_ATTN_CHUNK, default 256): sets the split grid of a context.
int attnChunkMin();
int attnChunkMax(int seqLen, int splitGrid);

// epoch (optional): one thread increments it - the per-forward epoch of the fused attention block.
// sync / nSync (optional): the measured-sync slots of the previous forward (syncFoldWords layout)
// are folded into their running totals, then cleared for this forward.
void launchEmbedding(const float *table, const int *tokens, float *x, int dim, int B, hipStream_t s,
                     unsigned *epoch = nullptr, unsigned *sync = nullptr, int nSync = 0,
                     const PrenormOut *pre = nullptr);  // B == 1: also the first layer's PRO_PRENORM input
// Measured-sync slot layout (u32 words) for S slots: [0, S) the longest peer wait of each exchange,
// [S, 2S) the longest exchange tail (span), [2S, 6S) a u64 stamp pair per slot (a separate
// collective), then 4 u64 running totals over folded forwards: wait, span, stamped, forwards.
inline size_t syncFoldWords(int S) { return 6 * (size_t)S + 8; }
// One s_memrealtime stamp (100 MHz) into *p: brackets a separate collective for the measured sync.
void launchStamp(unsigned long long *p, hipStream_t s);
// Parallel argmax over [B][vocab]; partials need B*256 floats + ints, counters B ints (zeroed).
// When `tokens` is non-null the result is also fed back (tokens[b] = id; hist[b][pos] = id; pos += 1).
struct ArgmaxArgs {
    const float *logits = nullptr;
    int vocab = 0;
    int *ids = nullptr;
    float *partV = nullptr;
    int *partI = nullptr;
    int *counters = nullptr;
    int *tokens = nullptr, *pos = nullptr, *hist = nullptr;
    int seqLen = 0;
    // tensor parallel: `logits` is this rank's vocab slice starting at vocabStart; the per-row
    // (value, index) winners are exchanged (tp.world > 1) and every rank picks the same global one
    TpXchg tp;
    int vocabStart = 0;
    // tensor parallel over separate collectives: the row's slice winner {value, global index bits}
    // goes to pairs[2b .. 2b+1] and nothing else; after an all-gather of the pairs,
    // launchArgmaxPick picks the same global winner on every rank
    float *pairs = nullptr;
};
// Device sampling of B rows of full-vocabulary logits (the reference's Sampler::sample:
// logits / temperature -> softmax -> coin -> multinomial in index order, or top-p: candidates
// >= (1 - p) / (V - 1), descending by probability, cut where the cumulative mass first exceeds p,
// draw r = coin * nucleus mass). spec[b] = (temperature, topp, coin, -): temperature 0 -> argmax,
// < 0 -> no draw (ids[b] = -1). sampleGroups(B) workgroups per row run 8 dependent phases; the
// top-p cut and the draw are 11/11/10-bit radix searches over the order-preserving key of
// logit / temperature. The scratch must be zero-initialised once; every call leaves it zero.
constexpr int kSampleMaxGroups = 64;
constexpr int kSampleStateWords = 16;
int sampleGroups(int B);
struct SampleScratch {
    float *hist = nullptr;  // [rows][G][2048] partial histograms (G = sampleGroups(rows))
    float *part = nullptr;  // [B][kSampleMaxGroups]
    int *partI = nullptr;   // [B][kSampleMaxGroups]
    uint32_t *state = nullptr;  // [B][kSampleStateWords]
    // partial-histogram slots for any batch of up to B rows
    static size_t histFloats(int B) {
        size_t m = 0;
        for (int r = 1; r <= B; r++) m = std::max(m, (size_t)r * sampleGroups(r));
        return m * 2048;
    }
    static size_t bytes(int B) { return (histFloats(B) + (size_t)B * (2 * kSampleMaxGroups + kSampleStateWords)) * 4; }
    void carve(void *base, int B) {
        float *f = static_cast<float *>(base);
        hist = f;
        part = f + histFloats(B);
        partI = reinterpret_cast<int *>(part + (size_t)B * kSampleMaxGroups);
        state = reinterpret_cast<uint32_t *>(partI + (size_t)B * kSampleMaxGroups);
    }
};
struct SampleArgs {
    const float *logits = nullptr;
    int vocab = 0;
    const float4 *spec = nullptr;
    int *ids = nullptr;
    SampleScratch scratch;
};
void launchSample(const SampleArgs &a, int B, hipStream_t s);

// Round-trip f32 partial sums through Q80 blocks in place (the reference's ZQ cast before the
// exchange) - used ahead of a plain all-reduce when the fused exchange is not available.
void launchQ80Roundtrip(float *x, size_t n, hipStream_t s);
void launchArgmax(const ArgmaxArgs &a, int B, hipStream_t s);
// all[p * 2B + 2b ..]: rank p's pairs of row b (ArgmaxArgs::pairs, all-gathered over W ranks)
void launchArgmaxPick(const ArgmaxArgs &a, const float *all, int B, int W, hipStream_t s);
// logits gathered rank-major [nRanks][B][vocab0] -> row-major [B][vocab]
void launchUnshardLogits(const float *in, float *out, int nRanks, int B, int vocab0, hipStream_t s);

// Synthetic weights: random Q40 nibbles with scale ~ scale*(0.5..1.5), f32 uniform(-a,a), or constant.
void launchFillQ40(uint8_t *qs, uint16_t *d, size_t nBlocks, float scale, uint64_t seed, hipStream_t s);
void launchFillF32Uniform(float *p, size_t n, float amp, uint64_t seed, hipStream_t s);
void launchFillF32Const(float *p, size_t n, float v, hipStream_t s);

// Load every code object of this library onto the current device now. HIP loads a translation
// unit's code object at the first launch of one of its kernels; on the CLI that cost landed in the
// first prompt chunk (+4.7 ms) and the first decode token (+3.2 ms). Engines call this once at
// construction, after the weights are resident.
void preloadModules();

}  // namespace hipk
}  // namespace dl
