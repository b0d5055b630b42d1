// Host-visible launchers for the gfx950 kernels (csrc/hip/kernels.hip).
//
// Kernel map vs the reference op inventory:
//   gemv<PRO_RESNORM, EPI_QKV>   OP_MERGE_ADD + OP_INV_RMS + OP_RMS_NORM + OP_CAST(Q80)
//                                + 3x OP_MATMUL (q,k,v) + 2x OP_ROPE_LLAMA + 2x OP_SHIFT
//   attention + attnCombine      OP_MULTIHEAD_ATT (flash-decoding split over the sequence)
//   gemv<PRO_QUANT, EPI_STORE>   OP_CAST(Q80) + OP_MATMUL (wo, w2)
//   gemv<PRO_RESNORM, EPI_ACT>   OP_MERGE_ADD + norm + OP_MATMUL (w1, w3) + OP_SILU/GELU + OP_MUL
//   gemv<PRO_RESNORM, EPI_STORE> final norm + OP_MATMUL (logits)
//   embedding                    OP_EMBEDDING
//   argmaxRows                   greedy sampling on device
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dl {
namespace hipk {

enum Prologue : int { PRO_QUANT = 0, PRO_RESNORM = 1 };
enum Epilogue : int { EPI_STORE = 0, EPI_ACT = 1, EPI_QKV = 2 };

struct GemvArgs {
    // weights: Q40 repacked (qs [rows][nb][16], d [rows][nb] f16) or F32 [rows][n]
    const uint8_t *qs = nullptr;
    const uint16_t *wd = nullptr;
    const float *wf = nullptr;
    int rows = 0, n = 0;
    int passes = 1;  // row passes per workgroup (rows per WG = passes * 256 / L)
    // prologue
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
    // EPI_QKV
    int q0 = 0, kv0 = 0, hs = 0, seqLen = 0;
    const float2 *rope = nullptr; // [seqLen][hs/2] (cos, sin)
    const int *pos = nullptr;     // per batch row
    const int *slot = nullptr;
    void *kcache = nullptr;       // layer base: [slot][seqLen][kv0]
    void *vcache = nullptr;
    int kvBf16 = 1;
};

// B = batch rows in this launch (1, 2 or 4); q40 = weight format.
void launchGemv(const GemvArgs &a, int B, int pro, int epi, bool q40, hipStream_t s);
// Rows per workgroup for a given n (used by the host to size partial passes).
int gemvLanesPerRow(int n, bool q40);
// Dynamic LDS bytes a gemv launch needs.
size_t gemvLdsBytes(int n, int B, bool q40, int rowsPerWg);

struct AttnArgs {
    const float *q = nullptr;   // [B][ldq], rotated queries
    int ldq = 0;
    const void *kcache = nullptr, *vcache = nullptr;  // layer base [slot][seqLen][kv0]
    const int *pos = nullptr, *slot = nullptr;
    int nHeads0 = 0, kvMul = 1, hs = 0, kv0 = 0, seqLen = 0;
    int splitGrid = 1;          // max sequence splits (grid.y)
    int chunkMax = 256;         // LDS capacity in positions per split
    float *partO = nullptr;     // [B][nHeads0][splitGrid][hs]
    float *partML = nullptr;    // [B][nHeads0][splitGrid][2]
    float *out = nullptr;       // [B][ldOut] (combined output)
    int ldOut = 0;
    int kvBf16 = 1;
};
void launchAttention(const AttnArgs &a, int B, hipStream_t s);
int attnSplitGrid(int seqLen);
int attnChunkMax(int seqLen, int splitGrid);

void launchEmbedding(const float *table, const int *tokens, float *x, int dim, int B, hipStream_t s);
void launchArgmax(const float *logits, int vocab, int B, int *outIds, hipStream_t s);
// logits gathered rank-major [nRanks][B][vocab0] -> row-major [B][vocab]
void launchUnshardLogits(const float *in, float *out, int nRanks, int B, int vocab0, hipStream_t s);
// Decode chaining: tokens[b] = ids[b]; pos[b] += 1
void launchAdvance(const int *ids, int *tokens, int *pos, int B, hipStream_t s);

// Synthetic weights: random Q40 nibbles with scale ~ scale*(0.5..1.5), f32 uniform(-a,a), or constant.
void launchFillQ40(uint8_t *qs, uint16_t *d, size_t nBlocks, float scale, uint64_t seed, hipStream_t s);
void launchFillF32Uniform(float *p, size_t n, float amp, uint64_t seed, hipStream_t s);
void launchFillF32Const(float *p, size_t n, float v, hipStream_t s);

}  // namespace hipk
}  // namespace dl
