// gfx950 (MI355X / CDNA4) kernels for decode and small-batch forward passes.
//
// Design notes (see csrc/hip/kernels.h for the op map):
// * Weights stream straight from HBM into VGPRs (16 B per lane per Q40 block); each lane's first
//   KMAX blocks are issued BEFORE the prologue so HBM latency overlaps the norm/quant work
//   (GEMV regime: operands read once, no LDS staging - cdna_hip_programming.md §5 table,
//   "GEMV / M <= 16 decode weights"). Loads are non-temporal (read-once weights).
// * Activations are Q80: either produced once per workgroup in LDS (norm prologue) or produced
//   upstream in the epilogue of the previous kernel and read straight from global (L2-resident).
//   The inner product is v_dot4_i32_i8 on nibbles with the "-8" folded into a per-block sum:
//   sum((q-8)*x) = dot(q, x) - 8*sum(x).
// * Row reductions use DPP (quad_perm / row_ror) inside 16-lane rows, shfl only across rows.
// * Every per-token input (token id, position, KV slot) is read from device memory so the whole
//   forward pass is captured once per batch size in a hipGraph and replayed.
// * Cross-workgroup hand-offs (attention split combine, argmax) follow the agent-scope
//   release/acquire counter recipe (cdna_hip_programming.md §5 "In-launch split-K reduction").
#include "../core/common.h"
#include "device_comm.h"
#include "device_common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <type_traits>

namespace dl {
namespace hipk {

using namespace dl::dev;

static constexpr int kThreads = 256;
static constexpr int kMaxHeadSize = 128;  // RoPE rows staged in LDS by the QKV epilogue
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

__host__ __device__ static inline size_t alignUp(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Tuning knob (experiments only): DL_GEMV_MIN_LANES=32 forces at least 32 lanes per row.
static int minLanesOverride() {
    static const int v = [] {
        const char *e = getenv("DL_GEMV_MIN_LANES");
        return e ? atoi(e) : 0;
    }();
    return v;
}

int gemvLanesPerRow(int n, int rows, int B, bool q40) {
    int L;
    if (q40) {
        // Ring kernel: the fewest lanes per row (longest per-lane step sequence, so the whole
        // ring is real work, cheapest reduction, fewest redundant prologues) that still spreads
        // over >= 3/4 of the CUs (measured: qkv 6144x4096 7.1 us at L=16 / 192 WGs vs 8.3 us at
        // L=32 / 384 WGs; wo 4096x4096 4.2 us at L=32 / 256 WGs vs 4.9 us at L=16 / 128 WGs).
        const int groups = (rows + 1) / 2;
        L = 16;
        while (L < 64 && (size_t)groups * L / kThreads < 192) L *= 2;
    } else {
        const int n4 = n / 4;
        L = n4 >= 2048 ? 64 : (n4 >= 512 ? 32 : 16);
        // skinny shards (tensor parallel): fewer rows per workgroup so the grid still covers the CUs
        while (L < 64 && rows / (kThreads / L * gemvRowGroup(B, q40)) < 256) L *= 2;
    }
    const int mo = minLanesOverride();
    if (mo > L) L = mo > 64 ? 64 : mo;
    return L;
}

struct GemvLds {
    size_t scratch, rope, res, hbuf, act, sc, total;
};

__host__ __device__ static GemvLds gemvLayout(int n, int B, bool q40, int rowsPerWg, int pro) {
    GemvLds l;
    size_t off = 0;
    l.scratch = off;
    off += 64 * sizeof(float);
    l.rope = off;  // RoPE rows of the batch's positions (QKV epilogue of the Q40 ring kernel)
    off += (size_t)B * (kMaxHeadSize / 2) * sizeof(float2);
    l.res = off;
    off = alignUp(off + (size_t)B * rowsPerWg * sizeof(float), 16);
    l.hbuf = off;
    off = alignUp(off + (size_t)B * (rowsPerWg / 2) * sizeof(float), 16);
    l.act = off;
    if (pro == PRO_RESNORM || q40) {
        if (q40) {
            off = alignUp(off + (size_t)B * n, 16);
            l.sc = off;
            off = alignUp(off + (size_t)B * (n / 32) * sizeof(float2), 16);
        } else {
            off = alignUp(off + (size_t)B * n * sizeof(float), 16);
            l.sc = off;
        }
    } else {
        l.sc = off;
    }
    l.total = off;
    return l;
}

Q40Tiling q40Tiling(int rows, int n, int L) {
    Q40Tiling t;
    t.L = L;
    t.NG = kThreads / L;
    const int nb = n / 32;
    t.K = (nb + L - 1) / L;
    t.groups = (rows + 2 * t.NG - 1) / (2 * t.NG);
    t.chunks = (size_t)t.groups * t.K;
    t.qsBytes = t.chunks * 2 * kThreads * 16;
    t.dBytes = t.chunks * kThreads * 4;
    return t;
}

// Tiled layout writer over pass groups [gBegin, gEnd): src(row, j, qs16Out) copies block j of
// `row` (16 nibble bytes) and returns its f16 scale.
template <typename Src>
static void tileQ40Groups(const Src &src, int rows, int nb, const Q40Tiling &t, int gBegin, int gEnd,
                          uint8_t *qsOut, uint32_t *dOut) {
    const int L = t.L;
    for (int g = gBegin; g < gEnd; g++)
        for (int k = 0; k < t.K; k++) {
            const size_t c = (size_t)g * t.K + k;
            for (int tid = 0; tid < kThreads; tid++) {
                const int gi = tid / L, li = tid % L, j = li + k * L;
                const int row0 = 2 * (g * t.NG + gi);
                uint32_t dd = 0;
                for (int r = 0; r < 2; r++) {
                    uint8_t *dst = qsOut + ((c * 2 + r) * kThreads + tid) * 16;
                    const int row = row0 + r;
                    if (row < rows && j < nb)
                        dd |= (uint32_t)src(row, j, dst) << (16 * r);
                    else
                        std::memset(dst, 0, 16);
                }
                dOut[c * kThreads + tid] = dd;
            }
        }
}

// Pass groups are independent output ranges: split them over host threads (a 405B TP8 shard is
// ~28 GB of Q40 per rank, so the repack at load time must not be single-threaded).
template <typename Src>
static void tileQ40Parallel(const Src &src, int rows, int n, int L, uint8_t *qsOut, uint32_t *dOut) {
    const Q40Tiling t = q40Tiling(rows, n, L);
    const int nb = n / 32;
    const int hw = (int)std::thread::hardware_concurrency();
    const int nThreads = std::max(1, std::min({hw > 0 ? hw : 1, 32, t.groups / 4}));
    if (nThreads > 1) {
        std::vector<std::thread> pool;
        for (int ti = 0; ti < nThreads; ti++)
            pool.emplace_back([&, ti] {
                const int g0 = (int)((long)t.groups * ti / nThreads), g1 = (int)((long)t.groups * (ti + 1) / nThreads);
                tileQ40Groups(src, rows, nb, t, g0, g1, qsOut, dOut);
            });
        for (auto &th : pool) th.join();
        return;
    }
    tileQ40Groups(src, rows, nb, t, 0, t.groups, qsOut, dOut);
}

void tileQ40(const uint8_t *qs, const uint16_t *d, int rows, int n, int L, uint8_t *qsOut, uint32_t *dOut) {
    const size_t nb = (size_t)n / 32;
    auto src = [&](int row, int j, uint8_t *dst) -> uint16_t {
        const size_t blk = (size_t)row * nb + j;
        std::memcpy(dst, qs + blk * 16, 16);
        return d[blk];
    };
    tileQ40Parallel(src, rows, n, L, qsOut, dOut);
}

void tileQ40AoS(const uint8_t *const *rowBlocks, int rows, int n, int L, uint8_t *qsOut, uint32_t *dOut) {
    // file layout: per block an f16 scale then 16 nibble bytes (18 B, unaligned)
    auto src = [&](int row, int j, uint8_t *dst) -> uint16_t {
        const uint8_t *b = rowBlocks[row] + (size_t)j * 18;
        std::memcpy(dst, b + 2, 16);
        uint16_t dv;
        std::memcpy(&dv, b, 2);
        return dv;
    };
    tileQ40Parallel(src, rows, n, L, qsOut, dOut);
}

int gemvDefaultPasses(int n, int rows, int B, bool q40, int epi) {
    static const int resident = [] {
        const char *e = getenv("DL_GEMV_RESIDENT");
        return e ? atoi(e) : 512;
    }();
    const int rp = gemvRowsPerPass(n, rows, B, q40);
    const int grid0 = (rows + rp - 1) / rp;
    int passes;
    if (q40) {
        passes = (grid0 + resident - 1) / resident;
        if (epi == EPI_ACT_Q80)
            while ((rp * passes) % 64) passes++;
    } else {
        if (epi == EPI_ACT_Q80) return 64 / rp;
        passes = grid0 / 1024;
        passes = passes < 1 ? 1 : (passes > 4 ? 4 : passes);
    }
    return passes;
}

size_t gemvLdsBytes(int n, int B, bool q40, int rowsPerWg, int pro) {
    return gemvLayout(n, B, q40, rowsPerWg, pro).total;
}

// ------------------------------------------------------------------------------------------------
// Prologue: (x + delta) -> RMS norm -> Q80 blocks (or f32) in LDS; workgroup 0 writes x + delta.
// ------------------------------------------------------------------------------------------------
// Quantize (or store) one 8-element chunk c of row b into the LDS activation image.
template <bool Q40>
__device__ __forceinline__ void stageChunk(float (&v)[8], int b, int c, int n, int8_t *sq, float2 *ssc, float *sf) {
    const int nb = n >> 5, tid = threadIdx.x;
    if constexpr (Q40) {
        float amax = 0.f;
#pragma unroll
        for (int i = 0; i < 8; i++) amax = fmaxf(amax, fabsf(v[i]));
        amax = quadMax(amax);  // the 4 lanes of a quad hold one 32-element block
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        int q[8];
        int qsum = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            q[i] = (int)rintf(v[i] * id);
            q[i] = q[i] > 127 ? 127 : (q[i] < -127 ? -127 : q[i]);
            qsum += q[i];
        }
        int2 packed;
        packed.x = packI8x4(q[0], q[1], q[2], q[3]);
        packed.y = packI8x4(q[4], q[5], q[6], q[7]);
        *reinterpret_cast<int2 *>(sq + (size_t)b * n + c * 8) = packed;
        qsum = quadSumI(qsum);
        if ((tid & 3) == 0) ssc[b * nb + (c >> 2)] = make_float2(roundF16(d), (float)qsum);
    } else {
        float *dst = sf + (size_t)b * n + c * 8;
        st4(dst, make_float4(v[0], v[1], v[2], v[3]));
        st4(dst + 4, make_float4(v[4], v[5], v[6], v[7]));
    }
}

// Single global pass: each thread keeps up to PMAX chunks of 8 elements per row in registers
// (n <= 256 * 8 * PMAX); larger inputs fall back to a second pass over L2.
template <int B, bool Q40>
__device__ __forceinline__ void resNormPrologue(const GemvArgs &a, float *scratch, int8_t *sq, float2 *ssc, float *sf,
                                                bool writeX = false) {
    constexpr int PMAX = 4;
    const int n = a.n, tid = threadIdx.x;
    const int nChunks = n >> 3;
    const bool inReg = nChunks <= kThreads * PMAX;
#pragma unroll
    for (int b = 0; b < B; b++) {
        const float *xi = a.in + (size_t)b * a.ldIn;
        const float *yi = a.addIn ? a.addIn + (size_t)b * a.ldIn : nullptr;
        float *xo = ((blockIdx.x == 0 || writeX) && a.xNext) ? a.xNext + (size_t)b * a.ldIn : nullptr;
        float v[PMAX][8];
        float4 nw[PMAX][2];  // norm weights, fetched in the same round trip as x and delta
        float ss = 0.f;
        if (inReg) {
#pragma unroll
            for (int k = 0; k < PMAX; k++) {
                const int c = tid + k * kThreads;
                if (c < nChunks) {
                    if (a.normW) {
                        nw[k][0] = ld4(a.normW + c * 8);
                        nw[k][1] = ld4(a.normW + c * 8 + 4);
                    }
                    float4 v0 = ld4(xi + c * 8), v1 = ld4(xi + c * 8 + 4);
                    if (yi) {
                        const float4 y0 = ld4(yi + c * 8), y1 = ld4(yi + c * 8 + 4);
                        v0.x += y0.x; v0.y += y0.y; v0.z += y0.z; v0.w += y0.w;
                        v1.x += y1.x; v1.y += y1.y; v1.z += y1.z; v1.w += y1.w;
                    }
                    if (xo) {
                        st4(xo + c * 8, v0);
                        st4(xo + c * 8 + 4, v1);
                    }
                    v[k][0] = v0.x; v[k][1] = v0.y; v[k][2] = v0.z; v[k][3] = v0.w;
                    v[k][4] = v1.x; v[k][5] = v1.y; v[k][6] = v1.z; v[k][7] = v1.w;
#pragma unroll
                    for (int i = 0; i < 8; i++) ss += v[k][i] * v[k][i];
                }
            }
        } else {
            for (int i = tid * 4; i < n; i += kThreads * 4) {
                float4 x = ld4(xi + i);
                if (yi) {
                    const float4 y = ld4(yi + i);
                    x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
                }
                ss += x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
                if (xo) st4(xo + i, x);
            }
        }
        float inv = 1.0f;
        if (a.normW) {
            ss = blockSum<kThreads>(ss, scratch);
            inv = 1.0f / sqrtf(ss / (float)n + a.eps);
        }
        if (inReg) {
#pragma unroll
            for (int k = 0; k < PMAX; k++) {
                const int c = tid + k * kThreads;
                if (c < nChunks) {
                    if (a.normW) {
                        const float4 w0 = nw[k][0], w1 = nw[k][1];
                        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                        for (int i = 0; i < 8; i++) v[k][i] = wv[i] * (inv * v[k][i]);
                    }
                    stageChunk<Q40>(v[k], b, c, n, sq, ssc, sf);
                }
            }
            continue;
        }
        for (int c = tid; c < nChunks; c += kThreads) {
            float4 v0 = ld4(xi + c * 8), v1 = ld4(xi + c * 8 + 4);
            if (yi) {
                const float4 y0 = ld4(yi + c * 8), y1 = ld4(yi + c * 8 + 4);
                v0.x += y0.x; v0.y += y0.y; v0.z += y0.z; v0.w += y0.w;
                v1.x += y1.x; v1.y += y1.y; v1.z += y1.z; v1.w += y1.w;
            }
            float w8[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
            if (a.normW) {
                const float4 w0 = ld4(a.normW + c * 8), w1 = ld4(a.normW + c * 8 + 4);
                w8[0] = w0.x; w8[1] = w0.y; w8[2] = w0.z; w8[3] = w0.w;
                w8[4] = w1.x; w8[5] = w1.y; w8[6] = w1.z; w8[7] = w1.w;
            }
            float vv[8] = {w8[0] * (inv * v0.x), w8[1] * (inv * v0.y), w8[2] * (inv * v0.z), w8[3] * (inv * v0.w),
                           w8[4] * (inv * v1.x), w8[5] * (inv * v1.y), w8[6] * (inv * v1.z), w8[7] * (inv * v1.w)};
            stageChunk<Q40>(vv, b, c, n, sq, ssc, sf);
        }
    }
    __syncthreads();
}

// One Q40 block (32 weights) of RG rows against B activation blocks; the activation block is
// loaded once and shared by the RG rows (halves activation traffic at batch 1).
template <int B, int RG>
__device__ __forceinline__ void q40Block(float (&acc)[RG][B], const u32x4 (&w)[RG], const float (&dw)[RG], int j,
                                         int n, int nb, const int8_t *act, const float2 *asc) {
    int lo[RG][4], hi[RG][4];
#pragma unroll
    for (int r = 0; r < RG; r++) {
        lo[r][0] = w[r].x & 0x0F0F0F0F; hi[r][0] = (w[r].x >> 4) & 0x0F0F0F0F;
        lo[r][1] = w[r].y & 0x0F0F0F0F; hi[r][1] = (w[r].y >> 4) & 0x0F0F0F0F;
        lo[r][2] = w[r].z & 0x0F0F0F0F; hi[r][2] = (w[r].z >> 4) & 0x0F0F0F0F;
        lo[r][3] = w[r].w & 0x0F0F0F0F; hi[r][3] = (w[r].w >> 4) & 0x0F0F0F0F;
    }
#pragma unroll
    for (int b = 0; b < B; b++) {
        const int4 *xp = reinterpret_cast<const int4 *>(act + (size_t)b * n + j * 32);
        const int4 xa = xp[0], xb = xp[1];
        const float2 sc = asc[b * nb + j];
        const int off8 = 8 * (int)sc.y;
#pragma unroll
        for (int r = 0; r < RG; r++) {
            int s = dot4(lo[r][0], xa.x, 0);
            s = dot4(lo[r][1], xa.y, s);
            s = dot4(lo[r][2], xa.z, s);
            s = dot4(lo[r][3], xa.w, s);
            s = dot4(hi[r][0], xb.x, s);
            s = dot4(hi[r][1], xb.y, s);
            s = dot4(hi[r][2], xb.z, s);
            s = dot4(hi[r][3], xb.w, s);
            acc[r][b] += (dw[r] * sc.x) * (float)(s - off8);
        }
    }
}

// Fused epilogues of a row pair (2k, 2k+1) --------------------------------------------------------
__device__ __forceinline__ float gateAct(const GemvArgs &a, float v) {
    if (a.act == 1) return v / (1.0f + __expf(-v));
    return 0.5f * v * (1.0f + tanhf(0.79788456080286535588f * v * (1.0f + 0.044715f * v * v)));
}

// Rows [0, q0) are Q, [q0, q0+kv0) K, then V. Q and K pairs are rotated (RoPE at this row's
// position); K and V are appended to the KV cache at [slot][pos].
__device__ __forceinline__ void qkvPairStore(const GemvArgs &a, int r0, float v0, float v1, const float2 *ropeRow,
                                             int p, int sl, float *qRow) {
    if (r0 < a.q0 + a.kv0) {
        const float2 cs = ropeRow[(r0 % a.hs) >> 1];
        const float o0 = v0 * cs.x - v1 * cs.y;
        const float o1 = v0 * cs.y + v1 * cs.x;
        if (r0 < a.q0) {
            *reinterpret_cast<float2 *>(qRow + r0) = make_float2(o0, o1);
        } else {
            const size_t off = ((size_t)sl * a.seqLen + p) * a.kv0 + (r0 - a.q0);
            if (a.kvBf16) {
                const uint32_t pk = (uint32_t)f32ToBf16(o0) | ((uint32_t)f32ToBf16(o1) << 16);
                *reinterpret_cast<uint32_t *>(reinterpret_cast<uint16_t *>(a.kcache) + off) = pk;
            } else {
                *reinterpret_cast<float2 *>(reinterpret_cast<float *>(a.kcache) + off) = make_float2(o0, o1);
            }
        }
    } else {
        const size_t off = ((size_t)sl * a.seqLen + p) * a.kv0 + (r0 - a.q0 - a.kv0);
        if (a.kvBf16) {
            const uint32_t pk = (uint32_t)f32ToBf16(v0) | ((uint32_t)f32ToBf16(v1) << 16);
            *reinterpret_cast<uint32_t *>(reinterpret_cast<uint16_t *>(a.vcache) + off) = pk;
        } else {
            *reinterpret_cast<float2 *>(reinterpret_cast<float *>(a.vcache) + off) = make_float2(v0, v1);
        }
    }
}

// Quantize a workgroup's `halfR` hidden units (multiple of 32, in LDS) to Q80 blocks in global.
template <int B>
__device__ __forceinline__ void storeHiddenQ80(const GemvArgs &a, const float *hbuf, int halfR, int hBase) {
    for (int i = threadIdx.x; i < B * halfR; i += kThreads) {  // 32-lane groups = one block
        const int b = i / halfR, k = i % halfR;
        if (hBase + k >= (a.rows >> 1)) continue;  // whole 32-unit blocks: uniform per lane group
        const float h = hbuf[b * halfR + k];
        const float amax = groupMax<32>(fabsf(h));
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        int q = (int)rintf(h * id);
        q = q > 127 ? 127 : (q < -127 ? -127 : q);
        a.oq[(size_t)b * a.ldOut + hBase + k] = (int8_t)q;
        const float qs = groupSum<32>((float)q);
        if ((k & 31) == 0) a.os[(size_t)b * (a.ldOut >> 5) + ((hBase + k) >> 5)] = make_float2(roundF16(d), qs);
    }
}

// Copy B rows of Q80 activations (n int8 + n/32 scale pairs) from global into the LDS image.
template <int B>
__device__ __forceinline__ void stageQ80(const GemvArgs &a, int8_t *sq, float2 *ssc) {
    const int n = a.n, nb = n >> 5;
#pragma unroll
    for (int b = 0; b < B; b++) {
        const int4 *src = reinterpret_cast<const int4 *>(a.aq + (size_t)b * n);
        int4 *dst = reinterpret_cast<int4 *>(sq + (size_t)b * n);
        for (int i = threadIdx.x; i < (n >> 4); i += kThreads) dst[i] = src[i];
        for (int i = threadIdx.x; i < nb; i += kThreads) ssc[b * nb + i] = a.as[(size_t)b * nb + i];
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// Fused tensor-parallel exchange (TpXchg, kernels.h). Peer words are 8-byte {payload, epoch}
// granules in uncached memory: one relaxed system-scope store publishes data and flag together,
// a relaxed system-scope load polls them (cdna_hip_programming.md Guideline 16 "R2": the data is
// the flag, no fence needed); a wait gives up after tp.timeoutTicks and raises tp.error.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t tpLoad(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool tpFailed(const TpXchg &x) {
    return __hip_atomic_load(x.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

// Push `payload` as exchange word `w` (epoch e) to every peer, then collect word `w` of every rank
// into vals[p] (this rank's own payload included). Peer loads are all issued before any wait.
__device__ __forceinline__ void tpPushCollect(const TpXchg &x, long long w, unsigned e, unsigned payload,
                                              unsigned (&vals)[kTpMaxRanks], bool failed) {
    const int me = x.rank, W = x.world;
    const long long par = e & 1;
    const uint64_t word = (uint64_t)payload | ((uint64_t)e << 32);
#pragma unroll
    for (int p = 0; p < kTpMaxRanks; p++)
        if (p < W && p != me)
            __hip_atomic_store(x.recv[p] + (par * W + me) * x.stride + w, word, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t *mine = x.recv[me] + par * W * x.stride + w;
    uint64_t got[kTpMaxRanks];
#pragma unroll
    for (int p = 0; p < kTpMaxRanks; p++) got[p] = (p < W && p != me) ? tpLoad(mine + p * x.stride) : word;
#pragma unroll
    for (int p = 0; p < kTpMaxRanks; p++) {
        if (p < W) {
            uint64_t v = got[p];
            if ((unsigned)(v >> 32) != e && !failed) {
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                while ((unsigned)(v >> 32) != e) {
                    __builtin_amdgcn_s_sleep(1);
                    v = tpLoad(mine + p * x.stride);
                    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > x.timeoutTicks) {
                        __hip_atomic_store(x.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                }
            }
            vals[p] = (unsigned)v;
        }
    }
}

// LDS bytes of the Q80 exchange staging for nEl elements over W ranks.
__host__ __device__ static inline size_t tpQ80Lds(int nEl, int W) {
    return alignUp((size_t)nEl, 16) + alignUp((size_t)nEl / 32 * 4, 16) + (size_t)W * (nEl / 32) * 9 * 4;
}

// f32 exchange of a workgroup's partial rows res[B][R] (rows rowBase..) -> a.out summed over ranks.
template <int B>
__device__ __forceinline__ void tpExchangeF32(const GemvArgs &a, const float *res, int R, int rowBase) {
    const TpXchg &x = a.tp;
    const bool failed = tpFailed(x);
    for (int i = threadIdx.x; i < B * R; i += kThreads) {
        const int b = i / R, row = rowBase + i % R;
        if (row >= a.rows) continue;
        const long long el = (long long)b * a.ldOut + row;
        const unsigned e = x.epochs[el] + 1;
        unsigned v[kTpMaxRanks];
        tpPushCollect(x, el, e, __float_as_uint(res[i]), v, failed);
        float s = 0.f;
#pragma unroll
        for (int p = 0; p < kTpMaxRanks; p++)
            if (p < x.world) s += __uint_as_float(v[p]);
        a.out[el] = s;
        x.epochs[el] = e;
    }
}

// Q80 exchange (the reference's ZQ pipe: every rank's partial quantized once to Q80 blocks of 32
// rows, all ranks' blocks dequantized and summed in rank order, own included). R and rowBase are
// multiples of 32. A block travels as 9 words: 8 x 4 int8 + the f16 scale. `lds` = free staging.
template <int B>
__device__ __forceinline__ void tpExchangeQ80(const GemvArgs &a, const float *res, int R, int rowBase, char *lds) {
    const TpXchg &x = a.tp;
    const int nEl = B * R, nBlk = nEl >> 5, W = x.world;
    int8_t *q8 = reinterpret_cast<int8_t *>(lds);
    uint32_t *dq = reinterpret_cast<uint32_t *>(lds + alignUp((size_t)nEl, 16));
    uint32_t *rv = reinterpret_cast<uint32_t *>(lds + alignUp((size_t)nEl, 16) + alignUp((size_t)nBlk * 4, 16));
    const bool failed = tpFailed(x);
    // 1. quantize this rank's partial (whole 32-lane groups per block: the loop is uniform)
    for (int base = 0; base < nEl; base += kThreads) {
        const int i = base + threadIdx.x;
        const float v = i < nEl ? res[i] : 0.f;
        const float amax = groupMax<32>(fabsf(v));
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        int q = (int)rintf(v * id);
        q = q > 127 ? 127 : (q < -127 ? -127 : q);
        if (i < nEl) {
            q8[i] = (int8_t)q;
            if ((i & 31) == 0) dq[i >> 5] = __half_as_ushort(__float2half(d));
        }
    }
    __syncthreads();
    auto blockId = [&](int blk, bool &live) -> long long {  // global block id in the exchange space
        const int b = (blk * 32) / R, row = rowBase + (blk * 32) % R;
        live = row < a.rows;
        return ((long long)b * a.ldOut + row) >> 5;
    };
    // 2. push / collect the 9 words of every block
    for (int j = threadIdx.x; j < nBlk * 9; j += kThreads) {
        const int blk = j / 9, w = j % 9;
        bool live;
        const long long gb = blockId(blk, live);
        if (!live) continue;
        const unsigned e = x.epochs[gb] + 1;
        const unsigned payload = w < 8 ? reinterpret_cast<const uint32_t *>(q8)[blk * 8 + w] : dq[blk];
        unsigned v[kTpMaxRanks];
        tpPushCollect(x, gb * 9 + w, e, payload, v, failed);
#pragma unroll
        for (int p = 0; p < kTpMaxRanks; p++)
            if (p < W) rv[(p * nBlk + blk) * 9 + w] = v[p];
    }
    __syncthreads();
    // 3. dequantize and sum in rank order
    for (int i = threadIdx.x; i < nEl; i += kThreads) {
        const int b = i / R, row = rowBase + i % R, blk = i >> 5;
        if (row >= a.rows) continue;
        float s = 0.f;
        for (int p = 0; p < W; p++) {
            const uint32_t *bw = rv + (p * nBlk + blk) * 9;
            const float d = __half2float(__ushort_as_half((uint16_t)(bw[8] & 0xFFFFu)));
            const int q = (int)(int8_t)(bw[(i & 31) >> 2] >> (8 * (i & 3)));
            s += (float)q * d;
        }
        a.out[(size_t)b * a.ldOut + row] = s;
    }
    // 4. advance the block epochs (every word of step 2 has read them)
    for (int blk = threadIdx.x; blk < nBlk; blk += kThreads) {
        bool live;
        const long long gb = blockId(blk, live);
        if (live) x.epochs[gb] += 1;
    }
}

// Sequence split of a decode-attention row of length `len`: nSplit chunks of ch positions
// (~256 per chunk, at most splitGrid chunks).
__device__ __forceinline__ void attnSplit(int len, int splitGrid, int &nSplit, int &ch) {
    int ns = (len + 255) / 256;
    if (ns > splitGrid) ns = splitGrid;
    if (ns < 1) ns = 1;
    ch = (((len + ns - 1) / ns) + 15) & ~15;
    nSplit = (len + ch - 1) / ch;
}

// ------------------------------------------------------------------------------------------------
// Q40 GEMV, register-ring pipeline.
//   Each lane group (L lanes) owns row pairs; lane li walks blocks j = li, li+L, ... of its rows
//   for every pass (row pair) of the workgroup as ONE flat sequence of T = passes * K steps
//   (K = ceil(nb / L)). kRing steps are kept in flight in a ring of VGPR slots: step t is
//   consumed from slot t % kRing and the slot is immediately refilled with step t + kRing, so the
//   HBM stream never drains between blocks, row pairs or passes (the previous design issued
//   4 blocks, computed, then issued the rest 2 at a time: ~1.6x the streaming floor measured by
//   scripts/microbench_stream.hip). Activations always come from LDS (norm prologue or a copy
//   of upstream Q80), row-pair epilogues (SwiGLU, RoPE + KV append) run in registers.
// ------------------------------------------------------------------------------------------------
static constexpr int kRing = 8;
#ifndef DL_GEMV_KE
#define DL_GEMV_KE 2
#endif
static constexpr int kEarlySlots = DL_GEMV_KE;  // ring slots issued before the early prologue's wait

template <int L, int B, int PRO, int EPI>
__global__ __launch_bounds__(kThreads) void gemvQ40Kernel(GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int RG = 2, NG = kThreads / L, RP = NG * RG, D = kRing;
    const int n = a.n, nb = n >> 5, K = (nb + L - 1) / L, P = a.passes, T = P * K;
    const int R = RP * P;
    const GemvLds lay = gemvLayout(n, B, true, R, PRO_RESNORM);
    float *scratch = reinterpret_cast<float *>(smem + lay.scratch);
    float *hbuf = reinterpret_cast<float *>(smem + lay.hbuf);
    int8_t *sq = reinterpret_cast<int8_t *>(smem + lay.act);
    float2 *ssc = reinterpret_cast<float2 *>(smem + lay.sc);
    float *res = reinterpret_cast<float *>(smem + lay.res);  // partial rows held for the TP exchange
    constexpr bool tpx = EPI == EPI_STORE_TP;
    const int tid = threadIdx.x, gi = tid / L, li = tid % L;
    const int rowBase = blockIdx.x * R;
    // timestamps stay in SGPRs until the end: a store here would join the ring's vmcnt accounting
    const unsigned long long tEntry = a.trace ? wall_clock64() : 0ull;
    unsigned long long tReady = 0ull, tLoaded = 0ull, tFirst = 0ull;

    // slot = 2 rows x 16 B of nibbles + the pair's two f16 scales in one 32-bit word
    u32x4 w[D][RG];
    uint32_t dh[D];
    const uint32_t *wd2 = reinterpret_cast<const uint32_t *>(a.wd);  // tiled pair scales
    // this workgroup's chunks are [blockIdx.x * T, blockIdx.x * T + T) of the tiled matrix
    const size_t cBase = (size_t)blockIdx.x * T;
    const size_t cLast = (size_t)((a.rows + RP - 1) / RP) * K - 1;
    int it = 0;  // issue cursor (steps)
    auto stepPtrs = [&](const u32x4 *&p0, const uint32_t *&pd) {
        const size_t c = min(cBase + (size_t)min(it, T - 1), cLast);
        p0 = reinterpret_cast<const u32x4 *>(a.qs) + (c * 2) * kThreads + tid;
        pd = wd2 + c * kThreads + tid;
        ++it;
    };
    // The ring's refills are inline asm with explicit vmcnt waits (cdna_hip_programming.md §5.7,
    // form ii): hipcc's own waitcnt pass flushes vmcnt(0) at the loop header, which turns the ring
    // into bulk-synchronous rounds. Each step is 3 loads; consuming a slot waits until only the
    // loads issued after it are outstanding. Refills past the last step re-read this workgroup's
    // last chunk (L2), keeping every slot unconditionally defined (no phi copies of in-flight
    // registers).
    auto issue = [&](u32x4(&ws)[RG], uint32_t &ds) {
        const u32x4 *p0;
        const uint32_t *pd;
        stepPtrs(p0, pd);
        asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(ws[0]) : "v"(p0));
        asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(ws[1]) : "v"(p0 + kThreads));
        asm volatile("global_load_dword %0, %1, off" : "=v"(ds) : "v"(pd));
    };
    // Late path: the prologue's compiler-visible loads were issued after the ring's, so waiting
    // for them waits for the whole first round anyway; this explicit wait also pins every slot
    // register before the loop, so no copy of an in-flight register can be made.
    auto waitAll = [&]() {
#pragma unroll
        for (int s = 0; s < D; s++) asm volatile("s_waitcnt vmcnt(0)" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(dh[s]));
    };

    float2 *sRope = reinterpret_cast<float2 *>(smem + lay.rope);
    int posB[B], slotB[B];  // uniform: scalar loads, kept out of the ring's vmcnt accounting
#pragma unroll
    for (int b = 0; b < B; b++) {
        posB[b] = EPI == EPI_QKV ? a.pos[b] : 0;
        slotB[b] = EPI == EPI_QKV ? a.slot[b] : 0;
    }
    // Early prologue (batch 1, activations small enough to sit in registers): the activation /
    // residual / norm-weight loads go out BEFORE the ring's first round, so the norm + Q80 work
    // overlaps the ring's HBM round trip instead of following it (~1 us per kernel).
    // PK = 8-float chunks (resnorm) or 16-byte Q80 units (copy) per thread, sized from n so no
    // load is wasted: resnorm n <= 2048 * PK, Q80 copy n <= 4096 * PK.
    auto earlyPath = [&](auto pkTag) {
        constexpr int PK = decltype(pkTag)::value, PS = (PK + 1) / 2;
        const int nChunks = n >> 3, n16 = n >> 4;
        f32x4 ex[PK][2], ey[PK][2], ew[PK][2];
        u32x4 eq[PK];
        u32x2 es[PS];
        // Every load of this path is inline asm with explicit waits: the compiler's waitcnt pass
        // does not see them, so nothing flushes vmcnt(0) before the loop and each ring slot is
        // waited for on its own inside it (the first slot's dot products start while the rest of
        // the first round is still in flight). Loads are unconditional and clamped.
        auto ld4a = [](f32x4 &r, const float *p) { asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p)); };
        u32x2 ropeV = {0u, 0u};
        if constexpr (EPI == EPI_QKV) {
            const float2 *rp = a.rope + (size_t)posB[0] * (a.hs >> 1) + min(tid, (a.hs >> 1) - 1);
            asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(ropeV) : "v"(rp));
        }
        if constexpr (PRO == PRO_RESNORM) {
            const float *yp = a.addIn ? a.addIn : a.in;
            const float *wp = a.normW ? a.normW : a.in;
#pragma unroll
            for (int k = 0; k < PK; k++) {
                const int c = min(tid + k * kThreads, nChunks - 1);
                ld4a(ex[k][0], a.in + c * 8);
                ld4a(ex[k][1], a.in + c * 8 + 4);
                ld4a(ey[k][0], yp + c * 8);
                ld4a(ey[k][1], yp + c * 8 + 4);
                ld4a(ew[k][0], wp + c * 8);
                ld4a(ew[k][1], wp + c * 8 + 4);
            }
        } else {
#pragma unroll
            for (int k = 0; k < PK; k++) {
                const u32x4 *src = reinterpret_cast<const u32x4 *>(a.aq) + min(tid + k * kThreads, n16 - 1);
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(eq[k]) : "v"(src));
            }
#pragma unroll
            for (int k = 0; k < PS; k++) {
                const u32x2 *src = reinterpret_cast<const u32x2 *>(a.as) + min(tid + k * kThreads, nb - 1);
                asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(es[k]) : "v"(src));
            }
        }
        // A CU returns vector loads in issue order across its waves: without this barrier a wave's
        // prologue loads queue behind the other waves' ring rounds (~3 us at the CU's share of
        // HBM bandwidth, measured with GemvArgs::trace). s_barrier alone, no fence: it does not
        // wait for the loads, only orders every wave's prologue issue before any ring issue.
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // KE slots go out before the prologue's wait, the rest of the ring once the prologue's
        // loads have landed (a full first round floods the memory queues and delays them)
        constexpr int KE = kEarlySlots < D ? kEarlySlots : D;
#pragma unroll
        for (int s = 0; s < KE; s++) {
            issue(w[s], dh[s]);
            __builtin_amdgcn_sched_barrier(0);
        }
        // the prologue's loads are older than the ring's 3 * KE: wait for them only
        if constexpr (EPI == EPI_QKV) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(ropeV) : "i"(3 * KE));
        if constexpr (PRO == PRO_RESNORM) {
#pragma unroll
            for (int k = 0; k < PK; k++)
                asm volatile("s_waitcnt vmcnt(%6)"
                             : "+v"(ex[k][0]), "+v"(ex[k][1]), "+v"(ey[k][0]), "+v"(ey[k][1]), "+v"(ew[k][0]), "+v"(ew[k][1])
                             : "i"(3 * KE));
        } else {
#pragma unroll
            for (int k = 0; k < PK; k++) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(eq[k]) : "i"(3 * KE));
#pragma unroll
            for (int k = 0; k < PS; k++) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(es[k]) : "i"(3 * KE));
        }
        if (a.trace) tLoaded = wall_clock64();
        if constexpr (EPI == EPI_QKV)
            if (tid < (a.hs >> 1)) sRope[tid] = make_float2(__uint_as_float(ropeV.x), __uint_as_float(ropeV.y));
        if constexpr (PRO == PRO_RESNORM) {
            float *xo = (blockIdx.x == 0 && a.xNext) ? a.xNext : nullptr;
            float v[PK][8];
            float ss = 0.f;
#pragma unroll
            for (int k = 0; k < PK; k++) {
                const int c = tid + k * kThreads;
                f32x4 v0 = ex[k][0], v1 = ex[k][1];
                if (a.addIn) {
                    v0 += ey[k][0];
                    v1 += ey[k][1];
                }
                if (xo && c < nChunks) {
                    *reinterpret_cast<f32x4 *>(xo + c * 8) = v0;
                    *reinterpret_cast<f32x4 *>(xo + c * 8 + 4) = v1;
                }
                v[k][0] = v0.x; v[k][1] = v0.y; v[k][2] = v0.z; v[k][3] = v0.w;
                v[k][4] = v1.x; v[k][5] = v1.y; v[k][6] = v1.z; v[k][7] = v1.w;
                if (c < nChunks) {
#pragma unroll
                    for (int i = 0; i < 8; i++) ss += v[k][i] * v[k][i];
                }
            }
            float inv = 1.0f;
            if (a.normW) {
                ss = blockSum<kThreads>(ss, scratch);
                inv = 1.0f / sqrtf(ss / (float)n + a.eps);
            }
#pragma unroll
            for (int k = 0; k < PK; k++) {
                const int c = tid + k * kThreads;
                if (c < nChunks) {
                    if (a.normW) {
                        const float wv[8] = {ew[k][0].x, ew[k][0].y, ew[k][0].z, ew[k][0].w,
                                             ew[k][1].x, ew[k][1].y, ew[k][1].z, ew[k][1].w};
#pragma unroll
                        for (int i = 0; i < 8; i++) v[k][i] = wv[i] * (inv * v[k][i]);
                    }
                    stageChunk<true>(v[k], 0, c, n, sq, ssc, nullptr);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < PK; k++)
                if (tid + k * kThreads < n16) reinterpret_cast<u32x4 *>(sq)[tid + k * kThreads] = eq[k];
#pragma unroll
            for (int k = 0; k < PS; k++)
                if (tid + k * kThreads < nb) reinterpret_cast<u32x2 *>(ssc)[tid + k * kThreads] = es[k];
        }
        __syncthreads();
        if (a.trace) tReady = wall_clock64();
        // The rest of the ring only now: a wave stalls at ISSUE once its CU's memory queue is full,
        // so issuing it before the prologue's arithmetic made the norm wait for most of the
        // matrix to stream in (trace: prologue loads landed at 0.6 us, prologue done at 2.8 us).
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = KE; s < D; s++) {
            issue(w[s], dh[s]);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto latePath = [&]() {
        // sched_barrier keeps issue order == slot order, so each step waits for exactly its own
        // slot (vmcnt = loads of the other kRing-1 slots) instead of the scheduler batching the ring.
#pragma unroll
        for (int s = 0; s < D; s++) {
            issue(w[s], dh[s]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (EPI == EPI_QKV) {  // the prologue's __syncthreads publishes these
            const int h2 = a.hs >> 1;
            for (int i = tid; i < B * h2; i += kThreads) {
                const int b = i / h2;
                sRope[b * (kMaxHeadSize / 2) + i % h2] = a.rope[(size_t)a.pos[b] * h2 + i % h2];
            }
        }
        if constexpr (PRO == PRO_RESNORM)
            resNormPrologue<B, true>(a, scratch, sq, ssc, nullptr);
        else
            stageQ80<B>(a, sq, ssc);
        waitAll();
        if (a.trace) tReady = wall_clock64();
    };

    // The ring's consume loop. Each prologue path below inlines its own copy, so no ring register
    // is live across a join of two paths (a join could copy a register whose load is in flight).
    auto mainLoop = [&]() __attribute__((always_inline)) {
    float acc[RG][B];
#pragma unroll
    for (int r = 0; r < RG; r++)
#pragma unroll
        for (int b = 0; b < B; b++) acc[r][b] = 0.f;
    int cp = 0, ck = 0;  // consume cursor
    // consume the step held in slot (ws, ds)
    auto consume = [&](const u32x4(&ws)[RG], uint32_t ds, bool live) {
        const int j = li + ck * L;
        const bool use = live && j < nb;
        float dw[RG];
        dw[0] = use ? __half2float(__ushort_as_half((uint16_t)(ds & 0xFFFFu))) : 0.f;
        dw[1] = use ? __half2float(__ushort_as_half((uint16_t)(ds >> 16))) : 0.f;
        q40Block<B, RG>(acc, ws, dw, min(j, nb - 1), n, nb, sq, ssc);
    };
    // after a step: at the end of a row pair, reduce over the lane group and run the fused
    // epilogue on its lane 0
    auto advance = [&]() {
        if (++ck < K) return;
#pragma unroll
        for (int r = 0; r < RG; r++)
#pragma unroll
            for (int b = 0; b < B; b++) acc[r][b] = groupSum<L>(acc[r][b]);
        const int r0 = rowBase + cp * RP + gi * RG;
        if (li == 0 && r0 < a.rows) {
#pragma unroll
            for (int b = 0; b < B; b++) {
                const float v0 = acc[0][b], v1 = acc[1][b];
                if constexpr (EPI == EPI_STORE_TP) {
                    res[b * R + (r0 - rowBase)] = v0;
                    res[b * R + (r0 - rowBase) + 1] = v1;
                } else if constexpr (EPI == EPI_STORE) {
                    float *o = a.out + (size_t)b * a.ldOut + r0;
                    o[0] = v0;
                    if (r0 + 1 < a.rows) o[1] = v1;
                } else if constexpr (EPI == EPI_ACT) {
                    a.out[(size_t)b * a.ldOut + (r0 >> 1)] = gateAct(a, v0) * v1;
                } else if constexpr (EPI == EPI_ACT_Q80) {
                    hbuf[b * (R >> 1) + ((r0 - rowBase) >> 1)] = gateAct(a, v0) * v1;
                } else {
                    qkvPairStore(a, r0, v0, v1, sRope + b * (kMaxHeadSize / 2), posB[b], slotB[b],
                                 a.out + (size_t)b * a.ldOut);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RG; r++)
#pragma unroll
            for (int b = 0; b < B; b++) acc[r][b] = 0.f;
        ck = 0;
        ++cp;
    };
    // Full rounds: every slot is consumed and refilled, so the slots stay in fixed registers and
    // consuming slot s waits until only the other kRing-1 slots are in flight.
    int t0 = 0;
    for (; t0 + D < T; t0 += D) {
#pragma unroll
        for (int s = 0; s < D; s++) {
            asm volatile("s_waitcnt vmcnt(%3)" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(dh[s]) : "i"(3 * (D - 1)));
            consume(w[s], dh[s], true);
            if (a.trace && s == 0 && t0 == 0) tFirst = wall_clock64();
            issue(w[s], dh[s]);
            advance();
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // Last round: no refills; slot s waits for the loads issued after it (slots s+1..kRing-1), so
    // every load has landed when the workgroup ends.
#pragma unroll
    for (int s = 0; s < D; s++) {
        asm volatile("s_waitcnt vmcnt(%3)" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(dh[s]) : "i"(3 * (D - 1 - s)));
        if (t0 + s < T) {
            consume(w[s], dh[s], true);
            if (a.trace && s == 0 && t0 == 0) tFirst = wall_clock64();
            advance();
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    };

    const int unitsPerThread = PRO == PRO_RESNORM ? (n + 8 * kThreads - 1) / (8 * kThreads)
                                                  : (n + 16 * kThreads - 1) / (16 * kThreads);
    if (B == 1 && unitsPerThread <= 1) {
        earlyPath(std::integral_constant<int, 1>{});
        mainLoop();
    } else if (B == 1 && unitsPerThread <= 2) {
        earlyPath(std::integral_constant<int, 2>{});
        mainLoop();
    } else if (B == 1 && unitsPerThread <= 4) {
        earlyPath(std::integral_constant<int, 4>{});
        mainLoop();
    } else {
        latePath();
        mainLoop();
    }
    if constexpr (EPI == EPI_ACT_Q80) {
        __syncthreads();
        storeHiddenQ80<B>(a, hbuf, R >> 1, rowBase >> 1);
    }
    if constexpr (tpx) {  // all-reduce the partial rows over the TP ranks, then store (sq is free now)
        __syncthreads();
        if (a.tp.q80) tpExchangeQ80<B>(a, res, R, rowBase, reinterpret_cast<char *>(sq));
        else tpExchangeF32<B>(a, res, R, rowBase);
    }
    if (a.trace) {
        __syncthreads();
        if (tid == 0) {
            const unsigned long long tExit = wall_clock64();
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
            unsigned long long *t = a.trace + 8 * (size_t)blockIdx.x;
            t[0] = tEntry;
            t[1] = tReady;
            t[2] = tExit;
            t[3] = ((unsigned long long)hw << 32) | xcc;
            t[4] = tLoaded;
            t[5] = tFirst;
        }
    }
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

// Dynamic LDS above 64 KB (up to the CU's 160 KB) has to be opted into per kernel.
static void allowLds(const void *fn, size_t bytes) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
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
    if (q40 && epi == EPI_STORE_TP && a.tp.q80) {  // Q80 exchange staging reuses `act`
        const GemvLds lay = gemvLayout(a.n, B, true, R, PRO_RESNORM);
        g.lds = std::max(g.lds, lay.act + tpQ80Lds(B * R, a.tp.world));
    }
    if (q40)
        g.fn = L == 16 ? gemvFnB<16, true>(B, pro, epi) : L == 32 ? gemvFnB<32, true>(B, pro, epi) : gemvFnB<64, true>(B, pro, epi);
    else
        g.fn = L == 16 ? gemvFnB<16, false>(B, pro, epi) : L == 32 ? gemvFnB<32, false>(B, pro, epi) : gemvFnB<64, false>(B, pro, epi);
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

// ------------------------------------------------------------------------------------------------
// Batched GEMM design notes (measured, profiles/r2_gemm_designs.md): two alternatives were built
// and measured slower than this kernel on every shape - (v2) weights HBM -> VGPR ring with the
// activations refilled through a 4-deep LDS ring (shared vmcnt capped the weight stream at 3 steps
// in flight), (v3) activations resident in LDS with a deep weight ring and 4 or 8 waves (1.4-1.7
// TB/s on w13, issue-stall bound per PMC: SQ_WAIT_INST_ANY 46 % of wave cycles). This v1 stays.
// Batched Q40 matmul on MFMA (prefill / multi-user decode, 2..32 tokens per launch).
//   out[t][row] = sum_k W[row][k] * x[t][k], W Q40 (the GEMV's tiled layout), x f16.
// Each workgroup owns 64 weight rows (4 waves x 16) and one K split, streamed in chunks of 16
// Q40 blocks. Both operands are copied HBM/L2 -> LDS with global_load_lds_dwordx4 (no VGPR
// staging; one 16-B unit per lane, contiguous 256-B+ runs per wave instruction), multi-buffered
// with counted vmcnt waits and raw barriers (kGemmStages buffers), into XOR-swizzled images so the fragment reads are
// bank-conflict free. Per block a lane dequantizes 8 nibbles of its row ((1024+q) - 1032 exact in
// f16, times d) into the B fragment of v_mfma_f32_16x16x32_f16; A fragments are read as is.
// Split-K partials are combined in split order by the last-arriving workgroup (agent-scope
// release/acquire counter: deterministic), which runs the fused epilogues (store / SwiGLU /
// SwiGLU -> f16 / SwiGLU -> Q80 / RoPE + KV append).
// ------------------------------------------------------------------------------------------------
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
static constexpr int kGemmRows = 64;
static constexpr int kGemmCh = 8;  // Q40 blocks per pipeline stage (~25 KB at 32 tokens)

// Split-K degree: grow S until the grid reaches the workgroup target (DL_GEMM_WG, read once) or
// a split would get fewer than kGemmCh blocks. The target is sized so every CU holds its 3
// resident workgroups: with one chunk in flight per workgroup, bytes in flight per CU (and so
// HBM bandwidth) scale with resident workgroups, not with tiles.
static int gemmWgTarget() {
    static const int v = [] {
        const char *e = std::getenv("DL_GEMM_WG");
        return e ? std::max(1, std::atoi(e)) : 256;
    }();
    return v;
}
static int gemmMaxSplits() {
    static const int v = [] {
        const char *e = std::getenv("DL_GEMM_MAXS");
        return e ? std::max(1, std::atoi(e)) : 8;
    }();
    return v;
}

GemmPlan gemmPlan(int rows, int n, int M) {
    GemmPlan p;
    p.rt = 1;
    p.tiles = (rows + kGemmRows - 1) / kGemmRows;
    p.splits = gemmSplits(rows, n, M);
    return p;
}

bool gemmSupported(int n) { return n % 32 == 0; }

int gemmSplits(int rows, int n, int M) {
    (void)M;
    const int tiles = (rows + kGemmRows - 1) / kGemmRows, nb = n / 32;
    const int target = gemmWgTarget(), maxS = gemmMaxSplits();
    int S = 1;
    while (2 * S <= maxS && tiles * S < target && nb % (2 * S) == 0 && nb / (2 * S) >= kGemmCh) S *= 2;
    // deep K (w2: 4096 x 14336): keep splitting up to two workgroups per CU while every split
    // still streams >= 4 chunks (measured w2 M=8 23.9 -> 19.6 us; shallower matrices lose)
    while (2 * S <= maxS && tiles * 2 * S <= 2 * target && nb % (2 * S) == 0 && nb / (2 * S) >= 4 * kGemmCh) S *= 2;
    return S;
}

int gemmTokenPad(int M) { return M <= 16 ? 16 : M <= 32 ? 32 : 64; }

size_t gemmPartFloats(int rows, int n, int maxTokens) {
    const int tiles = (rows + kGemmRows - 1) / kGemmRows, S = gemmSplits(rows, n, maxTokens);
    const int mp = gemmTokenPad(maxTokens);
    return S > 1 ? (size_t)S * tiles * mp * kGemmRows : 0;
}

// stage layout (bytes): weights [64 rows][8 units] x 16 B | scales [32 pairs][8] u32 | x [MP][32 units] x 16 B
static constexpr int kStW = kGemmRows * kGemmCh * 16, kStD = (kGemmRows / 2) * kGemmCh * 4;
__host__ __device__ static constexpr int gemmStageBytes(int MT) { return kStW + kStD + MT * 16 * kGemmCh * 64; }
#ifndef DL_GEMM_STAGES
#define DL_GEMM_STAGES 2  // 3 stages (2 WGs/CU) measured slower: batch-32 8.1k vs 8.8k tok/s
#endif
static constexpr int kGemmStages = DL_GEMM_STAGES;  // stage buffers (kGemmStages-1 chunks in flight)
static size_t gemmLds(int MT, int stages) { return stages * (size_t)gemmStageBytes(MT) + 16 + 320 * 4; }  // + flag, row scales

// 8 nibbles (lo or hi of 8 bytes) -> 8 f16 values (q - 8) * d via the 0x6400 | q magic (1024 + q)
__device__ __forceinline__ half8 dequantQ40x8(u32x2 wv, int nibHi, uint32_t d16) {
    const uint32_t lo = nibHi ? (wv.x >> 4) & 0x0F0F0F0Fu : wv.x & 0x0F0F0F0Fu;
    const uint32_t hi = nibHi ? (wv.y >> 4) & 0x0F0F0F0Fu : wv.y & 0x0F0F0F0Fu;
    const uint32_t p0 = __builtin_amdgcn_perm(0x64646464u, lo, 0x07010700u);
    const uint32_t p1 = __builtin_amdgcn_perm(0x64646464u, lo, 0x07030702u);
    const uint32_t p2 = __builtin_amdgcn_perm(0x64646464u, hi, 0x07010700u);
    const uint32_t p3 = __builtin_amdgcn_perm(0x64646464u, hi, 0x07030702u);
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const _Float16 d = __builtin_bit_cast(_Float16, (uint16_t)d16);
    // (1024 + q) - 1032 = q - 8 is exact in f16; one rounding in the multiply by d
    const h2 dd = {d, d};
    const h2 off = {(_Float16)-1032.0f, (_Float16)-1032.0f};
    const h2 r0 = (__builtin_bit_cast(h2, p0) + off) * dd;
    const h2 r1 = (__builtin_bit_cast(h2, p1) + off) * dd;
    const h2 r2 = (__builtin_bit_cast(h2, p2) + off) * dd;
    const h2 r3 = (__builtin_bit_cast(h2, p3) + off) * dd;
    half8 out;
    out[0] = r0[0]; out[1] = r0[1]; out[2] = r1[0]; out[3] = r1[1];
    out[4] = r2[0]; out[5] = r2[1]; out[6] = r3[0]; out[7] = r3[1];
    return out;
}

// one 16-B global -> LDS copy per lane; `lds` = this wave's base (lane l lands at lds + 16 l)
__device__ __forceinline__ void glds16(const void *g, void *lds) {
    __builtin_amdgcn_global_load_lds(const_cast<void *>(g), reinterpret_cast<__attribute__((address_space(3))) void *>(
                                         reinterpret_cast<uintptr_t>(lds)), 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void *g, void *lds) {
    __builtin_amdgcn_global_load_lds(const_cast<void *>(g), reinterpret_cast<__attribute__((address_space(3))) void *>(
                                         reinterpret_cast<uintptr_t>(lds)), 4, 0, 0);
}

// EPI_RES hand-off scale (power of two: exact) and the f16 store that saturates instead of
// overflowing to inf.
static constexpr float kResXScale = 1.0f / 32.0f;
__device__ __forceinline__ _Float16 satF16(float v) { return (_Float16)fminf(fmaxf(v, -65504.f), 65504.f); }

// Split-K combine and fused epilogues shared by the batched GEMMs (Q40 and f32): `acc` holds this
// lane's C fragments (weight row (local) wave*16 + col, token t*16 + h*4 + i); `smem` must hold
// MP x 64 floats and is free (all K-loop LDS reads retired behind a barrier); `flag` one int.
// tileIdx / tiles: this 64-row tile and the launch's tile count (split-K partial slots, counters).
template <int MT, int EPI>
__device__ __forceinline__ void gemmFinish(const GemmArgs &ga, const f32x4 (&acc)[MT], char *smem, int *flag,
                                           int tileIdx, int tiles) {
    const GemvArgs &a = ga.e;
    constexpr int MP = MT * 16;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int col = lane & 15, h = lane >> 4, rl = wave * 16 + col;
    const int sp = blockIdx.y, S = ga.splits;
    const int R0 = tileIdx * kGemmRows;
    float *tile = reinterpret_cast<float *>(smem);  // [MP][64], stages are free now
    // C layout: weight row (local) wave*16 + col, token t*16 + h*4 + i
    if (S == 1) {
#pragma unroll
        for (int t = 0; t < MT; t++)
#pragma unroll
            for (int i = 0; i < 4; i++) tile[(t * 16 + h * 4 + i) * kGemmRows + rl] = acc[t][i];
    } else {
        // Partials are written and read with agent-scope atomic accesses (global_store / load sc1:
        // performed at the coherence point, never held in or served from one XCD's L2), so the
        // hand-off needs no fence: an agent-scope release / acquire fence is a whole-L2 writeback
        // (buffer_wbl2) / invalidate (buffer_inv) on gfx950, which measured ~28 us per split level
        // on w13 (448 -> 896 workgroups) and evicted the other workgroups' cached activations.
        // vmcnt(0) before the arrival count: every partial store has been performed.
        float *part = ga.part + ((size_t)sp * tiles + tileIdx) * MP * kGemmRows;
#pragma unroll
        for (int t = 0; t < MT; t++)
#pragma unroll
            for (int i = 0; i < 4; i++)
                __hip_atomic_store(part + (t * 16 + h * 4 + i) * kGemmRows + rl, acc[t][i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const int old = __hip_atomic_fetch_add(ga.counters + tileIdx, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            flag[0] = old == S - 1;
        }
        __syncthreads();
        if (!flag[0]) return;
        if (tid == 0) __hip_atomic_store(ga.counters + tileIdx, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // combine in split order (deterministic), all of a thread's splits in flight at once: this
        // tail runs on one workgroup per tile after the others finished
        const float *P = ga.part + (size_t)tileIdx * MP * kGemmRows;
        const size_t stp = (size_t)tiles * MP * kGemmRows;
        auto ld = [](const float *q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
        for (int i = tid; i < MP * kGemmRows / 4; i += kThreads) {
            f32x4 v[8];
#pragma unroll
            for (int s2 = 0; s2 < 8; s2++)
                if (s2 < S) {
                    const float *q = P + s2 * stp + 4 * i;
                    v[s2] = f32x4{ld(q), ld(q + 1), ld(q + 2), ld(q + 3)};
                }
            f32x4 r = v[0];
#pragma unroll
            for (int s2 = 1; s2 < 8; s2++)
                if (s2 < S) r += v[s2];
            for (int s2 = 8; s2 < S; s2++) {
                const float *q = P + s2 * stp + 4 * i;
                r += f32x4{ld(q), ld(q + 1), ld(q + 2), ld(q + 3)};
            }
            reinterpret_cast<f32x4 *>(tile)[i] = r;
        }
    }
    // consumer of a fused residual + norm: per-token RMS scale from the producer's tile partials
    float *rsL = reinterpret_cast<float *>(flag + 4);  // [64]
    if (ga.ssIn) {
        // TPT threads per token each sum a strided slice of the tile partials (independent loads
        // in flight), then one thread per token adds the TPT slices in order (deterministic)
        float *slL = rsL + 64;  // [256]
        constexpr int TPT = kThreads / MP;
        const int t = tid / TPT, q = tid % TPT;
        float ssum = 0.f;
        if (t < ga.M) {
#pragma unroll 8
            for (int j = q; j < ga.ssTiles; j += TPT) ssum += ga.ssIn[(size_t)j * ga.ldSS + t];
        }
        slL[tid] = ssum;
        __syncthreads();
        if (tid < ga.M) {
            float tot = 0.f;
            for (int i = 0; i < TPT; i++) tot += slL[tid * TPT + i];
            rsL[tid] = (1.0f / kResXScale) / sqrtf(tot / (float)a.n + a.eps);
        }
    }
    __syncthreads();
    // fused epilogues on row pairs (2k, 2k+1) of the tile, 32 pairs per token
    for (int i = tid; i < ga.M * 32; i += kThreads) {
        const int t = i >> 5, k = i & 31, r0 = R0 + 2 * k;
        float v0 = tile[t * kGemmRows + 2 * k], v1 = tile[t * kGemmRows + 2 * k + 1];
        if (ga.ssIn) {
            v0 *= rsL[t];
            v1 *= rsL[t];
        }
        if constexpr (EPI == EPI_RES) {
            float x0 = 0.f, x1 = 0.f;
            if (r0 < a.rows) {  // a.rows even: whole pairs
                const size_t o = (size_t)t * a.ldOut + r0;
                x0 = ga.resIn[o] + v0;
                x1 = ga.resIn[o + 1] + v1;
                ga.resOut[o] = x0;
                ga.resOut[o + 1] = x1;
                // the un-normalised residual can be large (real checkpoints carry outlier channels
                // of 1e3-1e4): stored pre-scaled by 2^-5 (exact) and saturated, so f16 never
                // overflows to inf; the consumer folds 2^5 into its RMS scale
                ga.resX[o] = satF16(x0 * ga.resW[r0] * kResXScale);
                ga.resX[o + 1] = satF16(x1 * ga.resW[r0 + 1] * kResXScale);
            }
            const float ssq = groupSum<32>(x0 * x0 + x1 * x1);  // the 32 pairs of token t, in lane order
            if (k == 0) ga.ssOut[(size_t)tileIdx * ga.ldSS + t] = ssq;
        } else if constexpr (EPI == EPI_STORE) {
            if (r0 < a.rows) a.out[(size_t)t * a.ldOut + r0] = v0;
            if (r0 + 1 < a.rows) a.out[(size_t)t * a.ldOut + r0 + 1] = v1;
        } else if constexpr (EPI == EPI_ACT) {
            if (r0 < a.rows) a.out[(size_t)t * a.ldOut + (r0 >> 1)] = gateAct(a, v0) * v1;
        } else if constexpr (EPI == EPI_ACT_F16) {
            if (r0 < a.rows) ga.outH[(size_t)t * a.ldOut + (r0 >> 1)] = (_Float16)(gateAct(a, v0) * v1);
        } else if constexpr (EPI == EPI_ACT_Q80) {
            const int hBase = R0 >> 1;
            if (hBase >= (a.rows >> 1)) continue;  // whole 32-unit block: uniform per lane group
            const float hv = gateAct(a, v0) * v1;
            const float amax = groupMax<32>(fabsf(hv));
            const float d = amax / 127.0f;
            const float id = d != 0.f ? 1.0f / d : 0.f;
            int q = (int)rintf(hv * id);
            q = q > 127 ? 127 : (q < -127 ? -127 : q);
            a.oq[(size_t)t * a.ldOut + hBase + k] = (int8_t)q;
            const float qsum = groupSum<32>((float)q);
            if (k == 0) a.os[(size_t)t * (a.ldOut >> 5) + (hBase >> 5)] = make_float2(roundF16(d), qsum);
        } else {
            if (r0 < a.rows)
                qkvPairStore(a, r0, v0, v1, a.rope + (size_t)a.pos[t] * (a.hs >> 1), a.pos[t], a.slot[t],
                             a.out + (size_t)t * a.ldOut);
        }
    }
}

// STG = stage buffers: 2 double-buffers the chunk stream inside a workgroup; 1 (the 64-token
// tile) drops that to fit 3 workgroups per CU, which then overlap each other's loads.
template <int MT, int EPI, int STG>
__global__ __launch_bounds__(kThreads) void gemmQ40Kernel(GemmArgs ga) {
    const GemvArgs &a = ga.e;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int SB = gemmStageBytes(MT);
    constexpr int NW = kGemmRows * kGemmCh / kThreads, NX = MT * 16 * kGemmCh * 4 / kThreads;
    constexpr int NLD = NW + 1 + NX;  // glds instructions per thread per stage
    int *flag = reinterpret_cast<int *>(smem + STG * SB);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int col = lane & 15, h = lane >> 4;
    const int n = a.n, nb = n >> 5, L = a.lanes, NG = kThreads / L, KS = (nb + L - 1) / L;
    const int lgL = 31 - __builtin_clz(L);
    const int tileIdx = blockIdx.x, sp = blockIdx.y, S = ga.splits;
    const int R0 = tileIdx * kGemmRows;
    const int bps = nb / S, j0 = sp * bps, j1 = j0 + bps;
    const int nch = (bps + kGemmCh - 1) / kGemmCh;
    const uint8_t *qs = a.qs;
    const uint32_t *wd2 = reinterpret_cast<const uint32_t *>(a.wd);
    auto unitOf = [&](int row, int j) -> size_t {  // tiled 16-B unit of (row, block j), clamped
        row = min(row, a.rows - 1);
        j = min(j, j1 - 1);
        const int g = row / (2 * NG), rem = row % (2 * NG), gi = rem >> 1, rpar = rem & 1;
        const int k = j >> lgL, li = j & (L - 1);
        return (((size_t)g * KS + k) * 2 + rpar) * kThreads + gi * L + li;
    };
    auto scaleIdx = [&](int pairRow, int j) -> size_t {  // tiled u32 pair scale of (row pair, block j)
        const int row = min(pairRow, a.rows - 1);
        j = min(j, j1 - 1);
        const int g = row / (2 * NG), rem = row % (2 * NG), gi = rem >> 1;
        const int k = j >> lgL, li = j & (L - 1);
        return ((size_t)g * KS + k) * kThreads + gi * L + li;
    };
    // issue the copies of chunk c into stage buffer b
    auto issue = [&](int c, int b) {
        char *st = smem + b * SB;
        const int c0 = j0 + c * kGemmCh;
        // weights: unit u = s*256 + tid -> (row_l = u/8, position p = u%8) holds block p ^ ((row_l>>1)&7)
#pragma unroll
        for (int s = 0; s < NW; s++) {
            const int u = s * kThreads + tid, rl = u / kGemmCh, pp = u % kGemmCh;
            const size_t unit = unitOf(R0 + rl, c0 + (pp ^ ((rl >> 1) & (kGemmCh - 1))));
            glds16(qs + unit * 16, st + (size_t)(s * kThreads + wave * 64) * 16);
        }
        // pair scales: u = tid -> (pair_l = u/8, block u%8), 4 B each
        {
            const int pl = tid / kGemmCh, jj = tid % kGemmCh;
            glds4(wd2 + scaleIdx(R0 + 2 * pl, c0 + jj), st + kStW + (size_t)(wave * 64) * 4);
        }
        // activations: token row t = 4*kGemmCh units of 8 f16; position p holds unit p ^ (t&15)
#pragma unroll
        for (int s = 0; s < NX; s++) {
            const int u = s * kThreads + tid, t = u / (4 * kGemmCh), pp = u % (4 * kGemmCh);
            const int uu = pp ^ (t & 15);
            const int cb = min(c0 + (uu >> 2), j1 - 1);  // block of this unit (clamped)
            const _Float16 *src = ga.x + (size_t)t * n + (size_t)cb * 32 + (uu & 3) * 8;
            glds16(src, st + kStW + kStD + (size_t)(s * kThreads + wave * 64) * 16);
        }
    };

    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int rl = wave * 16 + col;  // this lane's weight row (local)
    const int byteHalf = h & 1, nibHi = h >> 1;

    constexpr int PF = STG - 1;  // chunks in flight ahead of the one consumed
    for (int c = 0; c < PF && c < nch; c++) issue(c, c);
    for (int c = 0; c < nch; c++) {
        if (c + PF < nch) issue(c + PF, (c + PF) % STG);
        // wait until chunk c landed (this thread): the chunks issued after it may stay in flight
        const int after = min(nch - 1, c + PF) - c;
        if (after >= 3)
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * NLD) : "memory");
        else if (after == 2)
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * NLD) : "memory");
        else if (after == 1)
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NLD) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // ... and for every thread
        const char *st = smem + (c % STG) * SB;
        const int cn = min(kGemmCh, bps - c * kGemmCh);
#pragma unroll
        for (int jj = 0; jj < kGemmCh; jj++) {
            // swizzle key (rl >> 1) & 7: the 16 rows of a wave's ds_read_b64 (two 8-B halves per
            // 16-B unit) land on 32 distinct bank pairs (rows 128 B apart alias every other row;
            // the old key rl & 7 left 2-way conflicts: SQ_LDS_BANK_CONFLICT 25 % of LDS cycles)
            const int pp = jj ^ ((rl >> 1) & (kGemmCh - 1));
            const u32x2 wv = *reinterpret_cast<const u32x2 *>(st + (size_t)(rl * kGemmCh + pp) * 16 + byteHalf * 8);
            const uint32_t dw = *reinterpret_cast<const uint32_t *>(st + kStW + (size_t)((rl >> 1) * kGemmCh + jj) * 4);
            const uint32_t d16 = jj < cn ? ((rl & 1) ? dw >> 16 : dw & 0xFFFFu) : 0u;
            const half8 b = dequantQ40x8(wv, nibHi, d16);
#pragma unroll
            for (int t = 0; t < MT; t++) {
                const int tok = t * 16 + col, up = (jj * 4 + h) ^ (tok & 15);
                const half8 av = *reinterpret_cast<const half8 *>(st + kStW + kStD + (size_t)(tok * 4 * kGemmCh + up) * 16);
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, b, acc[t], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage c % STG is refilled at iteration c + 1
    }

    gemmFinish<MT, EPI>(ga, acc, smem, flag, blockIdx.x, gridDim.x);
}

static int gemmStages4() {  // stage buffers of the 64-token tile (DL_GEMM_STG4, read once)
    static const int v = [] {
        const char *e = std::getenv("DL_GEMM_STG4");
        return e && std::atoi(e) == 2 ? 2 : 1;
    }();
    return v;
}

static int gemmStages2() {  // stage buffers of the 32-token tile (DL_GEMM_STG2, read once)
    static const int v = [] {
        const char *e = std::getenv("DL_GEMM_STG2");
        const int k = e ? std::atoi(e) : kGemmStages;
        return k >= 1 && k <= 3 ? k : kGemmStages;
    }();
    return v;
}

static int gemmStages1() {  // stage buffers of the 16-token tile (DL_GEMM_STG1 = 2..4, read once)
    static const int v = [] {
        const char *e = std::getenv("DL_GEMM_STG1");
        const int k = e ? std::atoi(e) : kGemmStages;
        return k >= 2 && k <= 4 ? k : kGemmStages;
    }();
    return v;
}

void launchGemmQ40(const GemmArgs &ga, int epi, hipStream_t s) {
    const int tiles = (ga.e.rows + kGemmRows - 1) / kGemmRows;
    const int MT = gemmTokenPad(ga.M) / 16;
    const int stg = MT == 4 ? gemmStages4() : MT == 2 ? gemmStages2() : gemmStages1();
    const dim3 grid(tiles, ga.splits);
    const size_t lds = gemmLds(MT, stg);
#define DL_GEMM_CASE(M_, E, G)                                                                    \
    if (MT == M_ && epi == E && stg == G) {                                                       \
        if (lds > 65536) allowLds((const void *)gemmQ40Kernel<M_, E, G>, lds); /* per device */  \
        hipLaunchKernelGGL((gemmQ40Kernel<M_, E, G>), grid, dim3(kThreads), lds, s, ga);         \
        return;                                                                                   \
    }
#define DL_GEMM_CASES(M_, G)                                                                      \
    DL_GEMM_CASE(M_, EPI_STORE, G) DL_GEMM_CASE(M_, EPI_ACT, G) DL_GEMM_CASE(M_, EPI_ACT_Q80, G)  \
    DL_GEMM_CASE(M_, EPI_QKV, G) DL_GEMM_CASE(M_, EPI_ACT_F16, G) DL_GEMM_CASE(M_, EPI_RES, G)
    DL_GEMM_CASES(1, kGemmStages) DL_GEMM_CASES(1, 3) DL_GEMM_CASES(1, 4) DL_GEMM_CASES(2, kGemmStages) DL_GEMM_CASES(2, 1) DL_GEMM_CASES(2, 3) DL_GEMM_CASES(4, 1) DL_GEMM_CASES(4, 2)
#undef DL_GEMM_CASES
#undef DL_GEMM_CASE
}

// Batched matmul for F32 weights on MFMA (the reference runs F32 batches through
// llamafile_sgemm, nn-cpu-ops.cpp:1018-1037): out[t][row] = sum_k W[row][k] x[t][k], W f32
// row-major [rows][n] (exact: v_mfma_f32_16x16x4_f32), x f16 as on the Q40 path (the only
// rounding). A wave owns 16 rows; per 32-k step lane (col, h) streams 32 B of its row col
// (k = 8h .. 8h+7: 4 lanes cover a 128-B line) straight into VGPRs - no LDS for the weights,
// which are read once - and the matching 16 B of f16 activations per token tile (L2-resident,
// shared by the workgroup's waves). Element e of those 8 feeds MFMA e on both operands (k = 8h+e,
// a permutation of k). 4 steps are issued per iteration so 4 x 32 B per lane stay in flight.
// Split-K, the deterministic combine and the fused epilogues are the Q40 GEMM's (gemmFinish).
template <int MT, int EPI>
__global__ __launch_bounds__(kThreads) void gemmF32Kernel(GemmArgs ga) {
    const GemvArgs &a = ga.e;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int *flag = reinterpret_cast<int *>(smem + MT * 16 * kGemmRows * 4);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 15, h = lane >> 4;
    const int n = a.n, kps = n / ga.splits, k0 = blockIdx.y * kps;
    const int row = min(blockIdx.x * kGemmRows + wave * 16 + col, a.rows - 1);  // clamped: outputs dropped
    const float *wp = a.wf + (size_t)row * n + k0 + 8 * h;
    const _Float16 *xp = ga.x + (size_t)col * n + k0 + 8 * h;
    f32x4 acc[MT];
#pragma unroll
    for (int t = 0; t < MT; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    constexpr int U = 4;
    int k = 0;
    for (; k + 32 * U <= kps; k += 32 * U) {
        f32x4 w[U][2];
        half8 xv[U][MT];
#pragma unroll
        for (int u = 0; u < U; u++) {
            w[u][0] = *reinterpret_cast<const f32x4 *>(wp + k + 32 * u);
            w[u][1] = *reinterpret_cast<const f32x4 *>(wp + k + 32 * u + 4);
#pragma unroll
            for (int t = 0; t < MT; t++) xv[u][t] = *reinterpret_cast<const half8 *>(xp + (size_t)t * 16 * n + k + 32 * u);
        }
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int e = 0; e < 8; e++)
#pragma unroll
                for (int t = 0; t < MT; t++)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)xv[u][t][e], w[u][e >> 2][e & 3], acc[t], 0, 0, 0);
    }
    for (; k < kps; k += 32) {  // remainder steps (kps is a multiple of 32)
        const f32x4 w0 = *reinterpret_cast<const f32x4 *>(wp + k), w1 = *reinterpret_cast<const f32x4 *>(wp + k + 4);
#pragma unroll
        for (int t = 0; t < MT; t++) {
            const half8 xv = *reinterpret_cast<const half8 *>(xp + (size_t)t * 16 * n + k);
#pragma unroll
            for (int e = 0; e < 8; e++)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32((float)xv[e], e < 4 ? w0[e] : w1[e - 4], acc[t], 0, 0, 0);
        }
    }
    gemmFinish<MT, EPI>(ga, acc, smem, flag, blockIdx.x, gridDim.x);
}

void launchGemmF32(const GemmArgs &ga, int epi, hipStream_t s) {
    const int tiles = (ga.e.rows + kGemmRows - 1) / kGemmRows;
    const int MT = gemmTokenPad(ga.M) / 16;
    const dim3 grid(tiles, ga.splits);
    const size_t lds = (size_t)MT * 16 * kGemmRows * 4 + 16 + 320 * 4;  // + flag, row scales
#define DL_GEMMF_CASE(M_, E)                                                              \
    if (MT == M_ && epi == E) {                                                           \
        if (lds > 65536) allowLds((const void *)gemmF32Kernel<M_, E>, lds);               \
        hipLaunchKernelGGL((gemmF32Kernel<M_, E>), grid, dim3(kThreads), lds, s, ga);     \
        return;                                                                           \
    }
#define DL_GEMMF_CASES(M_)                                                                \
    DL_GEMMF_CASE(M_, EPI_STORE) DL_GEMMF_CASE(M_, EPI_ACT) DL_GEMMF_CASE(M_, EPI_QKV)    \
    DL_GEMMF_CASE(M_, EPI_ACT_F16) DL_GEMMF_CASE(M_, EPI_RES)
    DL_GEMMF_CASES(1) DL_GEMMF_CASES(2) DL_GEMMF_CASES(4)
#undef DL_GEMMF_CASES
#undef DL_GEMMF_CASE
    throw Error("launchGemmF32: unsupported epilogue");
}

// Residual add + RMS norm (optional) of M rows -> f16 (one workgroup per row): the batched
// path's replacement for the GEMV's per-workgroup norm prologue.
__global__ __launch_bounds__(kThreads) void normF16Kernel(GemvArgs a, _Float16 *out) {
    __shared__ float scratch[64];
    constexpr int PV = 8;  // float4 per thread kept in registers (n <= 8192 in one pass)
    const int b = blockIdx.x, n = a.n, tid = threadIdx.x;
    const float *x = a.in + (size_t)b * a.ldIn;
    const float *y = a.addIn ? a.addIn + (size_t)b * a.ldIn : nullptr;
    float *xo = a.xNext ? a.xNext + (size_t)b * a.ldIn : nullptr;
    _Float16 *o = out + (size_t)b * n;
    const bool inReg = n <= kThreads * 4 * PV;
    float4 v[PV], gw[PV];
    float ss = 0.f;
    if (inReg) {
        // every load (x, the residual delta and the norm weights) is issued before any is used:
        // one memory round trip before the reduction instead of three
        float4 w[PV];
#pragma unroll
        for (int k = 0; k < PV; k++) {
            const int i = min((tid + k * kThreads) * 4, n - 4);
            v[k] = ld4(x + i);
            w[k] = y ? ld4(y + i) : make_float4(0.f, 0.f, 0.f, 0.f);
            gw[k] = a.normW ? ld4(a.normW + i) : make_float4(1.f, 1.f, 1.f, 1.f);
        }
#pragma unroll
        for (int k = 0; k < PV; k++) {
            const int i = (tid + k * kThreads) * 4;
            if (i < n) {
                v[k].x += w[k].x; v[k].y += w[k].y; v[k].z += w[k].z; v[k].w += w[k].w;
                if (xo) st4(xo + i, v[k]);
                ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
            }
        }
    } else {
        for (int i = tid * 4; i < n; i += kThreads * 4) {
            float4 u = ld4(x + i);
            if (y) {
                const float4 w = ld4(y + i);
                u.x += w.x; u.y += w.y; u.z += w.z; u.w += w.w;
            }
            if (xo) st4(xo + i, u);
            ss += u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w;
        }
    }
    float inv = 1.0f;
    if (a.normW) {
        ss = blockSum<kThreads>(ss, scratch);
        inv = 1.0f / sqrtf(ss / (float)n + a.eps);
    }
    auto emit = [&](int i, float4 u, const float4 *gp) {
        const float4 g = gp ? *gp : (a.normW ? ld4(a.normW + i) : make_float4(1.f, 1.f, 1.f, 1.f));
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        const h4 r = {(_Float16)(g.x * (inv * u.x)), (_Float16)(g.y * (inv * u.y)), (_Float16)(g.z * (inv * u.z)),
                      (_Float16)(g.w * (inv * u.w))};
        *reinterpret_cast<h4 *>(o + i) = r;
    };
    if (inReg) {
#pragma unroll
        for (int k = 0; k < PV; k++) {
            const int i = (tid + k * kThreads) * 4;
            if (i < n) emit(i, v[k], &gw[k]);
        }
    } else {
        for (int i = tid * 4; i < n; i += kThreads * 4) {
            float4 u = xo ? ld4(xo + i) : ld4(x + i);
            if (!xo && y) {
                const float4 w = ld4(y + i);
                u.x += w.x; u.y += w.y; u.z += w.z; u.w += w.w;
            }
            emit(i, u, nullptr);
        }
    }
}

void launchNormF16(const GemvArgs &a, _Float16 *out, int M, hipStream_t s) {
    hipLaunchKernelGGL(normF16Kernel, dim3(M), dim3(kThreads), 0, s, a, out);
}

// ------------------------------------------------------------------------------------------------
// Attention (decode / prefill rows): split the sequence [0, pos] into chunks, one workgroup per
// (head group, chunk, row). A single chunk writes the final output directly; with several chunks
// each workgroup publishes its online-softmax partial and the last arriver combines them.
// ------------------------------------------------------------------------------------------------
int attnSplitGrid(int seqLen) {
    int g = (seqLen + 255) / 256;
    return g < 1 ? 1 : (g > 128 ? 128 : g);
}

int attnChunkMax(int seqLen, int splitGrid) {
    int per = (seqLen + splitGrid - 1) / splitGrid;
    if (per < 256) per = 256;
    return ((per + 15) / 16) * 16 + 16;
}


template <int DPL, bool BF16>
__device__ __forceinline__ void loadKv(const void *base, size_t off, float (&v)[DPL]) {
    if constexpr (BF16) {
        const uint16_t *p = reinterpret_cast<const uint16_t *>(base) + off;
        if constexpr (DPL == 8) {
            const uint4 r = *reinterpret_cast<const uint4 *>(p);
            const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                v[2 * i] = __uint_as_float(w[i] << 16);
                v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
            }
        } else if constexpr (DPL == 4) {
            const uint2 r = *reinterpret_cast<const uint2 *>(p);
            v[0] = __uint_as_float(r.x << 16);
            v[1] = __uint_as_float(r.x & 0xFFFF0000u);
            v[2] = __uint_as_float(r.y << 16);
            v[3] = __uint_as_float(r.y & 0xFFFF0000u);
        } else if constexpr (DPL == 2) {
            const uint32_t r = *reinterpret_cast<const uint32_t *>(p);
            v[0] = __uint_as_float(r << 16);
            v[1] = __uint_as_float(r & 0xFFFF0000u);
        } else {
            v[0] = bf16ToF32(p[0]);
        }
    } else {
        const float *p = reinterpret_cast<const float *>(base) + off;
#pragma unroll
        for (int i = 0; i < DPL; i++) v[i] = p[i];
    }
}

// Final output of HG heads from LDS fin[HG][HS] -> f32 or Q80 (32-element blocks) in global.
template <int HG, int HS, int AT>
__device__ __forceinline__ void attnWriteOut(const AttnArgs &a, int b, int head0, const float *fin) {
    const int tid = threadIdx.x;
    if (a.outQ) {
        for (int i = tid; i < HG * HS; i += AT) {  // 32-lane groups = one Q80 block
            const float v = fin[i];
            const float amax = groupMax<32>(fabsf(v));
            const float d = amax / 127.0f;
            const float id = d != 0.f ? 1.0f / d : 0.f;
            int q = (int)rintf(v * id);
            q = q > 127 ? 127 : (q < -127 ? -127 : q);
            const int col = head0 * HS + i;
            a.outQ[(size_t)b * a.ldOut + col] = (int8_t)q;
            const float qs = groupSum<32>((float)q);
            if ((i & 31) == 0) a.outS[(size_t)b * (a.ldOut >> 5) + (col >> 5)] = make_float2(roundF16(d), qs);
        }
    } else if (a.outH) {
        for (int i = tid; i < HG * HS; i += AT) a.outH[(size_t)b * a.ldOut + head0 * HS + i] = (_Float16)fin[i];
    } else {
        for (int i = tid; i < HG * HS; i += AT) a.out[(size_t)b * a.ldOut + head0 * HS + i] = fin[i];
    }
}

// Online-softmax merge of (m2, l2, o2) into (m, l, o).
template <int D>
__device__ __forceinline__ void softmaxMerge(float &m, float &l, float (&o)[D], float m2, float l2, const float (&o2)[D]) {
    const float mn = fmaxf(m, m2);
    const float c1 = mn == -INFINITY ? 0.f : __expf(m - mn);
    const float c2 = mn == -INFINITY ? 0.f : __expf(m2 - mn);
    l = l * c1 + l2 * c2;
#pragma unroll
    for (int i = 0; i < D; i++) o[i] = o[i] * c1 + o2[i] * c2;
    m = mn;
}

static constexpr int kAttnThreads = 512;  // 8 waves = 32 groups of 16 lanes, one key per group

// Split epilogue of the attention kernel: redL [HG][HS] holds the unnormalised output of this
// workgroup's chunk, mlL [HG][2] its (max, sum). One chunk: normalise and write. Several: publish
// the partial and count arrivals; the last workgroup combines all chunks. The combine stages every
// chunk's (max, sum) in LDS (`scratch`, >= 2 * HG * splitGrid floats) with one load per thread and
// keeps 8 partial-output loads in flight per thread: a serial loop over the chunks costs one
// cross-XCD round trip per chunk (~30 us at 32 chunks).
template <int HG, int HS, int AT>
__device__ __forceinline__ bool attnFinish(const AttnArgs &a, int b, int hgIdx, int c, int nSplit, float *redL,
                                           float *mlL, int *flagL, float *scratch) {
    const int tid = threadIdx.x, head0 = hgIdx * HG;
    if (nSplit == 1) {
        for (int i = tid; i < HG * HS; i += AT) redL[i] = redL[i] / mlL[(i / HS) * 2 + 1];
        __syncthreads();
        attnWriteOut<HG, HS, AT>(a, b, head0, redL);
        return true;
    }
    const int G = a.splitGrid;
    const size_t pbase = ((size_t)b * a.nHeads0 + head0) * G;  // [HG][G] chunks of this head group
    // fence-free hand-off (as gemmFinish): partials stored and read back with agent-scope atomic
    // accesses (sc1, performed at the coherence point), vmcnt(0) before the arrival count; an
    // agent-scope fence would write back / invalidate this XCD's whole L2
    auto st = [](float *q, float v) { __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto ld = [](const float *q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    for (int i = tid; i < HG * HS; i += AT) {
        const int h = i / HS, d = i % HS;
        st(a.partO + ((pbase + (size_t)h * G) + c) * HS + d, redL[i]);
    }
    if (tid < HG) {
        st(a.partML + ((pbase + (size_t)tid * G) + c) * 2, mlL[tid * 2]);
        st(a.partML + ((pbase + (size_t)tid * G) + c) * 2 + 1, mlL[tid * 2 + 1]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int *cnt = a.counters + (size_t)b * (a.nHeads0 / HG) + hgIdx;
    if (tid == 0) {
        const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flagL[0] = old == nSplit - 1;
    }
    __syncthreads();
    if (!flagL[0]) return false;
    if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every chunk's (max, sum) -> LDS, then per head: global max and chunk weights w = exp(m - M)
    for (int i = tid; i < HG * nSplit; i += AT) {
        const int h = i / nSplit, cc = i % nSplit;
        const float *ml = a.partML + ((pbase + (size_t)h * G) + cc) * 2;
        scratch[2 * (h * G + cc)] = ld(ml);
        scratch[2 * (h * G + cc) + 1] = ld(ml + 1);
    }
    __syncthreads();
    if (tid < HG) {
        float M = -INFINITY;
        for (int cc = 0; cc < nSplit; cc++) M = fmaxf(M, scratch[2 * (tid * G + cc)]);
        float Ls = 0.f;
        for (int cc = 0; cc < nSplit; cc++) {
            float *ml = scratch + 2 * (tid * G + cc);
            const float w = M == -INFINITY ? 0.f : __expf(ml[0] - M);
            ml[0] = w;
            Ls += w * ml[1];
        }
        mlL[tid * 2 + 1] = Ls;
    }
    __syncthreads();
    constexpr int U = 8;
    for (int i = tid; i < HG * HS; i += AT) {
        const int h = i / HS, d = i % HS;
        const float *po = a.partO + (pbase + (size_t)h * G) * HS + d;
        const float *wv = scratch + 2 * h * G;
        float acc = 0.f;
        int cc = 0;
        for (; cc + U <= nSplit; cc += U) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = ld(po + (size_t)(cc + u) * HS);
#pragma unroll
            for (int u = 0; u < U; u++) acc += wv[2 * (cc + u)] * v[u];
        }
        for (; cc < nSplit; cc++) acc += wv[2 * cc] * ld(po + (size_t)cc * HS);
        redL[i] = acc / mlL[h * 2 + 1];
    }
    __syncthreads();
    attnWriteOut<HG, HS, AT>(a, b, head0, redL);
    return true;
}

// One attention task: query heads [hgIdx*HG, +HG) of row b over sequence chunk c, AT threads.
// Returns true when this call wrote the head group's final output (single chunk, or the last
// chunk to arrive combined all of them).
template <int HG, int HS, bool BF16, int AT>
__device__ __forceinline__ bool attnTask(const AttnArgs &a, int b, int hgIdx, int c, char *smem) {
    constexpr int NW = AT / 64, NG = AT / 16;
    constexpr int DPL = HS / 16;           // dims per lane: 16 lanes cover one position's head vector
    constexpr int TU = BF16 ? 8 : 4;       // keys per group loaded before any is consumed
    constexpr int RW = BF16 ? DPL / 2 : DPL;  // 32-bit words per lane per key (packed bf16 pairs)
    const int pos = a.pos[b], sl = a.slot[b];
    const int len = pos + 1;
    int nSplit, ch;
    attnSplit(len, a.splitGrid, nSplit, ch);
    if (c >= nSplit) return false;
    const int t0 = c * ch;
    const int t1 = min(t0 + ch, len);
    const int head0 = hgIdx * HG;
    const int kvh = head0 / a.kvMul;
    const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
    const int g16 = tid / 16, l16 = tid % 16;

    float *mW = reinterpret_cast<float *>(smem);    // [NW][HG]
    float *lW = mW + NW * HG;                       // [NW][HG]
    float *oW = lW + NW * HG;                       // [NW][HG][HS]
    float *redL = oW + NW * HG * HS;                // [HG][HS] final (unnormalized) o
    float *mlL = redL + HG * HS;                    // [HG][2]
    int *flagL = reinterpret_cast<int *>(mlL + 2 * HG);

    // this lane's slice of the HG query heads (pre-scaled), vector loads
    const float scale = 1.0f / sqrtf((float)HS);
    float qr[HG][DPL];
#pragma unroll
    for (int h = 0; h < HG; h++) {
        const float *qp = a.q + (size_t)b * a.ldq + (head0 + h) * HS + l16 * DPL;
#pragma unroll
        for (int i = 0; i < DPL; i += 4) {
            const float4 v = ld4(qp + i);
            qr[h][i] = v.x * scale;
            qr[h][i + 1] = v.y * scale;
            qr[h][i + 2] = v.z * scale;
            qr[h][i + 3] = v.w * scale;
        }
    }
    float m[HG], l[HG], o[HG][DPL];
#pragma unroll
    for (int h = 0; h < HG; h++) {
        m[h] = -INFINITY;
        l[h] = 0.f;
#pragma unroll
        for (int i = 0; i < DPL; i++) o[h][i] = 0.f;
    }
    // each 16-lane group walks keys g16, g16+NG, ... with a running softmax; TU keys per group are
    // in flight at once (NG*TU = 256 keys per memory round trip for bf16 caches)
    const size_t slotBase = (size_t)sl * a.seqLen;
    for (int tb = t0 + g16; tb < t1; tb += TU * NG) {
        uint32_t kr[TU][RW], vr[TU][RW];
#pragma unroll
        for (int u = 0; u < TU; u++) {
            const int t = min(tb + u * NG, t1 - 1);  // clamped: no divergent loads
            const size_t off = (slotBase + t) * a.kv0 + kvh * HS + l16 * DPL;
            const uint32_t *kp = reinterpret_cast<const uint32_t *>(
                BF16 ? (const void *)(reinterpret_cast<const uint16_t *>(a.kcache) + off)
                     : (const void *)(reinterpret_cast<const float *>(a.kcache) + off));
            const uint32_t *vp = reinterpret_cast<const uint32_t *>(
                BF16 ? (const void *)(reinterpret_cast<const uint16_t *>(a.vcache) + off)
                     : (const void *)(reinterpret_cast<const float *>(a.vcache) + off));
            if constexpr (RW == 4) {
                const uint4 k4 = *reinterpret_cast<const uint4 *>(kp), v4 = *reinterpret_cast<const uint4 *>(vp);
                kr[u][0] = k4.x; kr[u][1] = k4.y; kr[u][2] = k4.z; kr[u][3] = k4.w;
                vr[u][0] = v4.x; vr[u][1] = v4.y; vr[u][2] = v4.z; vr[u][3] = v4.w;
            } else if constexpr (RW == 8) {
                const uint4 k0 = reinterpret_cast<const uint4 *>(kp)[0], k1 = reinterpret_cast<const uint4 *>(kp)[1];
                const uint4 v0 = reinterpret_cast<const uint4 *>(vp)[0], v1 = reinterpret_cast<const uint4 *>(vp)[1];
                kr[u][0] = k0.x; kr[u][1] = k0.y; kr[u][2] = k0.z; kr[u][3] = k0.w;
                kr[u][4] = k1.x; kr[u][5] = k1.y; kr[u][6] = k1.z; kr[u][7] = k1.w;
                vr[u][0] = v0.x; vr[u][1] = v0.y; vr[u][2] = v0.z; vr[u][3] = v0.w;
                vr[u][4] = v1.x; vr[u][5] = v1.y; vr[u][6] = v1.z; vr[u][7] = v1.w;
            } else {
                const uint2 k2 = *reinterpret_cast<const uint2 *>(kp), v2 = *reinterpret_cast<const uint2 *>(vp);
                kr[u][0] = k2.x; kr[u][1] = k2.y;
                vr[u][0] = v2.x; vr[u][1] = v2.y;
            }
        }
#pragma unroll
        for (int u = 0; u < TU; u++) {
            if (tb + u * NG >= t1) break;  // uniform within the 16-lane group
            float kv[DPL], vv[DPL];
#pragma unroll
            for (int w = 0; w < RW; w++) {
                if constexpr (BF16) {
                    kv[2 * w] = __uint_as_float(kr[u][w] << 16);
                    kv[2 * w + 1] = __uint_as_float(kr[u][w] & 0xFFFF0000u);
                    vv[2 * w] = __uint_as_float(vr[u][w] << 16);
                    vv[2 * w + 1] = __uint_as_float(vr[u][w] & 0xFFFF0000u);
                } else {
                    kv[w] = __uint_as_float(kr[u][w]);
                    vv[w] = __uint_as_float(vr[u][w]);
                }
            }
#pragma unroll
            for (int h = 0; h < HG; h++) {
                float d = 0.f;
#pragma unroll
                for (int i = 0; i < DPL; i++) d += qr[h][i] * kv[i];
                d = groupSum<16>(d);
                const float mn = fmaxf(m[h], d);
                const float corr = __expf(m[h] - mn);  // m = -inf first time -> 0
                const float p = __expf(d - mn);
                l[h] = l[h] * corr + p;
#pragma unroll
                for (int i = 0; i < DPL; i++) o[h][i] = o[h][i] * corr + p * vv[i];
                m[h] = mn;
            }
        }
    }
    // merge the 4 position groups of each wave (lanes l, l^16, l^32, l^48 share dims)
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
#pragma unroll
        for (int h = 0; h < HG; h++) {
            const float m2 = __shfl_xor(m[h], off), l2 = __shfl_xor(l[h], off);
            float o2[DPL];
#pragma unroll
            for (int i = 0; i < DPL; i++) o2[i] = __shfl_xor(o[h][i], off);
            softmaxMerge<DPL>(m[h], l[h], o[h], m2, l2, o2);
        }
    }
    if (lane < 16) {
#pragma unroll
        for (int h = 0; h < HG; h++) {
            if (lane == 0) {
                mW[wave * HG + h] = m[h];
                lW[wave * HG + h] = l[h];
            }
#pragma unroll
            for (int i = 0; i < DPL; i++) oW[(wave * HG + h) * HS + lane * DPL + i] = o[h][i];
        }
    }
    __syncthreads();
    // merge the NW waves
    for (int i = tid; i < HG * HS; i += AT) {
        const int h = i / HS;
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < NW; w++) M = fmaxf(M, mW[w * HG + h]);
        float acc = 0.f, Ls = 0.f;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const float e = M == -INFINITY ? 0.f : __expf(mW[w * HG + h] - M);
            acc += e * oW[(w * HG + h) * HS + (i % HS)];
            Ls += e * lW[w * HG + h];
        }
        redL[i] = acc;
        if (i % HS == 0) {
            mlL[h * 2] = M;
            mlL[h * 2 + 1] = Ls;
        }
    }
    __syncthreads();

    return attnFinish<HG, HS, AT>(a, b, hgIdx, c, nSplit, redL, mlL, flagL, oW);
}

template <int HG, int HS, bool BF16>
__global__ __launch_bounds__(kAttnThreads) void attnKernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int hgx = a.nHeads0 / HG;  // attention workgroups per (split, row) slice
    if ((int)blockIdx.x >= hgx) {
        // MALL warm-up role: every extra workgroup of every slice streams its share of the next
        // GEMVs' weights with plain loads (allocating in the Infinity Cache) and discards them
        const int pfx = gridDim.x - hgx;
        const int id = (blockIdx.z * gridDim.y + blockIdx.y) * pfx + (blockIdx.x - hgx);
        const int nPf = pfx * gridDim.y * gridDim.z;
        typedef unsigned int u32x4l __attribute__((ext_vector_type(4)));
        const size_t n0 = a.pf0Bytes / 16, n1 = a.pf1Bytes / 16, tot = n0 + n1;
        const size_t per = (tot + nPf - 1) / nPf;
        const size_t i0 = (size_t)id * per, i1 = min(i0 + per, tot);
        const u32x4l *p0 = reinterpret_cast<const u32x4l *>(a.pf0), *p1 = reinterpret_cast<const u32x4l *>(a.pf1);
        u32x4l acc = {0u, 0u, 0u, 0u};
        for (size_t i = i0 + threadIdx.x; i < i1; i += 4 * kAttnThreads) {
            u32x4l v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const size_t j = min(i + (size_t)u * kAttnThreads, i1 - 1);
                v[u] = j < n0 ? p0[j] : p1[j - n0];
            }
#pragma unroll
            for (int u = 0; u < 4; u++) acc ^= v[u];
        }
        asm volatile("" ::"v"(acc.x), "v"(acc.y), "v"(acc.z), "v"(acc.w));
        return;
    }
    attnTask<HG, HS, BF16, kAttnThreads>(a, blockIdx.z, blockIdx.x, blockIdx.y, smem);
}

template <int HS, bool BF16>
static void attnDispatchHG(const AttnArgs &a, int B, int HG, hipStream_t s) {
    constexpr int NW = kAttnThreads / 64;
    int pfx = 0;  // extra MALL warm-up workgroups per slice (see attnKernel)
    if (a.pfBlocks > 0 && (a.pf0Bytes + a.pf1Bytes) >= 16) pfx = (a.pfBlocks + a.splitGrid * B - 1) / (a.splitGrid * B);
    const size_t lds = sizeof(float) * (2 * NW * HG + NW * HG * HS + HG * HS + 2 * HG) + 16;
    const dim3 grid(a.nHeads0 / HG + pfx, a.splitGrid, B);
    switch (HG) {
        case 1: hipLaunchKernelGGL((attnKernel<1, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
        case 2: hipLaunchKernelGGL((attnKernel<2, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
        case 4: hipLaunchKernelGGL((attnKernel<4, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
        default: hipLaunchKernelGGL((attnKernel<8, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
    }
}

void launchAttention(const AttnArgs &a, int B, hipStream_t s) {
    static const int hgOverride = [] {  // experiments: DL_ATTN_HG forces query heads per workgroup
        const char *e = getenv("DL_ATTN_HG");
        return e ? atoi(e) : 0;
    }();
    // Query heads per workgroup: sharing a KV head's loads between HG heads costs HG x the serial
    // work per workgroup, so take the fewest heads per workgroup that keep the grid (at the
    // longest context this launch can see) within one workgroup per CU. Measured on MI355X
    // (scripts/bench_attn.py, profiles/r1_attention.md): short contexts 7.9 -> 5.9 us (TP1) and
    // 7.7 -> 4.4 us (TP8) with one head per workgroup; long contexts keep 2-4 heads per workgroup.
    const int hgMax = (a.kvMul & (a.kvMul - 1)) == 0 ? (a.kvMul < 8 ? a.kvMul : 8) : 1;
    int HG = 1;
    while (HG < hgMax && (long)(a.nHeads0 / HG) * a.splitGrid * B > 256) HG *= 2;
    if (hgOverride > 0 && hgOverride <= hgMax && hgMax % hgOverride == 0) HG = hgOverride;
    if (a.hs == 128) {
        if (a.kvBf16) attnDispatchHG<128, true>(a, B, HG, s);
        else attnDispatchHG<128, false>(a, B, HG, s);
    } else if (a.hs == 64) {
        if (a.kvBf16) attnDispatchHG<64, true>(a, B, HG, s);
        else attnDispatchHG<64, false>(a, B, HG, s);
    }
}

// ------------------------------------------------------------------------------------------------
// Prefill attention on MFMA (batched path, bf16 KV cache; reference: the per-row causal attention of
// nn-cpu-ops.cpp:1135-1161 run for every prompt row). The decode kernel above walks the context once
// per row, so a 32-row chunk at position p re-reads 32 x p keys; here a workgroup owns one KV head
// and a block of rows of one slot (16 / kvMul rows per wave, one column per (row, query head)) and
// every key is read once per block:
//   S^T = K . Q^T   (v_mfma_f32_16x16x32_bf16: A = 16 keys x 32 dims from the LDS K tile,
//                    B = Q^T in registers), causal mask per column (key <= the row's position)
//   P^T = exp(S^T - m) with the online softmax per column (the lanes of column l & 15)
//   O^T += V^T . P^T (A = V^T from an LDS tile stored transposed, B = P^T straight from the S^T
//                    accumulators: both operands use the same permuted key order)
// K / V tiles of 32 keys are staged global -> registers -> LDS (double-buffered, the next tile's
// loads in flight during the current tile's MFMAs). Long contexts split the keys into chunks of
// 256 over grid.y; the last-arriving chunk combines the partials (as attnFinish).
// ------------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
static constexpr int kPfThreads = 256, kPfWaves = 4, kPfChunk = 256, kPfTile = 32;
static constexpr int kPfVtStride = 40;  // bf16 per transposed-V row in LDS (32 keys + 8 pad)

int attnPrefillRowsPerBlock(int kvMul) { return kPfWaves * (16 / kvMul); }
bool attnPrefillSupported(int hs, int kvMul, bool kvBf16) {
    return kvBf16 && (hs == 64 || hs == 128) && kvMul >= 1 && kvMul <= 16 && (kvMul & (kvMul - 1)) == 0;
}

__device__ __forceinline__ bf16x8 f32x8ToBf16(const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = (__bf16)v[j];
    return r;
}

template <int HS>
__global__ __launch_bounds__(kPfThreads) void attnPrefillKernel(AttnArgs a, int nRows) {
    constexpr int DS = HS / 32, NT = HS / 16;
    constexpr int U8 = HS / 8;                        // 16-byte units per key row
    constexpr int PER = kPfTile * U8 / kPfThreads;    // 16-byte units per thread per operand and tile
    static_assert(PER >= 1, "tile too small for the workgroup");
    __shared__ __attribute__((aligned(16))) __bf16 kT[2][kPfTile * HS];
    __shared__ __attribute__((aligned(16))) __bf16 vT[2][HS * kPfVtStride];
    __shared__ int flagL;
    const int kvMul = a.kvMul, rpw = 16 / kvMul, rpb = kPfWaves * rpw, nKv = a.nHeads0 / kvMul;
    const int g = blockIdx.x % nKv, rb = blockIdx.x / nKv, c = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 15, h = lane >> 4;
    const int b0 = rb * rpb;
    int maxLen = 0;
    for (int r = 0; r < rpb && b0 + r < nRows; r++) maxLen = max(maxLen, a.pos[b0 + r] + 1);
    int nSplit = (maxLen + kPfChunk - 1) / kPfChunk;
    nSplit = max(1, min(min(nSplit, a.splitGrid), HS / 2));  // combine weights: 64 columns x nSplit in the K tiles' LDS
    const int ch = ((maxLen + nSplit - 1) / nSplit + kPfTile - 1) / kPfTile * kPfTile;
    if (c >= nSplit) return;
    const int k0 = c * ch, k1 = min(k0 + ch, maxLen);
    const int sl = a.slot[b0];  // every row of the block (host-checked)
    // this lane's column
    const int row = b0 + wave * rpw + col / kvMul, head = g * kvMul + col % kvMul;
    const bool rowOk = row < nRows;
    const int myLen = rowOk ? a.pos[row] + 1 : 0;
    const float scale = 1.0f / sqrtf((float)HS);
    bf16x8 qf[DS];
#pragma unroll
    for (int s = 0; s < DS; s++) {
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (rowOk) {
            const float *qp = a.q + (size_t)row * a.ldq + (size_t)head * HS + 32 * s + 8 * h;
            const float4 x0 = ld4(qp), x1 = ld4(qp + 4);
            v[0] = x0.x * scale; v[1] = x0.y * scale; v[2] = x0.z * scale; v[3] = x0.w * scale;
            v[4] = x1.x * scale; v[5] = x1.y * scale; v[6] = x1.z * scale; v[7] = x1.w * scale;
        }
        qf[s] = f32x8ToBf16(v);
    }
    const uint16_t *kc = reinterpret_cast<const uint16_t *>(a.kcache);
    const uint16_t *vc = reinterpret_cast<const uint16_t *>(a.vcache);
    const size_t kvBase = (size_t)sl * a.seqLen * a.kv0 + (size_t)g * HS;
    u32x4 kr[PER], vr[PER];
    auto gload = [&](int t0) {
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int e = tid + u * kPfThreads;
            const int key = min(t0 + e / U8, a.seqLen - 1);  // past the range: masked in compute
            const size_t off = kvBase + (size_t)key * a.kv0 + (e % U8) * 8;
            kr[u] = *reinterpret_cast<const u32x4 *>(kc + off);
            vr[u] = *reinterpret_cast<const u32x4 *>(vc + off);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int e = tid + u * kPfThreads, kk = e / U8, d0 = (e % U8) * 8;
            *reinterpret_cast<u32x4 *>(&kT[buf][kk * HS + d0]) = kr[u];
            const uint32_t w[4] = {vr[u].x, vr[u].y, vr[u].z, vr[u].w};
            uint16_t *vt = reinterpret_cast<uint16_t *>(&vT[buf][0]);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                vt[(d0 + 2 * j) * kPfVtStride + kk] = (uint16_t)(w[j] & 0xFFFFu);
                vt[(d0 + 2 * j + 1) * kPfVtStride + kk] = (uint16_t)(w[j] >> 16);
            }
        }
    };
    f32x4 o[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    auto compute = [&](int buf, int t0) {
        f32x4 st[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            st[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < DS; s++) {
                const bf16x8 kf = *reinterpret_cast<const bf16x8 *>(&kT[buf][(16 * u + col) * HS + 32 * s + 8 * h]);
                st[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], st[u], 0, 0, 0);
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int t = t0 + 16 * u + 4 * h + i;
                if (t >= k1 || t >= myLen) st[u][i] = -INFINITY;
                mx = fmaxf(mx, st[u][i]);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        const float mn = fmaxf(m, mx);
        const float corr = m == -INFINITY ? 0.f : __expf(m - mn);
        float p[8], ps = 0.f;
#pragma unroll
        for (int u = 0; u < 2; u++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                p[4 * u + i] = st[u][i] == -INFINITY ? 0.f : __expf(st[u][i] - mn);
                ps += p[4 * u + i];
            }
        lsum = lsum * corr + ps;
        m = mn;
        const bf16x8 pf = f32x8ToBf16(p);
#pragma unroll
        for (int n = 0; n < NT; n++) {
            const __bf16 *vrow = &vT[buf][(16 * n + col) * kPfVtStride];
            const bf16x4 lo = *reinterpret_cast<const bf16x4 *>(vrow + 4 * h);
            const bf16x4 hi = *reinterpret_cast<const bf16x4 *>(vrow + 16 + 4 * h);
            const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            o[n] *= corr;
            o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[n], 0, 0, 0);
        }
    };
    gload(k0);
    lstore(0);
    __syncthreads();
    int buf = 0;
    for (int t0 = k0; t0 < k1; t0 += kPfTile, buf ^= 1) {
        const bool more = t0 + kPfTile < k1;
        if (more) gload(t0 + kPfTile);
        compute(buf, t0);
        if (more) lstore(buf ^ 1);
        __syncthreads();
    }
    lsum += __shfl_xor(lsum, 16);
    lsum += __shfl_xor(lsum, 32);
    // O^T accumulators: lane holds O[column][dim 16 n + 4 h + i]
    auto writeOut = [&](int r, int hd, int d, const float (&v)[4]) {
        const size_t at = (size_t)r * a.ldOut + (size_t)hd * HS + d;
        if (a.outH) {
            typedef _Float16 h4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<h4 *>(a.outH + at) = h4{(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
        } else {
            *reinterpret_cast<float4 *>(a.out + at) = make_float4(v[0], v[1], v[2], v[3]);
        }
    };
    if (nSplit == 1) {
        if (rowOk) {
            const float il = lsum > 0.f ? 1.0f / lsum : 0.f;
#pragma unroll
            for (int n = 0; n < NT; n++) {
                const float v[4] = {o[n][0] * il, o[n][1] * il, o[n][2] * il, o[n][3] * il};
                writeOut(row, head, 16 * n + 4 * h, v);
            }
        }
        return;
    }
    // several chunks: publish (every column of the block, masked ones as (-inf, 0, 0)), count in,
    // the last arriver combines
    const int G = a.splitGrid;
    // fence-free hand-off (see gemmFinish): agent-scope atomic stores here, atomic loads below
    auto st = [](float *q, float v) { __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    auto ld = [](const float *q) { return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    if (rowOk) {
        const size_t pb = ((size_t)row * a.nHeads0 + head) * G + c;
#pragma unroll
        for (int n = 0; n < NT; n++)
#pragma unroll
            for (int e = 0; e < 4; e++) st(a.partO + pb * HS + 16 * n + 4 * h + e, o[n][e]);
        if (h == 0) {
            st(a.partML + pb * 2, m);
            st(a.partML + pb * 2 + 1, lsum);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int *cnt = a.counters + (size_t)rb * nKv + g;
    if (tid == 0) flagL = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nSplit - 1;
    __syncthreads();
    if (!flagL) return;
    if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // per column: chunk weights exp(m_c - M) and the total sum (LDS: the tiles are free now)
    const int nCol = rpb * kvMul;  // 64 columns
    float *wts = reinterpret_cast<float *>(&kT[0][0]);  // [nCol][nSplit]
    float *tot = reinterpret_cast<float *>(&vT[0][0]);  // [nCol]
    if (tid < nCol) {
        const int r = b0 + tid / kvMul, hd = g * kvMul + tid % kvMul;
        float M = -INFINITY, L = 0.f;
        if (r < nRows) {
            const float *ml = a.partML + ((size_t)r * a.nHeads0 + hd) * G * 2;
            for (int cc = 0; cc < nSplit; cc++) M = fmaxf(M, ld(ml + 2 * cc));
            for (int cc = 0; cc < nSplit; cc++) {
                const float mc = ld(ml + 2 * cc);
                const float w = (M == -INFINITY || mc == -INFINITY) ? 0.f : __expf(mc - M);
                wts[tid * nSplit + cc] = w;
                L += w * ld(ml + 2 * cc + 1);
            }
        }
        tot[tid] = L;
    }
    __syncthreads();
    for (int i = tid; i < nCol * (HS / 4); i += kPfThreads) {
        const int cl = i / (HS / 4), d = (i % (HS / 4)) * 4;
        const int r = b0 + cl / kvMul, hd = g * kvMul + cl % kvMul;
        if (r >= nRows) continue;
        const float *po = a.partO + ((size_t)r * a.nHeads0 + hd) * G * HS + d;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        for (int cc = 0; cc < nSplit; cc++) {
            const float w = wts[cl * nSplit + cc];
            const float *x = po + (size_t)cc * HS;
            acc[0] += w * ld(x); acc[1] += w * ld(x + 1); acc[2] += w * ld(x + 2); acc[3] += w * ld(x + 3);
        }
        const float il = tot[cl] > 0.f ? 1.0f / tot[cl] : 0.f;
        const float v[4] = {acc[0] * il, acc[1] * il, acc[2] * il, acc[3] * il};
        writeOut(r, hd, d, v);
    }
}

void launchAttentionPrefill(const AttnArgs &a, int nRows, hipStream_t s) {
    const int nKv = a.nHeads0 / a.kvMul, rpb = attnPrefillRowsPerBlock(a.kvMul);
    const dim3 grid(nKv * ((nRows + rpb - 1) / rpb), a.splitGrid);
    if (a.hs == 128) hipLaunchKernelGGL(attnPrefillKernel<128>, grid, dim3(kPfThreads), 0, s, a, nRows);
    else hipLaunchKernelGGL(attnPrefillKernel<64>, grid, dim3(kPfThreads), 0, s, a, nRows);
}

// ------------------------------------------------------------------------------------------------
// Small kernels
// ------------------------------------------------------------------------------------------------
__global__ void embeddingKernel(const float *table, const int *tokens, float *x, int dim) {
    const int b = blockIdx.x;
    const float *src = table + (size_t)tokens[b] * dim;
    float *dst = x + (size_t)b * dim;
    // all of a thread's row loads in flight before the first store (one HBM round trip, not four)
    constexpr int U = 4;
    for (int i0 = threadIdx.x * 4; i0 < dim; i0 += U * blockDim.x * 4) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + u * blockDim.x * 4;
            if (i < dim) v[u] = ld4(src + i);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + u * blockDim.x * 4;
            if (i < dim) st4(dst + i, v[u]);
        }
    }
}

void launchEmbedding(const float *table, const int *tokens, float *x, int dim, int B, hipStream_t s) {
    hipLaunchKernelGGL(embeddingKernel, dim3(B), dim3(256), 0, s, table, tokens, x, dim);
}

__device__ __forceinline__ void argBetter(float &bv, int &bi, float ov, int oi) {
    if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
    }
}

__device__ __forceinline__ void blockArgmax(float &bv, int &bi, float *sv, int *si) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) argBetter(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
    const int w = threadIdx.x / 64;
    __syncthreads();
    if (threadIdx.x % 64 == 0) {
        sv[w] = bv;
        si[w] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0)
        for (int i = 1; i < (int)(blockDim.x / 64); i++) argBetter(bv, bi, sv[i], si[i]);
}

constexpr int kArgmaxBlocks = 64;

// grid (kArgmaxBlocks, B): each workgroup reduces a slice; the last arriver reduces the partials.
__global__ __launch_bounds__(256) void argmaxKernel(ArgmaxArgs a) {
    __shared__ float sv[4];
    __shared__ int si[4];
    __shared__ int last;
    const int b = blockIdx.y;
    const float *x = a.logits + (size_t)b * a.vocab;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    // 8 loads in flight per thread per round (a plain grid-stride loop waits for each load in turn)
    constexpr int U = 8;
    const int stride = gridDim.x * blockDim.x;
    for (int i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < a.vocab; i0 += U * stride) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + u * stride;
            v[u] = i < a.vocab ? x[i] : -INFINITY;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int i = i0 + u * stride;
            if (i < a.vocab) argBetter(bv, bi, v[u], i);
        }
    }
    blockArgmax(bv, bi, sv, si);
    // fence-free hand-off (see gemmFinish): agent-scope atomic stores / loads of the partials
    if (threadIdx.x == 0) {
        __hip_atomic_store(a.partV + b * kArgmaxBlocks + blockIdx.x, bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.partI + b * kArgmaxBlocks + blockIdx.x, bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int old = __hip_atomic_fetch_add(a.counters + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = old == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    if (threadIdx.x == 0) __hip_atomic_store(a.counters + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bv = -INFINITY;
    bi = 0x7fffffff;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x)
        argBetter(bv, bi, __hip_atomic_load(a.partV + b * kArgmaxBlocks + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                  __hip_atomic_load(a.partI + b * kArgmaxBlocks + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    blockArgmax(bv, bi, sv, si);
    if (threadIdx.x == 0 && a.tp.world > 1) {
        // tensor parallel: every rank offers its slice's winner (value, global index); all ranks
        // pick the same one in rank order (ties -> lowest index, like a full-vocabulary argmax)
        const TpXchg &x = a.tp;
        const bool failed = tpFailed(x);
        const unsigned e = x.epochs[b] + 1;
        unsigned vv[kTpMaxRanks], vi[kTpMaxRanks];
        tpPushCollect(x, 2LL * b, e, __float_as_uint(bv), vv, failed);
        tpPushCollect(x, 2LL * b + 1, e, (unsigned)(bi + a.vocabStart), vi, failed);
        bv = -INFINITY;
        bi = 0x7fffffff;
        for (int p = 0; p < x.world; p++) argBetter(bv, bi, __uint_as_float(vv[p]), (int)vi[p]);
        x.epochs[b] = e;
    }
    if (threadIdx.x == 0) {
        a.ids[b] = bi;
        if (a.tokens) {
            const int p = a.pos[b];
            a.hist[(size_t)b * a.seqLen + p] = bi;
            a.tokens[b] = bi;
            a.pos[b] = p + 1;
        }
    }
}

void launchArgmax(const ArgmaxArgs &a, int B, hipStream_t s) {
    hipLaunchKernelGGL(argmaxKernel, dim3(kArgmaxBlocks, B), dim3(256), 0, s, a);
}

// ------------------------------------------------------------------------------------------------
// Device sampling (SampleArgs in kernels.h), G workgroups per row and 8 dependent phases (kernel
// boundaries are the only grid-wide synchronisation; inside a phase the last-arriving workgroup of
// a row reduces what the row's workgroups produced and writes the row's state for the next phase).
// x = logit / T; the order-preserving key of x ranks probabilities; searches are 11/11/10-bit radix
// passes over that key, each building a 2048-bin histogram of probability mass (one LDS copy per
// wave, wave-aggregated adds); each workgroup stores its histogram and the row's last arriver
// sums them in workgroup order, so the result is bit-reproducible (no float atomics in memory).
//   0  stats: online max / sum of exp per workgroup, combined by the last arriver (T == 0: argmax)
//   1-3 nucleus cut (top-p): key where the descending cumulative mass first exceeds p
//       (multinomial rows, p <= 0 or >= 1: 1 = per-chunk mass, 2 = the chunk holding the coin
//        scans its elements in index order)
//   4-6 the draw: same search for coin * nucleus mass among keys >= the cut
//   7  the index: lowest index whose key is the drawn key
// Round 2's first version ran one 1024-thread workgroup per row through 11 passes over the
// vocabulary (607 us for 64 x 128256 logits, flat distribution; profiles/r2_sampler.md).
// ------------------------------------------------------------------------------------------------
static constexpr int kSampleWg = 256;
static constexpr int kSampleBins = 2048;

struct SampleRow {  // per-row state (SampleScratch::state, kSampleStateWords u32)
    float m, invZ, above, nucleus;
    uint32_t prefix, cutKey;
    int mode;     // 0 done, 1 nucleus, 2 multinomial
    int counter;  // last-arriver counter of the current phase (back to 0 after each phase)
    int chunk;    // multinomial: the chunk holding the coin
    float base;   // multinomial: mass of the chunks before it
    int result;
    int pad[5];
};
static_assert(sizeof(SampleRow) == kSampleStateWords * 4, "SampleRow size");

__device__ __forceinline__ uint32_t orderKey(float x) {
    const uint32_t u = __float_as_uint(x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename F>
__device__ __forceinline__ float wgReduce(float v, float *red, F op) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = op(v, __shfl_xor(v, off));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float r = red[0];
#pragma unroll
    for (int w = 1; w < kSampleWg / 64; w++) r = op(r, red[w]);
    __syncthreads();
    return r;
}

// Lanes that share the first active lane's bin are summed and added once (three times), the rest
// add directly: a flat distribution puts nearly every element of the top-digit pass in one bin,
// where per-lane LDS atomics would serialise 64-fold.
__device__ __forceinline__ void histAddWave(float *h, bool act, uint32_t bin, float p) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int rep = 0; rep < 3; rep++) {
        const unsigned long long am = __ballot(act);
        if (am == 0ull) return;
        const int leader = __builtin_ctzll(am);
        const uint32_t b0 = __shfl(bin, leader);
        const bool mine = act && bin == b0;
        float v = mine ? p : 0.f;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        if (lane == leader) atomicAdd(&h[b0], v);
        act = act && !mine;
    }
    if (act) atomicAdd(&h[bin], p);
}

struct SamplePhaseCtx {
    const float *l;
    int V, g, G, c0, c1;
    float T, P, coin;
    SampleRow *st;
    float *gh;    // the row's partial histograms [G][kSampleBins] (every slot rewritten each pass)
    float *part;  // the row's per-chunk values [G]
    int *partI;
};

// Last-arriver handshake. Every cross-workgroup value of a phase is written with agent-scope
// atomics (histogram adds, partial stores) and read back with agent-scope atomic loads, so no
// cache maintenance is needed: each thread waits until its own writes have been performed, then
// one thread counts the workgroup in. (A __threadfence() per thread here - an L2 writeback plus
// invalidate per wave, 4096 per phase at 64 rows - cost ~80 us per phase.)
__device__ __forceinline__ bool lastArrival(SampleRow *st, int G, int *flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        flag[0] = __hip_atomic_fetch_add(&st->counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
    __syncthreads();
    if (!flag[0]) return false;
    if (threadIdx.x == 0) __hip_atomic_store(&st->counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

__device__ __forceinline__ void gstore(float *p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void gstore(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Visit the workgroup's chunk: per round every thread loads kSampleVals elements (coalesced,
// index clamped so the loads are unconditional) before using any, so a phase costs about one
// memory round trip per 8192 elements instead of one per 256 (the first version's loop was
// latency-bound at ~25 us per phase). f(i, value, valid) runs uniformly on every lane.
static constexpr int kSampleVals = 32;
template <typename F>
__device__ __forceinline__ void forChunk(const SamplePhaseCtx &c, F f) {
    for (int r0 = c.c0; r0 < c.c1; r0 += kSampleVals * kSampleWg) {
        float v[kSampleVals];
#pragma unroll
        for (int j = 0; j < kSampleVals; j++) v[j] = c.l[min(r0 + j * kSampleWg + (int)threadIdx.x, c.c1 - 1)];
        __builtin_amdgcn_sched_barrier(0);  // all loads issued before the first use
#pragma unroll
        for (int j = 0; j < kSampleVals; j++) {
            const int i = r0 + j * kSampleWg + (int)threadIdx.x;
            f(i, v[j], i < c.c1);
        }
    }
}

// One radix pass (digit `pass` of 0..2) of a search for `target` among candidates with
// p >= cutoff and key >= minKey whose key matches st->prefix above this digit.
__device__ void sampleRadixPass(const SamplePhaseCtx &c, int pass, bool draw, float *h, float *red, int *flag) {
    const int tid = threadIdx.x;
    const int shift = pass == 0 ? 21 : (pass == 1 ? 10 : 0);
    const uint32_t width = pass == 2 ? 10 : 11, mask = (1u << width) - 1u;
    SampleRow *st = c.st;
    const float invT = 1.0f / c.T, m = st->m, invZ = st->invZ;
    const float cutoff = (1.0f - c.P) / (float)(c.V - 1);
    const uint32_t minKey = draw ? st->cutKey : 0u;
    const uint32_t prefix = pass == 0 ? 0u : st->prefix;
    const int hiShift = shift + (int)width;  // bits above this digit (32 for pass 0)
    float *hw = h + (tid >> 6) * kSampleBins;  // this wave's histogram
    for (int i = tid; i < kSampleBins * (kSampleWg / 64); i += kSampleWg) h[i] = 0.f;
    __syncthreads();
    forChunk(c, [&](int, float lv, bool act) {
        const float x = lv * invT;
        const float p = __expf(x - m) * invZ;
        const uint32_t k = orderKey(x);
        act = act && p >= cutoff && k >= minKey;
        if (hiShift < 32) act = act && (k >> hiShift) == (prefix >> hiShift);
        histAddWave(hw, act, (k >> shift) & mask, p);
    });
    __syncthreads();
    // this workgroup's histogram (the waves' copies summed in wave order) -> its partial slot
    constexpr int PER = kSampleBins / kSampleWg;  // 8 consecutive bins per thread
    float *mine = c.gh + (size_t)c.g * kSampleBins;
#pragma unroll
    for (int j = 0; j < PER; j++) {  // lane-consecutive bins: every store instruction is one 1 KB line run
        const int bin = j * kSampleWg + tid;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < kSampleWg / 64; w++) v += h[w * kSampleBins + bin];
        gstore(&mine[bin], v);
    }
    if (!lastArrival(st, c.G, flag)) return;
    // ---- last arriver: sum the G partial histograms in workgroup order (deterministic) into LDS,
    // then pick the bin where the descending cumulative mass crosses the target
    {
        float acc8[PER];
#pragma unroll
        for (int j = 0; j < PER; j++) acc8[j] = 0.f;
        for (int g0 = 0; g0 < c.G; g0 += 4) {
            float t4[4][PER];
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int j = 0; j < PER; j++)
                    t4[q][j] = __hip_atomic_load(&c.gh[(size_t)min(g0 + q, c.G - 1) * kSampleBins + j * kSampleWg + tid],
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (g0 + q < c.G)
#pragma unroll
                    for (int j = 0; j < PER; j++) acc8[j] += t4[q][j];
        }
#pragma unroll
        for (int j = 0; j < PER; j++) h[j * kSampleWg + tid] = acc8[j];
    }
    __syncthreads();
    float v[PER];
    float tot = 0.f;
#pragma unroll
    for (int j = 0; j < PER; j++) {
        v[j] = h[tid * PER + j];
        tot += v[j];
    }
    // mass of the bins of higher threads (exclusive suffix over threads)
    float inc = tot;  // inclusive suffix within the wave (lanes >= this lane)
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float y = __shfl_down(inc, off);
        if (lane + off < 64) inc += y;
    }
    if (lane == 0) red[wv] = inc;  // wave totals
    __syncthreads();
    float higher = inc - tot;
    for (int w = wv + 1; w < kSampleWg / 64; w++) higher += red[w];
    const float above0 = pass == 0 ? 0.f : st->above;
    const float target = draw ? st->nucleus * c.coin : c.P;
    const float t = target - above0;
    // highest bin b with (mass of bins > b) + v[b] > t
    int sel = -1;
    float selAbove = 0.f, acc = higher;
#pragma unroll
    for (int j = PER - 1; j >= 0; j--) {
        if (sel < 0 && v[j] > 0.f && acc + v[j] > t) {
            sel = tid * PER + j;
            selAbove = acc;
        }
        acc += v[j];
    }
    // lowest non-empty bin, for a target never exceeded (rounding)
    int low = 0x7fffffff;
    float lowAbove = 0.f;
    acc = higher;
#pragma unroll
    for (int j = PER - 1; j >= 0; j--) {
        if (v[j] > 0.f) {
            low = tid * PER + j;
            lowAbove = acc;
        }
        acc += v[j];
    }
    __shared__ int sSel[2];
    __shared__ float sAbove[2];
    if (tid == 0) {
        sSel[0] = -1;
        sSel[1] = 0x7fffffff;
    }
    __syncthreads();
    if (sel >= 0) atomicMax(&sSel[0], sel);
    if (low != 0x7fffffff) atomicMin(&sSel[1], low);
    __syncthreads();
    const int bin = sSel[0] >= 0 ? sSel[0] : sSel[1];
    if (bin != 0x7fffffff && bin / PER == tid) {  // the bin's owner publishes its numbers
        sAbove[0] = sSel[0] >= 0 ? selAbove : lowAbove;
        float bm = 0.f;
#pragma unroll
        for (int j = 0; j < PER; j++)
            if (tid * PER + j == bin) bm = v[j];
        sAbove[1] = bm;
    }
    __syncthreads();
    if (tid == 0 && bin != 0x7fffffff) {
        const float binMass = sAbove[1];
        st->prefix = prefix | ((uint32_t)bin << shift);
        st->above = above0 + sAbove[0];
        if (pass == 2) {
            if (!draw) {
                st->cutKey = st->prefix;
                st->nucleus = st->above + binMass;  // mass of keys >= the cut
            }
        }
    }
}

template <int PHASE>
__global__ __launch_bounds__(kSampleWg) void samplePhaseKernel(SampleArgs a) {
    __shared__ float h[kSampleBins * (kSampleWg / 64)];  // one histogram per wave (32 KB)
    __shared__ float red[kSampleWg / 64 + 2];
    __shared__ int flag[1];
    const int g = blockIdx.x, b = blockIdx.y, G = gridDim.x, tid = threadIdx.x, V = a.vocab;
    SampleRow *st = reinterpret_cast<SampleRow *>(a.scratch.state) + b;
    const float4 sp = a.spec[b];
    SamplePhaseCtx c;
    c.l = a.logits + (size_t)b * V;
    c.V = V;
    c.g = g;
    c.G = G;
    const int C = (V + G - 1) / G;
    c.c0 = min(g * C, V);
    c.c1 = min(c.c0 + C, V);
    c.T = sp.x;
    c.P = sp.y;
    c.coin = sp.z;
    c.st = st;
    c.gh = a.scratch.hist + (size_t)b * G * kSampleBins;
    c.part = a.scratch.part + (size_t)b * G;
    c.partI = a.scratch.partI + (size_t)b * G;
    const bool multinomial = c.P <= 0.f || c.P >= 1.f;

    if constexpr (PHASE == 0) {
        if (c.T < 0.f) {
            if (g == 0 && tid == 0) {
                a.ids[b] = -1;
                st->mode = 0;
            }
            return;
        }
        if (c.T == 0.f) {  // greedy row: lowest index of the maximum
            float bv = -INFINITY;
            int bi = 0x7fffffff;
            forChunk(c, [&](int i, float lv, bool ok) {
                if (ok) argBetter(bv, bi, lv, i);
            });
            const float mv = wgReduce(bv, red, [](float x, float y) { return fmaxf(x, y); });
            if (tid == 0) flag[0] = 0x7fffffff;
            __syncthreads();
            if (bv == mv && bi != 0x7fffffff) atomicMin(&flag[0], bi);
            __syncthreads();
            if (tid == 0) {
                gstore(&c.part[g], mv);
                gstore(&c.partI[g], flag[0]);
            }
            if (!lastArrival(st, G, flag)) return;
            if (tid == 0) {
                float best = -INFINITY;
                int bestI = 0x7fffffff;
                for (int j = 0; j < G; j++) {
                    const float pv = __hip_atomic_load(&c.part[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const int pi = __hip_atomic_load(&c.partI[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (pi != 0x7fffffff) argBetter(best, bestI, pv, pi);
                }
                a.ids[b] = bestI == 0x7fffffff ? 0 : bestI;
                st->mode = 0;
            }
            return;
        }
        // online max / sum of exp(x - max) over the chunk
        const float invT = 1.0f / c.T;
        float mx = -INFINITY, sm = 0.f;
        forChunk(c, [&](int, float lv, bool ok) {
            const float x = lv * invT;
            if (!ok) return;
            if (x > mx) {
                sm = sm * __expf(mx - x) + 1.f;
                mx = x;
            } else {
                sm += __expf(x - mx);
            }
        });
        const float M = wgReduce(mx, red, [](float x, float y) { return fmaxf(x, y); });
        const float S = wgReduce(mx == -INFINITY ? 0.f : sm * __expf(mx - M), red, [](float x, float y) { return x + y; });
        if (tid == 0) {
            gstore(&c.part[g], M);
            gstore(&c.partI[g], __float_as_int(S));
        }
        if (!lastArrival(st, G, flag)) return;
        if (tid == 0) {
            float gm = -INFINITY;
            for (int j = 0; j < G; j++) gm = fmaxf(gm, __hip_atomic_load(&c.part[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            float z = 0.f;
            for (int j = 0; j < G; j++) {
                const float pm = __hip_atomic_load(&c.part[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const float ps = __int_as_float(__hip_atomic_load(&c.partI[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (pm != -INFINITY) z += ps * __expf(pm - gm);
            }
            st->m = gm;
            st->invZ = 1.0f / z;
            st->mode = multinomial ? 2 : 1;
            st->result = 0x7fffffff;
        }
        return;
    } else {
        if (st->mode == 0) return;
        if (st->mode == 2) {  // multinomial in index order
            const float invT = 1.0f / c.T, m = st->m, invZ = st->invZ;
            if constexpr (PHASE == 1) {
                float s = 0.f;
                forChunk(c, [&](int, float lv, bool ok) {
                    if (ok) s += __expf(lv * invT - m) * invZ;
                });
                s = wgReduce(s, red, [](float x, float y) { return x + y; });
                if (tid == 0) gstore(&c.part[g], s);
                if (!lastArrival(st, G, flag)) return;
                if (tid == 0) {
                    float base = 0.f;
                    int ch = -1;
                    for (int j = 0; j < G; j++) {
                        const float pj = __hip_atomic_load(&c.part[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (ch < 0 && c.coin >= base && c.coin < base + pj) {
                            ch = j;
                            break;
                        }
                        base += pj;
                    }
                    st->chunk = ch;
                    st->base = base;
                    if (ch < 0) {  // the coin fell past the total mass (rounding): last token
                        a.ids[b] = V - 1;
                        st->mode = 0;
                    }
                }
            } else if constexpr (PHASE == 2) {
                if (g != st->chunk) return;
                // thread t owns a contiguous sub-range of the chunk (index order)
                const int n = c.c1 - c.c0, per = (n + kSampleWg - 1) / kSampleWg;
                const int i0 = c.c0 + min(tid * per, n), i1 = c.c0 + min(tid * per + per, n);
                // the thread's run, loaded at once (per <= kSampleVals for the chunk sizes used)
                float pv[kSampleVals];
                float s = 0.f;
#pragma unroll
                for (int k = 0; k < kSampleVals; k++) pv[k] = c.l[min(i0 + k, c.c1 - 1)];
#pragma unroll
                for (int k = 0; k < kSampleVals; k++) {
                    pv[k] = __expf(pv[k] * invT - m) * invZ;
                    if (i0 + k < i1) s += pv[k];
                }
                if (per > kSampleVals)  // large chunks (few rows, small G): the rest one by one
                    for (int i = i0 + kSampleVals; i < i1; i++) s += __expf(c.l[i] * invT - m) * invZ;
                float inc = s;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const float y = __shfl_up(inc, off);
                    if ((tid & 63) >= off) inc += y;
                }
                if ((tid & 63) == 63) red[tid >> 6] = inc;
                if (tid == 0) flag[0] = c.c1 - 1;
                __syncthreads();
                float base = st->base + inc - s;
                for (int w = 0; w < (tid >> 6); w++) base += red[w];
                if (i1 > i0 && c.coin >= base && c.coin < base + s) {
                    float cdf = base;
                    int pick = -1;
#pragma unroll
                    for (int k = 0; k < kSampleVals; k++)
                        if (pick < 0 && i0 + k < i1) {
                            cdf += pv[k];
                            if (c.coin < cdf) pick = i0 + k;
                        }
                    for (int i = i0 + kSampleVals; pick < 0 && i < i1; i++) {
                        cdf += __expf(c.l[i] * invT - m) * invZ;
                        if (c.coin < cdf) pick = i;
                    }
                    atomicMin(&flag[0], pick < 0 ? i1 - 1 : pick);
                }
                __syncthreads();
                if (tid == 0) {
                    a.ids[b] = flag[0];
                    st->mode = 0;
                }
            }
            return;
        }
        // nucleus rows
        if constexpr (PHASE >= 1 && PHASE <= 6) {
            sampleRadixPass(c, (PHASE - 1) % 3, PHASE >= 4, h, red, flag);
        } else if constexpr (PHASE == 7) {
            const float invT = 1.0f / c.T;
            const uint32_t key = st->prefix;
            if (tid == 0) flag[0] = 0x7fffffff;
            __syncthreads();
            int mine = 0x7fffffff;
            forChunk(c, [&](int i, float lv, bool ok) {
                if (ok && orderKey(lv * invT) == key) mine = min(mine, i);
            });
            if (mine != 0x7fffffff) atomicMin(&flag[0], mine);
            __syncthreads();
            if (tid == 0 && flag[0] != 0x7fffffff) atomicMin(&st->result, flag[0]);
            if (!lastArrival(st, G, flag)) return;
            if (tid == 0) {
                const int r = __hip_atomic_load(&st->result, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                a.ids[b] = r == 0x7fffffff ? 0 : r;
                st->mode = 0;
            }
        }
    }
}

int sampleGroups(int B) {
    int G = 1024 / (B > 0 ? B : 1);
    return G < 8 ? 8 : (G > kSampleMaxGroups ? kSampleMaxGroups : G);
}

void launchSample(const SampleArgs &a, int B, hipStream_t s) {
    const dim3 grid(sampleGroups(B), B);
    hipLaunchKernelGGL(samplePhaseKernel<0>, grid, dim3(kSampleWg), 0, s, a);
    hipLaunchKernelGGL(samplePhaseKernel<1>, grid, dim3(kSampleWg), 0, s, a);
    hipLaunchKernelGGL(samplePhaseKernel<2>, grid, dim3(kSampleWg), 0, s, a);
    hipLaunchKernelGGL(samplePhaseKernel<3>, grid, dim3(kSampleWg), 0, s, a);
    hipLaunchKernelGGL(samplePhaseKernel<4>, grid, dim3(kSampleWg), 0, s, a);
    hipLaunchKernelGGL(samplePhaseKernel<5>, grid, dim3(kSampleWg), 0, s, a);
    hipLaunchKernelGGL(samplePhaseKernel<6>, grid, dim3(kSampleWg), 0, s, a);
    hipLaunchKernelGGL(samplePhaseKernel<7>, grid, dim3(kSampleWg), 0, s, a);
}

// In-place Q80 round trip of f32 values (32-element blocks, rintf like every Q80 producer here).
__global__ void q80RoundtripKernel(float *x, size_t n) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;  // n % 32 == 0: whole groups
    const float v = i < n ? x[i] : 0.f;
    const float amax = groupMax<32>(fabsf(v));
    const float d = amax / 127.0f;
    const float id = d != 0.f ? 1.0f / d : 0.f;
    int q = (int)rintf(v * id);
    q = q > 127 ? 127 : (q < -127 ? -127 : q);
    if (i < n) x[i] = (float)q * __half2float(__float2half(d));
}

void launchQ80Roundtrip(float *x, size_t n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(q80RoundtripKernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n);
}

__global__ void unshardKernel(const float *in, float *out, int nRanks, int B, int vocab0) {
    const size_t total = (size_t)nRanks * B * vocab0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int v = (int)(i % vocab0);
        const size_t rb = i / vocab0;
        const int b = (int)(rb % B), r = (int)(rb / B);
        out[((size_t)b * nRanks + r) * vocab0 + v] = in[i];
    }
}

void launchUnshardLogits(const float *in, float *out, int nRanks, int B, int vocab0, hipStream_t s) {
    hipLaunchKernelGGL(unshardKernel, dim3(1024), dim3(256), 0, s, in, out, nRanks, B, vocab0);
}

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void fillQ40Kernel(uint8_t *qs, uint16_t *d, size_t nBlocks, float scale, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nBlocks; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t r0 = splitmix(seed ^ (i * 3 + 0)), r1 = splitmix(seed ^ (i * 3 + 1));
        uint4 v;
        v.x = (uint32_t)r0;
        v.y = (uint32_t)(r0 >> 32);
        v.z = (uint32_t)r1;
        v.w = (uint32_t)(r1 >> 32);
        reinterpret_cast<uint4 *>(qs)[i] = v;
        const uint64_t r2 = splitmix(seed ^ (i * 3 + 2));
        const float u = (float)(r2 >> 40) / 16777216.0f;
        d[i] = __half_as_ushort(__float2half(scale * (0.5f + u)));
    }
}

void launchFillQ40(uint8_t *qs, uint16_t *d, size_t nBlocks, float scale, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL(fillQ40Kernel, dim3(4096), dim3(256), 0, s, qs, d, nBlocks, scale, seed);
}

__global__ void fillF32Kernel(float *p, size_t n, float amp, uint64_t seed) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float u = (float)(splitmix(seed ^ i) >> 40) / 16777216.0f;
        p[i] = amp * (2.0f * u - 1.0f);
    }
}

void launchFillF32Uniform(float *p, size_t n, float amp, uint64_t seed, hipStream_t s) {
    hipLaunchKernelGGL(fillF32Kernel, dim3(4096), dim3(256), 0, s, p, n, amp, seed);
}

__global__ void fillConstKernel(float *p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

void launchFillF32Const(float *p, size_t n, float v, hipStream_t s) {
    hipLaunchKernelGGL(fillConstKernel, dim3(1024), dim3(256), 0, s, p, n, v);
}

}  // namespace hipk
}  // namespace dl
