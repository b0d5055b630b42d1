// Device-side building blocks of the decode path (gfx950), part 1: LDS layout of the GEMVs, the
// residual + RMS norm prologue, the Q40 block dot product, the fused epilogues (SwiGLU, RoPE + KV
// append, Q80 hand-offs), the write-through accessors and the fused tensor-parallel exchange.
// Included through decode_dev.h (with gemv_dev.h: the ring GEMV body, attn_dev.h: the decode
// attention task).
#pragma once

#include "../core/common.h"
#include "device_common.h"
#include "kernels.h"

#include <type_traits>

namespace dl {
namespace hipk {

using namespace dl::dev;

// Dynamic LDS above 64 KB (up to the CU's 160 KB) has to be opted into per kernel.
static inline void allowLds(const void *fn, size_t bytes) {
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

static constexpr int kThreads = 256;
static constexpr int kMaxHeadSize = 128;  // RoPE rows staged in LDS by the QKV epilogue
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

__host__ __device__ static inline size_t alignUp(size_t x, size_t a) { return (x + a - 1) / a * a; }

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
    l.res = off;  // TP partial rows
    off = alignUp(off + (size_t)2 * B * rowsPerWg * sizeof(float), 16);
    l.hbuf = off;
    off = alignUp(off + (size_t)B * (rowsPerWg / 2) * sizeof(float), 16);
    l.act = off;
    if (pro != PRO_GLOBAL || q40) {
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

// Write-through (agent-scope, sc1) stores / loads for data handed to other workgroups INSIDE one
// launch (cdna_hip_programming.md Guideline 16: L2s are per XCD and not coherent, so a plain store
// may sit in the writer's L2 and a plain load may hit a stale line): the producer's stores are
// performed at the coherence point, the consumer's loads bypass its caches. WT = false: plain.
template <bool WT>
__device__ __forceinline__ void st32(void *p, uint32_t v) {
    if constexpr (WT) __hip_atomic_store(reinterpret_cast<uint32_t *>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *reinterpret_cast<uint32_t *>(p) = v;
}
template <bool WT>
__device__ __forceinline__ void st64(void *p, uint64_t v) {
    if constexpr (WT) __hip_atomic_store(reinterpret_cast<uint64_t *>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *reinterpret_cast<uint64_t *>(p) = v;
}
template <bool WT>
__device__ __forceinline__ void stF2(float *p, float a, float b) {
    st64<WT>(p, (uint64_t)__float_as_uint(a) | ((uint64_t)__float_as_uint(b) << 32));
}
__device__ __forceinline__ uint32_t ldWT32(const void *p) {
    return __hip_atomic_load(reinterpret_cast<const uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ldWT64(const void *p) {
    return __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Rows [0, q0) are Q, [q0, q0+kv0) K, then V. Q and K pairs are rotated (RoPE at this row's
// position); K and V are appended to the KV cache at [slot][pos]. WT: write-through (the fused
// attention block's attention workgroups read them in the same launch).
template <bool WT = false>
__device__ __forceinline__ void qkvPairStore(const GemvArgs &a, int r0, float v0, float v1, const float2 *ropeRow,
                                             int p, int sl, float *qRow) {
    if (r0 < a.q0 + a.kv0) {
        const float2 cs = ropeRow[(r0 % a.hs) >> 1];
        const float o0 = v0 * cs.x - v1 * cs.y;
        const float o1 = v0 * cs.y + v1 * cs.x;
        if (r0 < a.q0) {
            stF2<WT>(qRow + r0, o0, o1);
        } else {
            const int x = r0 - a.q0;  // K row: head x / hs, dim x % hs (a row pair stays in one head)
            const int lg = __builtin_ctz(a.hs);  // hs is a power of two (64 / 128)
            const size_t off = kvOff(a.kvMap, a.seqLen, a.kv0 >> lg, a.hs, sl, p, x >> lg) + (x & (a.hs - 1));
            if (a.kvBf16) {
                const uint32_t pk = (uint32_t)f32ToBf16(o0) | ((uint32_t)f32ToBf16(o1) << 16);
                st32<WT>(reinterpret_cast<uint16_t *>(a.kcache) + off, pk);
            } else {
                stF2<WT>(reinterpret_cast<float *>(a.kcache) + off, o0, o1);
            }
        }
    } else {
        const int x = r0 - a.q0 - a.kv0, lg = __builtin_ctz(a.hs);
        const size_t off = kvOff(a.kvMap, a.seqLen, a.kv0 >> lg, a.hs, sl, p, x >> lg) + (x & (a.hs - 1));
        if (a.kvBf16) {
            const uint32_t pk = (uint32_t)f32ToBf16(v0) | ((uint32_t)f32ToBf16(v1) << 16);
            st32<WT>(reinterpret_cast<uint16_t *>(a.vcache) + off, pk);
        } else {
            stF2<WT>(reinterpret_cast<float *>(a.vcache) + off, v0, v1);
        }
    }
}

// Quantize a workgroup's `halfR` hidden units (multiple of 32, in LDS) to Q80 blocks in global.
// WT: the hidden rows are consumed in this launch (fused FFN block): 4 lanes' bytes packed into one
// write-through 32-bit store, the scale pair one write-through 64-bit store.
template <int B, bool WT = false>
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
        int8_t *dst = a.oq + (size_t)b * a.ldOut + hBase + k;
        if constexpr (WT) {
            const uint32_t u = (uint32_t)(uint8_t)q;
            const uint32_t w = u | ((uint32_t)__shfl_down((int)u, 1, 32) << 8) |
                               ((uint32_t)__shfl_down((int)u, 2, 32) << 16) | ((uint32_t)__shfl_down((int)u, 3, 32) << 24);
            if ((k & 3) == 0) st32<true>(dst, w);
        } else {
            *dst = (int8_t)q;
        }
        const float qs = groupSum<32>((float)q);
        if ((k & 31) == 0) stF2<WT>(reinterpret_cast<float *>(a.os + (size_t)b * (a.ldOut >> 5) + ((hBase + k) >> 5)),
                                    roundF16(d), qs);
    }
}

// Copy B rows of Q80 activations (n int8 + n/32 scale pairs) from global into the LDS image.
// WT: the rows were produced in this launch (write-through loads).
template <int B, bool WT = false>
__device__ __forceinline__ void stageQ80(const GemvArgs &a, int8_t *sq, float2 *ssc) {
    const int n = a.n, nb = n >> 5;
#pragma unroll
    for (int b = 0; b < B; b++) {
        if constexpr (WT) {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(a.aq + (size_t)b * n);
            uint32_t *dst = reinterpret_cast<uint32_t *>(sq + (size_t)b * n);
            for (int i = threadIdx.x; i < (n >> 2); i += kThreads) dst[i] = ldWT32(src + i);
            const uint64_t *ss = reinterpret_cast<const uint64_t *>(a.as + (size_t)b * nb);
            for (int i = threadIdx.x; i < nb; i += kThreads) reinterpret_cast<uint64_t *>(ssc)[b * nb + i] = ldWT64(ss + i);
        } else {
            const int4 *src = reinterpret_cast<const int4 *>(a.aq + (size_t)b * n);
            int4 *dst = reinterpret_cast<int4 *>(sq + (size_t)b * n);
            for (int i = threadIdx.x; i < (n >> 4); i += kThreads) dst[i] = src[i];
            for (int i = threadIdx.x; i < nb; i += kThreads) ssc[b * nb + i] = a.as[(size_t)b * nb + i];
        }
    }
    __syncthreads();
}

// B rows of f32 activations produced in this launch (write-through loads) quantized into the LDS
// Q80 image: the fused FFN block's w2 role when w13 hands the hidden rows off in f32. Same values
// as resNormPrologue without a norm (n % 32 == 0: the quads of a block stay together).
template <int B>
__device__ __forceinline__ void stageF32WT(const GemvArgs &a, int8_t *sq, float2 *ssc) {
    const int n = a.n, nChunks = n >> 3;
#pragma unroll
    for (int b = 0; b < B; b++) {
        const float *xi = a.in + (size_t)b * a.ldIn;
        for (int c = threadIdx.x; c < nChunks; c += kThreads) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                const uint64_t u = ldWT64(xi + c * 8 + i);
                v[i] = __uint_as_float((uint32_t)u);
                v[i + 1] = __uint_as_float((uint32_t)(u >> 32));
            }
            stageChunk<true>(v, b, c, n, sq, ssc, nullptr);
        }
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------------
// Fused tensor-parallel exchange (TpXchg, kernels.h). Peer words are 8-byte {payload, epoch}
// granules in uncached memory: one relaxed system-scope store publishes data and flag together,
// a relaxed system-scope load polls them (cdna_hip_programming.md Guideline 16 "R2": the data is
// the flag, no fence needed); a wait gives up after tp.timeoutTicks and raises tp.error.
// Every user keeps ONE epoch per exchange word (epochs[w] = the last epoch word w carried): every
// write of a word then carries a larger epoch than any earlier write of it, whichever user (f32 or
// Q80 rows, argmax winners, the self-test) or engine on the same comm wrote it, so a stale word
// can never pass for a fresh one.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t tpLoad(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool tpFailed(const TpXchg &x) {
    return __hip_atomic_load(x.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

// Push `payload` as exchange word `w` (epoch e) to every peer, then collect word `w` of every rank
// into vals[p] (this rank's own payload included). Peer loads are all issued before any wait.
// WM: compile-time bound on the ranks (x.world <= WM; tpDispatch picks it once per exchange): the
// rank loops are unrolled WM times, so a TP2 exchange is not compiled as 16 predicated ranks (the
// 16-way form measured ~1.1-2.3 us of scalar selects and spilled SGPRs per workgroup tail).
template <int WM>
__device__ __forceinline__ void tpPushCollect(const TpXchg &x, long long w, unsigned e, unsigned payload,
                                              unsigned (&vals)[WM], unsigned &waited) {
    const int me = x.rank, W = x.world;
    if (x.loopback) {
#pragma unroll
        for (int p = 0; p < WM; p++) vals[p] = p == me ? payload : 0u;
        return;
    }
    const long long par = e & 1;
    const uint64_t word = (uint64_t)payload | ((uint64_t)e << 32);
#pragma unroll
    for (int p = 0; p < WM; p++)
        if (p < W && p != me)
            __hip_atomic_store(x.recv[p] + (par * W + me) * x.stride + w, word, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    // this rank's region picked with compile-time indices: a runtime index into the kernel
    // argument's pointer array made the fused attention block copy its whole 1.2 KB argument
    // struct to scratch at entry (the memcpy of a by-value kernel argument that SROA cannot undo)
    const uint64_t *mine = nullptr;
#pragma unroll
    for (int p = 0; p < WM; p++)
        if (p == me) mine = x.recv[p];
    mine += par * W * x.stride + w;
    uint64_t got[WM];
#pragma unroll
    for (int p = 0; p < WM; p++) got[p] = (p < W && p != me) ? tpLoad(mine + p * x.stride) : word;
#pragma unroll
    for (int p = 0; p < WM; p++) {
        if (p < W) {
            uint64_t v = got[p];
            // the error word is read only when a wait is due (an earlier timeout: do not wait)
            if ((unsigned)(v >> 32) != e && !tpFailed(x)) {
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                while ((unsigned)(v >> 32) != e) {
                    __builtin_amdgcn_s_sleep(1);
                    v = tpLoad(mine + p * x.stride);
                    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > x.timeoutTicks) {
                        __hip_atomic_store(x.error, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // 3: fused exchange
                        break;
                    }
                }
                waited += (unsigned)((long long)__builtin_amdgcn_s_memrealtime() - t0);
            }
            vals[p] = (unsigned)v;
        }
    }
}

template <int WM>
__device__ __forceinline__ void tpPushCollect(const TpXchg &x, long long w, unsigned e, unsigned payload,
                                              unsigned (&vals)[WM]) {
    unsigned waited = 0;
    tpPushCollect<WM>(x, w, e, payload, vals, waited);
}

// Calls f(std::integral_constant<int, WM>) with the smallest rank bound WM in {2, 4, 8, 16} >= world.
template <typename F>
__device__ __forceinline__ void tpDispatch(int world, F &&f) {
    if (world <= 2) f(std::integral_constant<int, 2>{});
    else if (world <= 4) f(std::integral_constant<int, 4>{});
    else if (world <= 8) f(std::integral_constant<int, 8>{});
    else f(std::integral_constant<int, 16>{});
}

// Measured sync (ForwardStats::syncMs): the time a wave spends waiting for peers' words, read from
// s_memrealtime (10 ns ticks) only inside the wait loop - an exchange that finds every word
// already there costs nothing (a stamp at every exchange's start stalled the tail's next LDS
// access on the RTC read: ~4 % of a TP8 rank's decode). Per exchange the longest wave's wait is
// raised into x.ticks (one no-return atomic per wave that waited). Wave-uniform control flow.
__device__ __forceinline__ void tpWaitReport(const TpXchg &x, unsigned waited) {
    if (!x.ticks || __ballot(waited != 0u) == 0ull) return;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned o = (unsigned)__shfl_xor((int)waited, off);
        waited = o > waited ? o : waited;
    }
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_max(x.ticks, waited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The same from a single thread (argmax winners).
__device__ __forceinline__ void tpWaitReportThread(const TpXchg &x, unsigned waited) {
    if (x.ticks && waited) __hip_atomic_fetch_max(x.ticks, waited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Argmax reductions (value, index): larger value wins, ties -> lower index (a full-vocabulary
// argmax's pick). blockArgmax leaves the workgroup's winner in thread 0 (sv / si: NW scratch words).
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

// Tensor-parallel argmax: every rank offers its slice's winner (value, global index) in the
// argmax-winners exchange region (words 2b, 2b + 1); all ranks pick the same one in rank order.
// Thread 0 only.
template <int WM>
__device__ __forceinline__ void tpArgmaxPick(const TpXchg &x, int b, float &bv, int &bi) {
    // compute-only rank (loopback): no peer offers anything, this shard's winner stands (peers read
    // as zeros would otherwise offer value 0 at index 0 and win over a negative local maximum)
    if (x.loopback) return;
    const unsigned long long xs = x.span ? wall_clock64() : 0ull;
    unsigned waited = 0;
    const unsigned ev = x.epochs[2 * b] + 1, ei = x.epochs[2 * b + 1] + 1;  // one epoch per word
    unsigned vv[WM], vi[WM];
    tpPushCollect(x, 2LL * b, ev, __float_as_uint(bv), vv, waited);
    tpPushCollect(x, 2LL * b + 1, ei, (unsigned)bi, vi, waited);
    bv = -INFINITY;
    bi = 0x7fffffff;
#pragma unroll
    for (int p = 0; p < WM; p++)
        if (p < x.world) argBetter(bv, bi, __uint_as_float(vv[p]), (int)vi[p]);
    x.epochs[2 * b] = ev;
    x.epochs[2 * b + 1] = ei;
    tpWaitReportThread(x, waited);
    if (x.span)
        __hip_atomic_fetch_max(x.span, (unsigned)(wall_clock64() - xs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS bytes of the Q80 exchange staging for nEl elements over W ranks.
__host__ __device__ static inline size_t tpQ80Lds(int nEl, int W) {
    return alignUp((size_t)nEl, 16) + alignUp((size_t)nEl / 32 * 4, 16) + (size_t)W * (nEl / 32) * 9 * 4;
}

// f32 exchange of a workgroup's partial rows res[B][R] (rows rowBase..) -> a.out summed over ranks.
// Exchange words of a workgroup's partial rows, k-th of this thread (k = 0, 1, ...): f32 words are
// the elements b * ldOut + row, Q80 words 9 per 32-row block. Returns -1 for a dead word.
__device__ __forceinline__ long long tpWordOf(const GemvArgs &a, int R, int rowBase, int j, bool q80) {
    const int i = q80 ? (j / 9) * 32 : j;
    const int b = i / R, row = rowBase + i % R;
    if (row >= a.rows) return -1;
    const long long el = (long long)b * a.ldOut + row;
    return q80 ? (el >> 5) * 9 + j % 9 : el;
}

// Exchange epochs are read with plain (compiler-visible) loads in the tail. An inline-asm prefetch
// at kernel entry (round 5) saved nothing measurable and let the compiler copy the pending
// registers before their s_waitcnt (an asm operand moved to other VGPRs: v_mov of a register whose
// load was still in flight, ISA of gemvQ40Kernel<.., EPI_STORE_TP>), i.e. a stale-epoch hazard.
// TO_LDS (EPI_RESQ_TP): the rank-summed rows replace the partials in res[] (the tail continues
// from LDS) instead of going to a.out.
template <int B, int WM, bool TO_LDS = false>
__device__ __forceinline__ void tpExchangeF32(const GemvArgs &a, float *res, int R, int rowBase) {
    const TpXchg &x = a.tp;
    unsigned waited = 0;
    for (int i = threadIdx.x; i < B * R; i += kThreads) {
        const int b = B == 1 ? 0 : i / R, row = rowBase + (B == 1 ? i : i % R);
        if (row >= a.rows) continue;
        const long long el = (long long)b * a.ldOut + row;
        const unsigned e = x.epochs[el] + 1;
        unsigned v[WM];
        tpPushCollect(x, el, e, __float_as_uint(res[i]), v, waited);
        float s = 0.f;
#pragma unroll
        for (int p = 0; p < WM; p++)
            if (p < x.world) s += __uint_as_float(v[p]);
        if constexpr (TO_LDS) res[i] = s;
        else a.out[el] = s;
        x.epochs[el] = e;
    }
    tpWaitReport(x, waited);
}

// Q80 exchange (the reference's ZQ pipe: every rank's partial quantized once to Q80 blocks of 32
// rows, all ranks' blocks dequantized and summed in rank order, own included). R and rowBase are
// multiples of 32. A block travels as 9 words: 8 x 4 int8 + the f16 scale. `lds` = free staging.
// Q80 exchange of one row's partials (B = 1), wave-local: 32-row block g is quantized by the
// 32-lane group of threads 32g..32g+31 (lane l = row rowBase + 32g + l), lanes 0-8 push / collect
// the block's 9 words (8 x 4 int8 + the f16 scale), and every lane sums its row over the ranks
// from those words by shuffles: no LDS staging and no barrier (the LDS form spent ~1.6 us per
// workgroup tail, profiles/r5_tp_rank.md). Same rounding and rank order as tpExchangeQ80.
template <int WM, bool TO_LDS = false>
__device__ __forceinline__ void tpExchangeQ80Row(const GemvArgs &a, float *res, int R, int rowBase) {
    const TpXchg &x = a.tp;
    const int nBlk = R >> 5, W = x.world;
    unsigned waited = 0;
    const int l = threadIdx.x & 31;
    for (int base = 0; base < nBlk * 32; base += kThreads) {  // uniform per 32-lane group
        const int i = base + threadIdx.x, blk = i >> 5, row = rowBase + i;
        const bool blkLive = blk < nBlk && rowBase + blk * 32 < a.rows;
        const float v = blk < nBlk ? res[i] : 0.f;
        const float amax = groupMax<32>(fabsf(v));
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        int q = (int)rintf(v * id);
        q = q > 127 ? 127 : (q < -127 ? -127 : q);
        const unsigned d16 = __half_as_ushort(__float2half(d));
        // lane w < 8 packs the bytes of rows 4w .. 4w + 3; lane 8 carries the scale
        const unsigned b0 = (unsigned)__shfl(q, 4 * (l & 7), 32) & 0xFFu, b1 = (unsigned)__shfl(q, 4 * (l & 7) + 1, 32) & 0xFFu;
        const unsigned b2 = (unsigned)__shfl(q, 4 * (l & 7) + 2, 32) & 0xFFu, b3 = (unsigned)__shfl(q, 4 * (l & 7) + 3, 32) & 0xFFu;
        const unsigned payload = l < 8 ? (b0 | (b1 << 8) | (b2 << 16) | (b3 << 24)) : d16;
        unsigned vals[WM];
#pragma unroll
        for (int p = 0; p < WM; p++) vals[p] = 0u;
        if (blkLive && l < 9) {
            const long long wd = (long long)((rowBase >> 5) + blk) * 9 + l;
            const unsigned e = x.epochs[wd] + 1;
            tpPushCollect<WM>(x, wd, e, payload, vals, waited);
            x.epochs[wd] = e;
        }
        float sum = 0.f;
#pragma unroll
        for (int p = 0; p < WM; p++) {
            if (p < W) {
                const unsigned wq = (unsigned)__shfl((int)vals[p], l >> 2, 32);
                const unsigned ds = (unsigned)__shfl((int)vals[p], 8, 32);
                const int qq = (int)(int8_t)(wq >> (8 * (l & 3)));
                sum += (float)qq * __half2float(__ushort_as_half((uint16_t)(ds & 0xFFFFu)));
            }
        }
        if constexpr (TO_LDS) {
            if (blk < nBlk) res[i] = sum;  // this lane read res[i] above: no other lane touches it
        } else if (blkLive && row < a.rows) {
            a.out[row] = sum;
        }
    }
    tpWaitReport(x, waited);
}

template <int B, int WM>
__device__ __forceinline__ void tpExchangeQ80(const GemvArgs &a, const float *res, int R, int rowBase, char *lds) {
    const TpXchg &x = a.tp;
    const int nEl = B * R, nBlk = nEl >> 5, W = x.world;
    int8_t *q8 = reinterpret_cast<int8_t *>(lds);
    uint32_t *dq = reinterpret_cast<uint32_t *>(lds + alignUp((size_t)nEl, 16));
    uint32_t *rv = reinterpret_cast<uint32_t *>(lds + alignUp((size_t)nEl, 16) + alignUp((size_t)nBlk * 4, 16));
    unsigned waited = 0;
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
        const int b = B == 1 ? 0 : (blk * 32) / R, row = rowBase + (B == 1 ? blk * 32 : (blk * 32) % R);
        live = row < a.rows;
        return ((long long)b * a.ldOut + row) >> 5;
    };
    // 2. push / collect the 9 words of every block
    for (int j = threadIdx.x; j < nBlk * 9; j += kThreads) {
        const int blk = j / 9, w = j % 9;
        bool live;
        const long long gb = blockId(blk, live);
        if (!live) continue;
        const long long wd = gb * 9 + w;
        const unsigned e = x.epochs[wd] + 1;
        const unsigned payload = w < 8 ? reinterpret_cast<const uint32_t *>(q8)[blk * 8 + w] : dq[blk];
        unsigned v[WM];
        tpPushCollect(x, wd, e, payload, v, waited);
#pragma unroll
        for (int p = 0; p < WM; p++)
            if (p < W) rv[(p * nBlk + blk) * 9 + w] = v[p];
        x.epochs[wd] = e;
    }
    tpWaitReport(x, waited);
    __syncthreads();
    // 3. dequantize and sum in rank order
    for (int i = threadIdx.x; i < nEl; i += kThreads) {
        const int b = B == 1 ? 0 : i / R, row = rowBase + (B == 1 ? i : i % R), blk = i >> 5;
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
}

// EPI_RESQ_TP tail (one row; R a multiple of 32, rowBase too): res[i] holds the rank-summed delta
// of row rowBase + i. x' = resIn + delta -> resOut; x' * resW quantized to Q80 blocks (d' =
// amax / 127 unrounded: the consumer folds in 1 / rms and rounds) -> xq / xs; the workgroup's
// sum of x'^2 -> ssp[blk]. Uniform loop over whole 32-lane groups (one block each).
// resqPrefetch: this thread's residual and norm weight (R <= 256: one row per thread), loaded
// before the exchange so their round trip overlaps the peers' wait instead of following it.
struct ResqPre {
    float x = 0.f, w = 0.f;
};
__device__ __forceinline__ ResqPre resqPrefetch(const GemvArgs &a, int R, int rowBase) {
    ResqPre p;
    const int row = rowBase + (int)threadIdx.x;
    if ((int)threadIdx.x < R && row < a.rows) {
        p.x = a.rq.resIn[row];
        p.w = a.rq.resW[row];
    }
    return p;
}
__device__ __forceinline__ void resqTail(const GemvArgs &a, const float *res, int R, int rowBase, int blk,
                                         float *scratch, ResqPre pf) {
    const PrenormOut &o = a.rq;
    float ss = 0.f;
    for (int base = 0; base < R; base += kThreads) {
        const int i = base + threadIdx.x, row = rowBase + i;
        const bool live = i < R && row < a.rows;  // a.rows % 32 == 0: whole blocks live or dead
        float g = 0.f;
        if (live) {
            const bool pre1 = R <= kThreads;  // prefetched (one row per thread)
            const float xn = (pre1 ? pf.x : o.resIn[row]) + res[i];
            o.resOut[row] = xn;
            g = xn * (pre1 ? pf.w : o.resW[row]);
            ss += xn * xn;
        }
        const float amax = groupMax<32>(fabsf(g));
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        int q = (int)rintf(g * id);
        q = q > 127 ? 127 : (q < -127 ? -127 : q);
        const float qs = groupSum<32>((float)q);
        if (live) o.xq[row] = (int8_t)q;
        if (live && (i & 31) == 0) o.xs[row >> 5] = make_float2(d, qs);
    }
    if (R <= 64) {  // every row in wave 0: a wave reduction, no workgroup barrier
        if (threadIdx.x < 64) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) ss += __shfl_xor(ss, off);
            if (threadIdx.x == 0) o.ssp[blk] = ss;
        }
        return;
    }
    ss = blockSum<kThreads>(ss, scratch);
    if (threadIdx.x == 0) o.ssp[blk] = ss;
}

// Longest context (max position + 1) over rows [b0, b0 + n) below nRows, n <= 64: one load per
// lane and a wave max, the same value in every wave. (A loop of dependent per-row loads put ~16
// serial memory round trips at the start of every prefill-attention workgroup.)
__device__ __forceinline__ int rowsMaxLen(const int *pos, int b0, int n, int nRows) {
    const int lane = threadIdx.x & 63;
    int v = (lane < n && b0 + lane < nRows) ? pos[b0 + lane] + 1 : 0;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = max(v, __shfl_xor(v, off));
    return v;
}

// Sequence split of a decode-attention row of length `len`: nSplit chunks of ch positions
// (~256 per chunk, at most splitGrid chunks). Shorter chunks for the few heads of a TP8 shard
// (4 per rank) measured slower: 5.4 -> 7.6 us at 100 positions (profiles/r5_tp_rank.md).
__device__ __forceinline__ void attnSplit(int len, int splitGrid, int &nSplit, int &ch, int chunkMin = 256,
                                          int shortLen = 0) {
    // single decode rows (shortLen set) of <= shortLen keys split at 128 keys: one 256-thread task
    // walks 112-128 keys per memory round trip, so 129..256 keys in one chunk cost a second
    // dependent round trip per layer (decode at 164-204: 1.39-1.44 vs 1.35-1.37 ms/token,
    // r6_decode.md). Batched launches keep 256 (their grid would double for it).
    if (chunkMin >= 256 && len <= shortLen) chunkMin = kAttnShortChunk;
    int ns = (len + chunkMin - 1) / chunkMin;
    if (ns > splitGrid) ns = splitGrid;
    if (ns < 1) ns = 1;
    ch = (((len + ns - 1) / ns) + 15) & ~15;
    nSplit = (len + ch - 1) / ch;
}

}  // namespace hipk
}  // namespace dl
