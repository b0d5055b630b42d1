// Device-side building blocks of the decode path (gfx950), shared by the standalone kernels
// (kernels.hip) and the fused attention-block kernel (decode_block.hip): the Q40 ring GEMV body
// with its prologues / epilogues / fused TP exchange, and the decode attention task.
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
            const size_t off = kvRow(a.kvMap, a.seqLen, sl, p) * a.kv0 + (r0 - a.q0);
            if (a.kvBf16) {
                const uint32_t pk = (uint32_t)f32ToBf16(o0) | ((uint32_t)f32ToBf16(o1) << 16);
                st32<WT>(reinterpret_cast<uint16_t *>(a.kcache) + off, pk);
            } else {
                stF2<WT>(reinterpret_cast<float *>(a.kcache) + off, o0, o1);
            }
        }
    } else {
        const size_t off = kvRow(a.kvMap, a.seqLen, sl, p) * a.kv0 + (r0 - a.q0 - a.kv0);
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

// Ring-GEMV variants: GEMV_PLAIN (a standalone launch), GEMV_PRODUCER (rows published write-
// through to consumers in the same launch + arrival counts, see BlockSync), GEMV_CONSUMER (the
// Q80 activations are produced in the same launch: wait for them after the ring is issued).
enum GemvMode : int { GEMV_PLAIN = 0, GEMV_PRODUCER = 1, GEMV_CONSUMER = 2 };

// In-launch hand-off state of the fused attention block (decode_block.hip).
// Counters are monotonic across layers and forwards (never reset): after the s-th layer step
// (s = (forward epoch - 1) * nLayers + layer + 1) KV group g's counter has been incremented
// s * qkvExpect[g] times and the attention counter s * (head groups) times, so a waiter compares
// against a target computed from s in wrapping u32 arithmetic ((int)(cnt - target) >= 0).
// Every polled word sits on its own 256-byte line (kCntStride u32): 192 qkv workgroups adding into
// one line serialised their atomics (~4 us per layer, traced); the attention -> wo "ready" flag is
// replicated per XCD so 256 pollers do not hammer one line.
constexpr int kCntStride = 64;
struct BlockSync {
    unsigned *qkvCnt = nullptr;          // [kv groups * kCntStride] arrivals of qkv workgroups per group
    const unsigned *qkvExpect = nullptr; // [kv groups] qkv workgroups touching each group
    unsigned *attnCnt = nullptr;         // [1] arrivals of attention head groups (final outputs)
    unsigned *attnFlag = nullptr;        // [8 * kCntStride] per-XCD copies of the last step all heads finished
    unsigned *qkvAll = nullptr;          // [1] arrivals of every qkv workgroup
    unsigned *qkvFlag = nullptr;         // [8 * kCntStride] per-XCD copies of the last step the qkv phase finished
    unsigned qkvAllTarget = 0;           // s * qkv workgroups
    unsigned step = 0;                   // s (see above)
    int nKv = 0;                         // KV groups
    unsigned attnTarget = 0;             // s * head groups
    int *error = nullptr;                // set when a wait gave up (the engine raises)
    long long timeoutTicks = 0;
    int codeBase = 0;                    // added to the GEMV waits' error codes (3 data, 4 ring start)
    bool ringEarly = false;              // consumer: issue the weight ring at entry (no ring-start wait)
};
__device__ __forceinline__ int xccId() { return (int)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u); }

// One lane waits (relaxed agent-scope polls + s_sleep, bounded: a wait that gives up sets the
// error word and every later wait fails fast), then the workgroup's barrier releases the others.
__device__ __forceinline__ unsigned long long blockWait(const unsigned *cnt, unsigned target, const BlockSync &bs,
                                                        int code = 1) {
    unsigned long long stamp = 0ull;
    if (threadIdx.x == 0) {
        if (__hip_atomic_load(bs.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while ((int)(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
                __builtin_amdgcn_s_sleep(1);
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > bs.timeoutTicks) {
                    __hip_atomic_store(bs.error, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        stamp = wall_clock64();
    }
    __syncthreads();
    return stamp;
}

// Raise the per-XCD copies of a "step done" flag (the last arriver of a phase).
__device__ __forceinline__ void raiseFlags(unsigned *flag, unsigned step) {
#pragma unroll
    for (int k = 0; k < 8; k++) __hip_atomic_store(flag + k * kCntStride, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// After write-through stores: every wave drains its stores, the barrier, then one lane signals.
__device__ __forceinline__ void blockDrain() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// KV groups touched by qkv rows [r0, r1) (Q rows of the group's kvMul heads, its K and V rows):
// a bit mask (<= 64 groups). Shared by the producers and the host's expected counts.
__host__ __device__ inline unsigned long long qkvGroupMask(int r0, int r1, int q0, int kv0, int hs, int kvMul) {
    unsigned long long m = 0;
    auto span = [&](int lo, int hi, int base, int per) {  // rows [lo, hi) of a part starting at base
        if (lo >= hi) return;
        for (int g = (lo - base) / per; g <= (hi - 1 - base) / per; g++) m |= 1ull << g;
    };
    auto mx = [](int x, int y) { return x > y ? x : y; };
    auto mn = [](int x, int y) { return x < y ? x : y; };
    span(mx(r0, 0), mn(r1, q0), 0, kvMul * hs);
    span(mx(r0, q0), mn(r1, q0 + kv0), q0, hs);
    span(mx(r0, q0 + kv0), mn(r1, q0 + 2 * kv0), q0 + kv0, hs);
    return m;
}

template <int L, int B, int PRO, int EPI, int MODE = GEMV_PLAIN>
__device__ __forceinline__ void gemvQ40Body(const GemvArgs &a, const int blk, char *smem, const BlockSync *bs = nullptr) {
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
    const int rowBase = blk * R;
    // timestamps stay in SGPRs until the end: a store here would join the ring's vmcnt accounting
    const unsigned long long tEntry = a.trace ? wall_clock64() : 0ull;
    unsigned long long tReady = 0ull, tLoaded = 0ull, tFirst = 0ull, tWaited = 0ull;

    // slot = 2 rows x 16 B of nibbles + the pair's two f16 scales in one 32-bit word
    u32x4 w[D][RG];
    uint32_t dh[D];
    const uint32_t *wd2 = reinterpret_cast<const uint32_t *>(a.wd);  // tiled pair scales
    // this workgroup's chunks are [blk * T, blk * T + T) of the tiled matrix
    const size_t cBase = (size_t)blk * T;
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
            float *xo = (blk == 0 && a.xNext) ? a.xNext : nullptr;
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
        // consumer: the weight ring is issued once the qkv phase of the launch is done, so it streams
        // while HBM would idle during attention instead of competing with the qkv weights
        if constexpr (MODE == GEMV_CONSUMER)
            if (!bs->ringEarly) blockWait(bs->qkvFlag + xccId() * kCntStride, bs->step, *bs, bs->codeBase + 4);
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
        if constexpr (MODE == GEMV_CONSUMER) {
            // the activations are produced in this launch: wait for every producer (the ring's
            // weight loads are already in flight), then read them write-through
            tWaited = blockWait(bs->attnFlag + xccId() * kCntStride, bs->step, *bs, bs->codeBase + 3);
            stageQ80<B, true>(a, sq, ssc);
        } else if constexpr (PRO == PRO_RESNORM)
            resNormPrologue<B, true>(a, scratch, sq, ssc, nullptr);
        else {
            stageQ80<B>(a, sq, ssc);
        }
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
                    qkvPairStore<MODE == GEMV_PRODUCER>(a, r0, v0, v1, sRope + b * (kMaxHeadSize / 2), posB[b], slotB[b],
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

    const int unitsPerThread = PRO != PRO_GLOBAL ? (n + 8 * kThreads - 1) / (8 * kThreads)
                                                  : (n + 16 * kThreads - 1) / (16 * kThreads);
    static_assert(MODE != GEMV_CONSUMER || PRO == PRO_GLOBAL, "a consumer GEMV reads Q80 activations");
    if constexpr (MODE == GEMV_CONSUMER) {
        latePath();
        mainLoop();
    } else if (B == 1 && unitsPerThread <= 1) {
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
        storeHiddenQ80<B, MODE == GEMV_PRODUCER>(a, hbuf, R >> 1, rowBase >> 1);
    }
    if constexpr (MODE == GEMV_PRODUCER) {  // rows published write-through: drain, then count in
        blockDrain();
        if (tid == 0) {
            if constexpr (EPI == EPI_QKV) {  // attention block: per KV group arrivals
                unsigned long long m = qkvGroupMask(rowBase, min(rowBase + R, a.rows), a.q0, a.kv0, a.hs, a.kvMul);
                while (m) {
                    const int g = __builtin_ctzll(m);
                    m &= m - 1;
                    __hip_atomic_fetch_add(bs->qkvCnt + g * kCntStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            // the last producer workgroup of the step raises the per-XCD "phase done" flags: the
            // attention block's wo role starts its weight ring (so the wo weights stream while
            // attention runs instead of competing with qkv's), the FFN block's w2 role its ring + reads
            if (__hip_atomic_fetch_add(bs->qkvAll, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == bs->qkvAllTarget)
                raiseFlags(bs->qkvFlag, bs->step);
        }
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
            unsigned long long *t = a.trace + 8 * (size_t)blk;
            t[0] = tEntry;
            t[1] = tReady;
            t[2] = tExit;
            t[3] = ((unsigned long long)hw << 32) | xcc;
            t[4] = tLoaded;
            t[5] = tFirst;
            t[6] = tWaited;
        }
    }
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
// WT: write-through (the fused attention block's wo workgroups read the Q80 output in the same
// launch): 4 int8 per 32-bit store, the scale pair as one 64-bit store.
template <int HG, int HS, int AT, bool WT = false>
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
            if constexpr (WT) {
                const int q1 = __shfl_down(q, 1), q2 = __shfl_down(q, 2), q3 = __shfl_down(q, 3);
                if ((i & 3) == 0)
                    st32<true>(a.outQ + (size_t)b * a.ldOut + col, (uint32_t)(q & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) |
                                                                       ((uint32_t)(q2 & 0xFF) << 16) | ((uint32_t)q3 << 24));
            } else {
                a.outQ[(size_t)b * a.ldOut + col] = (int8_t)q;
            }
            const float qs = groupSum<32>((float)q);
            if ((i & 31) == 0) {
                float *sp = reinterpret_cast<float *>(a.outS + (size_t)b * (a.ldOut >> 5) + (col >> 5));
                stF2<WT>(sp, roundF16(d), qs);
            }
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
template <int HG, int HS, int AT, bool WT = false>
__device__ __forceinline__ bool attnFinish(const AttnArgs &a, int b, int hgIdx, int c, int nSplit, float *redL,
                                           float *mlL, int *flagL, float *scratch) {
    const int tid = threadIdx.x, head0 = hgIdx * HG;
    if (nSplit == 1) {
        for (int i = tid; i < HG * HS; i += AT) redL[i] = redL[i] / mlL[(i / HS) * 2 + 1];
        __syncthreads();
        attnWriteOut<HG, HS, AT, WT>(a, b, head0, redL);
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
    // Weighted sum of the chunks' partial outputs: (item = 4 dims of one head) x (part = a strided
    // subset of the chunks) per thread, the `parts` threads of an item adjacent lanes, every load
    // of a thread (16-B coherence-point loads, sc1 like the atomic loads above) in flight at once,
    // then a fixed butterfly over the parts (deterministic). One memory round trip for <= 8 chunks
    // per thread instead of one per 8 chunks of a head dimension (long contexts: 32 chunks).
    constexpr int U = 8, ITEMS = HG * (HS / 4), PARTS = ITEMS >= AT ? 1 : AT / ITEMS;
    for (int base = 0; base < ITEMS * PARTS; base += AT) {
        const int t = base + tid, item = t / PARTS, part = t % PARTS;
        const int h = min(item, ITEMS - 1) / (HS / 4), d = (min(item, ITEMS - 1) % (HS / 4)) * 4;
        const float *po = a.partO + (pbase + (size_t)h * G) * HS + d;
        const float *wv = scratch + 2 * h * G;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int c0 = part; c0 < nSplit; c0 += U * PARTS) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int cc = min(c0 + u * PARTS, nSplit - 1);
                asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[u]) : "v"(po + (size_t)cc * HS));
            }
#pragma unroll
            for (int u = 0; u < U; u++) {  // each wait pins its own load's registers (no early use)
                asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v[u]) : "i"(U - 1 - u) : "memory");
                if (c0 + u * PARTS < nSplit) acc += wv[2 * (c0 + u * PARTS)] * v[u];
            }
        }
#pragma unroll
        for (int off = 1; off < PARTS; off <<= 1)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[j] += __shfl_xor(acc[j], off);
        if (part == 0 && item < ITEMS) {
            const float il = 1.0f / mlL[h * 2 + 1];
#pragma unroll
            for (int j = 0; j < 4; j++) redL[h * HS + d + j] = acc[j] * il;
        }
    }
    __syncthreads();
    attnWriteOut<HG, HS, AT, WT>(a, b, head0, redL);
    return true;
}

// One attention task: query heads [hgIdx*HG, +HG) of row b over sequence chunk c, AT threads.
// Returns true when this call wrote the head group's final output (single chunk, or the last
// chunk to arrive combined all of them).
// SYNC (fused attention block): q and the current position's K / V rows are produced by the qkv
// workgroups of the same launch - wait for this KV group's producers, read those write-through.
template <int HG, int HS, bool BF16, int AT, bool SYNC = false>
__device__ __forceinline__ bool attnTask(const AttnArgs &a, int b, int hgIdx, int c, char *smem,
                                         const BlockSync *bs = nullptr, unsigned long long *trace = nullptr) {
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

    // SYNC: the first round's keys written by earlier forwards are loaded before the wait (their
    // latency overlaps the qkv workgroups); the current position's row after it, write-through

    uint32_t kr[TU][RW], vr[TU][RW];
    // phase 0: every key (the current one write-through under SYNC); 1: all but the current one;
    // 2: only the current one
    auto loadRound = [&](int tb, int phase) {
#pragma unroll
        for (int u = 0; u < TU; u++) {
            const int t = min(tb + u * NG, t1 - 1);  // clamped: no divergent loads
            const bool cur = SYNC && t == pos;
            if ((phase == 1 && cur) || (phase == 2 && !cur)) continue;
            const size_t off = kvRow(a.kvMap, a.seqLen, sl, t) * a.kv0 + kvh * HS + l16 * DPL;
            const uint32_t *kp = reinterpret_cast<const uint32_t *>(
                BF16 ? (const void *)(reinterpret_cast<const uint16_t *>(a.kcache) + off)
                     : (const void *)(reinterpret_cast<const float *>(a.kcache) + off));
            const uint32_t *vp = reinterpret_cast<const uint32_t *>(
                BF16 ? (const void *)(reinterpret_cast<const uint16_t *>(a.vcache) + off)
                     : (const void *)(reinterpret_cast<const float *>(a.vcache) + off));
            if (cur) {  // appended by this launch's qkv workgroups: write-through loads
#pragma unroll
                for (int w = 0; w < RW; w += 2) {
                    const uint64_t kk = ldWT64(kp + w), vv = ldWT64(vp + w);
                    kr[u][w] = (uint32_t)kk;
                    kr[u][w + 1] = (uint32_t)(kk >> 32);
                    vr[u][w] = (uint32_t)vv;
                    vr[u][w + 1] = (uint32_t)(vv >> 32);
                }
            } else if constexpr (RW == 4) {
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
    };
    int tb = t0 + g16;
    bool prefetched = false;
    unsigned long long tWaited = 0ull;
    if constexpr (SYNC) {
        if (tb < t1) {
            loadRound(tb, 1);
            prefetched = true;
        }
        tWaited = blockWait(bs->qkvCnt + kvh * kCntStride, bs->step * bs->qkvExpect[kvh], *bs, 2);
    }
    // this lane's slice of the HG query heads (pre-scaled), vector loads
    const float scale = 1.0f / sqrtf((float)HS);
    float qr[HG][DPL];
#pragma unroll
    for (int h = 0; h < HG; h++) {
        const float *qp = a.q + (size_t)b * a.ldq + (head0 + h) * HS + l16 * DPL;
#pragma unroll
        for (int i = 0; i < DPL; i += 4) {
            float4 v;
            if constexpr (SYNC) {
                const uint64_t lo = ldWT64(qp + i), hi = ldWT64(qp + i + 2);
                v = make_float4(__uint_as_float((uint32_t)lo), __uint_as_float((uint32_t)(lo >> 32)),
                                __uint_as_float((uint32_t)hi), __uint_as_float((uint32_t)(hi >> 32)));
            } else {
                v = ld4(qp + i);
            }
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
    for (; tb < t1; tb += TU * NG) {
        loadRound(tb, prefetched ? 2 : 0);
        prefetched = false;
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

    if (trace && threadIdx.x == 0) {
        trace[1] = tWaited;
        trace[2] = wall_clock64();
    }
    return attnFinish<HG, HS, AT, SYNC>(a, b, hgIdx, c, nSplit, redL, mlL, flagL, oW);
}


}  // namespace hipk
}  // namespace dl
