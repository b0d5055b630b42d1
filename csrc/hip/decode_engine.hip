// Persistent decode engine (kernels.h PdeArgs): one launch runs every layer of a single-row decode
// forward. One 768-thread workgroup per CU:
//   * 8 ring waves = 2 virtual workgroups (VWG) of 256 lanes. Each VWG owns a contiguous range of
//     8-row passes of every matrix (qkv, wo, w13, w2) of every layer and streams them as ONE
//     sequence of weight steps through a per-lane register ring (kPdeD steps of 2 x 16 B nibbles +
//     the pair's f16 scales in flight, inline-asm loads with counted vmcnt waits, as the standalone
//     GEMV): the ring runs ahead across matrices and layers, so the weights of the next phase are
//     already streaming while a phase waits for its inputs. Ring waves issue no other global
//     memory operation: they read the activation image from LDS, leave raw row results in LDS and
//     meet the aux waves at two workgroup barriers per phase (activations staged / results ready).
//   * 4 aux waves (256 threads) do everything else: residual add + RMS norm + Q80 of the
//     activation image, RoPE + KV-cache append, one attention head per workgroup, SwiGLU + Q80 of
//     the hidden vector, and the cross-workgroup hand-offs of every phase (write-through stores,
//     drained, then one agent-scope add to a per-XCD counter shard; consumers poll the shards with
//     write-through loads and read the payload write-through: MI355X_MICROARCH.md "Valid forms").
// Every wait is bounded (error word, fail-fast once set); ring waves only wait on barriers, so the
// launch always drains. Reference step chain this replaces: llm.cpp:200-391 (26 ops + 2 syncs per
// layer, nn-executor.cpp:124-187 barrier per op).
#include "decode_dev.h"
#include "device_comm.h"

#include <cstdlib>

namespace dl {
namespace hipk {

constexpr int kPdeRingThreads = 512;
constexpr int kPdeAuxThreads = 256;
constexpr int kPdeThreads = kPdeRingThreads + kPdeAuxThreads;
// Ring depth D (steps per lane, 3 loads each): the kernel is instantiated for several; deeper rings
// prefetch more of the next phase across a hand-off but queue the aux waves' loads behind more
// weight traffic on the same CU (pdeRingDepth picks; decode_engine trace in profiles/).

// LDS image of one workgroup.
struct PdeLds {
    size_t x, act, sc, res, rope, attn, misc, seg, total;
};
__host__ __device__ static inline PdeLds pdeLayout(int dim, int nMax, int nPhases) {
    PdeLds l;
    size_t off = 0;
    l.x = off;  // the residual stream (f32, replicated in every workgroup)
    off += (size_t)dim * 4;
    l.act = off;  // Q80 activation image of the current phase (at the end: the last w2 output, f32)
    off = alignUp(off + (size_t)(nMax > 4 * dim ? nMax : 4 * dim), 16);
    l.sc = off;
    off = alignUp(off + (size_t)(nMax / 32) * 8, 16);
    l.res = off;  // raw row results [2 VWGs][kPdeMaxRes]
    off += (size_t)2 * kPdeMaxRes * 4;
    l.rope = off;  // RoPE row of this forward's position
    off += (size_t)(kMaxHeadSize / 2) * 8;
    l.attn = off;  // attention: q, per-wave (m, l, o), output
    off += (size_t)(kMaxHeadSize + 4 * (2 + kMaxHeadSize) + kMaxHeadSize) * 4 + 64;
    l.misc = off;  // reductions + aux barrier counter + ring-wave trace stamps (PdeArgs::trace)
    off += 192;
    l.seg = off;  // [2 VWGs][4 * nLayers] stream segments
    off += (size_t)2 * nPhases * 32;
    l.total = alignUp(off, 16);
    return l;
}

// ------------------------------------------------------------------------------------------------
// aux-wave helpers (threads kPdeRingThreads .. +256)
// ------------------------------------------------------------------------------------------------
struct AuxCtx {
    unsigned *bar;     // LDS counter of the aux barrier
    unsigned gen = 0;  // aux barrier generation (each wave counts its own arrivals)
    float *red;        // LDS [4] reduction scratch
    int at, wave, lane;
};

// Barrier of the 4 aux waves (LDS counter; the ring waves are not involved).
__device__ __forceinline__ void auxSync(AuxCtx &c) {
    c.gen += 4;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (c.lane == 0) __hip_atomic_fetch_add(c.bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(c.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) - c.gen) < 0) {
        __builtin_amdgcn_s_sleep(0);
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > 200000000LL) break;  // 2 s: never hang the launch
    }
    asm volatile("" ::: "memory");
}

// Sum over the 256 aux threads (every thread gets it).
__device__ __forceinline__ float auxSum(AuxCtx &c, float v) {
    v = waveSum(v);
    if (c.lane == 0) c.red[c.wave] = v;
    auxSync(c);
    const float s = c.red[0] + c.red[1] + c.red[2] + c.red[3];
    auxSync(c);  // red is reused by the next reduction
    return s;
}

// Bounded wait until the sum of `shards` counters (8, one 256-B line apart) reaches `target`.
__device__ __forceinline__ void auxWait(const PdeArgs &a, const unsigned *cnt, int shards, unsigned target, int code,
                                        int lane) {
    if (__hip_atomic_load(a.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while (true) {
        unsigned v = lane < shards ? ldWT32(cnt + lane * kCntStride) : 0u;
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v = __shfl(v, 0);
        if ((int)(v - target) >= 0) return;
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > a.timeoutTicks) {
            if (lane == 0) __hip_atomic_store(a.error, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// After the aux waves' write-through stores: drain every wave, then one lane adds to the counter
// shard of this XCD (or to `cnt` itself when shards == 1).
__device__ __forceinline__ void auxSignal(AuxCtx &c, unsigned *cnt, bool sharded) {
    auxSync(c);  // includes every aux wave's vmcnt(0)
    if (c.at == 0)
        __hip_atomic_fetch_add(cnt + (sharded ? xccId() * kCntStride : 0), 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}

// Copy `bytes` (a multiple of 16) of a vector produced in this launch from global memory into LDS:
// 16-B write-through (sc1) loads, up to 8 per thread in flight per round.
__device__ __forceinline__ void auxCopyWT(const AuxCtx &c, const void *src, void *dst, int bytes) {
    const f32x4 *s4 = reinterpret_cast<const f32x4 *>(src);
    f32x4 *d4 = reinterpret_cast<f32x4 *>(dst);
    const int n16 = bytes >> 4;
    for (int base = 0; base < n16; base += 8 * kPdeAuxThreads) {
        f32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int i = min(base + c.at + k * kPdeAuxThreads, n16 - 1);
            asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[k]) : "v"(s4 + i));
        }
#pragma unroll
        for (int k = 0; k < 8; k++) {
            asm volatile("s_waitcnt vmcnt(%1)" : "+v"(v[k]) : "i"(7 - k) : "memory");
            const int i = base + c.at + k * kPdeAuxThreads;
            if (i < n16) d4[i] = v[k];
        }
    }
}

// The RMS norm's weights for auxResNorm, issued early (before the hand-off wait): <= 4 chunks of
// 8 floats per aux thread, asm loads waited inside auxResNorm.
struct NormW {
    f32x4 w[4][2];
};
__device__ __forceinline__ NormW auxNormIssue(const AuxCtx &c, const PdeArgs &a, const float *w) {
    NormW r;
    const int nChunks = a.dim >> 3;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ch = min(c.at + k * kPdeAuxThreads, nChunks - 1);
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r.w[k][0]) : "v"(w + ch * 8));
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r.w[k][1]) : "v"(w + ch * 8 + 4));
    }
    return r;
}

// x (LDS) += delta (write-through global, or the embedding output when init), then RMS norm with
// the pre-issued weights -> the Q80 activation image. dim is a multiple of 32 (whole Q80 blocks
// per quad of 8-float chunks), <= 8192.
__device__ __forceinline__ void auxResNorm(AuxCtx &c, const PdeArgs &a, float *xs, const float *delta, bool init,
                                           NormW &nw, int8_t *sq, float2 *ssc) {
    const int nChunks = a.dim >> 3;  // 8 floats per chunk, <= 4 chunks per thread
    f32x4 d[4][2];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // every delta / input load in flight at once
        const int ch = min(c.at + k * kPdeAuxThreads, nChunks - 1);
        const float *src = init ? a.xIn + ch * 8 : delta + ch * 8;
        if (init) {
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d[k][0]) : "v"(src));
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d[k][1]) : "v"(src + 4));
        } else {
            asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(d[k][0]) : "v"(src));
            asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(d[k][1]) : "v"(src + 4));
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(d[0][0]), "+v"(d[0][1]), "+v"(d[1][0]), "+v"(d[1][1]), "+v"(d[2][0]),
                 "+v"(d[2][1]), "+v"(d[3][0]), "+v"(d[3][1])::"memory");
    asm volatile("" : "+v"(nw.w[0][0]), "+v"(nw.w[0][1]), "+v"(nw.w[1][0]), "+v"(nw.w[1][1]), "+v"(nw.w[2][0]),
                 "+v"(nw.w[2][1]), "+v"(nw.w[3][0]), "+v"(nw.w[3][1]));  // (landed with the wait above)
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ch = c.at + k * kPdeAuxThreads;
        if (ch < nChunks) {
            f32x4 v0 = d[k][0], v1 = d[k][1];
            if (!init) {
                v0 += *reinterpret_cast<const f32x4 *>(xs + ch * 8);
                v1 += *reinterpret_cast<const f32x4 *>(xs + ch * 8 + 4);
            }
            *reinterpret_cast<f32x4 *>(xs + ch * 8) = v0;
            *reinterpret_cast<f32x4 *>(xs + ch * 8 + 4) = v1;
            d[k][0] = v0;
            d[k][1] = v1;
            ss += v0.x * v0.x + v0.y * v0.y + v0.z * v0.z + v0.w * v0.w + v1.x * v1.x + v1.y * v1.y + v1.z * v1.z +
                  v1.w * v1.w;
        }
    }
    ss = auxSum(c, ss);
    const float inv = 1.0f / sqrtf(ss / (float)a.dim + a.eps);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int ch = c.at + k * kPdeAuxThreads;
        if (ch < nChunks) {
            const f32x4 w0 = nw.w[k][0], w1 = nw.w[k][1], x0 = d[k][0], x1 = d[k][1];
            float v[8] = {w0.x * (inv * x0.x), w0.y * (inv * x0.y), w0.z * (inv * x0.z), w0.w * (inv * x0.w),
                          w1.x * (inv * x1.x), w1.y * (inv * x1.y), w1.z * (inv * x1.z), w1.w * (inv * x1.w)};
            stageChunk<true>(v, 0, ch, a.dim, sq, ssc, nullptr);
        }
    }
}

// Q80 vector (n int8 + n/32 scale pairs) produced in this launch -> the LDS activation image.
__device__ __forceinline__ void auxStageQ80(AuxCtx &c, const int8_t *q, const float2 *s, int n, int8_t *sq,
                                            float2 *ssc) {
    auxCopyWT(c, q, sq, n);
    auxCopyWT(c, s, ssc, (n >> 5) * 8);
}

// Quantize 32-element blocks of `v` (one value per lane, lanes of a 32-lane group = one block) and
// store them write-through: 4 int8 per 32-bit store, the (d, sum q) pair as one 64-bit store.
__device__ __forceinline__ void q80StoreWT(float v, int8_t *qDst, float2 *sDst, int idx) {
    const float amax = groupMax<32>(fabsf(v));
    const float d = amax / 127.0f;
    const float id = d != 0.f ? 1.0f / d : 0.f;
    int q = (int)rintf(v * id);
    q = q > 127 ? 127 : (q < -127 ? -127 : q);
    const uint32_t u = (uint32_t)(uint8_t)q;
    const uint32_t word = u | ((uint32_t)__shfl_down((int)u, 1, 32) << 8) | ((uint32_t)__shfl_down((int)u, 2, 32) << 16) |
                          ((uint32_t)__shfl_down((int)u, 3, 32) << 24);
    if ((idx & 3) == 0) st32<true>(qDst + idx, word);
    const float qs = groupSum<32>((float)q);
    if ((idx & 31) == 0) stF2<true>(reinterpret_cast<float *>(sDst + (idx >> 5)), roundF16(d), qs);
}

// RW 32-bit words (RW = 2, 4 or 8) of one cache row per lane, asm load (waited by the caller).
template <int RW>
__device__ __forceinline__ void ldRow(const uint32_t *p, uint32_t (&r)[RW]) {
    if constexpr (RW == 2) {
        u32x2 v;
        asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p));
        r[0] = v.x, r[1] = v.y;
    } else if constexpr (RW == 4) {
        u32x4 v;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p));
        r[0] = v.x, r[1] = v.y, r[2] = v.z, r[3] = v.w;
    } else {
        u32x4 v0, v1;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v0) : "v"(p));
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v1) : "v"(p + 4));
        r[0] = v0.x, r[1] = v0.y, r[2] = v0.z, r[3] = v0.w, r[4] = v1.x, r[5] = v1.y, r[6] = v1.z, r[7] = v1.w;
    }
}

// One decode attention head over keys [0, pos]: the current key / value rows come from the qkv
// hand-off (write-through), earlier ones from the cache. 16 groups of 16 lanes, HS/16 dims per
// lane, TU keys per group per round; the first round of cached keys is loaded BEFORE waiting for
// this head's qkv producers (those keys do not depend on them), so a context of <= 16 TU keys
// costs one memory round trip after the hand-off. Online softmax; output -> Q80 hand-off.
template <int HS, bool BF16>
__device__ __forceinline__ void auxAttention(AuxCtx &c, const PdeArgs &a, int head, int l, int pos, int sl, float *sm,
                                             const unsigned *groupCnt, unsigned target) {
    constexpr int DPL = HS / 16, RW = BF16 ? DPL / 2 : DPL, TU = 4;
    const int g16 = c.at >> 4, l16 = c.at & 15, kvh = head / a.kvMul;
    const void *kc = a.kcache[l], *vc = a.vcache[l];
    const float scale = 1.0f / sqrtf((float)HS);
    uint32_t kr[TU][RW], vr[TU][RW];
    auto loadRound = [&](int tb) {
#pragma unroll
        for (int u = 0; u < TU; u++) {
            const int t = max(min(tb + u * 16, pos - 1), 0);
            const size_t off = kvRow(a.kvMap, a.seqLen, sl, t) * a.kv0 + kvh * HS + l16 * DPL;
            const uint32_t *kp = reinterpret_cast<const uint32_t *>(
                BF16 ? (const void *)(reinterpret_cast<const uint16_t *>(kc) + off)
                     : (const void *)(reinterpret_cast<const float *>(kc) + off));
            const uint32_t *vp = reinterpret_cast<const uint32_t *>(
                BF16 ? (const void *)(reinterpret_cast<const uint16_t *>(vc) + off)
                     : (const void *)(reinterpret_cast<const float *>(vc) + off));
            ldRow<RW>(kp, kr[u]);
            ldRow<RW>(vp, vr[u]);
        }
    };
    auto waitRound = [&] {
#pragma unroll
        for (int u = 0; u < TU; u++)
#pragma unroll
            for (int w = 0; w < RW; w++) asm volatile("s_waitcnt vmcnt(0)" : "+v"(kr[u][w]), "+v"(vr[u][w])::"memory");
    };
    loadRound(g16);  // (clamped addresses: always valid, position 0 exists)
    auxWait(a, groupCnt, 1, target, 22, c.lane);
    float qr[DPL], kcur[DPL], vcur[DPL];
    {
        const float *qp = a.eQkv + head * HS + l16 * DPL;
        const float *kp = a.eQkv + a.q0 + kvh * HS + l16 * DPL;
        const float *vp = a.eQkv + a.q0 + a.kv0 + kvh * HS + l16 * DPL;
#pragma unroll
        for (int i = 0; i < DPL; i += 2) {
            const uint64_t q2 = ldWT64(qp + i), k2 = ldWT64(kp + i), v2 = ldWT64(vp + i);
            qr[i] = __uint_as_float((uint32_t)q2) * scale;
            qr[i + 1] = __uint_as_float((uint32_t)(q2 >> 32)) * scale;
            kcur[i] = __uint_as_float((uint32_t)k2);
            kcur[i + 1] = __uint_as_float((uint32_t)(k2 >> 32));
            vcur[i] = __uint_as_float((uint32_t)v2);
            vcur[i + 1] = __uint_as_float((uint32_t)(v2 >> 32));
        }
    }
    if constexpr (BF16) {  // the cache holds bf16: score the current key at the precision it is stored
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            kcur[i] = bf16ToF32(f32ToBf16(kcur[i]));
            vcur[i] = bf16ToF32(f32ToBf16(vcur[i]));
        }
    }
    float m = -INFINITY, lsum = 0.f, o[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) o[i] = 0.f;
    auto accum = [&](const float(&kv)[DPL], const float(&vv)[DPL]) {
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < DPL; i++) d += qr[i] * kv[i];
        d = groupSum<16>(d);
        const float mn = fmaxf(m, d);
        const float corr = __expf(m - mn);
        const float p = __expf(d - mn);
        lsum = lsum * corr + p;
#pragma unroll
        for (int i = 0; i < DPL; i++) o[i] = o[i] * corr + p * vv[i];
        m = mn;
    };
    for (int tb = g16; tb < pos; tb += TU * 16) {
        if (tb != g16) loadRound(tb);
        waitRound();
#pragma unroll
        for (int u = 0; u < TU; u++) {
            if (tb + u * 16 >= pos) break;
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
            accum(kv, vv);
        }
    }
    waitRound();  // (a context without cached keys still drains the prefetch)
    if (g16 == (pos & 15)) accum(kcur, vcur);  // key `pos` in the group that owns it
    // merge the 4 groups of each wave, then the 4 waves through LDS
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
        const float m2 = __shfl_xor(m, off), l2 = __shfl_xor(lsum, off);
        float o2[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++) o2[i] = __shfl_xor(o[i], off);
        softmaxMerge<DPL>(m, lsum, o, m2, l2, o2);
    }
    float *mW = sm, *lW = sm + 4, *oW = sm + 8;  // [4] [4] [4][HS]
    float *fin = oW + 4 * HS;                     // [HS]
    if (c.lane < 16) {
        if (c.lane == 0) {
            mW[c.wave] = m;
            lW[c.wave] = lsum;
        }
#pragma unroll
        for (int i = 0; i < DPL; i++) oW[c.wave * HS + c.lane * DPL + i] = o[i];
    }
    auxSync(c);
    if (c.at < HS) {
        float M = -INFINITY;
#pragma unroll
        for (int w = 0; w < 4; w++) M = fmaxf(M, mW[w]);
        float acc = 0.f, Ls = 0.f;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const float e = M == -INFINITY ? 0.f : __expf(mW[w] - M);
            acc += e * oW[w * HS + c.at];
            Ls += e * lW[w];
        }
        fin[c.at] = acc / Ls;
    }
    auxSync(c);
    if (c.at < HS) q80StoreWT(fin[c.at], a.eAttQ, a.eAttS, head * HS + c.at);
}

// ------------------------------------------------------------------------------------------------
// ring waves: the weight stream
// ------------------------------------------------------------------------------------------------
// One (layer, matrix) segment of a VWG's weight stream (LDS).
struct PdeSeg {
    const u32x4 *qs;    // first step's nibble chunk
    const uint32_t *d;  // first step's scale chunk
    int steps, K, n, pad;
};
// Per-matrix values are selected, never indexed by a runtime matrix number (a dynamically indexed
// kernel-argument or private array would go through scratch memory).
template <typename T>
__device__ __forceinline__ T sel4(int m, T x0, T x1, T x2, T x3) {
    return m == 0 ? x0 : (m == 1 ? x1 : (m == 2 ? x2 : x3));
}

template <int HS, bool BF16, int kPdeD>
__global__ __launch_bounds__(kPdeThreads) void pdeKernel(PdeArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nMax = max(max(a.dim, a.hidden), a.q0);
    const PdeLds lay = pdeLayout(a.dim, nMax, 4 * a.nLayers);
    float *xs = reinterpret_cast<float *>(smem + lay.x);
    int8_t *sq = reinterpret_cast<int8_t *>(smem + lay.act);
    float2 *ssc = reinterpret_cast<float2 *>(smem + lay.sc);
    float *res = reinterpret_cast<float *>(smem + lay.res);
    float2 *sRope = reinterpret_cast<float2 *>(smem + lay.rope);
    float *sAttn = reinterpret_cast<float *>(smem + lay.attn);
    unsigned *misc = reinterpret_cast<unsigned *>(smem + lay.misc);
    const int tid = threadIdx.x;
    const int nPhases = 4 * a.nLayers;
    const unsigned epoch = *a.epoch;
    auto stepOf = [&](int l) { return (epoch - 1u) * (unsigned)a.nLayers + (unsigned)l + 1u; };
    auto barrier = [] {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    if (tid < kPdeRingThreads) {  // the ring waves describe their VWG's stream segments
        const int u = tid >> 8, v = 2 * blockIdx.x + u, t256 = tid & 255, V = 2 * gridDim.x;
        PdeSeg *segs = reinterpret_cast<PdeSeg *>(smem + lay.seg) + u * nPhases;
        for (int ph = t256; ph < nPhases; ph += 256) {
            const int l = ph >> 2, m = ph & 3;
            const int pb = a.passStart[m * (V + 1) + v], pe = a.passStart[m * (V + 1) + v + 1];
            const int K = sel4(m, a.K[0], a.K[1], a.K[2], a.K[3]);
            PdeSeg sg;
            sg.qs = reinterpret_cast<const u32x4 *>(sel4(m, a.qs[0], a.qs[1], a.qs[2], a.qs[3]) +
                                                    (size_t)l * sel4(m, a.qsStride[0], a.qsStride[1], a.qsStride[2], a.qsStride[3])) +
                    (size_t)pb * K * 2 * kThreads;
            sg.d = sel4(m, a.d[0], a.d[1], a.d[2], a.d[3]) +
                   (size_t)l * sel4(m, a.dStride[0], a.dStride[1], a.dStride[2], a.dStride[3]) + (size_t)pb * K * kThreads;
            sg.steps = (pe - pb) * K;
            sg.K = K;
            sg.n = sel4(m, a.n[0], a.n[1], a.n[2], a.n[3]);
            segs[ph] = sg;
        }
    } else if (tid == kPdeRingThreads) {
        misc[0] = 0u;  // aux barrier counter
    }
    __syncthreads();  // every wave (no ring load is in flight yet)

    if (tid < kPdeRingThreads) {
        // ============================== ring waves ==============================
        // Each (layer, matrix) phase of this VWG is one segment of its weight stream, described in
        // LDS (built above, once): the ring cursors walk the segments with running pointers, so the
        // per-step work is two pointer increments and the per-matrix parameters stay out of SGPRs.
        const int u = tid >> 8;  // VWG within the workgroup
        const int t256 = tid & 255, w = t256 >> 6, lane = t256 & 63;
        const PdeSeg *segs = reinterpret_cast<const PdeSeg *>(smem + lay.seg) + u * nPhases;
        unsigned long long *rtr = reinterpret_cast<unsigned long long *>(misc + 16);  // [8] LDS stamps
        auto segSteps = [&](int ph) { return __builtin_amdgcn_readfirstlane(segs[ph].steps); };
        auto nextSeg = [&](int ph) {  // first non-empty segment after ph (nPhases: none)
            do {
                ++ph;
            } while (ph < nPhases && segSteps(ph) == 0);
            return ph;
        };
        auto segQs = [&](int ph) {
            const uint64_t p = (uint64_t)(uintptr_t)segs[ph].qs;
            return reinterpret_cast<const u32x4 *>(
                (uintptr_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(p >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)p)));
        };
        auto segD = [&](int ph) {
            const uint64_t p = (uint64_t)(uintptr_t)segs[ph].d;
            return reinterpret_cast<const uint32_t *>(
                (uintptr_t)(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(p >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)p)));
        };
        int Ttot = 0;
        for (int ph = 0; ph < nPhases; ph++) Ttot += segSteps(ph);
        // issue cursor: segment, steps left in it, running pointers
        int si = nextSeg(-1);
        bool idone = si >= nPhases;
        // (a VWG without rows keeps its slots defined by re-reading the first chunk of matrix 0)
        const u32x4 *pq = idone ? reinterpret_cast<const u32x4 *>(a.qs[0]) : segQs(si);
        const uint32_t *pd = idone ? a.d[0] : segD(si);
        int ri = idone ? 0 : segSteps(si);
        u32x4 wr[kPdeD][2];
        uint32_t dh[kPdeD];
        auto issue = [&](u32x4(&ws)[2], uint32_t &ds) {
            asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(ws[0]) : "v"(pq + t256));
            asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(ws[1]) : "v"(pq + kThreads + t256));
            asm volatile("global_load_dword %0, %1, off" : "=v"(ds) : "v"(pd + t256));
            if (idone) return;  // past the end: keep re-reading the last step
            if (--ri > 0) {
                pq += 2 * kThreads;
                pd += kThreads;
                return;
            }
            const int nx = nextSeg(si);
            if (nx >= nPhases) {
                idone = true;
                return;
            }
            si = nx;
            ri = segSteps(si);
            pq = segQs(si);
            pd = segD(si);
        };
#pragma unroll
        for (int s = 0; s < kPdeD; s++) {
            issue(wr[s], dh[s]);
            __builtin_amdgcn_sched_barrier(0);
        }
        // consume cursor
        int sc = nextSeg(-1), rc = 0, kc = 0, pc = 0, cK = 1, cN = 32;
        int entered = -1;  // phase whose activations this VWG is consuming
        float acc[2][1] = {{0.f}, {0.f}};
        auto consume = [&](const u32x4(&ws)[2], uint32_t ds) {
            if (sc != entered) {  // first step of a phase: close the previous one, skip empty ones
                if (entered >= 0) barrier();  // results of `entered` in LDS
                for (int q = entered + 1; q < sc; q++) {
                    barrier();
                    barrier();
                }
                barrier();  // activations of `sc` staged
                entered = sc;
                if (a.trace && (sc >> 2) == a.traceLayer && t256 == 0 && u == 0)
                    rtr[2 * (sc & 3)] = wall_clock64();
                rc = segSteps(sc);
                cK = __builtin_amdgcn_readfirstlane(segs[sc].K);
                cN = __builtin_amdgcn_readfirstlane(segs[sc].n);
                kc = pc = 0;
            }
            const int nb = cN >> 5, j = lane + 64 * kc;
            const bool use = j < nb;
            float dw[2];
            dw[0] = use ? __half2float(__ushort_as_half((uint16_t)(ds & 0xFFFFu))) : 0.f;
            dw[1] = use ? __half2float(__ushort_as_half((uint16_t)(ds >> 16))) : 0.f;
            q40Block<1, 2>(acc, ws, dw, min(j, nb - 1), cN, nb, sq, ssc);
            if (++kc == cK) {  // end of the pass: this wave's row pair
                const float v0 = waveSum(acc[0][0]), v1 = waveSum(acc[1][0]);
                if (lane == 0) {
                    const int i = pc * 8 + 2 * w;
                    res[u * kPdeMaxRes + i] = v0;
                    res[u * kPdeMaxRes + i + 1] = v1;
                }
                acc[0][0] = acc[1][0] = 0.f;
                kc = 0;
                ++pc;
            }
            if (--rc == 0) {
                if (a.trace && (sc >> 2) == a.traceLayer && t256 == 0 && u == 0) rtr[2 * (sc & 3) + 1] = wall_clock64();
                sc = nextSeg(sc);
            }
        };
        for (int t0 = 0; t0 < Ttot; t0 += kPdeD) {
#pragma unroll
            for (int s = 0; s < kPdeD; s++) {
                asm volatile("s_waitcnt vmcnt(%3)" : "+v"(wr[s][0]), "+v"(wr[s][1]), "+v"(dh[s]) : "i"(3 * (kPdeD - 1)));
                if (t0 + s < Ttot) consume(wr[s], dh[s]);
                issue(wr[s], dh[s]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // close the last phase and meet the aux waves at every remaining barrier
        if (entered >= 0) barrier();
        for (int q = entered + 1; q < nPhases; q++) {
            barrier();
            barrier();
        }
        return;
    }

    // ============================== aux waves ==============================
    AuxCtx c;
    c.bar = misc;
    c.red = reinterpret_cast<float *>(misc + 4);
    c.at = tid - kPdeRingThreads;
    c.wave = c.at >> 6;
    c.lane = c.at & 63;
    const int V = 2 * gridDim.x;
    const int G = gridDim.x;
    const int pos = a.pos[0], sl = a.slot[0];
    // this workgroup's pass ranges (two VWGs) per matrix
    int rb[4][2], re[4][2];
#pragma unroll
    for (int m = 0; m < 4; m++)
#pragma unroll
        for (int u = 0; u < 2; u++) {
            rb[m][u] = a.passStart[m * (V + 1) + 2 * blockIdx.x + u] * 8;
            re[m][u] = min(a.passStart[m * (V + 1) + 2 * blockIdx.x + u + 1] * 8, a.rows[m]);
        }
    unsigned *cntAtt = a.cnt + kPdeMaxKv * kCntStride;
    unsigned *cntWo = cntAtt + 8 * kCntStride, *cntH = cntWo + 8 * kCntStride, *cntW2 = cntH + 8 * kCntStride;
    const int h2 = HS / 2;
    unsigned long long *tr = a.trace ? a.trace + (size_t)blockIdx.x * 32 : nullptr;
    for (int l = 0; l < a.nLayers; l++) {
        const unsigned st = stepOf(l);
        const bool trL = tr && l == a.traceLayer && c.at == 0;
#define PDE_TR(k) \
    if (trL) tr[k] = wall_clock64();
        PDE_TR(0)
        // ---- qkv: x (+= w2 output of layer l - 1) -> norm -> Q80; RoPE row
        NormW nw = auxNormIssue(c, a, a.rmsAtt[l]);
        if (l > 0) auxWait(a, cntW2, 8, (st - 1u) * (unsigned)G, 21, c.lane);
        PDE_TR(1)
        auxResNorm(c, a, xs, a.eW2, l == 0, nw, sq, ssc);
        if (c.at < h2) sRope[c.at] = a.rope[(size_t)pos * h2 + c.at];
        PDE_TR(2)
        barrier();  // activations staged
        barrier();  // qkv rows in LDS
        PDE_TR(3)
        {
            // RoPE on q / k pairs, publish q | k | v write-through, append k / v to the cache
            unsigned long long gm = 0ull;
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int r0 = rb[0][u], nr = re[0][u] - r0;
                if (nr > 0) gm |= qkvGroupMask(r0, r0 + nr, a.q0, a.kv0, HS, a.kvMul);
                for (int i = 2 * c.at; i < nr; i += 2 * kPdeAuxThreads) {
                    const int r = r0 + i;
                    float v0 = res[u * kPdeMaxRes + i], v1 = res[u * kPdeMaxRes + i + 1];
                    if (r < a.q0 + a.kv0) {
                        const float2 cs = sRope[(r % HS) >> 1];
                        const float o0 = v0 * cs.x - v1 * cs.y, o1 = v0 * cs.y + v1 * cs.x;
                        v0 = o0, v1 = o1;
                    }
                    stF2<true>(a.eQkv + r, v0, v1);
                    if (r >= a.q0) {
                        const bool isK = r < a.q0 + a.kv0;
                        const size_t off = kvRow(a.kvMap, a.seqLen, sl, pos) * a.kv0 + (r - a.q0 - (isK ? 0 : a.kv0));
                        void *cache = isK ? a.kcache[l] : a.vcache[l];
                        if (BF16)
                            *reinterpret_cast<uint32_t *>(reinterpret_cast<uint16_t *>(cache) + off) =
                                (uint32_t)f32ToBf16(v0) | ((uint32_t)f32ToBf16(v1) << 16);
                        else
                            *reinterpret_cast<float2 *>(reinterpret_cast<float *>(cache) + off) = make_float2(v0, v1);
                    }
                }
            }
            auxSync(c);  // every aux wave's stores drained
            if (c.at == 0)
                while (gm) {
                    const int g = __builtin_ctzll(gm);
                    gm &= gm - 1;
                    __hip_atomic_fetch_add(a.cnt + g * kCntStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
        }
        PDE_TR(4)
        // ---- attention: workgroup h < nHeads0 owns query head h
        if ((int)blockIdx.x < a.nHeads0) {
            const int head = blockIdx.x, g = head / a.kvMul;
            PDE_TR(5)
            auxAttention<HS, BF16>(c, a, head, l, pos, sl, sAttn, a.cnt + g * kCntStride, st * a.groupExpect[g]);
            auxSignal(c, cntAtt, true);
            PDE_TR(6)
        }
        auxWait(a, cntAtt, 8, st * (unsigned)a.nHeads0, 23, c.lane);
        PDE_TR(7)
        auxStageQ80(c, a.eAttQ, a.eAttS, a.q0, sq, ssc);
        PDE_TR(8)
        barrier();  // wo activations staged
        barrier();  // wo rows in LDS
        PDE_TR(9)
#pragma unroll
        for (int u = 0; u < 2; u++)
            for (int i = c.at; i < re[1][u] - rb[1][u]; i += kPdeAuxThreads)
                st32<true>(a.eWo + rb[1][u] + i, __float_as_uint(res[u * kPdeMaxRes + i]));
        auxSignal(c, cntWo, true);
        PDE_TR(10)
        // ---- w13: x += wo output -> norm -> Q80
        nw = auxNormIssue(c, a, a.rmsFfn[l]);
        auxWait(a, cntWo, 8, st * (unsigned)G, 24, c.lane);
        PDE_TR(11)
        auxResNorm(c, a, xs, a.eWo, false, nw, sq, ssc);
        PDE_TR(12)
        barrier();  // w13 activations staged
        barrier();  // w13 rows in LDS
        PDE_TR(13)
        // SwiGLU of the row pairs (w1, w3 interleaved), Q80 blocks of 32 hidden units
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int h0 = rb[2][u] >> 1, nh = (re[2][u] - rb[2][u]) >> 1;  // whole blocks (host plan)
            for (int i = c.at; i < ((nh + 31) & ~31); i += kPdeAuxThreads) {
                float hv = 0.f;
                if (i < nh) {
                    const float g1 = res[u * kPdeMaxRes + 2 * i], g3 = res[u * kPdeMaxRes + 2 * i + 1];
                    hv = (a.act == 1 ? g1 / (1.0f + __expf(-g1))
                                     : 0.5f * g1 * (1.0f + tanhf(0.79788456080286535588f * g1 * (1.0f + 0.044715f * g1 * g1)))) *
                         g3;
                }
                q80StoreWT(hv, a.eHQ, a.eHS, h0 + i);
            }
        }
        auxSignal(c, cntH, true);
        PDE_TR(14)
        auxWait(a, cntH, 8, st * (unsigned)G, 25, c.lane);
        PDE_TR(15)
        auxStageQ80(c, a.eHQ, a.eHS, a.hidden, sq, ssc);
        PDE_TR(16)
        barrier();  // w2 activations staged
        barrier();  // w2 rows in LDS
        PDE_TR(17)
#pragma unroll
        for (int u = 0; u < 2; u++)
            for (int i = c.at; i < re[3][u] - rb[3][u]; i += kPdeAuxThreads)
                st32<true>(a.eW2 + rb[3][u] + i, __float_as_uint(res[u * kPdeMaxRes + i]));
        auxSignal(c, cntW2, true);
        PDE_TR(18)
#undef PDE_TR
    }
    if (tr && c.at < 8) tr[20 + c.at] = reinterpret_cast<const unsigned long long *>(misc + 16)[c.at];  // ring stamps
    if (tr && c.at == 0) tr[31] = (unsigned long long)xccId();
    // final residual for the logits GEMV (workgroup 0)
    if (blockIdx.x == 0) {
        auxWait(a, cntW2, 8, stepOf(a.nLayers - 1) * (unsigned)G, 26, c.lane);
        float *tmp = reinterpret_cast<float *>(sq);  // the activation image is free now
        auxCopyWT(c, a.eW2, tmp, a.dim * 4);
        auxSync(c);
        for (int i = c.at; i < a.dim; i += kPdeAuxThreads) a.xOut[i] = xs[i] + tmp[i];
    }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
int pdeRingDepth() {
    static const int v = [] {
        const char *e = std::getenv("DL_PDE_RING");
        const int d = e && *e ? std::atoi(e) : 8;
        return d == 4 || d == 6 || d == 8 || d == 12 ? d : 8;
    }();
    return v;
}

template <int D>
static const void *pdeFnD(int hs, bool bf16) {
    if (hs == 128) return bf16 ? (const void *)pdeKernel<128, true, D> : (const void *)pdeKernel<128, false, D>;
    if (hs == 64) return bf16 ? (const void *)pdeKernel<64, true, D> : (const void *)pdeKernel<64, false, D>;
    return nullptr;
}

static const void *pdeFn(int hs, bool bf16) {
    switch (pdeRingDepth()) {
        case 4: return pdeFnD<4>(hs, bf16);
        case 6: return pdeFnD<6>(hs, bf16);
        case 12: return pdeFnD<12>(hs, bf16);
        default: return pdeFnD<8>(hs, bf16);
    }
}

size_t pdeLdsBytes(int dim, int hidden, int q0, int nLayers) {
    return pdeLayout(dim, std::max(std::max(dim, hidden), q0), 4 * nLayers).total;
}

int pdeGrid(int dim, int hidden, int q0, int hs, int nLayers, bool bf16) {
    const void *fn = pdeFn(hs, bf16);
    if (!fn) return 0;
    const size_t lds = pdeLdsBytes(dim, hidden, q0, nLayers);
    if (lds > 160 * 1024) return 0;
    if (lds > 65536) allowLds(fn, lds);
    int dev = 0, cus = 0, perCu = 0;
    DL_HIP(hipGetDevice(&dev));
    DL_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, fn, kPdeThreads, lds) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return perCu >= 1 ? cus : 0;  // one workgroup per CU (the ring's registers leave room for no second)
}

PdePlan pdePlan(const int rows[4], const int n[4], int hidden, int grid) {
    PdePlan p;
    const int V = 2 * grid;
    long long steps[4], passes[4];
    for (int m = 0; m < 4; m++) {
        p.K[m] = ((n[m] >> 5) + 63) / 64;
        passes[m] = (rows[m] + 7) / 8;
        steps[m] = passes[m] * p.K[m];
    }
    p.passStart.assign((size_t)4 * (V + 1), 0);
    // w13 first, in whole Q80 blocks of 32 hidden units (8 passes): spread evenly over the VWGs
    const long long blocks = hidden / 32;
    std::vector<long long> w13v(V, 0);
    for (int v = 0; v <= V; v++) {
        const long long bStart = blocks * v / V;
        p.passStart[2 * (V + 1) + v] = (int)(bStart * 8);
        if (v < V) w13v[v] = (blocks * (v + 1) / V - bStart) * 8 * p.K[2];
    }
    // the other matrices fill each VWG up to the mean total (quota-weighted contiguous split)
    const long long total = steps[0] + steps[1] + steps[2] + steps[3];
    const double target = (double)total / V;
    std::vector<double> quota(V), cum(V + 1, 0.0);
    for (int v = 0; v < V; v++) {
        quota[v] = std::max(0.0, target - (double)w13v[v]);
        cum[v + 1] = cum[v] + quota[v];
    }
    for (int m : {0, 1, 3}) {
        for (int v = 0; v <= V; v++) {
            const double f = cum[V] > 0 ? cum[v] / cum[V] : (double)v / V;
            p.passStart[m * (V + 1) + v] = (int)std::llround(f * (double)passes[m]);
        }
        p.passStart[m * (V + 1) + V] = (int)passes[m];
    }
    return p;
}

void launchPde(const PdeArgs &a, int grid, hipStream_t s) {
    const void *fn = pdeFn(a.hs, a.kvBf16 != 0);
    if (!fn) throw Error("launchPde: unsupported head size");
    const size_t lds = pdeLdsBytes(a.dim, a.hidden, a.q0, a.nLayers);
    if (lds > 65536) allowLds(fn, lds);
    PdeArgs args = a;
    void *kargs[] = {&args};
    DL_HIP(hipLaunchKernel(fn, dim3(grid), dim3(kPdeThreads), kargs, lds, s));
}

std::vector<unsigned> pdeGroupExpect(const std::vector<int> &passStart, int grid, int rowsQkv, int q0, int kv0, int hs,
                                     int kvMul, int nKv) {
    std::vector<unsigned> out(nKv, 0u);
    const int V = 2 * grid;
    for (int b = 0; b < grid; b++) {
        unsigned long long m = 0ull;
        for (int u = 0; u < 2; u++) {
            const int r0 = passStart[2 * b + u] * 8, r1 = std::min(passStart[2 * b + u + 1] * 8, rowsQkv);
            if (r1 > r0) m |= qkvGroupMask(r0, r1, q0, kv0, hs, kvMul);
        }
        for (int g = 0; g < nKv; g++)
            if (m >> g & 1ull) out[g]++;
    }
    (void)V;
    return out;
}

// preloadModules(): one kernel of this translation unit's code object
const void *pdeModuleKernel() { return pdeFn(128, true); }

}  // namespace hipk
}  // namespace dl
