// Device-side building blocks of the decode path, part 3: the decode attention task (VALU, one
// row x head group x sequence chunk), its output writers and the split combine (attnFinish),
// shared by the attention kernels and the fused attention block. Included through decode_dev.h.
#pragma once

#include "gemv_dev.h"

namespace dl {
namespace hipk {

#ifndef DL_ATTN_TU_F32_BLOCK
#define DL_ATTN_TU_F32_BLOCK 7
#endif
#ifndef DL_ATTN_TU_F32
#define DL_ATTN_TU_F32 4  // f32 caches outside the block: keys per 16-lane group per round
#endif
#ifndef DL_ATTN_HOIST_SYNC
#define DL_ATTN_HOIST_SYNC 0  // fused block: per-key lookups measured 0.3-0.5 % faster (raw/r6_kvload_ab.txt)
#endif
#ifndef DL_ATTN_TU_BF16_BLOCK
#define DL_ATTN_TU_BF16_BLOCK 8
#endif

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
// the partial and count arrivals; the last workgroup combines all chunks, with 8 chunks' partial
// outputs and (max, sum) pairs in flight per thread (a serial loop over the chunks costs one
// cross-XCD round trip per chunk: ~30 us at 32 chunks). `scratch` is not used (kept for callers).
template <int HG, int HS, int AT, bool WT = false>
__device__ __forceinline__ bool attnFinish(const AttnArgs &a, int b, int hgIdx, int c, int nSplit, float *redL,
                                           float *mlL, int *flagL, float *scratch) {
    const int tid = threadIdx.x, head0 = hgIdx * HG;
    (void)scratch;
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
    // Weighted sum of the chunks' partial outputs in ONE memory round trip: (item = 4 dims of one
    // head) x (part = a strided subset of the chunks) per thread, the `parts` threads of an item
    // adjacent lanes. Every thread loads its chunks' partial outputs AND their (max, sum) pairs at
    // once (16-B / 8-B coherence-point loads, sc1 like the atomic accesses above), folds them with an
    // online softmax rescale in chunk order, then a fixed butterfly merges the parts: deterministic,
    // and every item of a head derives the same denominator from the same chunks in the same order.
    // (A separate (max, sum) pass with a serial per-head weight loop cost an extra round trip and
    // ~7 us per long-context combine: trace_attention.py.)
    constexpr int U = 8, ITEMS = HG * (HS / 4), PARTS = ITEMS >= AT ? 1 : AT / ITEMS;
    for (int base = 0; base < ITEMS * PARTS; base += AT) {
        const int t = base + tid, item = t / PARTS, part = t % PARTS;
        const int h = min(item, ITEMS - 1) / (HS / 4), d = (min(item, ITEMS - 1) % (HS / 4)) * 4;
        const float *po = a.partO + (pbase + (size_t)h * G) * HS + d;
        const float *pml = a.partML + (pbase + (size_t)h * G) * 2;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        float M = -INFINITY, Ls = 0.f;
        for (int c0 = part; c0 < nSplit; c0 += U * PARTS) {
            f32x4 v[U];
            u32x2 ml[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int cc = min(c0 + u * PARTS, nSplit - 1);
                asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v[u]) : "v"(po + (size_t)cc * HS));
                asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=v"(ml[u]) : "v"(pml + (size_t)cc * 2));
            }
#pragma unroll
            for (int u = 0; u < U; u++) {  // each wait pins its own loads' registers (no early use)
                asm volatile("s_waitcnt vmcnt(%2)" : "+v"(v[u]), "+v"(ml[u]) : "i"(2 * (U - 1 - u)) : "memory");
                if (c0 + u * PARTS < nSplit) {
                    const float mc = __uint_as_float(ml[u].x), lc = __uint_as_float(ml[u].y);
                    const float Mn = fmaxf(M, mc);
                    const float so = M == -INFINITY ? 0.f : __expf(M - Mn), w = mc == -INFINITY ? 0.f : __expf(mc - Mn);
                    acc = acc * so + w * v[u];
                    Ls = Ls * so + w * lc;
                    M = Mn;
                }
            }
        }
#pragma unroll
        for (int off = 1; off < PARTS; off <<= 1) {
            const float M2 = __shfl_xor(M, off), L2 = __shfl_xor(Ls, off);
            f32x4 a2;
#pragma unroll
            for (int j = 0; j < 4; j++) a2[j] = __shfl_xor(acc[j], off);
            const float Mn = fmaxf(M, M2);
            const float s1 = M == -INFINITY ? 0.f : __expf(M - Mn), s2 = M2 == -INFINITY ? 0.f : __expf(M2 - Mn);
            acc = acc * s1 + a2 * s2;
            Ls = Ls * s1 + L2 * s2;
            M = Mn;
        }
        if (part == 0 && item < ITEMS) {
            const float il = 1.0f / Ls;
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
// LOCAL (the wo GEMV's attention prologue, PRO_ATTN): the whole context in one chunk, nothing
// written to global memory: the normalised output of the HG heads is left in LDS at attnLocalOut.
template <int HG, int HS, int AT>
__host__ __device__ constexpr int attnLocalOut() {  // float offset of the LOCAL output in the task's LDS
    return 2 * (AT / 64) * HG + (AT / 64) * HG * HS;
}
template <int HG, int HS, int AT>
__host__ __device__ constexpr int attnTaskLdsBytes() {
    return (int)sizeof(float) * (attnLocalOut<HG, HS, AT>() + HG * HS + 2 * HG) + 16;
}
template <int HG, int HS, bool BF16, int AT, bool SYNC, bool LOCAL>
__device__ __forceinline__ bool attnTask(const AttnArgs &a, int b, int hgIdx, int c, char *smem,
                                         const BlockSync *bs, unsigned long long *trace) {
    constexpr int NW = AT / 64, NG = AT / 16;
    constexpr int DPL = HS / 16;           // dims per lane: 16 lanes cover one position's head vector
    // keys per group loaded before any is consumed. The fused block (SYNC) issues its first round
    // before waiting for the qkv workgroups: 7 keys per group there for f32 caches (112 keys per
    // round instead of 64: f32-KV decode 1.322 -> 1.291 ms/token, same box; 8 keys took the block
    // kernel to 178 VGPRs, 2 waves per SIMD, and off co-residency), bf16 stays at 8 (12 measured
    // 1.357 vs 1.289 ms/token): profiles/r6_decode.md
    constexpr int TU = BF16 ? (SYNC ? DL_ATTN_TU_BF16_BLOCK : 8) : (SYNC ? DL_ATTN_TU_F32_BLOCK : DL_ATTN_TU_F32);
    constexpr int RW = BF16 ? DPL / 2 : DPL;  // 32-bit words per lane per key (packed bf16 pairs)
    const int pos = a.pos[b], sl = a.slot[b];
    const int len = pos + 1;
    int nSplit, ch;
    if constexpr (LOCAL) {
        nSplit = 1;
        ch = len;
    } else {
        attnSplit(len, a.splitGrid, nSplit, ch, a.chunkMin, a.shortLen);
    }
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
        // the round's cache blocks first (pool pages of a paged cache, else the slot): a page-table
        // load inside the key loop put a full vmcnt(0) drain at its join before every key, so
        // the round's TU keys went out one memory round trip after another
        size_t blk[TU];
#pragma unroll
        for (int u = 0; u < TU; u++) {
            const int t = min(tb + u * NG, t1 - 1);
            if constexpr (SYNC && !DL_ATTN_HOIST_SYNC) blk[u] = 0;  // per key below (A/B switch)
            else blk[u] = a.kvMap.table ? kvPageOf(a.kvMap, sl, t) : (size_t)sl;
        }
#pragma unroll
        for (int u = 0; u < TU; u++) {
            const int t = min(tb + u * NG, t1 - 1);  // clamped: no divergent loads
            const bool cur = SYNC && t == pos;
            if ((phase == 1 && cur) || (phase == 2 && !cur)) continue;
            const size_t off = (SYNC && !DL_ATTN_HOIST_SYNC)
                                   ? kvOff(a.kvMap, a.seqLen, a.kv0 / HS, HS, sl, t, kvh) + l16 * DPL
                                   : kvOffAt(a.kvMap, a.seqLen, a.kv0 / HS, HS, blk[u], t, kvh) + l16 * DPL;
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
    // the first round of keys goes out before the query loads (the keys do not depend on q, so
    // both round trips overlap instead of following each other)
    if (tb < t1) {
        loadRound(tb, 1);
        prefetched = true;
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (SYNC) tWaited = blockWait(bs->qkvCnt + kvh * kCntStride, bs->step * bs->qkvExpect[kvh], *bs, 2);
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
    // in flight at once (NG*TU keys per memory round trip)
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
    if constexpr (LOCAL) {  // one chunk: normalise in place, the caller reads redL
        for (int i = tid; i < HG * HS; i += AT) redL[i] = redL[i] / mlL[(i / HS) * 2 + 1];
        __syncthreads();
        return true;
    }
    return attnFinish<HG, HS, AT, SYNC>(a, b, hgIdx, c, nSplit, redL, mlL, flagL, oW);
}

}  // namespace hipk
}  // namespace dl
