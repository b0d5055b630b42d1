// Device-side building blocks of the decode path, part 2: the Q40 register-ring GEMV body shared
// by the standalone GEMV kernels (gemv_inst.h) and the fused attention block (attn_block_inst.h),
// with the in-launch hand-off state (BlockSync). Included through decode_dev.h.
#pragma once

#include "decode_common.h"

namespace dl {
namespace hipk {

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
#ifndef DL_GEMV_RING
// 4 slots: same-box A/B of whole builds (profiles/r5_decode_profile.md): TP1 decode 1.308-1.314 vs
// 1.371-1.382 ms/token at 8 (fewer ring VGPRs, more waves per SIMD), long context 1.534-1.553 vs
// 1.60-1.62; 2 / 3 / 5 / 6 / 12 slower at TP1 (2 is ahead only on a TP8 rank's small shards)
#define DL_GEMV_RING 4
#endif
static constexpr int kRing = DL_GEMV_RING;

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>): ring slots addressed by
// compile-time indices (fixed registers) however large the body (the compiler may decline to
// unroll a loop, which would index the ring dynamically and spill it).
template <int I, int N, typename F>
__device__ __forceinline__ void staticForImpl(F &f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        staticForImpl<I + 1, N>(f);
    }
}
template <int N, typename F>
__device__ __forceinline__ void staticFor(F &&f) {
    staticForImpl<0, N>(f);
}
#ifndef DL_GEMV_KE
// 4: same-box A/B of whole builds (profiles/r5_decode_profile.md): TP1 decode 1.386 vs 1.397
// ms/token at 2, TP8 rank 0.965 vs 0.984; 1, 6 and 8 slower (6 and 8 at long context too)
#define DL_GEMV_KE 4
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

// attn_dev.h (included after this header): the decode attention task, used by PRO_ATTN
template <int HG, int HS, int AT>
__host__ __device__ constexpr int attnLocalOut();
template <int HG, int HS, bool BF16, int AT, bool SYNC = false, bool LOCAL = false>
__device__ __forceinline__ bool attnTask(const AttnArgs &a, int b, int hgIdx, int c, char *smem,
                                         const BlockSync *bs = nullptr, unsigned long long *trace = nullptr);

template <int L, int B, int PRO, int EPI, int MODE = GEMV_PLAIN, int AHG = 1, bool ABF16 = false>
__device__ __forceinline__ void gemvQ40Body(const GemvArgs &a, const int blk, char *smem, const BlockSync *bs = nullptr,
                                            const AttnArgs *at = nullptr) {
    constexpr int RG = 2, NG = kThreads / L, RP = NG * RG, D = kRing;
    const int n = a.n, nb = n >> 5, K = (nb + L - 1) / L, P = a.passes, T = P * K;
    const int R = RP * P;
    const GemvLds lay = gemvLayout(n, B, true, R, PRO_RESNORM);
    float *scratch = reinterpret_cast<float *>(smem + lay.scratch);
    float *hbuf = reinterpret_cast<float *>(smem + lay.hbuf);
    int8_t *sq = reinterpret_cast<int8_t *>(smem + lay.act);
    float2 *ssc = reinterpret_cast<float2 *>(smem + lay.sc);
    float *res = reinterpret_cast<float *>(smem + lay.res);  // partial rows held for the TP exchange
    constexpr bool tpx = EPI == EPI_STORE_TP || EPI == EPI_RESQ_TP;
    constexpr bool pren = PRO == PRO_PRENORM;  // pre-normalized Q80 input (copy + 1 / rms)
    static_assert(!pren || B == 1, "PRO_PRENORM: one row");
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
        uint32_t spv = 0u;  // PRO_PRENORM: the producer's partial sum of squares
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
            if constexpr (pren) {  // this thread's partial sum of squares (nSsp <= 256: one each)
                const float *src = a.sspIn + min(tid, a.nSsp - 1);
                asm volatile("global_load_dword %0, %1, off" : "=v"(spv) : "v"(src));
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
            if constexpr (pren) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(spv) : "i"(3 * KE));
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
            if (MODE == GEMV_PLAIN && a.trace) tWaited = wall_clock64();  // norm reduced (plain GEMVs)
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
            float inv = 1.0f;
            if constexpr (pren) {  // 1 / rms from the producer's partials, summed in workgroup order
                const float ss = blockSum<kThreads>(tid < a.nSsp ? __uint_as_float(spv) : 0.f, scratch);
                inv = 1.0f / sqrtf(ss / (float)n + a.eps);
            }
#pragma unroll
            for (int k = 0; k < PK; k++)
                if (tid + k * kThreads < n16) reinterpret_cast<u32x4 *>(sq)[tid + k * kThreads] = eq[k];
#pragma unroll
            for (int k = 0; k < PS; k++)
                if (tid + k * kThreads < nb) {
                    u32x2 e = es[k];
                    // the block's scale of x * normW / rms: f16(d' / rms), as the norm prologue's
                    // f16(amax(x * normW / rms) / 127) up to the last ulp (stageChunk)
                    if constexpr (pren) e.x = __float_as_uint(roundF16(__uint_as_float(e.x) * inv));
                    reinterpret_cast<u32x2 *>(ssc)[tid + k * kThreads] = e;
                }
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
            if constexpr (PRO == PRO_RESNORM) stageF32WT<B>(a, sq, ssc);  // f32 rows (FFN block, skinny w13)
            else stageQ80<B, true>(a, sq, ssc);
        } else if constexpr (PRO == PRO_RESNORM)
            resNormPrologue<B, true>(a, scratch, sq, ssc, nullptr);
        else {
            stageQ80<B>(a, sq, ssc);
        }
        waitAll();
        if (a.trace) tReady = wall_clock64();
    };

    // PRO_ATTN: the rank's attention heads, one KV group at a time (AHG query heads sharing its
    // keys), computed into this workgroup's LDS from the L2-resident cache and quantized to the Q80
    // image the main loop reads (32-lane groups = one block, the attention kernel's own rounding);
    // then the weight ring. The ring is NOT issued first: under the attention's register pressure
    // the compiler moved pending ring registers to AGPRs before their s_waitcnt (stale copies,
    // scripts/check_isa.py --hazards), so no inline-asm load is in flight during the attention.
    auto attnPath = [&]() {
      if constexpr (PRO == PRO_ATTN && B == 1) {
        char *asmem = smem + alignUp(lay.total, 16);
        const float *o = reinterpret_cast<const float *>(asmem) + attnLocalOut<AHG, 128, kThreads>();
        const int groups = at->nHeads0 / AHG;
        for (int g = 0; g < groups; g++) {
            attnTask<AHG, 128, ABF16, kThreads, false, true>(*at, 0, g, 0, asmem);
            for (int i = tid; i < AHG * 128; i += kThreads) {  // AHG * 128 is a multiple of 256
                const float v = o[i];
                const float amax = groupMax<32>(fabsf(v));
                const float d = amax / 127.0f;
                const float id = d != 0.f ? 1.0f / d : 0.f;
                int q = (int)rintf(v * id);
                q = q > 127 ? 127 : (q < -127 ? -127 : q);
                const int col = g * AHG * 128 + i;
                sq[col] = (int8_t)q;
                const float qs = groupSum<32>((float)q);
                if ((i & 31) == 0) ssc[col >> 5] = make_float2(roundF16(d), qs);
            }
            __syncthreads();  // the next group's task reuses the scratch
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < D; s++) {
            issue(w[s], dh[s]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (a.trace) tReady = wall_clock64();
      }
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
                if constexpr (EPI == EPI_STORE_TP || EPI == EPI_RESQ_TP || EPI == EPI_ARGMAX) {
                    res[b * R + (r0 - rowBase)] = v0;
                    res[b * R + (r0 - rowBase) + 1] = v1;
                } else if constexpr (EPI == EPI_STORE) {
                    float *o = a.out + (size_t)b * a.ldOut + r0;
                    o[0] = v0;
                    if (r0 + 1 < a.rows) o[1] = v1;
                } else if constexpr (EPI == EPI_ACT) {
                    float *o = a.out + (size_t)b * a.ldOut + (r0 >> 1);
                    if constexpr (MODE == GEMV_PRODUCER)  // read by the FFN block's w2 role in this launch
                        __hip_atomic_store(o, gateAct(a, v0) * v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else
                        *o = gateAct(a, v0) * v1;
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
    auto fullSlot = [&](auto sTag) {
        constexpr int s = decltype(sTag)::value;
        asm volatile("s_waitcnt vmcnt(%3)" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(dh[s]) : "i"(3 * (D - 1)));
        consume(w[s], dh[s], true);
        if (a.trace && s == 0 && t0 == 0) tFirst = wall_clock64();
        issue(w[s], dh[s]);
        advance();
        __builtin_amdgcn_sched_barrier(0);
    };
    for (; t0 + D < T; t0 += D) staticFor<D>(fullSlot);
    // Last round: no refills; slot s waits for the loads issued after it (slots s+1..kRing-1), so
    // every load has landed when the workgroup ends. (Slots expanded at compile time: the wait
    // count must be an immediate even where the compiler declines to unroll a large body.)
    auto lastSlot = [&](auto sTag) {
        constexpr int s = decltype(sTag)::value;
        asm volatile("s_waitcnt vmcnt(%3)" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(dh[s]) : "i"(3 * (D - 1 - s)));
        if (t0 + s < T) {
            consume(w[s], dh[s], true);
            if (a.trace && s == 0 && t0 == 0) tFirst = wall_clock64();
            advance();
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    staticFor<D>(lastSlot);
    };

    const int unitsPerThread = (PRO != PRO_GLOBAL && PRO != PRO_PRENORM) ? (n + 8 * kThreads - 1) / (8 * kThreads)
                                                                         : (n + 16 * kThreads - 1) / (16 * kThreads);
    static_assert(MODE != GEMV_CONSUMER || PRO == PRO_GLOBAL || PRO == PRO_RESNORM,
                  "a consumer GEMV reads Q80 activations (or un-normalized f32 rows: PRO_RESNORM, no norm)");
    if constexpr (PRO == PRO_ATTN) {
        attnPath();
        mainLoop();
    } else if constexpr (MODE == GEMV_CONSUMER) {
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
    const unsigned long long tLoop = a.trace ? wall_clock64() : 0ull;  // main loop done (this wave)
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
        // exchange span (DL_SYNC_MEASURE=2, a.tp.span set): this workgroup's tail, first push to
        // last summed store, raised into the exchange's slot (the longest tail of the launch)
        const unsigned long long xs = a.tp.span ? wall_clock64() : 0ull;
        ResqPre rpf;
        if constexpr (EPI == EPI_RESQ_TP) rpf = resqPrefetch(a, R, rowBase);
        tpDispatch(a.tp.world, [&](auto wm) {
            constexpr int WM = decltype(wm)::value;
            if constexpr (EPI == EPI_RESQ_TP) {  // sums back into res[], then the residual + norm tail
                static_assert(B == 1, "EPI_RESQ_TP: one row");
                if (a.tp.q80) tpExchangeQ80Row<WM, true>(a, res, R, rowBase);
                else tpExchangeF32<1, WM, true>(a, res, R, rowBase);
            } else if (a.tp.q80 && B == 1) {
                tpExchangeQ80Row<WM>(a, res, R, rowBase);
            } else if (a.tp.q80) {
                tpExchangeQ80<B, WM>(a, res, R, rowBase, reinterpret_cast<char *>(sq));
            } else {
                tpExchangeF32<B, WM>(a, res, R, rowBase);
            }
        });
        if constexpr (EPI == EPI_RESQ_TP) {
            __syncthreads();
            resqTail(a, res, R, rowBase, blk, scratch, rpf);
        }
        if (a.tp.span) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0)
                __hip_atomic_fetch_max(a.tp.span, (unsigned)(wall_clock64() - xs), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if constexpr (EPI == EPI_ARGMAX) {  // the row's argmax instead of its logits (ArgmaxTail)
        static_assert(B == 1, "EPI_ARGMAX: one row");
        __syncthreads();
        float *sv = scratch;
        int *si = reinterpret_cast<int *>(scratch + 8);
        int *last = reinterpret_cast<int *>(scratch + 16);
        float bv = -INFINITY;
        int bi = 0x7fffffff;
        for (int i = tid; i < R; i += kThreads)
            if (rowBase + i < a.rows) argBetter(bv, bi, res[i], rowBase + i);
        blockArgmax(bv, bi, sv, si);
        // fence-free hand-off (as argmaxKernel): agent-scope stores of the partial, drained, then counted
        if (tid == 0) {
            __hip_atomic_store(a.am.partV + blk, bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.am.partI + blk, bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const int old = __hip_atomic_fetch_add(a.am.counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *last = old == (int)gridDim.x - 1;
        }
        __syncthreads();
        if (*last) {
            if (tid == 0) __hip_atomic_store(a.am.counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bv = -INFINITY;
            bi = 0x7fffffff;
            for (int i = tid; i < (int)gridDim.x; i += kThreads)
                argBetter(bv, bi, __hip_atomic_load(a.am.partV + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                          __hip_atomic_load(a.am.partI + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            blockArgmax(bv, bi, sv, si);
            if (tid == 0) {
                bi += a.am.vocabStart;
                if (a.tp.world > 1)
                    tpDispatch(a.tp.world, [&](auto wm) { tpArgmaxPick<decltype(wm)::value>(a.tp, 0, bv, bi); });
                a.am.ids[0] = bi;
                if (a.am.tokens) {  // chained decode: feed the token back
                    const int p = a.am.pos[0];
                    a.am.hist[p] = bi;
                    a.am.tokens[0] = bi;
                    a.am.pos[0] = p + 1;
                }
            }
        }
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
            t[7] = tLoop;
        }
    }
}

}  // namespace hipk
}  // namespace dl
