// Device building blocks shared by the batched MFMA GEMMs (gemm.hip: 16..128-token tiles of 64
// rows; gemm_wide.hip: 128 x 128 tiles for prefill chunks): Q40 nibble dequantization to f16,
// global -> LDS copies, the range-safe f16 hand-off of EPI_RES and the fused epilogues.
#pragma once

#include "decode_dev.h"

namespace dl {
namespace hipk {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
static constexpr int kGemmRows = 64;  // weight rows per narrow-GEMM workgroup (4 waves x 16)

// 8 nibbles (lo or hi of 8 bytes) -> 8 f16 values (q - 8) * d. Low nibbles: f16 bits 0x64 | q =
// 1024 + q; high nibbles stay in place (byte & 0xF0 = 16 q) under exponent byte 0x54, whose ulp
// is 1/16: 64 + q. Subtracting 1032 / 72 gives q - 8 exactly; one rounding in the multiply by d.
// The mask, magic and offset depend on nibHi only (per lane, loop-invariant): no per-lane shift.
__device__ __forceinline__ half8 dequantQ40x8(u32x2 wv, int nibHi, uint32_t d16) {
    const uint32_t mask = nibHi ? 0xF0F0F0F0u : 0x0F0F0F0Fu;
    const uint32_t magic = nibHi ? 0x54545454u : 0x64646464u;
    const uint32_t lo = wv.x & mask;
    const uint32_t hi = wv.y & mask;
    const uint32_t p0 = __builtin_amdgcn_perm(magic, lo, 0x07010700u);
    const uint32_t p1 = __builtin_amdgcn_perm(magic, lo, 0x07030702u);
    const uint32_t p2 = __builtin_amdgcn_perm(magic, hi, 0x07010700u);
    const uint32_t p3 = __builtin_amdgcn_perm(magic, hi, 0x07030702u);
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const _Float16 d = __builtin_bit_cast(_Float16, (uint16_t)d16);
    const h2 dd = {d, d};
    const _Float16 o = nibHi ? (_Float16)-72.0f : (_Float16)-1032.0f;
    const h2 off = {o, o};
    const h2 r0 = (__builtin_bit_cast(h2, p0) + off) * dd;
    const h2 r1 = (__builtin_bit_cast(h2, p1) + off) * dd;
    const h2 r2 = (__builtin_bit_cast(h2, p2) + off) * dd;
    const h2 r3 = (__builtin_bit_cast(h2, p3) + off) * dd;
    half8 out;
    out[0] = r0[0]; out[1] = r0[1]; out[2] = r1[0]; out[3] = r1[1];
    out[4] = r2[0]; out[5] = r2[1]; out[6] = r3[0]; out[7] = r3[1];
    return out;
}

// one 16-B global -> LDS copy per lane; `lds` = this wave's base (lane l lands at lds + 16 l).
// NT: non-temporal (streamed once: weights, KV), as the GEMV ring's loads (cache policy nt = 2)
template <bool NT = false>
__device__ __forceinline__ void glds16(const void *g, void *lds) {
    __builtin_amdgcn_global_load_lds(const_cast<void *>(g), reinterpret_cast<__attribute__((address_space(3))) void *>(
                                         reinterpret_cast<uintptr_t>(lds)), 16, 0, NT ? 2 : 0);
}
__device__ __forceinline__ void glds4(const void *g, void *lds) {
    __builtin_amdgcn_global_load_lds(const_cast<void *>(g), reinterpret_cast<__attribute__((address_space(3))) void *>(
                                         reinterpret_cast<uintptr_t>(lds)), 4, 0, 0);
}

// EPI_RES hand-off scale (power of two: exact) and the f16 store that saturates instead of
// overflowing to inf.
static constexpr float kResXScale = 1.0f / 32.0f;
__device__ __forceinline__ _Float16 satF16(float v) { return (_Float16)fminf(fmaxf(v, -65504.f), 65504.f); }

// Fence-free cross-workgroup hand-off (split-K partials), one place for the pattern:
// * producer: every handed-off value stored with wtStore (agent-scope relaxed atomic store =
//   global_store ... sc1, performed at the device coherence point, never left dirty in one XCD's
//   L2), then splitArrive: s_waitcnt vmcnt(0) (all of this wave's stores performed), a workgroup
//   barrier, one relaxed agent-scope fetch_add on the tile counter;
// * consumer (the last arriver): loads with wtLoad (global_load ... sc1, served from the coherence
//   point, never from a stale L1/L2 line).
// This is the "Valid forms" alternative to a release/acquire pair in MI355X_MICROARCH.md
// (Correctness boundaries: inter-workgroup visibility). The release/acquire fences compile to a
// whole-L2 writeback / invalidate (buffer_wbl2 sc1 / buffer_inv sc1) on gfx950, ~28 us per split
// level on w13 (profiles/r2_splitk_fences.md). The asm vmcnt(0) carries a "memory" clobber so the
// compiler cannot move the stores below it; tests/test_gpu_ops.py::test_gemm_split_determinism
// pins the result of many splits across XCDs bitwise against one split.
__device__ __forceinline__ void wtStore(float *p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float wtLoad(const float *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// All S workgroups of a tile call this after their wtStores; true in the last arriver only (which
// also re-arms the counter for the next launch). flag: one int of LDS.
__device__ __forceinline__ bool splitArrive(int *counter, int S, int *flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = old == S - 1;
    }
    __syncthreads();
    const bool last = flag[0] != 0;
    if (last && threadIdx.x == 0) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return last;
}
// Sum S partials (P + s * stride, f32x4 units [0, n4)) in split order into dst (LDS; unit i lands
// at dst[(i / rowU) * ldU + i % rowU], a padded row stride): the loads of 4 splits are in flight
// before their adds. Register-lean on purpose: an 8-deep fully unrolled form set the whole
// narrow kernel's VGPR allocation (224-231 at <= 16 tokens: 2 waves per SIMD for the main loop).
__device__ __forceinline__ void splitCombine(const float *P, size_t stride, int S, int n4, f32x4 *dst, int rowU = 1,
                                             int ldU = 1) {
    auto ld = [](const float *q) { return f32x4{wtLoad(q), wtLoad(q + 1), wtLoad(q + 2), wtLoad(q + 3)}; };
#pragma clang loop unroll(disable)
    for (int i = threadIdx.x; i < n4; i += kThreads) {
        f32x4 r = ld(P + 4 * i);
#pragma clang loop unroll(disable)
        for (int s0 = 1; s0 < S; s0 += 4) {
            f32x4 v[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (s0 + j < S) v[j] = ld(P + (size_t)(s0 + j) * stride + 4 * i);
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (s0 + j < S) r += v[j];
        }
        dst[(i / rowU) * ldU + i % rowU] = r;
    }
}

// Tensor-parallel all-reduce of a GEMM output tile in LDS (tile[t * 64 + r]: tokens t < M, rows R0 +
// r of ldOut-wide outputs) through the fused exchange of the decode GEMVs (decode_dev.h
// tpPushCollect: every rank pushes its partials into each peer's receive region as {value, epoch}
// words, polls its own, sums in rank order: bitwise identical on every rank). Exchange element =
// token * ldOut + row, the GEMV's convention, so the per-element epochs stay in step. Q80: every
// rank's partial is quantized once to 32-row blocks (the reference's ZQ wire format, 9 words per
// block), dequantized and summed. The sums overwrite the tile. `lds` = free staging (Q80:
// tpTileQ80Lds bytes). Called by one whole workgroup; ends with a barrier.
__host__ __device__ inline size_t tpTileQ80Lds(int M, int W) {
    const int nEl = M * 64, nBlk = nEl / 32;
    return alignUp((size_t)nEl, 16) + alignUp((size_t)nBlk * 4, 16) + (size_t)W * nBlk * 9 * 4;
}
template <int WM>
__device__ __forceinline__ void tpExchangeTileW(const GemmArgs &ga, float *tile, int R0, char *lds) {
    const TpXchg &x = ga.e.tp;
    const int M = ga.M, nEl = M * 64, W = x.world;
    __syncthreads();
    unsigned waited = 0;
    if (!x.q80) {
        for (int i = threadIdx.x; i < nEl; i += kThreads) {
            const int t = i >> 6, row = R0 + (i & 63);
            if (row >= ga.e.rows) continue;
            const long long el = (long long)t * ga.e.ldOut + row;
            const unsigned e = x.epochs[el] + 1;
            unsigned v[WM];
            tpPushCollect(x, el, e, __float_as_uint(tile[i]), v, waited);
            float s = 0.f;
#pragma unroll
            for (int p = 0; p < WM; p++)
                if (p < W) s += __uint_as_float(v[p]);
            tile[i] = s;
            x.epochs[el] = e;
        }
        tpWaitReport(x, waited);
        __syncthreads();
        return;
    }
    const int nBlk = nEl >> 5;
    int8_t *q8 = reinterpret_cast<int8_t *>(lds);
    uint32_t *dq = reinterpret_cast<uint32_t *>(lds + alignUp((size_t)nEl, 16));
    uint32_t *rv = reinterpret_cast<uint32_t *>(lds + alignUp((size_t)nEl, 16) + alignUp((size_t)nBlk * 4, 16));
    for (int base = 0; base < nEl; base += kThreads) {  // whole 32-lane groups per block: uniform
        const int i = base + threadIdx.x;
        const float v = i < nEl ? tile[i] : 0.f;
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
    auto blockId = [&](int blk, bool &live) -> long long {  // 32-row block of (token, rows)
        const int t = blk >> 1, row = R0 + (blk & 1) * 32;
        live = row < ga.e.rows;
        return ((long long)t * ga.e.ldOut + row) >> 5;
    };
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
    for (int i = threadIdx.x; i < nEl; i += kThreads) {
        const int blk = i >> 5;
        float s = 0.f;
        for (int p = 0; p < W; p++) {
            const uint32_t *bw = rv + (p * nBlk + blk) * 9;
            const float d = __half2float(__ushort_as_half((uint16_t)(bw[8] & 0xFFFFu)));
            const int q = (int)(int8_t)(bw[(i & 31) >> 2] >> (8 * (i & 3)));
            s += (float)q * d;
        }
        tile[i] = s;
    }
    __syncthreads();
}
__device__ __forceinline__ void tpExchangeTile(const GemmArgs &ga, float *tile, int R0, char *lds) {
    tpDispatch(ga.e.tp.world, [&](auto wm) { tpExchangeTileW<decltype(wm)::value>(ga, tile, R0, lds); });
}

// Consumer of a fused residual + norm (ga.ssIn): per-token RMS scale of tokens [t0, t0 + nt) of the
// launch (nt <= 128) from the producer's 64-row tile partials, into rsL[0, nt). TPT threads per
// token each sum a strided slice (independent loads in flight), then one thread per token adds the
// slices in order (deterministic). slL: kThreads floats of scratch. Ends with a barrier.
__device__ __forceinline__ void gemmRowScales(const GemmArgs &ga, int t0, int nt, float *rsL, float *slL) {
    const int tid = threadIdx.x;
    // threads per token summing its partials; a batch-invariant launch (ga.fixed) always uses 2, so
    // the order of the sum does not depend on the launch's token count
    const int TPT = ga.fixed ? 2 : nt <= 16 ? 16 : nt <= 32 ? 8 : nt <= 64 ? 4 : 2;
    const int t = tid / TPT, q = tid % TPT;
    float ssum = 0.f;
    if (t < nt && t0 + t < ga.M) {
#pragma unroll 8
        for (int j = q; j < ga.ssTiles; j += TPT) ssum += ga.ssIn[(size_t)j * ga.ldSS + t0 + t];
    }
    slL[tid] = ssum;
    __syncthreads();
    if (tid < nt) {
        float tot = 0.f;
        for (int i = 0; i < TPT; i++) tot += slL[tid * TPT + i];
        rsL[tid] = (1.0f / kResXScale) / sqrtf(tot / (float)ga.e.n + ga.e.eps);
    }
    __syncthreads();
}

// Fused epilogues of an output tile in LDS: tile[tl * ldT + r] holds tokens tl in [tl0, tl1) (local
// to the tile; launch token = tokBase + tl) and the tile's rows r in [0, 2 * PAIRS) (global row
// R0 + r), processed as row pairs (2k, 2k+1). rsL (indexed tl - tl0): per-token RMS scales of an
// ssIn consumer, else null. EPI_RES writes one sum of squares per 64 rows (32 pairs) and token to
// ssOut[(ssSlot0 + k / 32) * ldSS + t].
template <int EPI, int PAIRS>
__device__ __forceinline__ void gemmEpilogue(const GemmArgs &ga, const float *tile, int ldT, int tl0, int tl1,
                                             int tokBase, int R0, int ssSlot0, const float *rsL) {
    const GemvArgs &a = ga.e;
    // not unrolled: a fully unrolled short trip (<= 16 tokens) hoisted every iteration's loads and
    // set the whole kernel's VGPR allocation (224+ -> 2 waves per SIMD for the main loop too)
#pragma clang loop unroll(disable)
    for (int i = threadIdx.x; i < (tl1 - tl0) * PAIRS; i += kThreads) {
        const int tl = tl0 + i / PAIRS, k = i % PAIRS, r0 = R0 + 2 * k, t = tokBase + tl;
        float v0 = tile[tl * ldT + 2 * k], v1 = tile[tl * ldT + 2 * k + 1];
        if (rsL) {
            v0 *= rsL[tl - tl0];
            v1 *= rsL[tl - tl0];
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
            const float ssq = groupSum<32>(x0 * x0 + x1 * x1);  // 32 pairs = 64 rows of token t, in lane order
            if ((k & 31) == 0 && R0 + 2 * k < a.rows) ga.ssOut[(size_t)(ssSlot0 + (k >> 5)) * ga.ldSS + t] = ssq;
        } else if constexpr (EPI == EPI_STORE) {
            if (r0 < a.rows) a.out[(size_t)t * a.ldOut + r0] = v0;
            if (r0 + 1 < a.rows) a.out[(size_t)t * a.ldOut + r0 + 1] = v1;
        } else if constexpr (EPI == EPI_ACT) {
            if (r0 < a.rows) a.out[(size_t)t * a.ldOut + (r0 >> 1)] = gateAct(a, v0) * v1;
        } else if constexpr (EPI == EPI_ACT_F16) {
            if (r0 < a.rows) ga.outH[(size_t)t * a.ldOut + (r0 >> 1)] = (_Float16)(gateAct(a, v0) * v1);
        } else if constexpr (EPI == EPI_ACT_Q80) {
            const int hBase = (R0 >> 1) + (k & ~31);
            if (hBase >= (a.rows >> 1)) continue;  // whole 32-unit block: uniform per lane group
            const float hv = gateAct(a, v0) * v1;
            const float amax = groupMax<32>(fabsf(hv));
            const float d = amax / 127.0f;
            const float id = d != 0.f ? 1.0f / d : 0.f;
            int q = (int)rintf(hv * id);
            q = q > 127 ? 127 : (q < -127 ? -127 : q);
            a.oq[(size_t)t * a.ldOut + hBase + (k & 31)] = (int8_t)q;
            const float qsum = groupSum<32>((float)q);
            if ((k & 31) == 0) a.os[(size_t)t * (a.ldOut >> 5) + (hBase >> 5)] = make_float2(roundF16(d), qsum);
        } else {
            if (r0 < a.rows)
                qkvPairStore(a, r0, v0, v1, a.rope + (size_t)a.pos[t] * (a.hs >> 1), a.pos[t], a.slot[t],
                             a.out + (size_t)t * a.ldOut);
        }
    }
}

// Split-K combine and fused epilogues shared by the batched GEMMs (Q40 and f32): `acc` holds this
// lane's C fragments (weight row (local) wave*16 + col, token t*16 + h*4 + i); `smem` must hold
// MP x 64 floats and is free (all K-loop LDS reads retired behind a barrier); `flag` one int.
// tileIdx / tiles: this 64-row tile and the launch's tile count (split-K partial slots, counters).
// Diagnostics (ga.e.trace): 8 u64 per workgroup (blockIdx.y * gridDim.x + blockIdx.x):
// [0] entry, [1] first stage / ring slot landed, [2] K loop done, [3] split hand-off done (the
// combining workgroup: partials summed; the others: arrival counted), [4] exit, [5] XCC id,
// [6] 1 if this workgroup combined the tile (thread 0's view; s_memrealtime, 100 MHz).
__device__ __forceinline__ void gemmTrace(const GemmArgs &ga, const unsigned long long (&t)[4], bool combined) {
    if (!ga.e.trace || threadIdx.x != 0) return;
    unsigned long long *o = ga.e.trace + 8 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x);
    o[0] = t[0];
    o[1] = t[1];
    o[2] = t[2];
    o[3] = t[3];
    o[4] = wall_clock64();
    o[5] = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;
    o[6] = combined ? 1ull : 0ull;
}

template <int MT, int EPI>
__device__ __forceinline__ void gemmFinish(const GemmArgs &ga, const f32x4 (&acc)[MT], char *smem, int *flag,
                                           int tileIdx, int tiles, unsigned long long t0 = 0,
                                           unsigned long long t1 = 0, unsigned long long t2 = 0) {
    unsigned long long tr[4] = {t0, t1, t2, 0ull};
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
            for (int i = 0; i < 4; i++) wtStore(part + (t * 16 + h * 4 + i) * kGemmRows + rl, acc[t][i]);
        if (!splitArrive(ga.counters + tileIdx, S, flag)) {
            if (ga.e.trace) {
                tr[3] = wall_clock64();
                gemmTrace(ga, tr, false);
            }
            return;
        }
        // combine in split order (deterministic): this tail runs on one workgroup per tile after
        // the others finished
        splitCombine(ga.part + (size_t)tileIdx * MP * kGemmRows, (size_t)tiles * MP * kGemmRows, S,
                     MP * kGemmRows / 4, reinterpret_cast<f32x4 *>(tile));
    }
    if (ga.e.trace) tr[3] = wall_clock64();
    // tensor parallel: the tile's partial sums all-reduced over the ranks in place (staging after
    // the [MP][64] tile; the host checked that the launch's LDS holds it)
    if (ga.tpx) tpExchangeTile(ga, tile, R0, smem + (size_t)MP * kGemmRows * 4);
    // consumer of a fused residual + norm: per-token RMS scale from the producer's tile partials
    float *rsL = reinterpret_cast<float *>(flag + 4);  // [128] + [256] scratch
    if (ga.ssIn) gemmRowScales(ga, 0, MP, rsL, rsL + 128);
    __syncthreads();
    gemmEpilogue<EPI, 32>(ga, tile, kGemmRows, 0, ga.M, 0, R0, tileIdx, ga.ssIn ? rsL : nullptr);
    if (ga.e.trace) gemmTrace(ga, tr, true);
}

}  // namespace hipk
}  // namespace dl
