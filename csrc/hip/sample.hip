// Argmax and device sampling of the logits rows (ArgmaxArgs / SampleArgs in kernels.h).
#include "decode_dev.h"

#include <cstdlib>

namespace dl {
namespace hipk {

constexpr int kArgmaxBlocks = 64;

// The row's winner: ids, and for a chained decode the next step's token / position / history.
__device__ __forceinline__ void argmaxStore(const ArgmaxArgs &a, int b, int bi) {
    a.ids[b] = bi;
    if (a.tokens) {
        const int p = a.pos[b];
        a.hist[(size_t)b * a.seqLen + p] = bi;
        a.tokens[b] = bi;
        a.pos[b] = p + 1;
    }
}

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
    if (a.pairs) {
        if (threadIdx.x == 0) {
            a.pairs[2 * b] = bv;
            a.pairs[2 * b + 1] = __int_as_float(bi + a.vocabStart);
        }
        return;
    }
    if (threadIdx.x == 0 && a.tp.world > 1) {
        // tensor parallel: every rank offers its slice's winner (value, global index)
        bi += a.vocabStart;
        tpDispatch(a.tp.world, [&](auto wm) { tpArgmaxPick<decltype(wm)::value>(a.tp, b, bv, bi); });
    }
    if (threadIdx.x == 0) argmaxStore(a, b, bi);
}

// One thread per row: the global winner of the all-gathered per-rank pairs, in rank order.
__global__ __launch_bounds__(64) void argmaxPickKernel(ArgmaxArgs a, const float *all, int B, int W) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= B) return;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int p = 0; p < W; p++)
        argBetter(bv, bi, all[(size_t)p * 2 * B + 2 * b], __float_as_int(all[(size_t)p * 2 * B + 2 * b + 1]));
    argmaxStore(a, b, bi);
}

void launchArgmax(const ArgmaxArgs &a, int B, hipStream_t s) {
    hipLaunchKernelGGL(argmaxKernel, dim3(kArgmaxBlocks, B), dim3(256), 0, s, a);
}

void launchArgmaxPick(const ArgmaxArgs &a, const float *all, int B, int W, hipStream_t s) {
    hipLaunchKernelGGL(argmaxPickKernel, dim3((B + 63) / 64), dim3(64), 0, s, a, all, B, W);
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

// (preloadModules: any kernel of this code object)
const void *sampleModuleKernel() { return (const void *)argmaxKernel; }

}  // namespace hipk
}  // namespace dl
