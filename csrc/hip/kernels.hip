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
#include "decode_dev.h"
#include "device_comm.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <type_traits>

namespace dl {
namespace hipk {


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
    return L;
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

int gemvDefaultPasses(int n, int rows, int B, bool q40, int epi, int lanes) {
    static const int resident = [] {
        const char *e = getenv("DL_GEMV_RESIDENT");
        return e ? atoi(e) : 512;
    }();
    const int rp = lanes > 0 ? kThreads / lanes * gemvRowGroup(B, q40) : gemvRowsPerPass(n, rows, B, q40);
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
// Attention (decode / prefill rows): split the sequence [0, pos] into chunks, one workgroup per
// (head group, chunk, row). A single chunk writes the final output directly; with several chunks
// each workgroup publishes its online-softmax partial and the last arriver combines them.
// ------------------------------------------------------------------------------------------------
int attnChunkMin() {
    static const int v = [] {
        const char *e = std::getenv("DL_ATTN_CHUNK");
        const int c = e ? std::atoi(e) : 256;
        return c >= 32 && c <= 1024 && (c & 15) == 0 ? c : 256;
    }();
    return v;
}

int attnSplitGrid(int seqLen, bool shortChunks) {
    const int cm = attnChunkMin();
    int g = (seqLen + cm - 1) / cm;
    if (shortChunks && cm >= 256)
        g = std::max(g, (std::min(seqLen, kAttnShortLen) + kAttnShortChunk - 1) / kAttnShortChunk);
    return g < 1 ? 1 : (g > 128 ? 128 : g);
}

int attnChunkMax(int seqLen, int splitGrid) {
    int per = (seqLen + splitGrid - 1) / splitGrid;
    if (per < 256) per = 256;
    return ((per + 15) / 16) * 16 + 16;
}


template <int HG, int HS, bool BF16>
__global__ __launch_bounds__(kAttnThreads) void attnKernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    attnTask<HG, HS, BF16, kAttnThreads>(a, blockIdx.z, blockIdx.x, blockIdx.y, smem);
}

template <int HS, bool BF16>
static void attnDispatchHG(const AttnArgs &a, int B, int HG, hipStream_t s) {
    constexpr int NW = kAttnThreads / 64;
    const size_t lds = sizeof(float) * (2 * NW * HG + NW * HG * HS + HG * HS + 2 * HG) + 16;
    const dim3 grid(a.nHeads0 / HG, a.splitGrid, B);
    switch (HG) {
        case 1: hipLaunchKernelGGL((attnKernel<1, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
        case 2: hipLaunchKernelGGL((attnKernel<2, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
        case 4: hipLaunchKernelGGL((attnKernel<4, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
        default: hipLaunchKernelGGL((attnKernel<8, HS, BF16>), grid, dim3(kAttnThreads), lds, s, a); break;
    }
}

void launchAttention(const AttnArgs &a, int B, hipStream_t s) {
    if (attnUsesMfma(a))  // bf16 cache, long context: MFMA kernel (attn_mfma.hip)
        launchAttentionMfma(a, B, s);
    else
        launchAttentionValu(a, B, s);
}

void launchAttentionValu(const AttnArgs &a, int B, hipStream_t s) {
    // Query heads per workgroup: sharing a KV head's loads between HG heads costs HG x the serial
    // work per workgroup, so take the fewest heads per workgroup that keep the grid (at the
    // longest context this launch can see) within one workgroup per CU. Measured on MI355X
    // (scripts/bench_attn.py, profiles/r1_attention.md): short contexts 7.9 -> 5.9 us (TP1) and
    // 7.7 -> 4.4 us (TP8) with one head per workgroup; long contexts keep 2-4 heads per workgroup.
    const int hgMax = (a.kvMul & (a.kvMul - 1)) == 0 ? (a.kvMul < 8 ? a.kvMul : 8) : 1;
    static const long gridMax = [] {
        const char *e = std::getenv("DL_ATTN_GRID_MAX");
        return e ? std::atol(e) : 256L;
    }();
    int HG = 1;
    while (HG < hgMax && (long)(a.nHeads0 / HG) * a.splitGrid * B > gridMax) HG *= 2;
    if (a.hs == 128) {
        if (a.kvBf16) attnDispatchHG<128, true>(a, B, HG, s);
        else attnDispatchHG<128, false>(a, B, HG, s);
    } else if (a.hs == 64) {
        if (a.kvBf16) attnDispatchHG<64, true>(a, B, HG, s);
        else attnDispatchHG<64, false>(a, B, HG, s);
    }
}

// ------------------------------------------------------------------------------------------------
// Small kernels
// ------------------------------------------------------------------------------------------------
__global__ void embeddingKernel(const float *table, const int *tokens, float *x, int dim, unsigned *epoch,
                                unsigned *sync, int S, PrenormOut pre) {
    const int b = blockIdx.x;
    // the forward's epoch, read by later kernels: a no-return atomic (the wave does not wait on a
    // read-modify-write round trip before its row loads)
    if (epoch && b == 0 && threadIdx.x == 0) __hip_atomic_fetch_add(epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (b == 0 && S > 0) {
        // fold the previous forward's measured-sync slots into the running totals, then clear them
        // (each thread reads and clears only its own slots: no barrier)
        unsigned long long *st = reinterpret_cast<unsigned long long *>(sync + 2 * S);
        unsigned long long *acc = reinterpret_cast<unsigned long long *>(sync + 6 * S);
        unsigned long long w = 0, sp = 0, sd = 0;
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            w += sync[i];
            sp += sync[S + i];
            const unsigned long long a = st[2 * i], e = st[2 * i + 1];
            if (a && e > a) sd += e - a;
            sync[i] = 0u;
            sync[S + i] = 0u;
            st[2 * i] = 0ull;
            st[2 * i + 1] = 0ull;
        }
        if (w) __hip_atomic_fetch_add(acc, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (sp) __hip_atomic_fetch_add(acc + 1, sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (sd) __hip_atomic_fetch_add(acc + 2, sd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (threadIdx.x == 0) __hip_atomic_fetch_add(acc + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const float *src = table + (size_t)tokens[b] * dim;
    float *dst = x + (size_t)b * dim;
    extern __shared__ float xs[];  // the row (pre.xq set: dim floats of dynamic LDS)
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
            if (pre.xq && i < dim) st4(xs + i, v[u]);
        }
    }
    if (!pre.xq) return;
    // one decode row (B == 1): the first layer's pre-normalized input (PrenormOut, PRO_PRENORM):
    // x * rmsAtt as Q80 blocks with the unrounded d' = amax / 127, and sum(x^2) as one partial
    __syncthreads();
    float ss = 0.f;
    constexpr int WU = 16;  // norm weights of 16 passes loaded at once (one round trip, not 16)
    float wv[WU];
    for (int base = 0; base < dim; base += blockDim.x) {  // dim % 32 == 0: whole 32-lane groups
        const int u = (base / blockDim.x) % WU;
        if (u == 0) {
#pragma unroll
            for (int k = 0; k < WU; k++) {
                const int j = base + k * blockDim.x + threadIdx.x;
                wv[k] = j < dim ? pre.resW[j] : 0.f;
            }
        }
        const int i = base + threadIdx.x;
        const float xv = i < dim ? xs[i] : 0.f;
        float w = 0.f;
#pragma unroll
        for (int k = 0; k < WU; k++) w = k == u ? wv[k] : w;
        const float g = i < dim ? xv * w : 0.f;
        ss += xv * xv;
        const float amax = groupMax<32>(fabsf(g));
        const float d = amax / 127.0f;
        const float id = d != 0.f ? 1.0f / d : 0.f;
        int q = (int)rintf(g * id);
        q = q > 127 ? 127 : (q < -127 ? -127 : q);
        const float qs = groupSum<32>((float)q);
        if (i < dim) pre.xq[i] = (int8_t)q;
        if (i < dim && (i & 31) == 0) pre.xs[i >> 5] = make_float2(d, qs);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ss += __shfl_xor(ss, off);
    __shared__ float red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += red[w];
        pre.ssp[0] = t;
    }
}

void launchEmbedding(const float *table, const int *tokens, float *x, int dim, int B, hipStream_t s, unsigned *epoch,
                     unsigned *sync, int nSync, const PrenormOut *pre) {
    PrenormOut p;
    size_t lds = 0;
    if (pre) {
        if (B != 1 || dim % 32 || (size_t)dim * 4 > 65536) throw Error("launchEmbedding: prenorm output needs one row, dim % 32 == 0, dim <= 16384");
        p = *pre;
        lds = (size_t)dim * 4;
    }
    hipLaunchKernelGGL(embeddingKernel, dim3(B), dim3(256), lds, s, table, tokens, x, dim, epoch, sync, nSync, p);
}

__global__ void stampKernel(unsigned long long *p) {
    if (threadIdx.x == 0) *p = wall_clock64();
}

void launchStamp(unsigned long long *p, hipStream_t s) { hipLaunchKernelGGL(stampKernel, dim3(1), dim3(64), 0, s, p); }

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

// one kernel per translation unit (each .hip file is its own code object)
const void *gemmModuleKernel();
const void *gemmWideModuleKernel();
const void *attnMfmaModuleKernel();
const void *xgmiModuleKernel();
const void *sampleModuleKernel();
const void *attnPrefillModuleKernel();
const void *tpCheckModuleKernel();
const void *gemvFnL16(bool q40, int B, int pro, int epi);
const void *gemvFnL32(bool q40, int B, int pro, int epi);
const void *gemvFnL64(bool q40, int B, int pro, int epi);
const void *attnBlockFn_16_16_128(int hg, bool bf16, int md);
const void *attnBlockFn_16_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_32_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_16_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_64_128(int hg, bool bf16, int md);
const void *attnBlockFn_32_64_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_64_64(int hg, bool bf16, int md);

void preloadModules() {
    typedef const void *(*BlockFn)(int, bool, int);
    const BlockFn blocks[] = {attnBlockFn_16_16_128, attnBlockFn_16_32_128, attnBlockFn_32_32_128, attnBlockFn_64_32_128, attnBlockFn_64_16_128,
                              attnBlockFn_64_64_128, attnBlockFn_32_64_128, attnBlockFn_64_64_64};
    std::vector<const void *> fns = {sampleModuleKernel(), attnPrefillModuleKernel(), tpCheckModuleKernel(),
                                     gemmModuleKernel(),   gemmWideModuleKernel(),    attnMfmaModuleKernel(),
                                     xgmiModuleKernel(),   gemvFnL16(true, 1, 0, 0),
                                     gemvFnL32(true, 1, 0, 0), gemvFnL64(true, 1, 0, 0)};
    for (BlockFn b : blocks) {  // any instance of the unit will do
        const void *f = nullptr;
        for (int hg = 1; hg <= 8 && !f; hg *= 2) f = b(hg, true, 0);
        fns.push_back(f);
    }
    // resolving a kernel's attributes builds (loads) its code object for the current device
    for (const void *f : fns) {
        if (!f) continue;
        hipFuncAttributes at;
        (void)hipFuncGetAttributes(&at, f);
    }
    (void)hipGetLastError();  // a unit without a usable instance must not leave a sticky error
}

}  // namespace hipk
}  // namespace dl
