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
int attnSplitGrid(int seqLen) {
    int g = (seqLen + 255) / 256;
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
    int HG = 1;
    while (HG < hgMax && (long)(a.nHeads0 / HG) * a.splitGrid * B > 256) HG *= 2;
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
    const size_t kvBase = (size_t)g * HS;
    u32x4 kr[PER], vr[PER];
    auto gload = [&](int t0) {
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int e = tid + u * kPfThreads;
            const int key = min(t0 + e / U8, k1 - 1);  // past the range: masked in compute (and mapped)
            const size_t off = kvBase + kvRow(a.kvMap, a.seqLen, sl, key) * a.kv0 + (e % U8) * 8;
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
    if (attnPrefillDmaSupported(a)) {  // LDS-DMA staged kernel (attn_mfma.hip)
        launchAttentionPrefillDma(a, nRows, s);
        return;
    }
    const int nKv = a.nHeads0 / a.kvMul, rpb = attnPrefillRowsPerBlock(a.kvMul);
    const dim3 grid(nKv * ((nRows + rpb - 1) / rpb), a.splitGrid);
    if (a.hs == 128) hipLaunchKernelGGL(attnPrefillKernel<128>, grid, dim3(kPfThreads), 0, s, a, nRows);
    else hipLaunchKernelGGL(attnPrefillKernel<64>, grid, dim3(kPfThreads), 0, s, a, nRows);
}

// ------------------------------------------------------------------------------------------------
// Small kernels
// ------------------------------------------------------------------------------------------------
__global__ void embeddingKernel(const float *table, const int *tokens, float *x, int dim, unsigned *epoch) {
    const int b = blockIdx.x;
    if (epoch && b == 0 && threadIdx.x == 0) *epoch += 1;  // read by later kernels of this forward
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

void launchEmbedding(const float *table, const int *tokens, float *x, int dim, int B, hipStream_t s, unsigned *epoch) {
    hipLaunchKernelGGL(embeddingKernel, dim3(B), dim3(256), 0, s, table, tokens, x, dim, epoch);
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

// one kernel per translation unit (each .hip file is its own code object)
const void *gemmModuleKernel();
const void *gemmWideModuleKernel();
const void *attnMfmaModuleKernel();
const void *xgmiModuleKernel();
const void *gemvFnL16(bool q40, int B, int pro, int epi);
const void *gemvFnL32(bool q40, int B, int pro, int epi);
const void *gemvFnL64(bool q40, int B, int pro, int epi);
const void *attnBlockFn_16_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_32_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_32_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_16_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_64_128(int hg, bool bf16, int md);
const void *attnBlockFn_32_64_128(int hg, bool bf16, int md);
const void *attnBlockFn_64_64_64(int hg, bool bf16, int md);

void preloadModules() {
    typedef const void *(*BlockFn)(int, bool, int);
    const BlockFn blocks[] = {attnBlockFn_16_32_128, attnBlockFn_32_32_128, attnBlockFn_64_32_128, attnBlockFn_64_16_128,
                              attnBlockFn_64_64_128, attnBlockFn_32_64_128, attnBlockFn_64_64_64};
    std::vector<const void *> fns = {(const void *)argmaxKernel, gemmModuleKernel(), gemmWideModuleKernel(),
                                     attnMfmaModuleKernel(), xgmiModuleKernel(), gemvFnL16(true, 1, 0, 0),
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
