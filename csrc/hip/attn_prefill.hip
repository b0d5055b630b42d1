// Prefill attention on MFMA for the batched path (split out of kernels.hip).
#include "decode_dev.h"

#include <cstdlib>
#include <type_traits>

namespace dl {
namespace hipk {

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
// An f32 cache (the reference's KV precision) runs the same schedule on v_mfma_f32_16x16x4_f32
// (attnPrefillF32Kernel below): f32 Q, K, V and P, no rounding beyond f32 reassociation.
// ------------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
static constexpr int kPfThreads = 256, kPfWaves = 4, kPfChunk = 256, kPfTile = 32;
static constexpr int kPfVtStride = 40;  // bf16 per transposed-V row in LDS (32 keys + 8 pad)
#ifndef DL_PF_F32_SMALL_CHUNK
#define DL_PF_F32_SMALL_CHUNK 128
#endif
static constexpr int kPfChunkF32Small = DL_PF_F32_SMALL_CHUNK;  // keys per split, f32 kernel, small grids
// Paged caches: the chunk's per-tile pool pages go to LDS once (a tile of 32 keys never crosses a
// page). A page-table load inside the tile loads put a full vmcnt(0) drain at its join before every
// 16-byte load - taken on the contiguous path too - and serialised the tile's memory round trips.
static constexpr int kPfMaxTiles = 256;
__device__ __forceinline__ void pfPages(const AttnArgs &a, int sl, int k0, int k1, int *pageL) {
    if (a.kvMap.table)
        for (int i = threadIdx.x; i < (k1 - k0 + kPfTile - 1) / kPfTile; i += kPfThreads)
            pageL[i] = (int)kvPageOf(a.kvMap, sl, k0 + i * kPfTile);
    __syncthreads();
}

int attnPrefillRowsPerBlock(int kvMul) { return kPfWaves * (16 / kvMul); }
bool attnPrefillSupported(int hs, int kvMul, bool kvBf16) {
    (void)kvBf16;  // bf16: attnPrefillKernel (or the LDS-DMA kernel), f32: attnPrefillF32Kernel
    return (hs == 64 || hs == 128) && kvMul >= 1 && kvMul <= 16 && (kvMul & (kvMul - 1)) == 0;
}

__device__ __forceinline__ bf16x8 f32x8ToBf16(const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; j++) r[j] = (__bf16)v[j];
    return r;
}

// Shared tail of both prefill kernels: normalize and store (one chunk), or publish the chunk's
// partials and let the last-arriving chunk combine them. wts ([64 columns][nSplit]) and tot ([64])
// reuse the workgroup's K / V tile LDS.
template <int HS>
__device__ __forceinline__ void pfFinish(const AttnArgs &a, int nRows, const f32x4 (&o)[HS / 16], float m, float lsum,
                                         int nSplit, int rb, int g, int c, int b0, int row, int head, float *wts,
                                         float *tot, int &flagL) {
    constexpr int NT = HS / 16;
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 4;
    const int kvMul = a.kvMul, rpb = kPfWaves * (16 / kvMul), nKv = a.nHeads0 / kvMul;
    const bool rowOk = row < nRows;
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
    const int maxLen = rowsMaxLen(a.pos, b0, rpb, nRows);
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
    __shared__ int pageL[kPfMaxTiles];
    pfPages(a, sl, k0, k1, pageL);
    u32x4 kr[PER], vr[PER];
    auto gload = [&](int t0) {
        const size_t blk = a.kvMap.table ? (size_t)pageL[(t0 - k0) / kPfTile] : (size_t)sl;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int e = tid + u * kPfThreads;
            const int key = min(t0 + e / U8, k1 - 1);  // past the range: masked in compute (and mapped)
            const size_t off = kvOffAt(a.kvMap, a.seqLen, nKv, HS, blk, key, g) + (e % U8) * 8;
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
    pfFinish<HS>(a, nRows, o, m, lsum, nSplit, rb, g, c, b0, row, head, reinterpret_cast<float *>(&kT[0][0]),
                 reinterpret_cast<float *>(&vT[0][0]), flagL);
}

// f32 cache: the same row-block schedule on v_mfma_f32_16x16x4_f32 (A: lane (col, h) holds
// A[col][h], B: B[h][col], D: D[4 h + i][col]). S^T: MFMA e multiplies K[key 16 u + col][dim
// QD h + e] by Q[column col][dim QD h + e] (lane group h owns a contiguous quarter of the head,
// read as 16-byte LDS vectors); O^T: MFMA (u, i) multiplies V[key 16 u + 4 h + i][dim 16 n + col]
// by P[key 16 u + 4 h + i][col], which is exactly the S^T accumulator lane (col, h) already holds,
// so P never moves. K and V stay row-major in LDS (row stride HS + 4 floats: the 16 columns of a
// K read and the two lane groups of a V read fall on distinct banks). One tile buffer (34 KB) so
// four workgroups share a CU; the next tile's loads are in flight during the MFMAs.
template <int HS>
__global__ __launch_bounds__(kPfThreads) void attnPrefillF32Kernel(AttnArgs a, int nRows) {
    constexpr int NT = HS / 16, QD = HS / 4, SR = HS + 4;
    constexpr int U4 = HS / 4;                        // 16-byte units per key row
    constexpr int PER = kPfTile * U4 / kPfThreads;    // 16-byte units per thread per operand and tile
    static_assert(PER >= 1 && kPfTile * U4 % kPfThreads == 0, "tile / workgroup shape");
    static_assert(kPfTile * SR >= 64 * (HS / 2), "combine weights must fit the K tile");
    __shared__ __attribute__((aligned(16))) float kT[1][kPfTile * SR];
    __shared__ __attribute__((aligned(16))) float vT[1][kPfTile * SR];
    __shared__ int flagL;
    const int kvMul = a.kvMul, rpw = 16 / kvMul, rpb = kPfWaves * rpw, nKv = a.nHeads0 / kvMul;
    const int g = blockIdx.x % nKv, rb = blockIdx.x / nKv, c = blockIdx.y;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, col = lane & 15, h = lane >> 4;
    const int b0 = rb * rpb;
    const int maxLen = rowsMaxLen(a.pos, b0, rpb, nRows);
    // with few row blocks (a 32-row chunk: 16 workgroups per split) the keys are split finer so
    // more CUs share them (4k prompt in 32-row chunks 0.1526 -> 0.1498 ms/token, raw/r6_prefill_f32_chunk_ab.txt)
    const int chunkKeys = gridDim.x >= 256 ? kPfChunk : kPfChunkF32Small;
    int nSplit = (maxLen + chunkKeys - 1) / chunkKeys;
    nSplit = max(1, min(min(nSplit, a.splitGrid), HS / 2));
    const int ch = ((maxLen + nSplit - 1) / nSplit + kPfTile - 1) / kPfTile * kPfTile;
    if (c >= nSplit) return;
    const int k0 = c * ch, k1 = min(k0 + ch, maxLen);
    const int sl = a.slot[b0];
    const int row = b0 + wave * rpw + col / kvMul, head = g * kvMul + col % kvMul;
    const bool rowOk = row < nRows;
    const int myLen = rowOk ? a.pos[row] + 1 : 0;
    const float scale = 1.0f / sqrtf((float)HS);
    float q[QD];
#pragma unroll
    for (int e = 0; e < QD; e += 4) {
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (rowOk) x = ld4(a.q + (size_t)row * a.ldq + (size_t)head * HS + QD * h + e);
        q[e] = x.x * scale; q[e + 1] = x.y * scale; q[e + 2] = x.z * scale; q[e + 3] = x.w * scale;
    }
    const float *kc = reinterpret_cast<const float *>(a.kcache);
    const float *vc = reinterpret_cast<const float *>(a.vcache);
    // two register staging sets: tile t + 2's loads go out while tile t computes and tile t + 1's
    // are still in flight (one set left each tile waiting on a full memory round trip)
    f32x4 kr[2][PER], vr[2][PER];
    __shared__ int pageL[kPfMaxTiles];
    pfPages(a, sl, k0, k1, pageL);
    auto gload = [&](auto sTag, int t0) {
        constexpr int S = decltype(sTag)::value;
        const size_t blk = a.kvMap.table ? (size_t)pageL[(t0 - k0) / kPfTile] : (size_t)sl;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int e = tid + u * kPfThreads;
            const int key = min(t0 + e / U4, k1 - 1);  // past the range: masked in compute
            const size_t off = kvOffAt(a.kvMap, a.seqLen, nKv, HS, blk, key, g) + (e % U4) * 4;
            kr[S][u] = *reinterpret_cast<const f32x4 *>(kc + off);
            vr[S][u] = *reinterpret_cast<const f32x4 *>(vc + off);
        }
    };
    auto lstore = [&](auto sTag) {
        constexpr int S = decltype(sTag)::value;
#pragma unroll
        for (int u = 0; u < PER; u++) {
            const int e = tid + u * kPfThreads, at = (e / U4) * SR + (e % U4) * 4;
            *reinterpret_cast<f32x4 *>(&kT[0][at]) = kr[S][u];
            *reinterpret_cast<f32x4 *>(&vT[0][at]) = vr[S][u];
        }
    };
    f32x4 o[NT];
#pragma unroll
    for (int n = 0; n < NT; n++) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    auto compute = [&](int t0) {
        f32x4 st[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int e = 0; e < QD; e += 4) {
#pragma unroll
            for (int u = 0; u < 2; u++) {  // two independent accumulator chains
                const f32x4 kf = *reinterpret_cast<const f32x4 *>(&kT[0][(16 * u + col) * SR + QD * h + e]);
#pragma unroll
                for (int j = 0; j < 4; j++) st[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(kf[j], q[e + j], st[u], 0, 0, 0);
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
#pragma unroll
        for (int n = 0; n < NT; n++) o[n] *= corr;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const float *vrow = &vT[0][(16 * (j >> 2) + 4 * h + (j & 3)) * SR + col];
#pragma unroll
            for (int n = 0; n < NT; n++) o[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(vrow[16 * n], p[j], o[n], 0, 0, 0);
        }
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    gload(S0{}, k0);
    if (k0 + kPfTile < k1) gload(S1{}, k0 + kPfTile);
    lstore(S0{});
    __syncthreads();
    // tile t in LDS (from set t & 1), tile t + 1 in flight in the other set: issue t + 2 into the
    // set just stored, compute t, then store t + 1 (the loop is unrolled by two: static sets)
    auto step = [&](auto cur, auto nxt, int t0) {
        if (t0 + 2 * kPfTile < k1) gload(cur, t0 + 2 * kPfTile);
        compute(t0);
        __syncthreads();
        if (t0 + kPfTile < k1) {
            lstore(nxt);
            __syncthreads();
        }
    };
    for (int t0 = k0; t0 < k1; t0 += 2 * kPfTile) {
        step(S0{}, S1{}, t0);
        if (t0 + kPfTile < k1) step(S1{}, S0{}, t0 + kPfTile);
    }
    pfFinish<HS>(a, nRows, o, m, lsum, nSplit, rb, g, c, b0, row, head, &kT[0][0], &vT[0][0], flagL);
}

void launchAttentionPrefill(const AttnArgs &a, int nRows, hipStream_t s) {
    if (attnPrefillDmaSupported(a)) {  // LDS-DMA staged kernel (attn_mfma.hip)
        launchAttentionPrefillDma(a, nRows, s);
        return;
    }
    const int nKv = a.nHeads0 / a.kvMul, rpb = attnPrefillRowsPerBlock(a.kvMul);
    const dim3 grid(nKv * ((nRows + rpb - 1) / rpb), a.splitGrid);
    if (!attnPrefillSupported(a.hs, a.kvMul, a.kvBf16 != 0) || a.nHeads0 % a.kvMul)
        throw Error("launchAttentionPrefill: head size 64 / 128 and a power-of-two GQA group <= 16");
    {  // the longest split chunk's tiles fit the kernels' LDS page list (pfPages)
        const int minSplits = std::max(1, std::min(a.splitGrid, a.hs / 2));
        if (a.kvMap.table && ((a.seqLen + minSplits - 1) / minSplits + kPfTile - 1) / kPfTile + 1 > kPfMaxTiles)
            throw Error("launchAttentionPrefill: paged context too long for the per-chunk page list");
    }
    if (!a.kvBf16) {
        if (a.hs == 128) hipLaunchKernelGGL(attnPrefillF32Kernel<128>, grid, dim3(kPfThreads), 0, s, a, nRows);
        else hipLaunchKernelGGL(attnPrefillF32Kernel<64>, grid, dim3(kPfThreads), 0, s, a, nRows);
        return;
    }
    if (a.hs == 128) hipLaunchKernelGGL(attnPrefillKernel<128>, grid, dim3(kPfThreads), 0, s, a, nRows);
    else hipLaunchKernelGGL(attnPrefillKernel<64>, grid, dim3(kPfThreads), 0, s, a, nRows);
}

const void *attnPrefillModuleKernel() { return (const void *)attnPrefillKernel<128>; }

}  // namespace hipk
}  // namespace dl
