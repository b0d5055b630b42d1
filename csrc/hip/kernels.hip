// gfx950 (MI355X / CDNA4) kernels for decode and small-batch forward passes.
//
// Design notes (see csrc/hip/kernels.h for the op map):
// * Weights stream straight from HBM into VGPRs (16 B per lane per Q40 block, several blocks in
//   flight per lane); no LDS staging for operands that are read once (GEMV regime).
// * Activations are quantized to Q80 ONCE per workgroup in the prologue and kept in LDS; the
//   inner product is four v_dot4_i32_i8 per 16 weights with the "-8" nibble offset folded into a
//   per-block activation sum: sum((q-8)*x) = dot(q, x) - 8*sum(x).
// * Row reductions use DPP (quad_perm / row_ror) inside 16-lane rows, shfl only across rows.
// * Every per-token input (token id, position, KV slot) is read from device memory so the whole
//   forward pass can be captured once in a hipGraph and replayed.
#include "device_common.h"
#include "kernels.h"

namespace dl {
namespace hipk {

using namespace dl::dev;

static constexpr int kThreads = 256;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

__host__ __device__ static inline size_t alignUp(size_t x, size_t a) { return (x + a - 1) / a * a; }

int gemvLanesPerRow(int n, bool q40) {
    if (q40) {
        const int nb = n / 32;
        if (nb >= 384) return 64;
        if (nb >= 192) return 32;
        return 16;
    }
    const int n4 = n / 4;
    if (n4 >= 2048) return 64;
    if (n4 >= 512) return 32;
    return 16;
}

struct GemvLds {
    size_t scratch, res, act, sc, total;
};

__host__ __device__ static GemvLds gemvLayout(int n, int B, bool q40, int rowsPerWg) {
    GemvLds l;
    size_t off = 0;
    l.scratch = off;
    off += 64 * sizeof(float);
    l.res = off;
    off = alignUp(off + (size_t)B * rowsPerWg * sizeof(float), 16);
    l.act = off;
    if (q40) {
        off = alignUp(off + (size_t)B * n, 16);
        l.sc = off;
        off = alignUp(off + (size_t)B * (n / 32) * sizeof(float2), 16);
    } else {
        off = alignUp(off + (size_t)B * n * sizeof(float), 16);
        l.sc = off;
    }
    l.total = off;
    return l;
}

size_t gemvLdsBytes(int n, int B, bool q40, int rowsPerWg) { return gemvLayout(n, B, q40, rowsPerWg).total; }

// ------------------------------------------------------------------------------------------------
// GEMV: out[b][row] = W[row,:] . act(in[b,:]), fused prologue/epilogue.
// ------------------------------------------------------------------------------------------------
template <int L, int B, int PRO, int EPI, bool Q40>
__global__ __launch_bounds__(kThreads) void gemvKernel(GemvArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int RP = kThreads / L;  // rows per pass
    const int n = a.n, nb = n >> 5;
    const int R = RP * a.passes;
    const GemvLds lay = gemvLayout(n, B, Q40, R);
    float *scratch = reinterpret_cast<float *>(smem + lay.scratch);
    float *res = reinterpret_cast<float *>(smem + lay.res);
    int8_t *sq = reinterpret_cast<int8_t *>(smem + lay.act);
    float *sf = reinterpret_cast<float *>(smem + lay.act);
    float2 *ssc = reinterpret_cast<float2 *>(smem + lay.sc);
    const int tid = threadIdx.x;

    // ---- prologue: (residual add) + (rms norm) + quantize activations into LDS ----------------
    float inv[B];
#pragma unroll
    for (int b = 0; b < B; b++) inv[b] = 1.0f;
    if constexpr (PRO == PRO_RESNORM) {
#pragma unroll
        for (int b = 0; b < B; b++) {
            const float *xi = a.in + (size_t)b * a.ldIn;
            const float *yi = a.addIn ? a.addIn + (size_t)b * a.ldIn : nullptr;
            float *xo = (blockIdx.x == 0 && a.xNext) ? a.xNext + (size_t)b * a.ldIn : nullptr;
            float ss = 0.f;
            for (int i = tid * 4; i < n; i += kThreads * 4) {
                float4 v = ld4(xi + i);
                if (yi) {
                    const float4 y = ld4(yi + i);
                    v.x += y.x;
                    v.y += y.y;
                    v.z += y.z;
                    v.w += y.w;
                }
                ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                if (xo) st4(xo + i, v);
            }
            if (a.normW) {
                ss = blockSum<kThreads>(ss, scratch);
                inv[b] = 1.0f / sqrtf(ss / (float)n + a.eps);
            }
        }
    }
#pragma unroll
    for (int b = 0; b < B; b++) {
        const float *xi = a.in + (size_t)b * a.ldIn;
        const float *yi = (PRO == PRO_RESNORM && a.addIn) ? a.addIn + (size_t)b * a.ldIn : nullptr;
        const float *w = (PRO == PRO_RESNORM) ? a.normW : nullptr;
        for (int c = tid; c < (n >> 3); c += kThreads) {
            float v[8];
            float4 v0 = ld4(xi + c * 8), v1 = ld4(xi + c * 8 + 4);
            if (yi) {
                const float4 y0 = ld4(yi + c * 8), y1 = ld4(yi + c * 8 + 4);
                v0.x += y0.x; v0.y += y0.y; v0.z += y0.z; v0.w += y0.w;
                v1.x += y1.x; v1.y += y1.y; v1.z += y1.z; v1.w += y1.w;
            }
            v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
            v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
            if (w) {
                const float4 w0 = ld4(w + c * 8), w1 = ld4(w + c * 8 + 4);
                const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
                for (int i = 0; i < 8; i++) v[i] = wv[i] * (inv[b] * v[i]);
            }
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
    }
    __syncthreads();

    // ---- main loop ------------------------------------------------------------------------------
    const int gi = tid / L, li = tid % L;
    const int rowBase = blockIdx.x * R;
    for (int p = 0; p < a.passes; p++) {
        const int row = rowBase + p * RP + gi;
        const int rowc = row < a.rows ? row : a.rows - 1;
        float acc[B];
#pragma unroll
        for (int b = 0; b < B; b++) acc[b] = 0.f;
        if constexpr (Q40) {
            constexpr int U = 4;
            const u32x4 *wrow = reinterpret_cast<const u32x4 *>(a.qs + (size_t)rowc * nb * 16);
            const uint16_t *drow = a.wd + (size_t)rowc * nb;
            for (int j0 = li; j0 < nb; j0 += L * U) {
                u32x4 w[U];
                float dw[U];
                int jj[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int j = j0 + u * L;
                    jj[u] = j < nb ? j : nb - 1;  // clamp: loads always issue, tail masked by dw=0
                    w[u] = __builtin_nontemporal_load(wrow + jj[u]);
                    const uint16_t hb = drow[jj[u]];
                    dw[u] = j < nb ? __half2float(__ushort_as_half(hb)) : 0.f;
                }
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const int j = jj[u];
                    const int lo0 = w[u].x & 0x0F0F0F0F, hi0 = (w[u].x >> 4) & 0x0F0F0F0F;
                    const int lo1 = w[u].y & 0x0F0F0F0F, hi1 = (w[u].y >> 4) & 0x0F0F0F0F;
                    const int lo2 = w[u].z & 0x0F0F0F0F, hi2 = (w[u].z >> 4) & 0x0F0F0F0F;
                    const int lo3 = w[u].w & 0x0F0F0F0F, hi3 = (w[u].w >> 4) & 0x0F0F0F0F;
#pragma unroll
                    for (int b = 0; b < B; b++) {
                        const int4 xa = *reinterpret_cast<const int4 *>(sq + (size_t)b * n + j * 32);
                        const int4 xb = *reinterpret_cast<const int4 *>(sq + (size_t)b * n + j * 32 + 16);
                        int s = dot4(lo0, xa.x, 0);
                        s = dot4(lo1, xa.y, s);
                        s = dot4(lo2, xa.z, s);
                        s = dot4(lo3, xa.w, s);
                        s = dot4(hi0, xb.x, s);
                        s = dot4(hi1, xb.y, s);
                        s = dot4(hi2, xb.z, s);
                        s = dot4(hi3, xb.w, s);
                        const float2 sc = ssc[b * nb + j];
                        acc[b] += (dw[u] * sc.x) * (float)(s - 8 * (int)sc.y);
                    }
                }
            }
        } else {
            const f32x4 *wrow = reinterpret_cast<const f32x4 *>(a.wf + (size_t)rowc * n);
            const int n4 = n >> 2;
#pragma unroll 4
            for (int k = li; k < n4; k += L) {
                const f32x4 wv = __builtin_nontemporal_load(wrow + k);
#pragma unroll
                for (int b = 0; b < B; b++) {
                    const float4 xv = *reinterpret_cast<const float4 *>(sf + (size_t)b * n + k * 4);
                    acc[b] += wv.x * xv.x + wv.y * xv.y + wv.z * xv.z + wv.w * xv.w;
                }
            }
        }
#pragma unroll
        for (int b = 0; b < B; b++) acc[b] = groupSum<L>(acc[b]);
        if (li == 0) {
            if constexpr (EPI == EPI_STORE) {
                if (row < a.rows) {
#pragma unroll
                    for (int b = 0; b < B; b++) a.out[(size_t)b * a.ldOut + row] = acc[b];
                }
            } else {
#pragma unroll
                for (int b = 0; b < B; b++) res[b * R + p * RP + gi] = acc[b];
            }
        }
    }
    if constexpr (EPI == EPI_STORE) return;
    __syncthreads();

    // ---- pair epilogues (rows 2k, 2k+1 of this workgroup) --------------------------------------
    const int halfR = R / 2;
    for (int i = tid; i < B * halfR; i += kThreads) {
        const int b = i / halfR, k = i % halfR;
        const int r0 = rowBase + 2 * k;
        if (r0 >= a.rows) continue;
        const float v0 = res[b * R + 2 * k], v1 = res[b * R + 2 * k + 1];
        if constexpr (EPI == EPI_ACT) {
            // interleaved rows: 2i = gate (w1), 2i+1 = up (w3)
            float g;
            if (a.act == 1) {
                g = v0 / (1.0f + __expf(-v0));
            } else {
                g = 0.5f * v0 * (1.0f + tanhf(0.79788456080286535588f * v0 * (1.0f + 0.044715f * v0 * v0)));
            }
            a.out[(size_t)b * a.ldOut + (r0 >> 1)] = g * v1;
        } else if constexpr (EPI == EPI_QKV) {
            const int p = a.pos[b];
            const int sl = a.slot[b];
            if (r0 < a.q0 + a.kv0) {
                const float2 cs = a.rope[(size_t)p * (a.hs >> 1) + ((r0 % a.hs) >> 1)];
                const float o0 = v0 * cs.x - v1 * cs.y;
                const float o1 = v0 * cs.y + v1 * cs.x;
                if (r0 < a.q0) {
                    a.out[(size_t)b * a.ldOut + r0] = o0;
                    a.out[(size_t)b * a.ldOut + r0 + 1] = o1;
                } else {
                    const size_t off = ((size_t)sl * a.seqLen + p) * a.kv0 + (r0 - a.q0);
                    if (a.kvBf16) {
                        uint32_t pk = (uint32_t)f32ToBf16(o0) | ((uint32_t)f32ToBf16(o1) << 16);
                        *reinterpret_cast<uint32_t *>(reinterpret_cast<uint16_t *>(a.kcache) + off) = pk;
                    } else {
                        *reinterpret_cast<float2 *>(reinterpret_cast<float *>(a.kcache) + off) = make_float2(o0, o1);
                    }
                }
            } else {
                const size_t off = ((size_t)sl * a.seqLen + p) * a.kv0 + (r0 - a.q0 - a.kv0);
                if (a.kvBf16) {
                    uint32_t pk = (uint32_t)f32ToBf16(v0) | ((uint32_t)f32ToBf16(v1) << 16);
                    *reinterpret_cast<uint32_t *>(reinterpret_cast<uint16_t *>(a.vcache) + off) = pk;
                } else {
                    *reinterpret_cast<float2 *>(reinterpret_cast<float *>(a.vcache) + off) = make_float2(v0, v1);
                }
            }
        }
    }
}

template <int L, int B, bool Q40>
static void gemvDispatchPE(const GemvArgs &a, int pro, int epi, size_t lds, int grid, hipStream_t s) {
#define DL_GEMV_CASE(P, E)                                                                     \
    if (pro == P && epi == E) {                                                                \
        hipLaunchKernelGGL((gemvKernel<L, B, P, E, Q40>), dim3(grid), dim3(kThreads), lds, s, a); \
        return;                                                                                \
    }
    DL_GEMV_CASE(PRO_QUANT, EPI_STORE)
    DL_GEMV_CASE(PRO_RESNORM, EPI_STORE)
    DL_GEMV_CASE(PRO_RESNORM, EPI_ACT)
    DL_GEMV_CASE(PRO_RESNORM, EPI_QKV)
    DL_GEMV_CASE(PRO_QUANT, EPI_ACT)
#undef DL_GEMV_CASE
}

template <int L, bool Q40>
static void gemvDispatchB(const GemvArgs &a, int B, int pro, int epi, size_t lds, int grid, hipStream_t s) {
    switch (B) {
        case 1: gemvDispatchPE<L, 1, Q40>(a, pro, epi, lds, grid, s); break;
        case 2: gemvDispatchPE<L, 2, Q40>(a, pro, epi, lds, grid, s); break;
        case 4: gemvDispatchPE<L, 4, Q40>(a, pro, epi, lds, grid, s); break;
        default: break;
    }
}

void launchGemv(const GemvArgs &a, int B, int pro, int epi, bool q40, hipStream_t s) {
    const int L = gemvLanesPerRow(a.n, q40);
    const int R = (kThreads / L) * a.passes;
    const int grid = (a.rows + R - 1) / R;
    const size_t lds = gemvLdsBytes(a.n, B, q40, R);
    if (q40) {
        switch (L) {
            case 16: gemvDispatchB<16, true>(a, B, pro, epi, lds, grid, s); break;
            case 32: gemvDispatchB<32, true>(a, B, pro, epi, lds, grid, s); break;
            default: gemvDispatchB<64, true>(a, B, pro, epi, lds, grid, s); break;
        }
    } else {
        switch (L) {
            case 16: gemvDispatchB<16, false>(a, B, pro, epi, lds, grid, s); break;
            case 32: gemvDispatchB<32, false>(a, B, pro, epi, lds, grid, s); break;
            default: gemvDispatchB<64, false>(a, B, pro, epi, lds, grid, s); break;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Attention (decode / prefill rows): split the sequence [0, pos] into chunks, one workgroup per
// (head group, chunk, row); online-softmax partials are merged by attnCombineKernel.
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

__device__ __forceinline__ void attnSplit(int len, int splitGrid, int &nSplit, int &ch) {
    int ns = (len + 255) / 256;
    if (ns > splitGrid) ns = splitGrid;
    if (ns < 1) ns = 1;
    ch = (((len + ns - 1) / ns) + 15) & ~15;
    nSplit = (len + ch - 1) / ch;
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

template <int HG, int HS, bool BF16>
__global__ __launch_bounds__(kThreads) void attnKernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int DPL = HS / 16;  // dims per lane in the score phase (16 lanes per position)
    constexpr int DPV = HS / 64;  // dims per lane in the PV phase (one wave per position)
    const int b = blockIdx.z;
    const int pos = a.pos[b], sl = a.slot[b];
    const int len = pos + 1;
    int nSplit, ch;
    attnSplit(len, a.splitGrid, nSplit, ch);
    const int c = blockIdx.y;
    if (c >= nSplit) return;
    const int t0 = c * ch;
    const int t1 = min(t0 + ch, len);
    const int nt = t1 - t0;
    const int head0 = blockIdx.x * HG;
    const int kvh = head0 / a.kvMul;
    const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;

    float *qL = reinterpret_cast<float *>(smem);          // [HG][HS]
    float *sL = qL + HG * HS;                              // [HG][chunkMax]
    float *mlL = sL + HG * a.chunkMax;                     // [HG][2]
    float *redL = mlL + 2 * HG + 2;                        // [4][HG][HS]

    const float scale = 1.0f / sqrtf((float)HS);
    for (int i = tid; i < HG * HS; i += kThreads) qL[i] = a.q[(size_t)b * a.ldq + head0 * HS + i] * scale;
    __syncthreads();

    // scores: 16 lanes per position
    const int g16 = tid / 16, l16 = tid % 16;
    float qr[HG][DPL];
#pragma unroll
    for (int h = 0; h < HG; h++)
#pragma unroll
        for (int i = 0; i < DPL; i++) qr[h][i] = qL[h * HS + l16 * DPL + i];
    const size_t slotBase = (size_t)sl * a.seqLen;
    for (int t = t0 + g16; t < t1; t += kThreads / 16) {
        float kv[DPL];
        loadKv<DPL, BF16>(a.kcache, (slotBase + t) * a.kv0 + kvh * HS + l16 * DPL, kv);
#pragma unroll
        for (int h = 0; h < HG; h++) {
            float d = 0.f;
#pragma unroll
            for (int i = 0; i < DPL; i++) d += qr[h][i] * kv[i];
            d = groupSum<16>(d);
            if (l16 == 0) sL[h * a.chunkMax + (t - t0)] = d;
        }
    }
    __syncthreads();

    // local softmax per head (one wave per head)
    for (int h = wave; h < HG; h += kThreads / 64) {
        float m = -INFINITY;
        for (int i = lane; i < nt; i += 64) m = fmaxf(m, sL[h * a.chunkMax + i]);
        m = waveMax(m);
        float l = 0.f;
        for (int i = lane; i < nt; i += 64) {
            const float e = __expf(sL[h * a.chunkMax + i] - m);
            sL[h * a.chunkMax + i] = e;
            l += e;
        }
        l = waveSum(l);
        if (lane == 0) {
            mlL[h * 2] = m;
            mlL[h * 2 + 1] = l;
        }
    }
    __syncthreads();

    // P.V: wave w takes positions t0+w, t0+w+4, ...; lanes cover the head dims
    float o[HG][DPV];
#pragma unroll
    for (int h = 0; h < HG; h++)
#pragma unroll
        for (int i = 0; i < DPV; i++) o[h][i] = 0.f;
#pragma unroll 2
    for (int t = wave; t < nt; t += kThreads / 64) {
        float vv[DPV];
        loadKv<DPV, BF16>(a.vcache, (slotBase + t0 + t) * a.kv0 + kvh * HS + lane * DPV, vv);
#pragma unroll
        for (int h = 0; h < HG; h++) {
            const float p = sL[h * a.chunkMax + t];
#pragma unroll
            for (int i = 0; i < DPV; i++) o[h][i] += p * vv[i];
        }
    }
#pragma unroll
    for (int h = 0; h < HG; h++)
#pragma unroll
        for (int i = 0; i < DPV; i++) redL[(wave * HG + h) * HS + lane * DPV + i] = o[h][i];
    __syncthreads();
    for (int i = tid; i < HG * HS; i += kThreads) {
        const int h = i / HS, d = i % HS;
        const float s = redL[(0 * HG + h) * HS + d] + redL[(1 * HG + h) * HS + d] + redL[(2 * HG + h) * HS + d] +
                        redL[(3 * HG + h) * HS + d];
        const size_t pidx = ((size_t)b * a.nHeads0 + head0 + h) * a.splitGrid + c;
        a.partO[pidx * HS + d] = s;
        if (d == 0) {
            a.partML[pidx * 2] = mlL[h * 2];
            a.partML[pidx * 2 + 1] = mlL[h * 2 + 1];
        }
    }
}

template <int HS>
__global__ __launch_bounds__(64) void attnCombineKernel(AttnArgs a) {
    constexpr int DPV = HS / 64;
    const int head = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const int len = a.pos[b] + 1;
    int nSplit, ch;
    attnSplit(len, a.splitGrid, nSplit, ch);
    const size_t base = ((size_t)b * a.nHeads0 + head) * a.splitGrid;
    float M = -INFINITY;
    for (int c = 0; c < nSplit; c++) M = fmaxf(M, a.partML[(base + c) * 2]);
    float o[DPV];
#pragma unroll
    for (int i = 0; i < DPV; i++) o[i] = 0.f;
    float Lsum = 0.f;
    for (int c = 0; c < nSplit; c++) {
        const float w = __expf(a.partML[(base + c) * 2] - M);
        Lsum += w * a.partML[(base + c) * 2 + 1];
#pragma unroll
        for (int i = 0; i < DPV; i++) o[i] += w * a.partO[(base + c) * HS + lane * DPV + i];
    }
    const float inv = 1.0f / Lsum;
#pragma unroll
    for (int i = 0; i < DPV; i++) a.out[(size_t)b * a.ldOut + head * HS + lane * DPV + i] = o[i] * inv;
}

template <int HS, bool BF16>
static void attnDispatchHG(const AttnArgs &a, int B, int HG, hipStream_t s) {
    const size_t lds = sizeof(float) * ((size_t)HG * HS + (size_t)HG * a.chunkMax + 2 * HG + 2 + 4 * HG * HS);
    const dim3 grid(a.nHeads0 / HG, a.splitGrid, B);
    switch (HG) {
        case 1: hipLaunchKernelGGL((attnKernel<1, HS, BF16>), grid, dim3(kThreads), lds, s, a); break;
        case 2: hipLaunchKernelGGL((attnKernel<2, HS, BF16>), grid, dim3(kThreads), lds, s, a); break;
        case 4: hipLaunchKernelGGL((attnKernel<4, HS, BF16>), grid, dim3(kThreads), lds, s, a); break;
        default: hipLaunchKernelGGL((attnKernel<8, HS, BF16>), grid, dim3(kThreads), lds, s, a); break;
    }
    hipLaunchKernelGGL((attnCombineKernel<HS>), dim3(a.nHeads0, B), dim3(64), 0, s, a);
}

void launchAttention(const AttnArgs &a, int B, hipStream_t s) {
    int HG = a.kvMul < 8 ? a.kvMul : 8;
    if (HG == 3 || HG == 5 || HG == 6 || HG == 7) HG = 1;
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
__global__ void embeddingKernel(const float *table, const int *tokens, float *x, int dim) {
    const int b = blockIdx.x;
    const float *src = table + (size_t)tokens[b] * dim;
    float *dst = x + (size_t)b * dim;
    for (int i = threadIdx.x * 4; i < dim; i += blockDim.x * 4) st4(dst + i, ld4(src + i));
}

void launchEmbedding(const float *table, const int *tokens, float *x, int dim, int B, hipStream_t s) {
    hipLaunchKernelGGL(embeddingKernel, dim3(B), dim3(256), 0, s, table, tokens, x, dim);
}

__global__ __launch_bounds__(1024) void argmaxKernel(const float *logits, int vocab, int *out) {
    __shared__ float sv[16];
    __shared__ int si[16];
    const int b = blockIdx.x;
    const float *x = logits + (size_t)b * vocab;
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < vocab; i += blockDim.x) {
        const float v = x[i];
        if (v > bv) {
            bv = v;
            bi = i;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const float ov = __shfl_xor(bv, off);
        const int oi = __shfl_xor(bi, off);
        if (ov > bv || (ov == bv && oi < bi)) {
            bv = ov;
            bi = oi;
        }
    }
    const int w = threadIdx.x / 64;
    if (threadIdx.x % 64 == 0) {
        sv[w] = bv;
        si[w] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < (int)(blockDim.x / 64); i++)
            if (sv[i] > bv || (sv[i] == bv && si[i] < bi)) {
                bv = sv[i];
                bi = si[i];
            }
        out[b] = bi;
    }
}

void launchArgmax(const float *logits, int vocab, int B, int *outIds, hipStream_t s) {
    hipLaunchKernelGGL(argmaxKernel, dim3(B), dim3(1024), 0, s, logits, vocab, outIds);
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

__global__ void advanceKernel(const int *ids, int *tokens, int *pos, int B) {
    const int b = threadIdx.x;
    if (b < B) {
        tokens[b] = ids[b];
        pos[b] += 1;
    }
}

void launchAdvance(const int *ids, int *tokens, int *pos, int B, hipStream_t s) {
    hipLaunchKernelGGL(advanceKernel, dim3(1), dim3(64), 0, s, ids, tokens, pos, B);
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

}  // namespace hipk
}  // namespace dl
