// Single-kernel entry points (see ops.h). Host staging is deliberately simple: synchronous copies,
// one allocation per operand, freed on return.
#include "ops.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "../core/quant.h"
#include "device_comm.h"
#include "kernels.h"

namespace dl {
namespace ops {

namespace {

// Device allocations of one op call, released on scope exit.
class Scratch {
  public:
    Scratch() { DL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
    ~Scratch() {
        for (void *p : mem_) (void)hipFree(p);
        (void)hipStreamDestroy(s);
    }
    template <typename T>
    T *alloc(size_t count) {
        void *p = nullptr;
        const size_t bytes = count * sizeof(T) < 16 ? 16 : count * sizeof(T);
        DL_HIP(hipMalloc(&p, bytes));
        DL_HIP(hipMemsetAsync(p, 0, bytes, s));
        mem_.push_back(p);
        return static_cast<T *>(p);
    }
    template <typename T>
    T *upload(const std::vector<T> &v) {
        if (v.empty()) return nullptr;
        T *p = alloc<T>(v.size());
        DL_HIP(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
        return p;
    }
    template <typename T>
    std::vector<T> download(const T *p, size_t count) {
        std::vector<T> v(count);
        DL_HIP(hipMemcpyAsync(v.data(), p, count * sizeof(T), hipMemcpyDeviceToHost, s));
        DL_HIP(hipStreamSynchronize(s));
        return v;
    }
    void sync() {
        DL_HIP(hipGetLastError());
        DL_HIP(hipStreamSynchronize(s));
    }
    hipStream_t s = nullptr;

  private:
    std::vector<void *> mem_;
};

// File-layout Q40 blocks -> the engine's tiled device layout (csrc/hip/kernels.h Q40Tiling).
struct DevQ40 {
    uint8_t *qs = nullptr;
    uint16_t *d = nullptr;
    int lanes = 0;
};

DevQ40 uploadQ40(Scratch &sc, const std::vector<uint8_t> &blocks, int rows, int n) {
    DL_CHECK(n % 32 == 0 && rows > 0, "Q40 shape");
    const size_t nb = (size_t)rows * (n / 32);
    DL_CHECK(blocks.size() == nb * sizeof(BlockQ40), "Q40 blocks size");
    std::vector<uint8_t> qs(nb * 16);
    std::vector<uint16_t> d(nb);
    const BlockQ40 *b = reinterpret_cast<const BlockQ40 *>(blocks.data());
    for (size_t i = 0; i < nb; i++) {
        std::memcpy(&qs[i * 16], b[i].qs, 16);
        d[i] = b[i].d;
    }
    DevQ40 m;
    m.lanes = hipk::gemvLanesPerRow(n, rows, 1, true);
    const hipk::Q40Tiling t = hipk::q40Tiling(rows, n, m.lanes);
    std::vector<uint8_t> qt(t.qsBytes);
    std::vector<uint32_t> dt(t.dBytes / 4);
    hipk::tileQ40(qs.data(), d.data(), rows, n, m.lanes, qt.data(), dt.data());
    m.qs = sc.upload(qt);
    m.d = reinterpret_cast<uint16_t *>(sc.upload(dt));
    return m;
}

void checkRows(const std::vector<float> &v, size_t want, const char *what) {
    DL_CHECK(v.empty() || v.size() == want, std::string("ops: bad size of ") + what);
}

}  // namespace

std::vector<float> gemvQ40(const std::vector<uint8_t> &blocks, int rows, int n, const std::vector<float> &in,
                           const std::vector<float> &residual, const std::vector<float> &normW, float eps, int B,
                           int epi, std::vector<float> *xNext) {
    DL_CHECK(B == 1 || B == 2 || B == 4, "gemv batch must be 1, 2 or 4");
    DL_CHECK(epi == 0 || (epi == 1 && rows % 2 == 0), "gemv epilogue");
    DL_CHECK(in.size() == (size_t)B * n, "gemv input size");
    checkRows(residual, (size_t)B * n, "residual");
    checkRows(normW, (size_t)n, "norm weights");
    Scratch sc;
    const DevQ40 w = uploadQ40(sc, blocks, rows, n);
    const int outRows = epi == 1 ? rows / 2 : rows;
    hipk::GemvArgs a;
    a.qs = w.qs;
    a.wd = w.d;
    a.rows = rows;
    a.n = n;
    a.lanes = w.lanes;
    const int ep = epi == 1 ? hipk::EPI_ACT : hipk::EPI_STORE;
    a.passes = hipk::gemvDefaultPasses(n, rows, B, true, ep);
    a.in = sc.upload(in);
    a.ldIn = n;
    a.addIn = sc.upload(residual);
    a.xNext = residual.empty() ? nullptr : sc.alloc<float>((size_t)B * n);
    a.normW = sc.upload(normW);
    a.eps = eps;
    a.out = sc.alloc<float>((size_t)B * outRows);
    a.ldOut = outRows;
    a.act = 1;
    const size_t lds = hipk::gemvLdsBytes(n, B, true, hipk::gemvRowsPerPass(n, rows, B, true) * a.passes,
                                          hipk::PRO_RESNORM);
    DL_CHECK(B == 1 || lds <= 64 * 1024, "gemv LDS footprint too large for this batch");
    hipk::launchGemv(a, B, hipk::PRO_RESNORM, ep, true, sc.s);
    sc.sync();
    if (xNext && a.xNext) *xNext = sc.download(a.xNext, (size_t)B * n);
    return sc.download(a.out, (size_t)B * outRows);
}

std::vector<float> gemvQ40Q80In(const std::vector<uint8_t> &blocks, int rows, int n, const std::vector<float> &in,
                                int B) {
    DL_CHECK(B == 1 || B == 2 || B == 4, "gemv batch must be 1, 2 or 4");
    DL_CHECK(in.size() == (size_t)B * n, "gemv input size");
    Scratch sc;
    const DevQ40 w = uploadQ40(sc, blocks, rows, n);
    // host Q80 (the reference quantizer) -> int8 codes + (d, sum of codes) per block, as the
    // attention / SwiGLU epilogues hand them to this kernel
    const int nb = n / 32;
    std::vector<BlockQ80> q((size_t)B * nb);
    quantizeQ80(in.data(), q.data(), (u64)B * n);
    std::vector<int8_t> codes((size_t)B * n);
    std::vector<float> scales((size_t)B * nb * 2);
    for (size_t i = 0; i < q.size(); i++) {
        int s = 0;
        for (int j = 0; j < 32; j++) {
            codes[i * 32 + j] = q[i].qs[j];
            s += q[i].qs[j];
        }
        scales[2 * i] = f16ToF32(q[i].d);
        scales[2 * i + 1] = (float)s;
    }
    hipk::GemvArgs a;
    a.qs = w.qs;
    a.wd = w.d;
    a.rows = rows;
    a.n = n;
    a.lanes = w.lanes;
    a.passes = hipk::gemvDefaultPasses(n, rows, B, true, hipk::EPI_STORE);
    a.aq = sc.upload(codes);
    a.as = reinterpret_cast<const float2 *>(sc.upload(scales));
    a.out = sc.alloc<float>((size_t)B * rows);
    a.ldOut = rows;
    hipk::launchGemv(a, B, hipk::PRO_GLOBAL, hipk::EPI_STORE, true, sc.s);
    sc.sync();
    return sc.download(a.out, (size_t)B * rows);
}

std::vector<float> gemmQ40(const std::vector<uint8_t> &blocks, int rows, int n, const std::vector<float> &in,
                           const std::vector<float> &residual, const std::vector<float> &normW, float eps, int M,
                           int splits) {
    DL_CHECK(splits == 0 || (splits > 0 && (n / 32) % splits == 0), "gemm splits must divide n / 32");
    DL_CHECK(M >= 1 && M <= 2048, "gemm tokens must be 1..2048");
    DL_CHECK(in.size() == (size_t)M * n, "gemm input size");
    DL_CHECK(hipk::gemmSupported(n), "gemm input width must be a multiple of 32");
    checkRows(residual, (size_t)M * n, "residual");
    checkRows(normW, (size_t)n, "norm weights");
    Scratch sc;
    const DevQ40 w = uploadQ40(sc, blocks, rows, n);
    hipk::GemvArgs nq;
    nq.n = n;
    nq.in = sc.upload(in);
    nq.ldIn = n;
    nq.addIn = sc.upload(residual);
    nq.normW = sc.upload(normW);
    nq.eps = eps;
    // rows past M are read by the last launch (padded to 16/32) and their outputs dropped
    const int rowsPad = (M + hipk::kGemmMaxTokens - 1) / hipk::kGemmMaxTokens * hipk::kGemmMaxTokens;
    _Float16 *xh = sc.alloc<_Float16>((size_t)rowsPad * n);
    hipk::launchNormF16(nq, xh, M, sc.s);
    float *out = sc.alloc<float>((size_t)M * rows);
    size_t part = hipk::gemmPartFloats(rows, n, M);
    if (splits > 0) part = std::max(part, (size_t)splits * ((rows + 127) / 128) * (size_t)rowsPad * 128);
    float *partBuf = part ? sc.alloc<float>(part) : nullptr;
    int *counters = sc.alloc<int>((size_t)hipk::gemmCounterInts(rows, M) + (size_t)(rows + 63) / 64 * (M / 128 + 1) + 1);
    // the engine's chunking: one wide launch, or <= 128 tokens per narrow launch
    const int chunk = hipk::gemmUsesWide(M) ? M : hipk::kGemmMaxTokens;
    for (int c0 = 0; c0 < M; c0 += chunk) {
        const int bc = std::min(chunk, M - c0);
        hipk::GemmArgs g;
        g.e.qs = w.qs;
        g.e.wd = w.d;
        g.e.rows = rows;
        g.e.n = n;
        g.e.lanes = w.lanes;
        g.e.out = out + (size_t)c0 * rows;
        g.e.ldOut = rows;
        g.x = xh + (size_t)c0 * n;
        g.M = bc;
        g.splits = splits > 0 ? splits : hipk::gemmSplits(rows, n, bc, w.lanes);
        g.part = partBuf;
        g.counters = counters;
        hipk::launchGemmQ40(g, hipk::EPI_STORE, sc.s);
    }
    sc.sync();
    return sc.download(out, (size_t)M * rows);
}

// Batched F32-weight GEMM (K5): RMS norm -> f16 activations -> gemmF32Kernel, EPI_STORE.
std::vector<float> gemmF32(const std::vector<float> &w, int rows, int n, const std::vector<float> &in,
                           const std::vector<float> &normW, float eps, int M) {
    DL_CHECK(M >= 1 && M <= 256, "gemm tokens must be 1..256");
    DL_CHECK(w.size() == (size_t)rows * n && in.size() == (size_t)M * n, "gemm operand sizes");
    DL_CHECK(hipk::gemmSupported(n), "gemm input width must be a multiple of 32");
    checkRows(normW, (size_t)n, "norm weights");
    Scratch sc;
    hipk::GemvArgs nq;
    nq.n = n;
    nq.in = sc.upload(in);
    nq.ldIn = n;
    nq.normW = sc.upload(normW);
    nq.eps = eps;
    const int rowsPad = (M + hipk::kGemmF32MaxTokens - 1) / hipk::kGemmF32MaxTokens * hipk::kGemmF32MaxTokens;
    _Float16 *xh = sc.alloc<_Float16>((size_t)rowsPad * n);
    hipk::launchNormF16(nq, xh, M, sc.s);
    const float *wd = sc.upload(w);
    float *out = sc.alloc<float>((size_t)M * rows);
    const size_t part = hipk::gemmPartFloats(rows, n, M);
    float *partBuf = part ? sc.alloc<float>(part) : nullptr;
    int *counters = sc.alloc<int>((size_t)(rows + 63) / 64 + 1);
    for (int c0 = 0; c0 < M; c0 += hipk::kGemmF32MaxTokens) {
        const int bc = std::min(hipk::kGemmF32MaxTokens, M - c0);
        hipk::GemmArgs g;
        g.e.wf = wd;
        g.e.rows = rows;
        g.e.n = n;
        g.e.out = out + (size_t)c0 * rows;
        g.e.ldOut = rows;
        g.x = xh + (size_t)c0 * n;
        g.M = bc;
        g.splits = hipk::gemmSplits(rows, n, bc);
        g.part = partBuf;
        g.counters = counters;
        hipk::launchGemmF32(g, hipk::EPI_STORE, sc.s);
    }
    sc.sync();
    return sc.download(out, (size_t)M * rows);
}

std::vector<float> qkvRope(const std::vector<uint8_t> &blocks, int q0, int kv0, int hs, int n,
                           const std::vector<float> &in, const std::vector<float> &normW, float eps,
                           const std::vector<float> &rope, int seqLen, const std::vector<int> &pos, bool kvBf16,
                           std::vector<float> *kOut, std::vector<float> *vOut) {
    const int B = (int)pos.size(), rows = q0 + 2 * kv0;
    DL_CHECK(B == 1 || B == 2 || B == 4, "qkv batch must be 1, 2 or 4");
    DL_CHECK(hs % 2 == 0 && hs <= 128 && q0 % hs == 0 && kv0 % hs == 0, "qkv head layout");
    DL_CHECK(in.size() == (size_t)B * n && rope.size() == (size_t)seqLen * hs, "qkv operand sizes");
    checkRows(normW, (size_t)n, "norm weights");
    for (int p : pos) DL_CHECK(p >= 0 && p < seqLen, "qkv position out of range");
    Scratch sc;
    const DevQ40 w = uploadQ40(sc, blocks, rows, n);
    std::vector<int> slots(B);
    for (int b = 0; b < B; b++) slots[b] = b;
    const size_t cacheElems = (size_t)B * seqLen * kv0;
    void *kc = kvBf16 ? (void *)sc.alloc<uint16_t>(cacheElems) : (void *)sc.alloc<float>(cacheElems);
    void *vc = kvBf16 ? (void *)sc.alloc<uint16_t>(cacheElems) : (void *)sc.alloc<float>(cacheElems);
    hipk::GemvArgs a;
    a.qs = w.qs;
    a.wd = w.d;
    a.rows = rows;
    a.n = n;
    a.lanes = w.lanes;
    a.passes = hipk::gemvDefaultPasses(n, rows, B, true, hipk::EPI_QKV);
    a.in = sc.upload(in);
    a.ldIn = n;
    a.normW = sc.upload(normW);
    a.eps = eps;
    a.out = sc.alloc<float>((size_t)B * q0);
    a.ldOut = q0;
    a.q0 = q0;
    a.kv0 = kv0;
    a.hs = hs;
    a.seqLen = seqLen;
    a.rope = reinterpret_cast<const float2 *>(sc.upload(rope));
    a.pos = sc.upload(pos);
    a.slot = sc.upload(slots);
    a.kcache = kc;
    a.vcache = vc;
    a.kvBf16 = kvBf16 ? 1 : 0;
    hipk::launchGemv(a, B, hipk::PRO_RESNORM, hipk::EPI_QKV, true, sc.s);
    sc.sync();
    auto row = [&](void *cache, int b) {  // the [kv0] row of (slot b, pos[b]) from the head-major cache
        std::vector<float> r(kv0);
        for (int kh = 0; kh < kv0 / hs; kh++) {
            const size_t off = hipk::kvOff(hipk::KvMap{}, seqLen, kv0 / hs, hs, b, pos[b], kh);
            if (kvBf16) {
                const std::vector<uint16_t> h = sc.download(static_cast<uint16_t *>(cache) + off, hs);
                for (int i = 0; i < hs; i++) {
                    const uint32_t u = (uint32_t)h[i] << 16;
                    std::memcpy(&r[kh * hs + i], &u, 4);
                }
            } else {
                const std::vector<float> f = sc.download(static_cast<float *>(cache) + off, hs);
                std::copy(f.begin(), f.end(), r.begin() + (size_t)kh * hs);
            }
        }
        return r;
    };
    if (kOut) kOut->clear();
    if (vOut) vOut->clear();
    for (int b = 0; b < B; b++) {
        if (kOut) {
            const std::vector<float> r = row(kc, b);
            kOut->insert(kOut->end(), r.begin(), r.end());
        }
        if (vOut) {
            const std::vector<float> r = row(vc, b);
            vOut->insert(vOut->end(), r.begin(), r.end());
        }
    }
    return sc.download(a.out, (size_t)B * q0);
}

std::vector<float> attention(const std::vector<float> &q, const std::vector<float> &k, const std::vector<float> &v,
                             int nSlots, int seqLen, int nHeads0, int kvMul, int hs, const std::vector<int> &pos,
                             const std::vector<int> &slot, bool kvBf16, int impl) {
    const int B = (int)pos.size();
    DL_CHECK(B >= 1 && slot.size() == pos.size(), "attention rows");
    if (impl == 1) {
        DL_CHECK(hipk::attnPrefillSupported(hs, kvMul, kvBf16), "prefill attention: head size 64 / 128, power-of-two GQA group");
        const int rpb = hipk::attnPrefillRowsPerBlock(kvMul);
        for (int b = 0; b < B; b++) DL_CHECK(slot[b] == slot[b - b % rpb], "prefill row blocks must share a slot");
    }
    DL_CHECK(kvMul >= 1 && nHeads0 % kvMul == 0 && (hs == 64 || hs == 128), "attention head layout");
    const int q0 = nHeads0 * hs, kv0 = nHeads0 / kvMul * hs;
    const size_t cacheElems = (size_t)nSlots * seqLen * kv0;
    DL_CHECK(q.size() == (size_t)B * q0 && k.size() == cacheElems && v.size() == cacheElems, "attention sizes");
    for (int b = 0; b < B; b++)
        DL_CHECK(pos[b] >= 0 && pos[b] < seqLen && slot[b] >= 0 && slot[b] < nSlots, "attention row out of range");
    Scratch sc;
    auto cache = [&](const std::vector<float> &xs) -> void * {
        // the caller's [slot][seqLen][kv0] rows -> the engine's head-major [slot][nKv][seqLen][hs]
        const int nKv = kv0 / hs;
        std::vector<float> x(xs.size());
        for (int sl = 0; sl < nSlots; sl++)
            for (int p = 0; p < seqLen; p++)
                for (int kh = 0; kh < nKv; kh++)
                    std::memcpy(&x[hipk::kvOff(hipk::KvMap{}, seqLen, nKv, hs, sl, p, kh)],
                                &xs[((size_t)sl * seqLen + p) * kv0 + (size_t)kh * hs], hs * sizeof(float));
        if (!kvBf16) return sc.upload(x);
        std::vector<uint16_t> h(x.size());
        for (size_t i = 0; i < x.size(); i++) {  // round to nearest even, as the QKV epilogue stores
            uint32_t u;
            std::memcpy(&u, &x[i], 4);
            h[i] = (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
        }
        return sc.upload(h);
    };
    hipk::AttnArgs a;
    a.q = sc.upload(q);
    a.ldq = q0;
    a.kcache = cache(k);
    a.vcache = cache(v);
    a.pos = sc.upload(pos);
    a.slot = sc.upload(slot);
    a.nHeads0 = nHeads0;
    a.kvMul = kvMul;
    a.hs = hs;
    a.kv0 = kv0;
    a.seqLen = seqLen;
    a.splitGrid = hipk::attnSplitGrid(seqLen);
    a.chunkMax = hipk::attnChunkMax(seqLen, a.splitGrid);
    a.chunkMin = hipk::attnChunkMin();
    a.partO = sc.alloc<float>((size_t)B * nHeads0 * a.splitGrid * hs);
    a.partML = sc.alloc<float>((size_t)B * nHeads0 * a.splitGrid * 2);
    a.out = sc.alloc<float>((size_t)B * q0);
    a.ldOut = q0;
    a.kvBf16 = kvBf16 ? 1 : 0;
    a.counters = sc.alloc<int>((size_t)B * nHeads0);
    DL_HIP(hipMemsetAsync(a.counters, 0, sizeof(int) * (size_t)B * nHeads0, sc.s));
    if (impl == 1)
        hipk::launchAttentionPrefill(a, B, sc.s);
    else if (impl == 2)
        hipk::launchAttentionValu(a, B, sc.s);
    else if (impl == 3) {
        DL_CHECK(hipk::attnMfmaSupported(a), "MFMA decode attention: bf16 cache, head size 128, kvMul 1/2/4/8");
        hipk::launchAttentionMfma(a, B, sc.s);
    } else
        hipk::launchAttention(a, B, sc.s);
    sc.sync();
    return sc.download(a.out, (size_t)B * q0);
}

std::vector<int> argmax(const std::vector<float> &logits, int B, int vocab) {
    DL_CHECK(B >= 1 && vocab >= 1 && logits.size() == (size_t)B * vocab, "argmax sizes");
    Scratch sc;
    hipk::ArgmaxArgs g;
    g.logits = sc.upload(logits);
    g.vocab = vocab;
    g.ids = sc.alloc<int>(B);
    g.partV = sc.alloc<float>((size_t)B * 64);
    g.partI = sc.alloc<int>((size_t)B * 64);
    g.counters = sc.alloc<int>(B);
    hipk::launchArgmax(g, B, sc.s);
    sc.sync();
    return sc.download(g.ids, B);
}

std::vector<int> sample(const std::vector<float> &logits, int B, int vocab, const std::vector<float> &specs) {
    DL_CHECK(B >= 1 && vocab >= 2 && logits.size() == (size_t)B * vocab && specs.size() == (size_t)B * 4,
             "sample sizes");
    Scratch sc;
    hipk::SampleArgs g;
    g.logits = sc.upload(logits);
    g.vocab = vocab;
    g.spec = reinterpret_cast<const float4 *>(sc.upload(specs));
    g.ids = sc.alloc<int>(B);
    void *ss = sc.alloc<uint8_t>(hipk::SampleScratch::bytes(B));
    DL_HIP(hipMemsetAsync(ss, 0, hipk::SampleScratch::bytes(B), sc.s));
    g.scratch.carve(ss, B);
    hipk::launchSample(g, B, sc.s);
    sc.sync();
    return sc.download(g.ids, B);
}

std::vector<float> embedding(const std::vector<float> &table, int vocab, int dim, const std::vector<int> &tokens) {
    const int B = (int)tokens.size();
    DL_CHECK(dim % 4 == 0 && table.size() == (size_t)vocab * dim, "embedding sizes");
    for (int t : tokens) DL_CHECK(t >= 0 && t < vocab, "embedding token out of range");
    Scratch sc;
    const float *tab = sc.upload(table);
    const int *tok = sc.upload(tokens);
    float *x = sc.alloc<float>((size_t)B * dim);
    hipk::launchEmbedding(tab, tok, x, dim, B, sc.s);
    sc.sync();
    return sc.download(x, (size_t)B * dim);
}

}  // namespace ops
}  // namespace dl
