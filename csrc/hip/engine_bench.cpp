// Kernel microbenchmarks (scripts/bench_gemv.py, bench_gemm.py, bench_attn.py): each cycles
// `copies` operand sets through a graph of `iters` launches so the 256 MB Infinity Cache cannot
// serve them, and returns microseconds per launch.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "engine.h"
#include "kernels.h"

namespace dl {

double benchGemvQ40(int rows, int n, int pro, int epi, int B, int lanes, int passes, int copies, int iters,
                    std::vector<unsigned long long> *trace) {
    hipStream_t s;
    DL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void *> mem;
    auto alloc = [&](size_t bytes) {
        void *p;
        DL_HIP(hipMalloc(&p, bytes));
        mem.push_back(p);
        return p;
    };
    const int L = lanes > 0 ? lanes : hipk::gemvLanesPerRow(n, rows, B, true);
    const hipk::Q40Tiling t = hipk::q40Tiling(rows, n, L);
    std::vector<uint8_t *> qs(copies);
    std::vector<uint16_t *> d(copies);
    for (int c = 0; c < copies; c++) {
        qs[c] = (uint8_t *)alloc(t.qsBytes);
        d[c] = (uint16_t *)alloc(t.dBytes);
        hipk::launchFillQ40(qs[c], d[c], t.qsBytes / 16, 0.01f, 77 + c, s);
    }
    float *x = (float *)alloc((size_t)B * n * 4), *y = (float *)alloc((size_t)B * n * 4);
    float *xn = (float *)alloc((size_t)B * n * 4), *w = (float *)alloc((size_t)n * 4);
    hipk::launchFillF32Uniform(x, (size_t)B * n, 1.f, 1, s);
    hipk::launchFillF32Uniform(y, (size_t)B * n, 1.f, 2, s);
    hipk::launchFillF32Const(w, n, 1.f, s);
    int8_t *aq = (int8_t *)alloc((size_t)B * n);
    float2 *as = (float2 *)alloc((size_t)B * n / 32 * 8);
    DL_HIP(hipMemsetAsync(aq, 1, (size_t)B * n, s));
    DL_HIP(hipMemsetAsync(as, 0, (size_t)B * n / 32 * 8, s));
    const int outRows = epi == hipk::EPI_ACT_Q80 ? rows / 2 : rows;
    float *out = (float *)alloc((size_t)B * rows * 4);
    int8_t *oq = (int8_t *)alloc((size_t)B * outRows);
    float2 *os = (float2 *)alloc((size_t)B * outRows / 32 * 8);
    hipk::GemvArgs a;
    a.rows = rows;
    a.n = n;
    a.lanes = L;
    a.passes = passes > 0 ? passes : hipk::gemvDefaultPasses(n, rows, B, true, epi);
    if (passes <= 0 && lanes > 0) {  // forced lane count: same residency rule with its rows/pass
        const int rp = 256 / lanes * 2, grid0 = (rows + rp - 1) / rp;
        a.passes = (grid0 + 511) / 512;
        if (epi == hipk::EPI_ACT_Q80)
            while ((rp * a.passes) % 64) a.passes++;
    }
    a.in = x;
    a.ldIn = n;
    a.addIn = y;
    a.xNext = xn;
    a.normW = w;
    a.aq = aq;
    a.as = as;
    a.out = out;
    a.ldOut = outRows;
    a.oq = oq;
    a.os = os;
    if (epi == hipk::EPI_QKV) {  // Llama-like split: q = 2/3 of the rows, k = v = 1/6, one position
        a.hs = 128;
        a.kv0 = rows / 6;
        a.q0 = rows - 2 * a.kv0;
        a.seqLen = 1;
        a.kvBf16 = 1;
        float2 *rope = (float2 *)alloc(64 * sizeof(float2));
        int *zeros = (int *)alloc(64 * sizeof(int));
        DL_HIP(hipMemsetAsync(rope, 0, 64 * sizeof(float2), s));
        DL_HIP(hipMemsetAsync(zeros, 0, 64 * sizeof(int), s));
        a.rope = rope;
        a.pos = zeros;
        a.slot = zeros;
        a.kcache = alloc((size_t)a.kv0 * 2);
        a.vcache = alloc((size_t)a.kv0 * 2);
    }
    if (epi == hipk::EPI_STORE_TP) {  // the TP tail in loopback (ComputeOnlyComm's exchange):
        // DL_BENCH_TP_WORLD ranks (default 8), DL_BENCH_TP_Q80=0 for the f32 wire format
        const char *w = std::getenv("DL_BENCH_TP_WORLD"), *q = std::getenv("DL_BENCH_TP_Q80");
        a.tp.world = w ? std::atoi(w) : 8;
        a.tp.q80 = q && *q == '0' ? 0 : 1;
        a.tp.loopback = 1;
        a.tp.stride = (long long)B * rows * 9;
        a.tp.epochs = (unsigned *)alloc((size_t)a.tp.stride * 4);
        a.tp.error = (int *)alloc(4);
        DL_HIP(hipMemsetAsync(a.tp.epochs, 0, (size_t)a.tp.stride * 4, s));
        DL_HIP(hipMemsetAsync(a.tp.error, 0, 4, s));
        if (a.tp.q80 && passes <= 0)  // whole Q80 blocks of 32 rows per workgroup (engine tpPasses)
            while ((256 / L * 2 * a.passes) % 32) a.passes++;
    }
    const int grid = (rows + (256 / L) * 2 * a.passes - 1) / ((256 / L) * 2 * a.passes);
    unsigned long long *tbuf = trace ? (unsigned long long *)alloc((size_t)iters * grid * 8 * 8) : nullptr;
    auto launch = [&](int c) {
        a.qs = qs[c % copies];
        a.wd = d[c % copies];
        a.trace = tbuf ? tbuf + (size_t)c * grid * 8 : nullptr;
        hipk::launchGemv(a, B, pro, epi, true, s);
    };
    launch(0);
    DL_HIP(hipGetLastError());
    hipGraph_t g;
    hipGraphExec_t ge;
    DL_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < iters; i++) launch(i);
    DL_HIP(hipStreamEndCapture(s, &g));
    DL_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    DL_HIP(hipGraphLaunch(ge, s));
    DL_HIP(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    DL_HIP(hipEventCreate(&e0));
    DL_HIP(hipEventCreate(&e1));
    DL_HIP(hipEventRecord(e0, s));
    DL_HIP(hipGraphLaunch(ge, s));
    DL_HIP(hipEventRecord(e1, s));
    DL_HIP(hipEventSynchronize(e1));
    float ms = 0;
    DL_HIP(hipEventElapsedTime(&ms, e0, e1));
    if (trace) {
        trace->resize((size_t)iters * grid * 8);
        DL_HIP(hipMemcpy(trace->data(), tbuf, trace->size() * 8, hipMemcpyDeviceToHost));
    }
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (void *p : mem) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return ms * 1000.0 / iters;
}

double benchGemmQ40(int rows, int n, int M, int epi, int copies, int iters, std::vector<unsigned long long> *trace) {
    DL_CHECK(M >= 1 && M <= hipk::kGemmMaxTokens && hipk::gemmSupported(n) && rows % 64 == 0, "bad gemm bench shape");
    hipStream_t s;
    DL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void *> mem;
    auto alloc = [&](size_t bytes) {
        void *p;
        DL_HIP(hipMalloc(&p, bytes));
        DL_HIP(hipMemsetAsync(p, 0, bytes, s));
        mem.push_back(p);
        return p;
    };
    const int L = hipk::gemvLanesPerRow(n, rows, 1, true);
    const hipk::Q40Tiling t = hipk::q40Tiling(rows, n, L);
    std::vector<uint8_t *> qs(copies);
    std::vector<uint16_t *> d(copies);
    for (int c = 0; c < copies; c++) {
        qs[c] = (uint8_t *)alloc(t.qsBytes);
        d[c] = (uint16_t *)alloc(t.dBytes);
        hipk::launchFillQ40(qs[c], d[c], t.qsBytes / 16, 0.01f, 77 + c, s);
    }
    // the operand rows a launch reads: the narrow kernel's 16/32/64/128-row pad, the wide kernel's
    // whole 128-token tiles
    const int MP = hipk::gemmUsesWide(M) ? (M + 127) / 128 * 128 : hipk::gemmTokenPad(M);
    _Float16 *x = (_Float16 *)alloc((size_t)MP * n * 2);
    hipk::launchFillF32Uniform((float *)x, (size_t)MP * n / 2, 1e-3f, 3, s);  // small finite f16 pairs
    const size_t part = hipk::gemmPartFloats(rows, n, M);
    hipk::GemmArgs g;
    g.e.rows = rows;
    g.e.n = n;
    g.e.lanes = L;
    g.e.out = (float *)alloc((size_t)M * rows * 4);
    g.e.ldOut = epi == hipk::EPI_STORE ? rows : rows / 2;
    g.outH = (_Float16 *)alloc((size_t)M * rows * 2);
    g.x = x;
    g.M = M;
    g.splits = hipk::gemmSplits(rows, n, M, L);
    g.part = part ? (float *)alloc(part * 4) : nullptr;
    g.counters = (int *)alloc((size_t)std::max(rows / 64 + 1, hipk::gemmCounterInts(rows, M)) * 4);
    auto launch = [&](int c) {
        g.e.qs = qs[c % copies];
        g.e.wd = d[c % copies];
        hipk::launchGemmQ40(g, epi, s);
    };
    launch(0);
    DL_HIP(hipGetLastError());
    hipGraph_t gr;
    hipGraphExec_t ge;
    DL_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < iters; i++) launch(i);
    DL_HIP(hipStreamEndCapture(s, &gr));
    DL_HIP(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    DL_HIP(hipGraphLaunch(ge, s));
    DL_HIP(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    DL_HIP(hipEventCreate(&e0));
    DL_HIP(hipEventCreate(&e1));
    DL_HIP(hipEventRecord(e0, s));
    DL_HIP(hipGraphLaunch(ge, s));
    DL_HIP(hipEventRecord(e1, s));
    DL_HIP(hipEventSynchronize(e1));
    float ms = 0;
    DL_HIP(hipEventElapsedTime(&ms, e0, e1));
    if (trace) {
        const size_t words = 8 * (size_t)((rows + 63) / 64) * g.splits;
        unsigned long long *tb = (unsigned long long *)alloc(words * 8);
        g.e.trace = tb;
        launch(1);
        DL_HIP(hipStreamSynchronize(s));
        trace->resize(words);
        DL_HIP(hipMemcpy(trace->data(), tb, words * 8, hipMemcpyDeviceToHost));
        g.e.trace = nullptr;
    }
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(gr);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (void *p : mem) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return ms * 1000.0 / iters;
}

double benchAttention(int nHeads0, int kvMul, int hs, int seqLen, int pos, int B, int copies, int iters,
                      std::vector<unsigned long long> *trace, bool kvBf16) {
    hipStream_t s;
    DL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void *> mem;
    auto alloc = [&](size_t bytes) {
        void *p;
        DL_HIP(hipMalloc(&p, bytes));
        DL_HIP(hipMemsetAsync(p, 0, bytes, s));
        mem.push_back(p);
        return p;
    };
    DL_CHECK(kvMul >= 1 && nHeads0 % kvMul == 0 && pos >= 0 && pos < seqLen && B >= 1, "bad attention bench shape");
    const int kv0 = nHeads0 / kvMul * hs, q0 = nHeads0 * hs;
    const size_t kvElems = (size_t)B * seqLen * kv0;  // one slot per row
    std::vector<void *> kc(copies), vc(copies);
    const size_t kvWords = kvBf16 ? kvElems / 2 : kvElems;  // bf16 pairs of small values, or f32
    for (int c = 0; c < copies; c++) {
        kc[c] = alloc(kvWords * 4);
        vc[c] = alloc(kvWords * 4);
        hipk::launchFillF32Uniform((float *)kc[c], kvWords, 1.f, 5 + c, s);
        hipk::launchFillF32Uniform((float *)vc[c], kvWords, 1.f, 9 + c, s);
    }
    float *q = (float *)alloc((size_t)B * q0 * 4);
    hipk::launchFillF32Uniform(q, (size_t)B * q0, 1.f, 3, s);
    std::vector<int> hp(B), hsl(B);
    for (int b = 0; b < B; b++) hp[b] = pos, hsl[b] = b;
    int *dpos = (int *)alloc(B * 4), *dslot = (int *)alloc(B * 4);
    DL_HIP(hipMemcpyAsync(dpos, hp.data(), B * 4, hipMemcpyHostToDevice, s));
    DL_HIP(hipMemcpyAsync(dslot, hsl.data(), B * 4, hipMemcpyHostToDevice, s));
    hipk::AttnArgs a;
    a.q = q;
    a.ldq = q0;
    a.pos = dpos;
    a.slot = dslot;
    a.nHeads0 = nHeads0;
    a.kvMul = kvMul;
    a.hs = hs;
    a.kv0 = kv0;
    a.seqLen = seqLen;
    a.splitGrid = hipk::attnSplitGrid(seqLen);
    a.chunkMax = hipk::attnChunkMax(seqLen, a.splitGrid);
    a.chunkMin = hipk::attnChunkMin();
    a.partO = (float *)alloc((size_t)B * nHeads0 * a.splitGrid * hs * 4);
    a.partML = (float *)alloc((size_t)B * nHeads0 * a.splitGrid * 2 * 4);
    a.outQ = (int8_t *)alloc((size_t)B * q0);
    a.outS = (float2 *)alloc((size_t)B * q0 / 32 * 8);
    a.ldOut = q0;
    a.kvBf16 = kvBf16 ? 1 : 0;
    a.counters = (int *)alloc((size_t)B * nHeads0 * 4);
    DL_HIP(hipStreamSynchronize(s));
    auto launch = [&](int c) {
        a.kcache = kc[c % copies];
        a.vcache = vc[c % copies];
        hipk::launchAttention(a, B, s);
    };
    launch(0);
    DL_HIP(hipGetLastError());
    hipGraph_t g;
    hipGraphExec_t ge;
    DL_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < iters; i++) launch(i);
    DL_HIP(hipStreamEndCapture(s, &g));
    DL_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    DL_HIP(hipGraphLaunch(ge, s));
    DL_HIP(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    DL_HIP(hipEventCreate(&e0));
    DL_HIP(hipEventCreate(&e1));
    DL_HIP(hipEventRecord(e0, s));
    DL_HIP(hipGraphLaunch(ge, s));
    DL_HIP(hipEventRecord(e1, s));
    DL_HIP(hipEventSynchronize(e1));
    float ms = 0;
    DL_HIP(hipEventElapsedTime(&ms, e0, e1));
    if (trace) {  // one more (eager) launch with per-workgroup stamps (MFMA decode kernel)
        const size_t words = 8 * (size_t)(nHeads0 / kvMul) * a.splitGrid * B;
        a.trace = (unsigned long long *)alloc(words * 8);
        launch(iters);
        DL_HIP(hipStreamSynchronize(s));
        trace->resize(words);
        DL_HIP(hipMemcpy(trace->data(), a.trace, words * 8, hipMemcpyDeviceToHost));
    }
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (void *p : mem) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return ms * 1000.0 / iters;
}

}  // namespace dl

namespace dl {

// The separate-collective schedule of a tensor-parallel forward (engine_forward.cpp: per layer two
// Q80-rounded all-reduces of [rows][dim] partial sums, then the logits slices gathered to the root
// and the argmax winner pairs all-gathered), on `comm`, run eagerly or captured once into a hipGraph
// and replayed. Rank r contributes c * k(r, i) with integer k and c = 2^-4 (every Q80 block holds a
// 127 * c element, so the Q80 round trip and the sums are exact); returns the largest |got - want|
// over every output of every run (0 when the transport is right), checked on the host.
double commScheduleCheck(DeviceComm &comm, int layers, int rows, int dim, int vocab0, int runs, bool graph) {
    DL_CHECK(layers >= 1 && rows >= 1 && dim % 32 == 0 && vocab0 >= 1 && runs >= 1, "bad schedule shape");
    const int W = comm.size(), me = comm.rank();
    const float c = 1.0f / 16.0f;
    auto k = [](int r, size_t i) { return (i % 32) == 0 ? 127.f : (float)((int)((i * 37 + (size_t)r * 11) % 255) - 127); };
    const size_t ny = (size_t)rows * dim, nl = (size_t)rows * vocab0, np = 2 * (size_t)rows;
    std::vector<float> hy(ny), hl(nl), hp(np);
    for (size_t i = 0; i < ny; i++) hy[i] = c * k(me, i);
    for (size_t i = 0; i < nl; i++) hl[i] = (float)(me * 1000 + (int)(i % 997));
    for (size_t i = 0; i < np; i++) hp[i] = (float)(me * 7 + (int)i);
    hipStream_t s;
    DL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void *> mem;
    auto alloc = [&](size_t floats) {
        void *p;
        DL_HIP(hipMalloc(&p, floats * sizeof(float)));
        DL_HIP(hipMemset(p, 0, floats * sizeof(float)));
        mem.push_back(p);
        return (float *)p;
    };
    float *ySrc = alloc(ny), *y = alloc(ny), *outs = alloc(ny * layers), *lg = alloc(nl), *lgAll = alloc(nl * W);
    float *pr = alloc(np), *prAll = alloc(np * W);
    DL_HIP(hipMemcpy(ySrc, hy.data(), ny * 4, hipMemcpyHostToDevice));
    DL_HIP(hipMemcpy(lg, hl.data(), nl * 4, hipMemcpyHostToDevice));
    DL_HIP(hipMemcpy(pr, hp.data(), np * 4, hipMemcpyHostToDevice));
    auto schedule = [&]() {
        for (int l = 0; l < layers; l++) {
            DL_HIP(hipMemcpyAsync(y, ySrc, ny * 4, hipMemcpyDeviceToDevice, s));
            hipk::launchQ80Roundtrip(y, ny, s);
            comm.allReduceSum(y, ny, s);
            DL_HIP(hipMemcpyAsync(outs + (size_t)l * ny, y, ny * 4, hipMemcpyDeviceToDevice, s));
        }
        comm.gatherToRoot(lg, lgAll, nl, s);
        comm.allGather(pr, prAll, np, s);
    };
    hipGraphExec_t ge = nullptr;
    if (graph) {
        hipGraph_t g;
        DL_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        schedule();
        DL_HIP(hipStreamEndCapture(s, &g));
        DL_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
    }
    double err = 0;
    std::vector<float> got;
    for (int run = 0; run < runs; run++) {
        DL_HIP(hipMemsetAsync(outs, 0, ny * layers * 4, s));
        DL_HIP(hipMemsetAsync(lgAll, 0, nl * W * 4, s));
        DL_HIP(hipMemsetAsync(prAll, 0, np * W * 4, s));
        if (graph)
            DL_HIP(hipGraphLaunch(ge, s));
        else
            schedule();
        DL_HIP(hipStreamSynchronize(s));
        got.resize(ny * layers);
        DL_HIP(hipMemcpy(got.data(), outs, ny * layers * 4, hipMemcpyDeviceToHost));
        for (int l = 0; l < layers; l++)
            for (size_t i = 0; i < ny; i++) {
                float want = 0;
                for (int r = 0; r < W; r++) want += c * k(r, i);
                err = std::max(err, (double)std::fabs(got[(size_t)l * ny + i] - want));
            }
        if (me == 0) {
            got.resize(nl * W);
            DL_HIP(hipMemcpy(got.data(), lgAll, nl * W * 4, hipMemcpyDeviceToHost));
            for (int r = 0; r < W; r++)
                for (size_t i = 0; i < nl; i++)
                    err = std::max(err, (double)std::fabs(got[r * nl + i] - (float)(r * 1000 + (int)(i % 997))));
        }
        got.resize(np * W);
        DL_HIP(hipMemcpy(got.data(), prAll, np * W * 4, hipMemcpyDeviceToHost));
        for (int r = 0; r < W; r++)
            for (size_t i = 0; i < np; i++) err = std::max(err, (double)std::fabs(got[r * np + i] - (float)(r * 7 + (int)i)));
    }
    if (ge) (void)hipGraphExecDestroy(ge);
    for (void *p : mem) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return err;
}

}  // namespace dl
