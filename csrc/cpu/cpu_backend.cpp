// CPU reference backend.
//
// Matmuls are AVX2/FMA (x86-64-v3) and batched: every weight row is read once per forward for all
// of its activation rows (the reference reaches the same reuse with vendored tinyBLAS for
// batch > 1, nn-cpu-ops.cpp:1000-1016 / sgemm.cpp; here one kernel serves decode and prefill).
// Q40 x Q80 blocks are int8 dot products (maddubs on |w| and sign-transferred x, exact int32 per
// block) scaled by d_w * d_x in f32, like matmul_Q80_Q40_F32 (nn-cpu-ops.cpp:222-440).
// Semantics follow the reference's CPU ops (src/nn/nn-cpu-ops.cpp): invRms/rmsNorm (105-166),
// Q80xQ40 and F32 matmul (182-440), SiLU/GELU (445-491), RoPE over adjacent pairs (1090-1120),
// KV append at `pos` (1253-1275) and multi-head attention with GQA (749-784). It is the test
// oracle for the HIP engine and the `--nthreads` CPU path (BASELINE config #1). Partial sums are
// exchanged in the reference's wire format by default: with `--buffer-float-type q80` the
// `--sync-type` is Q80 (every rank's partial quantized once to 32-value blocks, all ranks' blocks
// dequantized and summed in rank order, llm.cpp:150); `--sync-type f32` exchanges exact f32
// partials. Neither is bitwise TP=1: a rank-order sum of partials rounds differently from one
// accumulation (the tests bound the difference). Deliberate differences from the reference:
// every row carries its own KV slot; GELU is honoured (Q6).
#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "../core/quant.h"
#include "../runtime/backend.h"
#include "cpu_ops.h"
#include "thread_pool.h"

namespace dl {

void LocalComm::gatherToRoot(const float *local, u64 nLocal, float *out) {
    if (out && out != local) std::memcpy(out, local, nLocal * sizeof(float));
}

struct ThreadGroupComm::Group {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    u64 generation = 0;
    std::vector<const void *> ptr;
    std::vector<std::vector<BlockQ80>> q80;
    explicit Group(int w) : world(w), ptr(w), q80(w) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const u64 gen = generation;
        if (++arrived == world) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};

std::vector<std::unique_ptr<ThreadGroupComm>> ThreadGroupComm::make(int world) {
    auto g = std::make_shared<Group>(world);
    std::vector<std::unique_ptr<ThreadGroupComm>> out;
    for (int r = 0; r < world; r++) out.emplace_back(new ThreadGroupComm(g, r));
    return out;
}

int ThreadGroupComm::size() const { return g_->world; }

void ThreadGroupComm::allReduceSum(float *data, u64 n) {
    g_->ptr[rank_] = data;
    g_->barrier();
    tmp_.assign(n, 0.f);
    for (int r = 0; r < g_->world; r++) {
        const float *p = static_cast<const float *>(g_->ptr[r]);
        for (u64 i = 0; i < n; i++) tmp_[i] += p[i];
    }
    g_->barrier();  // every rank has read every partial before any overwrites its own
    std::memcpy(data, tmp_.data(), n * sizeof(float));
}

void ThreadGroupComm::allReduceSumQ80(float *data, u64 n) {
    DL_CHECK(n % kQBlock == 0, "Q80 sync needs 32-aligned vectors");
    auto &mine = g_->q80[rank_];
    mine.resize(n / kQBlock);
    quantizeQ80(data, mine.data(), n);
    g_->barrier();
    tmp_.resize(n);
    std::vector<float> acc(n, 0.f);
    for (int r = 0; r < g_->world; r++) {
        dequantizeQ80(g_->q80[r].data(), tmp_.data(), n);
        for (u64 i = 0; i < n; i++) acc[i] += tmp_[i];
    }
    g_->barrier();
    std::memcpy(data, acc.data(), n * sizeof(float));
}

void ThreadGroupComm::gatherToRoot(const float *local, u64 nLocal, float *out) {
    g_->ptr[rank_] = local;
    g_->barrier();
    if (rank_ == 0 && out)
        for (int r = 0; r < g_->world; r++)
            std::memcpy(out + (u64)r * nLocal, g_->ptr[r], nLocal * sizeof(float));
    g_->barrier();
}

namespace {

struct Mat {
    const u8 *data = nullptr;  // row-major [rows][cols] of `type`
    FloatType type = FloatType::F32;
    u32 rows = 0, cols = 0;
    std::vector<u8> owned;
};

struct Layer {
    Mat wq, wk, wv, wo, w1, w2, w3;
    const float *rmsAtt = nullptr, *rmsFfn = nullptr;
};

// Activation vector, optionally quantized to Q80.
struct Act {
    std::vector<float> f;
    std::vector<BlockQ80> q;
};

class CpuBackend : public Backend {
  public:
    CpuBackend(const EngineConfig &cfg, HostComm *comm) : cfg_(cfg), comm_(comm), pool_(cfg.nThreads) {
        DL_CHECK(!cfg.synthetic, "CPU backend needs a model file");
        file_.reset(new ModelFile(cfg.modelPath, cfg.maxSeqLen));
        h_ = file_->header();
        plan_ = ShardPlan::make(h_, comm_->size(), comm_->rank());
        q80_ = cfg.bufferType == FloatType::Q80;
        DL_CHECK(cfg.syncType == FloatType::F32 || cfg.syncType == FloatType::Q80, "sync type must be f32 or q80");
        syncQ80_ = cfg.syncType == FloatType::Q80;
        if (h_.weightType == FloatType::Q40 && !q80_)
            throw Error("This version supports only Q40 weights with Q80 sync type");
        if (h_.weightType == FloatType::F32 && q80_)
            throw Error("F32 weights require --buffer-float-type f32");
        load();
        rope_ = buildRopeTable(h_);
        const u64 kvPerLayer = (u64)cfg_.nSlots * h_.seqLen * plan_.kv0;
        kcache_.assign(kvPerLayer * h_.nLayers, 0.f);
        vcache_.assign(kvPerLayer * h_.nLayers, 0.f);
    }

    const ModelHeader &header() const override { return h_; }
    const ShardPlan &plan() const override { return plan_; }
    std::string name() const override { return "cpu"; }

    void forward(int n, const int *tokens, const int *positions, const int *slots, float *logits) override {
        std::vector<float> full;
        forwardImpl(n, tokens, positions, slots, logits);
    }

    void forwardArgmax(int n, const int *tokens, const int *positions, const int *slots, int *out) override {
        std::vector<float> logits;
        if (comm_->rank() == 0) logits.resize((u64)n * h_.vocabSize);
        forwardImpl(n, tokens, positions, slots, comm_->rank() == 0 ? logits.data() : nullptr);
        std::vector<float> ids(n, 0.f);
        if (comm_->rank() == 0)
            for (int i = 0; i < n; i++) ids[i] = (float)argmaxRow(&logits[(u64)i * h_.vocabSize]);
        // broadcast the ids through the all-reduce (non-root ranks contribute zeros)
        comm_->allReduceSum(ids.data(), n);
        for (int i = 0; i < n; i++) out[i] = (int)ids[i];
    }

  private:
    int argmaxRow(const float *x) const {
        int best = 0;
        for (u32 i = 1; i < h_.vocabSize; i++)
            if (x[i] > x[best]) best = (int)i;
        return best;
    }

    void makeMat(Mat &m, const TensorInfo &t, bool rowSlice, u32 start, u32 count) {
        m.type = t.type;
        if (rowSlice) {
            m.rows = count;
            m.cols = t.cols;
            if (plan_.nRanks == 1) {
                m.data = file_->ptr(t);
                return;
            }
            m.owned.resize(floatTypeBytes(t.type, (u64)count * t.cols));
            sliceRows(file_->ptr(t), t.type, t.cols, start, count, m.owned.data());
        } else {
            m.rows = t.rows;
            m.cols = count;
            if (plan_.nRanks == 1) {
                m.data = file_->ptr(t);
                return;
            }
            m.owned.resize(floatTypeBytes(t.type, (u64)t.rows * count));
            sliceCols(file_->ptr(t), t.type, t.rows, t.cols, start, count, m.owned.data());
        }
        m.data = m.owned.data();
    }

    void load() {
        const ShardPlan &p = plan_;
        layers_.resize(h_.nLayers);
        for (u32 l = 0; l < h_.nLayers; l++) {
            Layer &L = layers_[l];
            makeMat(L.wq, file_->find(TensorKind::WQ, l), true, p.qStart(), p.q0);
            makeMat(L.wk, file_->find(TensorKind::WK, l), true, p.kvStart(), p.kv0);
            makeMat(L.wv, file_->find(TensorKind::WV, l), true, p.kvStart(), p.kv0);
            makeMat(L.wo, file_->find(TensorKind::WO, l), false, p.qStart(), p.q0);
            makeMat(L.w1, file_->find(TensorKind::W1, l), true, p.hiddenStart(), p.hidden0);
            makeMat(L.w2, file_->find(TensorKind::W2, l), false, p.hiddenStart(), p.hidden0);
            makeMat(L.w3, file_->find(TensorKind::W3, l), true, p.hiddenStart(), p.hidden0);
            L.rmsAtt = (const float *)file_->ptr(file_->find(TensorKind::RMS_ATT, l));
            L.rmsFfn = (const float *)file_->ptr(file_->find(TensorKind::RMS_FFN, l));
        }
        emb_ = (const float *)file_->ptr(file_->find(TensorKind::EMBEDDING, -1));
        rmsFinal_ = (const float *)file_->ptr(file_->find(TensorKind::RMS_FINAL, -1));
        makeMat(wcls_, file_->find(TensorKind::WCLS, -1), true, p.vocabStart(), p.vocab0);
    }

    void setAct(Act &a, const float *x, u32 n) {
        a.f.assign(x, x + n);
        if (q80_) {
            a.q.resize(n / kQBlock);
            quantizeQ80(x, a.q.data(), n);
        }
    }

    void matmul(const Mat &W, const Act *const *xs, int B, float *const *ys) {
        if (W.type == FloatType::F32) {
            std::vector<const float *> xf(B);
            for (int t = 0; t < B; t++) xf[t] = xs[t]->f.data();
            cpu::matmulF32((const float *)W.data, W.rows, W.cols, xf.data(), B, ys, pool_);
            return;
        }
        DL_CHECK(W.type == FloatType::Q40 && q80_, "Q40 matmul needs Q80 activations");
        std::vector<const BlockQ80 *> xq(B);
        for (int t = 0; t < B; t++) xq[t] = xs[t]->q.data();
        cpu::matmulQ40Q80((const BlockQ40 *)W.data, W.rows, W.cols, xq.data(), B, ys, pool_);
    }

    void allReduce(float *y, u64 n) {
        if (syncQ80_)
            comm_->allReduceSumQ80(y, n);
        else
            comm_->allReduceSum(y, n);
    }

    void rmsNorm(const float *x, const float *w, float *out) {
        const float inv = cpu::invRms(x, h_.dim, h_.normEpsilon);
        for (u32 i = 0; i < h_.dim; i++) out[i] = w[i] * (inv * x[i]);
    }

    void rope(float *v, u32 len, u32 pos) { cpu::ropeApply(v, len, pos, plan_.headSize, rope_.data()); }

    float *kc(u32 layer, int slot, u32 pos) {
        return &kcache_[(((u64)layer * cfg_.nSlots + slot) * h_.seqLen + pos) * plan_.kv0];
    }
    float *vc(u32 layer, int slot, u32 pos) {
        return &vcache_[(((u64)layer * cfg_.nSlots + slot) * h_.seqLen + pos) * plan_.kv0];
    }

    void forwardImpl(int n, const int *tokens, const int *positions, const int *slots, float *logitsOut) {
        Timer timer;
        double syncMs = 0;
        const u32 dim = h_.dim, hs = plan_.headSize;
        const ShardPlan &p = plan_;
        for (int b = 0; b < n; b++) {
            DL_CHECK(positions[b] >= 0 && (u32)positions[b] < h_.seqLen, "position out of range");
            DL_CHECK(slots[b] >= 0 && (u32)slots[b] < cfg_.nSlots, "slot out of range");
            DL_CHECK(tokens[b] >= 0 && (u32)tokens[b] < h_.vocabSize, "token out of range");
        }
        std::vector<float> x((u64)n * dim), xn(dim), q((u64)n * p.q0), k((u64)n * p.kv0), v((u64)n * p.kv0);
        std::vector<float> att((u64)n * p.q0), y((u64)n * dim), hbuf((u64)n * p.hidden0), gbuf((u64)n * p.hidden0);
        std::vector<Act> acts(n);
        std::vector<const Act *> ap(n);
        for (int b = 0; b < n; b++) ap[b] = &acts[b];
        // row pointers of an [n][width] buffer
        auto rows = [n](std::vector<float> &buf, u32 width) {
            std::vector<float *> r(n);
            for (int b = 0; b < n; b++) r[b] = &buf[(u64)b * width];
            return r;
        };
        const std::vector<float *> qR = rows(q, p.q0), kR = rows(k, p.kv0), vR = rows(v, p.kv0), yR = rows(y, dim),
                                   hR = rows(hbuf, p.hidden0), gR = rows(gbuf, p.hidden0);
        for (int b = 0; b < n; b++) std::memcpy(&x[(u64)b * dim], emb_ + (u64)tokens[b] * dim, dim * sizeof(float));

        for (u32 l = 0; l < h_.nLayers; l++) {
            Layer &L = layers_[l];
            // attention block: norm -> q,k,v (one pass over each weight for all rows) -> rope ->
            // kv append (all rows first, then attention)
            for (int b = 0; b < n; b++) {
                rmsNorm(&x[(u64)b * dim], L.rmsAtt, xn.data());
                setAct(acts[b], xn.data(), dim);
            }
            matmul(L.wq, ap.data(), n, qR.data());
            matmul(L.wk, ap.data(), n, kR.data());
            matmul(L.wv, ap.data(), n, vR.data());
            for (int b = 0; b < n; b++) {
                rope(qR[b], p.q0, positions[b]);
                rope(kR[b], p.kv0, positions[b]);
                std::memcpy(kc(l, slots[b], positions[b]), kR[b], p.kv0 * sizeof(float));
                std::memcpy(vc(l, slots[b], positions[b]), vR[b], p.kv0 * sizeof(float));
            }
            const float scale = 1.0f / std::sqrt((float)hs);
            for (int b = 0; b < n; b++) {
                const u32 pos = positions[b];
                const int slot = slots[b];
                pool_.parallelFor(p.nHeads0, [&](long hs0, long hs1) {
                    std::vector<float> sc(pos + 1);
                    for (long h = hs0; h < hs1; h++) {
                        const float *qh = &q[(u64)b * p.q0 + h * hs];
                        const u32 kvh = (u32)h / p.kvMul;
                        for (u32 t = 0; t <= pos; t++) {
                            const float *kt = kc(l, slot, t) + kvh * hs;
                            float d = 0.f;
                            for (u32 i = 0; i < hs; i++) d += qh[i] * kt[i];
                            sc[t] = d * scale;
                        }
                        float mx = sc[0];
                        for (u32 t = 1; t <= pos; t++) mx = std::fmax(mx, sc[t]);
                        float sum = 0.f;
                        for (u32 t = 0; t <= pos; t++) {
                            sc[t] = std::exp(sc[t] - mx);
                            sum += sc[t];
                        }
                        float *o = &att[(u64)b * p.q0 + h * hs];
                        std::memset(o, 0, hs * sizeof(float));
                        for (u32 t = 0; t <= pos; t++) {
                            const float w = sc[t] / sum;
                            const float *vt = vc(l, slot, t) + kvh * hs;
                            for (u32 i = 0; i < hs; i++) o[i] += w * vt[i];
                        }
                    }
                });
            }
            for (int b = 0; b < n; b++) setAct(acts[b], &att[(u64)b * p.q0], p.q0);
            matmul(L.wo, ap.data(), n, yR.data());
            Timer st;
            allReduce(y.data(), (u64)n * dim);
            syncMs += st.elapsedMs();
            for (u64 i = 0; i < (u64)n * dim; i++) x[i] += y[i];

            // feed-forward block
            for (int b = 0; b < n; b++) {
                rmsNorm(&x[(u64)b * dim], L.rmsFfn, xn.data());
                setAct(acts[b], xn.data(), dim);
            }
            matmul(L.w1, ap.data(), n, hR.data());
            matmul(L.w3, ap.data(), n, gR.data());
            for (int b = 0; b < n; b++) {
                float *hb = hR[b];
                const float *gb = gR[b];
                for (u32 i = 0; i < p.hidden0; i++) {
                    const float z = hb[i];
                    const float act = h_.hiddenAct == HiddenAct::GELU ? cpu::gelu(z) : cpu::silu(z);
                    hb[i] = act * gb[i];
                }
                setAct(acts[b], hb, p.hidden0);
            }
            matmul(L.w2, ap.data(), n, yR.data());
            st.reset();
            allReduce(y.data(), (u64)n * dim);
            syncMs += st.elapsedMs();
            for (u64 i = 0; i < (u64)n * dim; i++) x[i] += y[i];
        }

        // final norm + vocab-sharded classifier, gathered to the root
        std::vector<float> lg((u64)n * p.vocab0);
        const std::vector<float *> lR = rows(lg, p.vocab0);
        for (int b = 0; b < n; b++) {
            rmsNorm(&x[(u64)b * dim], rmsFinal_, xn.data());
            setAct(acts[b], xn.data(), dim);
        }
        matmul(wcls_, ap.data(), n, lR.data());
        Timer st;
        if (comm_->size() == 1) {
            if (logitsOut) std::memcpy(logitsOut, lg.data(), lg.size() * sizeof(float));
        } else {
            // gather rank-major [rank][n][vocab0] then transpose to [n][vocab]
            std::vector<float> g(comm_->rank() == 0 ? (u64)n * h_.vocabSize : 0);
            comm_->gatherToRoot(lg.data(), lg.size(), comm_->rank() == 0 ? g.data() : nullptr);
            if (comm_->rank() == 0 && logitsOut) {
                for (u32 r = 0; r < p.nRanks; r++)
                    for (int b = 0; b < n; b++)
                        std::memcpy(&logitsOut[(u64)b * h_.vocabSize + (u64)r * p.vocab0],
                                    &g[((u64)r * n + b) * p.vocab0], p.vocab0 * sizeof(float));
            }
        }
        syncMs += st.elapsedMs();
        stats_.syncMs = syncMs;
        stats_.xchgMs = syncMs;  // the whole exchange step is timed (reference nn-executor.cpp:150-155)
        stats_.computeMs = timer.elapsedMs() - syncMs;
        comm_->stats(stats_.sentBytes, stats_.recvBytes);
    }

    EngineConfig cfg_;
    HostComm *comm_;
    ThreadPool pool_;
    std::unique_ptr<ModelFile> file_;
    ModelHeader h_;
    ShardPlan plan_;
    bool q80_ = false, syncQ80_ = false;
    std::vector<Layer> layers_;
    const float *emb_ = nullptr, *rmsFinal_ = nullptr;
    Mat wcls_;
    std::vector<float> rope_;
    std::vector<float> kcache_, vcache_;
};

}  // namespace

std::unique_ptr<Backend> makeCpuBackend(const EngineConfig &cfg, HostComm *comm) {
    static LocalComm local;
    return std::unique_ptr<Backend>(new CpuBackend(cfg, comm ? comm : &local));
}

}  // namespace dl
