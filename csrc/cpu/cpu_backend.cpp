// CPU reference backend.
//
// Semantics follow the reference's CPU ops (src/nn/nn-cpu-ops.cpp): invRms/rmsNorm (105-166),
// Q80xQ40 and F32 matmul (182-440), SiLU/GELU (445-491), RoPE over adjacent pairs (1090-1120),
// KV append at `pos` (1253-1275) and multi-head attention with GQA (749-784). It is the test
// oracle for the HIP engine and the `--nthreads` CPU path (BASELINE config #1). Differences
// from the reference, all deliberate: partial sums are exchanged in f32 (the reference quantizes
// them to Q80, llm.cpp:150); every row carries its own KV slot; GELU is honoured (Q6).
#include <cmath>
#include <cstring>
#include <vector>

#include "../core/quant.h"
#include "../runtime/backend.h"
#include "thread_pool.h"

namespace dl {

void LocalComm::gatherToRoot(const float *local, u64 nLocal, float *out) {
    if (out && out != local) std::memcpy(out, local, nLocal * sizeof(float));
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

    // y[r] = W[r,:] . x  for r in [0, rows)
    void matmul(const Mat &W, const Act &x, float *y) {
        if (W.type == FloatType::F32) {
            const float *w = (const float *)W.data;
            const float *xv = x.f.data();
            const u32 n = W.cols;
            pool_.parallelFor(W.rows, [&](long s, long e) {
                for (long r = s; r < e; r++) {
                    const float *wr = w + (u64)r * n;
                    float acc = 0.f;
                    for (u32 i = 0; i < n; i++) acc += wr[i] * xv[i];
                    y[r] = acc;
                }
            });
        } else {
            DL_CHECK(W.type == FloatType::Q40 && q80_, "Q40 matmul needs Q80 activations");
            const BlockQ40 *w = (const BlockQ40 *)W.data;
            const BlockQ80 *xq = x.q.data();
            const u32 nb = W.cols / kQBlock;
            std::vector<float> xd(nb);
            for (u32 b = 0; b < nb; b++) xd[b] = f16ToF32(xq[b].d);
            pool_.parallelFor(W.rows, [&](long s, long e) {
                for (long r = s; r < e; r++) {
                    const BlockQ40 *wr = w + (u64)r * nb;
                    float acc = 0.f;
                    for (u32 b = 0; b < nb; b++) {
                        int isum = 0;
                        for (int j = 0; j < 16; j++) {
                            const int lo = (wr[b].qs[j] & 0x0F) - 8;
                            const int hi = (wr[b].qs[j] >> 4) - 8;
                            isum += lo * xq[b].qs[j] + hi * xq[b].qs[j + 16];
                        }
                        acc += (float)isum * f16ToF32(wr[b].d) * xd[b];
                    }
                    y[r] = acc;
                }
            });
        }
    }

    static float invRms(const float *x, u32 n, float eps) {
        float s = 0.f;
        for (u32 i = 0; i < n; i++) s += x[i] * x[i];
        s /= (float)n;
        s += eps;
        return 1.0f / std::sqrt(s);
    }

    void rmsNorm(const float *x, const float *w, float *out) {
        const float inv = invRms(x, h_.dim, h_.normEpsilon);
        for (u32 i = 0; i < h_.dim; i++) out[i] = w[i] * (inv * x[i]);
    }

    // rotate pairs (i, i+1) of a vector whose element i sits at within-head index i % headSize
    void rope(float *v, u32 len, u32 pos) {
        const u32 hs = plan_.headSize, half = hs / 2;
        const float *t = &rope_[(u64)pos * half * 2];
        for (u32 i = 0; i < len; i += 2) {
            const u32 fi = (i % hs) / 2;
            const float c = t[fi * 2], s = t[fi * 2 + 1];
            const float v0 = v[i], v1 = v[i + 1];
            v[i] = v0 * c - v1 * s;
            v[i + 1] = v0 * s + v1 * c;
        }
    }

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
        std::vector<float> x((u64)n * dim), xn(dim), q((u64)n * p.q0), k(p.kv0), v(p.kv0);
        std::vector<float> att((u64)n * p.q0), y((u64)n * dim), hbuf(p.hidden0), gbuf(p.hidden0);
        std::vector<float> scores(h_.seqLen);
        Act a;
        for (int b = 0; b < n; b++) std::memcpy(&x[(u64)b * dim], emb_ + (u64)tokens[b] * dim, dim * sizeof(float));

        for (u32 l = 0; l < h_.nLayers; l++) {
            Layer &L = layers_[l];
            // attention block: norm -> q,k,v -> rope -> kv append (all rows first, then attention)
            for (int b = 0; b < n; b++) {
                rmsNorm(&x[(u64)b * dim], L.rmsAtt, xn.data());
                setAct(a, xn.data(), dim);
                matmul(L.wq, a, &q[(u64)b * p.q0]);
                matmul(L.wk, a, k.data());
                matmul(L.wv, a, v.data());
                rope(&q[(u64)b * p.q0], p.q0, positions[b]);
                rope(k.data(), p.kv0, positions[b]);
                std::memcpy(kc(l, slots[b], positions[b]), k.data(), p.kv0 * sizeof(float));
                std::memcpy(vc(l, slots[b], positions[b]), v.data(), p.kv0 * sizeof(float));
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
            for (int b = 0; b < n; b++) {
                setAct(a, &att[(u64)b * p.q0], p.q0);
                matmul(L.wo, a, &y[(u64)b * dim]);
            }
            Timer st;
            comm_->allReduceSum(y.data(), (u64)n * dim);
            syncMs += st.elapsedMs();
            for (u64 i = 0; i < (u64)n * dim; i++) x[i] += y[i];

            // feed-forward block
            for (int b = 0; b < n; b++) {
                rmsNorm(&x[(u64)b * dim], L.rmsFfn, xn.data());
                setAct(a, xn.data(), dim);
                matmul(L.w1, a, hbuf.data());
                matmul(L.w3, a, gbuf.data());
                for (u32 i = 0; i < p.hidden0; i++) {
                    const float z = hbuf[i];
                    float act;
                    if (h_.hiddenAct == HiddenAct::GELU)
                        act = 0.5f * z * (1.0f + std::tanh(0.79788456080286535588f * z * (1.0f + 0.044715f * z * z)));
                    else
                        act = z / (1.0f + std::exp(-z));
                    hbuf[i] = act * gbuf[i];
                }
                setAct(a, hbuf.data(), p.hidden0);
                matmul(L.w2, a, &y[(u64)b * dim]);
            }
            st.reset();
            comm_->allReduceSum(y.data(), (u64)n * dim);
            syncMs += st.elapsedMs();
            for (u64 i = 0; i < (u64)n * dim; i++) x[i] += y[i];
        }

        // final norm + vocab-sharded classifier, gathered to the root
        std::vector<float> lg((u64)n * p.vocab0);
        for (int b = 0; b < n; b++) {
            rmsNorm(&x[(u64)b * dim], rmsFinal_, xn.data());
            setAct(a, xn.data(), dim);
            matmul(wcls_, a, &lg[(u64)b * p.vocab0]);
        }
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
        stats_.computeMs = timer.elapsedMs() - syncMs;
        comm_->stats(stats_.sentBytes, stats_.recvBytes);
    }

    EngineConfig cfg_;
    HostComm *comm_;
    ThreadPool pool_;
    std::unique_ptr<ModelFile> file_;
    ModelHeader h_;
    ShardPlan plan_;
    bool q80_ = false;
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
