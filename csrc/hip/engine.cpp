// HipEngine implementation (host side).
//
// Weight residency: every rank repacks ITS shard of the mmapped `.m` file on the host into the
// GPU layout and uploads it once (reference: root streams shards to workers over TCP,
// nn-network.cpp:766-901; llm.cpp:447-483 defines the slices). Q40 matrices become SoA
// (16-byte nibble rows + f16 scale plane) so a lane's 16-byte load is one whole block.
// Fusions baked into the layout:
//   Wq|Wk|Wv row slices concatenated -> one QKV GEMV (+RoPE +KV append epilogue)
//   W1/W3 row slices interleaved      -> one GEMV whose epilogue computes act(w1 x) * (w3 x)
#include "engine.h"

#include <cstdlib>

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <unordered_set>
#include <vector>

#include "../core/quant.h"
#include "../runtime/metrics.h"
#include "kernels.h"

namespace dl {


int hipDeviceCount() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

namespace {

struct DevMat {
    uint8_t *qs = nullptr;  // Q40: tiled for `lanes` lanes per row (hipk::Q40Tiling)
    uint16_t *d = nullptr;
    float *f = nullptr;
    int rows = 0, n = 0, lanes = 0;
};

struct DevLayer {
    DevMat qkv, wo, w13, w2;
    float *rmsAtt = nullptr, *rmsFfn = nullptr;
    void *k = nullptr, *v = nullptr;
};

class HipEngineImpl : public HipEngine {
  public:
    HipEngineImpl(const EngineConfig &cfg, DeviceComm *comm) : cfg_(cfg), comm_(comm) {
        const int nDev = hipDeviceCount();
        if (nDev <= 0) throw Error("No HIP device available");
        dev_ = cfg.gpuIndex >= 0 ? cfg.gpuIndex : 0;
        DL_CHECK(dev_ < nDev, "gpu index out of range");
        DL_HIP(hipSetDevice(dev_));
        DL_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));

        const u32 nRanks = comm_ ? comm_->size() : 1, rank = comm_ ? comm_->rank() : 0;
        if (cfg.synthetic) {
            h_ = cfg.syntheticHeader;
            h_.origSeqLen = h_.seqLen;
            if (cfg.maxSeqLen > 0 && h_.seqLen > cfg.maxSeqLen) h_.seqLen = cfg.maxSeqLen;
        } else {
            file_.reset(new ModelFile(cfg.modelPath, cfg.maxSeqLen));
            h_ = file_->header();
        }
        plan_ = ShardPlan::make(h_, nRanks, rank);
        q40_ = h_.weightType == FloatType::Q40;
        if (q40_ && cfg.bufferType != FloatType::Q80)
            throw Error("This version supports only Q40 weights with Q80 sync type");
        if (!q40_ && h_.weightType != FloatType::F32) throw Error("unsupported weight type");
        DL_CHECK(h_.headSize() == 64 || h_.headSize() == 128, "GPU kernels support head size 64 or 128");
        DL_CHECK(cfg.maxBatch >= 1 && cfg.nSlots >= 1, "maxBatch/nSlots");
        kvBf16_ = cfg.kvBf16;
        syncQ80_ = cfg.syncType == FloatType::Q80;
        if (comm_ && plan_.nRanks > 1) {
            const char *e = std::getenv("DL_TP_FUSED");  // 0: separate all-reduce kernels (comparison)
            tpFused_ = !(e && *e == '0') && comm_->fusedXchg(0, &tpVec_) && comm_->fusedXchg(1, &tpArg_) &&
                       (size_t)std::min<u32>(cfg.maxBatch, 4) * h_.dim <= (size_t)tpVec_.stride &&
                       (size_t)2 * cfg.maxBatch <= (size_t)tpArg_.stride;
            tpVec_.q80 = syncQ80_ ? 1 : 0;
        }
        checkFits();
        if (tpFused_) checkFusedResidency();
        {  // path knobs, read once: a captured graph replays the path it was captured with
            const char *e = std::getenv("DL_GEMM_MIN");
            gemmMin_ = e && *e ? std::atoi(e) : (plan_.nRanks > 1 ? 5 : 3);
            const char *f = std::getenv("DL_GEMM_FUSE_NORM");
            fuseNormEnv_ = !(f && *f == '0');
        }
        Timer timer;
        allocBuffers();
        if (cfg.synthetic)
            loadSynthetic();
        else
            loadFromFile();
        uploadRope();
        DL_HIP(hipStreamSynchronize(stream_));
        setupAttnBlock();
        setupFfnBlock();
        setupUn();
        hipk::preloadModules();  // no code-object load inside the first forwards
        load_.ms = timer.elapsedMs();
        load_.deviceBytes = deviceBytes_;
    }

    LoadStats loadStats() const override { return load_; }

    // ---------------------------------------------------------------- paged KV cache
    // With cfg.kvPages > 0 each layer's K / V cache is a pool of kvPages pages of kvPageSize
    // positions and a page table maps (slot, pos) to a pool row (kernels.h KvMap): a slot holds only
    // the pages its sequence reached, so many slots can share HBM sized for the tokens actually in
    // flight instead of nSlots x seqLen. Pages are mapped at setInputs for every position a forward
    // (or a decode chain) writes and released when a slot restarts at position 0: the same
    // deterministic rule on every tensor-parallel rank, so no page messages are exchanged.
    size_t kvPoolRows() const {
        return cfg_.kvPages ? (size_t)cfg_.kvPages * cfg_.kvPageSize : (size_t)cfg_.nSlots * h_.seqLen;
    }
    bool paged() const { return cfg_.kvPages > 0; }
    int kvPagesFree() const override { return paged() ? (int)freePages_.size() : -1; }
    int kvPageSize() const override { return paged() ? (int)cfg_.kvPageSize : 0; }
    void releaseSlot(int slot) override {
        if (!paged() || slot < 0 || (u32)slot >= cfg_.nSlots) return;
        for (int i = 0; i < slotPages_[slot]; i++) {
            int &e = hostTable_[(size_t)slot * pagesPerSlot_ + i];
            freePages_.push_back(e);
            e = -1;
        }
        if (slotPages_[slot]) tableDirty_ = true;  // uploaded with the next forward's mapping
        slotPages_[slot] = 0;
    }
    void setupPages() {
        if (!paged()) return;
        const u32 P = cfg_.kvPageSize;
        DL_CHECK(P >= 32 && (P & (P - 1)) == 0, "--kv-page-size must be a power of two >= 32");
        pageShift_ = 0;
        while ((1u << pageShift_) < P) pageShift_++;
        pagesPerSlot_ = (int)((h_.seqLen + P - 1) / P);
        const size_t entries = (size_t)cfg_.nSlots * pagesPerSlot_;
        hostTable_.assign(entries, -1);
        slotPages_.assign(cfg_.nSlots, 0);
        for (int pg = (int)cfg_.kvPages - 1; pg >= 0; pg--) freePages_.push_back(pg);
        dKvTable_ = dalloc<int>(entries);
        // unmapped entries read page 0 (valid memory, masked out): never a stray address
        DL_HIP(hipMemsetAsync(dKvTable_, 0, entries * sizeof(int), stream_));
        for (int i = 0; i < 2; i++) hTableStage_[i] = halloc<int>(entries);
    }
    hipk::KvMap kvMap() const {
        hipk::KvMap m;
        if (paged()) {
            m.table = dKvTable_;
            m.pageShift = pageShift_;
            m.pagesPerSlot = pagesPerSlot_;
        }
        return m;
    }
    // Map the pages every row's positions [pos, pos + ahead] need; a row at position 0 starts a new
    // sequence in its slot and releases the slot's old pages first. Uploads the table if it changed
    // (stream-ordered before the forward that reads it).
    void mapPages(int n, const int *positions, const int *slots, int ahead) {
        if (!paged()) return;
        bool dirty = tableDirty_;
        tableDirty_ = false;
        auto release = [&](int s) {
            for (int i = 0; i < slotPages_[s]; i++) {
                int &e = hostTable_[(size_t)s * pagesPerSlot_ + i];
                freePages_.push_back(e);
                e = -1;
            }
            if (slotPages_[s]) dirty = true;
            slotPages_[s] = 0;
        };
        for (int b = 0; b < n; b++)
            if (positions[b] == 0) release(slots[b]);
        for (int b = 0; b < n; b++) {
            const int s = slots[b];
            const int need = std::min(pagesPerSlot_, ((positions[b] + ahead) >> pageShift_) + 1);
            while (slotPages_[s] < need) {
                if (freePages_.empty())
                    throw Error("KV page pool exhausted: " + std::to_string(cfg_.kvPages) + " pages of " +
                                std::to_string(cfg_.kvPageSize) + " positions are all mapped; raise --kv-pages " +
                                "or lower the concurrent context");
                hostTable_[(size_t)s * pagesPerSlot_ + slotPages_[s]++] = freePages_.back();
                freePages_.pop_back();
                dirty = true;
            }
        }
        if (!dirty) return;
        // a pinned copy per upload, alternating: the previous upload may still be reading the other
        int *st = hTableStage_[tableFlip_ ^= 1];
        if (inputsInFlight_) DL_HIP(hipStreamSynchronize(stream_));
        for (size_t i = 0; i < hostTable_.size(); i++) st[i] = hostTable_[i] < 0 ? 0 : hostTable_[i];
        DL_HIP(hipMemcpyAsync(dKvTable_, st, hostTable_.size() * sizeof(int), hipMemcpyHostToDevice, stream_));
    }

    // Refuse a configuration whose weights + KV cache cannot be resident, with the numbers, before
    // allocating anything (KV is preallocated as nSlots x seqLen per layer).
    void checkFits() {
        size_t freeB = 0, totalB = 0;
        DL_HIP(hipMemGetInfo(&freeB, &totalB));
        const ShardPlan &p = plan_;
        const double GB = 1e9;
        const size_t kv = (size_t)h_.nLayers * 2 * kvPoolRows() * p.kv0 * (kvBf16_ ? 2 : 4);
        size_t w = (size_t)h_.nLayers * (matStageBytes(p.q0 + 2 * p.kv0, h_.dim) + matStageBytes(h_.dim, p.q0) +
                                         matStageBytes(2 * p.hidden0, h_.dim) + matStageBytes(h_.dim, p.hidden0));
        w += matStageBytes(p.vocab0, h_.dim) + (size_t)h_.vocabSize * h_.dim * 4;
        const size_t act = (size_t)cfg_.maxBatch * h_.vocabSize * 4 * 3 + ((size_t)256 << 20);
        if (kv + w + act > freeB) {
            // the page pool that would fit (positions shared by all slots), as a hint
            const size_t perPos = (size_t)h_.nLayers * 2 * p.kv0 * (kvBf16_ ? 2 : 4);
            const long long spare = (long long)freeB - (long long)(w + act);
            const long long pages = spare > 0 ? spare / (long long)(perPos * cfg_.kvPageSize) : 0;
            char msg[768];
            std::snprintf(msg, sizeof(msg), "Model does not fit on GPU %d: weights %.2f GB + KV cache %.2f GB (%s x %u "
                                  "layers, %s) + buffers %.2f GB > %.2f GB free of %.2f GB. Lower "
                                  "--max-seq-len or the number of slots, add tensor-parallel ranks, or use a paged "
                                  "KV cache sized to the tokens in flight (--kv-pages %lld fits %lld positions).",
                                  dev_, w / GB, kv / GB,
                                  paged() ? (std::to_string(cfg_.kvPages) + " pages").c_str()
                                          : (std::to_string(cfg_.nSlots) + " slots x " + std::to_string(h_.seqLen) +
                                             " positions").c_str(),
                                  h_.nLayers, kvBf16_ ? "bf16" : "f32", act / GB, freeB / GB, totalB / GB, pages,
                                  pages * (long long)cfg_.kvPageSize);
            throw Error(msg);
        }
    }

    // The fused TP exchange spins inside the wo / w2 GEMV workgroups until every peer published the
    // same rows: deadlock-free only if every workgroup of such a launch is resident at once (a
    // waiting workgroup must never keep a peer's producer, or its own rank's later workgroups, off
    // the CUs). Check every launch shape the fused path can take against the device's occupancy
    // (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs at the launch's LDS size); if any would
    // not fit, fall back to the separate all-reduce kernels, whose grids are a few workgroups.
    void checkFusedResidency() {
        const ShardPlan &p = plan_;
        // ranks sharing this GPU (same-GPU rehearsals) share its resident slots; DL_FUSED_RESIDENT
        // overrides the limit (diagnostics / tests of the fallback)
        const int share = std::max(1, comm_->ranksOnDevice());
        const char *ov = std::getenv("DL_FUSED_RESIDENT");
        const bool hQ80 = p.hidden0 / 32 >= 192;
        struct Shape {
            int rows, n, pro;
        } shapes[2] = {{(int)h_.dim, (int)p.q0, hipk::PRO_GLOBAL},
                       {(int)h_.dim, (int)p.hidden0, hQ80 ? hipk::PRO_GLOBAL : hipk::PRO_RESNORM}};
        for (const Shape &sh : shapes) {
            DevMat m;
            m.rows = sh.rows;
            m.n = sh.n;
            m.lanes = hipk::gemvLanesPerRow(sh.n, sh.rows, 1, true);
            const int bcMax = std::min<int>(batchChunk(m, sh.pro, hipk::EPI_STORE_TP), (int)cfg_.maxBatch);
            for (int bc = 1; bc <= bcMax; bc *= 2) {
                hipk::GemvArgs a;
                a.rows = m.rows;
                a.n = m.n;
                a.lanes = m.lanes;
                a.passes = tpPasses(m, bc);
                a.tp = tpVec_;
                const hipk::GemvResidency r = hipk::gemvResidency(a, bc, sh.pro, hipk::EPI_STORE_TP, true);
                const int limit = ov && *ov ? std::atoi(ov) : r.maxResident / share;
                fusedGridMax_ = std::max(fusedGridMax_, r.grid);
                if (limit <= 0 || r.grid > limit) {
                    std::fprintf(stderr,
                                 "⚠️  fused TP exchange disabled: a %dx%d GEMV at batch %d needs %d co-resident "
                                 "workgroups, this rank may hold %d (%d per device, %d rank(s) on it); using "
                                 "separate all-reduce kernels\n",
                                 sh.rows, sh.n, bc, r.grid, limit, r.maxResident, share);
                    tpFused_ = false;
                    return;
                }
            }
        }
    }
    int tpPasses(const DevMat &m, int bc) const {
        int passes = passesFor(m, hipk::EPI_STORE_TP, bc);
        if (tpVec_.q80)  // whole Q80 blocks of 32 rows per workgroup
            while ((256 / m.lanes * 2 * passes) % 32) passes++;
        return passes;
    }

  public:
    bool tpFused() const override { return tpFused_; }
    bool attnBlock() const override { return blockOn_; }
    bool unNorm() const override { return unOn_; }
    bool ffnBlock() const override { return ffnOn_; }
    std::vector<unsigned long long> traceAttnBlock(int token, int pos, int slot, int layer, bool ffn) override {
        if (ffn ? !ffnOn_ : !blockOn_) return {};
        int g[3] = {0, 0, 0};
        if (ffn) {
            const hipk::FfnBlockPlan pl = hipk::ffnBlockPlan(ffnBlockArgs(layers_[0], 0, 0), fusedTp(false));
            g[0] = pl.g13;
            g[2] = pl.g2;
        } else {
            const hipk::AttnBlockPlan pl = hipk::attnBlockPlan(attnBlockArgs(layers_[0], 0, 0), fusedTp(false));
            g[0] = pl.gq;
            g[1] = pl.ga;
            g[2] = pl.gw;
        }
        const size_t words = 8 * (size_t)(g[0] + g[1] + g[2]);
        traceBuf_ = dalloc<unsigned long long>(words);
        DL_HIP(hipMemsetAsync(traceBuf_, 0, words * 8, stream_));
        traceLayer_ = layer;
        traceFfn_ = ffn;
        setInputs(1, &token, &pos, &slot);
        enqueueForward(1, GraphKind::LOGITS);
        syncAndCheckComm();
        inputsInFlight_ = false;
        std::vector<unsigned long long> out(3 + words);
        for (int i = 0; i < 3; i++) out[i] = (unsigned long long)g[i];
        DL_HIP(hipMemcpy(out.data() + 3, traceBuf_, words * 8, hipMemcpyDeviceToHost));
        traceLayer_ = -1;
        traceFfn_ = false;
        traceBuf_ = nullptr;  // (one small buffer per call, released with the engine)
        return out;
    }
    int fusedGridMax() const override { return fusedGridMax_; }

    ~HipEngineImpl() override {
        (void)hipSetDevice(dev_);
        for (auto &kv : graphs_) (void)hipGraphExecDestroy(kv.second);
        for (void *p : allocs_) (void)hipFree(p);
        for (void *p : hostAllocs_) (void)hipHostFree(p);
        if (stream_) (void)hipStreamDestroy(stream_);
    }

    const ModelHeader &header() const override { return h_; }
    const ShardPlan &plan() const override { return plan_; }
    std::string name() const override { return "hip"; }
    size_t deviceBytes() const override { return deviceBytes_; }
    void synchronize() override { DL_HIP(hipStreamSynchronize(stream_)); }

    void forward(int n, const int *tokens, const int *positions, const int *slots, float *logits) override {
        Timer t;
        setInputs(n, tokens, positions, slots);
        runGraph(n, GraphKind::LOGITS);
        const bool root = rank() == 0;
        if (root && logits) {
            const float *src = plan_.nRanks > 1 ? dLogitsFull_ : dLogits_;
            DL_HIP(hipMemcpyAsync(hLogits_, src, (size_t)n * h_.vocabSize * sizeof(float), hipMemcpyDeviceToHost,
                                  stream_));
        }
        syncAndCheckComm();
        inputsInFlight_ = false;
        if (root && logits) std::memcpy(logits, hLogits_, (size_t)n * h_.vocabSize * sizeof(float));
        stats_.computeMs = t.elapsedMs();
        stats_.syncMs = 0;
    }

    void forwardArgmax(int n, const int *tokens, const int *positions, const int *slots, int *out) override {
        Timer t;
        setInputs(n, tokens, positions, slots);
        runGraph(n, GraphKind::ARGMAX);
        DL_HIP(hipMemcpyAsync(hIds_, dIds_, n * sizeof(int), hipMemcpyDeviceToHost, stream_));
        syncAndCheckComm();
        inputsInFlight_ = false;
        std::memcpy(out, hIds_, n * sizeof(int));
        stats_.computeMs = t.elapsedMs();
    }

    void forwardSample(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs,
                       int *out) override {
        Timer t;
        setInputs(n, tokens, positions, slots, specs);
        runGraph(n, GraphKind::SAMPLE);
        DL_HIP(hipMemcpyAsync(hIds_, dIds_, n * sizeof(int), hipMemcpyDeviceToHost, stream_));
        syncAndCheckComm();
        inputsInFlight_ = false;
        std::memcpy(out, hIds_, n * sizeof(int));
        stats_.computeMs = t.elapsedMs();
    }

    // Pipelined serving: the forward and the D2H copy of its ids are enqueued; the host returns at
    // once (inputs are staged in pinned memory: the previous forward was collected before).
    void launchIds(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs) override {
        DL_CHECK(pendingN_ == 0, "launchIds: the previous forward was not collected");
        Timer t;
        setInputs(n, tokens, positions, slots, specs);
        runGraph(n, specs ? GraphKind::SAMPLE : GraphKind::ARGMAX);
        DL_HIP(hipMemcpyAsync(hIds_, dIds_, n * sizeof(int), hipMemcpyDeviceToHost, stream_));
        pendingN_ = n;
        stats_.computeMs = t.elapsedMs();
    }
    void collectIds(int *out) override {
        DL_CHECK(pendingN_ > 0, "collectIds: nothing launched");
        const int n = pendingN_;
        pendingN_ = 0;
        syncAndCheckComm();
        inputsInFlight_ = false;
        std::memcpy(out, hIds_, n * sizeof(int));
    }

    double decodeGreedy(int steps, int token, int pos, int slot, int *outTokens) override {
        return decodeGreedyBatch(steps, 1, &token, &pos, &slot, outTokens);
    }

    double decodeGreedyBatch(int steps, int nSeq, const int *tokens, const int *pos, const int *slots,
                             int *outTokens) override {
        DL_CHECK(nSeq >= 1 && (u32)nSeq <= cfg_.maxBatch, "nSeq");
        for (int b = 0; b < nSeq; b++) DL_CHECK((u32)(pos[b] + steps) <= h_.seqLen, "decode exceeds seqLen");
        setInputs(nSeq, tokens, pos, slots, nullptr, steps - 1);
        DL_HIP(hipMemsetAsync(dHist_, 0xff, sizeof(int) * (size_t)cfg_.maxBatch * h_.seqLen, stream_));
        hipEvent_t e0, e1;
        DL_HIP(hipEventCreate(&e0));
        DL_HIP(hipEventCreate(&e1));
        // the chained graph: forward -> argmax -> (tokens := ids, pos += 1)
        DL_HIP(hipEventRecord(e0, stream_));
        for (int s = 0; s < steps; s++) runGraph(nSeq, GraphKind::CHAIN);
        DL_HIP(hipEventRecord(e1, stream_));
        DL_HIP(hipEventSynchronize(e1));
        float ms = 0;
        DL_HIP(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        syncAndCheckComm();
        inputsInFlight_ = false;
        if (outTokens) {
            std::vector<int> hist((size_t)cfg_.maxBatch * h_.seqLen);
            DL_HIP(hipMemcpy(hist.data(), dHist_, hist.size() * sizeof(int), hipMemcpyDeviceToHost));
            for (int b = 0; b < nSeq; b++)
                for (int s = 0; s < steps; s++) outTokens[b * steps + s] = hist[(size_t)b * h_.seqLen + pos[b] + s];
        }
        return ms;
    }

    void profileForward(int n, const int *tokens, const int *positions, const int *slots) override {
        setInputs(n, tokens, positions, slots);
        profile_ = true;
        profTimes_.clear();
        enqueueForward(n, GraphKind::LOGITS);
        DL_HIP(hipStreamSynchronize(stream_));
        inputsInFlight_ = false;
        profile_ = false;
        std::map<std::string, double> agg;
        for (auto &p : profTimes_) {
            float ms = 0;
            DL_HIP(hipEventElapsedTime(&ms, p.second.first, p.second.second));
            agg[p.first] += ms;
            (void)hipEventDestroy(p.second.first);
            (void)hipEventDestroy(p.second.second);
        }
        double total = 0;
        for (auto &kv : agg) total += kv.second;
        std::printf("⏱️  per-kernel-class device time (eager, batch %d):\n", n);
        for (auto &kv : agg) std::printf("   %-14s %8.3f ms (%5.1f%%)\n", kv.first.c_str(), kv.second, 100.0 * kv.second / total);
        std::printf("   %-14s %8.3f ms\n", "total", total);
        profTimes_.clear();
    }

  private:
    enum class GraphKind { LOGITS = 0, ARGMAX = 1, CHAIN = 2, SAMPLE = 3 };

    // Wait for the stream, then turn a tensor-parallel transport failure into an exception (the
    // worker loop re-serves, the root reports it) instead of returning results computed from a
    // peer's stale data: the xGMI collectives flag a peer that did not arrive within 2 s, RCCL
    // reports asynchronous errors (the communicator is then released without waiting).
    void syncAndCheckComm() {
        const int *flag = comm_ ? comm_->deviceErrorFlag() : nullptr;
        if (flag) DL_HIP(hipMemcpyAsync(hErr_, flag, sizeof(int), hipMemcpyDeviceToHost, stream_));
        const bool anyBlock = blockOn_ || ffnOn_;
        if (anyBlock) DL_HIP(hipMemcpyAsync(hErr_ + 1, dBlockErr_, sizeof(int), hipMemcpyDeviceToHost, stream_));
        DL_HIP(hipStreamSynchronize(stream_));
        if (anyBlock && hErr_[1] != 0) {
            const int code = hErr_[1];
            hErr_[1] = 0;
            resetAttnBlockState();
            throw Error("fused layer block: a hand-off wait timed out (code " + std::to_string(code) +
                        ": 2 qkv->attention, 3 attention->wo, 4 qkv phase, 13 w13->w2, 14 w13 phase; not all "
                        "workgroups resident?)");
        }
        if (flag && *hErr_ != 0)
            throw Error("tensor-parallel collective timed out: a peer rank did not arrive within 2 s (worker lost?)");
        if (comm_) {
            const std::string e = comm_->asyncError();
            if (!e.empty()) {
                comm_->shutdownNow();
                throw Error("tensor-parallel transport failed: " + e);
            }
        }
    }

    int rank() const { return comm_ ? comm_->rank() : 0; }

    template <typename T>
    T *dalloc(size_t count) {
        void *p = nullptr;
        const size_t bytes = count * sizeof(T);
        DL_HIP(hipMalloc(&p, bytes < 16 ? 16 : bytes));
        allocs_.push_back(p);
        deviceBytes_ += bytes;
        return (T *)p;
    }
    template <typename T>
    T *halloc(size_t count) {
        void *p = nullptr;
        DL_HIP(hipHostMalloc(&p, count * sizeof(T) < 16 ? 16 : count * sizeof(T), hipHostMallocDefault));
        hostAllocs_.push_back(p);
        return (T *)p;
    }

    void allocBuffers() {
        const u32 MB = cfg_.maxBatch;
        const ShardPlan &p = plan_;
        // [tokens | positions | slots | sample specs (4 floats per row)]: one H2D copy per forward
        dTok_ = dalloc<int>(7 * (size_t)MB);
        dPos_ = dTok_ + MB;
        dSlot_ = dTok_ + 2 * MB;
        dSpec_ = reinterpret_cast<float4 *>(dTok_ + 3 * MB);
        dIds_ = dalloc<int>(MB);
        dHist_ = dalloc<int>((size_t)MB * h_.seqLen);
        hIn_ = halloc<int>(7 * MB);
        hIds_ = halloc<int>(MB);
        hErr_ = halloc<int>(2);
        hErr_[0] = hErr_[1] = 0;
        hLogits_ = halloc<float>((size_t)MB * h_.vocabSize);
        dX_[0] = dalloc<float>((size_t)MB * h_.dim);
        dX_[1] = dalloc<float>((size_t)MB * h_.dim);
        dY_ = dalloc<float>((size_t)MB * h_.dim);
        for (int i = 0; i < 2; i++) {
            dU_[i] = dalloc<float>(h_.dim);
            dUnSS_[i] = dalloc<float>(hipk::kUnMaxPartials);
        }
        dQ_ = dalloc<float>((size_t)MB * p.q0);
        dAtt_ = dalloc<float>((size_t)MB * p.q0);
        dH_ = dalloc<float>((size_t)MB * p.hidden0);
        dAttQ_ = dalloc<int8_t>((size_t)MB * p.q0);
        dAttS_ = dalloc<float2>((size_t)MB * p.q0 / 32);
        dHQ_ = dalloc<int8_t>((size_t)MB * p.hidden0);
        dHS_ = dalloc<float2>((size_t)MB * p.hidden0 / 32);
        {  // batched (MFMA) path, Q40 and F32 weights: f16 activations, split-K partials, counters
            const size_t rowsH = ((size_t)MB + 2 * kGemmMaxTokens - 1) / kGemmMaxTokens * kGemmMaxTokens;
            dXh_ = dalloc<_Float16>(rowsH * h_.dim);
            dAttH_ = dalloc<_Float16>(rowsH * p.q0);
            dHh_ = dalloc<_Float16>(rowsH * p.hidden0);
            DL_HIP(hipMemsetAsync(dXh_, 0, rowsH * h_.dim * 2, stream_));
            DL_HIP(hipMemsetAsync(dAttH_, 0, rowsH * p.q0 * 2, stream_));
            DL_HIP(hipMemsetAsync(dHh_, 0, rowsH * p.hidden0 * 2, stream_));
            const int mt = (int)MB;
            size_t part = 0;
            int cnt = 0;
            auto acc = [&](int rows, int n) {
                part = std::max(part, hipk::gemmPartFloats(rows, n, mt));
                cnt = std::max(cnt, hipk::gemmCounterInts(rows, mt));
            };
            acc(p.q0 + 2 * p.kv0, h_.dim);
            acc(h_.dim, p.q0);
            acc(2 * p.hidden0, h_.dim);
            acc(h_.dim, p.hidden0);
            acc(p.vocab0, h_.dim);
            if (part) dPart_ = dalloc<float>(part);
            const int maxTiles = cnt;
            dGemmCnt_ = dalloc<int>(maxTiles);
            // fused residual + norm hand-off between batched GEMMs (TP1): per 64-row tile of dim,
            // per token, the partial sum of squares
            dSS_ = dalloc<float>((size_t)((h_.dim + 63) / 64) * MB);
            DL_HIP(hipMemsetAsync(dGemmCnt_, 0, sizeof(int) * maxTiles, stream_));
        }
        {  // fused attention block: epoch, monotonic counters, expected counts, timeout flag
            dEpoch_ = dalloc<unsigned>(4);
            dBlockCnt_ = dalloc<unsigned>(kBlockCntWords);
            dBlockExpect_ = dalloc<unsigned>(kMaxKvGroups);
            dBlockErr_ = dalloc<int>(4);
            DL_HIP(hipMemsetAsync(dEpoch_, 0, 4 * sizeof(unsigned), stream_));
            DL_HIP(hipMemsetAsync(dBlockCnt_, 0, kBlockCntWords * sizeof(unsigned), stream_));
            DL_HIP(hipMemsetAsync(dBlockExpect_, 0, kMaxKvGroups * sizeof(unsigned), stream_));
            DL_HIP(hipMemsetAsync(dBlockErr_, 0, 4 * sizeof(int), stream_));
        }
        dAttCnt_ = dalloc<int>((size_t)MB * p.nHeads0);
        DL_HIP(hipMemsetAsync(dAttCnt_, 0, sizeof(int) * (size_t)MB * p.nHeads0, stream_));
        dArgV_ = dalloc<float>((size_t)MB * 64);
        dArgI_ = dalloc<int>((size_t)MB * 64);
        {
            void *ss = dalloc<uint8_t>(hipk::SampleScratch::bytes((int)MB));
            DL_HIP(hipMemsetAsync(ss, 0, hipk::SampleScratch::bytes((int)MB), stream_));
            sampleScratch_.carve(ss, (int)MB);
        }
        dArgCnt_ = dalloc<int>(MB);
        DL_HIP(hipMemsetAsync(dArgCnt_, 0, sizeof(int) * MB, stream_));
        dLogits_ = dalloc<float>((size_t)MB * p.vocab0);
        if (p.nRanks > 1) {
            dLogitsAll_ = dalloc<float>((size_t)MB * h_.vocabSize);
            dLogitsFull_ = dalloc<float>((size_t)MB * h_.vocabSize);
        }
        splitGrid_ = hipk::attnSplitGrid(h_.seqLen);
        chunkMax_ = hipk::attnChunkMax(h_.seqLen, splitGrid_);
        dPartO_ = dalloc<float>((size_t)MB * p.nHeads0 * splitGrid_ * p.headSize);
        dPartML_ = dalloc<float>((size_t)MB * p.nHeads0 * splitGrid_ * 2);
        dRope_ = dalloc<float2>((size_t)h_.seqLen * (p.headSize / 2));
        layers_.resize(h_.nLayers);
        const size_t kvElems = kvPoolRows() * p.kv0;
        setupPages();
        for (auto &L : layers_) {
            if (kvBf16_) {
                L.k = dalloc<uint16_t>(kvElems);
                L.v = dalloc<uint16_t>(kvElems);
            } else {
                L.k = dalloc<float>(kvElems);
                L.v = dalloc<float>(kvElems);
            }
            DL_HIP(hipMemsetAsync(L.k, 0, kvElems * (kvBf16_ ? 2 : 4), stream_));
            DL_HIP(hipMemsetAsync(L.v, 0, kvElems * (kvBf16_ ? 2 : 4), stream_));
        }
    }

    void uploadRope() {
        std::vector<float> t = buildRopeTable(h_);
        DL_HIP(hipMemcpy(dRope_, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
    }

    // ---------------------------------------------------------------- weight upload
    // The file load is a three-stage pipeline per matrix:
    //   1. parallel pread of exactly this rank's rows / row slices (ParallelReader, 16 threads);
    //   2. multi-threaded repack of the file's AoS Q40 blocks straight into the GEMV's tiled layout,
    //      written into one of two pinned staging buffers;
    //   3. hipMemcpyAsync on a dedicated copy stream (DMA at pinned-memory speed), which runs while
    //      the host reads and tiles the next matrix; a staging buffer is reused only after the
    //      event of its previous copy has completed.
    // (Round 1 repacked into std::vectors and uploaded with synchronous pageable hipMemcpy.)
    struct RowSrc {
        const TensorInfo *t;
        u32 r0, nr;
    };
    struct Loader {
        std::unique_ptr<ParallelReader> reader;
        hipStream_t copy = nullptr;
        u8 *stage[2] = {nullptr, nullptr};
        hipEvent_t done[2] = {nullptr, nullptr};
        bool busy[2] = {false, false};
        size_t stageBytes = 0;
        int cur = 0;
        std::vector<u8> raw;
        std::vector<const u8 *> rowPtr;
    };

    u8 *stageAcquire(Loader &ld) {
        ld.cur ^= 1;
        if (ld.busy[ld.cur]) DL_HIP(hipEventSynchronize(ld.done[ld.cur]));
        ld.busy[ld.cur] = false;
        return ld.stage[ld.cur];
    }
    void stageCopy(Loader &ld, void *dst, const u8 *src, size_t bytes) {
        DL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ld.copy));
    }
    void stageRelease(Loader &ld) {
        DL_HIP(hipEventRecord(ld.done[ld.cur], ld.copy));
        ld.busy[ld.cur] = true;
    }

    // Read the rows of every source (restricted to columns [c0, c0 + nc)) into ld.raw and point
    // ld.rowPtr at each output row (w1/w3 interleaved row by row when `interleave`).
    void readRows(Loader &ld, const std::vector<RowSrc> &srcs, bool interleave, u32 c0, u32 nc) {
        const u64 esz = q40_ ? 0 : 4;
        auto rowBytes = [&](u32 cols) { return q40_ ? (u64)cols / kQBlock * kQ40BlockBytes : (u64)cols * esz; };
        const u64 slice = rowBytes(nc);
        u64 total = 0;
        for (const auto &s : srcs) total += (u64)s.nr * slice;
        if (ld.raw.size() < total) ld.raw.resize(total);
        std::vector<ParallelReader::Range> ranges;
        std::vector<std::vector<const u8 *>> perSrc(srcs.size());
        u64 at = 0;
        for (size_t i = 0; i < srcs.size(); i++) {
            const RowSrc &s = srcs[i];
            const u64 full = rowBytes(s.t->cols), skip = rowBytes(c0);
            u8 *dst = ld.raw.data() + at;
            if (c0 == 0 && nc == s.t->cols) {  // whole rows: one contiguous range
                ranges.push_back({s.t->offset + (u64)s.r0 * full, (u64)s.nr * full, dst});
            } else {  // column slice (row-split wo / w2 of tensor parallelism): one range per row
                for (u32 r = 0; r < s.nr; r++)
                    ranges.push_back({s.t->offset + (u64)(s.r0 + r) * full + skip, slice, dst + (u64)r * slice});
            }
            for (u32 r = 0; r < s.nr; r++) perSrc[i].push_back(dst + (u64)r * slice);
            at += (u64)s.nr * slice;
        }
        ld.reader->readMany(ranges);
        ld.rowPtr.clear();
        if (interleave) {
            DL_CHECK(srcs.size() == 2 && srcs[0].nr == srcs[1].nr, "interleave");
            for (u32 i = 0; i < srcs[0].nr; i++) {
                ld.rowPtr.push_back(perSrc[0][i]);
                ld.rowPtr.push_back(perSrc[1][i]);
            }
        } else {
            for (auto &v : perSrc) ld.rowPtr.insert(ld.rowPtr.end(), v.begin(), v.end());
        }
    }

    size_t matStageBytes(u32 rows, u32 n) const {
        if (!q40_) return (size_t)rows * n * 4;
        const hipk::Q40Tiling t = hipk::q40Tiling((int)rows, (int)n, hipk::gemvLanesPerRow((int)n, (int)rows, 1, true));
        return t.qsBytes + t.dBytes;
    }

    void buildMat(Loader &ld, DevMat &m, const std::vector<RowSrc> &srcs, bool interleave, u32 c0, u32 nc) {
        readRows(ld, srcs, interleave, c0, nc);
        const int rows = (int)ld.rowPtr.size();
        m.rows = rows;
        m.n = (int)nc;
        u8 *st = stageAcquire(ld);
        if (q40_) {
            m.lanes = hipk::gemvLanesPerRow((int)nc, rows, 1, true);
            const hipk::Q40Tiling t = hipk::q40Tiling(rows, (int)nc, m.lanes);
            DL_CHECK(t.qsBytes + t.dBytes <= ld.stageBytes, "staging buffer too small");
            hipk::tileQ40AoS(ld.rowPtr.data(), rows, (int)nc, m.lanes, st, reinterpret_cast<uint32_t *>(st + t.qsBytes));
            m.qs = dalloc<uint8_t>(t.qsBytes);
            m.d = dalloc<uint16_t>(t.dBytes / 2);
            stageCopy(ld, m.qs, st, t.qsBytes);
            stageCopy(ld, m.d, st + t.qsBytes, t.dBytes);
        } else {
            const size_t rb = (size_t)nc * 4;
            DL_CHECK((size_t)rows * rb <= ld.stageBytes, "staging buffer too small");
            for (int r = 0; r < rows; r++) std::memcpy(st + (size_t)r * rb, ld.rowPtr[r], rb);
            m.f = dalloc<float>((size_t)rows * nc);
            stageCopy(ld, m.f, st, (size_t)rows * rb);
        }
        stageRelease(ld);
    }

    // A whole f32 tensor (norm weights, embedding), streamed through the staging buffers.
    float *uploadF32(Loader &ld, const TensorInfo &t) {
        const size_t bytes = (size_t)t.rows * t.cols * 4;
        float *p = dalloc<float>((size_t)t.rows * t.cols);
        for (size_t o = 0; o < bytes; o += ld.stageBytes) {
            const size_t len = std::min(ld.stageBytes, bytes - o);
            u8 *st = stageAcquire(ld);
            ld.reader->read(t.offset + o, len, st);
            stageCopy(ld, reinterpret_cast<u8 *>(p) + o, st, len);
            stageRelease(ld);
        }
        return p;
    }

    void loadFromFile() {
        const ShardPlan &p = plan_;
        const ModelFile &f = *file_;
        Loader ld;
        ld.reader.reset(new ParallelReader(file_->path()));
        // staging: the largest tiled matrix of this shard (at least 64 MB for the f32 tensors)
        size_t sb = (size_t)64 << 20;
        sb = std::max(sb, matStageBytes(p.q0 + 2 * p.kv0, h_.dim));
        sb = std::max(sb, matStageBytes(h_.dim, p.q0));
        sb = std::max(sb, matStageBytes(2 * p.hidden0, h_.dim));
        sb = std::max(sb, matStageBytes(h_.dim, p.hidden0));
        sb = std::max(sb, matStageBytes(p.vocab0, h_.dim));
        ld.stageBytes = sb;
        for (int i = 0; i < 2; i++) {
            DL_HIP(hipHostMalloc(reinterpret_cast<void **>(&ld.stage[i]), sb, hipHostMallocDefault));
            DL_HIP(hipEventCreateWithFlags(&ld.done[i], hipEventDisableTiming));
        }
        DL_HIP(hipStreamCreateWithFlags(&ld.copy, hipStreamNonBlocking));
        auto cleanup = [&] {
            (void)hipStreamSynchronize(ld.copy);
            for (int i = 0; i < 2; i++) {
                (void)hipHostFree(ld.stage[i]);
                (void)hipEventDestroy(ld.done[i]);
            }
            (void)hipStreamDestroy(ld.copy);
        };
        try {
            for (u32 l = 0; l < h_.nLayers; l++) {
                DevLayer &L = layers_[l];
                const TensorInfo &wq = f.find(TensorKind::WQ, l), &wk = f.find(TensorKind::WK, l),
                                 &wv = f.find(TensorKind::WV, l), &wo = f.find(TensorKind::WO, l),
                                 &w1 = f.find(TensorKind::W1, l), &w2 = f.find(TensorKind::W2, l),
                                 &w3 = f.find(TensorKind::W3, l);
                buildMat(ld, L.qkv, {{&wq, p.qStart(), p.q0}, {&wk, p.kvStart(), p.kv0}, {&wv, p.kvStart(), p.kv0}},
                         false, 0, h_.dim);
                buildMat(ld, L.wo, {{&wo, 0, h_.dim}}, false, p.qStart(), p.q0);
                buildMat(ld, L.w13, {{&w1, p.hiddenStart(), p.hidden0}, {&w3, p.hiddenStart(), p.hidden0}}, true, 0,
                         h_.dim);
                buildMat(ld, L.w2, {{&w2, 0, h_.dim}}, false, p.hiddenStart(), p.hidden0);
                L.rmsAtt = uploadF32(ld, f.find(TensorKind::RMS_ATT, l));
                L.rmsFfn = uploadF32(ld, f.find(TensorKind::RMS_FFN, l));
            }
            emb_ = uploadF32(ld, f.find(TensorKind::EMBEDDING, -1));
            rmsFinal_ = uploadF32(ld, f.find(TensorKind::RMS_FINAL, -1));
            buildMat(ld, wcls_, {{&f.find(TensorKind::WCLS, -1), p.vocabStart(), p.vocab0}}, false, 0, h_.dim);
            DL_HIP(hipStreamSynchronize(ld.copy));
        } catch (...) {
            cleanup();
            throw;
        }
        cleanup();
        load_.fileBytes = ld.reader->bytesRead();
    }

    void synthMat(DevMat &m, int rows, int n, u64 seed) {
        m.rows = rows;
        m.n = n;
        const float scale = 1.0f / std::sqrt(21.5f * (float)n);
        if (q40_) {
            m.lanes = hipk::gemvLanesPerRow(n, rows, 1, true);
            const hipk::Q40Tiling t = hipk::q40Tiling(rows, n, m.lanes);
            const size_t nBlocks = t.qsBytes / 16;  // == t.dBytes / 2 f16 scales
            m.qs = dalloc<uint8_t>(t.qsBytes);
            m.d = dalloc<uint16_t>(nBlocks);
            hipk::launchFillQ40(m.qs, m.d, nBlocks, scale, seed, stream_);
        } else {
            m.f = dalloc<float>((size_t)rows * n);
            hipk::launchFillF32Uniform(m.f, (size_t)rows * n, std::sqrt(3.0f / (float)n), seed, stream_);
        }
        DL_HIP(hipGetLastError());
    }

    void loadSynthetic() {
        const ShardPlan &p = plan_;
        u64 seed = cfg_.seed * 1000003ull + (u64)p.rank * 7919ull;
        for (u32 l = 0; l < h_.nLayers; l++) {
            DevLayer &L = layers_[l];
            synthMat(L.qkv, p.q0 + 2 * p.kv0, h_.dim, seed++);
            synthMat(L.wo, h_.dim, p.q0, seed++);
            synthMat(L.w13, 2 * p.hidden0, h_.dim, seed++);
            synthMat(L.w2, h_.dim, p.hidden0, seed++);
            L.rmsAtt = dalloc<float>(h_.dim);
            L.rmsFfn = dalloc<float>(h_.dim);
            hipk::launchFillF32Const(L.rmsAtt, h_.dim, 1.0f, stream_);
            hipk::launchFillF32Const(L.rmsFfn, h_.dim, 1.0f, stream_);
        }
        emb_ = dalloc<float>((size_t)h_.vocabSize * h_.dim);
        hipk::launchFillF32Uniform(emb_, (size_t)h_.vocabSize * h_.dim, 1.0f, cfg_.seed ^ 0xE3B, stream_);
        rmsFinal_ = dalloc<float>(h_.dim);
        hipk::launchFillF32Const(rmsFinal_, h_.dim, 1.0f, stream_);
        synthMat(wcls_, p.vocab0, h_.dim, seed++);
        DL_HIP(hipGetLastError());
    }

    // ---------------------------------------------------------------- forward schedule
    void setInputs(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs = nullptr,
                   int ahead = 0) {
        DL_CHECK(n >= 1 && (u32)n <= cfg_.maxBatch, "batch size out of range");
        for (int b = 0; b < n; b++) {
            DL_CHECK(tokens[b] >= 0 && (u32)tokens[b] < h_.vocabSize, "token out of range");
            DL_CHECK(positions[b] >= 0 && (u32)positions[b] < h_.seqLen, "position out of range");
            DL_CHECK(slots[b] >= 0 && (u32)slots[b] < cfg_.nSlots, "slot out of range");
        }
        mapPages(n, positions, slots, ahead);
        // decode attention kernel for this forward (part of the graph key): the MFMA kernel once a
        // row's context reaches kAttnMfmaMinPos keys (measured faster from ~1.5K keys, slower on
        // short contexts: profiles/r3_prefill_attention.md), else the VALU kernel
        int maxPos = 0;
        for (int b = 0; b < n; b++) maxPos = std::max(maxPos, positions[b] + ahead);
        attnLong_ = maxPos >= kAttnMfmaMinPos;
        const u32 MB = cfg_.maxBatch;
        // keep the pinned staging buffer stable while a previous copy may still read it (every
        // public entry point ends with a stream sync, so this only waits after an async path)
        if (inputsInFlight_) DL_HIP(hipStreamSynchronize(stream_));
        std::memcpy(hIn_, tokens, n * sizeof(int));
        std::memcpy(hIn_ + MB, positions, n * sizeof(int));
        std::memcpy(hIn_ + 2 * MB, slots, n * sizeof(int));
        size_t words = 2 * (size_t)MB + n;
        // prefill attention on MFMA: every block of rows it assigns to one workgroup is one slot
        prefillOk_ = kvBf16_ && hipk::attnPrefillSupported(plan_.headSize, plan_.kvMul, true);
        const int rpb = prefillOk_ ? hipk::attnPrefillRowsPerBlock(plan_.kvMul) : 1;
        for (int b = 0; prefillOk_ && b < n; b++) prefillOk_ = slots[b] == slots[b - b % rpb];
        if (specs) {
            static_assert(sizeof(SampleSpec) == 4 * sizeof(float), "spec layout");
            std::memcpy(hIn_ + 3 * MB, specs, n * sizeof(SampleSpec));
            words = 3 * (size_t)MB + 4 * (size_t)n;
        }
        // one copy of the row arrays (the unused tail of each is never read)
        DL_HIP(hipMemcpyAsync(dTok_, hIn_, words * sizeof(int), hipMemcpyHostToDevice, stream_));
        inputsInFlight_ = true;
    }

    void runGraph(int n, GraphKind kind) {
        if (!cfg_.useGraphs || graphsBroken_) {
            enqueueForward(n, kind);
            return;
        }
        const int key = ((n * 4 + (int)kind) * 2 + (prefillOk_ ? 1 : 0)) * 2 + (attnLong_ ? 1 : 0);
        auto it = graphs_.find(key);
        if (it == graphs_.end()) {
            // capture on the second use of a shape: a one-off row count (the tail chunk of a prompt,
            // a serving batch seen once) runs eagerly instead of paying capture + instantiation
            // (several ms for ~170 kernel nodes) for a graph that would never be replayed
            if (graphSeen_.insert(key).second) {
                enqueueForward(n, kind);
                return;
            }
            hipGraphExec_t ge = captureForward(n, kind);
            if (!ge) {
                // e.g. a collective library build that cannot be stream-captured: stay correct, run eagerly
                graphsBroken_ = true;
                std::fprintf(stderr, "⚠️  hipGraph capture failed; falling back to eager launches\n");
                enqueueForward(n, kind);
                return;
            }
            it = graphs_.emplace(key, ge).first;
        }
        DL_HIP(hipGraphLaunch(it->second, stream_));
    }

    hipGraphExec_t captureForward(int n, GraphKind kind) {
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        if (hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal) != hipSuccess) return nullptr;
        bool ok = true;
        try {
            enqueueForward(n, kind);
        } catch (const std::exception &e) {
            std::fprintf(stderr, "capture error: %s\n", e.what());
            ok = false;
        }
        const hipError_t ec = hipStreamEndCapture(stream_, &g);
        if (ec != hipSuccess || !ok || !g) {
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();
            return nullptr;
        }
        const hipError_t ei = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ei != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        return ge;
    }

    // timing hook for profileForward (eager only)
    struct ProfScope {
        HipEngineImpl *e;
        std::string name;
        TraceRange trace;  // roctx range (DL_ROCTX=1): per kernel class in eager runs
        hipEvent_t a = nullptr, b = nullptr;
        ProfScope(HipEngineImpl *e_, const char *n_) : e(e_), name(n_), trace(n_) {
            if (e->profile_) {
                (void)hipEventCreate(&a);
                (void)hipEventCreate(&b);
                (void)hipEventRecord(a, e->stream_);
            }
        }
        ~ProfScope() {
            if (e->profile_) {
                (void)hipEventRecord(b, e->stream_);
                e->profTimes_.push_back({name, {a, b}});
            }
        }
    };

    int batchChunk(const DevMat &m, int pro, int epi) const {
        // largest batch chunk (1/2/4) whose LDS footprint stays <= 64 KiB for this input width
        int bc = 4;
        while (bc > 1) {
            const int rpw = hipk::gemvRowsPerPass(m.n, m.rows, bc, q40_) * passesFor(m, epi, bc);
            if (hipk::gemvLdsBytes(m.n, bc, q40_, rpw, pro) <= 64 * 1024) break;  // B > 1 only; B = 1 may use up to 160 KB
            bc >>= 1;
        }
        return bc;
    }

    int passesFor(const DevMat &m, int epi, int B) const {
        return hipk::gemvDefaultPasses(m.n, m.rows, B, q40_, epi);
    }

    // Launch a GEMV over all n rows, in batch chunks of <= 4. tp: all-reduce the EPI_STORE output
    // over the tensor-parallel ranks in the kernel tail (fused exchange).
    // Arguments of one GEMV launch over rows [c0, c0 + bc) of the batch (see gemv()).
    hipk::GemvArgs gemvArgs(const DevMat &m, int c0, int bc, int epi, const float *in, int ldIn, const float *add,
                            float *xNext, const float *normW, float *out, int ldOut, const DevLayer *L,
                            const int8_t *aq, const float2 *as, int8_t *oq, float2 *os, bool tp) const {
        hipk::GemvArgs a;
        a.qs = m.qs;
        a.wd = m.d;
        a.wf = m.f;
        a.rows = m.rows;
        a.n = m.n;
        a.passes = tp ? tpPasses(m, bc) : passesFor(m, epi, bc);
        a.lanes = m.lanes;
        if (tp) a.tp = tpVec_;
        a.in = in ? in + (size_t)c0 * ldIn : nullptr;
        a.aq = aq ? aq + (size_t)c0 * m.n : nullptr;
        a.as = as ? as + (size_t)c0 * (m.n / 32) : nullptr;
        a.oq = oq ? oq + (size_t)c0 * ldOut : nullptr;
        a.os = os ? os + (size_t)c0 * (ldOut / 32) : nullptr;
        a.ldIn = ldIn;
        a.addIn = add ? add + (size_t)c0 * ldIn : nullptr;
        a.xNext = xNext ? xNext + (size_t)c0 * ldIn : nullptr;
        a.normW = normW;
        a.eps = h_.normEpsilon;
        a.out = out ? out + (size_t)c0 * ldOut : nullptr;
        a.ldOut = ldOut;
        a.act = h_.hiddenAct == HiddenAct::GELU ? 0 : 1;
        if (L) {
            a.q0 = plan_.q0;
            a.kv0 = plan_.kv0;
            a.hs = plan_.headSize;
            a.kvMul = plan_.kvMul;
            a.seqLen = h_.seqLen;
            a.rope = dRope_;
            a.pos = dPos_ + c0;
            a.slot = dSlot_ + c0;
            a.kcache = L->k;
            a.kvMap = kvMap();
            a.vcache = L->v;
            a.kvBf16 = kvBf16_ ? 1 : 0;
        }
        return a;
    }

    // Launch a GEMV over all n rows, in batch chunks of <= 4. tp: all-reduce the EPI_STORE output
    // over the tensor-parallel ranks in the kernel tail (fused exchange).
    void gemv(const DevMat &m, int n, int pro, int epi, const float *in, int ldIn, const float *add, float *xNext,
              const float *normW, float *out, int ldOut, const DevLayer *L, const int8_t *aq = nullptr,
              const float2 *as = nullptr, int8_t *oq = nullptr, float2 *os = nullptr, bool tp = false) {
        if (tp) epi = hipk::EPI_STORE_TP;
        const int bcMax = batchChunk(m, pro, epi);
        for (int c0 = 0; c0 < n;) {
            int bc = n - c0;
            if (bc > bcMax) bc = bcMax;
            if (bc == 3) bc = 2;
            const hipk::GemvArgs a = gemvArgs(m, c0, bc, epi, in, ldIn, add, xNext, normW, out, ldOut, L, aq, as, oq, os, tp);
            hipk::launchGemv(a, bc, pro, epi, q40_, stream_);
            c0 += bc;
        }
    }

    // Decode attention of this layer (rows 0..n of the forward).
    hipk::AttnArgs attnArgs(const DevLayer &L, bool bat) const {
        const ShardPlan &p = plan_;
        hipk::AttnArgs a;
        a.q = dQ_;
        a.ldq = p.q0;
        a.kcache = L.k;
        a.kvMap = kvMap();
        a.vcache = L.v;
        a.pos = dPos_;
        a.slot = dSlot_;
        a.nHeads0 = p.nHeads0;
        a.kvMul = p.kvMul;
        a.hs = p.headSize;
        a.kv0 = p.kv0;
        a.seqLen = h_.seqLen;
        a.splitGrid = splitGrid_;
        a.chunkMax = chunkMax_;
        a.partO = dPartO_;
        a.partML = dPartML_;
        a.out = dAtt_;
        a.outQ = q40_ && !bat ? dAttQ_ : nullptr;
        a.outS = q40_ && !bat ? dAttS_ : nullptr;
        a.outH = bat ? dAttH_ : nullptr;
        a.ldOut = p.q0;
        a.kvBf16 = kvBf16_ ? 1 : 0;
        a.mfma = attnLong_ ? 1 : 0;
        a.counters = dAttCnt_;
        return a;
    }

    // The fused attention block of a single decode row (kernels.h AttnBlockArgs): qkv GEMV +
    // attention + wo GEMV in one launch. Layer l, residual input dX_[cur].
    hipk::AttnBlockArgs attnBlockArgs(const DevLayer &L, u32 l, int cur) const {
        const ShardPlan &p = plan_;
        const bool hasDelta = l > 0;
        hipk::AttnBlockArgs b;
        b.qkv = gemvArgs(L.qkv, 0, 1, hipk::EPI_QKV, dX_[cur], h_.dim, hasDelta ? dY_ : nullptr,
                         hasDelta ? dX_[cur ^ 1] : nullptr, L.rmsAtt, dQ_, p.q0, &L, nullptr, nullptr, nullptr, nullptr,
                         false);
        b.at = attnArgs(L, false);
        const bool tp = fusedTp(false);
        b.wo = gemvArgs(L.wo, 0, 1, tp ? hipk::EPI_STORE_TP : hipk::EPI_STORE, nullptr, p.q0, nullptr, nullptr, nullptr,
                        dY_, h_.dim, nullptr, dAttQ_, dAttS_, nullptr, nullptr, tp);
        b.hg = hipk::attnBlockHG(b.at);
        b.layer = (int)l;
        b.nLayers = (int)h_.nLayers;
        b.epoch = dEpoch_;
        b.qkvCnt = dBlockCnt_;
        b.attnCnt = dBlockCnt_ + kMaxKvGroups * 64;
        b.attnFlag = dBlockCnt_ + kMaxKvGroups * 64 + 64;
        b.qkvExpect = dBlockExpect_;
        b.error = dBlockErr_;
        return b;
    }

    // Decide once whether decode rows run the fused attention block: Q40 weights, a compiled
    // instance for this shape, <= 64 KV groups, and the whole grid co-resident (shared with the
    // other ranks on this GPU). DL_ATTN_BLOCK=0 keeps the three separate launches.
    void setupAttnBlock() {
        const char *e = std::getenv("DL_ATTN_BLOCK");
        if ((e && *e == '0') || !q40_ || plan_.nKvHeads0 > kMaxKvGroups) return;
        const hipk::AttnBlockArgs b = attnBlockArgs(layers_[0], 0, 0);
        if (!hipk::attnBlockPlan(b, fusedTp(false)).fn) return;
        const hipk::GemvResidency r = hipk::attnBlockResidency(b, fusedTp(false));
        const int share = comm_ ? std::max(1, comm_->ranksOnDevice()) : 1;
        if (r.maxResident <= 0 || r.grid > r.maxResident / share) {
            std::fprintf(stderr, "ℹ️  fused attention block off: grid %d > %d co-resident workgroups per rank\n", r.grid,
                         r.maxResident / share);
            return;
        }
        std::vector<unsigned> expect(kMaxKvGroups, 0);
        hipk::attnBlockExpect(b.qkv, (int)plan_.nKvHeads0, expect.data());
        DL_HIP(hipMemcpy(dBlockExpect_, expect.data(), expect.size() * sizeof(unsigned), hipMemcpyHostToDevice));
        blockGrid_ = r.grid;
        blockOn_ = true;
    }

    // The fused FFN block of a single decode row (kernels.h FfnBlockArgs): w13 GEMV (SwiGLU -> Q80
    // hidden, write-through) + w2 GEMV in one launch. Layer l, residual input dX_[cur] + dY_.
    hipk::FfnBlockArgs ffnBlockArgs(const DevLayer &L, u32 l, int cur) const {
        const ShardPlan &p = plan_;
        const bool tp = fusedTp(false);
        hipk::FfnBlockArgs b;
        b.w13 = gemvArgs(L.w13, 0, 1, hipk::EPI_ACT_Q80, dX_[cur], h_.dim, dY_, dX_[cur ^ 1], L.rmsFfn, dH_, p.hidden0,
                         nullptr, nullptr, nullptr, dHQ_, dHS_, false);
        b.w13.passes *= ffnW13PassMul_;
        b.w2 = gemvArgs(L.w2, 0, 1, tp ? hipk::EPI_STORE_TP : hipk::EPI_STORE, nullptr, p.hidden0, nullptr, nullptr,
                        nullptr, dY_, h_.dim, nullptr, dHQ_, dHS_, nullptr, nullptr, tp);
        b.layer = (int)l;
        b.nLayers = (int)h_.nLayers;
        b.epoch = dEpoch_;
        b.cnt = dBlockCnt_ + kFfnCntOff;
        b.flag = dBlockCnt_ + kFfnCntOff + 64;
        b.error = dBlockErr_;
        b.ringEarly = ffnRingEarly_;
        b.sameWg = ffnSameWg_;
        return b;
    }

    // Decide once whether decode rows run the fused FFN block: Q40 weights with the Q80 hidden
    // hand-off, a compiled instance for the (w13, w2) lane counts, and the whole grid co-resident
    // (shared with the other ranks on this GPU); w13's passes are doubled (fewer, longer
    // workgroups) until it fits. DL_FFN_BLOCK=1 enables it (default: the two launches); DL_FFN_RING_EARLY=1 issues
    // w2's weight ring at entry instead of after the w13 phase; DL_FFN_W13_PASSES sets w13's
    // passes multiplier.
    void setupFfnBlock() {
        // opt-in: 1 = producer / consumer workgroups (measured slower, profiles/r3_attn_block.md),
        // 2 = the same workgroups run w13 then w2
        const char *e = std::getenv("DL_FFN_BLOCK");
        if (!(e && (*e == '1' || *e == '2')) || !q40_ || plan_.hidden0 / 32 < 192) return;
        ffnSameWg_ = *e == '2' ? 1 : 0;
        const char *re = std::getenv("DL_FFN_RING_EARLY");
        ffnRingEarly_ = re && *re == '1' ? 1 : 0;
        const char *pm = std::getenv("DL_FFN_W13_PASSES");
        const int share = comm_ ? std::max(1, comm_->ranksOnDevice()) : 1;
        for (int mul = pm && *pm ? std::max(1, std::atoi(pm)) : 1; mul <= 8; mul *= 2) {
            ffnW13PassMul_ = mul;
            const hipk::FfnBlockArgs b = ffnBlockArgs(layers_[0], 0, 0);
            if (!hipk::ffnBlockPlan(b, fusedTp(false)).fn) break;
            const hipk::GemvResidency r = hipk::ffnBlockResidency(b, fusedTp(false));
            if (r.maxResident > 0 && r.grid <= r.maxResident / share) {
                ffnOn_ = true;
                return;
            }
            if (pm && *pm) {
                std::fprintf(stderr, "ℹ️  fused FFN block off: grid %d > %d co-resident workgroups per rank\n", r.grid,
                             r.maxResident / share);
                break;
            }
        }
        ffnW13PassMul_ = 1;
    }

    // Decide once whether single decode rows split each residual update + RMS norm between the GEMV
    // that produces the update and the one that consumes the norm (kernels.h EPI_STORE_UN /
    // PRO_UNORM): the wo / w2 epilogues add their rows into x in place and leave u = normW * x plus
    // one partial sum of squares per workgroup, so the qkv / w13 / logits prologues read u and the
    // partials instead of x, delta and normW per workgroup (qkv 6.0 -> 4.8 us, w13 14.3 -> 13.8 us
    // with fully precomputed activations, scripts/bench_gemv.py). TP1, Q40, Q80 hidden hand-off,
    // no fused FFN block. Opt-in (DL_UNORM=1): measured a wash on 8B decode (1.3453 -> 1.3496
    // ms/token: w13 14.64 -> 14.17 us, but the w2 producer 7.94 -> 8.49 us and the attention block
    // 16.29 -> 16.52 us; profiles/r3_prefill_attention.md).
    void setupUn() {
        const char *e = std::getenv("DL_UNORM");
        if (!(e && *e == '1') || !q40_ || plan_.nRanks != 1 || ffnOn_ || plan_.hidden0 / 32 < 192 || h_.dim > 8192)
            return;
        const DevLayer &L = layers_[0];
        auto rowsPerWg = [&](const DevMat &m) {
            return (256 / m.lanes) * 2 * passesFor(m, hipk::EPI_STORE_UN, 1);
        };
        if (rowsPerWg(L.wo) > 256 || rowsPerWg(L.w2) > 256) return;
        unWoGrid_ = (L.wo.rows + rowsPerWg(L.wo) - 1) / rowsPerWg(L.wo);
        unW2Grid_ = (L.w2.rows + rowsPerWg(L.w2) - 1) / rowsPerWg(L.w2);
        if (unWoGrid_ > hipk::kUnMaxPartials || unW2Grid_ > hipk::kUnMaxPartials) return;
        if (blockOn_) {
            hipk::AttnBlockArgs b = attnBlockArgs(L, 0, 0);
            unBlockArgs(b, L, 0);
            if (!hipk::attnBlockPlan(b, false).fn) return;
            const hipk::GemvResidency r = hipk::attnBlockResidency(b, false);
            if (r.maxResident <= 0 || r.grid > r.maxResident) return;
        }
        unOn_ = true;
    }
    const float *unNextNorm(u32 l) const { return l + 1 < h_.nLayers ? layers_[l + 1].rmsAtt : rmsFinal_; }
    // PRO_UNORM consumer of u[i] / ss[i] with `count` partials
    void unIn(hipk::GemvArgs &a, int i, int count) const {
        a.in = dU_[i];
        a.addIn = nullptr;
        a.xNext = nullptr;
        a.normW = nullptr;
        a.ssIn = dUnSS_[i];
        a.ssCount = count;
    }
    // EPI_STORE_UN producer: x updated in place, u[i] = w * x, ss[i][workgroup]
    void unOut(hipk::GemvArgs &a, int i, const float *w) const {
        a.out = dX_[0];
        a.uOut = dU_[i];
        a.unW = w;
        a.ssOut = dUnSS_[i];
    }
    void unBlockArgs(hipk::AttnBlockArgs &b, const DevLayer &L, u32 l) const {
        b.un = 1;
        unIn(b.qkv, 1, l == 0 ? 1 : unW2Grid_);
        unOut(b.wo, 0, L.rmsFfn);
    }

    // A fused-block wait gave up (a workgroup of the launch never arrived): reset the monotonic
    // counters and the epoch so the engine stays usable, then raise.
    void resetAttnBlockState() {
        DL_HIP(hipMemsetAsync(dBlockCnt_, 0, sizeof(unsigned) * kBlockCntWords, stream_));
        DL_HIP(hipMemsetAsync(dEpoch_, 0, sizeof(unsigned), stream_));
        DL_HIP(hipMemsetAsync(dBlockErr_, 0, sizeof(int), stream_));
        DL_HIP(hipStreamSynchronize(stream_));
    }

    // rows per forward from which the MFMA GEMM replaces the GEMV (DL_GEMM_MIN, read at construction)
    // Default: GEMV up to 2 rows at TP1 (8B ms/step GEMV vs MFMA GEMM: 1.90 vs 2.64 at 2 rows, 3.15 vs
    // 2.67 at 3, 2.92 vs 2.66 at 4, after the fence-free split-K); up to 4 rows at TP > 1, where the
    // GEMV path carries the fused exchange.
    int gemmMinTokens() const { return gemmMin_; }

    bool batchedPath(int n) const {
        return n >= gemmMinTokens() && hipk::gemmSupported(h_.dim) && hipk::gemmSupported(plan_.q0) &&
               hipk::gemmSupported(plan_.hidden0);
    }

    // MALL warm-up of wo + the head of w13 beside attention (DL_MALL_PREFETCH=1 enables;
    // DL_MALL_PREFETCH_MB sets the w13 head size)
    static bool mallPrefetch() {  // opt-in: measured slower on MI355X (profiles/r1_mall_prefetch.md)
        const char *e = std::getenv("DL_MALL_PREFETCH");
        return e && *e == '1';
    }
    static size_t mallPrefetchBytes() {
        const char *e = std::getenv("DL_MALL_PREFETCH_MB");
        return (size_t)(e && *e ? std::atoi(e) : 24) << 20;
    }

    // Batched path (>= gemmMinTokens rows, Q40 or F32 weights): per chunk of <= 64 tokens, a norm kernel (f32 ->
    // f16, RESNORM) or the producer's f16 rows (xh) feed the MFMA GEMM with the fused epilogue.
    // Residual + norm fusion between batched GEMMs at TP1 (DL_GEMM_FUSE_NORM=0 disables, read at
    // construction): wo / w2 end with EPI_RES (x' = x + out, x' * normW -> f16, per-tile sums of squares)
    // and the next GEMM applies the RMS scale per token in its epilogue: no norm kernel between.
    struct ResFuse {
        const float *resIn;
        float *resOut;
        const float *w;
    };
    // At TP > 1 the batched path keeps the fused residual + norm too when the wo / w2 tiles can be
    // all-reduced inside their GEMM epilogue (GemmArgs::tpx over the fused exchange: narrow
    // launches of <= 64 rows whose tile + Q80 staging fit the launch's LDS); otherwise a separate
    // all-reduce kernel and a norm kernel follow each of them. DL_TP_BATCHED=0 disables it.
    bool tpBatchedOk(int n) const {
        static const bool on = [] {
            const char *e = std::getenv("DL_TP_BATCHED");
            return !(e && *e == '0');
        }();
        return on && tpFused_ && q40_ && !hipk::gemmUsesWide(n) &&
               (size_t)n * h_.dim <= (size_t)tpVec_.stride && hipk::gemmTpxFits(n, plan_.nRanks, tpVec_.q80 != 0);
    }
    bool fuseNorm(int n) const { return fuseNormEnv_ && (plan_.nRanks == 1 || tpBatchedOk(n)); }

  public:
    bool tpBatchedFused(int n) const override { return plan_.nRanks > 1 && batchedPath(n) && fuseNorm(n); }

  private:

    void gemmBatched(const DevMat &m, int n, int epi, const float *in, int ldIn, const float *add, float *xNext,
                     const float *normW, const _Float16 *xh, float *out, int ldOut, _Float16 *outH,
                     const DevLayer *L, const ResFuse *rf = nullptr, bool ssIn = false) {
        // tokens per launch: the wide Q40 kernel takes the whole forward in one launch (one weight
        // pass per token tile, all tiles of a row tile on one XCD), the narrow one <= 128
        const int chunk = q40_ ? (hipk::gemmUsesWide(n) ? n : kGemmMaxTokens) : hipk::kGemmF32MaxTokens;
        for (int c0 = 0; c0 < n; c0 += chunk) {
            const int bc = std::min(chunk, n - c0);
            hipk::GemmArgs g;
            hipk::GemvArgs &a = g.e;
            a.qs = m.qs;
            a.wd = m.d;
            a.wf = m.f;
            a.rows = m.rows;
            a.n = m.n;
            a.lanes = m.lanes;
            a.eps = h_.normEpsilon;
            if (ssIn) {  // input = the producer's x' * normW rows; RMS scale applied per token
                g.x = dXh_ + (size_t)c0 * m.n;
                g.ssIn = dSS_ + c0;
                g.ssTiles = (h_.dim + 63) / 64;
                g.ldSS = (int)cfg_.maxBatch;
            } else if (!xh) {
                hipk::GemvArgs nq;
                nq.n = m.n;
                nq.in = in + (size_t)c0 * ldIn;
                nq.ldIn = ldIn;
                nq.addIn = add ? add + (size_t)c0 * ldIn : nullptr;
                nq.xNext = xNext ? xNext + (size_t)c0 * ldIn : nullptr;
                nq.normW = normW;
                nq.eps = h_.normEpsilon;
                hipk::launchNormF16(nq, dXh_, bc, stream_);
                g.x = dXh_;
            } else {
                g.x = xh + (size_t)c0 * m.n;
            }
            a.out = out ? out + (size_t)c0 * ldOut : nullptr;
            g.outH = outH ? outH + (size_t)c0 * ldOut : nullptr;
            a.ldOut = ldOut;
            a.act = h_.hiddenAct == HiddenAct::GELU ? 0 : 1;
            if (L) {
                a.q0 = plan_.q0;
                a.kv0 = plan_.kv0;
                a.hs = plan_.headSize;
                a.seqLen = h_.seqLen;
                a.rope = dRope_;
                a.pos = dPos_ + c0;
                a.slot = dSlot_ + c0;
                a.kcache = L->k;
                a.kvMap = kvMap();
                a.vcache = L->v;
                a.kvBf16 = kvBf16_ ? 1 : 0;
            }
            if (rf && plan_.nRanks > 1) {  // the residual update needs the rank-summed tile
                g.tpx = 1;
                a.tp = tpVec_;
            }
            if (rf) {
                g.resIn = rf->resIn + (size_t)c0 * ldOut;
                g.resOut = rf->resOut + (size_t)c0 * ldOut;
                g.resW = rf->w;
                g.resX = dXh_ + (size_t)c0 * ldOut;
                g.ssOut = dSS_ + c0;
                g.ldSS = (int)cfg_.maxBatch;
            }
            g.M = bc;
            g.splits = hipk::gemmSplits(m.rows, m.n, bc);
            g.part = dPart_;
            g.counters = dGemmCnt_;
            if (q40_)
                hipk::launchGemmQ40(g, epi, stream_);
            else
                hipk::launchGemmF32(g, epi, stream_);
        }
    }

    // Separate all-reduce of partial sums (batched path, RCCL, f32 weights). Q80 sync: every rank's
    // partial is first rounded through Q80 blocks, as the reference's ZQ cast (llm.cpp:308-314).
    void allReduce(float *buf, size_t count) {
        if (plan_.nRanks > 1) {
            ProfScope ps(this, "allreduce");
            if (syncQ80_) hipk::launchQ80Roundtrip(buf, count, stream_);
            comm_->allReduceSum(buf, count, stream_);
        }
    }
    // Decode rows (GEMV path, Q40) exchange their wo / w2 partials inside the GEMV tail.
    bool fusedTp(bool bat) const { return tpFused_ && !bat && q40_; }

    void enqueueForward(int n, GraphKind kind) {
        const ShardPlan &p = plan_;
        const int dim = h_.dim;
        int cur = 0;
        const bool bat = batchedPath(n);  // MFMA GEMMs on f16 activations instead of GEMVs
        const bool fz = bat && fuseNorm(n);  // residual + norm carried by the GEMM epilogues
        const bool blk = blockOn_ && n == 1 && !bat;  // fused attention block per layer
        const bool fb = ffnOn_ && n == 1 && !bat;     // fused FFN block per layer
        const bool un = unOn_ && n == 1 && !bat;      // residual + norm split (setupUn): x stays in dX_[0]
        {
            ProfScope ps(this, "embedding");
            // the epoch counts the forwards that run a fused block (its counters' targets)
            if (un)
                hipk::launchEmbeddingUn(emb_, dTok_, dX_[0], dim, stream_, blk ? dEpoch_ : nullptr, layers_[0].rmsAtt,
                                        dU_[1], dUnSS_[1]);
            else
                hipk::launchEmbedding(emb_, dTok_, dX_[0], dim, n, stream_, blk || fb ? dEpoch_ : nullptr);
        }
        for (u32 l = 0; l < h_.nLayers; l++) {
            DevLayer &L = layers_[l];
            const bool hasDelta = l > 0;
            if (blk) {
                ProfScope ps(this, "attn_block");
                hipk::AttnBlockArgs ba = attnBlockArgs(L, l, cur);
                if (un) unBlockArgs(ba, L, l);
                if ((int)l == traceLayer_ && !traceFfn_) ba.trace = traceBuf_;
                hipk::launchAttnBlock(ba, fusedTp(false), stream_);
                if (hasDelta && !un) cur ^= 1;
            } else {
            {
                ProfScope ps(this, "gemv_qkv");
                if (fz && hasDelta)
                    gemmBatched(L.qkv, n, hipk::EPI_QKV, nullptr, dim, nullptr, nullptr, nullptr, nullptr, dQ_, p.q0,
                                nullptr, &L, nullptr, true);
                else if (bat)
                    gemmBatched(L.qkv, n, hipk::EPI_QKV, dX_[cur], dim, hasDelta ? dY_ : nullptr,
                                hasDelta ? dX_[cur ^ 1] : nullptr, L.rmsAtt, nullptr, dQ_, p.q0, nullptr, &L);
                else if (un) {
                    hipk::GemvArgs a = gemvArgs(L.qkv, 0, 1, hipk::EPI_QKV, nullptr, dim, nullptr, nullptr, nullptr, dQ_,
                                                p.q0, &L, nullptr, nullptr, nullptr, nullptr, false);
                    unIn(a, 1, l == 0 ? 1 : unW2Grid_);
                    hipk::launchGemv(a, 1, hipk::PRO_UNORM, hipk::EPI_QKV, true, stream_);
                } else
                    gemv(L.qkv, n, hipk::PRO_RESNORM, hipk::EPI_QKV, dX_[cur], dim, hasDelta ? dY_ : nullptr,
                         hasDelta ? dX_[cur ^ 1] : nullptr, L.rmsAtt, dQ_, p.q0, &L);
            }
            if (hasDelta && !un) cur ^= 1;
            const bool pf = mallPrefetch() && q40_ && !profile_;
            {
                ProfScope ps(this, "attention");
                hipk::AttnArgs a = attnArgs(L, bat);
                if (pf) {
                    // attention keeps a handful of CUs busy for several µs while HBM idles: extra
                    // workgroups of the same launch pull wo and the head of w13 into the MALL
                    const hipk::Q40Tiling two = hipk::q40Tiling(L.wo.rows, L.wo.n, L.wo.lanes);
                    const hipk::Q40Tiling t13 = hipk::q40Tiling(L.w13.rows, L.w13.n, L.w13.lanes);
                    a.pf0 = L.wo.qs;
                    a.pf0Bytes = two.qsBytes;
                    a.pf1 = L.w13.qs;
                    a.pf1Bytes = std::min(t13.qsBytes, mallPrefetchBytes());
                    a.pfBlocks = 256;
                }
                if (bat && prefillOk_)
                    hipk::launchAttentionPrefill(a, n, stream_);
                else
                    hipk::launchAttention(a, n, stream_);
            }
            {
                ProfScope ps(this, "gemv_wo");
                if (fz) {
                    const ResFuse rf{dX_[cur], dX_[cur ^ 1], L.rmsFfn};
                    gemmBatched(L.wo, n, hipk::EPI_RES, nullptr, 0, nullptr, nullptr, nullptr, dAttH_, nullptr, dim,
                                nullptr, nullptr, &rf);
                } else if (bat)
                    gemmBatched(L.wo, n, hipk::EPI_STORE, nullptr, 0, nullptr, nullptr, nullptr, dAttH_, dY_, dim,
                                nullptr, nullptr);
                else if (un) {
                    hipk::GemvArgs a = gemvArgs(L.wo, 0, 1, hipk::EPI_STORE_UN, nullptr, p.q0, nullptr, nullptr, nullptr,
                                                nullptr, dim, nullptr, dAttQ_, dAttS_, nullptr, nullptr, false);
                    unOut(a, 0, L.rmsFfn);
                    hipk::launchGemv(a, 1, hipk::PRO_GLOBAL, hipk::EPI_STORE_UN, true, stream_);
                } else
                    gemv(L.wo, n, hipk::PRO_GLOBAL, hipk::EPI_STORE, q40_ ? nullptr : dAtt_, p.q0, nullptr, nullptr,
                         nullptr, dY_, dim, nullptr, dAttQ_, dAttS_, nullptr, nullptr, fusedTp(bat));
            }
            }
            if (!fusedTp(bat) && !fz) allReduce(dY_, (size_t)n * dim);
            // Q80 hand-off of h needs one workgroup per 32 hidden units; for skinny TP shards the
            // w13 epilogue emits f32 and w2 quantizes in its prologue instead.
            const bool hQ80 = q40_ && p.hidden0 / 32 >= 192;
            if (fb) {
                ProfScope ps(this, "ffn_block");
                hipk::FfnBlockArgs fa = ffnBlockArgs(L, l, cur);
                if ((int)l == traceLayer_ && traceFfn_) fa.trace = traceBuf_;
                hipk::launchFfnBlock(fa, fusedTp(false), stream_);
                cur ^= 1;
            } else {
            {
                ProfScope ps(this, "gemv_w13");
                if (fz)
                    gemmBatched(L.w13, n, hipk::EPI_ACT_F16, nullptr, dim, nullptr, nullptr, nullptr, nullptr, nullptr,
                                p.hidden0, dHh_, nullptr, nullptr, true);
                else if (bat)
                    gemmBatched(L.w13, n, hipk::EPI_ACT_F16, dX_[cur], dim, dY_, dX_[cur ^ 1], L.rmsFfn, nullptr,
                                nullptr, p.hidden0, dHh_, nullptr);
                else if (un) {
                    hipk::GemvArgs a = gemvArgs(L.w13, 0, 1, hipk::EPI_ACT_Q80, nullptr, dim, nullptr, nullptr, nullptr,
                                                dH_, p.hidden0, nullptr, nullptr, nullptr, dHQ_, dHS_, false);
                    unIn(a, 0, unWoGrid_);
                    hipk::launchGemv(a, 1, hipk::PRO_UNORM, hipk::EPI_ACT_Q80, true, stream_);
                } else
                    gemv(L.w13, n, hipk::PRO_RESNORM, hQ80 ? hipk::EPI_ACT_Q80 : hipk::EPI_ACT, dX_[cur], dim, dY_,
                         dX_[cur ^ 1], L.rmsFfn, dH_, p.hidden0, nullptr, nullptr, nullptr, dHQ_, dHS_);
            }
            if (!un) cur ^= 1;
            {
                ProfScope ps(this, "gemv_w2");
                if (fz) {
                    const float *wNext = l + 1 < h_.nLayers ? layers_[l + 1].rmsAtt : rmsFinal_;
                    const ResFuse rf{dX_[cur], dX_[cur ^ 1], wNext};
                    gemmBatched(L.w2, n, hipk::EPI_RES, nullptr, 0, nullptr, nullptr, nullptr, dHh_, nullptr, dim,
                                nullptr, nullptr, &rf);
                } else if (bat)
                    gemmBatched(L.w2, n, hipk::EPI_STORE, nullptr, 0, nullptr, nullptr, nullptr, dHh_, dY_, dim,
                                nullptr, nullptr);
                else if (un) {
                    hipk::GemvArgs a = gemvArgs(L.w2, 0, 1, hipk::EPI_STORE_UN, nullptr, p.hidden0, nullptr, nullptr,
                                                nullptr, nullptr, dim, nullptr, dHQ_, dHS_, nullptr, nullptr, false);
                    unOut(a, 1, unNextNorm(l));
                    hipk::launchGemv(a, 1, hipk::PRO_GLOBAL, hipk::EPI_STORE_UN, true, stream_);
                } else if (hQ80 || !q40_)
                    gemv(L.w2, n, hipk::PRO_GLOBAL, hipk::EPI_STORE, q40_ ? nullptr : dH_, p.hidden0, nullptr,
                         nullptr, nullptr, dY_, dim, nullptr, dHQ_, dHS_, nullptr, nullptr, fusedTp(bat));
                else
                    gemv(L.w2, n, hipk::PRO_RESNORM, hipk::EPI_STORE, dH_, p.hidden0, nullptr, nullptr, nullptr, dY_,
                         dim, nullptr, nullptr, nullptr, nullptr, nullptr, fusedTp(bat));
            }
            }
            if (!fusedTp(bat) && !fz) allReduce(dY_, (size_t)n * dim);
        }
        {
            ProfScope ps(this, "gemv_logits");
            if (fz)
                gemmBatched(wcls_, n, hipk::EPI_STORE, nullptr, dim, nullptr, nullptr, nullptr, nullptr, dLogits_,
                            p.vocab0, nullptr, nullptr, nullptr, true);
            else if (bat)
                gemmBatched(wcls_, n, hipk::EPI_STORE, dX_[cur], dim, dY_, nullptr, rmsFinal_, nullptr, dLogits_,
                            p.vocab0, nullptr, nullptr);
            else if (un) {
                hipk::GemvArgs a = gemvArgs(wcls_, 0, 1, hipk::EPI_STORE, nullptr, dim, nullptr, nullptr, nullptr, dLogits_,
                                            p.vocab0, nullptr, nullptr, nullptr, nullptr, nullptr, false);
                unIn(a, 1, unW2Grid_);
                hipk::launchGemv(a, 1, hipk::PRO_UNORM, hipk::EPI_STORE, true, stream_);
            } else
                gemv(wcls_, n, hipk::PRO_RESNORM, hipk::EPI_STORE, dX_[cur], dim, dY_, nullptr, rmsFinal_, dLogits_,
                     p.vocab0, nullptr);
        }
        const float *full = dLogits_;
        // greedy rows on a fused TP data plane: each rank reduces its own vocab slice and only the
        // (value, index) winners cross the links (reference: logits gathered to the root,
        // llm.cpp:432); the full logits are gathered only when the host samples them
        const bool distArgmax = tpFused_ && (kind == GraphKind::ARGMAX || kind == GraphKind::CHAIN);
        // logits for the host (LOGITS) and sampled rows (SAMPLE) are needed on the root only: the
        // vocab slices are gathered to rank 0 (the reference's SYNC_NODE_SLICES_EXCEPT_ROOT), the
        // other ranks publish theirs and skip the unshard and the draw (the root's ids are used)
        const bool rootOnly = kind == GraphKind::LOGITS || kind == GraphKind::SAMPLE;
        if (p.nRanks > 1 && !distArgmax) {
            ProfScope ps(this, "allgather");
            if (rootOnly)
                comm_->gatherToRoot(dLogits_, dLogitsAll_, (size_t)n * p.vocab0, stream_);
            else
                comm_->allGather(dLogits_, dLogitsAll_, (size_t)n * p.vocab0, stream_);
            if (!rootOnly || rank() == 0)
                hipk::launchUnshardLogits(dLogitsAll_, dLogitsFull_, p.nRanks, n, p.vocab0, stream_);
            full = dLogitsFull_;
        }
        if (kind == GraphKind::SAMPLE && (p.nRanks == 1 || rank() == 0)) {
            ProfScope ps(this, "sample");
            hipk::SampleArgs g;
            g.logits = full;
            g.vocab = h_.vocabSize;
            g.spec = dSpec_;
            g.ids = dIds_;
            g.scratch = sampleScratch_;
            hipk::launchSample(g, n, stream_);
        } else if (kind != GraphKind::LOGITS) {
            ProfScope ps(this, "argmax");
            hipk::ArgmaxArgs g;
            g.logits = full;
            g.vocab = h_.vocabSize;
            if (distArgmax) {
                g.vocab = p.vocab0;
                g.vocabStart = p.vocabStart();
                g.tp = tpArg_;
            }
            g.ids = dIds_;
            g.partV = dArgV_;
            g.partI = dArgI_;
            g.counters = dArgCnt_;
            if (kind == GraphKind::CHAIN) {
                // feed the sampled token back: tokens := ids, hist[b][pos] := ids, pos += 1
                g.tokens = dTok_;
                g.pos = dPos_;
                g.hist = dHist_;
                g.seqLen = h_.seqLen;
            }
            hipk::launchArgmax(g, n, stream_);
        }
        DL_HIP(hipGetLastError());
    }

    static constexpr int kGemmMaxTokens = hipk::kGemmMaxTokens;  // tokens per MFMA GEMM launch (one weight pass)
    _Float16 *dXh_ = nullptr, *dAttH_ = nullptr, *dHh_ = nullptr;
    float *dPart_ = nullptr;
    int *dGemmCnt_ = nullptr;
    std::unordered_set<int> graphSeen_;  // graph keys used once (captured on the second use)
    float *dSS_ = nullptr;

    EngineConfig cfg_;
    DeviceComm *comm_;
    int dev_ = 0;
    hipStream_t stream_ = nullptr;

    std::unique_ptr<ModelFile> file_;
    ModelHeader h_;
    ShardPlan plan_;
    bool q40_ = true, kvBf16_ = true, syncQ80_ = false, tpFused_ = false;
    int fusedGridMax_ = 0;  // largest grid of a fused-exchange GEMV launch (checked co-resident)
    static constexpr int kMaxKvGroups = 64;
    // counters: [64 groups x 64 words] qkv arrivals, [64] attention arrivals, [8 x 64] ready flags
    // + [64] qkv arrivals, [8 x 64] qkv-done flags (attn_block_inst.h carves them after attnFlag)
    // attention block: qkv counters per KV group | attention counter | 8 flags | qkv counter | 8 flags |
    // spare line; FFN block: w13 counter | 8 flags (every word on its own 256-B line)
    static constexpr int kFfnCntOff = kMaxKvGroups * 64 + 64 + 8 * 64 + 64 + 8 * 64 + 64;
    static constexpr int kBlockCntWords = kFfnCntOff + 64 + 8 * 64;
    unsigned *dEpoch_ = nullptr, *dBlockCnt_ = nullptr, *dBlockExpect_ = nullptr;
    int *dBlockErr_ = nullptr;
    bool blockOn_ = false;  // decode rows run the fused attention block (setupAttnBlock)
    bool unOn_ = false;     // decode rows split residual + norm between producer and consumer (setupUn)
    int unWoGrid_ = 0, unW2Grid_ = 0;  // partial sums the wo / w2 producers leave (one per workgroup)
    bool ffnOn_ = false;
    static constexpr int kAttnMfmaMinPos = 1024;
    bool attnLong_ = false;  // this forward's decode attention runs the MFMA kernel (setInputs)
    // paged KV cache (setupPages / mapPages)
    int *dKvTable_ = nullptr;
    int *hTableStage_[2] = {nullptr, nullptr};
    int tableFlip_ = 0, pageShift_ = 0, pagesPerSlot_ = 0;
    bool tableDirty_ = false;
    std::vector<int> hostTable_, slotPages_, freePages_;
    int ffnSameWg_ = 0;     // DL_FFN_BLOCK=2: w13 and w2 rows on the same workgroups    // decode rows run the fused FFN block (setupFfnBlock)
    int ffnRingEarly_ = 0, ffnW13PassMul_ = 1;
    bool traceFfn_ = false;  // traceAttnBlock(layer, ffn=true) traces the FFN block instead
    int traceLayer_ = -1;   // traceAttnBlock: the layer whose block launch is traced
    unsigned long long *traceBuf_ = nullptr;
    int blockGrid_ = 0;
    int gemmMin_ = 3;       // DL_GEMM_MIN: rows per forward from which the batched MFMA path runs
    bool fuseNormEnv_ = true;  // DL_GEMM_FUSE_NORM
    hipk::TpXchg tpVec_, tpArg_;
    std::vector<void *> allocs_, hostAllocs_;
    size_t deviceBytes_ = 0;
    LoadStats load_;
    hipk::SampleScratch sampleScratch_;
    std::vector<DevLayer> layers_;
    DevMat wcls_;
    float *emb_ = nullptr, *rmsFinal_ = nullptr;
    int *dTok_ = nullptr, *dPos_ = nullptr, *dSlot_ = nullptr, *dIds_ = nullptr, *dHist_ = nullptr;
    float4 *dSpec_ = nullptr;
    int *hIn_ = nullptr, *hIds_ = nullptr, *hErr_ = nullptr;
    float *hLogits_ = nullptr;
    float *dX_[2] = {nullptr, nullptr};
    float *dU_[2] = {nullptr, nullptr};   // normW * x from EPI_STORE_UN producers ([0] wo, [1] w2 / embedding)
    float *dUnSS_[2] = {nullptr, nullptr};  // their per-workgroup partial sums of squares
    float *dY_ = nullptr, *dQ_ = nullptr, *dAtt_ = nullptr, *dH_ = nullptr, *dLogits_ = nullptr;
    float *dLogitsAll_ = nullptr, *dLogitsFull_ = nullptr;
    float *dPartO_ = nullptr, *dPartML_ = nullptr;
    int8_t *dAttQ_ = nullptr, *dHQ_ = nullptr;
    float2 *dAttS_ = nullptr, *dHS_ = nullptr;
    int *dAttCnt_ = nullptr, *dArgCnt_ = nullptr, *dArgI_ = nullptr;
    float *dArgV_ = nullptr;
    float2 *dRope_ = nullptr;
    int splitGrid_ = 1, chunkMax_ = 256;
    bool prefillOk_ = false;  // this forward's rows qualify for the MFMA prefill attention
    std::map<int, hipGraphExec_t> graphs_;
    bool profile_ = false;
    bool graphsBroken_ = false;
    bool inputsInFlight_ = false;  // an H2D copy from hIn_ may still be pending
    int pendingN_ = 0;             // rows of a launchIds forward not collected yet
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> profTimes_;
};

}  // namespace

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

double benchGemmQ40(int rows, int n, int M, int epi, int copies, int iters) {
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
    const int MP = hipk::gemmTokenPad(M);
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
    g.splits = hipk::gemmSplits(rows, n, M);
    g.part = part ? (float *)alloc(part * 4) : nullptr;
    g.counters = (int *)alloc((size_t)(rows / 64 + 1) * 4);
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
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(gr);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (void *p : mem) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return ms * 1000.0 / iters;
}

double benchAttention(int nHeads0, int kvMul, int hs, int seqLen, int pos, int B, int copies, int iters) {
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
    for (int c = 0; c < copies; c++) {
        kc[c] = alloc(kvElems * 2);
        vc[c] = alloc(kvElems * 2);
        hipk::launchFillF32Uniform((float *)kc[c], kvElems / 2, 1.f, 5 + c, s);  // bf16 pairs of small values
        hipk::launchFillF32Uniform((float *)vc[c], kvElems / 2, 1.f, 9 + c, s);
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
    a.partO = (float *)alloc((size_t)B * nHeads0 * a.splitGrid * hs * 4);
    a.partML = (float *)alloc((size_t)B * nHeads0 * a.splitGrid * 2 * 4);
    a.outQ = (int8_t *)alloc((size_t)B * q0);
    a.outS = (float2 *)alloc((size_t)B * q0 / 32 * 8);
    a.ldOut = q0;
    a.kvBf16 = 1;
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
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (void *p : mem) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return ms * 1000.0 / iters;
}

std::unique_ptr<HipEngine> makeHipEngine(const EngineConfig &cfg, DeviceComm *comm) {
    return std::unique_ptr<HipEngine>(new HipEngineImpl(cfg, comm));
}

}  // namespace dl
