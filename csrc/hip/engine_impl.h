// HipEngine implementation class, shared by the engine's translation units:
//   engine.cpp          construction, public entry points, hipGraph cache, error checks
//   engine_load.cpp     device buffers, weight upload (file pipeline / synthetic), capacity checks
//   engine_kv.cpp       paged KV cache (page table per slot over per-layer pools)
//   engine_forward.cpp  the per-forward kernel schedule (GEMV / GEMM / attention / block launches)
//   engine_bench.cpp    kernel microbenchmarks (scripts/bench_*.py)
//
// Weight residency: every rank repacks ITS shard of the mmapped `.m` file on the host into the
// GPU layout and uploads it once (reference: root streams shards to workers over TCP,
// nn-network.cpp:766-901; llm.cpp:447-483 defines the slices). Q40 matrices become SoA
// (16-byte nibble rows + f16 scale plane) so a lane's 16-byte load is one whole block.
// Fusions baked into the layout:
//   Wq|Wk|Wv row slices concatenated -> one QKV GEMV (+RoPE +KV append epilogue)
//   W1/W3 row slices interleaved      -> one GEMV whose epilogue computes act(w1 x) * (w3 x)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <unordered_set>
#include <vector>

#include "../core/model_file.h"
#include "../core/plan.h"
#include "../runtime/metrics.h"
#include "engine.h"
#include "kernels.h"

namespace dl {
namespace engine_detail {

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

// Decode context bucket: the attention launches of a forward are sized for the longest context
// this forward can reach (the bucket's upper bound), not for the engine's capacity, so a
// 4K / 128K-capacity engine decodes short contexts with the grids of a short engine (and keeps
// the fused attention block). Part of the graph key.
struct CtxBucket {
    int maxLen = 0;     // positions covered (<= seqLen)
    int splitGrid = 1;  // attention sequence splits at this length (single decode rows: short chunks)
    int splitGridBat = 1;  // the same for batched rows (256-key chunks throughout)
    int chunkMax = 256;
    bool block = false; // the fused attention block fits co-resident at this bucket's grid
};

class HipEngineImpl : public HipEngine {
  public:
    HipEngineImpl(const EngineConfig &cfg, DeviceComm *comm);
    ~HipEngineImpl() override;

    // Backend
    const ModelHeader &header() const override { return h_; }
    const ShardPlan &plan() const override { return plan_; }
    std::string name() const override { return "hip"; }
    LoadStats loadStats() const override { return load_; }
    void forward(int n, const int *tokens, const int *positions, const int *slots, float *logits) override;
    void forwardArgmax(int n, const int *tokens, const int *positions, const int *slots, int *out) override;
    void forwardSample(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs,
                       int *out) override;
    void launchIds(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs) override;
    void collectIds(int *out) override;
    bool chainSupported() const override { return true; }
    void chainLaunch(int token, int pos, int slot) override;
    int chainCollect() override;
    int chainInFlight() const override { return (int)(chainHead_ - chainTail_); }
    int kvPagesFree() const override { return paged() ? (int)freePages_.size() : -1; }
    int kvPageSize() const override { return paged() ? (int)cfg_.kvPageSize : 0; }
    void releaseSlot(int slot) override;

    // HipEngine
    double decodeGreedy(int steps, int token, int pos, int slot, int *outTokens) override {
        return decodeGreedyBatch(steps, 1, &token, &pos, &slot, outTokens);
    }
    double decodeGreedyBatch(int steps, int nSeq, const int *tokens, const int *pos, const int *slots,
                             int *outTokens) override;
    void synchronize() override { DL_HIP(hipStreamSynchronize(stream_)); }
    size_t deviceBytes() const override { return deviceBytes_; }
    void profileForward(int n, const int *tokens, const int *positions, const int *slots) override;
    bool tpFused() const override { return tpFused_; }
    bool attnBlock() const override { return blockOn_; }
    bool woAttn() const override { return woAttnOn_; }
    bool prenorm() const override { return prenormOn_; }
    bool ffnBlock() const override { return ffnOn_; }
    std::vector<unsigned long long> traceAttnBlock(int token, int pos, int slot, int layer) override;
    int fusedGridMax() const override { return fusedGridMax_; }
    bool tpBatchedFused(int n) const override { return plan_.nRanks > 1 && batchedPath(n) && fuseNorm(n); }

    // ------------------------------------------------------------------ internals
    enum class GraphKind { LOGITS = 0, ARGMAX = 1, CHAIN = 2, SAMPLE = 3 };

    // engine.cpp
    void syncAndCheckComm();
    void enqueueErrorCopies();
    void checkErrorWords();
    int rank() const { return comm_ ? comm_->rank() : 0; }
    // syncDst: host copy of the forward's measured-sync slots (null: none, e.g. inside a decode chain)
    void runGraph(int n, GraphKind kind, unsigned *syncDst);
    void runGraph(int n, GraphKind kind) { runGraph(n, kind, hSync_); }
    void accountForward(int n, GraphKind kind, int times);
    // measured sync (ForwardStats::syncMs / xchgMs): one slot per (exchange, launch) of a forward
    // (exchange xSlot_: layer l's wo 2l, w2 2l + 1, the logits / argmax exchange 2L; launch xChunk_:
    // the batch chunks of one GEMV / GEMM, each its own slot so their waits add up): a u32 of
    // fused-exchange wait ticks (max over the waves), a u32 of exchange-tail ticks (max over the
    // workgroups, DL_SYNC_MEASURE=2) and a pair of u64 stamps around a separate collective
    // (hipk::syncFoldWords layout). Each forward's embedding kernel folds the previous forward's
    // slots into device running totals and clears them; the host copies them after a forward
    // (or one chain step) and reads the totals after a whole decode chain.
    static constexpr int kSyncChunks = 4;
    int syncSlots() const { return (2 * (int)h_.nLayers + 2) * kSyncChunks; }
    // DL_SYNC_MEASURE: 0 off (comparison runs: no wait ticks, no stamp kernels), 1 (default) the
    // longest peer wait per exchange, 2 also the longest exchange tail per exchange (the xchg span:
    // a stamp pair and an atomic per workgroup tail, ~2.5 % of a TP8 rank's decode, r5_tp_rank.md)
    const int syncLevel_ = [] {
        const char *e = std::getenv("DL_SYNC_MEASURE");
        return e && *e ? std::max(0, std::min(2, std::atoi(e))) : 1;
    }();
    int xChunk_ = 0;  // launch index within the exchange being enqueued
    int syncSlotNow() const { return xSlot_ * kSyncChunks + std::min(xChunk_, kSyncChunks - 1); }
    unsigned *syncTicks() const { return syncLevel_ ? dSync_ + syncSlotNow() : nullptr; }
    unsigned *syncSpan() const { return syncLevel_ >= 2 ? dSync_ + syncSlots() + syncSlotNow() : nullptr; }
    unsigned long long *syncStamps() const {
        return reinterpret_cast<unsigned long long *>(dSync_ + 2 * syncSlots()) + 2 * syncSlotNow();
    }
    struct SyncRead {
        double waitMs = 0, spanMs = -1;  // spanMs < 0: not measured (DL_SYNC_MEASURE < 2, no collective)
    };
    // buf: a host copy of the slots; totals: add the running totals of the folded forwards
    SyncRead readSync(const unsigned *buf, bool totals) const;
    void setSyncStats(const SyncRead &r, double capMs);
    template <typename F>
    void stamped(F &&collective) {  // a separate collective, bracketed by stamps (when measured)
        if (syncLevel_) launchStampAt(syncStamps());
        collective();
        if (syncLevel_) launchStampAt(syncStamps() + 1);
    }
    void launchStampAt(unsigned long long *p);
    void tpFusedSelfTest();
    hipGraphExec_t captureForward(int n, GraphKind kind);
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

    // engine_load.cpp
    void checkFits();
    void checkFusedResidency();
    void allocBuffers();
    void uploadRope();
    size_t matStageBytes(u32 rows, u32 n) const;
    // lanes per row of a matrix's Q40 tiling (the GEMV's choice)
    static int lanesFor(int rows, int n) { return hipk::gemvLanesPerRow(n, rows, 1, true); }
    void placeQ40(DevMat &m, const hipk::Q40Tiling &t, int mi, u32 l);
    struct RowSrc {
        const TensorInfo *t;
        u32 r0, nr;
    };
    struct Loader;
    u8 *stageAcquire(Loader &ld);
    void stageCopy(Loader &ld, void *dst, const u8 *src, size_t bytes);
    void stageRelease(Loader &ld);
    void readRows(Loader &ld, const std::vector<RowSrc> &srcs, bool interleave, u32 c0, u32 nc);
    void buildMat(Loader &ld, DevMat &m, const std::vector<RowSrc> &srcs, bool interleave, u32 c0, u32 nc, int mi,
                  u32 l);
    float *uploadF32(Loader &ld, const TensorInfo &t);
    void loadFromFile();
    void synthMat(DevMat &m, int rows, int n, u64 seed, int mi, u32 l);
    void loadSynthetic();

    // engine_kv.cpp
    size_t kvPoolRows() const {
        return cfg_.kvPages ? (size_t)cfg_.kvPages * cfg_.kvPageSize : (size_t)cfg_.nSlots * h_.seqLen;
    }
    bool paged() const { return cfg_.kvPages > 0; }
    void setupPages();
    hipk::KvMap kvMap() const;
    void mapPages(int n, const int *positions, const int *slots, int ahead);

    // engine_forward.cpp
    void setupBuckets();
    const CtxBucket &bucketFor(int maxPos) const;
    void setInputs(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs = nullptr,
                   int ahead = 0);
    int tpPasses(const DevMat &m, int bc) const;
    int batchChunk(const DevMat &m, int pro, int epi) const;
    int passesFor(const DevMat &m, int epi, int B) const {
        return hipk::gemvDefaultPasses(m.n, m.rows, B, q40_, epi, q40_ ? m.lanes : 0);
    }
    hipk::GemvArgs gemvArgs(const DevMat &m, int c0, int bc, int epi, const float *in, int ldIn, const float *add,
                            float *xNext, const float *normW, float *out, int ldOut, const DevLayer *L,
                            const int8_t *aq, const float2 *as, int8_t *oq, float2 *os, bool tp) const;
    void gemv(const DevMat &m, int n, int pro, int epi, const float *in, int ldIn, const float *add, float *xNext,
              const float *normW, float *out, int ldOut, const DevLayer *L, const int8_t *aq = nullptr,
              const float2 *as = nullptr, int8_t *oq = nullptr, float2 *os = nullptr, bool tp = false);
    hipk::AttnArgs attnArgs(const DevLayer &L, bool bat) const;
    hipk::AttnBlockArgs attnBlockArgs(const DevLayer &L, u32 l, int cur) const;
    void setupAttnBlock();
    void resetAttnBlockState();
    // the wo GEMV with the attention in its prologue (PRO_ATTN) for single decode rows of short
    // contexts when a rank holds few heads: decided once (setupWoAttn), taken per forward (woAttnNow)
    void setupWoAttn();
    // pre-normalized hand-off for single decode rows (EPI_RESQ_TP producers -> PRO_PRENORM
    // consumers): decided once (setupPrenorm), taken per forward (prenormNow)
    void setupPrenorm();
    bool prenormNow(int n, bool bat, bool blk) const { return prenormOn_ && n == 1 && !bat && !blk; }
    // fused FFN block (w13 + w2 roles in one launch) inside the pre-normalized layers: setupFfnBlock
    void setupFfnBlock();
    hipk::FfnBlockArgs ffnBlockArgs(const hipk::GemvArgs &w13, const hipk::GemvArgs &w2, u32 l);
    void enqueuePrenormLayers(GraphKind kind, bool argTail);
    bool woAttnNow(int n, bool bat, bool blk) const {
        return woAttnOn_ && n == 1 && !bat && !blk && buckets_[bucket_].maxLen <= woAttnMaxLen_;
    }
    bool batchedPath(int n) const {
        return n >= gemmMin_ && hipk::gemmSupported(h_.dim) && hipk::gemmSupported(plan_.q0) &&
               hipk::gemmSupported(plan_.hidden0);
    }
    struct ResFuse {
        const float *resIn;
        float *resOut;
        const float *w;
    };
    bool tpBatchedOk(int n) const;
    bool fuseNorm(int n) const { return fuseNormEnv_ && (plan_.nRanks == 1 || tpBatchedOk(n)); }
    void gemmBatched(const DevMat &m, int n, int epi, const float *in, int ldIn, const float *add, float *xNext,
                     const float *normW, const _Float16 *xh, float *out, int ldOut, _Float16 *outH,
                     const DevLayer *L, const ResFuse *rf = nullptr, bool ssIn = false);
    void allReduce(float *buf, size_t count);
    bool fusedTp(bool bat) const { return tpFused_ && !bat && q40_; }
    void enqueueForward(int n, GraphKind kind);

    // timing hook for profileForward (eager only)
    struct ProfScope;

    // ------------------------------------------------------------------ state
    static constexpr int kGemmMaxTokens = hipk::kGemmMaxTokens;  // tokens per MFMA GEMM launch (one weight pass)
    static constexpr int kMaxKvGroups = 64;
    // attention block counters: qkv counters per KV group | attention counter | 8 flags | qkv counter |
    // 8 flags | spare line (every word on its own 256-B line; attn_block_inst.h carves them)
    static constexpr int kBlockCntWords = kMaxKvGroups * 64 + 64 + 8 * 64 + 64 + 8 * 64 + 64;
    // the FFN block's words after the attention block's: [64] arrivals, [8 * 64] per-XCD flags
    static constexpr int kFfnCntOff = kBlockCntWords, kAllCntWords = kBlockCntWords + 64 + 8 * 64;
    static constexpr int kAttnMfmaMinPos = 1024;
    static constexpr int kAttnMfmaMinRows = 16;

    EngineConfig cfg_;
    DeviceComm *comm_;
    int dev_ = 0;
    hipStream_t stream_ = nullptr;
    std::unique_ptr<ModelFile> file_;
    ModelHeader h_;
    ShardPlan plan_;
    bool q40_ = true, kvBf16_ = true, syncQ80_ = false, tpFused_ = false;
    bool tpTested_ = false;  // tpFusedSelfTest ran (first forward)
    int fusedGridMax_ = 0;  // largest grid of a fused-exchange GEMV launch (checked co-resident)
    hipk::TpXchg tpVec_, tpArg_;
    int gemmMin_ = 3;          // DL_GEMM_MIN: rows per forward from which the batched MFMA path runs
    int decodeRows_ = 1;       // EngineConfig::maxDecode (<= maxBatch): greedy-chain rows, fused argmax rows
    int attRows_ = 1;          // rows per attention launch (the split partials hold this many rows)
    bool fuseNormEnv_ = true;  // DL_GEMM_FUSE_NORM
    bool invariant_ = false;   // EngineConfig::batchInvariant
    // single-row decode: w13 hands h to w2 as Q80 blocks (64-row w13 workgroups) when the shard has
    // >= 192 blocks of 32 hidden units, else as f32 that w2 quantizes in its prologue (DL_H_Q80=0/1
    // forces either)
    bool hQ80_ = true;
    std::vector<void *> allocs_, hostAllocs_;
    size_t deviceBytes_ = 0;
    LoadStats load_;

    // weights (layer matrices of one kind in one slab per kind: placeQ40)
    uint8_t *qsSlab_[4] = {};
    uint16_t *dSlab_[4] = {};
    size_t qsStride_[4] = {}, dStride_[4] = {};
    std::vector<DevLayer> layers_;
    DevMat wcls_;
    float *emb_ = nullptr, *rmsFinal_ = nullptr;
    float2 *dRope_ = nullptr;

    // per-forward inputs and outputs
    int *dTok_ = nullptr, *dPos_ = nullptr, *dSlot_ = nullptr, *dIds_ = nullptr, *dHist_ = nullptr;
    float4 *dSpec_ = nullptr;
    int *hIn_ = nullptr, *hIds_ = nullptr, *hErr_ = nullptr;
    float *hLogits_ = nullptr;  // pinned logits staging (forward with host logits), grown on demand
    size_t hLogitsCap_ = 0;
    bool inputsInFlight_ = false;  // an H2D copy from hIn_ may still be pending
    int pendingN_ = 0;             // rows of a launchIds forward not collected yet
    // chained decode (chainLaunch / chainCollect): a ring of pinned id words and their events
    // the logits GEMV of a greedy decode row ends in its argmax (EPI_ARGMAX; DL_ARGMAX_TAIL=0: the
    // separate argmax kernel, comparison runs)
    const bool argTailOn_ = [] {
        const char *e = std::getenv("DL_ARGMAX_TAIL");
        return !(e && *e == '0');
    }();
    static constexpr int kChainDepth = 4;
    int *hChain_ = nullptr;
    hipEvent_t chainEv_[kChainDepth] = {};
    long long chainHead_ = 0, chainTail_ = 0;  // steps launched / collected
    int chainSlot_ = 0;

    // activations
    float *dX_[2] = {nullptr, nullptr};
    float *dY_ = nullptr, *dQ_ = nullptr, *dAtt_ = nullptr, *dH_ = nullptr, *dLogits_ = nullptr;
    float *dLogitsAll_ = nullptr, *dLogitsFull_ = nullptr;
    int8_t *dAttQ_ = nullptr, *dHQ_ = nullptr;
    // pre-normalized hand-off (one row), by residual parity: Q80 of x * normW, scales, partial sums
    int8_t *dXQ_[2] = {nullptr, nullptr};
    float2 *dXS_[2] = {nullptr, nullptr};
    float *dSSP_[2] = {nullptr, nullptr};
    float2 *dAttS_ = nullptr, *dHS_ = nullptr;
    _Float16 *dXh_ = nullptr, *dAttH_ = nullptr, *dHh_ = nullptr;
    float *dPart_ = nullptr;
    size_t partFloats_ = 0;
    int *dGemmCnt_ = nullptr;
    float *dSS_ = nullptr;
    float *dPartO_ = nullptr, *dPartML_ = nullptr;
    int *dAttCnt_ = nullptr, *dArgCnt_ = nullptr, *dArgI_ = nullptr;
    float *dArgV_ = nullptr;
    float *dArgPairs_ = nullptr, *dArgPairsAll_ = nullptr;  // separate-collective TP argmax
    hipk::SampleScratch sampleScratch_;
    // measured-sync slots (syncSlots, hipk::syncFoldWords) and their host copies: [0] the last
    // forward / chain, [1 + k] chain step k % kChainDepth (chainLaunch / chainCollect)
    unsigned *dSync_ = nullptr, *hSync_ = nullptr;
    unsigned *hSyncAt(int i) const { return hSync_ + (size_t)i * hipk::syncFoldWords(syncSlots()); }
    int xSlot_ = 0;                                  // slot of the exchange being enqueued

    // attention: context buckets (setupBuckets) and this forward's choices (setInputs, graph key)
    std::vector<CtxBucket> buckets_;
    int bucket_ = 0;          // index into buckets_
    bool attnLong_ = false;   // decode attention runs the MFMA kernel
    bool prefillOk_ = false;  // the rows qualify for the MFMA prefill attention

    // fused attention block
    unsigned *dEpoch_ = nullptr, *dBlockCnt_ = nullptr, *dBlockExpect_ = nullptr;
    int *dBlockErr_ = nullptr;
    bool blockOn_ = false;   // decode rows may run the fused attention block (per bucket: CtxBucket::block)
    bool woAttnOn_ = false;  // setupWoAttn
    bool prenormOn_ = false; // setupPrenorm
    bool ffnOn_ = false;     // setupFfnBlock (prenorm forwards only)
    static constexpr int kMaxSsp = 256;  // producer workgroups of a pre-normalized hand-off
    int woAttnMaxLen_ = 256; // DL_WO_ATTN_LEN: context buckets up to this length
    int blockPassMul_ = 1;   // qkv / wo passes multiplier of the block's roles (same-GPU rehearsals)
    int traceLayer_ = -1;    // traceAttnBlock: the layer whose block launch is traced
    unsigned long long *traceBuf_ = nullptr;

    // paged KV cache (setupPages / mapPages)
    int *dKvTable_ = nullptr;
    int *hTableStage_[2] = {nullptr, nullptr};
    int tableFlip_ = 0, pageShift_ = 0, pagesPerSlot_ = 0;
    bool tableDirty_ = false;
    std::vector<int> hostTable_, slotPages_, freePages_;

    // graphs
    std::map<int, hipGraphExec_t> graphs_;
    std::unordered_set<int> graphSeen_;  // graph keys used once (captured on the second use)
    bool graphsBroken_ = false;
    bool profile_ = false;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> profTimes_;
};

struct HipEngineImpl::ProfScope {
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

}  // namespace engine_detail
}  // namespace dl
