// HipEngine: construction, public entry points, hipGraph cache and error checks (engine_impl.h
// lists the other translation units of the engine).
#include "engine_impl.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace dl {

int hipDeviceCount() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

namespace engine_detail {

HipEngineImpl::HipEngineImpl(const EngineConfig &cfg, DeviceComm *comm) : cfg_(cfg), comm_(comm) {
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
    decodeRows_ = (int)(cfg.maxDecode ? std::min(cfg.maxDecode, cfg.maxBatch) : cfg.maxBatch);
    if (comm_ && plan_.nRanks > 1) {
        const char *e = std::getenv("DL_TP_FUSED");  // 0: separate all-reduce kernels (comparison)
        tpFused_ = !(e && *e == '0') && comm_->fusedXchg(0, &tpVec_) && comm_->fusedXchg(1, &tpArg_) &&
                   (size_t)std::min<u32>(cfg.maxBatch, 4) * h_.dim <= (size_t)tpVec_.stride &&
                   (size_t)2 * decodeRows_ <= (size_t)tpArg_.stride;  // larger argmax forwards: all-gather
        tpVec_.q80 = syncQ80_ ? 1 : 0;
    }
    checkFits();
    {
        const char *hq = std::getenv("DL_H_Q80");
        hQ80_ = hq && *hq ? *hq == '1' : plan_.hidden0 / 32 >= 192;
    }
    if (tpFused_) checkFusedResidency();
    {  // path knobs, read once: a captured graph replays the path it was captured with
        const char *e = std::getenv("DL_GEMM_MIN");
        gemmMin_ = e && *e ? std::atoi(e) : (plan_.nRanks > 1 ? 5 : 3);
        // batch-invariant serving: every row of every forward takes the narrow MFMA GEMMs (fixed
        // splits, no 16-lane / wide variants) and the VALU decode attention, so a row's math does
        // not depend on how many rows share its forward (EngineConfig::batchInvariant)
        invariant_ = cfg.batchInvariant;
        if (invariant_) gemmMin_ = 1;
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
    setupWoAttn();
    setupPrenorm();
    setupFfnBlock();
    hipk::preloadModules();  // no code-object load inside the first forwards
    load_.ms = timer.elapsedMs();
    load_.deviceBytes = deviceBytes_;
}

HipEngineImpl::~HipEngineImpl() {
    (void)hipSetDevice(dev_);
    for (auto &kv : graphs_) (void)hipGraphExecDestroy(kv.second);
    for (void *p : allocs_) (void)hipFree(p);
    for (void *p : hostAllocs_) (void)hipHostFree(p);
    if (hLogits_) (void)hipHostFree(hLogits_);
    for (auto &e : chainEv_)
        if (e) (void)hipEventDestroy(e);
    if (stream_) (void)hipStreamDestroy(stream_);
}

std::vector<unsigned long long> HipEngineImpl::traceAttnBlock(int token, int pos, int slot, int layer) {
    if (!blockOn_) return {};
    bucket_ = (int)(&bucketFor(pos) - buckets_.data());
    if (!buckets_[bucket_].block) return {};
    const hipk::AttnBlockPlan pl = hipk::attnBlockPlan(attnBlockArgs(layers_[0], 0, 0), fusedTp(false));
    const int g[3] = {pl.gq, pl.ga, pl.gw};
    const size_t words = 8 * (size_t)(g[0] + g[1] + g[2]);
    traceBuf_ = dalloc<unsigned long long>(words);
    DL_HIP(hipMemsetAsync(traceBuf_, 0, words * 8, stream_));
    traceLayer_ = layer;
    setInputs(1, &token, &pos, &slot);
    enqueueForward(1, GraphKind::LOGITS);
    syncAndCheckComm();
    inputsInFlight_ = false;
    std::vector<unsigned long long> out(3 + words);
    for (int i = 0; i < 3; i++) out[i] = (unsigned long long)g[i];
    DL_HIP(hipMemcpy(out.data() + 3, traceBuf_, words * 8, hipMemcpyDeviceToHost));
    traceLayer_ = -1;
    traceBuf_ = nullptr;  // (one small buffer per call, released with the engine)
    return out;
}

void HipEngineImpl::forward(int n, const int *tokens, const int *positions, const int *slots, float *logits) {
    Timer t;
    setInputs(n, tokens, positions, slots);
    runGraph(n, GraphKind::LOGITS);
    const bool root = rank() == 0;
    if (root && logits && (size_t)n * h_.vocabSize > hLogitsCap_) {  // pinned staging, grown on demand
        if (hLogits_) DL_HIP(hipHostFree(hLogits_));
        hLogitsCap_ = (size_t)n * h_.vocabSize;
        DL_HIP(hipHostMalloc(reinterpret_cast<void **>(&hLogits_), hLogitsCap_ * sizeof(float), hipHostMallocDefault));
    }
    if (root && logits) {
        const float *src = plan_.nRanks > 1 ? dLogitsFull_ : dLogits_;
        DL_HIP(hipMemcpyAsync(hLogits_, src, (size_t)n * h_.vocabSize * sizeof(float), hipMemcpyDeviceToHost, stream_));
    }
    syncAndCheckComm();
    inputsInFlight_ = false;
    if (root && logits) std::memcpy(logits, hLogits_, (size_t)n * h_.vocabSize * sizeof(float));
    stats_.computeMs = t.elapsedMs();
    setSyncStats(readSync(hSync_, false), stats_.computeMs);
}

void HipEngineImpl::forwardArgmax(int n, const int *tokens, const int *positions, const int *slots, int *out) {
    Timer t;
    setInputs(n, tokens, positions, slots);
    runGraph(n, GraphKind::ARGMAX);
    DL_HIP(hipMemcpyAsync(hIds_, dIds_, n * sizeof(int), hipMemcpyDeviceToHost, stream_));
    syncAndCheckComm();
    inputsInFlight_ = false;
    std::memcpy(out, hIds_, n * sizeof(int));
    stats_.computeMs = t.elapsedMs();
    setSyncStats(readSync(hSync_, false), stats_.computeMs);
}

void HipEngineImpl::forwardSample(int n, const int *tokens, const int *positions, const int *slots,
                                  const SampleSpec *specs, int *out) {
    Timer t;
    setInputs(n, tokens, positions, slots, specs);
    runGraph(n, GraphKind::SAMPLE);
    DL_HIP(hipMemcpyAsync(hIds_, dIds_, n * sizeof(int), hipMemcpyDeviceToHost, stream_));
    syncAndCheckComm();
    inputsInFlight_ = false;
    std::memcpy(out, hIds_, n * sizeof(int));
    stats_.computeMs = t.elapsedMs();
    setSyncStats(readSync(hSync_, false), stats_.computeMs);
}

// Pipelined serving: the forward and the D2H copy of its ids are enqueued; the host returns at
// once (inputs are staged in pinned memory: the previous forward was collected before).
void HipEngineImpl::launchIds(int n, const int *tokens, const int *positions, const int *slots,
                              const SampleSpec *specs) {
    DL_CHECK(pendingN_ == 0, "launchIds: the previous forward was not collected");
    Timer t;
    setInputs(n, tokens, positions, slots, specs);
    runGraph(n, specs ? GraphKind::SAMPLE : GraphKind::ARGMAX);
    DL_HIP(hipMemcpyAsync(hIds_, dIds_, n * sizeof(int), hipMemcpyDeviceToHost, stream_));
    pendingN_ = n;
    stats_.computeMs = t.elapsedMs();  // host enqueue time; the sync is read when collected
}

void HipEngineImpl::collectIds(int *out) {
    DL_CHECK(pendingN_ > 0, "collectIds: nothing launched");
    const int n = pendingN_;
    pendingN_ = 0;
    syncAndCheckComm();
    inputsInFlight_ = false;
    std::memcpy(out, hIds_, n * sizeof(int));
    setSyncStats(readSync(hSync_, false), -1);
}

// Chained decode for the CLI: the CHAIN graph (forward -> argmax -> tokens := ids, pos += 1 on
// the device) per step, each followed by the D2H copy of its id into a ring slot and an event. The
// host keeps a step in flight while it decodes and prints the previous one (the reference's loop
// waits for every token before starting the next: dllama.cpp:74-96). Graph / bucket choice
// follow the step's position as in setInputs; error words are checked at every collect.
void HipEngineImpl::chainLaunch(int token, int pos, int slot) {
    DL_CHECK(pendingN_ == 0, "chainLaunch: a launchIds forward was not collected");
    DL_CHECK(chainHead_ - chainTail_ < kChainDepth, "chainLaunch: too many steps in flight");
    DL_CHECK(pos >= 0 && (u32)pos < h_.seqLen, "position out of range");
    if (!hChain_) {
        hChain_ = halloc<int>(kChainDepth);
        for (auto &e : chainEv_) DL_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (token >= 0) {
        DL_CHECK(chainHead_ == chainTail_, "chainLaunch: a chain restarted with steps in flight");
        setInputs(1, &token, &pos, &slot, nullptr, 0);
        chainSlot_ = slot;
    } else {  // dTok_ / dPos_ hold the previous step's id and position + 1 (written on the device)
        DL_CHECK(chainHead_ > 0, "chainLaunch: no chain started");
        mapPages(1, &pos, &chainSlot_, 0);
        attnLong_ = !invariant_ && pos >= kAttnMfmaMinPos;
        bucket_ = (int)(&bucketFor(pos) - buckets_.data());
    }
    const int k = (int)(chainHead_ % kChainDepth);
    runGraph(1, GraphKind::CHAIN, hSyncAt(1 + k));  // this step's own copy (steps in flight overlap)
    DL_HIP(hipMemcpyAsync(hChain_ + k, dIds_, sizeof(int), hipMemcpyDeviceToHost, stream_));
    enqueueErrorCopies();
    DL_HIP(hipEventRecord(chainEv_[k], stream_));
    chainHead_++;
}

int HipEngineImpl::chainCollect() {
    DL_CHECK(chainHead_ > chainTail_, "chainCollect: no step in flight");
    const int k = (int)(chainTail_ % kChainDepth);
    DL_HIP(hipEventSynchronize(chainEv_[k]));
    chainTail_++;
    if (chainTail_ == chainHead_) inputsInFlight_ = false;
    checkErrorWords();
    setSyncStats(readSync(hSyncAt(1 + k), false), -1);
    return hChain_[k];
}

double HipEngineImpl::decodeGreedyBatch(int steps, int nSeq, const int *tokens, const int *pos, const int *slots,
                                        int *outTokens) {
    DL_CHECK(nSeq >= 1 && nSeq <= decodeRows_, "nSeq exceeds the engine's decode rows (max_decode)");
    for (int b = 0; b < nSeq; b++) DL_CHECK((u32)(pos[b] + steps) <= h_.seqLen, "decode exceeds seqLen");
    if (!tpTested_) tpFusedSelfTest();
    setInputs(nSeq, tokens, pos, slots, nullptr, steps - 1);
    // the history window the chain writes: rows 0..nSeq, positions [p0, p1) (not the whole
    // maxBatch x seqLen buffer: 16 MB at a 131072-position capacity, set and copied every call)
    int p0 = pos[0], p1 = pos[0] + steps;
    for (int b = 1; b < nSeq; b++) {
        p0 = std::min(p0, pos[b]);
        p1 = std::max(p1, pos[b] + steps);
    }
    const size_t pitch = sizeof(int) * (size_t)h_.seqLen, width = sizeof(int) * (size_t)(p1 - p0);
    DL_HIP(hipMemset2DAsync(dHist_ + p0, pitch, 0xff, width, nSeq, stream_));
    hipEvent_t e0, e1;
    DL_HIP(hipEventCreate(&e0));
    DL_HIP(hipEventCreate(&e1));
    // measured sync of every step: the slots and running totals start at zero, each step's
    // embedding folds the previous step's slots into the totals, one copy after the last step
    if (plan_.nRanks > 1)
        DL_HIP(hipMemsetAsync(dSync_, 0, hipk::syncFoldWords(syncSlots()) * sizeof(unsigned), stream_));
    // the chained graph: forward -> argmax -> (tokens := ids, pos += 1)
    DL_HIP(hipEventRecord(e0, stream_));
    for (int s = 0; s < steps; s++) runGraph(nSeq, GraphKind::CHAIN, s + 1 == steps ? hSync_ : nullptr);
    accountForward(nSeq, GraphKind::CHAIN, steps);
    DL_HIP(hipEventRecord(e1, stream_));
    DL_HIP(hipEventSynchronize(e1));
    float ms = 0;
    DL_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    syncAndCheckComm();
    inputsInFlight_ = false;
    setSyncStats(readSync(hSync_, true), ms);  // every step's exchanges, measured
    if (outTokens) {
        const int w = p1 - p0;
        std::vector<int> hist((size_t)nSeq * w);
        DL_HIP(hipMemcpy2D(hist.data(), width, dHist_ + p0, pitch, width, nSeq, hipMemcpyDeviceToHost));
        for (int b = 0; b < nSeq; b++)
            for (int s = 0; s < steps; s++) outTokens[b * steps + s] = hist[(size_t)b * w + pos[b] - p0 + s];
    }
    return ms;
}

void HipEngineImpl::profileForward(int n, const int *tokens, const int *positions, const int *slots) {
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

// Wait for the stream, then turn a tensor-parallel transport failure into an exception (the
// worker loop re-serves, the root reports it) instead of returning results computed from a
// peer's stale data: the xGMI collectives flag a peer that did not arrive within 2 s, RCCL
// reports asynchronous errors (the communicator is then released without waiting).
void HipEngineImpl::syncAndCheckComm() {
    enqueueErrorCopies();
    DL_HIP(hipStreamSynchronize(stream_));
    checkErrorWords();
}

// The device error words (transport timeout, in-launch hand-off timeout) to pinned host words, in
// stream order behind the work they judge.
void HipEngineImpl::enqueueErrorCopies() {
    const int *flag = comm_ ? comm_->deviceErrorFlag() : nullptr;
    if (flag) DL_HIP(hipMemcpyAsync(hErr_, flag, sizeof(int), hipMemcpyDeviceToHost, stream_));
    if (blockOn_ || ffnOn_) DL_HIP(hipMemcpyAsync(hErr_ + 1, dBlockErr_, sizeof(int), hipMemcpyDeviceToHost, stream_));
}

void HipEngineImpl::checkErrorWords() {
    const int *flag = comm_ ? comm_->deviceErrorFlag() : nullptr;
    const bool inLaunch = blockOn_ || ffnOn_;  // kernels with in-launch hand-offs
    if (inLaunch && hErr_[1] != 0) {
        const int code = hErr_[1];
        hErr_[1] = 0;
        resetAttnBlockState();
        throw Error("in-launch hand-off wait timed out (code " + std::to_string(code) +
                    ": attention block 2 qkv->attention, 3 attention->wo, 4 qkv phase; FFN block 7 w13->w2; not all workgroups "
                    "resident?)");
    }
    if (flag && *hErr_ != 0)
        throw Error(std::string("tensor-parallel collective timed out: a peer rank did not arrive in time (2 s; 20 s for ranks sharing a GPU; ") +
                    (*hErr_ == 1 ? "all-reduce / all-gather" : *hErr_ == 2 ? "low-latency all-reduce" : "fused exchange") +
                    "; worker lost?)");
    if (comm_) {
        const std::string e = comm_->asyncError();
        if (!e.empty()) {
            comm_->shutdownNow();
            throw Error("tensor-parallel transport failed: " + e);
        }
    }
}

// Tensor-parallel data-plane bytes of one forward of n rows on this rank, in the reference's
// accounting (nn-network.cpp:493-508 counts socket payload): every residual update
// sends this rank's partial [n][dim] to each peer and receives each peer's (Q80 blocks of 34 B per
// 32 values with --sync-type q80, the reference's ZQ format, else f32), two per layer; greedy rows
// then trade one (value, index) winner per row (in the fused exchange or one all-gather), host
// logits and sampled rows gather the vocab slices to the root. The transport's own framing (the 8-byte
// {value, epoch} words of the fused exchange) is not payload and not counted.
void HipEngineImpl::accountForward(int n, GraphKind kind, int times) {
    stats_.sentBytes = stats_.recvBytes = 0;
    const ShardPlan &p = plan_;
    if (p.nRanks <= 1) return;
    const u64 peers = p.nRanks - 1;
    const u64 row = syncQ80_ ? (u64)h_.dim / 32 * 34 : (u64)h_.dim * 4;
    u64 sent = 2ull * h_.nLayers * peers * (u64)n * row, recv = sent;
    const u64 slice = (u64)n * p.vocab0 * 4;
    if (kind == GraphKind::ARGMAX || kind == GraphKind::CHAIN) {  // (value, index) winners only
        sent += peers * (u64)n * 8;
        recv += peers * (u64)n * 8;
    } else if (rank() == 0) {  // LOGITS / SAMPLE: the vocab slices go to the root
        recv += peers * slice;
    } else {
        sent += slice;
    }
    stats_.sentBytes = sent * (u64)times;
    stats_.recvBytes = recv * (u64)times;
}

// Measured sync of a forward (a host copy of its slots, enqueued by runGraph), summed over the
// forward's exchanges and their launches: wait = per exchange launch the longest time a wave of the
// fused exchange waited for peers' words (tpWaitReport); span = the longest exchange tail of a
// workgroup (DL_SYNC_MEASURE=2); a separate collective counts its stamped span (launch gaps
// included) in both. totals: plus the device running totals of every earlier folded forward (a
// whole decode chain). The reference times its sync steps per forward (nn-executor.cpp:150-155,
// printed per token dllama.cpp:57-64).
HipEngineImpl::SyncRead HipEngineImpl::readSync(const unsigned *buf, bool totals) const {
    SyncRead r;
    if (plan_.nRanks <= 1 || !buf) return r;
    const int S = syncSlots();
    const unsigned long long *st = reinterpret_cast<const unsigned long long *>(buf + 2 * S);
    const unsigned long long *acc = reinterpret_cast<const unsigned long long *>(buf + 6 * S);
    double wait = 0, span = 0, stamp = 0;
    for (int i = 0; i < S; i++) {
        wait += buf[i];
        span += buf[S + i];
        if (st[2 * i] && st[2 * i + 1] > st[2 * i]) stamp += (double)(st[2 * i + 1] - st[2 * i]);
    }
    if (totals) {
        wait += (double)acc[0];
        span += (double)acc[1];
        stamp += (double)acc[2];
    }
    r.waitMs = (wait + stamp) * 1e-5;  // s_memrealtime: 100 MHz
    if (syncLevel_ >= 2 || stamp > 0) r.spanMs = (span + stamp) * 1e-5;
    return r;
}

// capMs >= 0: the forward's wall time bounds both (a wait cannot exceed the forward it is part of)
void HipEngineImpl::setSyncStats(const SyncRead &r, double capMs) {
    stats_.syncMs = capMs >= 0 ? std::min(r.waitMs, capMs) : r.waitMs;
    stats_.xchgMs = r.spanMs < 0 ? -1 : (capMs >= 0 ? std::min(r.spanMs, capMs) : r.spanMs);
}

void HipEngineImpl::launchStampAt(unsigned long long *p) { hipk::launchStamp(p, stream_); }

// The first forward of a tensor-parallel engine with the fused exchange runs its self-test on the
// real devices (every rank reaches this point in the same forward: the ranks run forwards in
// lockstep). Pass: rank-order sums of known element-dependent values through both exchange
// regions, no peer timed out, and every rank's verdict exchanged over region 0 sums to the world
// size. Anything else switches the fused exchange off on every rank (the verdict sum is the same
// everywhere), which then runs the separate collectives of the same comm (xGMI all-reduce, itself
// self-tested at start-up, or RCCL). DL_TP_FUSED=fail makes rank 1 report a failure (tests).
void HipEngineImpl::tpFusedSelfTest() {
    tpTested_ = true;
    if (!tpFused_ || comm_->computeOnly()) return;
    const int W = plan_.nRanks, me = rank();
    const char *e = std::getenv("DL_TP_FUSED");
    bool ok = !(e && std::strcmp(e, "fail") == 0 && me == 1);
    const int *errFlag = comm_->deviceErrorFlag();
    auto timedOut = [&]() {
        if (!errFlag) return false;
        int v = 0;
        DL_HIP(hipMemcpy(&v, errFlag, sizeof(int), hipMemcpyDeviceToHost));
        return v != 0;
    };
    // the first pass is also the rendezvous: ranks reach their first forward seconds apart (model
    // load / synthetic init time differs per rank), so the self-test waits up to 60 s for a peer
    // instead of the data plane's 2 s
    auto patient = [](hipk::TpXchg x) {
        x.timeoutTicks = 6000LL * 1000 * 1000;
        return x;
    };
    std::vector<float> got;
    std::string why = ok ? "" : "DL_TP_FUSED=fail";
    for (int r = 0; r < 2; r++) {
        const hipk::TpXchg &x = r == 0 ? tpVec_ : tpArg_;
        // dY_ holds maxBatch x dim floats: a small engine tests fewer elements
        const int n = (int)std::min<long long>(std::min<long long>(4096, x.stride), (long long)cfg_.maxBatch * h_.dim);
        hipk::launchTpSelfTest(patient(x), dY_, n, (float)(me + 1), stream_);
        DL_HIP(hipStreamSynchronize(stream_));
        got.resize(n);
        DL_HIP(hipMemcpy(got.data(), dY_, n * sizeof(float), hipMemcpyDeviceToHost));
        for (int el = 0; el < n && ok; el++) {
            const float want = (float)(W * (W + 1) / 2) + (float)(W * (el & 1023));
            if (got[el] != want) {
                ok = false;
                why = "region " + std::to_string(r) + " element " + std::to_string(el) + ": got " +
                      std::to_string(got[el]) + ", want " + std::to_string(want);
            }
        }
    }
    if (timedOut()) {
        ok = false;
        why += " (a peer wait timed out)";
    }
    comm_->resetError();
    hipk::launchTpSelfTest(patient(tpVec_), dY_, 1, ok ? 1.f : 0.f, stream_);  // the verdicts (+ element 0's 0)
    DL_HIP(hipStreamSynchronize(stream_));
    float all = 0.f;
    DL_HIP(hipMemcpy(&all, dY_, sizeof(float), hipMemcpyDeviceToHost));
    bool allOk = !timedOut() && all == (float)W;
    comm_->resetError();
    // The decision must be the same on every rank: a rank whose verdict wait timed out (a peer
    // more than 60 s late) would switch the fused exchange off while the late peer, seeing every
    // verdict, keeps it, and their next forward would wait on different data planes. So the ranks
    // agree through the separate collectives (self-tested at start-up) on the sum of verdicts.
    float agree = allOk ? 1.f : 0.f;
    DL_HIP(hipMemcpy(dY_, &agree, sizeof(float), hipMemcpyHostToDevice));
    comm_->allReduceSum(dY_, 1, stream_);
    DL_HIP(hipStreamSynchronize(stream_));
    DL_HIP(hipMemcpy(&agree, dY_, sizeof(float), hipMemcpyDeviceToHost));
    if (timedOut()) throw Error("tensor-parallel self-test: a peer never reached the verdict agreement");
    if (agree != (float)W && allOk) why = "a peer's verdict";
    allOk = agree == (float)W;
    if (allOk) return;
    std::fprintf(stderr, "⚠️  rank %d: fused tensor-parallel exchange self-test failed (%s); using the separate "
                 "%s collectives\n", me, ok ? "on a peer" : ("here: " + why).c_str(), comm_->name().c_str());
    tpFused_ = false;
    blockOn_ = false;  // the attention block's wo role was chosen for the fused exchange: decide again
    for (CtxBucket &b : buckets_) b.block = false;
    setupAttnBlock();
    setupWoAttn();
    setupPrenorm();
    setupFfnBlock();
}

void HipEngineImpl::runGraph(int n, GraphKind kind, unsigned *syncDst) {
    if (!tpTested_) tpFusedSelfTest();
    accountForward(n, kind, 1);
    auto copySync = [&]() {  // the forward's measured-sync slots to the host (read after the sync)
        if (plan_.nRanks > 1 && syncDst)
            DL_HIP(hipMemcpyAsync(syncDst, dSync_, hipk::syncFoldWords(syncSlots()) * sizeof(unsigned),
                                  hipMemcpyDeviceToHost, stream_));
    };
    if (!cfg_.useGraphs || graphsBroken_) {
        enqueueForward(n, kind);
        copySync();
        return;
    }
    const int key = ((((n * 4 + (int)kind) * 2 + (prefillOk_ ? 1 : 0)) * 2 + (attnLong_ ? 1 : 0)) << 4) + bucket_;
    auto it = graphs_.find(key);
    if (it == graphs_.end()) {
        // capture on the second use of a shape: a one-off row count (the tail chunk of a prompt,
        // a serving batch seen once) runs eagerly instead of paying capture + instantiation
        // (several ms for ~170 kernel nodes) for a graph that would never be replayed
        if (graphSeen_.insert(key).second) {
            enqueueForward(n, kind);
            copySync();
            return;
        }
        hipGraphExec_t ge = captureForward(n, kind);
        if (!ge) {
            // e.g. a collective library build that cannot be stream-captured: stay correct, run eagerly
            graphsBroken_ = true;
            std::fprintf(stderr, "⚠️  hipGraph capture failed; falling back to eager launches\n");
            enqueueForward(n, kind);
            copySync();
            return;
        }
        it = graphs_.emplace(key, ge).first;
    }
    DL_HIP(hipGraphLaunch(it->second, stream_));
    copySync();
}

hipGraphExec_t HipEngineImpl::captureForward(int n, GraphKind kind) {
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

}  // namespace engine_detail

std::unique_ptr<HipEngine> makeHipEngine(const EngineConfig &cfg, DeviceComm *comm) {
    return std::unique_ptr<HipEngine>(new engine_detail::HipEngineImpl(cfg, comm));
}

}  // namespace dl
