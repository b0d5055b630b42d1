// The per-forward kernel schedule of the HIP engine (engine_impl.h): inputs and context buckets,
// GEMV / batched GEMM / attention / fused attention block launches, tensor-parallel collectives.
#include "engine_impl.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace dl {
namespace engine_detail {

// Context buckets: decode capacity seqLen is covered by buckets of 256 x 4^k positions (and seqLen
// itself); a forward whose rows reach at most position p runs the launches of the smallest bucket
// holding p + 1 positions. Within a bucket the sequence split of every row is the one the full
// capacity would give (attnSplit caps ceil(len / 256) chunks at the bucket's split grid, which is
// >= that count), so a bucketed forward is bitwise the forward of an engine sized to the bucket.
void HipEngineImpl::setupBuckets() {
    buckets_.clear();
    for (int len = 256; len < (int)h_.seqLen; len *= 4) {
        CtxBucket b;
        b.maxLen = len;
        buckets_.push_back(b);
    }
    CtxBucket last;
    last.maxLen = (int)h_.seqLen;
    buckets_.push_back(last);
    DL_CHECK(buckets_.size() <= 16, "too many context buckets");
    for (CtxBucket &b : buckets_) {
        b.splitGrid = hipk::attnSplitGrid(b.maxLen, true);
        b.splitGridBat = hipk::attnSplitGrid(b.maxLen, false);
        b.chunkMax = hipk::attnChunkMax(b.maxLen, b.splitGridBat);
    }
    bucket_ = (int)buckets_.size() - 1;
}

const CtxBucket &HipEngineImpl::bucketFor(int maxPos) const {
    for (const CtxBucket &b : buckets_)
        if (maxPos < b.maxLen) return b;
    return buckets_.back();
}

void HipEngineImpl::setInputs(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs,
                              int ahead) {
    DL_CHECK(n >= 1 && (u32)n <= cfg_.maxBatch, "batch size out of range");
    DL_CHECK(chainHead_ == chainTail_, "a chained decode step is still in flight");
    for (int b = 0; b < n; b++) {
        DL_CHECK(tokens[b] >= 0 && (u32)tokens[b] < h_.vocabSize, "token out of range");
        DL_CHECK(positions[b] >= 0 && (u32)positions[b] < h_.seqLen, "position out of range");
        DL_CHECK(slots[b] >= 0 && (u32)slots[b] < cfg_.nSlots, "slot out of range");
    }
    mapPages(n, positions, slots, ahead);
    // decode attention kernel for this forward (part of the graph key): the MFMA kernel once a
    // row's context reaches kAttnMfmaMinPos keys (measured faster from ~1.5K keys, slower on
    // short contexts: profiles/r3_prefill_attention.md) or the forward has kAttnMfmaMinRows rows
    // (batch 16 / 64 at 150 keys: 8.2 / 17.2 us vs 9.5 / 22.8 on the VALU kernel, which stays
    // ahead up to batch 8: profiles/r5_batched_attention.md), else the VALU kernel
    int maxPos = 0;
    for (int b = 0; b < n; b++) maxPos = std::max(maxPos, positions[b] + ahead);
    attnLong_ = !invariant_ && (maxPos >= kAttnMfmaMinPos || n >= kAttnMfmaMinRows);
    bucket_ = (int)(&bucketFor(maxPos) - buckets_.data());
    const u32 MB = cfg_.maxBatch;
    // keep the pinned staging buffer stable while a previous copy may still read it (every
    // public entry point ends with a stream sync, so this only waits after an async path)
    if (inputsInFlight_) DL_HIP(hipStreamSynchronize(stream_));
    std::memcpy(hIn_, tokens, n * sizeof(int));
    std::memcpy(hIn_ + MB, positions, n * sizeof(int));
    std::memcpy(hIn_ + 2 * MB, slots, n * sizeof(int));
    size_t words = 2 * (size_t)MB + n;
    // prefill attention on MFMA: every block of rows it assigns to one workgroup is one slot
    prefillOk_ = !invariant_ && hipk::attnPrefillSupported(plan_.headSize, plan_.kvMul, kvBf16_);
    const int rpb = prefillOk_ ? hipk::attnPrefillRowsPerBlock(plan_.kvMul) : 1;
    for (int b = 0; prefillOk_ && b < n; b++) prefillOk_ = slots[b] == slots[b - b % rpb];
    // f32 caches: the f32 MFMA prefill kernel from 128 keys on; below, the per-row decode attention
    // is faster (a 32-row chunk at positions 0-63: eval 0.0957 vs 0.0993 ms/token; crossover ~135
    // keys from the 4k-prompt slopes, profiles/r6_decode.md). DL_PREFILL_F32_MIN overrides.
    if (prefillOk_ && !kvBf16_) {
        static const int f32Min = [] {
            const char *e = std::getenv("DL_PREFILL_F32_MIN");
            return e ? std::atoi(e) : 128;
        }();
        int mx = 0;
        for (int b = 0; b < n; b++) mx = std::max(mx, positions[b] + 1);
        prefillOk_ = mx >= f32Min;
    }
    if (specs) {
        static_assert(sizeof(SampleSpec) == 4 * sizeof(float), "spec layout");
        std::memcpy(hIn_ + 3 * MB, specs, n * sizeof(SampleSpec));
        words = 3 * (size_t)MB + 4 * (size_t)n;
    }
    // one copy of the row arrays (the unused tail of each is never read)
    DL_HIP(hipMemcpyAsync(dTok_, hIn_, words * sizeof(int), hipMemcpyHostToDevice, stream_));
    inputsInFlight_ = true;
}

int HipEngineImpl::batchChunk(const DevMat &m, int pro, int epi) const {
    // largest batch chunk (1/2/4) whose LDS footprint stays <= 64 KiB for this input width (8 rows
    // measured 2x slower than the MFMA GEMM: the GEMV's per-row int8 dots are VALU-bound there)
    int bc = 4;
    while (bc > 1) {
        const int rp = q40_ ? 256 / m.lanes * hipk::gemvRowGroup(bc, true) : hipk::gemvRowsPerPass(m.n, m.rows, bc, false);
        const int rpw = rp * passesFor(m, epi, bc);
        if (hipk::gemvLdsBytes(m.n, bc, q40_, rpw, pro) <= 64 * 1024) break;  // B > 1 only; B = 1 may use up to 160 KB
        bc >>= 1;
    }
    return bc;
}

// Arguments of one GEMV launch over rows [c0, c0 + bc) of the batch (see gemv()).
hipk::GemvArgs HipEngineImpl::gemvArgs(const DevMat &m, int c0, int bc, int epi, const float *in, int ldIn, const float *add,
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
    if (tp) {
        a.tp = tpVec_;
        a.tp.ticks = syncTicks();
        a.tp.span = syncSpan();
    }
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
void HipEngineImpl::gemv(const DevMat &m, int n, int pro, int epi, const float *in, int ldIn, const float *add, float *xNext,
          const float *normW, float *out, int ldOut, const DevLayer *L, const int8_t *aq,
                         const float2 *as, int8_t *oq, float2 *os, bool tp) {
    if (tp) epi = hipk::EPI_STORE_TP;
    const int bcMax = batchChunk(m, pro, epi);
    xChunk_ = 0;  // each launch's exchange waits in a measured-sync slot of its own
    for (int c0 = 0; c0 < n; xChunk_++) {
        int bc = n - c0;
        if (bc > bcMax) bc = bcMax;
        while (bc & (bc - 1)) bc &= bc - 1;  // 1, 2 or 4 rows per launch
        const hipk::GemvArgs a = gemvArgs(m, c0, bc, epi, in, ldIn, add, xNext, normW, out, ldOut, L, aq, as, oq, os, tp);
        hipk::launchGemv(a, bc, pro, epi, q40_, stream_);
        c0 += bc;
    }
    xChunk_ = 0;
}

// Decode attention of this layer (rows 0..n of the forward).
hipk::AttnArgs HipEngineImpl::attnArgs(const DevLayer &L, bool bat) const {
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
    a.splitGrid = bat ? buckets_[bucket_].splitGridBat : buckets_[bucket_].splitGrid;
    a.shortLen = bat ? 0 : hipk::kAttnShortLen;
    a.chunkMax = buckets_[bucket_].chunkMax;
    a.chunkMin = hipk::attnChunkMin();
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
hipk::AttnBlockArgs HipEngineImpl::attnBlockArgs(const DevLayer &L, u32 l, int cur) const {
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
    b.qkv.passes *= blockPassMul_;  // same-GPU rehearsals: longer workgroups (setupAttnBlock)
    b.wo.passes *= blockPassMul_;
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

// Decide once per context bucket whether decode rows run the fused attention block: Q40 weights, a
// compiled instance for this shape, <= 64 KV groups, and the whole grid (whose attention role grows
// with the bucket's sequence splits) co-resident, shared with the other ranks on this GPU.
// DL_ATTN_BLOCK=0 keeps the three separate launches.
void HipEngineImpl::setupAttnBlock() {
    const char *e = std::getenv("DL_ATTN_BLOCK");
    if ((e && *e == '0') || !q40_ || plan_.nKvHeads0 > kMaxKvGroups) return;
    // one KV group per rank (8 KV heads at TP8): the attention role is a handful of workgroups
    // the whole wo role waits on - measured 2x the three launches (8B TP8 rank: 38 vs ~18 us per
    // layer, profiles/r5_tp_rank.md); DL_ATTN_BLOCK=1 forces it
    if (plan_.nKvHeads0 < 2 && !(e && *e == '1')) return;
    const int share = comm_ ? std::max(1, comm_->ranksOnDevice()) : 1;
    const int keep = bucket_;
    // qkv / wo passes per workgroup: the GEMVs' own grids. A grid beyond one round of co-resident
    // workgroups keeps the three launches: longer qkv / wo workgroups measured slower on a GPU of
    // its own (70B 8.10 -> 8.26, 405B 40.4 -> 43.3 ms/token) and in same-GPU rehearsals (ranks
    // sharing one GPU's resident slots: 8B TP2 2.91 vs 1.63 ms/token with the three launches), so
    // a rehearsal makes the production choice. Only a forced block (DL_ATTN_BLOCK=1, tests of the
    // block's exchange on one GPU) doubles the passes until the shared slots hold it.
    const bool forced = e && *e == '1';
    bucket_ = 0;
    for (blockPassMul_ = 1; forced && share > 1 && blockPassMul_ < 8; blockPassMul_ *= 2) {
        const hipk::AttnBlockArgs b = attnBlockArgs(layers_[0], 0, 0);
        if (!hipk::attnBlockPlan(b, fusedTp(false)).fn) break;
        const hipk::GemvResidency r = hipk::attnBlockResidency(b, fusedTp(false));
        if (r.maxResident > 0 && r.grid <= r.maxResident / share) break;
    }
    int lastOn = -1;
    hipk::GemvResidency off;
    for (size_t i = 0; i < buckets_.size(); i++) {
        bucket_ = (int)i;
        const hipk::AttnBlockArgs b = attnBlockArgs(layers_[0], 0, 0);
        if (!hipk::attnBlockPlan(b, fusedTp(false)).fn) break;
        const hipk::GemvResidency r = hipk::attnBlockResidency(b, fusedTp(false));
        if (r.maxResident <= 0 || r.grid > r.maxResident / share) {
            off = r;
            break;
        }
        buckets_[i].block = true;
        lastOn = (int)i;
        if (!blockOn_) {
            std::vector<unsigned> expect(kMaxKvGroups, 0);
            hipk::attnBlockExpect(b.qkv, (int)plan_.nKvHeads0, expect.data());
            DL_HIP(hipMemcpy(dBlockExpect_, expect.data(), expect.size() * sizeof(unsigned), hipMemcpyHostToDevice));
            blockOn_ = true;
        }
    }
    bucket_ = keep;
    if (lastOn < 0 && off.grid > 0)
        std::fprintf(stderr, "ℹ️  fused attention block off: grid %d > %d co-resident workgroups per rank\n", off.grid,
                     off.maxResident / share);
}

// Pre-normalized hand-off between the single-row GEMVs of a tensor-parallel rank (kernels.h
// PRO_PRENORM / EPI_RESQ_TP): the wo / w2 exchange tails, which already hold the rank-summed rows,
// also apply the residual update and the next RMS norm's weights and quantize x * normW to Q80
// blocks, plus one sum of squares per workgroup; the consumers (qkv, w13, logits) copy those blocks
// and fold in 1 / rms instead of re-reading x and the delta and reducing 4096 values in every
// workgroup. Measured per launch (scripts/trace_gemv.py, norm vs copy prologue): qkv 5.71 vs 4.69
// us at TP1 shapes, and at a TP8 rank's shards qkv 4.35 vs 3.13, w13 5.18 vs 3.96.
// Needs producers whose workgroups own whole 32-row blocks (the Q80 exchange's tpPasses) and at
// most kMaxSsp of them, the fused exchange (separate collectives keep the norm prologue) and
// no attention block in the forward (the block's roles keep theirs). DL_PRENORM=0 disables it.
void HipEngineImpl::setupPrenorm() {
    prenormOn_ = false;
    const char *e = std::getenv("DL_PRENORM");
    if ((e && *e == '0') || !q40_ || !fusedTp(false) || h_.dim % 32 || h_.dim > 16384) return;
    const int share = comm_ ? std::max(1, comm_->ranksOnDevice()) : 1;
    for (int w = 0; w < 2; w++) {
        const DevMat &m = w == 0 ? layers_[0].wo : layers_[0].w2;
        const int pro = w == 1 && !hQ80_ ? hipk::PRO_RESNORM : hipk::PRO_GLOBAL;
        const hipk::GemvArgs a = gemvArgs(m, 0, 1, hipk::EPI_RESQ_TP, nullptr, m.n, nullptr, nullptr, nullptr, dY_,
                                          h_.dim, nullptr, nullptr, nullptr, nullptr, nullptr, true);
        const int R = (256 / a.lanes) * 2 * a.passes, grid = (a.rows + R - 1) / R;
        if (R % 32 || grid > kMaxSsp) return;
        const hipk::GemvResidency r = hipk::gemvResidency(a, 1, pro, hipk::EPI_RESQ_TP, true);
        if (r.maxResident <= 0 || r.grid > r.maxResident / share) return;
    }
    prenormOn_ = true;
}

hipk::FfnBlockArgs HipEngineImpl::ffnBlockArgs(const hipk::GemvArgs &w13, const hipk::GemvArgs &w2, u32 l) {
    hipk::FfnBlockArgs f;
    f.w13 = w13;
    f.w2 = w2;
    f.hQ80 = hQ80_ ? 1 : 0;
    f.layer = (int)l;
    f.nLayers = (int)h_.nLayers;
    f.epoch = dEpoch_ + 1;
    f.cnt = dBlockCnt_ + kFfnCntOff;
    f.flag = dBlockCnt_ + kFfnCntOff + 64;
    f.error = dBlockErr_;
    return f;
}

// Fused FFN block (kernels.h FfnBlockArgs) for the pre-normalized single rows of a TP rank: a
// compiled (w13 lanes, w2 lanes) instance and the whole w13 + w2 grid co-resident, shared with the
// other ranks on this GPU. DL_FFN_BLOCK=0 keeps the two launches.
void HipEngineImpl::setupFfnBlock() {
    ffnOn_ = false;
    const char *e = std::getenv("DL_FFN_BLOCK");
    if (!prenormOn_ || !(e && *e == '1')) return;
    const DevLayer &L = layers_[0];
    const int epi = hQ80_ ? hipk::EPI_ACT_Q80 : hipk::EPI_ACT;
    const hipk::GemvArgs a13 = gemvArgs(L.w13, 0, 1, epi, nullptr, h_.dim, nullptr, nullptr, nullptr, dH_,
                                        plan_.hidden0, nullptr, nullptr, nullptr, dHQ_, dHS_, false);
    const hipk::GemvArgs a2 = gemvArgs(L.w2, 0, 1, hipk::EPI_RESQ_TP, hQ80_ ? nullptr : dH_, plan_.hidden0, nullptr,
                                       nullptr, nullptr, dY_, h_.dim, nullptr, hQ80_ ? dHQ_ : nullptr,
                                       hQ80_ ? dHS_ : nullptr, nullptr, nullptr, true);
    const hipk::FfnBlockArgs f = ffnBlockArgs(a13, a2, 0);
    if (!hipk::ffnBlockPlan(f).fn) return;
    const int share = comm_ ? std::max(1, comm_->ranksOnDevice()) : 1;
    const hipk::GemvResidency r = hipk::ffnBlockResidency(f);
    if (r.maxResident <= 0 || r.grid > r.maxResident / share) {
        std::fprintf(stderr, "ℹ️  fused FFN block off: grid %d > %d co-resident workgroups per rank\n", r.grid,
                     r.maxResident / share);
        return;
    }
    ffnOn_ = true;
}

// The layers + logits of one decode row with the pre-normalized hand-offs (setupPrenorm). The
// residual lives in dX_[cur]; its Q80 image for the next consumer in dXQ_ / dXS_ [cur] with sspN
// partial sums in dSSP_[cur]; each producer writes the other parity and flips cur.
void HipEngineImpl::enqueuePrenormLayers(GraphKind kind, bool argTail) {
    const ShardPlan &p = plan_;
    const int dim = h_.dim;
    const bool hQ80 = hQ80_;
    // layer 0's qkv normalizes the embedding's row itself (norm prologue): the one-workgroup
    // embedding kernel measured 12.8 vs 4.9 us with the pre-normalized output (PrenormOut)
    int cur = 0, sspN[2] = {0, 0};
    auto consumer = [&](hipk::GemvArgs &a) {
        a.aq = dXQ_[cur];
        a.as = dXS_[cur];
        a.sspIn = dSSP_[cur];
        a.nSsp = sspN[cur];
    };
    auto producer = [&](hipk::GemvArgs &a, const float *normW) {
        a.rq.resIn = dX_[cur];
        a.rq.resOut = dX_[cur ^ 1];
        a.rq.resW = normW;
        a.rq.xq = dXQ_[cur ^ 1];
        a.rq.xs = dXS_[cur ^ 1];
        a.rq.ssp = dSSP_[cur ^ 1];
        const int R = (256 / a.lanes) * 2 * a.passes;
        sspN[cur ^ 1] = (a.rows + R - 1) / R;
    };
    for (u32 l = 0; l < h_.nLayers; l++) {
        DevLayer &L = layers_[l];
        xSlot_ = 2 * (int)l;
        xChunk_ = 0;
        if (l == 0) {
            ProfScope ps(this, "gemv_qkv");
            gemv(L.qkv, 1, hipk::PRO_RESNORM, hipk::EPI_QKV, dX_[0], dim, nullptr, nullptr, L.rmsAtt, dQ_, p.q0, &L);
        } else {
            ProfScope ps(this, "gemv_qkv");
            hipk::GemvArgs a = gemvArgs(L.qkv, 0, 1, hipk::EPI_QKV, nullptr, dim, nullptr, nullptr, nullptr, dQ_, p.q0, &L,
                                        nullptr, nullptr, nullptr, nullptr, false);
            consumer(a);
            hipk::launchGemv(a, 1, hipk::PRO_PRENORM, hipk::EPI_QKV, true, stream_);
        }
        {
            ProfScope ps(this, "attention");
            hipk::launchAttention(attnArgs(L, false), 1, stream_);
        }
        {
            ProfScope ps(this, "gemv_wo");
            hipk::GemvArgs a = gemvArgs(L.wo, 0, 1, hipk::EPI_RESQ_TP, nullptr, p.q0, nullptr, nullptr, nullptr, dY_, dim,
                                        nullptr, dAttQ_, dAttS_, nullptr, nullptr, true);
            producer(a, L.rmsFfn);
            hipk::launchGemv(a, 1, hipk::PRO_GLOBAL, hipk::EPI_RESQ_TP, true, stream_);
            cur ^= 1;
        }
        xSlot_ = 2 * (int)l + 1;
        {
            const int epi = hQ80 ? hipk::EPI_ACT_Q80 : hipk::EPI_ACT;
            hipk::GemvArgs a13 = gemvArgs(L.w13, 0, 1, epi, nullptr, dim, nullptr, nullptr, nullptr, dH_, p.hidden0,
                                          nullptr, nullptr, nullptr, dHQ_, dHS_, false);
            consumer(a13);
            const float *wNext = l + 1 < h_.nLayers ? layers_[l + 1].rmsAtt : rmsFinal_;
            hipk::GemvArgs a2 = gemvArgs(L.w2, 0, 1, hipk::EPI_RESQ_TP, hQ80 ? nullptr : dH_, p.hidden0, nullptr, nullptr,
                                         nullptr, dY_, dim, nullptr, hQ80 ? dHQ_ : nullptr, hQ80 ? dHS_ : nullptr, nullptr,
                                         nullptr, true);
            producer(a2, wNext);
            if (ffnOn_) {  // one launch: w13 role + w2 role (weights prefetched before the hand-off wait)
                ProfScope ps(this, "ffn_block");
                hipk::launchFfnBlock(ffnBlockArgs(a13, a2, l), stream_);
            } else {
                {
                    ProfScope ps(this, "gemv_w13");
                    hipk::launchGemv(a13, 1, hipk::PRO_PRENORM, epi, true, stream_);
                }
                ProfScope ps(this, "gemv_w2");
                hipk::launchGemv(a2, 1, hQ80 ? hipk::PRO_GLOBAL : hipk::PRO_RESNORM, hipk::EPI_RESQ_TP, true, stream_);
            }
            cur ^= 1;
        }
    }
    xSlot_ = 2 * (int)h_.nLayers;  // logits gather / argmax winners
    ProfScope ps(this, "gemv_logits");
    if (argTail) {
        hipk::GemvArgs a = gemvArgs(wcls_, 0, 1, hipk::EPI_ARGMAX, nullptr, dim, nullptr, nullptr, nullptr, nullptr,
                                    p.vocab0, nullptr, nullptr, nullptr, nullptr, nullptr, false);
        consumer(a);
        a.am.ids = dIds_;
        a.am.partV = dArgV_;
        a.am.partI = dArgI_;
        a.am.counter = dArgCnt_;
        a.am.vocabStart = p.vocabStart();
        if (kind == GraphKind::CHAIN) {
            a.am.tokens = dTok_;
            a.am.pos = dPos_;
            a.am.hist = dHist_;
        }
        a.tp = tpArg_;
        a.tp.ticks = syncTicks();
        a.tp.span = syncSpan();
        hipk::launchGemv(a, 1, hipk::PRO_PRENORM, hipk::EPI_ARGMAX, true, stream_);
    } else {
        hipk::GemvArgs a = gemvArgs(wcls_, 0, 1, hipk::EPI_STORE, nullptr, dim, nullptr, nullptr, nullptr, dLogits_,
                                    p.vocab0, nullptr, nullptr, nullptr, nullptr, nullptr, false);
        consumer(a);
        hipk::launchGemv(a, 1, hipk::PRO_PRENORM, hipk::EPI_STORE, true, stream_);
    }
}

// The wo GEMV with the layer's attention in its prologue (PRO_ATTN, gemv_dev.h): every wo workgroup
// recomputes the rank's decode attention from the L2-resident cache instead of waiting for an
// attention launch, which at a TP-N rank's few heads is a handful of workgroups and a whole kernel
// boundary (TP8 rank of 8B: 4 heads, attention launch 5.8 us of a ~28 us layer, r5_decode_profile.md).
// The redundant work grows with the heads and the context, so it is taken for <= DL_WO_ATTN_HEADS
// (default 8) query heads per rank and context buckets of <= DL_WO_ATTN_LEN (256) positions; the
// block (TP1) and batched rows keep their own attention. With the fused exchange the kernel spins
// on peers, so its grid must be co-resident like the plain wo GEMV's.
// Measured (8B TP8 rank, f32 KV, same box): 0.973 ms/token with it vs 0.894 without - one
// workgroup computing all 4 heads of the rank serially (2 dependent key rounds, the per-key
// softmax of 4 heads on 256 lanes, then the ring's HBM latency, which cannot be issued before the
// attention: check_isa.py --hazards) costs more than the 4-workgroup attention launch it replaces.
// Opt-in (DL_WO_ATTN=1) for that reason; profiles/r6_tp_rank.md.
void HipEngineImpl::setupWoAttn() {
    woAttnOn_ = false;
    const char *e = std::getenv("DL_WO_ATTN");
    if (!(e && *e == '1') || !q40_) return;
    const char *hm = std::getenv("DL_WO_ATTN_HEADS");
    const char *lm = std::getenv("DL_WO_ATTN_LEN");
    const int maxHeads = hm && *hm ? std::atoi(hm) : 8;
    woAttnMaxLen_ = lm && *lm ? std::atoi(lm) : 256;
    if ((int)plan_.nHeads0 > maxHeads) return;
    const bool tp = fusedTp(false);
    const int epi = tp ? hipk::EPI_STORE_TP : hipk::EPI_STORE;
    const hipk::GemvArgs a = gemvArgs(layers_[0].wo, 0, 1, epi, nullptr, plan_.q0, nullptr, nullptr, nullptr, dY_,
                                      h_.dim, nullptr, dAttQ_, dAttS_, nullptr, nullptr, tp);
    const hipk::AttnArgs at = attnArgs(layers_[0], false);
    if (!hipk::gemvAttnSupported(a, at, epi)) return;
    if (tp) {
        const int share = comm_ ? std::max(1, comm_->ranksOnDevice()) : 1;
        const hipk::GemvResidency r = hipk::gemvAttnResidency(a, at, epi);
        if (r.maxResident <= 0 || r.grid > r.maxResident / share) return;
    }
    woAttnOn_ = true;
}

// A fused-block wait gave up (a workgroup of the launch never arrived): reset the monotonic
// counters and the epoch so the engine stays usable, then raise.
void HipEngineImpl::resetAttnBlockState() {
    DL_HIP(hipMemsetAsync(dBlockCnt_, 0, sizeof(unsigned) * kAllCntWords, stream_));
    DL_HIP(hipMemsetAsync(dEpoch_, 0, 2 * sizeof(unsigned), stream_));
    DL_HIP(hipMemsetAsync(dBlockErr_, 0, sizeof(int), stream_));
    DL_HIP(hipStreamSynchronize(stream_));
}

// Batched path (>= gemmMinTokens rows, Q40 or F32 weights): per chunk of <= 64 tokens, a norm kernel (f32 ->
// f16, RESNORM) or the producer's f16 rows (xh) feed the MFMA GEMM with the fused epilogue.
// Residual + norm fusion between batched GEMMs at TP1 (DL_GEMM_FUSE_NORM=0 disables, read at
// construction): wo / w2 end with EPI_RES (x' = x + out, x' * normW -> f16, per-tile sums of squares)
// and the next GEMM applies the RMS scale per token in its epilogue: no norm kernel between.
// At TP > 1 the batched path keeps the fused residual + norm too when the wo / w2 tiles can be
// all-reduced inside their GEMM epilogue (GemmArgs::tpx over the fused exchange: narrow
// launches of <= 64 rows whose tile + Q80 staging fit the launch's LDS); otherwise a separate
// all-reduce kernel and a norm kernel follow each of them. DL_TP_BATCHED=0 disables it.
bool HipEngineImpl::tpBatchedOk(int n) const {
    static const bool on = [] {
        const char *e = std::getenv("DL_TP_BATCHED");
        return !(e && *e == '0');
    }();
    return on && !invariant_ && tpFused_ && q40_ && !hipk::gemmUsesWide(n) &&
           (size_t)n * h_.dim <= (size_t)tpVec_.stride && hipk::gemmTpxFits(n, plan_.nRanks, tpVec_.q80 != 0);
}

void HipEngineImpl::gemmBatched(const DevMat &m, int n, int epi, const float *in, int ldIn, const float *add, float *xNext,
                 const float *normW, const _Float16 *xh, float *out, int ldOut, _Float16 *outH,
                 const DevLayer *L, const ResFuse *rf, bool ssIn) {
    // tokens per launch: the wide Q40 kernel takes the whole forward in one launch (one weight
    // pass per token tile, all tiles of a row tile on one XCD), the narrow one <= 128
    // (batch-invariant engines: narrow launches only, the split count of a 16-token launch for all)
    const int chunk = q40_ ? (hipk::gemmUsesWide(n) && !invariant_ ? n : kGemmMaxTokens) : hipk::kGemmF32MaxTokens;
    for (int c0 = 0; c0 < n; c0 += chunk) {
        const int bc = std::min(chunk, n - c0);
        xChunk_ = c0 / chunk;  // each launch's tile exchange waits in a measured-sync slot of its own
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
            a.tp.ticks = syncTicks();
            a.tp.span = syncSpan();
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
        g.splits = invariant_ ? hipk::gemmSplits(m.rows, m.n, 16, 0) : hipk::gemmSplits(m.rows, m.n, bc, q40_ ? m.lanes : 0);
        g.fixed = invariant_ ? 1 : 0;
        g.part = dPart_;
        g.partFloats = partFloats_;
        g.counters = dGemmCnt_;
        if (q40_)
            hipk::launchGemmQ40(g, epi, stream_);
        else
            hipk::launchGemmF32(g, epi, stream_);
    }
}

// Separate all-reduce of partial sums (batched path, RCCL, f32 weights). Q80 sync: every rank's
// partial is first rounded through Q80 blocks, as the reference's ZQ cast (llm.cpp:308-314).
void HipEngineImpl::allReduce(float *buf, size_t count) {
    if (plan_.nRanks > 1) {
        ProfScope ps(this, "allreduce");
        stamped([&] {
            if (syncQ80_) hipk::launchQ80Roundtrip(buf, count, stream_);
            comm_->allReduceSum(buf, count, stream_);
        });
    }
}

// The forward of n rows: embedding -> nLayers x [qkv (+RoPE, KV append) -> attention -> wo
// (-> all-reduce) -> w13 (SwiGLU) -> w2 (-> all-reduce)] -> logits -> (gather) -> argmax / sample.
// Single decode rows (GEMV path) run qkv + attention + wo as one fused attention-block launch when
// the context bucket allows it; batched rows run the MFMA GEMMs with residual + norm fused into
// their epilogues (reference step list: llm.cpp:200-434, ~840 barrier steps per forward).
void HipEngineImpl::enqueueForward(int n, GraphKind kind) {
    const ShardPlan &p = plan_;
    const int dim = h_.dim;
    int cur = 0;
    const bool bat = batchedPath(n);                                   // MFMA GEMMs on f16 activations
    const bool fz = bat && fuseNorm(n);                                // residual + norm in the GEMM epilogues
    const bool blk = blockOn_ && buckets_[bucket_].block && n == 1 && !bat;  // fused attention block
    const bool pre = prenormNow(n, bat, blk);  // pre-normalized Q80 hand-offs between the GEMVs
    {
        ProfScope ps(this, "embedding");
        // the epochs count the forwards that run the fused attention block / the FFN block (their
        // counters' targets); the two never run in the same forward (prenormNow excludes blk)
        unsigned *ep = blk ? dEpoch_ : (pre && ffnOn_) ? dEpoch_ + 1 : nullptr;
        hipk::launchEmbedding(emb_, dTok_, dX_[0], dim, n, stream_, ep,
                              p.nRanks > 1 ? dSync_ : nullptr, p.nRanks > 1 ? syncSlots() : 0);
    }
    // one greedy decode row: the logits GEMV ends in the row's argmax (EPI_ARGMAX: no logits
    // written, no argmax launch; under TP the winners trade over the fused exchange's region)
    const bool argTail = argTailOn_ && q40_ && !bat && !fz && n == 1 &&
                         (kind == GraphKind::ARGMAX || kind == GraphKind::CHAIN) &&
                         (p.nRanks == 1 || (tpFused_ && tpArg_.stride >= 2));
    if (pre) {
        enqueuePrenormLayers(kind, argTail);
        if (argTail) {
            DL_HIP(hipGetLastError());
            return;
        }
    }
    // Q80 hand-off of h needs one workgroup per 32 hidden units; for skinny TP shards the w13
    // epilogue emits f32 and w2 quantizes in its prologue instead.
    const bool hQ80 = q40_ && hQ80_;
    const bool woAttn = woAttnNow(n, bat, blk);  // attention inside the wo GEMV's prologue
    for (u32 l = 0; l < h_.nLayers && !pre; l++) {
        DevLayer &L = layers_[l];
        const bool hasDelta = l > 0;
        xSlot_ = 2 * (int)l;  // the wo exchange (fused in the wo kernel, or the all-reduce after it)
        if (blk) {
            ProfScope ps(this, "attn_block");
            hipk::AttnBlockArgs ba = attnBlockArgs(L, l, cur);
            if ((int)l == traceLayer_) ba.trace = traceBuf_;
            hipk::launchAttnBlock(ba, fusedTp(false), stream_);
            if (hasDelta) cur ^= 1;
        } else {
            {
                ProfScope ps(this, "gemv_qkv");
                if (fz && hasDelta)
                    gemmBatched(L.qkv, n, hipk::EPI_QKV, nullptr, dim, nullptr, nullptr, nullptr, nullptr, dQ_, p.q0,
                                nullptr, &L, nullptr, true);
                else if (bat)
                    gemmBatched(L.qkv, n, hipk::EPI_QKV, dX_[cur], dim, hasDelta ? dY_ : nullptr,
                                hasDelta ? dX_[cur ^ 1] : nullptr, L.rmsAtt, nullptr, dQ_, p.q0, nullptr, &L);
                else
                    gemv(L.qkv, n, hipk::PRO_RESNORM, hipk::EPI_QKV, dX_[cur], dim, hasDelta ? dY_ : nullptr,
                         hasDelta ? dX_[cur ^ 1] : nullptr, L.rmsAtt, dQ_, p.q0, &L);
            }
            if (hasDelta) cur ^= 1;
            if (!woAttn) {
                ProfScope ps(this, "attention");
                const hipk::AttnArgs a = attnArgs(L, bat);
                for (int r0 = 0; r0 < n; r0 += attRows_) {  // one launch unless the partials cap the rows
                    const int nr = std::min(attRows_, n - r0);
                    hipk::AttnArgs ar = a;
                    ar.q += (size_t)r0 * a.ldq;
                    ar.pos += r0;
                    ar.slot += r0;
                    ar.out += (size_t)r0 * a.ldOut;
                    if (ar.outH) ar.outH += (size_t)r0 * a.ldOut;
                    if (ar.outQ) ar.outQ += (size_t)r0 * a.ldOut;
                    if (ar.outS) ar.outS += (size_t)r0 * (a.ldOut / 32);
                    if (bat && prefillOk_)
                        hipk::launchAttentionPrefill(ar, nr, stream_);
                    else
                        hipk::launchAttention(ar, nr, stream_);
                }
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
                else if (woAttn) {
                    const bool tp = fusedTp(bat);
                    const int epi = tp ? hipk::EPI_STORE_TP : hipk::EPI_STORE;
                    xChunk_ = 0;
                    const hipk::GemvArgs a = gemvArgs(L.wo, 0, 1, epi, nullptr, p.q0, nullptr, nullptr, nullptr, dY_, dim,
                                                      nullptr, dAttQ_, dAttS_, nullptr, nullptr, tp);
                    hipk::launchGemvAttn(a, attnArgs(L, false), epi, stream_);
                } else
                    gemv(L.wo, n, hipk::PRO_GLOBAL, hipk::EPI_STORE, q40_ ? nullptr : dAtt_, p.q0, nullptr, nullptr,
                         nullptr, dY_, dim, nullptr, dAttQ_, dAttS_, nullptr, nullptr, fusedTp(bat));
            }
        }
        if (!fusedTp(bat) && !fz) allReduce(dY_, (size_t)n * dim);
        xSlot_ = 2 * (int)l + 1;  // the w2 exchange
        {
            ProfScope ps(this, "gemv_w13");
            if (fz)
                gemmBatched(L.w13, n, hipk::EPI_ACT_F16, nullptr, dim, nullptr, nullptr, nullptr, nullptr, nullptr,
                            p.hidden0, dHh_, nullptr, nullptr, true);
            else if (bat)
                gemmBatched(L.w13, n, hipk::EPI_ACT_F16, dX_[cur], dim, dY_, dX_[cur ^ 1], L.rmsFfn, nullptr, nullptr,
                            p.hidden0, dHh_, nullptr);
            else
                gemv(L.w13, n, hipk::PRO_RESNORM, hQ80 ? hipk::EPI_ACT_Q80 : hipk::EPI_ACT, dX_[cur], dim, dY_,
                     dX_[cur ^ 1], L.rmsFfn, dH_, p.hidden0, nullptr, nullptr, nullptr, dHQ_, dHS_);
        }
        cur ^= 1;
        {
            ProfScope ps(this, "gemv_w2");
            if (fz) {
                const float *wNext = l + 1 < h_.nLayers ? layers_[l + 1].rmsAtt : rmsFinal_;
                const ResFuse rf{dX_[cur], dX_[cur ^ 1], wNext};
                gemmBatched(L.w2, n, hipk::EPI_RES, nullptr, 0, nullptr, nullptr, nullptr, dHh_, nullptr, dim, nullptr,
                            nullptr, &rf);
            } else if (bat)
                gemmBatched(L.w2, n, hipk::EPI_STORE, nullptr, 0, nullptr, nullptr, nullptr, dHh_, dY_, dim, nullptr,
                            nullptr);
            else if (hQ80 || !q40_)
                gemv(L.w2, n, hipk::PRO_GLOBAL, hipk::EPI_STORE, q40_ ? nullptr : dH_, p.hidden0, nullptr, nullptr,
                     nullptr, dY_, dim, nullptr, dHQ_, dHS_, nullptr, nullptr, fusedTp(bat));
            else
                gemv(L.w2, n, hipk::PRO_RESNORM, hipk::EPI_STORE, dH_, p.hidden0, nullptr, nullptr, nullptr, dY_, dim,
                     nullptr, nullptr, nullptr, nullptr, nullptr, fusedTp(bat));
        }
        if (!fusedTp(bat) && !fz) allReduce(dY_, (size_t)n * dim);
    }
    xSlot_ = 2 * (int)h_.nLayers;  // logits gather / argmax winners
    if (!pre) {
        ProfScope ps(this, "gemv_logits");
        if (fz)
            gemmBatched(wcls_, n, hipk::EPI_STORE, nullptr, dim, nullptr, nullptr, nullptr, nullptr, dLogits_, p.vocab0,
                        nullptr, nullptr, nullptr, true);
        else if (bat)
            gemmBatched(wcls_, n, hipk::EPI_STORE, dX_[cur], dim, dY_, nullptr, rmsFinal_, nullptr, dLogits_, p.vocab0,
                        nullptr, nullptr);
        else if (argTail) {
            hipk::GemvArgs a = gemvArgs(wcls_, 0, 1, hipk::EPI_ARGMAX, dX_[cur], dim, dY_, nullptr, rmsFinal_, nullptr,
                                        p.vocab0, nullptr, nullptr, nullptr, nullptr, nullptr, false);
            a.am.ids = dIds_;
            a.am.partV = dArgV_;
            a.am.partI = dArgI_;
            a.am.counter = dArgCnt_;
            a.am.vocabStart = p.vocabStart();
            if (kind == GraphKind::CHAIN) {
                a.am.tokens = dTok_;
                a.am.pos = dPos_;
                a.am.hist = dHist_;
            }
            if (p.nRanks > 1) {
                a.tp = tpArg_;
                a.tp.ticks = syncTicks();
                a.tp.span = syncSpan();
            }
            hipk::launchGemv(a, 1, hipk::PRO_RESNORM, hipk::EPI_ARGMAX, true, stream_);
        } else
            gemv(wcls_, n, hipk::PRO_RESNORM, hipk::EPI_STORE, dX_[cur], dim, dY_, nullptr, rmsFinal_, dLogits_,
                 p.vocab0, nullptr);
    }
    if (argTail) {
        DL_HIP(hipGetLastError());
        return;
    }
    const float *full = dLogits_;
    // greedy rows under tensor parallelism: each rank reduces its own vocab slice and only the
    // (value, index) winners cross the links (reference: logits gathered to the root,
    // llm.cpp:432) - inside the argmax kernel on the fused data plane, else as one all-gather of
    // 2 floats per row; the full logits are gathered only when the host samples them
    const bool greedy = kind == GraphKind::ARGMAX || kind == GraphKind::CHAIN;
    const bool distArgmax = p.nRanks > 1 && greedy;
    // logits for the host (LOGITS) and sampled rows (SAMPLE) are needed on the root only: the
    // vocab slices are gathered to rank 0 (the reference's SYNC_NODE_SLICES_EXCEPT_ROOT), the
    // other ranks publish theirs and skip the unshard and the draw (the root's ids are used)
    const bool rootOnly = kind == GraphKind::LOGITS || kind == GraphKind::SAMPLE;
    if (p.nRanks > 1 && !distArgmax) {
        ProfScope ps(this, "allgather");
        stamped([&] {
            if (rootOnly)
                comm_->gatherToRoot(dLogits_, dLogitsAll_, (size_t)n * p.vocab0, stream_);
            else
                comm_->allGather(dLogits_, dLogitsAll_, (size_t)n * p.vocab0, stream_);
        });
        if (!rootOnly || rank() == 0) hipk::launchUnshardLogits(dLogitsAll_, dLogitsFull_, p.nRanks, n, p.vocab0, stream_);
        full = dLogitsFull_;
    }
    if (kind == GraphKind::SAMPLE) {
        if (p.nRanks == 1 || rank() == 0) {  // the other ranks' ids are not used (no draw, no argmax)
            ProfScope ps(this, "sample");
            hipk::SampleArgs g;
            g.logits = full;
            g.vocab = h_.vocabSize;
            g.spec = dSpec_;
            g.ids = dIds_;
            g.scratch = sampleScratch_;
            hipk::launchSample(g, n, stream_);
        }
    } else if (kind != GraphKind::LOGITS) {
        ProfScope ps(this, "argmax");
        hipk::ArgmaxArgs g;
        g.logits = full;
        g.vocab = h_.vocabSize;
        if (distArgmax) {
            g.vocab = p.vocab0;
            g.vocabStart = p.vocabStart();
            // fused winners exchange up to its region's rows (2 words per row), else one all-gather
            if (tpFused_ && (size_t)2 * n <= (size_t)tpArg_.stride) {
                g.tp = tpArg_;
                g.tp.ticks = syncTicks();
                g.tp.span = syncSpan();
            } else {
                g.pairs = dArgPairs_;
            }
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
        if (g.pairs) {
            stamped([&] { comm_->allGather(dArgPairs_, dArgPairsAll_, 2 * (size_t)n, stream_); });
            hipk::launchArgmaxPick(g, dArgPairsAll_, n, p.nRanks, stream_);
        }
    }
    DL_HIP(hipGetLastError());
}

}  // namespace engine_detail
}  // namespace dl
