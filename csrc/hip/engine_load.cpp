// Device buffers, capacity checks and the weight upload of the HIP engine (engine_impl.h).
#include "engine_impl.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../core/quant.h"

namespace dl {
namespace engine_detail {

// Refuse a configuration whose weights + KV cache cannot be resident, with the numbers, before
// allocating anything (KV is preallocated as nSlots x seqLen per layer).
void HipEngineImpl::checkFits() {
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
void HipEngineImpl::checkFusedResidency() {
    const ShardPlan &p = plan_;
    // ranks sharing this GPU (same-GPU rehearsals) share its resident slots; DL_FUSED_RESIDENT
    // overrides the limit (diagnostics / tests of the fallback)
    const int share = std::max(1, comm_->ranksOnDevice());
    const char *ov = std::getenv("DL_FUSED_RESIDENT");
    const bool hQ80 = hQ80_;
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

int HipEngineImpl::tpPasses(const DevMat &m, int bc) const {
    int passes = passesFor(m, hipk::EPI_STORE_TP, bc);
    if (tpVec_.q80)  // whole Q80 blocks of 32 rows per workgroup
        while ((256 / m.lanes * 2 * passes) % 32) passes++;
    return passes;
}

void HipEngineImpl::allocBuffers() {
    const u32 MB = cfg_.maxBatch;
    const ShardPlan &p = plan_;
    // [tokens | positions | slots | sample specs (4 floats per row)]: one H2D copy per forward
    dTok_ = dalloc<int>(7 * (size_t)MB);
    dPos_ = dTok_ + MB;
    dSlot_ = dTok_ + 2 * MB;
    dSpec_ = reinterpret_cast<float4 *>(dTok_ + 3 * MB);
    dIds_ = dalloc<int>(MB);
    dHist_ = dalloc<int>((size_t)decodeRows_ * h_.seqLen);  // greedy chains only (decode rows)
    hIn_ = halloc<int>(7 * MB);
    hIds_ = halloc<int>(MB);
    hErr_ = halloc<int>(2);
    hErr_[0] = hErr_[1] = 0;
    dX_[0] = dalloc<float>((size_t)MB * h_.dim);
    dX_[1] = dalloc<float>((size_t)MB * h_.dim);
    dY_ = dalloc<float>((size_t)MB * h_.dim);
    dQ_ = dalloc<float>((size_t)MB * p.q0);
    dAtt_ = dalloc<float>((size_t)MB * p.q0);
    dH_ = dalloc<float>((size_t)MB * p.hidden0);
    dAttQ_ = dalloc<int8_t>((size_t)MB * p.q0);
    dAttS_ = dalloc<float2>((size_t)MB * p.q0 / 32);
    dHQ_ = dalloc<int8_t>((size_t)MB * p.hidden0);
    dHS_ = dalloc<float2>((size_t)MB * p.hidden0 / 32);
    for (int i = 0; i < 2; i++) {
        dXQ_[i] = dalloc<int8_t>(h_.dim);
        dXS_[i] = dalloc<float2>((h_.dim + 31) / 32);
        dSSP_[i] = dalloc<float>(kMaxSsp);
    }
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
            if (invariant_ && q40_) part = std::max(part, hipk::gemmPartFloatsFixed(rows, n));
            cnt = std::max(cnt, hipk::gemmCounterInts(rows, mt));
        };
        acc(p.q0 + 2 * p.kv0, h_.dim);
        acc(h_.dim, p.q0);
        acc(2 * p.hidden0, h_.dim);
        acc(h_.dim, p.hidden0);
        acc(p.vocab0, h_.dim);
        if (part) dPart_ = dalloc<float>(part);
        partFloats_ = part;
        const int maxTiles = cnt;
        dGemmCnt_ = dalloc<int>(maxTiles);
        // fused residual + norm hand-off between batched GEMMs (TP1): per 64-row tile of dim,
        // per token, the partial sum of squares
        dSS_ = dalloc<float>((size_t)((h_.dim + 63) / 64) * MB);
        DL_HIP(hipMemsetAsync(dGemmCnt_, 0, sizeof(int) * maxTiles, stream_));
    }
    {  // fused attention block: epoch, monotonic counters, expected counts, timeout flag
        dEpoch_ = dalloc<unsigned>(4);
        // measured-sync slots (hipk::syncFoldWords: folded and cleared by the embedding kernel of
        // every forward) and their host copies (the last forward + one per chain step in flight)
        const size_t sw = hipk::syncFoldWords(syncSlots());
        dSync_ = dalloc<unsigned>(sw);
        hSync_ = halloc<unsigned>(sw * (1 + kChainDepth));
        DL_HIP(hipMemsetAsync(dSync_, 0, sw * sizeof(unsigned), stream_));
        std::memset(hSync_, 0, sw * (1 + kChainDepth) * sizeof(unsigned));
        dBlockCnt_ = dalloc<unsigned>(kAllCntWords);
        dBlockExpect_ = dalloc<unsigned>(kMaxKvGroups);
        dBlockErr_ = dalloc<int>(4);
        DL_HIP(hipMemsetAsync(dEpoch_, 0, 4 * sizeof(unsigned), stream_));
        DL_HIP(hipMemsetAsync(dBlockCnt_, 0, kAllCntWords * sizeof(unsigned), stream_));
        DL_HIP(hipMemsetAsync(dBlockExpect_, 0, kMaxKvGroups * sizeof(unsigned), stream_));
        DL_HIP(hipMemsetAsync(dBlockErr_, 0, 4 * sizeof(int), stream_));
    }
    dAttCnt_ = dalloc<int>((size_t)MB * p.nHeads0);
    DL_HIP(hipMemsetAsync(dAttCnt_, 0, sizeof(int) * (size_t)MB * p.nHeads0, stream_));
    // argmax partials: 64 workgroups per row (argmaxKernel), or one per workgroup of the logits
    // GEMV (EPI_ARGMAX: >= 8 rows per workgroup)
    const size_t argParts = std::max<size_t>((size_t)MB * 64, p.vocab0 / 8 + 1);
    dArgV_ = dalloc<float>(argParts);
    dArgI_ = dalloc<int>(argParts);
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
        dArgPairs_ = dalloc<float>((size_t)MB * 2);
        dArgPairsAll_ = dalloc<float>((size_t)MB * 2 * p.nRanks);
    }
    setupBuckets();  // the largest bucket sizes the split-attention partials
    const int splitMax = buckets_.back().splitGrid;
    {  // attention split partials: every row of a forward while they stay <= 256 MB, else the
       // launches take row chunks (multiples of 64 rows: whole prefill row blocks of one slot)
        const size_t perRow = (size_t)p.nHeads0 * splitMax * (p.headSize + 2) * sizeof(float);
        const size_t fit = ((size_t)256 << 20) / perRow / 64 * 64;
        attRows_ = (int)std::min<size_t>(MB, std::max<size_t>({fit, (size_t)decodeRows_, 64}));
    }
    dPartO_ = dalloc<float>((size_t)attRows_ * p.nHeads0 * splitMax * p.headSize);
    dPartML_ = dalloc<float>((size_t)attRows_ * p.nHeads0 * splitMax * 2);
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

void HipEngineImpl::uploadRope() {
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
struct HipEngineImpl::Loader {
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

u8 *HipEngineImpl::stageAcquire(Loader &ld) {
    ld.cur ^= 1;
    if (ld.busy[ld.cur]) DL_HIP(hipEventSynchronize(ld.done[ld.cur]));
    ld.busy[ld.cur] = false;
    return ld.stage[ld.cur];
}

void HipEngineImpl::stageCopy(Loader &ld, void *dst, const u8 *src, size_t bytes) {
    DL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ld.copy));
}

void HipEngineImpl::stageRelease(Loader &ld) {
    DL_HIP(hipEventRecord(ld.done[ld.cur], ld.copy));
    ld.busy[ld.cur] = true;
}

// Read the rows of every source (restricted to columns [c0, c0 + nc)) into ld.raw and point
// ld.rowPtr at each output row (w1/w3 interleaved row by row when `interleave`).
void HipEngineImpl::readRows(Loader &ld, const std::vector<RowSrc> &srcs, bool interleave, u32 c0, u32 nc) {
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

size_t HipEngineImpl::matStageBytes(u32 rows, u32 n) const {
    if (!q40_) return (size_t)rows * n * 4;
    const hipk::Q40Tiling t = hipk::q40Tiling((int)rows, (int)n, lanesFor((int)rows, (int)n));
    return t.qsBytes + t.dBytes;
}

// Device storage of a Q40 matrix: layer matrix `mi` (0 qkv, 1 wo, 2 w13, 3 w2) of layer l lives in
// one slab per matrix kind, all layers back to back (4 allocations instead of 4 x nLayers);
// other matrices get their own allocation.
void HipEngineImpl::placeQ40(DevMat &m, const hipk::Q40Tiling &t, int mi, u32 l) {
    if (mi < 0) {
        m.qs = dalloc<uint8_t>(t.qsBytes);
        m.d = dalloc<uint16_t>(t.dBytes / 2);
        return;
    }
    if (!qsSlab_[mi]) {
        qsStride_[mi] = t.qsBytes;
        dStride_[mi] = t.dBytes;
        qsSlab_[mi] = dalloc<uint8_t>(t.qsBytes * h_.nLayers);
        dSlab_[mi] = dalloc<uint16_t>(t.dBytes / 2 * h_.nLayers);
    }
    DL_CHECK(qsStride_[mi] == t.qsBytes && dStride_[mi] == t.dBytes, "layer matrices of one kind differ in size");
    m.qs = qsSlab_[mi] + (size_t)l * qsStride_[mi];
    m.d = dSlab_[mi] + (size_t)l * (dStride_[mi] / 2);
}

void HipEngineImpl::buildMat(Loader &ld, DevMat &m, const std::vector<RowSrc> &srcs, bool interleave, u32 c0, u32 nc,
                             int mi, u32 l) {
    readRows(ld, srcs, interleave, c0, nc);
    const int rows = (int)ld.rowPtr.size();
    m.rows = rows;
    m.n = (int)nc;
    u8 *st = stageAcquire(ld);
    if (q40_) {
        m.lanes = lanesFor(rows, (int)nc);
        const hipk::Q40Tiling t = hipk::q40Tiling(rows, (int)nc, m.lanes);
        DL_CHECK(t.qsBytes + t.dBytes <= ld.stageBytes, "staging buffer too small");
        hipk::tileQ40AoS(ld.rowPtr.data(), rows, (int)nc, m.lanes, st, reinterpret_cast<uint32_t *>(st + t.qsBytes));
        placeQ40(m, t, mi, l);
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
float *HipEngineImpl::uploadF32(Loader &ld, const TensorInfo &t) {
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

void HipEngineImpl::loadFromFile() {
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
                     false, 0, h_.dim, 0, l);
            buildMat(ld, L.wo, {{&wo, 0, h_.dim}}, false, p.qStart(), p.q0, 1, l);
            buildMat(ld, L.w13, {{&w1, p.hiddenStart(), p.hidden0}, {&w3, p.hiddenStart(), p.hidden0}}, true, 0,
                     h_.dim, 2, l);
            buildMat(ld, L.w2, {{&w2, 0, h_.dim}}, false, p.hiddenStart(), p.hidden0, 3, l);
            L.rmsAtt = uploadF32(ld, f.find(TensorKind::RMS_ATT, l));
            L.rmsFfn = uploadF32(ld, f.find(TensorKind::RMS_FFN, l));
        }
        emb_ = uploadF32(ld, f.find(TensorKind::EMBEDDING, -1));
        rmsFinal_ = uploadF32(ld, f.find(TensorKind::RMS_FINAL, -1));
        buildMat(ld, wcls_, {{&f.find(TensorKind::WCLS, -1), p.vocabStart(), p.vocab0}}, false, 0, h_.dim, -1, 0);
        DL_HIP(hipStreamSynchronize(ld.copy));
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
    load_.fileBytes = ld.reader->bytesRead();
}

void HipEngineImpl::synthMat(DevMat &m, int rows, int n, u64 seed, int mi, u32 l) {
    m.rows = rows;
    m.n = n;
    const float scale = 1.0f / std::sqrt(21.5f * (float)n);
    if (q40_) {
        m.lanes = lanesFor(rows, n);
        const hipk::Q40Tiling t = hipk::q40Tiling(rows, n, m.lanes);
        const size_t nBlocks = t.qsBytes / 16;  // == t.dBytes / 2 f16 scales
        placeQ40(m, t, mi, l);
        hipk::launchFillQ40(m.qs, m.d, nBlocks, scale, seed, stream_);
    } else {
        m.f = dalloc<float>((size_t)rows * n);
        hipk::launchFillF32Uniform(m.f, (size_t)rows * n, std::sqrt(3.0f / (float)n), seed, stream_);
    }
    DL_HIP(hipGetLastError());
}

void HipEngineImpl::loadSynthetic() {
    const ShardPlan &p = plan_;
    u64 seed = cfg_.seed * 1000003ull + (u64)p.rank * 7919ull;
    for (u32 l = 0; l < h_.nLayers; l++) {
        DevLayer &L = layers_[l];
        synthMat(L.qkv, p.q0 + 2 * p.kv0, h_.dim, seed++, 0, l);
        synthMat(L.wo, h_.dim, p.q0, seed++, 1, l);
        synthMat(L.w13, 2 * p.hidden0, h_.dim, seed++, 2, l);
        synthMat(L.w2, h_.dim, p.hidden0, seed++, 3, l);
        L.rmsAtt = dalloc<float>(h_.dim);
        L.rmsFfn = dalloc<float>(h_.dim);
        hipk::launchFillF32Const(L.rmsAtt, h_.dim, 1.0f, stream_);
        hipk::launchFillF32Const(L.rmsFfn, h_.dim, 1.0f, stream_);
    }
    emb_ = dalloc<float>((size_t)h_.vocabSize * h_.dim);
    hipk::launchFillF32Uniform(emb_, (size_t)h_.vocabSize * h_.dim, 1.0f, cfg_.seed ^ 0xE3B, stream_);
    rmsFinal_ = dalloc<float>(h_.dim);
    hipk::launchFillF32Const(rmsFinal_, h_.dim, 1.0f, stream_);
    synthMat(wcls_, p.vocab0, h_.dim, seed++, -1, 0);
    DL_HIP(hipGetLastError());
}

}  // namespace engine_detail
}  // namespace dl
