// Paged KV cache of the HIP engine (engine_impl.h).
#include "engine_impl.h"

namespace dl {
namespace engine_detail {

// ---------------------------------------------------------------- paged KV cache
// With cfg.kvPages > 0 each layer's K / V cache is a pool of kvPages pages of kvPageSize
// positions and a page table maps (slot, pos) to a pool row (kernels.h KvMap): a slot holds only
// the pages its sequence reached, so many slots can share HBM sized for the tokens actually in
// flight instead of nSlots x seqLen. Pages are mapped at setInputs for every position a forward
// (or a decode chain) writes and released when a slot restarts at position 0: the same
// deterministic rule on every tensor-parallel rank, so no page messages are exchanged.
void HipEngineImpl::releaseSlot(int slot) {
    if (!paged() || slot < 0 || (u32)slot >= cfg_.nSlots) return;
    for (int i = 0; i < slotPages_[slot]; i++) {
        int &e = hostTable_[(size_t)slot * pagesPerSlot_ + i];
        freePages_.push_back(e);
        e = -1;
    }
    if (slotPages_[slot]) tableDirty_ = true;  // uploaded with the next forward's mapping
    slotPages_[slot] = 0;
}

void HipEngineImpl::setupPages() {
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

hipk::KvMap HipEngineImpl::kvMap() const {
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
void HipEngineImpl::mapPages(int n, const int *positions, const int *slots, int ahead) {
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

}  // namespace engine_detail
}  // namespace dl
