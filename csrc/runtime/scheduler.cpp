#include "scheduler.h"

#include <algorithm>
#include <cstring>

namespace dl {

std::string GenRequest::wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
    return text;
}

bool GenRequest::nextDelta(std::string &out) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done || !deltas.empty(); });
    if (!deltas.empty()) {
        out = std::move(deltas.front());
        deltas.pop_front();
        return true;
    }
    return false;
}

void GenRequest::emit(const std::string &d) {
    if (d.empty()) return;
    std::lock_guard<std::mutex> lk(mu);
    text += d;
    deltas.push_back(d);
    cv.notify_all();
}

void GenRequest::finish(const std::string &reason) {
    std::lock_guard<std::mutex> lk(mu);
    finishReason = reason;
    done = true;
    cv.notify_all();
}

Scheduler::Scheduler(InferenceSession &sess) : sess_(sess), tok_(sess.tokenizer()) {
    for (int s = sess.nSlots() - 1; s >= 0; s--) freeSlots_.push_back(s);
    pagesTotal_ = sess.kvPagesFree();
    pageSize_ = sess.kvPageSize();
    slotPages_.assign(sess.nSlots(), 0);
    thread_ = std::thread([this] { loop(); });
}

Scheduler::~Scheduler() { stop(); }

void Scheduler::stop() {
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (stop_) return;
        stop_ = true;
    }
    cv_.notify_all();
    if (thread_.joinable()) thread_.join();
    // fail anything still pending
    for (auto &r : queue_) r->finish("error");
    for (auto &r : active_) r->finish("error");
}

std::shared_ptr<GenRequest> Scheduler::submit(std::vector<int> prompt, const GenParams &params) {
    auto r = std::make_shared<GenRequest>();
    r->prompt = std::move(prompt);
    r->params = params;
    {
        std::lock_guard<std::mutex> lk(mu_);
        r->id = nextId_++;
        if (stop_) {
            r->error = "scheduler stopped";
            r->finish("error");
            return r;
        }
        queue_.push_back(r);
    }
    cv_.notify_all();
    return r;
}

SchedulerStats Scheduler::stats() {
    std::lock_guard<std::mutex> lk(mu_);
    SchedulerStats s = stats_;
    s.queued = (int)queue_.size();
    return s;
}

void Scheduler::loop() {
    while (true) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || !queue_.empty() || !active_.empty() || inflight_; });
            if (stop_) break;
        }
        try {
            step();
        } catch (const std::exception &e) {
            // a failed forward poisons every in-flight request; the session stays usable
            failAll(e.what());
        }
    }
    if (inflight_) {  // leave no forward running on the backend
        try {
            std::vector<int> ids(flight_.n);
            sess_.collectIds(flight_.n, ids.data());
        } catch (const std::exception &) {
        }
        inflight_ = false;
    }
}

// Under mu_. A request's slot becomes free. With a paged KV cache its pages go back to the pool
// on every rank first: the slot waits in releasing_ until flushReleases() has sent the RELEASE
// (network I/O, never under mu_, so submit() / stats() on the HTTP threads do not stall).
void Scheduler::returnSlot(int slot) {
    if (pagesTotal_ >= 0 && slotPages_[slot])
        releasing_.push_back(slot);
    else
        freeSlots_.push_back(slot);
}

// Scheduler thread, without mu_: release the pages of the slots returned since the last call,
// then make the slots admissible again (before the next admission / launch).
void Scheduler::flushReleases() {
    std::vector<int> rel;
    {
        std::lock_guard<std::mutex> lk(mu_);
        rel.swap(releasing_);
    }
    if (rel.empty()) return;
    for (int s : rel) {
        try {
            sess_.releaseSlot(s);
        } catch (const std::exception &) {  // a lost worker surfaces on the next forward
        }
    }
    std::lock_guard<std::mutex> lk(mu_);
    for (int s : rel) {
        slotPages_[s] = 0;
        freeSlots_.push_back(s);
    }
}

void Scheduler::failAll(const std::string &what) {
    // the launched forward (if any) is collected first: it still writes the slots handed back
    // below, and the backend refuses the next launch until it has been collected
    bool hadFlight;
    {
        std::lock_guard<std::mutex> lk(mu_);
        hadFlight = inflight_;
    }
    if (hadFlight) {
        try {
            std::vector<int> ids(flight_.n);
            sess_.collectIds(flight_.n, ids.data());
        } catch (const std::exception &) {
        }
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        inflight_ = false;
        flight_.picks.clear();
        for (auto &r : active_) {
            r->error = what;
            r->finished = true;
            r->finish("error");
            returnSlot(r->slot);
        }
        for (auto &r : draining_) returnSlot(r->slot);
        active_.clear();
        draining_.clear();
    }
    flushReleases();
}

// Under mu_. Finished requests leave active_; their KV slot is reused only once no forward in
// flight still writes it (rows launched before the host saw the EOS are dropped at collection).
void Scheduler::finishRequest(const std::shared_ptr<GenRequest> &r, const char *reason) {
    r->finished = true;
    r->finish(reason);
    bool inFlight = false;
    if (inflight_)
        for (auto &p : flight_.picks)
            if (p.r == r) inFlight = true;
    if (inFlight)
        draining_.push_back(r);
    else
        returnSlot(r->slot);
    active_.erase(std::remove(active_.begin(), active_.end(), r), active_.end());
}

bool Scheduler::step() {
    const u32 seqLen = sess_.header().seqLen;
    const int vocab = (int)sess_.header().vocabSize;

    // 0) collect the forward in flight: token ids and prompt progress only (cheap); the text work
    //    for these tokens runs after the next forward has been launched (step 4)
    std::vector<Pick> done;
    std::vector<int> ids;
    int doneRows = 0, doneDecode = 0;
    double doneMs = 0;
    if (inflight_) {
        ids.resize(flight_.n);
        sess_.collectIds(flight_.n, ids.data());
        doneMs = flight_.t.elapsedMs();
        doneRows = flight_.n;
        doneDecode = flight_.nDecode;
        for (auto &p : flight_.picks) {
            GenRequest *r = p.r.get();
            if (r->finished) continue;  // finished while its row was in flight: dropped
            r->prefilled += p.prefill;
            if (p.sample) r->generated.push_back(ids[p.row]);
        }
        done.swap(flight_.picks);
        inflight_ = false;
        std::lock_guard<std::mutex> lk(mu_);
        for (auto &r : draining_) returnSlot(r->slot);  // their last rows have completed
        draining_.clear();
    }
    flushReleases();  // slots freed by the previous step's text work and by the collection above

    // 1) admission: one free KV slot per request (and, with a paged KV cache, the pages its prompt +
    //    max_tokens can reach; FIFO: the head waits until enough pages are free); cancelled requests
    //    give their slot back
    {
        std::lock_guard<std::mutex> lk(mu_);
        while (!queue_.empty() && !freeSlots_.empty()) {
            auto r = queue_.front();
            if (r->isCancelled()) {
                queue_.pop_front();
                r->finish("cancelled");
                stats_.cancelled++;
                continue;
            }
            if (r->prompt.empty() || r->prompt.size() >= seqLen) {
                queue_.pop_front();
                r->error = r->prompt.empty() ? "empty prompt" : "prompt longer than the context";
                r->finish("error");
                continue;
            }
            const int slot = freeSlots_.back();
            if (pagesTotal_ >= 0) {
                const u64 span = r->params.maxTokens > 0 ? (u64)r->prompt.size() + (u64)r->params.maxTokens + 1 : seqLen;
                const int need = (int)((std::min<u64>(span, seqLen) + pageSize_ - 1) / pageSize_);
                int held = 0;  // pages reserved by the active requests
                for (int p : slotPages_) held += p;
                if (need > pagesTotal_) {
                    queue_.pop_front();
                    r->error = "request needs more KV pages than the pool holds";
                    r->finish("error");
                    continue;
                }
                if (need > pagesTotal_ - held) break;  // wait for pages
                slotPages_[slot] = need;
            }
            queue_.pop_front();
            r->slot = slot;
            freeSlots_.pop_back();
            r->prefilled = 0;
            r->sampler.reset(new Sampler(vocab, r->params.temperature, r->params.topp, r->params.seed));
            r->decoder.reset(new TokenDecoder(tok_));
            ChatStops cs(tok_);
            std::vector<std::string> stops = cs.stops;
            size_t maxLen = cs.maxStopLength;
            for (auto &s : r->params.stop)
                if (!s.empty()) {
                    stops.push_back(s);
                    maxLen = std::max(maxLen, s.size());
                }
            std::vector<int> eosIds = tok_.eosTokenIds();
            while (eosIds.size() < stops.size()) eosIds.push_back(-1);
            r->eos.reset(new EosDetector(eosIds, stops, (int)maxLen, (int)maxLen));
            active_.push_back(r);
        }
        // the cancel flag is read ONCE per request (cancel() runs on HTTP threads without mu_)
        std::vector<std::shared_ptr<GenRequest>> cancelled;
        for (auto &r : active_)
            if (r->isCancelled()) cancelled.push_back(r);
        for (auto &r : cancelled) {
            finishRequest(r, "cancelled");
            stats_.cancelled++;
        }
        stats_.active = (int)active_.size();
    }

    // 2) build the next batch: decode rows first (latency), then prefill chunks with the remaining
    //    budget. A decode row is launched before the host has decoded the previous token: a request
    //    whose last token turns out to end it (EOS / stop string) wastes one row, dropped at collection.
    // decode rows first (<= --max-batch), then prompt rows up to the prefill chunk
    const int maxRows = std::max(sess_.maxBatch(), sess_.prefillChunk());
    std::vector<int> tokens, positions, slots;
    Flight next;
    for (auto &rp : active_) {
        GenRequest *r = rp.get();
        if (r->prefilled < r->prompt.size()) continue;
        if ((int)tokens.size() >= sess_.maxBatch()) break;
        const int pos = (int)(r->prompt.size() + r->generated.size()) - 1;
        if ((r->params.maxTokens > 0 && (int)r->generated.size() >= r->params.maxTokens) || (u32)(pos + 1) >= seqLen)
            continue;  // ends at this step's text work (length)
        tokens.push_back(r->generated.back());
        positions.push_back(pos);
        slots.push_back(r->slot);
        next.picks.push_back({rp, (int)tokens.size() - 1, true, 0});
    }
    next.nDecode = (int)tokens.size();
    for (auto &rp : active_) {
        GenRequest *r = rp.get();
        if (r->prefilled >= r->prompt.size()) continue;
        const int budget = maxRows - (int)tokens.size();
        if (budget <= 0) break;
        const int take = (int)std::min<size_t>(budget, r->prompt.size() - r->prefilled);
        for (int i = 0; i < take; i++) {
            tokens.push_back(r->prompt[r->prefilled + i]);
            positions.push_back((int)(r->prefilled + i));
            slots.push_back(r->slot);
        }
        const bool completes = r->prefilled + take == r->prompt.size();
        next.picks.push_back({rp, (int)tokens.size() - 1, completes, take});
    }
    next.n = (int)tokens.size();

    // 3) launch: device argmax when every sampled row is greedy; otherwise per-row draws on the
    //    backend (the device sampler on GPUs) with each request's own temperature / top-p and the
    //    coin its own seeded generator yields, so only token ids come back
    if (next.n > 0) {
        bool allGreedy = true;
        for (auto &p : next.picks)
            if (p.sample && p.r->params.temperature != 0.0f) allGreedy = false;
        next.t.reset();
        if (allGreedy) {
            sess_.launchIds(next.n, tokens.data(), positions.data(), slots.data(), nullptr);
        } else {
            std::vector<SampleSpec> specs(next.n);
            for (auto &sp : specs) sp.temperature = -1.f;  // rows that are not sampled
            for (auto &p : next.picks) {
                if (!p.sample) continue;
                SampleSpec &sp = specs[p.row];
                sp.temperature = p.r->params.temperature;
                sp.topp = p.r->params.topp;
                sp.coin = p.r->sampler->drawCoin();
            }
            sess_.launchIds(next.n, tokens.data(), positions.data(), slots.data(), specs.data());
        }
        std::lock_guard<std::mutex> lk(mu_);
        flight_ = std::move(next);
        inflight_ = true;
    }

    // 4) text work of the collected forward (overlaps the forward just launched): decode, detect
    //    stops, stream deltas, finish
    std::lock_guard<std::mutex> lk(mu_);
    if (doneRows > 0) {
        stats_.forwards++;
        stats_.rows += doneRows;
        stats_.decodeRows += doneDecode;
        stats_.prefillRows += doneRows - doneDecode;
        stats_.busyMs += doneMs;
    }
    for (auto &p : done) {
        const std::shared_ptr<GenRequest> &rp = p.r;
        GenRequest *r = rp.get();
        if (!p.sample || r->finished) continue;
        const int token = ids[p.row];
        r->completionTokens = (int)r->generated.size();
        std::string piece, delta;
        const bool has = r->decoder->decode(token, piece);
        const EosResult er = r->eos->append(token, has ? piece.c_str() : nullptr);
        if (er == EosResult::NOT_EOS || er == EosResult::EOS) {
            if (r->eos->getDelta(delta)) r->emit(delta);
            r->eos->reset();
        }
        const int nextPos = (int)(r->prompt.size() + r->generated.size());
        const char *reason = nullptr;
        if (er == EosResult::EOS)
            reason = "stop";
        else if ((r->params.maxTokens > 0 && (int)r->generated.size() >= r->params.maxTokens) || (u32)nextPos >= seqLen)
            reason = "length";
        if (reason) {
            stats_.completed++;
            stats_.generatedTokens += r->generated.size();
            finishRequest(rp, reason);
        }
    }
    stats_.active = (int)active_.size();
    return next.n > 0 || doneRows > 0;
}

}  // namespace dl
