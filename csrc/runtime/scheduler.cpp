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
            cv_.wait(lk, [&] { return stop_ || !queue_.empty() || !active_.empty(); });
            if (stop_) return;
        }
        try {
            step();
        } catch (const std::exception &e) {
            // a failed forward poisons every in-flight request; the session stays usable
            std::lock_guard<std::mutex> lk(mu_);
            for (auto &r : active_) {
                r->error = e.what();
                r->finish("error");
                freeSlots_.push_back(r->slot);
            }
            active_.clear();
        }
    }
}

bool Scheduler::step() {
    const u32 seqLen = sess_.header().seqLen;
    const int vocab = (int)sess_.header().vocabSize;
    // 1) admission: one free KV slot per request
    {
        std::lock_guard<std::mutex> lk(mu_);
        while (!queue_.empty() && !freeSlots_.empty()) {
            auto r = queue_.front();
            queue_.pop_front();
            if (r->isCancelled()) {
                r->finish("cancelled");
                stats_.cancelled++;
                continue;
            }
            if (r->prompt.empty() || r->prompt.size() >= seqLen) {
                r->error = r->prompt.empty() ? "empty prompt" : "prompt longer than the context";
                r->finish("error");
                continue;
            }
            r->slot = freeSlots_.back();
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
        // requests whose client disconnected give their slot back before the batch is built; the
        // flag is read ONCE per request (cancel() runs on HTTP threads without mu_), so a request
        // is either finished + freed + dropped, or kept - never dropped with its slot still held
        std::vector<std::shared_ptr<GenRequest>> keep;
        keep.reserve(active_.size());
        for (auto &r : active_) {
            if (r->isCancelled()) {
                r->finish("cancelled");
                freeSlots_.push_back(r->slot);
                stats_.cancelled++;
            } else {
                keep.push_back(r);
            }
        }
        active_.swap(keep);
        stats_.active = (int)active_.size();
    }
    if (active_.empty()) return false;

    // 2) build the batch: decode rows first (latency), then prefill chunks with the remaining budget
    const int maxRows = sess_.maxBatch();
    std::vector<int> tokens, positions, slots;
    struct Pick {
        GenRequest *r;
        int row;       // batch row whose logits are sampled
        bool sample;
        int prefill;   // prompt tokens consumed this step
    };
    std::vector<Pick> picks;
    for (auto &rp : active_) {
        GenRequest *r = rp.get();
        if (r->prefilled < r->prompt.size()) continue;
        if ((int)tokens.size() >= maxRows) break;
        const int pos = (int)(r->prompt.size() + r->generated.size()) - 1;
        tokens.push_back(r->generated.back());
        positions.push_back(pos);
        slots.push_back(r->slot);
        picks.push_back({r, (int)tokens.size() - 1, true, 0});
    }
    const int nDecode = (int)tokens.size();
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
        picks.push_back({r, (int)tokens.size() - 1, completes, take});
    }
    const int n = (int)tokens.size();
    if (n == 0) return false;

    // 3) forward: device argmax when every sampled row is greedy; otherwise per-row draws on the
    //    backend (the device sampler on GPUs) with each request's own temperature / top-p and the
    //    coin its own seeded generator yields, so only token ids come back
    bool allGreedy = true;
    for (auto &p : picks)
        if (p.sample && p.r->params.temperature != 0.0f) allGreedy = false;
    Timer t;
    std::vector<int> ids(n);
    if (allGreedy) {
        sess_.forwardArgmax(n, tokens.data(), positions.data(), slots.data(), ids.data());
    } else {
        std::vector<SampleSpec> specs(n);
        for (auto &sp : specs) sp.temperature = -1.f;  // rows that are not sampled
        for (auto &p : picks) {
            if (!p.sample) continue;
            SampleSpec &sp = specs[p.row];
            sp.temperature = p.r->params.temperature;
            sp.topp = p.r->params.topp;
            sp.coin = p.r->sampler->drawCoin();
        }
        sess_.forwardSample(n, tokens.data(), positions.data(), slots.data(), specs.data(), ids.data());
    }
    (void)vocab;
    const double ms = t.elapsedMs();

    // 4) sample, detect stops, stream deltas
    std::vector<GenRequest *> finished;
    for (auto &p : picks) {
        GenRequest *r = p.r;
        r->prefilled += p.prefill;
        if (!p.sample) continue;
        const int token = ids[p.row];
        r->generated.push_back(token);
        r->completionTokens = (int)r->generated.size();
        std::string piece, delta;
        const bool has = r->decoder->decode(token, piece);
        const EosResult er = r->eos->append(token, has ? piece.c_str() : nullptr);
        if (er == EosResult::NOT_EOS || er == EosResult::EOS) {
            if (r->eos->getDelta(delta)) r->emit(delta);
            r->eos->reset();
        }
        const int nextPos = (int)(r->prompt.size() + r->generated.size());
        if (er == EosResult::EOS) {
            r->finish("stop");
            finished.push_back(r);
        } else if ((r->params.maxTokens > 0 && (int)r->generated.size() >= r->params.maxTokens) ||
                   (u32)nextPos >= seqLen) {
            r->finish("length");
            finished.push_back(r);
        }
    }

    std::lock_guard<std::mutex> lk(mu_);
    stats_.forwards++;
    stats_.rows += n;
    stats_.decodeRows += nDecode;
    stats_.prefillRows += n - nDecode;
    stats_.busyMs += ms;
    for (GenRequest *r : finished) {
        stats_.completed++;
        stats_.generatedTokens += r->generated.size();
        freeSlots_.push_back(r->slot);
        active_.erase(std::remove_if(active_.begin(), active_.end(),
                                     [r](const std::shared_ptr<GenRequest> &x) { return x.get() == r; }),
                      active_.end());
    }
    stats_.active = (int)active_.size();
    return true;
}

}  // namespace dl
