// Multi-user continuous-batching scheduler (replaces the reference's Request/RequestQueue +
// inference_loop, src/Request.hpp:11-64, src/app.cpp:314-402).
//
// Fixes the reference defects SURVEY §2.9 Q1-Q5: every request owns a KV-cache slot and its own
// positions; prompts are really prefilled (chunked, mixed with other requests' decode rows in the
// same forward); each request has its own sampler/seed/temperature/stop strings and UTF-8 decoder;
// the loop has a lifecycle (stop()) and the API front end is concurrent.
#pragma once

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "app.h"

namespace dl {

struct GenParams {
    int maxTokens = 128;      // reference default (Request.hpp:33); <= 0 = until EOS / context end
    float temperature = 0.8f;
    float topp = 0.9f;
    u64 seed = 0;
    std::vector<std::string> stop;  // extra stop strings
};

class GenRequest {
  public:
    u64 id = 0;
    std::vector<int> prompt;
    GenParams params;

    // ---- results (guarded by mu) ----
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::string> deltas;  // streamed text pieces not yet consumed
    std::string text;                // full generated text
    std::string finishReason;        // "stop" | "length" | "error"
    std::string error;
    bool done = false;
    int completionTokens = 0;

    // The client went away (e.g. a streaming connection dropped): the scheduler finishes the
    // request at its next step and frees its KV slot instead of generating to max_tokens.
    void cancel() { cancelled.store(true); }
    bool isCancelled() const { return cancelled.load(); }

    // Blocks until finished; returns the full text.
    std::string wait();
    // Pops the next delta (blocking); returns false once the request is done and drained.
    bool nextDelta(std::string &out);

  private:
    friend class Scheduler;
    std::atomic<bool> cancelled{false};
    bool finished = false;  // scheduler thread only: finish() ran (rows still in flight are dropped)
    int slot = -1;
    size_t prefilled = 0;
    std::vector<int> generated;
    std::unique_ptr<Sampler> sampler;
    std::unique_ptr<TokenDecoder> decoder;
    std::unique_ptr<EosDetector> eos;
    void emit(const std::string &d);
    void finish(const std::string &reason);
};

struct SchedulerStats {
    u64 forwards = 0, rows = 0, prefillRows = 0, decodeRows = 0, completed = 0, generatedTokens = 0, cancelled = 0;
    double busyMs = 0;
    int active = 0, queued = 0;
};

class Scheduler {
  public:
    explicit Scheduler(InferenceSession &sess);
    ~Scheduler();
    std::shared_ptr<GenRequest> submit(std::vector<int> prompt, const GenParams &params);
    void stop();
    SchedulerStats stats();

  private:
    // One batched forward in flight (pipelined serving): while the device runs it, the host
    // decodes, EOS-checks and streams the previous forward's tokens.
    struct Pick {
        std::shared_ptr<GenRequest> r;
        int row;      // batch row whose id belongs to the request
        bool sample;  // the row yields the request's next token
        int prefill;  // prompt tokens consumed by this forward
    };
    struct Flight {
        std::vector<Pick> picks;
        int n = 0, nDecode = 0;
        Timer t;
    };
    void loop();
    bool step();  // collect the forward in flight, launch the next, post-process the collected one
    void finishRequest(const std::shared_ptr<GenRequest> &r, const char *reason);
    void failAll(const std::string &what);

    InferenceSession &sess_;
    Tokenizer &tok_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<GenRequest>> queue_;
    std::vector<std::shared_ptr<GenRequest>> active_;
    std::vector<std::shared_ptr<GenRequest>> draining_;  // finished, rows still in the forward in flight
    std::vector<int> freeSlots_;
    // paged KV cache: pages reserved for each slot's request at admission (prompt + max_tokens);
    // returned to the pool through releaseSlot (a RELEASE to every rank) when the slot is freed,
    // see flushReleases; admission needs enough unreserved pages
    int pagesTotal_ = -1, pageSize_ = 0;
    std::vector<int> slotPages_;
    std::vector<int> releasing_;  // freed slots whose pages are not released yet (under mu_)
    void returnSlot(int slot);
    void flushReleases();
    Flight flight_;
    bool inflight_ = false;
    bool stop_ = false;
    u64 nextId_ = 1;
    SchedulerStats stats_;
    std::vector<float> logits_;
    std::thread thread_;
};

}  // namespace dl
