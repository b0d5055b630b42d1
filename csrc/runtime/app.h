// Application runtime shared by `dllama` and `dllama-api`.
//
// CLI parity with the reference (src/app.cpp:33-136; flag table SURVEY §5.6): every reference
// flag is accepted with the same name and default; MI355X additions: --tp-gpus / --max-batch /
// --slots / --kv-dtype / --graph / --log-level / --synthetic / --metrics / --profile.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "../net/tcp.h"
#include "../text/tokenizer.h"
#include "backend.h"

namespace dl {

struct AppArgs {
    bool help = false;
    std::string mode;
    std::string modelPath, tokenizerPath, prompt;
    FloatType bufferType = FloatType::F32;
    // --sync-type: tensor-parallel wire format of the partial sums (f32 exact | q80). Unset = the
    // buffer float type, as in the reference (syncType = bufferFloatType, src/app.cpp:81, llm.cpp:150)
    FloatType syncType = FloatType::UNK;
    std::vector<std::string> workerHosts;
    std::vector<int> workerPorts;
    int port = 9990;
    int nThreads = 1;
    int nBatches = 32;  // max decode rows per forward (reference constant, now --max-batch)
    // --prefill-chunk: prompt rows per forward (0 = 1024 on GPUs, where one wide-GEMM launch covers
    // every 128-token tile of a chunk, and --max-batch on the CPU backend)
    int prefillChunk = 0;
    int steps = 0;
    float temperature = 0.8f;
    float topp = 0.9f;
    u64 seed = 0;
    ChatTemplateType chatTemplate = ChatTemplateType::UNKNOWN;
    u32 maxSeqLen = 0;
    bool netTurbo = true;
    int gpuIndex = -1;
    int gpuSegmentFrom = -1, gpuSegmentTo = -1;  // accepted for CLI compatibility (no effect)
    int slots = 0;                               // KV slots (0 = 1 for CLI modes, 8 for the API)
    bool kvBf16 = false;  // --kv-dtype: f32 by default (the reference's KV precision, llm.cpp:197-198)
    int kvPages = 0;       // --kv-pages: paged KV pool pages per layer (0 = contiguous per slot)
    bool batchInvariant = false;  // --batch-invariant 1: rows take the same kernels whatever the batch
    int kvPageSize = 256;  // --kv-page-size: positions per page
    bool graphs = true;
    int logLevel = 1;
    std::string synthetic;                       // "llama3_1_8b" etc: random-init weights on device
    std::string webUi;                           // dllama-api: directory served at GET /
    bool streamWeights = false;                  // worker: always fetch slices from the root
    std::string weightsCache = "/tmp";           // worker: directory for streamed weight files
    std::string metricsPath;                     // --metrics: JSON-lines sink ("-" = stderr)
    bool profile = false;                        // --profile 1: per-kernel-class table (GPU, eager)

    static AppArgs parse(int argc, char **argv, bool requireMode);
};


// Root-side inference: local backend + (optional) remote workers in lockstep.
class InferenceSession {
  public:
    explicit InferenceSession(const AppArgs &args, int nSlots);
    ~InferenceSession();

    const ModelHeader &header() const { return backend_->header(); }
    Tokenizer &tokenizer() { return *tokenizer_; }
    Sampler &sampler() { return *sampler_; }
    int nSlots() const { return nSlots_; }
    int maxBatch() const { return maxBatch_; }          // decode rows per forward
    int prefillChunk() const { return prefillChunk_; }  // prompt rows per forward (engine rows >= both)
    // paged KV cache of the (root) backend: free pages and positions per page (-1 / 0: contiguous)
    int kvPagesFree() const { return backend_->kvPagesFree(); }
    // a sequence ended: its KV slot's pages return to the pool on every rank (no-op when contiguous)
    void releaseSlot(int slot);
    int kvPageSize() const { return backend_->kvPageSize(); }
    bool isGpu() const { return gpu_; }
    int nNodes() const { return 1 + (int)workers_.size(); }

    // logits: [n][vocab]
    void forward(int n, const int *tokens, const int *positions, const int *slots, float *logits);
    void forwardArgmax(int n, const int *tokens, const int *positions, const int *slots, int *out);
    // per-row sampling on the backend (device sampler on GPUs: only token ids leave the device)
    void forwardSample(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs,
                       int *out);
    // Pipelined serving (Backend::launchIds / collectIds; workers run the forward in lockstep).
    void launchIds(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs);
    void collectIds(int n, int *out);
    // Chained greedy decode of one sequence (Backend::chainLaunch; workers follow each step).
    bool chainSupported() const { return backend_->chainSupported(); }
    void chainLaunch(int token, int pos, int slot);
    int chainCollect();
    ForwardStats lastStats();
    void finish();  // stop workers (they return to listening)
    // GPU only: one eager forward of these rows with a per-kernel-class device-time table.
    bool profileForward(int n, const int *tokens, const int *positions, const int *slots);

  private:
    void sendControl(Cmd cmd, int n, const int *tokens, const int *positions, const int *slots);
    void recordMetrics(const char *kind, int n, double ms);

    AppArgs args_;
    int nSlots_, maxBatch_, prefillChunk_ = 32;
    bool gpu_ = false;
    std::vector<Socket> workers_;
    std::unique_ptr<HostComm> hostComm_;
    std::unique_ptr<class DeviceComm> devComm_;
    std::unique_ptr<Backend> backend_;
    std::unique_ptr<Tokenizer> tokenizer_;
    std::unique_ptr<Sampler> sampler_;
    bool finished_ = false;
    unsigned long long mSent_ = 0, mRecv_ = 0;  // control-plane bytes at the previous metrics record
    Timer launchTimer_;                          // launchIds -> collectIds (metrics)
    bool launchedSample_ = false;
};

// `dllama worker`: serve forever; a root disconnect returns to listening.
void runWorker(const AppArgs &args);

// Builds the synthetic header for a named shape (see --synthetic).
ModelHeader syntheticHeader(const std::string &name, u32 seqLen);

}  // namespace dl
