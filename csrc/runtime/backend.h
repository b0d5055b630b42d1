// Backend interface shared by the CPU reference backend and the HIP (MI355X) engine.
//
// One Backend instance = one rank's shard of the model. A forward call processes `n` rows;
// every row carries its own token, position and KV slot, so rows of different requests
// (multi-user batching) and rows of one prompt chunk (prefill) can be mixed in one call.
// This replaces the reference's pipes + executor step list (nn-executor.cpp:124-187,
// app.cpp:169-209) with a fixed per-layer schedule.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "../core/model_file.h"
#include "../core/plan.h"

namespace dl {

struct EngineConfig {
    std::string modelPath;          // .m file (ignored when synthetic)
    u32 maxSeqLen = 0;              // clamp of header seqLen (0 = model's)
    u32 maxBatch = 32;              // max rows per forward (reference nBatches, app.cpp:37)
    u32 maxDecode = 0;              // rows of decode-only state (greedy-chain history, fused argmax
                                    // exchange); 0 = maxBatch. The CLI / API set --max-batch here and
                                    // size maxBatch by the (larger) prefill chunk.
    u32 nSlots = 1;                 // independent KV-cache slots (concurrent sequences)
    FloatType bufferType = FloatType::F32;  // activation quantization: Q80 or F32
    FloatType syncType = FloatType::F32;    // CPU tensor-parallel wire format of partial sums:
                                            // F32 (exact, TP=N == TP=1) or Q80 (the reference's
                                            // quantized all-gather, llm.cpp:150, 3.8x fewer bytes)
    int nThreads = 1;               // CPU backend threads
    int gpuIndex = -1;              // HIP device ordinal (-1 = CPU backend)
    bool useGraphs = true;          // capture per-batch-size hipGraphs
    bool kvBf16 = true;             // GPU KV cache dtype (bf16 default, f32 when false)
    u32 kvPages = 0;                // GPU paged KV cache: pool pages per layer (0 = contiguous
                                    // nSlots x seqLen, no page table)
    u32 kvPageSize = 256;           // positions per page (power of two, >= 32)
    bool synthetic = false;         // random-init weights of the header's shape (no file)
    ModelHeader syntheticHeader;    // used when synthetic
    u64 seed = 1234;                // synthetic weight seed
    bool batchInvariant = false;    // GPU: every row takes the same kernels and reduction order
                                    // whatever else shares its forward (reproducible serving: a
                                    // request's tokens do not depend on who else is being served)
};

struct ForwardStats {
    double computeMs = 0;
    double syncMs = 0;
    double xchgMs = -1;  // exchange span (GPU: DL_SYNC_MEASURE=2 or separate collectives; CPU: = syncMs); < 0 unmeasured
    u64 sentBytes = 0;
    u64 recvBytes = 0;
};

// Per-row sampling request (reference Sampler::sample, tokenizer.cpp:416-502): temperature 0 =
// greedy, < 0 = row not sampled (prefill rows), otherwise softmax(logits / temperature) then a
// multinomial draw (topp <= 0 or >= 1) or nucleus (top-p) draw with the given coin in [0, 1).
struct SampleSpec {
    float temperature = 0.f;
    float topp = 0.f;
    float coin = 0.f;
    float pad = 0.f;
};

// Host implementation of one row's draw (the CPU path and the reference for the device sampler).
int sampleHost(float *logits, int vocab, const SampleSpec &s);

class Backend {
  public:
    virtual ~Backend() = default;
    virtual const ModelHeader &header() const = 0;
    virtual const ShardPlan &plan() const = 0;
    // logits (root only, may be null): [n][vocabSize] full vocabulary.
    virtual void forward(int n, const int *tokens, const int *positions, const int *slots, float *logits) = 0;
    // Greedy decode helper: out[i] = argmax over the full vocabulary (every rank gets it).
    virtual void forwardArgmax(int n, const int *tokens, const int *positions, const int *slots, int *out) = 0;
    // Forward + per-row sampling: out[i] = the sampled token (-1 for rows with temperature < 0).
    // Default: full logits to the root, host draw, ids shared through forwardArgmax's channel.
    virtual void forwardSample(int n, const int *tokens, const int *positions, const int *slots,
                               const SampleSpec *specs, int *out);
    // Pipelined serving (scheduler.cpp): launchIds enqueues a forward whose result is one token id
    // per row (argmax when specs is null, else per-row sampling) and may return before it ran;
    // collectIds waits for it and writes the ids. At most one launch is outstanding. The default
    // runs the forward synchronously inside launchIds (host backends: no overlap).
    virtual void launchIds(int n, const int *tokens, const int *positions, const int *slots, const SampleSpec *specs);
    virtual void collectIds(int *out);
    // Chained greedy decode of one sequence (GPU engines; dllama inference): each step's input
    // token is the previous step's argmax, fed back on the device, so step k + 1 is enqueued
    // before the host has read step k (the host decodes and prints while the device runs).
    // chainLaunch: token >= 0 starts a chain at (token, pos, slot); token < 0 enqueues the next
    // step, at position pos. chainCollect waits for the oldest step in flight and returns its id.
    virtual bool chainSupported() const { return false; }
    virtual void chainLaunch(int token, int pos, int slot);
    virtual int chainCollect();
    virtual int chainInFlight() const { return 0; }
    virtual ForwardStats lastStats() const { return stats_; }
    // Weight residency: time to load (file read + repack + upload, or on-device init), bytes read
    // from the model file by this rank, bytes resident on its device (0 for host backends).
    struct LoadStats {
        double ms = 0;
        u64 fileBytes = 0, deviceBytes = 0;
    };
    virtual LoadStats loadStats() const { return {}; }
    // Paged KV cache (GPU, EngineConfig::kvPages > 0): free pages of the pool and positions per page
    // (the scheduler admits requests by pages); -1 / 0 when the cache is contiguous per slot.
    virtual int kvPagesFree() const { return -1; }
    virtual int kvPageSize() const { return 0; }
    // The sequence in this slot ended: a paged cache returns its pages to the pool (no-op otherwise).
    virtual void releaseSlot(int slot) { (void)slot; }
    virtual std::string name() const = 0;

  protected:
    ForwardStats stats_;
    std::vector<int> pendingIds_;  // default launchIds / collectIds
};

// Host data plane used by the CPU backend for tensor parallelism.
class HostComm {
  public:
    virtual ~HostComm() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    virtual void allReduceSum(float *data, u64 n) = 0;
    // Reference semantics of SYNC_NODE_SLICES with Q80 buffers (nn-network.cpp:537-569,
    // llm.cpp:212-217): every rank's partial is quantized to Q80 once, every rank receives all
    // ranks' quantized partials and sums them dequantized in rank order (identical on all ranks).
    virtual void allReduceSumQ80(float *data, u64 n) { allReduceSum(data, n); }
    // every rank contributes nLocal floats; root receives size()*nLocal floats in rank order
    virtual void gatherToRoot(const float *local, u64 nLocal, float *out) = 0;
    virtual void stats(u64 &sent, u64 &recv) const {
        sent = 0;
        recv = 0;
    }
};

class LocalComm : public HostComm {
  public:
    int rank() const override { return 0; }
    int size() const override { return 1; }
    void allReduceSum(float *, u64) override {}
    void gatherToRoot(const float *local, u64 nLocal, float *out) override;
};

// `world` ranks of one process (threads) exchanging through shared memory with exactly the TCP
// data plane's arithmetic (f32 sum in rank order; Q80: every partial quantized once, dequantized
// sums in rank order). Used to pin the GPU tensor-parallel paths against the CPU reference in
// tests without sockets.
class ThreadGroupComm : public HostComm {
  public:
    struct Group;
    static std::vector<std::unique_ptr<ThreadGroupComm>> make(int world);
    int rank() const override { return rank_; }
    int size() const override;
    void allReduceSum(float *data, u64 n) override;
    void allReduceSumQ80(float *data, u64 n) override;
    void gatherToRoot(const float *local, u64 nLocal, float *out) override;

  private:
    ThreadGroupComm(std::shared_ptr<Group> g, int rank) : g_(std::move(g)), rank_(rank) {}
    std::shared_ptr<Group> g_;
    int rank_;
    std::vector<float> tmp_;
};

std::unique_ptr<Backend> makeCpuBackend(const EngineConfig &cfg, HostComm *comm);

}  // namespace dl
