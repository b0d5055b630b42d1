// MI355X engine: one rank's shard resident in HBM, fused per-layer kernel schedule captured into
// one hipGraph per batch size (replaces the reference's per-op executor + barrier).
#pragma once

#include <memory>
#include <vector>

#include "../runtime/backend.h"
#include "device_comm.h"

namespace dl {

class HipEngine : public Backend {
  public:
    virtual ~HipEngine() = default;
    // Greedy decode of `steps` tokens for one sequence entirely on device: the token produced by
    // step i is fed to step i+1 without a host round trip (graph replay back to back).
    // Writes the generated ids to `outTokens` (may be null). Returns device wall ms.
    virtual double decodeGreedy(int steps, int token, int pos, int slot, int *outTokens) = 0;
    // Same, for `nSeq` independent sequences decoded together (multi-user batch).
    virtual double decodeGreedyBatch(int steps, int nSeq, const int *tokens, const int *pos, const int *slots,
                                     int *outTokens) = 0;
    virtual void synchronize() = 0;
    virtual size_t deviceBytes() const = 0;
    // Run one forward eagerly with a per-kernel-class timing breakdown (ms) printed to stdout.
    virtual void profileForward(int n, const int *tokens, const int *positions, const int *slots) = 0;
    // Tensor parallel: whether the partial-sum exchange runs fused in the wo / w2 GEMV tails (it is
    // switched off when a launch's grid would not be fully co-resident), and the largest grid of
    // such a launch (checked against the device's occupancy at construction).
    virtual bool tpFused() const { return false; }
    // Single decode rows run the fused attention block (qkv + attention + wo in one launch).
    virtual bool attnBlock() const { return false; }
    virtual bool woAttn() const { return false; }  // DL_WO_ATTN: the wo GEMV with the attention prologue
    virtual bool ffnBlock() const { return false; } // fused w13 + w2 launch in the pre-normalized layers
    virtual bool prenorm() const { return false; } // pre-normalized Q80 hand-offs of single decode rows
    // Diagnostics: one eager single-row forward with the fused attention block of `layer` traced
    // (kernels.h AttnBlockArgs::trace, 8 u64 per workgroup); returns {gq, ga, gw, trace...}.
    virtual std::vector<unsigned long long> traceAttnBlock(int token, int pos, int slot, int layer) {
        (void)token, (void)pos, (void)slot, (void)layer;
        return {};
    }
    virtual int fusedGridMax() const { return 0; }
    // Tensor parallel: a batched forward of n rows all-reduces its wo / w2 tiles inside the GEMM
    // epilogues (no separate all-reduce / norm kernels).
    virtual bool tpBatchedFused(int n) const {
        (void)n;
        return false;
    }
};

// comm may be null (single GPU). The engine does not own comm.
std::unique_ptr<HipEngine> makeHipEngine(const EngineConfig &cfg, DeviceComm *comm);
int hipDeviceCount();

// Micro-benchmark of one Q40 GEMV configuration: `copies` weight matrices (to defeat the 256 MB
// infinity cache) are cycled through a graph of `iters` launches. Returns microseconds per launch.
// trace: per launch x workgroup 8 u64 (GemvArgs::trace layout; s_memrealtime, 100 MHz)
double benchGemvQ40(int rows, int n, int pro, int epi, int B, int lanes, int passes, int copies, int iters,
                    std::vector<unsigned long long> *trace = nullptr);
// Micro-benchmark of the batched MFMA GEMM (M tokens, epilogue epi: EPI_STORE or EPI_ACT_F16),
// `copies` weight matrices cycled through a graph of `iters` launches. Returns us per launch.
// trace: one extra launch with per-workgroup stamps (gemm_dev.h gemmTrace layout, 8 u64 per
// workgroup, grid x then splits) appended after the timed graph.
double benchGemmQ40(int rows, int n, int M, int epi, int copies, int iters,
                    std::vector<unsigned long long> *trace = nullptr);
// Micro-benchmark of the decode attention kernel (bf16 or f32 KV, Q80 output): `copies` KV caches
// cycled through a graph of `iters` launches, every row at position `pos`. Returns microseconds per
// launch.
double benchAttention(int nHeads0, int kvMul, int hs, int seqLen, int pos, int B, int copies, int iters,
                      std::vector<unsigned long long> *trace = nullptr, bool kvBf16 = true);
// Check a transport on the engine's separate-collective schedule (per layer Q80-rounded
// all-reduces, root gather of logits slices, all-gather of argmax pairs), eagerly or captured in a
// hipGraph and replayed `runs` times: returns the largest error against exact host sums (engine_bench.cpp).
double commScheduleCheck(DeviceComm &comm, int layers, int rows, int dim, int vocab0, int runs, bool graph);

}  // namespace dl

namespace dl {
// Test helper: `world` tensor-parallel ranks simulated on one GPU (host-staged collectives).
// Returns rank 0's logits for single-token forwards of `tokens` at positions 0.., [n][vocab].
// attnBlocks (optional): per rank, whether its single decode rows run the fused attention block.
std::vector<float> simulateTensorParallel(const EngineConfig &cfg, int world, const std::vector<int> &tokens,
                                          std::vector<int> *attnBlocks = nullptr);
}  // namespace dl
