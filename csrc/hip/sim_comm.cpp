// Test-only DeviceComm: N tensor-parallel ranks simulated as N threads/engines on ONE GPU,
// exchanging partial sums through host memory. Used to validate the multi-rank engine logic
// (shard plan, per-layer all-reduce placement, logits all-gather + unshard) on hardware where
// only one GPU is available. The production data planes are the one-shot xGMI collectives and the
// exchange fused into the wo / w2 kernels (xgmi_comm.cpp, decode_common.h), with RCCL
// (rccl_comm.cpp) as the fallback when their self-test fails.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../core/common.h"
#include "device_comm.h"
#include "engine.h"
#include "kernels.h"

namespace dl {

namespace {

class Barrier {
  public:
    explicit Barrier(int n) : n_(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        const long gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            gen_++;
            cv_.notify_all();
        } else {
            cv_.wait(lk, [&] { return gen_ != gen; });
        }
    }

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    int n_, count_ = 0;
    long gen_ = 0;
};

struct SimShared {
    explicit SimShared(int n) : world(n), barrier(n), slots(n) {}
    int world;
    Barrier barrier;
    std::vector<std::vector<float>> slots;
};

class SimComm : public DeviceComm {
  public:
    SimComm(SimShared *sh, int rank) : sh_(sh), rank_(rank) {}
    int rank() const override { return rank_; }
    int size() const override { return sh_->world; }
    std::string name() const override { return "sim"; }
    void allReduceSum(float *buf, size_t n, hipStream_t s) override {
        stage(buf, n, s);
        std::vector<float> sum(n, 0.f);
        for (int r = 0; r < sh_->world; r++)  // same summation order on every rank
            for (size_t i = 0; i < n; i++) sum[i] += sh_->slots[r][i];
        sh_->barrier.wait();
        if (hipMemcpy(buf, sum.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) throw Error("sim memcpy");
    }
    void allGather(const float *send, float *recv, size_t nPerRank, hipStream_t s) override {
        stage(send, nPerRank, s);
        for (int r = 0; r < sh_->world; r++)
            if (hipMemcpy(recv + (size_t)r * nPerRank, sh_->slots[r].data(), nPerRank * 4, hipMemcpyHostToDevice) !=
                hipSuccess)
                throw Error("sim memcpy");
        sh_->barrier.wait();
    }
    void broadcastInts(int *, size_t, int, hipStream_t) override { throw Error("not supported by SimComm"); }

  private:
    void stage(const float *buf, size_t n, hipStream_t s) {
        if (hipStreamSynchronize(s) != hipSuccess) throw Error("sim sync");
        sh_->slots[rank_].resize(n);
        if (hipMemcpy(sh_->slots[rank_].data(), buf, n * 4, hipMemcpyDeviceToHost) != hipSuccess)
            throw Error("sim memcpy");
        sh_->barrier.wait();
    }
    SimShared *sh_;
    int rank_;
};

// Compute-only rank (device_comm.h makeComputeOnlyComm): the shard shapes and kernels of rank
// `rank` of `world`, nothing exchanged. The fused exchange keeps its local work (Q80 quantize,
// rank-order sum, epochs) with every peer's words read as zeros; the separate collectives are
// no-ops except that an all-gather places this rank's own slice and fills the peers' with -inf
// (gathered logits / argmax winners: a peer never wins over this shard's own maximum).
class ComputeOnlyComm : public DeviceComm {
  public:
    ComputeOnlyComm(int rank, int world) : rank_(rank), world_(world) {
        if (world < 2 || world > hipk::kTpMaxRanks || rank < 0 || rank >= world)
            throw Error("compute-only comm: bad rank / world");
        DL_HIP(hipMalloc(&epochs_, (kVec + kArg) * sizeof(unsigned)));
        DL_HIP(hipMemset(epochs_, 0, (kVec + kArg) * sizeof(unsigned)));
        DL_HIP(hipMalloc(&error_, sizeof(int)));
        DL_HIP(hipMemset(error_, 0, sizeof(int)));
    }
    ~ComputeOnlyComm() override {
        (void)hipFree(epochs_);
        (void)hipFree(error_);
    }
    int rank() const override { return rank_; }
    int size() const override { return world_; }
    std::string name() const override { return "compute-only"; }
    bool computeOnly() const override { return true; }
    const int *deviceErrorFlag() const override { return error_; }
    void resetError() override { DL_HIP(hipMemset(error_, 0, sizeof(int))); }
    void allReduceSum(float *, size_t, hipStream_t) override {}
    void allGather(const float *send, float *recv, size_t nPerRank, hipStream_t s) override {
        for (int p = 0; p < world_; p++)
            if (p != rank_) hipk::launchFillF32Const(recv + (size_t)p * nPerRank, nPerRank, -INFINITY, s);
        DL_HIP(hipMemcpyAsync(recv + (size_t)rank_ * nPerRank, send, nPerRank * sizeof(float),
                              hipMemcpyDeviceToDevice, s));
    }
    void broadcastInts(int *, size_t, int, hipStream_t) override {}
    bool fusedXchg(int region, hipk::TpXchg *x) const override {
        *x = hipk::TpXchg{};
        x->epochs = region == 0 ? epochs_ : epochs_ + kVec;
        x->error = error_;
        x->stride = region == 0 ? kVec : kArg;
        x->timeoutTicks = 1;
        x->rank = rank_;
        x->world = world_;
        x->loopback = 1;
        return true;
    }

  private:
    static constexpr long long kVec = 1 << 18, kArg = 2048;  // the xGMI comm's fused regions
    int rank_, world_;
    unsigned *epochs_ = nullptr;
    int *error_ = nullptr;
};

}  // namespace

std::unique_ptr<DeviceComm> makeComputeOnlyComm(int rank, int world) {
    return std::unique_ptr<DeviceComm>(new ComputeOnlyComm(rank, world));
}

// Runs `steps` single-token forwards (token i at position i) on `world` simulated ranks and
// returns rank 0's logits, [steps][vocab].
std::vector<float> simulateTensorParallel(const EngineConfig &cfg0, int world, const std::vector<int> &tokens,
                                          std::vector<int> *attnBlocks) {
    SimShared sh(world);
    std::vector<std::unique_ptr<SimComm>> comms;
    std::vector<std::unique_ptr<HipEngine>> engines;
    EngineConfig cfg = cfg0;
    cfg.useGraphs = false;  // host-staged collectives cannot be captured
    for (int r = 0; r < world; r++) {
        comms.emplace_back(new SimComm(&sh, r));
        engines.push_back(makeHipEngine(cfg, comms.back().get()));
    }
    if (attnBlocks)
        for (auto &e : engines) attnBlocks->push_back(e->attnBlock() ? 1 : 0);
    const u32 vocab = engines[0]->header().vocabSize;
    std::vector<float> out((size_t)tokens.size() * vocab);
    std::vector<std::thread> th;
    std::vector<std::string> errors(world);
    for (int r = 0; r < world; r++) {
        th.emplace_back([&, r] {
            try {
                (void)hipSetDevice(cfg.gpuIndex >= 0 ? cfg.gpuIndex : 0);
                std::vector<float> lg(vocab);
                for (size_t i = 0; i < tokens.size(); i++) {
                    const int t = tokens[i], p = (int)i, s = 0;
                    engines[r]->forward(1, &t, &p, &s, r == 0 ? lg.data() : nullptr);
                    if (r == 0) std::memcpy(&out[i * vocab], lg.data(), vocab * 4);
                }
            } catch (const std::exception &e) {
                errors[r] = e.what();
            }
        });
    }
    for (auto &t : th) t.join();
    for (auto &e : errors)
        if (!e.empty()) throw Error("simulated TP rank failed: " + e);
    return out;
}

}  // namespace dl
