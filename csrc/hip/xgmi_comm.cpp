// One-shot all-reduce / all-gather over xGMI peer-to-peer, for the small per-layer tensor-parallel
// exchanges of decode (16 KB per all-reduce at batch 1 for an 8B model).
//
// Replaces both the reference's star all-gather over TCP (nn-network.cpp:537-569) and, on the
// hot path, RCCL's ring/LL collectives: for a few KB the cost is latency, so every rank publishes
// its vector once in its own HBM and every rank reads all peers' copies directly over xGMI
// (one hop, all links in parallel) and reduces them locally in rank order, so the results are
// bitwise identical on all ranks.
//
// Buffers (one hipMalloc per rank, shared with peers through IPC handles):
//   pub[2][maxFloats]   published vectors, double-buffered by epoch parity
//   flags[W][kSlots]    flags[p][g] = last epoch rank p published for slot g (written remotely)
//   epochs[kSlots]      local epoch per slot
//   error               set when a wait timed out
// Small all-reduces (<= kLLMax floats, i.e. every decode-time residual update) use a second,
// lower-latency protocol instead ("LL", after the low-latency protocol of NCCL/RCCL): every rank
// PUSHES its chunk straight into each peer's receive buffer as 8-byte words {float bits, epoch}
// and each rank polls its OWN buffer until every word carries the current epoch, then sums the
// ranks' values in rank order. Data and flag travel in the same atomic 8-byte store, so there is
// no release fence, no separate flag store and no remote read: one one-way xGMI trip per call
// (the pull protocol below needs a flag trip and a remote read round trip, no fence). Receive
// buffers alternate by epoch parity per chunk; a rank can only write epoch e+2 into a peer's
// buffer after finishing call e+1, which needed that peer's e+1 data, which the peer only sends
// after it finished reading epoch e.
// Memory: the whole shared region is allocated UNCACHED (hipDeviceMallocUncached): every flag poll,
// LL word poll and remote read goes to HBM instead of a cache line that a peer's xGMI write does
// not invalidate (a plain coarse-grained hipMalloc would let a local L2 line go stale while the
// peer writes the HBM copy). Writers use system-scope atomic stores, readers system-scope atomic
// loads, so neither side depends on cache maintenance.
// Fused-exchange regions (TpXchg in kernels.h): producer kernels (wo / w2 GEMV tails, argmax)
// push their partials straight into these, so TP decode needs no separate all-reduce kernel.
// Elements are owned by fixed slots: chunk c (kChunk floats) belongs to slot c % kSlots, for
// every message size, so a slot only ever races with the same slot on other ranks. Protocol per
// call and slot (workgroup g): e = ++epochs[g]; write my chunks to pub[e&1]; release (system);
// store e into every peer's flags[me][g]; wait until my flags[p][g] >= e for all peers; acquire;
// read the chunks from every rank's pub[e&1]. A rank can only reuse pub[e&1] at epoch e+2 after
// every peer published e+1 for that slot, i.e. after they finished reading epoch e.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../core/common.h"
#include "device_comm.h"
#include "kernels.h"

namespace dl {

namespace {

constexpr int kSlots = 64;          // workgroups per call (max)
constexpr int kChunk = 1024;        // floats per chunk (256 threads x float4)
constexpr int kMaxRanks = 16;
constexpr int kThreads = 256;
constexpr int kLLMax = 16384;       // largest LL all-reduce (floats per rank)
constexpr int kLLSlots = kLLMax / kChunk;
// fused residual exchange: words per (parity, sender); decode rows use <= 4 x dim, the batched
// GEMMs' exchange (gemm_dev.h tpExchangeTile) up to 64 tokens x dim of the 8B
constexpr long long kFusedVec = 1 << 18;
constexpr long long kFusedArg = 2048;      // fused argmax exchange: 2 words per batch row
constexpr long long kTimeoutTicks = 200LL * 1000 * 1000;  // 2 s at 100 MHz
// ranks sharing one GPU (rehearsals, tests) time-share its CUs: a rank spinning in a collective
// can hold off its peer's kernels for seconds (seen: 2-4 s around wide prefill launches), so
// their waits give up after 20 s instead
constexpr long long kSharedTimeoutTicks = 2000LL * 1000 * 1000;

struct XgmiPeers {
    float *pub[kMaxRanks];          // each rank's pub base (pub[p] + parity * maxFloats)
    int *flags[kMaxRanks];          // each rank's flags base: [W][kSlots]
    uint64_t *ll[kMaxRanks];        // each rank's LL receive buffer: [2 parities][kMaxRanks senders][kLLMax]
};

struct XgmiCall {
    XgmiPeers peers;
    int *epochs;                    // local
    int *error;                     // local
    const float *in;                // local input (n floats)
    float *out;                     // local output (n floats for reduce, W*n for gather)
    long long maxFloats;
    long long n;
    int rank, world, gather;        // gather: 0 all-reduce, 1 all-gather, 2 gather to rank 0
    int fenced;                     // system-scope release / acquire fences around the flags
    long long timeoutTicks;         // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ long long rtClock() { return (long long)__builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(kThreads) void xgmiKernel(XgmiCall a) {
    const int g = blockIdx.x, tid = threadIdx.x;
    const long long nChunks = (a.n + kChunk - 1) / kChunk;
    if (g >= nChunks) return;  // no chunk for this slot at this size (same on every rank)
    __shared__ int sEpoch;
    if (tid == 0) sEpoch = a.epochs[g] + 1;
    __syncthreads();
    const int e = sEpoch, q = e & 1;
    float *myPub = a.peers.pub[a.rank] + (long long)q * a.maxFloats;
    // Published data is written and read with system-scope atomic accesses (performed at the
    // memory side, never served from a cached line), so no fence is needed around the flags: a
    // system-scope release / acquire fence is a whole-L2 writeback / invalidate on gfx950.
    auto pst = [](float *p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    auto pld = [](const float *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    // 1. publish my chunks
    for (long long c = g; c < nChunks; c += kSlots) {
        const long long i = c * kChunk + tid * 4;
        if (i + 3 < a.n) {
            const float4 v = *reinterpret_cast<const float4 *>(a.in + i);
            pst(myPub + i, v.x);
            pst(myPub + i + 1, v.y);
            pst(myPub + i + 2, v.z);
            pst(myPub + i + 3, v.w);
        } else {
            for (long long k = i; k < a.n; k++) pst(myPub + k, a.in[k]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every publish store performed
    // ranks on different GPUs: a system-scope release before the flag store as well (not needed
    // for the uncached, atomically accessed buffers on paper; kept until the fence-free protocol
    // has been validated across separate devices - see fencedDefault())
    if (a.fenced) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    // 2. signal every peer, then wait for every peer's signal (one lane per peer)
    if (tid < a.world) {
        if (tid != a.rank) {
            int *remote = a.peers.flags[tid] + a.rank * kSlots + g;
            __hip_atomic_store(remote, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            int *local = a.peers.flags[a.rank] + tid * kSlots + g;
            const long long t0 = rtClock();
            // after a first timeout every later call fails fast instead of waiting again
            const bool failed = __hip_atomic_load(a.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
            while (!failed && __hip_atomic_load(local, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
                __builtin_amdgcn_s_sleep(1);
                if (rtClock() - t0 > a.timeoutTicks) {  // a peer never arrived: give up, flag it
                    __hip_atomic_store(a.error, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
        }
    }
    __syncthreads();
    if (a.fenced) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    // 3. reduce (rank order, identical on every rank) or gather (gather to rank 0: the other
    //    ranks only publish and take part in the flag protocol, which keeps the double buffer safe)
    if (a.gather == 2 && a.rank != 0) {
        if (tid == 0) a.epochs[g] = e;
        return;
    }
    for (long long c = g; c < nChunks; c += kSlots) {
        const long long i = c * kChunk + tid * 4;
        const long long cnt = i + 3 < a.n ? 4 : (i < a.n ? a.n - i : 0);
        if (cnt <= 0) continue;
        if (!a.gather) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            if (cnt == 4) {
                float4 v[kMaxRanks];  // all peers' loads in flight at once
#pragma unroll
                for (int p = 0; p < kMaxRanks; p++)
                    if (p < a.world) {
                        const float *src = a.peers.pub[p] + (long long)q * a.maxFloats + i;
                        v[p] = make_float4(pld(src), pld(src + 1), pld(src + 2), pld(src + 3));
                    }
#pragma unroll
                for (int p = 0; p < kMaxRanks; p++)
                    if (p < a.world) {
                        acc.x += v[p].x;
                        acc.y += v[p].y;
                        acc.z += v[p].z;
                        acc.w += v[p].w;
                    }
                *reinterpret_cast<float4 *>(a.out + i) = acc;
            } else {
                for (long long k = 0; k < cnt; k++) {
                    float s = 0.f;
                    for (int p = 0; p < a.world; p++) s += pld(a.peers.pub[p] + (long long)q * a.maxFloats + i + k);
                    a.out[i + k] = s;
                }
            }
        } else {
            for (int p = 0; p < a.world; p++) {
                const float *src = a.peers.pub[p] + (long long)q * a.maxFloats + i;
                float *dst = a.out + (long long)p * a.n + i;
                for (long long k = 0; k < cnt; k++) dst[k] = pld(src + k);
            }
        }
    }
    if (tid == 0) a.epochs[g] = e;
}

// LL all-reduce (see the header): grid = chunks of kChunk floats, thread = 4 consecutive floats.
// W = world size as a template parameter so every peer loop unrolls with constant indices (peer
// pointers stay in SGPRs, polled words in VGPRs; no scratch).
template <int W>
__global__ __launch_bounds__(kThreads) void xgmiLLKernel(XgmiCall a, unsigned *llEpochs) {
    const int g = blockIdx.x, tid = threadIdx.x, me = a.rank;
    __shared__ unsigned sEpoch;
    if (tid == 0) sEpoch = llEpochs[g] + 1;
    __syncthreads();
    const unsigned e = sEpoch, q = e & 1;
    const long long i0 = (long long)g * kChunk + tid * 4;
    const int cnt = a.n - i0 >= 4 ? 4 : (a.n > i0 ? (int)(a.n - i0) : 0);
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = k < cnt ? a.in[i0 + k] : 0.f;
    // 1. push my values to every peer: {float bits, epoch} in one 8-byte store
#pragma unroll
    for (int p = 0; p < W; p++) {
        if (p == me) continue;
        uint64_t *dst = a.peers.ll[p] + ((size_t)q * kMaxRanks + me) * kLLMax + i0;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < cnt)
                __hip_atomic_store(dst + k, (uint64_t)__float_as_uint(v[k]) | ((uint64_t)e << 32), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // 2. sum every rank's values in rank order (bitwise identical on all ranks); my own are in v.
    //    All peers' words are loaded first (independent loads in flight together); only words that
    //    had not arrived yet are polled again.
    const uint64_t *mine = a.peers.ll[me] + (size_t)q * kMaxRanks * kLLMax + i0;
    uint64_t w[W][4];
#pragma unroll
    for (int p = 0; p < W; p++)
#pragma unroll
        for (int k = 0; k < 4; k++)
            w[p][k] = (p != me && k < cnt)
                          ? __hip_atomic_load(mine + (size_t)p * kLLMax + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                          : ((uint64_t)e << 32);
    const bool failed = __hip_atomic_load(a.error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < W; p++) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint64_t x = w[p][k];
            if ((unsigned)(x >> 32) != e && !failed) {
                const long long t0 = rtClock();
                while ((unsigned)(x >> 32) != e) {
                    __builtin_amdgcn_s_sleep(1);
                    x = __hip_atomic_load(mine + (size_t)p * kLLMax + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (rtClock() - t0 > a.timeoutTicks) {  // a peer never arrived: flag it, stop waiting
                        __hip_atomic_store(a.error, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                }
            }
            acc[k] += p == me ? v[k] : __uint_as_float((unsigned)x);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (k < cnt) a.out[i0 + k] = acc[k];
    __syncthreads();
    if (tid == 0) llEpochs[g] = e;
}

class XgmiComm : public DeviceComm {
  public:
    XgmiComm(int rank, int world, size_t maxFloats) : rank_(rank), world_(world), maxFloats_(maxFloats) {
        DL_CHECK(world >= 1 && world <= kMaxRanks, "xgmi comm: world size must be 1..16");
        DL_CHECK(rank >= 0 && rank < world, "xgmi comm: bad rank");
        maxFloats_ = (maxFloats_ + kChunk - 1) / kChunk * kChunk;
        pubBytes_ = 2 * maxFloats_ * sizeof(float);
        flagsBytes_ = (size_t)kMaxRanks * kSlots * sizeof(int);
        llOff_ = (pubBytes_ + flagsBytes_ + kSlots * sizeof(int) + 64 + 255) / 256 * 256;
        const size_t llBytes = (size_t)2 * kMaxRanks * kLLMax * sizeof(uint64_t);
        fvOff_ = (llOff_ + llBytes + kLLSlots * sizeof(unsigned) + 255) / 256 * 256;
        faOff_ = fvOff_ + (size_t)2 * world * kFusedVec * sizeof(uint64_t);
        const size_t total = faOff_ + (size_t)2 * world * kFusedArg * sizeof(uint64_t);
        DL_HIP(hipExtMallocWithFlags(&base_, total, hipDeviceMallocUncached));
        DL_HIP(hipMemset(base_, 0, total));
        DL_HIP(hipMalloc(&fusedEpochs_, (kFusedVec + kFusedArg) * sizeof(unsigned)));
        DL_HIP(hipMemset(fusedEpochs_, 0, (kFusedVec + kFusedArg) * sizeof(unsigned)));
        DL_HIP(hipDeviceSynchronize());
        epochs_ = reinterpret_cast<int *>(static_cast<char *>(base_) + pubBytes_ + flagsBytes_);
        error_ = epochs_ + kSlots;
        llEpochs_ = reinterpret_cast<unsigned *>(static_cast<char *>(base_) + llOff_ + llBytes);
        hipIpcMemHandle_t h;
        DL_HIP(hipIpcGetMemHandle(&h, base_));
        handle_.assign(reinterpret_cast<const char *>(&h), reinterpret_cast<const char *>(&h) + sizeof(h));
        // the handle travels with this rank's PCI bus id, so every rank knows whether its peers
        // are other GPUs (cross-device: fenced pull protocol by default) or the same one
        int dev = 0;
        DL_HIP(hipGetDevice(&dev));
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, sizeof(bus) - 1, dev) != hipSuccess) std::snprintf(bus, sizeof(bus), "dev%d", dev);
        busId_ = bus;
        handle_ += busId_;
    }
    ~XgmiComm() override {
        for (int p = 0; p < world_; p++)
            if (p != rank_ && peerBase_[p]) (void)hipIpcCloseMemHandle(peerBase_[p]);
        if (base_) (void)hipFree(base_);
        if (fusedEpochs_) (void)hipFree(fusedEpochs_);
    }
    const std::string &handle() const { return handle_; }
    // handles[p] = rank p's handle() bytes; call on every rank after all ranks were created.
    void connect(const std::vector<std::string> &handles) {
        DL_CHECK((int)handles.size() == world_, "xgmi comm: need one handle per rank");
        for (int p = 0; p < world_; p++) {
            if (p == rank_) {
                peerBase_[p] = base_;
            } else {
                DL_CHECK(handles[p].size() >= sizeof(hipIpcMemHandle_t), "xgmi comm: bad handle size");
                if (handles[p].substr(sizeof(hipIpcMemHandle_t)) != busId_) crossDevice_ = true;
                else sameDevice_++;
                hipIpcMemHandle_t h;
                std::memcpy(&h, handles[p].data(), sizeof(h));
                DL_HIP(hipIpcOpenMemHandle(&peerBase_[p], h, hipIpcMemLazyEnablePeerAccess));
            }
            peers_.pub[p] = static_cast<float *>(peerBase_[p]);
            peers_.flags[p] = reinterpret_cast<int *>(static_cast<char *>(peerBase_[p]) + pubBytes_);
            peers_.ll[p] = reinterpret_cast<uint64_t *>(static_cast<char *>(peerBase_[p]) + llOff_);
            fusedVec_[p] = reinterpret_cast<uint64_t *>(static_cast<char *>(peerBase_[p]) + fvOff_);
            fusedArg_[p] = reinterpret_cast<uint64_t *>(static_cast<char *>(peerBase_[p]) + faOff_);
        }
        connected_ = true;
        fenced_ = crossDevice_ && fencedDefault();
    }
    bool crossDevice() const { return crossDevice_; }
    int ranksOnDevice() const override { return sameDevice_; }
    bool fenced() const { return fenced_; }
    int rank() const override { return rank_; }
    int size() const override { return world_; }
    std::string name() const override { return "xgmi"; }
    void allReduceSum(float *buf, size_t n, hipStream_t s) override {
        if (ll_ && n <= (size_t)kLLMax && !pullOnly() && (world_ == 2 || world_ == 4 || world_ == 8))
            launchLL(buf, n, s);
        else
            launch(buf, buf, n, 0, s);
    }
    void allGather(const float *send, float *recv, size_t nPerRank, hipStream_t s) override {
        launch(send, recv, nPerRank, 1, s);
    }
    void gatherToRoot(const float *send, float *recv, size_t nPerRank, hipStream_t s) override {
        launch(send, recv, nPerRank, 2, s);
    }
    void broadcastInts(int *, size_t, int, hipStream_t) override {
        throw Error("xgmi comm: broadcastInts is not used on the device data plane");
    }
    const int *deviceErrorFlag() const override { return error_; }
    bool fusedXchg(int region, hipk::TpXchg *x) const override {
        if (!connected_ || world_ < 2) return false;
        *x = hipk::TpXchg{};
        for (int p = 0; p < world_; p++) x->recv[p] = region == 0 ? fusedVec_[p] : fusedArg_[p];
        x->epochs = region == 0 ? fusedEpochs_ : fusedEpochs_ + kFusedVec;
        x->error = error_;
        x->stride = region == 0 ? kFusedVec : kFusedArg;
        x->timeoutTicks = timeoutTicks();
        x->rank = rank_;
        x->world = world_;
        return true;
    }
    // The LL protocol can be switched off (e.g. when its pre-flight test fails on a platform);
    // resetError clears a timed-out flag so the other protocol can be tested.
    void setLowLatency(bool on) { ll_ = on; }
    void resetError() override {
        DL_HIP(hipMemset(error_, 0, sizeof(int)));
        DL_HIP(hipDeviceSynchronize());
    }
    bool timedOut() {
        int v = 0;
        DL_HIP(hipMemcpy(&v, error_, sizeof(int), hipMemcpyDeviceToHost));
        return v != 0;
    }

  private:
    // DL_XGMI_FENCE=0 runs the pull protocol fence-free across devices too (as on one device);
    // =1 fences even on one device (comparison runs).
    static bool fencedDefault() {
        const char *e = std::getenv("DL_XGMI_FENCE");
        return !(e && *e == '0');
    }
    long long timeoutTicks() const { return sameDevice_ > 1 ? kSharedTimeoutTicks : kTimeoutTicks; }
    static bool pullOnly() {  // DL_XGMI_LL=0: always the pull protocol (comparison runs)
        static const bool v = [] {
            const char *e = std::getenv("DL_XGMI_LL");
            return e && *e == '0';
        }();
        return v;
    }
    XgmiCall call(const float *in, float *out, size_t n, int gather) const {
        XgmiCall c;
        c.peers = peers_;
        c.epochs = epochs_;
        c.error = error_;
        c.in = in;
        c.out = out;
        c.maxFloats = (long long)maxFloats_;
        c.n = (long long)n;
        c.rank = rank_;
        c.world = world_;
        c.gather = gather;
        const char *fe = std::getenv("DL_XGMI_FENCE");
        c.fenced = fenced_ || (fe && *fe == '1') ? 1 : 0;
        c.timeoutTicks = timeoutTicks();
        return c;
    }
    void launchLL(float *buf, size_t n, hipStream_t s) {
        DL_CHECK(connected_, "xgmi comm: connect() was not called");
        const int grid = (int)((n + kChunk - 1) / kChunk);
        if (grid == 0) return;
        const XgmiCall c = call(buf, buf, n, 0);
        switch (world_) {
            case 2: hipLaunchKernelGGL(xgmiLLKernel<2>, dim3(grid), dim3(kThreads), 0, s, c, llEpochs_); break;
            case 4: hipLaunchKernelGGL(xgmiLLKernel<4>, dim3(grid), dim3(kThreads), 0, s, c, llEpochs_); break;
            default: hipLaunchKernelGGL(xgmiLLKernel<8>, dim3(grid), dim3(kThreads), 0, s, c, llEpochs_); break;
        }
        DL_HIP(hipGetLastError());
    }
    void launch(const float *in, float *out, size_t n, int gather, hipStream_t s) {
        DL_CHECK(connected_, "xgmi comm: connect() was not called");
        DL_CHECK(n <= maxFloats_, "xgmi comm: message larger than the published buffer");
        const XgmiCall c = call(in, out, n, gather);
        const long long chunks = ((long long)n + kChunk - 1) / kChunk;
        const int grid = (int)(chunks < kSlots ? chunks : kSlots);
        if (grid == 0) return;
        hipLaunchKernelGGL(xgmiKernel, dim3(grid), dim3(kThreads), 0, s, c);
        DL_HIP(hipGetLastError());
    }

    int rank_, world_;
    size_t maxFloats_, pubBytes_ = 0, flagsBytes_ = 0, llOff_ = 0, fvOff_ = 0, faOff_ = 0;
    uint64_t *fusedVec_[kMaxRanks] = {}, *fusedArg_[kMaxRanks] = {};
    unsigned *fusedEpochs_ = nullptr;
    unsigned *llEpochs_ = nullptr;
    void *base_ = nullptr;
    void *peerBase_[kMaxRanks] = {};
    XgmiPeers peers_{};
    int *epochs_ = nullptr, *error_ = nullptr;
    std::string handle_, busId_;
    bool connected_ = false, crossDevice_ = false, fenced_ = false;
    int sameDevice_ = 1;  // ranks on this GPU, this one included
    bool ll_ = true;
};

}  // namespace

std::unique_ptr<DeviceComm> makeXgmiComm(int rank, int world, size_t maxFloats) {
    return std::unique_ptr<DeviceComm>(new XgmiComm(rank, world, maxFloats));
}
std::string xgmiHandle(DeviceComm *c) { return static_cast<XgmiComm *>(c)->handle(); }
void xgmiConnect(DeviceComm *c, const std::vector<std::string> &handles) {
    static_cast<XgmiComm *>(c)->connect(handles);
}
bool xgmiTimedOut(DeviceComm *c) { return static_cast<XgmiComm *>(c)->timedOut(); }
void xgmiSetLowLatency(DeviceComm *c, bool on) { static_cast<XgmiComm *>(c)->setLowLatency(on); }
void xgmiResetError(DeviceComm *c) { static_cast<XgmiComm *>(c)->resetError(); }
bool xgmiCrossDevice(DeviceComm *c) { return static_cast<XgmiComm *>(c)->crossDevice(); }
bool xgmiFenced(DeviceComm *c) { return static_cast<XgmiComm *>(c)->fenced(); }
namespace hipk {
// preloadModules(): one kernel of this translation unit's code object
const void *xgmiModuleKernel() { return (const void *)xgmiKernel; }
}  // namespace hipk

}  // namespace dl
