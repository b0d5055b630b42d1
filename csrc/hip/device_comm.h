// Device data plane for tensor parallelism: RCCL over xGMI, one process per GPU.
//
// Replaces the reference's TCP all-gather + local merge-add (nn-network.cpp:537-569,
// llm.cpp:212-217, 308-314) with a single in-place f32 all-reduce per residual update and an
// all-gather of the vocab-sharded logits (nn-network.cpp SYNC_NODE_SLICES_EXCEPT_ROOT).
// Collectives are enqueued on the engine's stream so they are captured in the forward hipGraph.
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>
#include <vector>

namespace dl {

namespace hipk {
struct TpXchg;
}

class DeviceComm {
  public:
    virtual ~DeviceComm() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    virtual void allReduceSum(float *buf, size_t n, hipStream_t s) = 0;
    virtual void allGather(const float *send, float *recv, size_t nPerRank, hipStream_t s) = 0;
    // Rank 0 receives every rank's nPerRank floats in rank order (the reference gathers the logits
    // slices to the root only: SYNC_NODE_SLICES_EXCEPT_ROOT, llm.cpp:432); recv is only written on
    // rank 0. Default: an all-gather.
    virtual void gatherToRoot(const float *send, float *recv, size_t nPerRank, hipStream_t s) {
        allGather(send, recv, nPerRank, s);
    }
    virtual void broadcastInts(int *buf, size_t n, int root, hipStream_t s) = 0;
    virtual std::string name() const = 0;
    // Health reporting: device int set non-zero when a collective stopped waiting
    // for a peer (null if the transport has none), and the transport's host-side error text.
    virtual const int *deviceErrorFlag() const { return nullptr; }
    virtual std::string asyncError() { return ""; }
    // Release the communicator without waiting for peers (used after an error).
    virtual void shutdownNow() {}
    // Clear the device error flag (after a self-test whose failure was handled).
    virtual void resetError() {}
    // Ranks of this communicator that run on this rank's GPU (1 on a real multi-GPU node; all of
    // them in a same-GPU rehearsal): they share the device's resident workgroup slots.
    virtual int ranksOnDevice() const { return 1; }
    // Targets of the exchange fused into producer kernels (hipk::TpXchg): region 0 = residual
    // partial sums (elements b * dim + row, up to 65536), region 1 = argmax winners (2 words per
    // row). False when the transport has none (RCCL): the engine launches separate collectives.
    virtual bool fusedXchg(int region, hipk::TpXchg *x) const {
        (void)region;
        (void)x;
        return false;
    }    // No data plane at all (makeComputeOnlyComm): the engine skips the fused-exchange self-test.
    virtual bool computeOnly() const { return false; }
};

// Rank `rank` of a `world`-rank tensor-parallel group with no peers (sim_comm.cpp): collectives
// are no-ops and the fused exchange runs in loopback (TpXchg::loopback), so one GPU times a TP-N
// rank's shard kernels with the exchange removed (bench.py --tp-rank-compute). Not a data plane:
// the model's outputs are those of one shard.
std::unique_ptr<DeviceComm> makeComputeOnlyComm(int rank, int world);

// 128-byte RCCL unique id (generated on rank 0, distributed over the control plane).
std::vector<unsigned char> rcclGetUniqueId();
// Must be called with the HIP device of this rank already selected.
std::unique_ptr<DeviceComm> makeRcclComm(const std::vector<unsigned char> &uid, int rank, int size);

#define DL_HIP(x)                                                                                        \
    do {                                                                                                 \
        hipError_t e_ = (x);                                                                             \
        if (e_ != hipSuccess) throw Error(std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x); \
    } while (0)

// One-shot xGMI collectives over IPC-shared buffers (xgmi_comm.cpp). Bootstrap: create on every
// rank (device selected), exchange xgmiHandle() bytes over the control plane, xgmiConnect() with
// all ranks' handles, barrier, then use. maxFloats bounds any single message (per rank).
std::unique_ptr<DeviceComm> makeXgmiComm(int rank, int world, size_t maxFloats);
std::string xgmiHandle(DeviceComm *c);
void xgmiConnect(DeviceComm *c, const std::vector<std::string> &handles);
bool xgmiTimedOut(DeviceComm *c);
void xgmiSetLowLatency(DeviceComm *c, bool on);  // LL push protocol for small all-reduces (default on)
void xgmiResetError(DeviceComm *c);
// Peers on other GPUs (PCI bus ids differ)? Then the pull protocol runs with system-scope fences
// around its flags unless DL_XGMI_FENCE=0 (the LL / fused exchanges carry data and epoch in one
// 64-bit word and need no fence on any topology).
bool xgmiCrossDevice(DeviceComm *c);
bool xgmiFenced(DeviceComm *c);

}  // namespace dl
