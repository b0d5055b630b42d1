#include <rccl/rccl.h>

#include <cstring>

#include "../core/common.h"
#include "device_comm.h"

namespace dl {

#define DL_NCCL(x)                                                                                     \
    do {                                                                                               \
        ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) throw Error(std::string("RCCL error: ") + ncclGetErrorString(r_) + " at " #x); \
    } while (0)

std::vector<unsigned char> rcclGetUniqueId() {
    ncclUniqueId id;
    DL_NCCL(ncclGetUniqueId(&id));
    std::vector<unsigned char> v(sizeof(id.internal));
    std::memcpy(v.data(), id.internal, v.size());
    return v;
}

namespace {
class RcclComm : public DeviceComm {
  public:
    RcclComm(const std::vector<unsigned char> &uid, int rank, int size) : rank_(rank), size_(size) {
        ncclUniqueId id;
        DL_CHECK(uid.size() == sizeof(id.internal), "bad RCCL unique id size");
        std::memcpy(id.internal, uid.data(), uid.size());
        DL_NCCL(ncclCommInitRank(&comm_, size, id, rank));
    }
    ~RcclComm() override {
        if (comm_) ncclCommDestroy(comm_);
    }
    std::string asyncError() override {
        if (!comm_) return "communicator released after an error";
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) return "ncclCommGetAsyncError failed";
        return st == ncclSuccess || st == ncclInProgress ? "" : std::string("RCCL async error: ") + ncclGetErrorString(st);
    }
    void shutdownNow() override {
        if (comm_) (void)ncclCommAbort(comm_);
        comm_ = nullptr;
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    std::string name() const override { return "rccl"; }
    void allReduceSum(float *buf, size_t n, hipStream_t s) override {
        DL_NCCL(ncclAllReduce(buf, buf, n, ncclFloat32, ncclSum, comm_, s));
    }
    void allGather(const float *send, float *recv, size_t nPerRank, hipStream_t s) override {
        DL_NCCL(ncclAllGather(send, recv, nPerRank, ncclFloat32, comm_, s));
    }
    // Root-only gather (the reference's SYNC_NODE_SLICES_EXCEPT_ROOT, llm.cpp:432): point-to-point
    // sends to rank 0 move 1/N of an all-gather's bytes; rank 0 places its own slice locally.
    void gatherToRoot(const float *send, float *recv, size_t nPerRank, hipStream_t s) override {
        if (rank_ == 0) DL_HIP(hipMemcpyAsync(recv, send, nPerRank * sizeof(float), hipMemcpyDeviceToDevice, s));
        if (size_ == 1) return;
        DL_NCCL(ncclGroupStart());
        if (rank_ == 0) {
            for (int p = 1; p < size_; p++) DL_NCCL(ncclRecv(recv + (size_t)p * nPerRank, nPerRank, ncclFloat32, p, comm_, s));
        } else {
            DL_NCCL(ncclSend(send, nPerRank, ncclFloat32, 0, comm_, s));
        }
        DL_NCCL(ncclGroupEnd());
    }
    void broadcastInts(int *buf, size_t n, int root, hipStream_t s) override {
        DL_NCCL(ncclBroadcast(buf, buf, n, ncclInt32, root, comm_, s));
    }

  private:
    int rank_, size_;
    ncclComm_t comm_ = nullptr;
};
}  // namespace

std::unique_ptr<DeviceComm> makeRcclComm(const std::vector<unsigned char> &uid, int rank, int size) {
    return std::unique_ptr<DeviceComm>(new RcclComm(uid, rank, size));
}

}  // namespace dl
