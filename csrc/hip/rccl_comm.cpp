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
