// TCP control plane between the root and its workers (+ the CPU backend's data plane).
//
// Reference behaviour kept: workers listen on --port, the root connects to every worker given by
// --workers host:port..., sends the configuration, workers load their shard and run forwards on
// command, and a worker whose root disconnects goes back to listening (nn-network.cpp:264-348,
// app.cpp:405-463). What changed: the root sends a small versioned, explicitly packed config
// (not raw struct memcpy, nn-network.cpp:621-683) plus the RCCL unique id; each worker loads its
// own shard from the model file; on GPUs the per-token data plane is RCCL, not these sockets.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "../core/common.h"
#include "../runtime/backend.h"

namespace dl {

class NetError : public Error {
  public:
    using Error::Error;
};

class Socket {
  public:
    Socket() = default;
    explicit Socket(int fd) : fd_(fd) {}
    ~Socket();
    Socket(Socket &&o) noexcept
        : fd_(o.fd_), sent_(o.sent_), recv_(o.recv_), totalSent_(o.totalSent_), totalRecv_(o.totalRecv_) {
        o.fd_ = -1;
    }
    Socket &operator=(Socket &&o) noexcept;
    Socket(const Socket &) = delete;
    Socket &operator=(const Socket &) = delete;

    static Socket connectTo(const std::string &host, int port, int retries = 50, int retryMs = 100);
    void sendAll(const void *data, u64 n);
    void recvAll(void *data, u64 n);
    void setRecvTimeout(int ms);
    bool valid() const { return fd_ >= 0; }
    int fd() const { return fd_; }
    void close();
    u64 sentBytes() const { return sent_; }
    u64 recvBytes() const { return recv_; }
    void resetStats() { sent_ = recv_ = 0; }
    void addStats(u64 sent, u64 recv) {
        sent_ += sent;
        recv_ += recv;
        totalSent_ += sent;
        totalRecv_ += recv;
    }
    // never reset (metrics deltas)
    u64 totalSentBytes() const { return totalSent_; }
    u64 totalRecvBytes() const { return totalRecv_; }

    template <typename T>
    void sendPod(const T &v) {
        sendAll(&v, sizeof(T));
    }
    template <typename T>
    T recvPod() {
        T v;
        recvAll(&v, sizeof(T));
        return v;
    }
    void sendString(const std::string &s);
    std::string recvString();

  private:
    int fd_ = -1;
    u64 sent_ = 0, recv_ = 0;
    u64 totalSent_ = 0, totalRecv_ = 0;
};

class ServerSocket {
  public:
    explicit ServerSocket(int port);
    ~ServerSocket();
    Socket accept();
    int port() const { return port_; }

  private:
    int fd_ = -1;
    int port_;
};

// Send `n` bytes to every non-null peer and receive `n` bytes from each into recv[i], multiplexed
// with poll() so no pair of ranks can deadlock on full socket buffers (the reference's
// non-blocking round-robin writeMany/readMany, nn-network.cpp:419-491).
void exchangeAll(const std::vector<Socket *> &peers, const void *send, u64 n, const std::vector<void *> &recv);

// ---- control protocol ------------------------------------------------------------------------
constexpr u32 kProtoMagic = 0xD11A3355;  // "dllama MI355"
constexpr u32 kMeshMagic = 0xD11A3356;   // worker -> worker data-plane connection
constexpr u32 kProtoVersion = 1;
constexpr u32 kAck = 23571114;           // same ACK value as the reference (nn-network.cpp:23)

// RELEASE: the first n ints of the payload are KV slots whose sequences ended (paged KV cache:
// their pages return to the pool on every rank).
// CHAIN: one step of a chained greedy decode (Backend::chainLaunch), n = 1: token (< 0: continue
// the chain on the device), position, slot. Workers keep at most 2 steps in flight and drain them
// before any other command.
enum class Cmd : u32 { FORWARD = 1, FORWARD_ARGMAX = 2, STOP = 3, PING = 4, FORWARD_SAMPLE = 5, RELEASE = 6, CHAIN = 7 };

struct ControlHeader {
    u32 cmd;
    u32 n;  // rows
};

// Serialized run configuration sent root -> worker.
struct WorkerConfig {
    u32 rank = 0, world = 1;
    bool gpu = false;
    EngineConfig engine;
    std::vector<unsigned char> rcclUid;
    std::string devComm = "xgmi";  // GPU data plane: "xgmi" (IPC one-shot) or "rccl"
    u64 xgmiMaxFloats = 0;          // largest single message per rank (xgmi)
    // CPU data plane: every worker's address by rank (index rank - 1), for the worker-to-worker mesh
    std::vector<std::string> peerHosts;
    std::vector<int> peerPorts;
};
std::string encodeWorkerConfig(const WorkerConfig &c);
WorkerConfig decodeWorkerConfig(const std::string &s);

// CPU-backend data plane over a full mesh of sockets (reference: every node holds N-1 sockets and
// writes its slice to all peers, nn-network.cpp:264-348, 537-569): every rank sends its partial to
// every other rank and sums all partials in rank order, so all ranks get bitwise the same result
// and no rank relays another's traffic.
class TcpHostComm : public HostComm {
  public:
    // peers[r] = socket to rank r (nullptr at r == rank); rank 0 is the root
    TcpHostComm(int rank, int size, std::vector<Socket *> peers) : rank_(rank), size_(size), peers_(std::move(peers)) {
        DL_CHECK((int)peers_.size() == size_, "TcpHostComm: one socket slot per rank");
    }
    int rank() const override { return rank_; }
    int size() const override { return size_; }
    void allReduceSum(float *data, u64 n) override;
    void allReduceSumQ80(float *data, u64 n) override;
    void gatherToRoot(const float *local, u64 nLocal, float *out) override;
    void stats(u64 &sent, u64 &recv) const override;

  private:
    int rank_, size_;
    std::vector<Socket *> peers_;
    std::vector<float> tmp_;
    std::vector<u8> q80_;
};

}  // namespace dl
