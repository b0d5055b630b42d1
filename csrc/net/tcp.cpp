#include "tcp.h"

#include "../core/quant.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <sstream>
#include <thread>

namespace dl {

Socket::~Socket() { close(); }

Socket &Socket::operator=(Socket &&o) noexcept {
    if (this != &o) {
        close();
        fd_ = o.fd_;
        sent_ = o.sent_;
        recv_ = o.recv_;
        totalSent_ = o.totalSent_;
        totalRecv_ = o.totalRecv_;
        o.fd_ = -1;
    }
    return *this;
}

void Socket::close() {
    if (fd_ >= 0) {
        ::shutdown(fd_, SHUT_RDWR);
        ::close(fd_);
        fd_ = -1;
    }
}

static void tuneSocket(int fd) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
#ifdef TCP_QUICKACK
    setsockopt(fd, IPPROTO_TCP, TCP_QUICKACK, &one, sizeof(one));
#endif
    setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof(one));
}

Socket Socket::connectTo(const std::string &host, int port, int retries, int retryMs) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    const std::string p = std::to_string(port);
    if (getaddrinfo(host.c_str(), p.c_str(), &hints, &res) != 0 || !res)
        throw NetError("Cannot resolve host " + host);
    for (int attempt = 0;; attempt++) {
        int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) {
            freeaddrinfo(res);
            throw NetError("Cannot create socket");
        }
        if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
            freeaddrinfo(res);
            tuneSocket(fd);
            return Socket(fd);
        }
        ::close(fd);
        if (attempt >= retries) {
            freeaddrinfo(res);
            throw NetError("Cannot connect to " + host + ":" + p);
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(retryMs));
    }
}

void Socket::sendAll(const void *data, u64 n) {
    const char *p = (const char *)data;
    while (n > 0) {
        ssize_t s = ::send(fd_, p, n > (1u << 20) ? (1u << 20) : n, MSG_NOSIGNAL);
        if (s < 0) {
            if (errno == EINTR) continue;
            throw NetError(std::string("Error writing to socket: ") + std::strerror(errno));
        }
        if (s == 0) throw NetError("Socket closed");
        p += s;
        n -= (u64)s;
        sent_ += (u64)s;
        totalSent_ += (u64)s;
    }
}

void Socket::recvAll(void *data, u64 n) {
    char *p = (char *)data;
    while (n > 0) {
        ssize_t r = ::recv(fd_, p, n, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == EWOULDBLOCK) throw NetError("Socket read timeout");
            throw NetError(std::string("Error reading from socket: ") + std::strerror(errno));
        }
        if (r == 0) throw NetError("Socket closed");
        p += r;
        n -= (u64)r;
        recv_ += (u64)r;
        totalRecv_ += (u64)r;
    }
}

void exchangeAll(const std::vector<Socket *> &peers, const void *send, u64 n, const std::vector<void *> &recv) {
    const size_t P = peers.size();
    std::vector<u64> sent(P, 0), got(P, 0);
    std::vector<pollfd> fds;
    std::vector<size_t> idx;
    for (;;) {
        fds.clear();
        idx.clear();
        for (size_t i = 0; i < P; i++) {
            if (!peers[i]) continue;
            short ev = 0;
            if (sent[i] < n) ev |= POLLOUT;
            if (got[i] < n) ev |= POLLIN;
            if (!ev) continue;
            fds.push_back(pollfd{peers[i]->fd(), ev, 0});
            idx.push_back(i);
        }
        if (fds.empty()) return;
        const int r = ::poll(fds.data(), fds.size(), 60000);
        if (r < 0) {
            if (errno == EINTR) continue;
            throw NetError(std::string("poll: ") + std::strerror(errno));
        }
        if (r == 0) throw NetError("Socket exchange timeout");
        for (size_t k = 0; k < fds.size(); k++) {
            const size_t i = idx[k];
            if (fds[k].revents & (POLLERR | POLLHUP | POLLNVAL) && !(fds[k].revents & POLLIN))
                throw NetError("Socket closed during exchange");
            if ((fds[k].revents & POLLOUT) && sent[i] < n) {
                const u64 left = n - sent[i];
                const ssize_t w = ::send(fds[k].fd, (const char *)send + sent[i], left > (1u << 20) ? (1u << 20) : left,
                                         MSG_NOSIGNAL | MSG_DONTWAIT);
                if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
                    throw NetError(std::string("Error writing to socket: ") + std::strerror(errno));
                if (w > 0) {
                    sent[i] += (u64)w;
                    peers[i]->addStats((u64)w, 0);
                }
            }
            if ((fds[k].revents & POLLIN) && got[i] < n) {
                const ssize_t g = ::recv(fds[k].fd, (char *)recv[i] + got[i], n - got[i], MSG_DONTWAIT);
                if (g == 0) throw NetError("Socket closed");
                if (g < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)
                    throw NetError(std::string("Error reading from socket: ") + std::strerror(errno));
                if (g > 0) {
                    got[i] += (u64)g;
                    peers[i]->addStats(0, (u64)g);
                }
            }
        }
    }
}

void Socket::setRecvTimeout(int ms) {
    timeval tv;
    tv.tv_sec = ms / 1000;
    tv.tv_usec = (ms % 1000) * 1000;
    setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

void Socket::sendString(const std::string &s) {
    sendPod<u32>((u32)s.size());
    if (!s.empty()) sendAll(s.data(), s.size());
}

std::string Socket::recvString() {
    const u32 n = recvPod<u32>();
    if (n > (64u << 20)) throw NetError("message too large");
    std::string s(n, '\0');
    if (n) recvAll(&s[0], n);
    return s;
}

ServerSocket::ServerSocket(int port) : port_(port) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd_ < 0) throw NetError("Cannot create server socket");
    int one = 1;
    setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = INADDR_ANY;
    addr.sin_port = htons((u16)port);
    if (::bind(fd_, (sockaddr *)&addr, sizeof(addr)) < 0) {
        ::close(fd_);
        throw NetError("Cannot bind port " + std::to_string(port));
    }
    if (::listen(fd_, 16) < 0) {
        ::close(fd_);
        throw NetError("Cannot listen on port " + std::to_string(port));
    }
}

ServerSocket::~ServerSocket() {
    if (fd_ >= 0) ::close(fd_);
}

Socket ServerSocket::accept() {
    while (true) {
        int fd = ::accept(fd_, nullptr, nullptr);
        if (fd >= 0) {
            tuneSocket(fd);
            return Socket(fd);
        }
        if (errno != EINTR) throw NetError("accept failed");
    }
}

// ---- config serialization (key=value lines, hex for binary) -------------------------------------
static std::string hexOf(const std::vector<unsigned char> &v) {
    static const char *d = "0123456789abcdef";
    std::string s;
    for (unsigned char c : v) {
        s.push_back(d[c >> 4]);
        s.push_back(d[c & 15]);
    }
    return s;
}
static std::vector<unsigned char> unhex(const std::string &s) {
    std::vector<unsigned char> v(s.size() / 2);
    for (size_t i = 0; i < v.size(); i++) v[i] = (unsigned char)std::stoi(s.substr(2 * i, 2), nullptr, 16);
    return v;
}

std::string encodeWorkerConfig(const WorkerConfig &c) {
    std::ostringstream o;
    const EngineConfig &e = c.engine;
    const ModelHeader &h = e.syntheticHeader;
    o << "magic=" << kProtoMagic << "\nversion=" << kProtoVersion << "\nrank=" << c.rank << "\nworld=" << c.world
      << "\ngpu=" << (c.gpu ? 1 : 0) << "\nmodel=" << e.modelPath << "\nmax_seq_len=" << e.maxSeqLen
      << "\nmax_batch=" << e.maxBatch << "\nmax_decode=" << e.maxDecode << "\nn_slots=" << e.nSlots << "\nbuffer=" << (int)e.bufferType
      << "\nsync=" << (int)e.syncType
      << "\ngraphs=" << (e.useGraphs ? 1 : 0) << "\nkv_bf16=" << (e.kvBf16 ? 1 : 0) << "\nkv_pages=" << e.kvPages
      << "\nkv_page_size=" << e.kvPageSize << "\nbatch_invariant=" << (e.batchInvariant ? 1 : 0)
      << "\nsynthetic=" << (e.synthetic ? 1 : 0) << "\nseed=" << e.seed << "\nh_dim=" << h.dim
      << "\nh_hidden=" << h.hiddenDim << "\nh_layers=" << h.nLayers << "\nh_heads=" << h.nHeads
      << "\nh_kv=" << h.nKvHeads << "\nh_vocab=" << h.vocabSize << "\nh_seq=" << h.seqLen
      << "\nh_theta=" << h.ropeTheta << "\nh_wtype=" << (int)h.weightType << "\nh_act=" << (int)h.hiddenAct
      << "\nh_rsf=" << h.ropeScalingFactor << "\nh_rlo=" << h.ropeScalingLowFreqFactor
      << "\nh_rhi=" << h.ropeScalingHighFreqFactor << "\nh_rorig=" << h.ropeScalingOrigMaxSeqLen
      << "\nuid=" << hexOf(c.rcclUid) << "\ndev_comm=" << c.devComm << "\nxgmi_max=" << c.xgmiMaxFloats << "\n";
    for (size_t i = 0; i < c.peerHosts.size(); i++) o << "peer=" << c.peerHosts[i] << ":" << c.peerPorts[i] << "\n";
    return o.str();
}

WorkerConfig decodeWorkerConfig(const std::string &s) {
    WorkerConfig c;
    std::istringstream in(s);
    std::string line;
    EngineConfig &e = c.engine;
    ModelHeader &h = e.syntheticHeader;
    bool magicOk = false;
    while (std::getline(in, line)) {
        const size_t eq = line.find('=');
        if (eq == std::string::npos) continue;
        const std::string k = line.substr(0, eq), v = line.substr(eq + 1);
        if (k == "magic") magicOk = std::stoul(v) == kProtoMagic;
        else if (k == "version" && std::stoul(v) != kProtoVersion) throw NetError("protocol version mismatch");
        else if (k == "rank") c.rank = std::stoul(v);
        else if (k == "world") c.world = std::stoul(v);
        else if (k == "gpu") c.gpu = v == "1";
        else if (k == "model") e.modelPath = v;
        else if (k == "max_seq_len") e.maxSeqLen = std::stoul(v);
        else if (k == "max_batch") e.maxBatch = std::stoul(v);
        else if (k == "max_decode") e.maxDecode = std::stoul(v);
        else if (k == "n_slots") e.nSlots = std::stoul(v);
        else if (k == "buffer") e.bufferType = (FloatType)std::stoi(v);
        else if (k == "sync") e.syncType = (FloatType)std::stoi(v);
        else if (k == "graphs") e.useGraphs = v == "1";
        else if (k == "kv_bf16") e.kvBf16 = v == "1";
        else if (k == "kv_pages") e.kvPages = std::stoul(v);
        else if (k == "kv_page_size") e.kvPageSize = std::stoul(v);
        else if (k == "batch_invariant") e.batchInvariant = v == "1";
        else if (k == "synthetic") e.synthetic = v == "1";
        else if (k == "seed") e.seed = std::stoull(v);
        else if (k == "h_dim") h.dim = std::stoul(v);
        else if (k == "h_hidden") h.hiddenDim = std::stoul(v);
        else if (k == "h_layers") h.nLayers = std::stoul(v);
        else if (k == "h_heads") h.nHeads = std::stoul(v);
        else if (k == "h_kv") h.nKvHeads = std::stoul(v);
        else if (k == "h_vocab") h.vocabSize = std::stoul(v);
        else if (k == "h_seq") h.seqLen = std::stoul(v);
        else if (k == "h_theta") h.ropeTheta = std::stof(v);
        else if (k == "h_wtype") h.weightType = (FloatType)std::stoi(v);
        else if (k == "h_act") h.hiddenAct = (HiddenAct)std::stoi(v);
        else if (k == "h_rsf") h.ropeScalingFactor = std::stof(v);
        else if (k == "h_rlo") h.ropeScalingLowFreqFactor = std::stof(v);
        else if (k == "h_rhi") h.ropeScalingHighFreqFactor = std::stof(v);
        else if (k == "h_rorig") h.ropeScalingOrigMaxSeqLen = std::stoul(v);
        else if (k == "uid") c.rcclUid = unhex(v);
        else if (k == "dev_comm") c.devComm = v;
        else if (k == "xgmi_max") c.xgmiMaxFloats = std::stoull(v);
        else if (k == "peer") {
            const size_t colon = v.rfind(':');
            if (colon == std::string::npos) throw NetError("bad peer address in config");
            c.peerHosts.push_back(v.substr(0, colon));
            c.peerPorts.push_back(std::stoi(v.substr(colon + 1)));
        }
    }
    if (!magicOk) throw NetError("bad control-plane magic");
    h.origSeqLen = h.seqLen;
    return c;
}

// ---- CPU data plane ----------------------------------------------------------------------------
void TcpHostComm::allReduceSum(float *data, u64 n) {
    if (size_ == 1) return;
    tmp_.resize(n * size_);
    std::vector<void *> recv(size_);
    for (int r = 0; r < size_; r++) recv[r] = tmp_.data() + (u64)r * n;
    exchangeAll(peers_, data, n * sizeof(float), recv);
    std::memcpy(tmp_.data() + (u64)rank_ * n, data, n * sizeof(float));
    // every rank sums the same partials in the same (rank) order: bitwise identical results
    std::memcpy(data, tmp_.data(), n * sizeof(float));
    for (int r = 1; r < size_; r++) {
        const float *src = tmp_.data() + (u64)r * n;
        for (u64 i = 0; i < n; i++) data[i] += src[i];
    }
}

void TcpHostComm::allReduceSumQ80(float *data, u64 n) {
    if (size_ == 1) return;
    DL_CHECK(n % kQBlock == 0, "Q80 sync needs 32-aligned vectors");
    const u64 part = n / kQBlock * sizeof(BlockQ80);
    q80_.resize(part * size_);
    // my quantized partial goes to slot [rank] and to every peer; theirs land in their slots
    quantizeQ80(data, reinterpret_cast<BlockQ80 *>(q80_.data() + part * rank_), n);
    std::vector<void *> recv(size_);
    for (int r = 0; r < size_; r++) recv[r] = q80_.data() + part * r;
    exchangeAll(peers_, q80_.data() + part * rank_, part, recv);
    tmp_.resize(n);
    std::fill(data, data + n, 0.f);
    for (int r = 0; r < size_; r++) {
        dequantizeQ80(reinterpret_cast<const BlockQ80 *>(q80_.data() + part * r), tmp_.data(), n);
        for (u64 i = 0; i < n; i++) data[i] += tmp_[i];
    }
}

void TcpHostComm::gatherToRoot(const float *local, u64 nLocal, float *out) {
    if (rank_ == 0) {
        if (out) std::memcpy(out, local, nLocal * sizeof(float));
        for (int r = 1; r < size_; r++) {
            float *dst = out ? out + (u64)r * nLocal : nullptr;
            if (dst) {
                peers_[r]->recvAll(dst, nLocal * sizeof(float));
            } else {
                tmp_.resize(nLocal);
                peers_[r]->recvAll(tmp_.data(), nLocal * sizeof(float));
            }
        }
    } else {
        peers_[0]->sendAll(local, nLocal * sizeof(float));
    }
}

void TcpHostComm::stats(u64 &sent, u64 &recv) const {
    sent = recv = 0;
    for (Socket *s : peers_) {
        if (!s) continue;
        sent += s->sentBytes();
        recv += s->recvBytes();
    }
}

}  // namespace dl
