#include "app.h"

#include <cstdlib>

#include <cstdio>
#include <cstring>
#include <ctime>

#include <unistd.h>

#include "../hip/engine.h"
#include "metrics.h"
#include "weight_stream.h"

namespace dl {

AppArgs AppArgs::parse(int argc, char **argv, bool requireMode) {
    AppArgs a;
    a.seed = (u64)std::time(nullptr);
    int i = 1;
    if (requireMode && argc > 1) {
        a.mode = argv[1];
        i++;
    }
    for (int x = 0; x < argc; x++) {
        if (!std::strcmp(argv[x], "--usage") || !std::strcmp(argv[x], "--help") || !std::strcmp(argv[x], "-h")) {
            a.help = true;
            return a;
        }
    }
    for (; i + 1 < argc; i += 2) {
        const std::string name = argv[i];
        const char *value = argv[i + 1];
        if (name == "--model") a.modelPath = value;
        else if (name == "--tokenizer") a.tokenizerPath = value;
        else if (name == "--prompt") a.prompt = value;
        else if (name == "--buffer-float-type") a.bufferType = parseFloatType(value);
        else if (name == "--workers") {
            int j = i + 1;
            for (; j < argc && argv[j][0] != '-'; j++) {
                const char *v = argv[j];
                const char *sep = std::strchr(v, ':');
                if (!sep) throw Error(std::string("Invalid worker address: ") + v);
                a.workerHosts.emplace_back(v, sep - v);
                a.workerPorts.push_back(std::atoi(sep + 1));
            }
            i = j - 2;
        } else if (name == "--port") a.port = std::atoi(value);
        else if (name == "--nthreads") a.nThreads = std::atoi(value);
        else if (name == "--steps") a.steps = std::atoi(value);
        else if (name == "--temperature") a.temperature = (float)std::atof(value);
        else if (name == "--topp") a.topp = (float)std::atof(value);
        else if (name == "--seed") a.seed = std::strtoull(value, nullptr, 10);
        else if (name == "--chat-template") a.chatTemplate = parseChatTemplateType(value);
        else if (name == "--max-seq-len") a.maxSeqLen = (u32)std::atoi(value);
        else if (name == "--gpu-index") a.gpuIndex = std::atoi(value);
        else if (name == "--gpu-segments") {
            const char *sep = std::strchr(value, ':');
            if (!sep) throw Error("GPU segments expected in the format <from>:<to>");
            a.gpuSegmentFrom = std::atoi(value);
            a.gpuSegmentTo = std::atoi(sep + 1);
        } else if (name == "--net-turbo") a.netTurbo = std::atoi(value) == 1;
        else if (name == "--max-batch") a.nBatches = std::atoi(value);
        else if (name == "--prefill-chunk") a.prefillChunk = std::atoi(value);
        else if (name == "--slots") a.slots = std::atoi(value);
        else if (name == "--kv-dtype") {
            const std::string v = value;
            if (v == "bf16") a.kvBf16 = true;
            else if (v == "f32") a.kvBf16 = false;
            else throw Error("Invalid --kv-dtype (bf16|f32): " + v);
        } else if (name == "--kv-pages") a.kvPages = std::atoi(value);
        else if (name == "--kv-page-size") a.kvPageSize = std::atoi(value);
        else if (name == "--batch-invariant") a.batchInvariant = std::atoi(value) != 0;
        else if (name == "--graph") a.graphs = std::atoi(value) != 0;
        else if (name == "--log-level") a.logLevel = std::atoi(value);
        else if (name == "--synthetic") a.synthetic = value;
        else if (name == "--web-ui") a.webUi = value;
        else if (name == "--stream-weights") a.streamWeights = std::atoi(value) != 0;
        else if (name == "--weights-cache") a.weightsCache = value;
        else if (name == "--metrics") a.metricsPath = value;
        else if (name == "--sync-type") a.syncType = parseFloatType(value);
        else if (name == "--profile") a.profile = std::atoi(value) != 0;
        else throw Error("Unknown option: " + name);
    }
    if (a.syncType == FloatType::UNK) a.syncType = a.bufferType == FloatType::Q80 ? FloatType::Q80 : FloatType::F32;
    setLogLevel(a.logLevel);
    return a;
}

ModelHeader syntheticHeader(const std::string &name, u32 seqLen) {
    ModelHeader h;
    h.weightType = FloatType::Q40;
    h.vocabSize = 128256;
    h.nKvHeads = 8;
    h.ropeTheta = 500000.f;
    h.ropeType = RopeType::LLAMA3_1;
    h.ropeScalingFactor = 8.f;
    h.ropeScalingLowFreqFactor = 1.f;
    h.ropeScalingHighFreqFactor = 4.f;
    h.ropeScalingOrigMaxSeqLen = 8192;
    if (name == "llama3_2_1b") { h.dim = 2048; h.hiddenDim = 8192; h.nLayers = 16; h.nHeads = 32; }
    else if (name == "llama3_2_3b") { h.dim = 3072; h.hiddenDim = 8192; h.nLayers = 28; h.nHeads = 24; }
    else if (name == "llama3_1_8b") { h.dim = 4096; h.hiddenDim = 14336; h.nLayers = 32; h.nHeads = 32; }
    else if (name == "llama3_3_70b") { h.dim = 8192; h.hiddenDim = 28672; h.nLayers = 80; h.nHeads = 64; }
    else if (name == "llama3_1_405b") { h.dim = 16384; h.hiddenDim = 53248; h.nLayers = 126; h.nHeads = 128; }
    else throw Error("unknown synthetic model: " + name);
    h.seqLen = seqLen > 0 ? seqLen : 8192;
    h.origSeqLen = h.seqLen;
    return h;
}

// Prompt rows per forward: --prefill-chunk, else 1024 on GPUs (one wide-GEMM launch per matrix
// covers every 128-token tile of the chunk: 0.04 vs 0.13 ms/token at 32-row chunks, r3 bench) and
// --max-batch on the CPU backend (the reference's nBatches).
static int prefillChunkOf(const AppArgs &a) {
    const bool gpu = a.gpuIndex >= 0 || !a.synthetic.empty();
    return a.prefillChunk > 0 ? a.prefillChunk : (gpu ? std::max(1024, a.nBatches) : a.nBatches);
}

static EngineConfig engineConfigFrom(const AppArgs &a, int nSlots) {
    EngineConfig c;
    c.modelPath = a.modelPath;
    c.maxSeqLen = a.maxSeqLen;
    c.maxBatch = (u32)std::max(a.nBatches, prefillChunkOf(a));  // rows the engine's buffers hold
    c.maxDecode = (u32)a.nBatches;  // decode-only state (chain history, argmax exchange) for decode rows
    c.nSlots = (u32)nSlots;
    c.bufferType = a.bufferType;
    c.syncType = a.syncType;
    c.nThreads = a.nThreads;
    c.gpuIndex = a.gpuIndex;
    c.useGraphs = a.graphs;
    c.kvBf16 = a.kvBf16;
    c.kvPages = (u32)std::max(0, a.kvPages);
    c.kvPageSize = (u32)std::max(32, a.kvPageSize);
    c.batchInvariant = a.batchInvariant;
    if (!a.synthetic.empty()) {
        c.synthetic = true;
        c.syntheticHeader = syntheticHeader(a.synthetic, a.maxSeqLen);
        c.bufferType = FloatType::Q80;
    }
    return c;
}

static std::unique_ptr<Backend> makeBackend(const EngineConfig &c, bool gpu, HostComm *hc, DeviceComm *dc) {
    if (gpu) return std::unique_ptr<Backend>(makeHipEngine(c, dc).release());
    return makeCpuBackend(c, hc);
}

InferenceSession::InferenceSession(const AppArgs &args, int nSlots) : args_(args), nSlots_(nSlots) {
    if (!args.metricsPath.empty()) MetricsSink::global().open(args.metricsPath);
    maxBatch_ = args.nBatches;
    prefillChunk_ = prefillChunkOf(args);
    gpu_ = args.gpuIndex >= 0 || !args.synthetic.empty();
    AppArgs a = args;
    if (gpu_ && a.gpuIndex < 0) a.gpuIndex = 0;
    EngineConfig ec = engineConfigFrom(a, nSlots);
    const int world = 1 + (int)args.workerHosts.size();

    if (args.synthetic.empty()) {
        ModelHeader h = loadModelHeader(args.modelPath, args.maxSeqLen);
        if ((u32)world > h.nKvHeads)
            throw Error("This version does not support more nodes than the number of KV heads in the model");
        if (h.weightType == FloatType::Q40 && args.bufferType != FloatType::Q80)
            throw Error("This version supports only Q40 weights with Q80 sync type");
    }

    WorkerConfig wc;
    wc.world = (u32)world;
    wc.gpu = gpu_;
    wc.engine = ec;
    if (world > 1) {
        if (gpu_) {
            const char *dcEnv = std::getenv("DL_TP_COMM");
            wc.devComm = dcEnv && *dcEnv ? dcEnv : "xgmi";
            const ModelHeader h = args.synthetic.empty() ? loadModelHeader(args.modelPath, args.maxSeqLen)
                                                         : syntheticHeader(args.synthetic, args.maxSeqLen);
            const u64 vocab0 = (h.vocabSize + world - 1) / world;
            wc.xgmiMaxFloats = (u64)ec.maxBatch * std::max<u64>(h.dim, vocab0);
            if (wc.devComm == "rccl") wc.rcclUid = rcclGetUniqueId();
        }
        for (size_t i = 0; i < args.workerHosts.size(); i++) {
            if (logLevel() >= 1)
                std::printf("⭕ Connecting to worker %s:%d\n", args.workerHosts[i].c_str(), args.workerPorts[i]);
            workers_.push_back(Socket::connectTo(args.workerHosts[i], args.workerPorts[i]));
        }
        // every worker learns every other worker's address (the CPU data plane is a full mesh)
        wc.peerHosts = args.workerHosts;
        wc.peerPorts = args.workerPorts;
        for (size_t i = 0; i < workers_.size(); i++) {
            wc.rank = (u32)(i + 1);
            workers_[i].sendPod<u32>(kProtoMagic);
            workers_[i].sendString(encodeWorkerConfig(wc));
        }
        // workers without the model file get their slices streamed
        for (size_t i = 0; i < workers_.size(); i++) {
            const u32 st = workers_[i].recvPod<u32>();
            if (st == kWantWeights) {
                if (logLevel() >= 1) std::printf("💿 Streaming weights to worker %zu\n", i + 1);
                serveWeights(workers_[i], args.modelPath);
            } else if (st != kHaveWeights) {
                throw NetError("worker failed before loading weights");
            }
        }
        std::vector<Socket *> peers{nullptr};  // by rank: the root's data sockets are its control sockets
        for (auto &s : workers_) peers.push_back(&s);
        if (gpu_) {
            DL_HIP(hipSetDevice(a.gpuIndex));
            if (wc.devComm == "xgmi") {
                // every rank publishes an IPC handle of its buffers; the root redistributes them
                devComm_ = makeXgmiComm(0, world, wc.xgmiMaxFloats);
                std::vector<std::string> handles{xgmiHandle(devComm_.get())};
                for (auto &s : workers_) {
                    if (s.recvPod<u32>() != kAck) throw NetError("worker failed to create its device comm: " + s.recvString());
                    handles.push_back(s.recvString());
                }
                for (auto &s : workers_)
                    for (auto &hnd : handles) s.sendString(hnd);
                xgmiConnect(devComm_.get(), handles);
            } else {
                devComm_ = makeRcclComm(wc.rcclUid, 0, world);
            }
        } else {
            hostComm_.reset(new TcpHostComm(0, world, peers));
        }
        if (logLevel() >= 1) std::printf("⭕ Network is initialized (%d nodes)\n", world);
        // ranks sharing one GPU (same-GPU rehearsals): a rank spinning in its exchange on a
        // 256+-row forward can keep its peer's kernels off the CUs until the collective times out,
        // so the default prompt chunk drops to 32 rows there (an explicit --prefill-chunk stays)
        if (devComm_ && devComm_->ranksOnDevice() > 1 && args.prefillChunk <= 0 && prefillChunk_ > 32) {
            prefillChunk_ = std::max(32, args.nBatches);
            if (logLevel() >= 1)
                std::printf("ℹ️  %d ranks share this GPU: prompt chunks of %d rows\n", devComm_->ranksOnDevice(),
                            prefillChunk_);
        }
    }
    backend_ = makeBackend(ec, gpu_, hostComm_.get(), devComm_.get());
    for (auto &s : workers_) {
        const u32 ack = s.recvPod<u32>();
        if (ack != kAck) throw NetError("worker failed to initialize: " + s.recvString());
    }
    if (logLevel() >= 1) {
        printModelHeader(backend_->header());
        const Backend::LoadStats ls = backend_->loadStats();
        if (ls.fileBytes > 0)
            std::printf("💿 Weights: %.2f GB read in %.2f s (%.2f GB/s)%s\n", ls.fileBytes / 1e9, ls.ms / 1e3,
                        ls.fileBytes / 1e6 / std::max(ls.ms, 1e-3),
                        ls.deviceBytes ? (", " + std::to_string(ls.deviceBytes >> 20) + " MB on device").c_str() : "");
    }
    if (!args.tokenizerPath.empty()) {
        tokenizer_.reset(new Tokenizer(args.tokenizerPath, true));
        if ((u32)tokenizer_->vocabSize() != backend_->header().vocabSize)
            throw Error("Tokenizer vocab size does not match the model vocab size");
    }
    sampler_.reset(new Sampler((int)backend_->header().vocabSize, args.temperature, args.topp, args.seed));
    for (auto &s : workers_) s.resetStats();
}

InferenceSession::~InferenceSession() {
    try {
        finish();
    } catch (...) {
    }
}

void InferenceSession::sendControl(Cmd cmd, int n, const int *tokens, const int *positions, const int *slots) {
    if (workers_.empty()) return;
    std::vector<int> buf(2 + 3 * (size_t)n);
    buf[0] = (int)cmd;
    buf[1] = n;
    std::memcpy(&buf[2], tokens, n * sizeof(int));
    std::memcpy(&buf[2 + n], positions, n * sizeof(int));
    std::memcpy(&buf[2 + 2 * n], slots, n * sizeof(int));
    for (auto &s : workers_) s.sendAll(buf.data(), buf.size() * sizeof(int));
}

void InferenceSession::releaseSlot(int slot) {
    const int zero = 0;
    sendControl(Cmd::RELEASE, 1, &slot, &zero, &zero);
    backend_->releaseSlot(slot);
}

void InferenceSession::forward(int n, const int *tokens, const int *positions, const int *slots, float *logits) {
    TraceRange tr("dllama.forward");
    Timer t;
    sendControl(Cmd::FORWARD, n, tokens, positions, slots);
    backend_->forward(n, tokens, positions, slots, logits);
    recordMetrics("forward", n, t.elapsedMs());
}

void InferenceSession::forwardArgmax(int n, const int *tokens, const int *positions, const int *slots, int *out) {
    TraceRange tr("dllama.forward_argmax");
    Timer t;
    sendControl(Cmd::FORWARD_ARGMAX, n, tokens, positions, slots);
    backend_->forwardArgmax(n, tokens, positions, slots, out);
    recordMetrics("forward_argmax", n, t.elapsedMs());
}

void InferenceSession::forwardSample(int n, const int *tokens, const int *positions, const int *slots,
                                     const SampleSpec *specs, int *out) {
    TraceRange tr("dllama.forward_sample");
    Timer t;
    sendControl(Cmd::FORWARD_SAMPLE, n, tokens, positions, slots);
    if (!workers_.empty()) {  // the specs follow the row arrays (every rank runs the same draw graph)
        for (auto &s : workers_) s.sendAll(specs, n * sizeof(SampleSpec));
    }
    backend_->forwardSample(n, tokens, positions, slots, specs, out);
    recordMetrics("forward_sample", n, t.elapsedMs());
}

void InferenceSession::launchIds(int n, const int *tokens, const int *positions, const int *slots,
                                 const SampleSpec *specs) {
    launchTimer_.reset();
    if (specs) {
        sendControl(Cmd::FORWARD_SAMPLE, n, tokens, positions, slots);
        for (auto &s : workers_) s.sendAll(specs, n * sizeof(SampleSpec));
    } else {
        sendControl(Cmd::FORWARD_ARGMAX, n, tokens, positions, slots);
    }
    backend_->launchIds(n, tokens, positions, slots, specs);
    launchedSample_ = specs != nullptr;
}

void InferenceSession::chainLaunch(int token, int pos, int slot) {
    if (token >= 0) launchTimer_.reset();
    sendControl(Cmd::CHAIN, 1, &token, &pos, &slot);
    backend_->chainLaunch(token, pos, slot);
}

int InferenceSession::chainCollect() {
    const int id = backend_->chainCollect();
    recordMetrics("forward_argmax", 1, launchTimer_.elapsedMs());
    launchTimer_.reset();
    return id;
}

void InferenceSession::collectIds(int n, int *out) {
    backend_->collectIds(out);
    recordMetrics(launchedSample_ ? "forward_sample" : "forward_argmax", n, launchTimer_.elapsedMs());
}

void InferenceSession::recordMetrics(const char *kind, int n, double ms) {
    MetricsSink &m = MetricsSink::global();
    if (!m.enabled()) return;
    unsigned long long sent = 0, recv = 0;  // cumulative socket bytes (control plane; CPU data plane)
    for (auto &w : workers_) {
        sent += w.totalSentBytes();
        recv += w.totalRecvBytes();
    }
    const ForwardStats st = backend_->lastStats();
    // this forward: the sockets' bytes since the previous record, plus (GPUs) the device data plane
    // the engine counted for this forward alone (the CPU data plane is the sockets above)
    const unsigned long long fs = sent - mSent_ + (gpu_ ? st.sentBytes : 0);
    const unsigned long long fr = recv - mRecv_ + (gpu_ ? st.recvBytes : 0);
    mSent_ = sent;
    mRecv_ = recv;
    char buf[512], xchg[32];
    // xchg_ms: the exchange span (null when not measured: DL_SYNC_MEASURE < 2 on the fused exchange)
    if (st.xchgMs >= 0) std::snprintf(xchg, sizeof(xchg), "%.4f", st.xchgMs);
    else std::snprintf(xchg, sizeof(xchg), "null");
    std::snprintf(buf, sizeof(buf),
                  "{\"ts_ms\":%.3f,\"event\":\"%s\",\"rows\":%d,\"ms\":%.4f,\"compute_ms\":%.4f,\"sync_ms\":%.4f,"
                  "\"xchg_ms\":%s,\"sent_bytes\":%llu,\"recv_bytes\":%llu,\"nodes\":%d,\"backend\":\"%s\"}",
                  epochMs(), kind, n, ms, st.computeMs, st.syncMs, xchg, fs, fr, nNodes(), gpu_ ? "hip" : "cpu");
    m.write(buf);
}

bool InferenceSession::profileForward(int n, const int *tokens, const int *positions, const int *slots) {
    HipEngine *e = dynamic_cast<HipEngine *>(backend_.get());
    if (!e || !workers_.empty()) return false;  // single-process GPU runs only
    e->profileForward(n, tokens, positions, slots);
    return true;
}

ForwardStats InferenceSession::lastStats() {
    // bytes since the previous call (the reference resets its counters on read, nn-network.cpp:493-501):
    // the backend's device data plane (GPU tensor parallelism over xGMI / RCCL: the engine's own count
    // of the exchanged partials and logits) plus the control plane's sockets (and, on CPUs, the TCP
    // data plane, whose sockets are these same ones: the CPU backend's own count is not added).
    ForwardStats s = backend_->lastStats();
    if (!gpu_) s.sentBytes = s.recvBytes = 0;
    for (auto &w : workers_) {
        s.sentBytes += w.sentBytes();
        s.recvBytes += w.recvBytes();
        w.resetStats();
    }
    return s;
}

void InferenceSession::finish() {
    if (finished_) return;
    finished_ = true;
    int hdr[2] = {(int)Cmd::STOP, 0};
    for (auto &s : workers_) {
        try {
            s.sendAll(hdr, sizeof(hdr));
        } catch (...) {
        }
    }
}

void runWorker(const AppArgs &args) {
    ServerSocket server(args.port);
    while (true) {
        if (logLevel() >= 1) std::printf("⭕ Listening on port %d...\n", args.port);
        std::fflush(stdout);
        Socket root = server.accept();
        try {
            if (root.recvPod<u32>() != kProtoMagic) throw NetError("bad magic from root");
            WorkerConfig wc = decodeWorkerConfig(root.recvString());
            if (logLevel() >= 1) std::printf("⭕ Root connected; rank %u of %u (%s)\n", wc.rank, wc.world, wc.gpu ? "gpu" : "cpu");
            EngineConfig ec = wc.engine;
            std::string streamedFile;
            if (!ec.synthetic && (args.streamWeights || ::access(ec.modelPath.c_str(), R_OK) != 0)) {
                root.sendPod<u32>(kWantWeights);
                const size_t slash = ec.modelPath.find_last_of('/');
                streamedFile = args.weightsCache + "/dllama_r" + std::to_string(wc.rank) + "_" +
                               (slash == std::string::npos ? ec.modelPath : ec.modelPath.substr(slash + 1));
                const u64 got = fetchWeights(root, streamedFile, wc.rank, wc.world);
                if (logLevel() >= 1)
                    std::printf("💿 Received %llu MB of weight slices -> %s\n", (unsigned long long)(got >> 20),
                                streamedFile.c_str());
                ec.modelPath = streamedFile;
            } else {
                root.sendPod<u32>(kHaveWeights);
            }
            struct Cleanup {
                std::string path;
                ~Cleanup() {
                    if (!path.empty()) ::unlink(path.c_str());
                }
            } cleanup{streamedFile};
            ec.nThreads = args.nThreads;
            ec.gpuIndex = args.gpuIndex >= 0 ? args.gpuIndex : (wc.gpu ? (int)wc.rank : -1);
            ec.useGraphs = ec.useGraphs && args.graphs;
            std::vector<Socket> mesh;  // CPU data plane sockets to the other workers
            std::unique_ptr<HostComm> hc;
            std::unique_ptr<DeviceComm> dc;
            std::unique_ptr<Backend> backend;
            try {
                if (wc.gpu) {
                    DL_HIP(hipSetDevice(ec.gpuIndex));
                    if (wc.devComm == "xgmi") {
                        dc = makeXgmiComm((int)wc.rank, (int)wc.world, wc.xgmiMaxFloats);  // failure: reported below
                        root.sendPod<u32>(kAck);
                        root.sendString(xgmiHandle(dc.get()));
                        std::vector<std::string> handles(wc.world);
                        for (auto &hnd : handles) hnd = root.recvString();
                        xgmiConnect(dc.get(), handles);
                    } else {
                        dc = makeRcclComm(wc.rcclUid, (int)wc.rank, (int)wc.world);
                    }
                } else {
                    // full mesh: connect to the higher ranks (their listen backlog takes the
                    // connection before they accept), then accept the lower ones
                    mesh.reserve(wc.world);
                    std::vector<Socket *> byRank(wc.world, nullptr);
                    byRank[0] = &root;
                    for (u32 r = wc.rank + 1; r < wc.world; r++) {
                        DL_CHECK(r - 1 < wc.peerHosts.size(), "config lacks peer addresses");
                        mesh.push_back(Socket::connectTo(wc.peerHosts[r - 1], wc.peerPorts[r - 1]));
                        mesh.back().sendPod<u32>(kMeshMagic);
                        mesh.back().sendPod<u32>(wc.rank);
                        byRank[r] = &mesh.back();
                    }
                    for (u32 k = 1; k < wc.rank; k++) {
                        mesh.push_back(server.accept());
                        if (mesh.back().recvPod<u32>() != kMeshMagic) throw NetError("bad magic from a peer worker");
                        const u32 r = mesh.back().recvPod<u32>();
                        if (r == 0 || r >= wc.rank || byRank[r]) throw NetError("unexpected peer rank");
                        byRank[r] = &mesh.back();
                    }
                    if (logLevel() >= 1)
                        std::printf("⭕ Data-plane mesh: %u peer sockets\n", wc.world - 1);
                    hc.reset(new TcpHostComm((int)wc.rank, (int)wc.world, byRank));
                }
                backend = makeBackend(ec, wc.gpu, hc.get(), dc.get());
            } catch (const std::exception &e) {
                root.sendPod<u32>(0);
                root.sendString(e.what());
                throw;
            }
            root.sendPod<u32>(kAck);
            if (logLevel() >= 1) std::printf("💿 Weights loaded\n");
            std::fflush(stdout);
            std::vector<int> buf, ids;
            std::vector<SampleSpec> specs;
            while (true) {
                int hdr[2];
                root.recvAll(hdr, sizeof(hdr));
                const Cmd cmd = (Cmd)hdr[0];
                const int n = hdr[1];
                if (cmd != Cmd::CHAIN)  // chained steps finish before anything else runs
                    while (backend->chainInFlight() > 0) backend->chainCollect();
                if (cmd == Cmd::STOP) {
                    if (logLevel() >= 1) std::printf("🛑 Stop signal\n");
                    break;
                }
                buf.resize(3 * (size_t)n);
                root.recvAll(buf.data(), buf.size() * sizeof(int));
                if (cmd == Cmd::FORWARD) {
                    backend->forward(n, &buf[0], &buf[n], &buf[2 * n], nullptr);
                } else if (cmd == Cmd::FORWARD_ARGMAX) {
                    ids.resize(n);
                    backend->forwardArgmax(n, &buf[0], &buf[n], &buf[2 * n], ids.data());
                } else if (cmd == Cmd::CHAIN) {
                    backend->chainLaunch(buf[0], buf[n], buf[2 * n]);
                    while (backend->chainInFlight() > 2) backend->chainCollect();
                } else if (cmd == Cmd::RELEASE) {
                    for (int i = 0; i < n; i++) backend->releaseSlot(buf[i]);
                } else if (cmd == Cmd::FORWARD_SAMPLE) {
                    ids.resize(n);
                    specs.resize(n);
                    root.recvAll(specs.data(), n * sizeof(SampleSpec));
                    backend->forwardSample(n, &buf[0], &buf[n], &buf[2 * n], specs.data(), ids.data());
                }
            }
        } catch (const NetError &e) {
            std::printf("Network exception: %s\n", e.what());
        } catch (const std::exception &e) {
            std::printf("🚨 Worker error: %s\n", e.what());
        }
        std::fflush(stdout);
    }
}

}  // namespace dl
