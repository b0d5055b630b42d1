#include "model_file.h"

#include <atomic>
#include <cerrno>
#include <thread>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

namespace dl {

namespace {
enum HeaderKey {
    K_VERSION = 0,
    K_ARCH_TYPE = 1,
    K_DIM = 2,
    K_HIDDEN_DIM = 3,
    K_N_LAYERS = 4,
    K_N_HEADS = 5,
    K_N_KV_HEADS = 6,
    K_N_EXPERTS = 7,
    K_N_ACTIVE_EXPERTS = 8,
    K_VOCAB_SIZE = 9,
    K_SEQ_LEN = 10,
    K_HIDDEN_ACT = 11,
    K_ROPE_THETA = 12,
    K_WEIGHT_FLOAT_TYPE = 13,
    K_ROPE_SCALING_FACTOR = 14,
    K_ROPE_SCALING_LOW = 15,
    K_ROPE_SCALING_HIGH = 16,
    K_ROPE_SCALING_ORIG = 17,
    K_ROPE_TYPE = 18,
};
}  // namespace

ModelHeader parseModelHeader(const u8 *data, u64 size) {
    DL_CHECK(size >= 8, "model file too small");
    i32 magic, headerSize;
    std::memcpy(&magic, data, 4);
    std::memcpy(&headerSize, data + 4, 4);
    if (magic == 0xABCD00 || magic == 0xABCD01) throw Error("Old model format is not supported");
    if (magic != kModelMagic) throw Error("Unsupported magic number");
    DL_CHECK(headerSize >= 8 && (u64)headerSize <= size, "bad header size");
    ModelHeader h;
    h.headerSize = headerSize;
    const int nInts = (headerSize - 8) / 4;
    DL_CHECK(nInts % 2 == 0, "odd number of header ints");
    for (int i = 0; i < nInts; i += 2) {
        i32 key, value;
        std::memcpy(&key, data + 8 + 4 * i, 4);
        std::memcpy(&value, data + 8 + 4 * (i + 1), 4);
        switch (key) {
            case K_VERSION: h.version = value; break;
            case K_ARCH_TYPE: h.archType = value; break;
            case K_DIM: h.dim = value; break;
            case K_HIDDEN_DIM: h.hiddenDim = value; break;
            case K_N_LAYERS: h.nLayers = value; break;
            case K_N_HEADS: h.nHeads = value; break;
            case K_N_KV_HEADS: h.nKvHeads = value; break;
            case K_N_EXPERTS: h.nExperts = value; break;
            case K_N_ACTIVE_EXPERTS: h.nActiveExperts = value; break;
            case K_VOCAB_SIZE: h.vocabSize = value; break;
            case K_SEQ_LEN: h.seqLen = value; break;
            case K_HIDDEN_ACT: h.hiddenAct = (HiddenAct)value; break;
            case K_ROPE_THETA: h.ropeTheta = (float)value; break;
            case K_WEIGHT_FLOAT_TYPE: h.weightType = (FloatType)value; break;
            case K_ROPE_SCALING_FACTOR: h.ropeScalingFactor = (float)value; break;
            case K_ROPE_SCALING_LOW: h.ropeScalingLowFreqFactor = (float)value; break;
            case K_ROPE_SCALING_HIGH: h.ropeScalingHighFreqFactor = (float)value; break;
            case K_ROPE_SCALING_ORIG: h.ropeScalingOrigMaxSeqLen = value; break;
            case K_ROPE_TYPE: h.ropeType = (RopeType)value; break;
            default: throw Error("Unsupported header key: " + std::to_string(key));
        }
    }
    if (h.weightType == FloatType::UNK) throw Error("Model does not specify weight type");
    if (h.archType != kArchLlama) throw Error("Unsupported architecture");
    DL_CHECK(h.dim > 0 && h.nHeads > 0 && h.nKvHeads > 0 && h.nLayers > 0 && h.vocabSize > 0, "incomplete header");
    DL_CHECK(h.dim % h.nHeads == 0 && h.nHeads % h.nKvHeads == 0, "head dims");
    h.origSeqLen = h.seqLen;
    h.fileSize = (i64)size;
    return h;
}

ModelHeader loadModelHeader(const std::string &path, u32 maxSeqLen) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) throw Error("Cannot open model file: " + path);
    std::vector<u8> buf(8);
    if (std::fread(buf.data(), 1, 8, f) != 8) {
        std::fclose(f);
        throw Error("Cannot read model header");
    }
    i32 headerSize;
    std::memcpy(&headerSize, buf.data() + 4, 4);
    if (headerSize > 8 && headerSize < (1 << 20)) {
        buf.resize(headerSize);
        if (std::fread(buf.data() + 8, 1, headerSize - 8, f) != (size_t)(headerSize - 8)) {
            std::fclose(f);
            throw Error("Cannot read header values");
        }
    }
    std::fseek(f, 0, SEEK_END);
    const i64 fileSize = std::ftell(f);
    std::fclose(f);
    ModelHeader h = parseModelHeader(buf.data(), buf.size());
    h.fileSize = fileSize;
    if (maxSeqLen > 0 && h.seqLen > maxSeqLen) h.seqLen = maxSeqLen;
    return h;
}

static const char *hiddenActName(HiddenAct a) { return a == HiddenAct::GELU ? "Gelu" : "Silu"; }
static const char *ropeTypeName(RopeType t) {
    switch (t) {
        case RopeType::LLAMA: return "Llama";
        case RopeType::FALCON: return "Falcon";
        case RopeType::LLAMA3_1: return "Llama3.1";
    }
    return "Unknown";
}

void printModelHeader(const ModelHeader &h) {
    if (logLevel() < 1) return;
    std::printf("💡 Arch: Llama\n");
    std::printf("💡 HiddenAct: %s\n", hiddenActName(h.hiddenAct));
    std::printf("💡 Dim: %u\n", h.dim);
    std::printf("💡 KvDim: %u\n", h.kvDim());
    std::printf("💡 HiddenDim: %u\n", h.hiddenDim);
    std::printf("💡 VocabSize: %u\n", h.vocabSize);
    std::printf("💡 nLayers: %u\n", h.nLayers);
    std::printf("💡 nHeads: %u\n", h.nHeads);
    std::printf("💡 nKvHeads: %u\n", h.nKvHeads);
    if (h.seqLen != h.origSeqLen) std::printf("💡 OrigSeqLen: %u\n", h.origSeqLen);
    std::printf("💡 SeqLen: %u\n", h.seqLen);
    std::printf("💡 NormEpsilon: %f\n", h.normEpsilon);
    std::printf("💡 RopeType: %s\n", ropeTypeName(h.ropeType));
    std::printf("💡 RopeTheta: %.0f\n", h.ropeTheta);
    if (h.ropeType == RopeType::LLAMA3_1)
        std::printf("💡 RopeScaling: f=%.1f, l=%.1f, h=%.1f, o=%u\n", h.ropeScalingFactor, h.ropeScalingLowFreqFactor,
                    h.ropeScalingHighFreqFactor, h.ropeScalingOrigMaxSeqLen);
    std::fflush(stdout);
}

const char *tensorKindName(TensorKind k) {
    switch (k) {
        case TensorKind::EMBEDDING: return "embedding";
        case TensorKind::WQ: return "block_matmul_q";
        case TensorKind::WK: return "block_matmul_k";
        case TensorKind::WV: return "block_matmul_v";
        case TensorKind::WO: return "block_matmul_wo";
        case TensorKind::W1: return "block_matmul_w1";
        case TensorKind::W2: return "block_matmul_w2";
        case TensorKind::W3: return "block_matmul_w3";
        case TensorKind::RMS_ATT: return "block_rms_norm_0";
        case TensorKind::RMS_FFN: return "block_rms_norm_1";
        case TensorKind::RMS_FINAL: return "final_rms_norm";
        case TensorKind::WCLS: return "final_matmul_logits";
    }
    return "?";
}

std::vector<TensorInfo> buildTensorTable(const ModelHeader &h) {
    if (h.nExperts > 0) throw Error("Mixture-of-experts models are not supported by this runtime");
    if (h.weightType != FloatType::F32 && h.weightType != FloatType::Q40)
        throw Error(std::string("Unsupported weight type: ") + floatTypeName(h.weightType));
    std::vector<TensorInfo> t;
    u64 off = (u64)h.headerSize;
    auto add = [&](TensorKind k, int layer, FloatType type, u32 rows, u32 cols) {
        const u64 bytes = floatTypeBytes(type, (u64)rows * cols);
        t.push_back(TensorInfo{k, layer, off, bytes, type, rows, cols});
        off += bytes;
    };
    const FloatType w = h.weightType;
    const u32 kv = h.kvDim();
    add(TensorKind::EMBEDDING, -1, FloatType::F32, h.vocabSize, h.dim);
    for (u32 l = 0; l < h.nLayers; l++) {
        add(TensorKind::WQ, l, w, h.dim, h.dim);
        add(TensorKind::WK, l, w, kv, h.dim);
        add(TensorKind::WV, l, w, kv, h.dim);
        add(TensorKind::WO, l, w, h.dim, h.dim);
        add(TensorKind::W1, l, w, h.hiddenDim, h.dim);
        add(TensorKind::W2, l, w, h.dim, h.hiddenDim);
        add(TensorKind::W3, l, w, h.hiddenDim, h.dim);
        add(TensorKind::RMS_ATT, l, FloatType::F32, 1, h.dim);
        add(TensorKind::RMS_FFN, l, FloatType::F32, 1, h.dim);
    }
    add(TensorKind::RMS_FINAL, -1, FloatType::F32, 1, h.dim);
    add(TensorKind::WCLS, -1, w, h.vocabSize, h.dim);
    if (h.fileSize > 0 && (i64)off != h.fileSize)
        throw Error("Missing bytes in weight file: " + std::to_string((i64)off - h.fileSize));
    return t;
}

MappedFile::MappedFile(const std::string &path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw Error("Cannot open file: " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0) throw Error("fstat failed: " + path);
    size_ = (u64)st.st_size;
    void *p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) throw Error("mmap failed: " + path);
    data_ = (const u8 *)p;
}

MappedFile::~MappedFile() {
    if (data_) ::munmap((void *)data_, size_);
    if (fd_ >= 0) ::close(fd_);
}

ParallelReader::ParallelReader(const std::string &path, int threads, u64 piece) : piece_(piece), path_(path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw Error("Cannot open file: " + path);
    if (threads <= 0) {
        const unsigned hw = std::thread::hardware_concurrency();
        threads = (int)std::min<unsigned>(hw ? hw : 4, 16);
    }
    threads_ = threads;
}

ParallelReader::~ParallelReader() {
    if (fd_ >= 0) ::close(fd_);
}

void ParallelReader::read(u64 off, u64 len, void *dst) { readMany({{off, len, dst}}); }

void ParallelReader::readMany(const std::vector<Range> &ranges) {
    struct Part {
        u64 off, len;
        u8 *dst;
    };
    std::vector<Part> parts;
    u64 total = 0;
    for (const Range &r : ranges) {
        total += r.len;
        for (u64 o = 0; o < r.len; o += piece_)
            parts.push_back({r.off + o, std::min(piece_, r.len - o), (u8 *)r.dst + o});
    }
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    auto work = [&] {
        for (size_t i = next++; i < parts.size() && !failed; i = next++) {
            const Part &p = parts[i];
            u64 done = 0;
            while (done < p.len) {
                const ssize_t r = ::pread(fd_, p.dst + done, p.len - done, (off_t)(p.off + done));
                if (r < 0 && errno == EINTR) continue;
                if (r <= 0) {
                    failed = true;
                    break;
                }
                done += (u64)r;
            }
        }
    };
    const int nt = (int)std::min<size_t>((size_t)threads_, parts.size());
    if (nt <= 1) {
        work();
    } else {
        std::vector<std::thread> pool;
        for (int t = 0; t < nt; t++) pool.emplace_back(work);
        for (auto &t : pool) t.join();
    }
    if (failed) throw Error("short read from " + path_);
    bytes_ += total;
}

ModelFile::ModelFile(const std::string &path, u32 maxSeqLen) : path_(path) {
    file_.reset(new MappedFile(path));
    header_ = parseModelHeader(file_->data(), file_->size());
    if (maxSeqLen > 0 && header_.seqLen > maxSeqLen) header_.seqLen = maxSeqLen;
    tensors_ = buildTensorTable(header_);
}

const TensorInfo &ModelFile::find(TensorKind kind, int layer) const {
    for (const auto &t : tensors_)
        if (t.kind == kind && t.layer == layer) return t;
    throw Error(std::string("tensor not found: ") + tensorKindName(kind));
}

}  // namespace dl
