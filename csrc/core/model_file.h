// `.m` model file: header parsing, tensor table and memory-mapped access.
//
// Byte-compatible with the reference format:
//   header keys / defaults / magic       src/llm.hpp:8-67, src/llm.cpp:26-98, converter/writer.py:109-145
//   tensor order                         src/llm.cpp:447-483
// The tensor table is computed once from the header (no graph IR), and every rank reads
// its own shard straight out of the mapping.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "common.h"

namespace dl {

enum class HiddenAct : int { GELU = 0, SILU = 1 };
enum class RopeType : int { LLAMA = 0, FALCON = 1, LLAMA3_1 = 2 };
constexpr int kArchLlama = 0xABCD00;
constexpr int kModelMagic = 0xA00ABCD;

struct ModelHeader {
    i64 headerSize = 0;
    i64 fileSize = 0;
    int version = 0;
    int archType = kArchLlama;
    u32 dim = 0;
    u32 hiddenDim = 0;
    u32 nLayers = 0;
    u32 nHeads = 0;
    u32 nKvHeads = 0;
    u32 nExperts = 0;
    u32 nActiveExperts = 0;
    u32 vocabSize = 0;
    u32 origSeqLen = 0;
    u32 seqLen = 0;
    HiddenAct hiddenAct = HiddenAct::SILU;
    float ropeTheta = 10000.0f;
    RopeType ropeType = RopeType::LLAMA;
    float ropeScalingFactor = 1.0f;
    float ropeScalingLowFreqFactor = 0.0f;
    float ropeScalingHighFreqFactor = 0.0f;
    u32 ropeScalingOrigMaxSeqLen = 0;
    float normEpsilon = 1e-5f;
    FloatType weightType = FloatType::UNK;

    u32 headSize() const { return dim / nHeads; }
    u32 kvDim() const { return dim / nHeads * nKvHeads; }
};

// Parse a header from a file; `maxSeqLen` > 0 clamps seqLen (llm.cpp:88-91).
ModelHeader loadModelHeader(const std::string &path, u32 maxSeqLen = 0);
// Parse from raw bytes (the first bytes of a file).
ModelHeader parseModelHeader(const u8 *data, u64 size);
void printModelHeader(const ModelHeader &h);

enum class TensorKind : int { EMBEDDING, WQ, WK, WV, WO, W1, W2, W3, RMS_ATT, RMS_FFN, RMS_FINAL, WCLS };
const char *tensorKindName(TensorKind k);

struct TensorInfo {
    TensorKind kind;
    int layer;       // -1 for global tensors
    u64 offset;      // byte offset in the file
    u64 bytes;
    FloatType type;
    u32 rows;        // output dim (d)
    u32 cols;        // input dim (n)
};

// All tensors in file order. Throws if the header and file size disagree (llm.cpp:477-479).
std::vector<TensorInfo> buildTensorTable(const ModelHeader &h);

class MappedFile {
  public:
    explicit MappedFile(const std::string &path);
    ~MappedFile();
    MappedFile(const MappedFile &) = delete;
    MappedFile &operator=(const MappedFile &) = delete;
    const u8 *data() const { return data_; }
    u64 size() const { return size_; }

  private:
    const u8 *data_ = nullptr;
    u64 size_ = 0;
    int fd_ = -1;
};

// Positional reads of a file split over a pool of threads (pread, no page-cache mapping faults
// on the load path): large weight slices are read in `piece`-byte parts concurrently, which is
// what lets a multi-GB shard leave NVMe / the page cache at several GB/s (the mapping is
// single-threaded per fault). Thread-safe for concurrent read() calls on disjoint outputs.
class ParallelReader {
  public:
    explicit ParallelReader(const std::string &path, int threads = 0, u64 piece = 8ull << 20);
    ~ParallelReader();
    ParallelReader(const ParallelReader &) = delete;
    ParallelReader &operator=(const ParallelReader &) = delete;
    // [off, off + len) of the file into dst; throws on a short read.
    void read(u64 off, u64 len, void *dst);
    // Several ranges at once (one parallel batch): ranges[i] = {file offset, length, dst}.
    struct Range {
        u64 off, len;
        void *dst;
    };
    void readMany(const std::vector<Range> &ranges);
    u64 bytesRead() const { return bytes_; }
    int threads() const { return threads_; }

  private:
    int fd_ = -1;
    int threads_ = 1;
    u64 piece_;
    u64 bytes_ = 0;
    std::string path_;
};

// A model opened for reading: header + table + mapping.
class ModelFile {
  public:
    ModelFile(const std::string &path, u32 maxSeqLen = 0);
    const ModelHeader &header() const { return header_; }
    const std::vector<TensorInfo> &tensors() const { return tensors_; }
    const TensorInfo &find(TensorKind kind, int layer) const;
    const u8 *ptr(const TensorInfo &t) const { return file_->data() + t.offset; }
    const std::string &path() const { return path_; }

  private:
    std::string path_;
    ModelHeader header_;
    std::vector<TensorInfo> tensors_;
    std::unique_ptr<MappedFile> file_;
};

}  // namespace dl
