#include "weight_stream.h"

#include <algorithm>
#include <cstdio>
#include <cstring>

#include <fcntl.h>
#include <unistd.h>

namespace dl {

std::vector<ByteRange> shardByteRanges(const ModelHeader &h, const std::vector<TensorInfo> &tensors,
                                       const ShardPlan &p) {
    std::vector<ByteRange> r;
    auto rowsOf = [&](const TensorInfo &t, u32 r0, u32 nr) {
        const u64 rowBytes = floatTypeBytes(t.type, t.cols);
        r.push_back({t.offset + r0 * rowBytes, nr * rowBytes});
    };
    auto colsOf = [&](const TensorInfo &t, u32 c0, u32 nc) {
        const u64 rowBytes = floatTypeBytes(t.type, t.cols);
        const u64 off = floatTypeBytes(t.type, c0), len = floatTypeBytes(t.type, nc);
        for (u32 row = 0; row < t.rows; row++) r.push_back({t.offset + row * rowBytes + off, len});
    };
    for (const TensorInfo &t : tensors) {
        switch (t.kind) {
            case TensorKind::WQ: rowsOf(t, p.qStart(), p.q0); break;
            case TensorKind::WK:
            case TensorKind::WV: rowsOf(t, p.kvStart(), p.kv0); break;
            case TensorKind::WO: colsOf(t, p.qStart(), p.q0); break;
            case TensorKind::W1:
            case TensorKind::W3: rowsOf(t, p.hiddenStart(), p.hidden0); break;
            case TensorKind::W2: colsOf(t, p.hiddenStart(), p.hidden0); break;
            case TensorKind::WCLS: rowsOf(t, p.vocabStart(), p.vocab0); break;
            default: r.push_back({t.offset, t.bytes}); break;  // embedding, norms
        }
    }
    (void)h;
    std::sort(r.begin(), r.end(), [](const ByteRange &a, const ByteRange &b) { return a.offset < b.offset; });
    std::vector<ByteRange> merged;
    for (const ByteRange &x : r) {
        if (x.length == 0) continue;
        if (!merged.empty() && merged.back().offset + merged.back().length >= x.offset) {
            const u64 end = std::max(merged.back().offset + merged.back().length, x.offset + x.length);
            merged.back().length = end - merged.back().offset;
        } else {
            merged.push_back(x);
        }
    }
    return merged;
}

void serveWeights(Socket &s, const std::string &modelPath) {
    MappedFile f(modelPath);
    const ModelHeader h = parseModelHeader(f.data(), f.size());
    s.sendPod<u64>(f.size());
    s.sendPod<u64>((u64)h.headerSize);
    s.sendAll(f.data(), (u64)h.headerSize);
    const u64 n = s.recvPod<u64>();
    std::vector<ByteRange> ranges(n);
    if (n) s.recvAll(ranges.data(), n * sizeof(ByteRange));
    for (const ByteRange &r : ranges) {
        if (r.offset + r.length > f.size()) throw NetError("weight request out of range");
        s.sendAll(f.data() + r.offset, r.length);
    }
}

u64 fetchWeights(Socket &root, const std::string &cachePath, u32 rank, u32 world) {
    const u64 fileSize = root.recvPod<u64>();
    const u64 headerSize = root.recvPod<u64>();
    std::vector<u8> header(headerSize);
    root.recvAll(header.data(), headerSize);
    ModelHeader h = parseModelHeader(header.data(), headerSize);
    h.fileSize = (i64)fileSize;
    const std::vector<TensorInfo> tensors = buildTensorTable(h);
    const ShardPlan plan = ShardPlan::make(h, world, rank);
    const std::vector<ByteRange> ranges = shardByteRanges(h, tensors, plan);
    root.sendPod<u64>(ranges.size());
    if (!ranges.empty()) root.sendAll(ranges.data(), ranges.size() * sizeof(ByteRange));

    const int fd = ::open(cachePath.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
    if (fd < 0) throw Error("cannot create weight cache file " + cachePath);
    u64 received = 0;
    try {
        if (::ftruncate(fd, (off_t)fileSize) != 0) throw Error("cannot size weight cache file");
        if (::pwrite(fd, header.data(), headerSize, 0) != (ssize_t)headerSize) throw Error("write failed");
        std::vector<u8> buf(8u << 20);
        for (const ByteRange &r : ranges) {
            u64 done = 0;
            while (done < r.length) {
                const u64 chunk = std::min<u64>(buf.size(), r.length - done);
                root.recvAll(buf.data(), chunk);
                if (::pwrite(fd, buf.data(), chunk, (off_t)(r.offset + done)) != (ssize_t)chunk)
                    throw Error("write failed on weight cache file");
                done += chunk;
            }
            received += r.length;
        }
    } catch (...) {
        ::close(fd);
        throw;
    }
    ::close(fd);
    return received;
}

}  // namespace dl
