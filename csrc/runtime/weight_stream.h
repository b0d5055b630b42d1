// Root -> worker weight streaming for workers that do not have the model file (reference:
// NnRootWeightLoader / NnWorkerWeightReader, nn-network.cpp:799-901).
//
// The worker receives the header bytes, builds the tensor table and its own ShardPlan, asks for
// exactly the byte ranges its backend reads (row slices, per-row column slices, whole norms and the
// embedding), and writes them into a sparse local copy of the model file at their original offsets;
// the normal mmap loader then opens that copy. Only ~1/N of the weights crosses the wire per worker.
#pragma once

#include <string>
#include <vector>

#include "../core/model_file.h"
#include "../core/plan.h"
#include "../net/tcp.h"

namespace dl {

struct ByteRange {
    u64 offset, length;
};

// File byte ranges a rank's backend reads (sorted, adjacent ranges merged).
std::vector<ByteRange> shardByteRanges(const ModelHeader &h, const std::vector<TensorInfo> &tensors,
                                       const ShardPlan &plan);

constexpr u32 kHaveWeights = 0x57454931u;   // worker found the model file locally
constexpr u32 kWantWeights = 0x57454932u;   // worker asks the root to stream its slices

// Root side: answer one worker's requests from the root's model file.
void serveWeights(Socket &s, const std::string &modelPath);
// Worker side: fetch this rank's slices into `cachePath` (sparse file); returns bytes received.
u64 fetchWeights(Socket &root, const std::string &cachePath, u32 rank, u32 world);

}  // namespace dl
