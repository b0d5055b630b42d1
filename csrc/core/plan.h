// Tensor-parallel shard plan: which slice of every tensor a rank owns.
//
// Same partition as the reference's slicers (src/nn/nn-core.cpp:198-266, llm.cpp:131-142):
//   Wq/Wk/Wv/W1/W3/Wcls: row (output) slices   -> "column-parallel"
//   Wo/W2:               column (input) slices  -> partial sums, all-reduced
//   norms / embedding:   replicated on every rank (every rank gathers its own embedding row,
//                        removing the reference's per-token X broadcast, llm.cpp:193)
// Constraint: nRanks divides nKvHeads (app.cpp:237-238 only requires <=, divisibility is what
// the slicers assert).
#pragma once

#include <vector>

#include "model_file.h"

namespace dl {

struct ShardPlan {
    u32 nRanks = 1;
    u32 rank = 0;
    u32 dim = 0;
    u32 headSize = 0;
    u32 nHeads0 = 0;    // query heads on this rank
    u32 nKvHeads0 = 0;  // kv heads on this rank
    u32 q0 = 0;         // = nHeads0 * headSize
    u32 kv0 = 0;        // = nKvHeads0 * headSize
    u32 hidden0 = 0;    // hiddenDim / nRanks
    u32 vocab0 = 0;     // vocabSize / nRanks
    u32 kvMul = 1;      // query heads per kv head

    // global start offsets of this rank's slices
    u32 qStart() const { return rank * q0; }
    u32 kvStart() const { return rank * kv0; }
    u32 hiddenStart() const { return rank * hidden0; }
    u32 vocabStart() const { return rank * vocab0; }

    static ShardPlan make(const ModelHeader &h, u32 nRanks, u32 rank);
};

// Row-major [rows][cols] tensor of type `type`: copy rows [r0, r0+nr) (a contiguous byte range).
void sliceRows(const u8 *src, FloatType type, u32 cols, u32 r0, u32 nr, u8 *dst);
// Copy the column range [c0, c0+nc) of every row (block aligned for quantized types).
void sliceCols(const u8 *src, FloatType type, u32 rows, u32 cols, u32 c0, u32 nc, u8 *dst);

// RoPE cos/sin table [seqLen][headSize/2] of (cos, sin) pairs, with the Llama-3.1 frequency
// scaling applied when ropeScalingFactor != 1 (nn-core.cpp:307-340).
std::vector<float> buildRopeTable(const ModelHeader &h);

}  // namespace dl
