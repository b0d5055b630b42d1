#include "plan.h"

#include <cmath>
#include <cstring>

namespace dl {

ShardPlan ShardPlan::make(const ModelHeader &h, u32 nRanks, u32 rank) {
    DL_CHECK(nRanks >= 1 && rank < nRanks, "bad rank/world");
    if (nRanks > h.nKvHeads)
        throw Error("This version does not support more nodes than the number of KV heads in the model");
    DL_CHECK(h.nKvHeads % nRanks == 0, "nKvHeads must be divisible by the number of ranks");
    DL_CHECK(h.hiddenDim % (nRanks * kQBlock) == 0, "hiddenDim must split into 32-aligned shards");
    DL_CHECK(h.vocabSize % nRanks == 0, "vocabSize must be divisible by the number of ranks");
    ShardPlan p;
    p.nRanks = nRanks;
    p.rank = rank;
    p.dim = h.dim;
    p.headSize = h.headSize();
    p.nHeads0 = h.nHeads / nRanks;
    p.nKvHeads0 = h.nKvHeads / nRanks;
    p.q0 = p.nHeads0 * p.headSize;
    p.kv0 = p.nKvHeads0 * p.headSize;
    p.hidden0 = h.hiddenDim / nRanks;
    p.vocab0 = h.vocabSize / nRanks;
    p.kvMul = h.nHeads / h.nKvHeads;
    DL_CHECK(p.q0 % kQBlock == 0, "q shard must be 32-aligned");
    return p;
}

void sliceRows(const u8 *src, FloatType type, u32 cols, u32 r0, u32 nr, u8 *dst) {
    const u64 rowBytes = floatTypeBytes(type, cols);
    std::memcpy(dst, src + rowBytes * r0, rowBytes * nr);
}

void sliceCols(const u8 *src, FloatType type, u32 rows, u32 cols, u32 c0, u32 nc, u8 *dst) {
    const u64 rowBytes = floatTypeBytes(type, cols);
    const u64 offBytes = floatTypeBytes(type, c0);
    const u64 sliceBytes = floatTypeBytes(type, nc);
    for (u32 r = 0; r < rows; r++) std::memcpy(dst + r * sliceBytes, src + r * rowBytes + offBytes, sliceBytes);
}

static float scaleFreqLlama31(float freq, const ModelHeader &h) {
    // Llama 3.1 frequency scaling: keep high frequencies, divide low ones by the factor and
    // blend in between.
    const float waveLen = 2.0f * (float)M_PI / freq;
    const float orig = (float)h.ropeScalingOrigMaxSeqLen;
    const float highWave = orig / h.ropeScalingHighFreqFactor;
    if (waveLen < highWave) return freq;
    const float lowWave = orig / h.ropeScalingLowFreqFactor;
    if (waveLen > lowWave) return freq / h.ropeScalingFactor;
    const float smooth =
        (orig / waveLen - h.ropeScalingLowFreqFactor) / (h.ropeScalingHighFreqFactor - h.ropeScalingLowFreqFactor);
    return (1.0f - smooth) * freq / h.ropeScalingFactor + smooth * freq;
}

std::vector<float> buildRopeTable(const ModelHeader &h) {
    const u32 hs = h.headSize();
    const u32 half = hs / 2;
    std::vector<float> t((size_t)h.seqLen * half * 2);
    const bool scale = h.ropeScalingFactor != 1.0f;
    std::vector<float> freqs(half);
    for (u32 i = 0; i < half; i++) {
        float f = 1.0f / powf(h.ropeTheta, (float)(2 * i) / (float)hs);
        freqs[i] = scale ? scaleFreqLlama31(f, h) : f;
    }
    for (u32 pos = 0; pos < h.seqLen; pos++) {
        for (u32 i = 0; i < half; i++) {
            const float v = (float)pos * freqs[i];
            t[((size_t)pos * half + i) * 2 + 0] = cosf(v);
            t[((size_t)pos * half + i) * 2 + 1] = sinf(v);
        }
    }
    return t;
}

}  // namespace dl
