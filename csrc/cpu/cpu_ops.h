// CPU reference primitives shared by the CPU backend (cpu_backend.cpp) and the golden tests
// (bindings `cpu_ops`). Semantics of the reference's CPU ops (src/nn/nn-cpu-ops.cpp): invRms
// (105-134), SiLU / GELU (445-491), Q80 x Q40 and F32 matmuls (182-440), RoPE over adjacent pairs
// (1090-1120); softmax as the sampler's (tokenizer.cpp).
#pragma once

#include <cmath>

#include "../core/quant.h"
#include "thread_pool.h"

namespace dl {
namespace cpu {

float invRms(const float *x, u32 n, float eps);
inline float silu(float z) { return z / (1.0f + std::exp(-z)); }
inline float gelu(float z) {
    return 0.5f * z * (1.0f + std::tanh(0.79788456080286535588f * z * (1.0f + 0.044715f * z * z)));
}
// rotate pairs (i, i+1) of v[0, len) whose element i sits at within-head index i % headSize, by
// the table row of `pos` ([seqLen][headSize/2] (cos, sin), plan.h buildRopeTable)
void ropeApply(float *v, u32 len, u32 pos, u32 headSize, const float *table);
// ys[t][r] = W[r,:] . xs[t] for r < rows, t < B; every weight row is read once for all B rows
void matmulQ40Q80(const BlockQ40 *w, u32 rows, u32 cols, const BlockQ80 *const *xs, int B, float *const *ys,
                  ThreadPool &pool);
void matmulF32(const float *w, u32 rows, u32 cols, const float *const *xs, int B, float *const *ys, ThreadPool &pool);

}  // namespace cpu
}  // namespace dl
