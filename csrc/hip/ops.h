// Single-kernel entry points for kernel-level numerics tests and the Python `ops` package.
//
// Each call uploads host operands, runs ONE of the gfx950 kernels of csrc/hip/kernels.hip exactly as
// the engine launches it (same tiling, same fused prologue/epilogue), and copies the result back.
// They are not on the inference hot path; they exist so that every hot kernel can be compared
// against a plain PyTorch fp32 reference of the same op (tests/test_gpu_ops.py).
#pragma once

#include <cstdint>
#include <vector>

namespace dl {
namespace ops {

// Q40 GEMV (decode kernel, B rows <= 4) over `blocks` = [rows][n/32] Q40 blocks in file layout
// (18 bytes: f16 d + 16 nibble bytes). Prologue: in (+ residual) -> RMS norm with normW (if given,
// else plain) -> Q80 in LDS. epi 0: out[b][r] = W[r] . xq; epi 1: rows interleaved (w1, w3) pairs,
// out[b][r/2] = silu(W[2i] . xq) * (W[2i+1] . xq). Returns out; xNext (if residual) = in + residual.
std::vector<float> gemvQ40(const std::vector<uint8_t> &blocks, int rows, int n, const std::vector<float> &in,
                           const std::vector<float> &residual, const std::vector<float> &normW, float eps, int B,
                           int epi, std::vector<float> *xNext);

// Same weights, activations already Q80 (the wo / w2 path: prologue-free, Q80 blocks read from
// global): `in` is quantized on the host with the reference Q80 quantizer first.
std::vector<float> gemvQ40Q80In(const std::vector<uint8_t> &blocks, int rows, int n, const std::vector<float> &in,
                                int B);

// Batched F32 matmul on MFMA: norm kernel -> f16 -> gemmF32Kernel (store epilogue).
std::vector<float> gemmF32(const std::vector<float> &w, int rows, int n, const std::vector<float> &in,
                           const std::vector<float> &normW, float eps, int M);
std::vector<float> gemmQ40(const std::vector<uint8_t> &blocks, int rows, int n, const std::vector<float> &in,
                           const std::vector<float> &residual, const std::vector<float> &normW, float eps, int M,
                           int splits = 0);  // Batched Q40 matmul on MFMA (narrow <= 64 tokens, wide above);
                                             // splits > 0 forces the K split (must divide n / 32)

// QKV GEMV with the RoPE + KV-append epilogue (rows = q0 + 2*kv0, head size hs): returns rotated q
// [B][q0]; kOut/vOut receive the appended cache rows [B][kv0] (f32 view of the bf16 or f32 cache).
// rope = [seqLen][hs/2] (cos, sin) pairs; pos[b] < seqLen; each row b writes cache slot b.
std::vector<float> qkvRope(const std::vector<uint8_t> &blocks, int q0, int kv0, int hs, int n,
                           const std::vector<float> &in, const std::vector<float> &normW, float eps,
                           const std::vector<float> &rope, int seqLen, const std::vector<int> &pos, bool kvBf16,
                           std::vector<float> *kOut, std::vector<float> *vOut);

// Decode attention over caches k/v [nSlots][seqLen][kv0] (f32 values, stored bf16 when kvBf16),
// q [B][nHeads0*hs] (already rotated), row b at position pos[b] in slot slot[b]. Returns f32 [B][q0].
std::vector<float> attention(const std::vector<float> &q, const std::vector<float> &k, const std::vector<float> &v,
                             int nSlots, int seqLen, int nHeads0, int kvMul, int hs, const std::vector<int> &pos,
                             const std::vector<int> &slot, bool kvBf16, int impl = 0);
// attention impl: 0 = launchAttention's choice, 1 = MFMA prefill kernel, 2 = VALU decode kernel,
// 3 = MFMA decode kernel

// Parallel argmax over [B][vocab] (ties -> lowest index).
std::vector<int> argmax(const std::vector<float> &logits, int B, int vocab);
// device sampler (launchSample): spec rows (temperature, topp, coin, -)
std::vector<int> sample(const std::vector<float> &logits, int B, int vocab, const std::vector<float> &specs);

// Embedding row gather: table [vocab][dim] -> [B][dim].
std::vector<float> embedding(const std::vector<float> &table, int vocab, int dim, const std::vector<int> &tokens);

}  // namespace ops
}  // namespace dl
