// CPU reference primitives (see cpu_ops.h). Matmuls are AVX2/FMA (x86-64-v3) and batched: every
// weight row is read once for all activation rows (the reference reaches the same reuse with
// vendored tinyBLAS for batch > 1, nn-cpu-ops.cpp:1000-1016). Q40 x Q80 blocks are int8 dot
// products (maddubs on |w| and sign-transferred x, exact int32 per block) scaled by d_w * d_x in
// f32, like matmul_Q80_Q40_F32 (nn-cpu-ops.cpp:222-440).
#include "cpu_ops.h"

#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <vector>

namespace dl {
namespace cpu {

float invRms(const float *x, u32 n, float eps) {
    float s = 0.f;
    for (u32 i = 0; i < n; i++) s += x[i] * x[i];
    s /= (float)n;
    s += eps;
    return 1.0f / std::sqrt(s);
}

void ropeApply(float *v, u32 len, u32 pos, u32 headSize, const float *table) {
    const u32 half = headSize / 2;
    const float *t = &table[(u64)pos * half * 2];
    for (u32 i = 0; i < len; i += 2) {
        const u32 fi = (i % headSize) / 2;
        const float c = t[fi * 2], s = t[fi * 2 + 1];
        const float v0 = v[i], v1 = v[i + 1];
        v[i] = v0 * c - v1 * s;
        v[i + 1] = v0 * s + v1 * c;
    }
}

// groups of kGroup activation rows keep their accumulators in registers
static constexpr int kGroup = 8;

static float hsum(__m256 v) {
    __m128 s = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
    s = _mm_add_ps(s, _mm_movehl_ps(s, s));
    s = _mm_add_ss(s, _mm_movehdup_ps(s));
    return _mm_cvtss_f32(s);
}

void matmulF32(const float *w, u32 rows, u32 n, const float *const *xs, int B, float *const *ys, ThreadPool &pool) {
    DL_CHECK(n % 8 == 0, "f32 matmul: columns must be a multiple of 8");
    pool.parallelFor(rows, [&](long s, long e) {
        for (long r = s; r < e; r++) {
            const float *wr = w + (u64)r * n;
            for (int t0 = 0; t0 < B; t0 += kGroup) {
                const int g = std::min(kGroup, B - t0);
                __m256 acc[kGroup];
                for (int t = 0; t < g; t++) acc[t] = _mm256_setzero_ps();
                for (u32 i = 0; i < n; i += 8) {
                    const __m256 wv = _mm256_loadu_ps(wr + i);
                    for (int t = 0; t < g; t++) acc[t] = _mm256_fmadd_ps(wv, _mm256_loadu_ps(xs[t0 + t] + i), acc[t]);
                }
                for (int t = 0; t < g; t++) ys[t0 + t][r] = hsum(acc[t]);
            }
        }
    });
}

void matmulQ40Q80(const BlockQ40 *w, u32 rows, u32 cols, const BlockQ80 *const *xs, int B, float *const *ys,
                  ThreadPool &pool) {
    const u32 nb = cols / kQBlock;
    // activation scales as f32, once per call
    std::vector<float> xd((size_t)B * nb);
    for (int t = 0; t < B; t++)
        for (u32 b = 0; b < nb; b++) xd[(size_t)t * nb + b] = f16ToF32(xs[t][b].d);
    pool.parallelFor(rows, [&](long s, long e) {
        const __m256i low4 = _mm256_set1_epi8(0x0F), eight = _mm256_set1_epi8(8);
        const __m256i ones = _mm256_set1_epi16(1);
        for (long r = s; r < e; r++) {
            const BlockQ40 *wr = w + (u64)r * nb;
            for (int t0 = 0; t0 < B; t0 += kGroup) {
                const int g = std::min(kGroup, B - t0);
                __m256 acc[kGroup];
                for (int t = 0; t < g; t++) acc[t] = _mm256_setzero_ps();
                for (u32 b = 0; b < nb; b++) {
                    // 32 weights in Q80 element order: [lo nibbles 0..15 | hi nibbles 0..15] - 8
                    const __m128i raw = _mm_loadu_si128(reinterpret_cast<const __m128i *>(wr[b].qs));
                    const __m256i nib = _mm256_set_m128i(_mm_srli_epi16(raw, 4), raw);
                    const __m256i wq = _mm256_sub_epi8(_mm256_and_si256(nib, low4), eight);
                    const __m256i aw = _mm256_sign_epi8(wq, wq);
                    const float dw = f16ToF32(wr[b].d);
                    for (int t = 0; t < g; t++) {
                        const __m256i xq = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(xs[t0 + t][b].qs));
                        const __m256i p16 = _mm256_maddubs_epi16(aw, _mm256_sign_epi8(xq, wq));
                        const __m256i p32 = _mm256_madd_epi16(p16, ones);
                        const __m256 sc = _mm256_set1_ps(dw * xd[(size_t)(t0 + t) * nb + b]);
                        acc[t] = _mm256_fmadd_ps(_mm256_cvtepi32_ps(p32), sc, acc[t]);
                    }
                }
                for (int t = 0; t < g; t++) ys[t0 + t][r] = hsum(acc[t]);
            }
        }
    });
}

}  // namespace cpu
}  // namespace dl
