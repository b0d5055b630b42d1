// Host-side float16 / Q40 / Q80 codecs.
//
// Block semantics match the reference's on-disk format
// (src/nn/nn-quants.hpp:64-72, nn-quants.cpp:67-246, converter/writer.py:29-74):
//   Q40 block: f16 d, 16 bytes; element j = (lo nibble of byte j) - 8, element j+16 = (hi nibble) - 8.
//   Q80 block: f16 d, 32 x int8.
// Rounding of the Q80 quantizer is round-half-to-even (the reference's x86/AVX2 behaviour,
// nn-quants.cpp:139); the GPU kernels use the same rule so CPU and GPU agree bit-for-bit on codes.
#pragma once

#include "common.h"

namespace dl {

struct BlockQ40 {
    u16 d;
    u8 qs[kQBlock / 2];
};
static_assert(sizeof(BlockQ40) == kQ40BlockBytes, "BlockQ40 layout");

struct BlockQ80 {
    u16 d;
    i8 qs[kQBlock];
};
static_assert(sizeof(BlockQ80) == kQ80BlockBytes, "BlockQ80 layout");

float f16ToF32(u16 h);
u16 f32ToF16(float f);

// n elements -> n/32 blocks
void quantizeQ80(const float *x, BlockQ80 *out, u64 n);
void dequantizeQ80(const BlockQ80 *in, float *out, u64 n);
void quantizeQ40(const float *x, BlockQ40 *out, u64 n);
void dequantizeQ40(const BlockQ40 *in, float *out, u64 n);

// Split-of-range helper identical in spirit to SPLIT_THREADS (nn-quants.hpp:82-86).
inline void splitRange(u64 len, u32 nParts, u32 part, u64 &start, u64 &end) {
    u64 slice = len / nParts, rest = len % nParts;
    start = part * slice + (part < rest ? part : rest);
    end = start + slice + (part < rest ? 1 : 0);
}

}  // namespace dl
