// Device-side helpers for gfx950 (CDNA4, wave64).
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dl {
namespace dev {

constexpr int kWave = 64;

// ---- DPP cross-lane moves (stay in the VALU, no LDS round trip) -------------------------------
// dpp_ctrl codes: quad_perm [1,0,3,2] = 0xB1, quad_perm [2,3,0,1] = 0x4E,
// row_ror:4 = 0x124, row_ror:8 = 0x128.
template <int CTRL>
__device__ __forceinline__ float dppF(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppI(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// Sum over the 4 lanes of a quad (all 4 lanes receive it).
__device__ __forceinline__ float quadSum(float v) {
    v += dppF<0xB1>(v);
    v += dppF<0x4E>(v);
    return v;
}
__device__ __forceinline__ int quadSumI(int v) {
    v += dppI<0xB1>(v);
    v += dppI<0x4E>(v);
    return v;
}
__device__ __forceinline__ float quadMax(float v) {
    v = fmaxf(v, dppF<0xB1>(v));
    v = fmaxf(v, dppF<0x4E>(v));
    return v;
}

// Sum over aligned groups of L lanes (L in {4, 16, 32, 64}); every lane of the group gets it.
template <int L>
__device__ __forceinline__ float groupSum(float v) {
    v = quadSum(v);
    if constexpr (L >= 16) {
        v += dppF<0x124>(v);
        v += dppF<0x128>(v);
    }
    if constexpr (L >= 32) v += __shfl_xor(v, 16);
    if constexpr (L >= 64) v += __shfl_xor(v, 32);
    return v;
}
template <int L>
__device__ __forceinline__ float groupMax(float v) {
    v = quadMax(v);
    if constexpr (L >= 16) {
        v = fmaxf(v, dppF<0x124>(v));
        v = fmaxf(v, dppF<0x128>(v));
    }
    if constexpr (L >= 32) v = fmaxf(v, __shfl_xor(v, 16));
    if constexpr (L >= 64) v = fmaxf(v, __shfl_xor(v, 32));
    return v;
}

__device__ __forceinline__ float waveSum(float v) { return groupSum<64>(v); }
__device__ __forceinline__ float waveMax(float v) { return groupMax<64>(v); }

// Block-wide sum for blockDim.x == NT (multiple of 64). `scratch` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float blockSum(float v, float *scratch) {
    v = waveSum(v);
    const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    __syncthreads();
    if (lane == 0) scratch[w] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NT / kWave; i++) s += scratch[i];
    return s;
}

__device__ __forceinline__ float bf16ToF32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ uint16_t f32ToBf16(float f) {
    return __builtin_bit_cast(uint16_t, __float2bfloat16(f));
}
__device__ __forceinline__ float roundF16(float f) { return __half2float(__float2half(f)); }

// int8 dot of 4 packed bytes, accumulate into c (v_dot4_i32_i8).
__device__ __forceinline__ int dot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

__device__ __forceinline__ int packI8x4(int a, int b, int c, int d) {
    return (a & 0xFF) | ((b & 0xFF) << 8) | ((c & 0xFF) << 16) | ((d & 0xFF) << 24);
}

}  // namespace dev
}  // namespace dl
