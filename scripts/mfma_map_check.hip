#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
// A[16][32], B[32][16] (B[k][n]); expected map: lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]; C col=l&15,row=(l>>4)*4+i
__global__ void k(const float *A, const float *B, float *C) {
    int l = threadIdx.x;
    half8 a, b;
    for (int j = 0; j < 8; j++) {
        a[j] = (_Float16)A[(l & 15) * 32 + 8 * (l >> 4) + j];
        b[j] = (_Float16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];
    }
    f32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; i++) C[((l >> 4) * 4 + i) * 16 + (l & 15)] = c[i];
}
int main() {
    float hA[512], hB[512], hC[256], ref[256];
    for (int i = 0; i < 512; i++) { hA[i] = (float)((i * 7) % 5 - 2); hB[i] = (float)((i * 3) % 7 - 3); }
    for (int r = 0; r < 16; r++) for (int c = 0; c < 16; c++) { float s = 0; for (int k = 0; k < 32; k++) s += hA[r * 32 + k] * hB[k * 16 + c]; ref[r * 16 + c] = s; }
    float *dA, *dB, *dC;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dC, 1024);
    hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    k<<<1, 64>>>(dA, dB, dC);
    hipMemcpy(hC, dC, 1024, hipMemcpyDeviceToHost);
    int bad = 0; for (int i = 0; i < 256; i++) bad += hC[i] != ref[i];
    printf("mfma 16x16x32 f16 map: %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);
    return bad != 0;
}
