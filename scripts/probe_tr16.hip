// Probe of ds_read_b64_tr_b16 lane mapping on gfx950: LDS holds element e = (row << 8) | col for a
// [16 rows][64 cols] u16 image; lane l supplies address (row = 4*(l/16) + (l%16)/4, cols 4*(l%4)..)
// and we print what every lane receives. Build: hipcc --offload-arch=gfx950 -O2 probe_tr16.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
__global__ void probe(unsigned short *out) {
    __shared__ unsigned short img[16 * 64];
    for (int i = threadIdx.x; i < 16 * 64; i += 64) img[i] = (unsigned short)(((i / 64) << 8) | (i % 64));
    __syncthreads();
    const int l = threadIdx.x, g = l / 16, li = l % 16, q = li / 4, p = li % 4;
    const int row = 4 * g + q, col = 4 * p;
    const char *ad = reinterpret_cast<const char *>(img) + (row * 64 + col) * 2;
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) s16x4 *>(reinterpret_cast<uintptr_t>(ad)));
    for (int e = 0; e < 4; e++) out[l * 4 + e] = (unsigned short)v[e];
}
int main() {
    unsigned short *d, h[256];
    hipMalloc(&d, 512);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l++) {
        printf("lane %2d:", l);
        for (int e = 0; e < 4; e++) printf(" (r%d,c%d)", h[l * 4 + e] >> 8, h[l * 4 + e] & 255);
        printf("\n");
    }
    return 0;
}
