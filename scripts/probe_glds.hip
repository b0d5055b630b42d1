// Probe of the MFMA decode attention's LDS staging (attn_mfma.hip): 4 waves each DMA a 32-row x
// 256-B tile (rows = keys of a [keys][128] bf16 matrix whose element (r, d) = r * 256 + d) into a
// per-wave buffer with the chunk swizzle, wait (vmcnt + barrier), then read every (row, chunk) back
// through the kernel's row-read addressing and compare on the host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ __forceinline__ int amSwz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__global__ void probe(const uint16_t *src, uint16_t *out, int *bad) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    char *kb = smem + wave * 32768 + 16384;  // the kernel's buffer 1 of each wave
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int r = 4 * j + (lane >> 4), p = lane & 15;
        const size_t off = (size_t)(wave * 32 + r) * 128 + (size_t)(p ^ amSwz(r)) * 8;
        __builtin_amdgcn_global_load_lds(const_cast<uint16_t *>(src + off),
                                         reinterpret_cast<__attribute__((address_space(3))) void *>(
                                             reinterpret_cast<uintptr_t>(kb + j * 1024)), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // every lane reads rows lane>>1 .. with chunk ch: element (r, 8 ch + e)
    for (int q = lane; q < 32 * 16; q += 64) {
        const int r = q >> 4, ch = q & 15;
        const uint16_t *p = reinterpret_cast<const uint16_t *>(kb + r * 256 + 16 * (ch ^ amSwz(r)));
        for (int e = 0; e < 8; e++) {
            const uint16_t v = p[e];
            out[((wave * 32 + r) * 128) + ch * 8 + e] = v;
            if (v != (uint16_t)((wave * 32 + r) * 256 + ch * 8 + e)) atomicAdd(bad, 1);
        }
    }
}
int main() {
    const int n = 128 * 128;
    uint16_t *h = new uint16_t[n], *d, *o;
    int *bad, hb = 0;
    for (int r = 0; r < 128; r++)
        for (int c = 0; c < 128; c++) h[r * 128 + c] = (uint16_t)(r * 256 + c);
    (void)hipMalloc(&d, n * 2);
    (void)hipMalloc(&o, n * 2);
    (void)hipMalloc(&bad, 4);
    (void)hipMemcpy(d, h, n * 2, hipMemcpyHostToDevice);
    (void)hipMemset(bad, 0, 4);
    (void)hipFuncSetAttribute((const void *)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    hipLaunchKernelGGL(probe, dim3(1), dim3(256), 131072, 0, d, o, bad);
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h, o, n * 2, hipMemcpyDeviceToHost);
    printf("mismatches: %d\n", hb);
    for (int r = 0; r < 6; r++) {
        printf("row %3d:", r);
        for (int c = 0; c < 16; c++) printf(" %04x", h[r * 128 + c * 8]);
        printf("\n");
    }
    for (int r = 32; r < 34; r++) {
        printf("row %3d:", r);
        for (int c = 0; c < 16; c++) printf(" %04x", h[r * 128 + c * 8]);
        printf("\n");
    }
    return 0;
}
