// Microbenchmark: cost of a chain of dependent kernels replayed from a hipGraph on MI355X.
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_launch.hip -o build/microbench_launch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            return 1;                                                               \
        }                                                                           \
    } while (0)

__global__ void emptyKernel(int *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

__global__ void copyKernel(const float4 *a, float4 *b, int n4) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) b[i] = a[i];
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Streaming read of `bytes` with U 16-byte loads in flight per lane (nontemporal), grid-stride.
template <int U>
__global__ __launch_bounds__(256) void streamKernel(const u32x4 *p, size_t n16, unsigned *out) {
    unsigned acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += stride * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t j = i + u * stride;
            j = j < n16 ? j : n16 - 1;
            v[u] = __builtin_nontemporal_load(p + j);
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <int U>
static float timeStream(hipStream_t s, const u32x4 *p, size_t bytes, int grid, unsigned *out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(streamKernel<U>, dim3(grid), dim3(256), 0, s, p, bytes / 16, out);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(streamKernel<U>, dim3(grid), dim3(256), 0, s, p, bytes / 16, out);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return (float)(bytes * 5 / (ms * 1e-3) / 1e12);
}

static float timeGraph(hipStream_t s, int nKernels, int grid, int mode, int *flag, float4 *a, float4 *b, int n4) {
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < nKernels; i++) {
        if (mode == 0)
            hipLaunchKernelGGL(emptyKernel, dim3(grid), dim3(256), 0, s, flag);
        else
            hipLaunchKernelGGL(copyKernel, dim3(grid), dim3(256), 0, s, (i & 1) ? b : a, (i & 1) ? a : b, n4);
    }
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 3; w++) (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int reps = 10;
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < reps; r++) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return ms * 1000.f / reps / nKernels;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *flag;
    CK(hipMalloc(&flag, 64));
    CK(hipMemset(flag, 0, 64));
    const int n4 = (64 << 20) / 16;  // 64 MiB
    float4 *a, *b;
    CK(hipMalloc(&a, (size_t)n4 * 16));
    CK(hipMalloc(&b, (size_t)n4 * 16));
    CK(hipMemset(a, 0, (size_t)n4 * 16));
    for (int grid : {1, 64, 256, 1024, 4096}) {
        printf("empty kernels, grid %5d: %.2f us per kernel (graph of 160)\n", grid, timeGraph(s, 160, grid, 0, flag, a, b, n4));
    }
    for (int kb : {16, 256, 4096, 65536}) {
        const int m4 = kb * 1024 / 16;
        const int grid = m4 / 256 < 1 ? 1 : (m4 / 256 > 2048 ? 2048 : m4 / 256);
        const float us = timeGraph(s, 160, grid, 1, flag, a, b, m4);
        printf("copy %6d KiB (grid %d): %.2f us per kernel, %.1f GB/s\n", kb, grid, us, 2.0 * kb * 1024 / us / 1e3);
    }
    const size_t big = (size_t)4 << 30;  // 4 GiB >> 256 MiB infinity cache
    u32x4 *w;
    CK(hipMalloc(&w, big));
    CK(hipMemset(w, 1, big));
    for (int grid : {256, 512, 1024, 2048, 4096, 8192}) {
        printf("stream-read 4 GiB grid %5d: U=1 %.2f  U=4 %.2f  U=8 %.2f TB/s\n", grid,
               timeStream<1>(s, w, big, grid, (unsigned *)flag), timeStream<4>(s, w, big, grid, (unsigned *)flag),
               timeStream<8>(s, w, big, grid, (unsigned *)flag));
    }
    return 0;
}
