// Microbenchmark: the floor for a weight-streaming decode kernel of a given size on MI355X.
// Pure nontemporal reads of S bytes (cycling 8 copies so nothing is served from the 256 MB MALL),
// one launch per matrix, 200 launches back to back in a hipGraph: us per launch includes the
// dependent-kernel boundary exactly like the GEMV kernels do in the decode graph.
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_stream.hip -o build/microbench_stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Each workgroup streams one contiguous chunk; every lane keeps U 16-byte loads in flight.
template <int U>
__global__ __launch_bounds__(256) void chunkKernel(const u32x4 *p, size_t n16, unsigned *out) {
    const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const size_t b0 = blockIdx.x * per, b1 = b0 + per < n16 ? b0 + per : n16;
    unsigned acc = 0;
    for (size_t i = b0 + threadIdx.x; i < b1; i += 256 * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t j = i + u * 256;
            j = j < b1 ? j : b1 - 1;
            v[u] = __builtin_nontemporal_load(p + j);
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 0x12345678) out[0] = acc;
}

template <int U>
static float run(hipStream_t s, std::vector<u32x4 *> &bufs, size_t bytes, int grid, unsigned *out) {
    hipGraph_t g;
    hipGraphExec_t ge;
    const int n = 200;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < n; i++)
        hipLaunchKernelGGL(chunkKernel<U>, dim3(grid), dim3(256), 0, s, bufs[i % bufs.size()], bytes / 16, out);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < 3; r++) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    return ms * 1000.f / (3 * n);
}

int main() {
    hipStream_t s;
    (void)hipStreamCreate(&s);
    const size_t maxBytes = 296u << 20;
    std::vector<u32x4 *> bufs(8);
    for (auto &b : bufs) {
        if (hipMalloc(&b, maxBytes) != hipSuccess) return 1;
        (void)hipMemset(b, 1, maxBytes);
    }
    unsigned *out;
    (void)hipMalloc(&out, 64);
    const double sizes[] = {1.2, 4.1, 9.4, 14.2, 33.0, 66.1, 295.5};
    const int grids[] = {256, 512, 768, 1024, 2048};
    for (double mb : sizes) {
        const size_t bytes = ((size_t)(mb * 1e6) + 4095) / 4096 * 4096;
        for (int g : grids) {
            printf("%6.1f MB grid %4d |", mb, g);
            const float a = run<4>(s, bufs, bytes, g, out), b = run<8>(s, bufs, bytes, g, out),
                        c = run<16>(s, bufs, bytes, g, out);
            printf(" U4 %7.2f us %5.2f TB/s | U8 %7.2f us %5.2f TB/s | U16 %7.2f us %5.2f TB/s\n", a,
                   bytes / a / 1e6, b, bytes / b / 1e6, c, bytes / c / 1e6);
        }
    }
    return 0;
}
