// Microbenchmark: device-wide barrier cost in a persistent kernel on MI355X, and the cost of a
// "stage" (stream S bytes of weights, then synchronise the grid) in a persistent kernel versus one
// dependent kernel per stage replayed from a hipGraph.
// hipcc --offload-arch=gfx950 -O3 scripts/microbench_barrier.hip -o build/microbench_barrier
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);    \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Bar {
    unsigned count[8 * 32];  // per-group counters, 128 B apart
    unsigned top;
    unsigned pad0[31];
    unsigned gen;
    unsigned pad1[31];
    unsigned abort;
};

__device__ __forceinline__ long long rt() { return (long long)__builtin_amdgcn_s_memrealtime(); }

// Sense-reversal barrier; HIER = per-XCD (blockIdx % 8) counters first, then one top counter.
// FENCE = agent-scope release/acquire fences around it (on gfx950: whole-L2 writeback /
// invalidate); without, stage data must be handed over with agent-scope atomic (sc1) accesses.
template <bool HIER, bool FENCE = true>
__device__ __forceinline__ bool gridBarrier(Bar *b) {
    __shared__ int ok;
    __syncthreads();
    if (threadIdx.x == 0) {
        ok = 1;
        const unsigned g = __hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        bool last;
        if (HIER) {
            const int grp = blockIdx.x & 7;
            const unsigned nGrp = (gridDim.x - grp + 7) / 8;
            last = __hip_atomic_fetch_add(&b->count[grp * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nGrp - 1;
            if (last) {
                __hip_atomic_store(&b->count[grp * 32], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned nTop = gridDim.x < 8 ? gridDim.x : 8;
                last = __hip_atomic_fetch_add(&b->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nTop - 1;
                if (last) __hip_atomic_store(&b->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            last = __hip_atomic_fetch_add(&b->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
            if (last) __hip_atomic_store(&b->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (last) {
            if (FENCE) __hip_atomic_store(&b->gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            else __hip_atomic_store(&b->gen, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const long long t0 = rt();
            while (__hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (rt() - t0 > 100000000LL ||
                    __hip_atomic_load(&b->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    __hip_atomic_store(&b->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
            }
        }
        if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    return ok;
}

template <bool HIER, bool FENCE = true>
__global__ __launch_bounds__(256) void barrierLoop(Bar *b, int iters, unsigned *out) {
    for (int i = 0; i < iters; i++)
        if (!gridBarrier<HIER, FENCE>(b)) return;
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}

// stream this workgroup's contiguous share of buf (n16 x 16 B), D loads in flight per lane
__device__ __forceinline__ unsigned streamShare(const u32x4 *p, size_t n16) {
    const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const size_t i0 = blockIdx.x * per, i1 = i0 + per < n16 ? i0 + per : n16;
    unsigned acc = 0;
    for (size_t i = i0 + threadIdx.x; i < i1; i += 8 * 256) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            size_t j = i + u * 256;
            j = j < i1 ? j : i1 - 1;
            v[u] = __builtin_nontemporal_load(p + j);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    return acc;
}

template <bool HIER, bool FENCE = true>
__global__ __launch_bounds__(256) void persistentStages(const u32x4 *const *bufs, int nBufs, size_t n16, int stages,
                                                        Bar *b, unsigned *out) {
    unsigned acc = 0;
    for (int s = 0; s < stages; s++) {
        acc ^= streamShare(bufs[s % nBufs], n16);
        if (!gridBarrier<HIER, FENCE>(b)) return;
    }
    if (acc == 0x12345678) out[1] = acc;
}

__global__ __launch_bounds__(256) void oneStage(const u32x4 *p, size_t n16, unsigned *out) {
    const unsigned acc = streamShare(p, n16);
    if (acc == 0x12345678) out[1] = acc;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    Bar *bar;
    CK(hipMalloc(&bar, sizeof(Bar)));
    CK(hipMemset(bar, 0, sizeof(Bar)));
    unsigned *out;
    CK(hipMalloc(&out, 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("CUs: %d\n", cus);

    const int iters = 2000;
    for (int G : {cus, 2 * cus}) {
        for (int hier = 0; hier < 4; hier++) {  // 0/1 flat/hier with fences, 2/3 fence-free
            auto run = [&]() {
                if (hier == 1) hipLaunchKernelGGL((barrierLoop<true, true>), dim3(G), dim3(256), 0, s, bar, iters, out);
                else if (hier == 0) hipLaunchKernelGGL((barrierLoop<false, true>), dim3(G), dim3(256), 0, s, bar, iters, out);
                else if (hier == 3) hipLaunchKernelGGL((barrierLoop<true, false>), dim3(G), dim3(256), 0, s, bar, iters, out);
                else hipLaunchKernelGGL((barrierLoop<false, false>), dim3(G), dim3(256), 0, s, bar, iters, out);
            };
            run();
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            run();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            unsigned ab = 0;
            CK(hipMemcpy(&ab, &bar->abort, 4, hipMemcpyDeviceToHost));
            printf("barrier G=%d %s%s: %.3f us per barrier%s\n", G, (hier & 1) ? "hier" : "flat",
                   hier >= 2 ? " fence-free" : "", ms * 1000 / iters,
                   ab ? " (ABORTED)" : "");
            if (ab) return 1;
        }
    }

    // stages: persistent (stream + barrier) vs one kernel per stage in a hipGraph
    const int nBufs = 8, stages = 400;
    for (double mb : {1.2, 9.4, 14.2, 33.0, 66.1}) {
        const size_t bytes = (size_t)(mb * 1e6) / 4096 * 4096;
        std::vector<u32x4 *> bufs(nBufs);
        for (auto &p : bufs) {
            CK(hipMalloc(&p, bytes));
            CK(hipMemset(p, 1, bytes));
        }
        u32x4 **dBufs;
        CK(hipMalloc(&dBufs, nBufs * sizeof(void *)));
        CK(hipMemcpy(dBufs, bufs.data(), nBufs * sizeof(void *), hipMemcpyHostToDevice));
        const size_t n16 = bytes / 16;
        float msP[4] = {0, 0, 0, 0};
        for (int hier = 0; hier < 4; hier++) {
            auto run = [&]() {
                if (hier == 1) hipLaunchKernelGGL((persistentStages<true, true>), dim3(cus), dim3(256), 0, s, dBufs, nBufs, n16, stages, bar, out);
                else if (hier == 0) hipLaunchKernelGGL((persistentStages<false, true>), dim3(cus), dim3(256), 0, s, dBufs, nBufs, n16, stages, bar, out);
                else if (hier == 3) hipLaunchKernelGGL((persistentStages<true, false>), dim3(cus), dim3(256), 0, s, dBufs, nBufs, n16, stages, bar, out);
                else hipLaunchKernelGGL((persistentStages<false, false>), dim3(cus), dim3(256), 0, s, dBufs, nBufs, n16, stages, bar, out);
            };
            run();
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            run();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&msP[hier], e0, e1));
        }
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < stages; i++) hipLaunchKernelGGL(oneStage, dim3(cus), dim3(256), 0, s, bufs[i % nBufs], n16, out);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float msG = 0;
        CK(hipEventElapsedTime(&msG, e0, e1));
        printf("stage %5.1f MB: persistent flat %.2f us, hier %.2f us, fence-free flat %.2f us, hier %.2f us | graph of "
               "kernels %.2f us per stage\n", mb, msP[0] * 1000 / stages, msP[1] * 1000 / stages, msP[2] * 1000 / stages,
               msP[3] * 1000 / stages, msG * 1000 / stages);
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
        for (auto p : bufs) CK(hipFree(p));
        CK(hipFree(dBufs));
    }
    return 0;
}
