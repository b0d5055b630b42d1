// Per-CU intake of a long-context decode-attention workgroup (attn_mfma.hip's load shape): each of
// G workgroups (256 threads, one per CU) takes in 128 KB of distinct HBM data - 4 waves x 2 tiles x
// (K + V) 8 KB, 1-KB wave instructions - either by LDS-DMA (global_load_lds_dwordx4, the kernel's
// path) or into registers (global_load_dwordx4). Per workgroup: s_memrealtime at entry and after
// the last byte landed (100 MHz), so the table separates launch skew from the intake itself.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/intake scripts/microbench_intake.hip && /tmp/intake
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kBytesPerWg = 128 * 1024;
constexpr int kInstrPerWave = kBytesPerWg / 4 / 1024;  // 32 one-KB wave instructions

__global__ __launch_bounds__(256) void intakeLds(const char *src, unsigned long long *stamps) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const char *base = src + (size_t)blockIdx.x * kBytesPerWg + (size_t)wave * (kBytesPerWg / 4);
    char *dst = smem + wave * (kBytesPerWg / 4);
#pragma unroll
    for (int j = 0; j < kInstrPerWave; j++)
        __builtin_amdgcn_global_load_lds(const_cast<char *>(base + j * 1024 + lane * 16),
                                         reinterpret_cast<__attribute__((address_space(3))) void *>(
                                             reinterpret_cast<uintptr_t>(dst + j * 1024)), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        stamps[2 * blockIdx.x] = t0;
        stamps[2 * blockIdx.x + 1] = t1;
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void intakeReg(const char *src, unsigned long long *stamps, unsigned *sink) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const char *base = src + (size_t)blockIdx.x * kBytesPerWg + (size_t)wave * (kBytesPerWg / 4);
    u32x4 v[kInstrPerWave];
#pragma unroll
    for (int j = 0; j < kInstrPerWave; j++)
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v[j]) : "v"(base + j * 1024 + lane * 16));
    unsigned x = 0;
#pragma unroll
    for (int j = 0; j < kInstrPerWave; j++) {
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[j])::"memory");
        x ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        stamps[2 * blockIdx.x] = t0;
        stamps[2 * blockIdx.x + 1] = t1;
    }
    if (x == 0x12345678u) sink[tid] = x;
}

int main() {
    const int maxG = 256;
    const size_t bytes = (size_t)maxG * kBytesPerWg;
    const int copies = 16;  // rotate buffers so every run starts cold in L2 (64 MB per copy set)
    std::vector<char *> bufs(copies);
    for (auto &b : bufs) {
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(b, 1, bytes));
    }
    unsigned long long *st;
    unsigned *sink;
    CK(hipMalloc(&st, 2 * maxG * sizeof(unsigned long long)));
    CK(hipMalloc(&sink, 256 * 4));
    CK(hipFuncSetAttribute((const void *)intakeLds, hipFuncAttributeMaxDynamicSharedMemorySize, kBytesPerWg));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("per-workgroup intake of 128 KB (us from the workgroup's entry, median / max over workgroups; launch us)\n");
    for (int mode = 0; mode < 2; mode++) {
        for (int G : {32, 64, 128, 256}) {
            std::vector<double> med, mx, ln;
            for (int it = 0; it < 12; it++) {
                const char *src = bufs[it % copies];
                CK(hipEventRecord(e0));
                if (mode == 0)
                    hipLaunchKernelGGL(intakeLds, dim3(G), dim3(256), kBytesPerWg, 0, src, st);
                else
                    hipLaunchKernelGGL(intakeReg, dim3(G), dim3(256), 0, 0, src, st, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms = 0.f;
                CK(hipEventElapsedTime(&ms, e0, e1));
                std::vector<unsigned long long> h(2 * G);
                CK(hipMemcpy(h.data(), st, 2 * G * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                std::vector<double> d(G);
                for (int g = 0; g < G; g++) d[g] = (h[2 * g + 1] - h[2 * g]) * 0.01;  // 100 MHz ticks -> us
                std::sort(d.begin(), d.end());
                if (it >= 2) {
                    med.push_back(d[G / 2]);
                    mx.push_back(d[G - 1]);
                    ln.push_back(ms * 1000.0);
                }
            }
            auto m = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
            const double um = m(med);
            printf("%s G=%3d: intake median %6.2f us (%6.1f GB/s per CU), max %6.2f us, launch %6.2f us, chip %6.2f TB/s\n",
                   mode == 0 ? "lds-dma" : "regs   ", G, um, kBytesPerWg / um / 1e3, m(mx), m(ln),
                   (double)G * kBytesPerWg / m(ln) / 1e6);
        }
    }
    return 0;
}
