// Start-up self-test of the tensor-parallel exchange fused into the producer kernels (kernels.h
// TpXchg, decode_dev.h tpPushCollect): every rank pushes known values through the same transport
// the GEMV / GEMM epilogues use and checks the rank-order sums, then the ranks exchange their
// verdicts over it, so they all agree whether to keep the fused exchange or fall back to the
// separate collectives (engine.cpp HipEngineImpl::tpFusedSelfTest). Cross-device the exchange's
// 8-byte {payload, epoch} granules are trusted only after this passes on the real devices.
#include "decode_dev.h"
#include "device_comm.h"

namespace dl {
namespace hipk {

__global__ __launch_bounds__(kThreads) void tpSelfTestKernel(TpXchg x, float *out, int n, float val) {
    for (int el = blockIdx.x * kThreads + threadIdx.x; el < n; el += gridDim.x * kThreads) {
        const unsigned e = x.epochs[el] + 1;
        // element-dependent payload: a stale or misrouted word cannot pass as a correct one
        unsigned v[kTpMaxRanks];
        tpPushCollect(x, el, e, __float_as_uint(val + (float)(el & 1023)), v);
        float s = 0.f;
#pragma unroll
        for (int p = 0; p < kTpMaxRanks; p++)
            if (p < x.world) s += __uint_as_float(v[p]);
        out[el] = s;
        x.epochs[el] = e;
    }
}

void launchTpSelfTest(const TpXchg &x, float *out, int n, float val, hipStream_t s) {
    const int grid = std::min(64, (n + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(tpSelfTestKernel, dim3(grid), dim3(kThreads), 0, s, x, out, n, val);
    DL_HIP(hipGetLastError());
}

const void *tpCheckModuleKernel() { return (const void *)tpSelfTestKernel; }

}  // namespace hipk
}  // namespace dl
