// tabs_cw.h -- Tabs::cw / icw for the dev tools' own twiddle tables (round 6: the NTT column
// passes read the wave-uniform stages' w = rint(wq q) from a small table beside w / q).
// tools_make_cw(dpsif, dq, np, logN) builds [np][kColW] on the device from a w / q table.
#pragma once
#include <hip/hip_runtime.h>

__global__ void k_tools_make_cw(const double* __restrict__ psif, const aesfhe::u64* __restrict__ q, double* cw,
                                int np, int logN) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np * aesfhe::kColW) return;
    const int p = i / aesfhe::kColW, k = i % aesfhe::kColW;
    cw[i] = __builtin_rint(psif[((long)p << logN) + k] * (double)q[p]);
}
inline double* tools_make_cw(const double* dpsif, const aesfhe::u64* dq, int np, int logN) {
    if (!dpsif) return nullptr;
    double* d = nullptr;
    if (hipMalloc(&d, (size_t)np * aesfhe::kColW * 8) != hipSuccess) return nullptr;
    hipLaunchKernelGGL(k_tools_make_cw, dim3((np * aesfhe::kColW + 255) / 256), dim3(256), 0, 0, dpsif, dq, d, np, logN);
    if (hipDeviceSynchronize() != hipSuccess) return nullptr;
    return d;
}
