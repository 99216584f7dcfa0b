// NTT pass microbenchmark (dev tool): each N=2^16 pass kernel over 248 limbs, real vs
// load/store-only (NTT_NOCOMPUTE) builds, to separate memory time from arithmetic time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../aes-fhe_amd/csrc/ntt256.h"
using namespace aesfhe;
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("%s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_copy(const u64* __restrict__ a, u64* __restrict__ b, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

int main() {
    const int logN = 16, N = 1 << 16, L = 248, np = 1;
    u64 q = 1125899906826241ULL % (1ULL << 50);
    q = 1125899906629633ULL;  // any odd < 2^50 works for timing
    std::vector<u64> hq(np, q);
    std::vector<double> hqi(np, 1.0 / q);
    std::vector<Tw> htw(N);
    for (int i = 0; i < N; i++) htw[i] = Tw{(u64)(i * 7919ULL % q), (double)(i * 7919ULL % q) / q};
    u64 *dq, *data, *data2; double* dqi; Tw* dtw; u64* dninv; double* dninvf;
    CK(hipMalloc(&dq, 8)); CK(hipMalloc(&dqi, 8)); CK(hipMalloc(&dtw, N * 16)); CK(hipMalloc(&dninv, 8)); CK(hipMalloc(&dninvf, 8));
    CK(hipMemcpy(dq, hq.data(), 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dqi, hqi.data(), 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dtw, htw.data(), N * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(dninv, hq.data(), 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dninvf, hqi.data(), 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&data, (size_t)L * N * 8)); CK(hipMalloc(&data2, (size_t)L * N * 8));
    CK(hipMemset(data, 0, (size_t)L * N * 8));
    Tabs T{}; T.q = dq; T.qinv = dqi; T.tw = dtw; T.itw = dtw; T.ninv = dninv; T.ninvf = dninvf; T.logN = logN; T.Lp1 = 1;
    // every limb uses prime index 0: Span with nq = 0, spid0 = 0
    Span s{data, (long)N, 1, 0, 0, 0};
    Span s2{data2, (long)N, 1, 0, 0, 0};
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto timeit = [&](const char* name, auto fn) {
        for (int w = 0; w < 3; w++) fn();
        hipEventRecord(a);
        const int it = 20;
        for (int i = 0; i < it; i++) fn();
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        double us = ms * 1000 / it;
        printf("%-28s %8.1f us  %7.1f GB/s (r+w)\n", name, us, 2.0 * L * N * 8 / (us * 1e3));
    };
    timeit("copy", [&] { hipLaunchKernelGGL(k_copy, dim3(L * N / 256), dim3(256), 0, 0, data, data2, (long)L * N); });
    timeit("fwd_cols (src!=dst)", [&] { hipLaunchKernelGGL(k_ntt256_fwd_cols, dim3(16, L), dim3(256), 0, 0, s, s2, T); });
    timeit("fwd_cols (in place)", [&] { hipLaunchKernelGGL(k_ntt256_fwd_cols, dim3(16, L), dim3(256), 0, 0, s, s, T); });
    timeit("fwd_rows", [&] { hipLaunchKernelGGL(k_ntt256_fwd_rows, dim3(16, L), dim3(256), 0, 0, s, T); });
    timeit("inv_rows", [&] { hipLaunchKernelGGL(k_ntt256_inv_rows, dim3(16, L), dim3(256), 0, 0, s, s2, T); });
    timeit("inv_cols", [&] { hipLaunchKernelGGL(k_ntt256_inv_cols, dim3(16, L), dim3(256), 0, 0, s, T); });
    return 0;
}
