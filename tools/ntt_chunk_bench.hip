// Chunked / pipelined forward NTT microbenchmark (dev tool): does keeping the column-pass
// intermediate of a chunk of limbs resident in the Infinity Cache (256 MiB) speed up the row
// pass?  Full two-pass NTT over 496 limbs (B = 16 x 31) vs chunks of C limbs, serial on one
// stream or pipelined on two streams (rows of chunk k beside cols of chunk k + 1).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../aes-fhe_amd/csrc/ntt256f.h"
#include "tabs_cw.h"
using namespace aesfhe;
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("%s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
    const int logN = 16, N = 1 << 16, L = argc > 1 ? atoi(argv[1]) : 496;
    const u64 q = 1099511480321ULL;  // 40-bit prime (no folding path)
    u64 *dq, *src, *dst; double *dqi, *dw8;
    CK(hipMalloc(&dq, 8)); CK(hipMalloc(&dqi, 8)); CK(hipMalloc(&dw8, N * 8));
    double qi = 1.0 / q;
    CK(hipMemcpy(dq, &q, 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dqi, &qi, 8, hipMemcpyHostToDevice));
    { std::vector<double> h(N); for (int i = 0; i < N; i++) h[i] = (double)(i * 7919ULL % q) / q; CK(hipMemcpy(dw8, h.data(), N * 8, hipMemcpyHostToDevice)); }
    CK(hipMalloc(&src, (size_t)L * N * 8)); CK(hipMalloc(&dst, (size_t)L * N * 8));
    CK(hipMemset(src, 0, (size_t)L * N * 8));
    Tabs T{}; T.q = dq; T.qinv = dqi; T.psif = dw8; T.ipsif = dw8; T.logN = logN; T.Lp1 = 1;
    T.cw = T.icw = tools_make_cw(dw8, dq, 1, logN);
    hipStream_t s1, s2; CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(1024);
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    auto span = [&](u64* p, int off) { return Span{p + (long)off * N, (long)N, 1, 0, 0, 0}; };
    auto run = [&](int C, bool pipe) {
        for (int off = 0, k = 0; off < L; off += C, k++) {
            const int n = std::min(C, L - off);
            hipLaunchKernelGGL(k_nttf_fwd_cols, dim3(16, n), dim3(256), 0, s1, span(src, off), span(dst, off), T);
            hipStream_t sr = s1;
            if (pipe) { hipEventRecord(ev[k], s1); hipStreamWaitEvent(s2, ev[k], 0); sr = s2; }
            hipLaunchKernelGGL(k_nttf_fwd_rows_t<false>, dim3(16, n), dim3(256), 0, sr, span(dst, off), T, RowFin{});
        }
        if (pipe) { hipEventRecord(ev[1023], s2); hipStreamWaitEvent(s1, ev[1023], 0); }
    };
    auto timeit = [&](const char* name, int C, bool pipe) {
        for (int w = 0; w < 3; w++) run(C, pipe);
        hipEventRecord(a, s1);
        const int it = 10;
        for (int i = 0; i < it; i++) run(C, pipe);
        hipEventRecord(b, s1); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1000 / it;
        printf("%-10s C=%4d %9.1f us  %7.1f GB/s algorithmic (16N B/limb)\n", name, C, us, 2.0 * L * N * 8 / (us * 1e3));
    };
    timeit("full", L, false);
    for (int C : {8, 16, 32, 64, 128}) { timeit("serial", C, false); timeit("pipelined", C, true); }
    return 0;
}
