// NOTE: a measurement record (round 1: the integer passes of the removed ntt256.h against the fp64
// passes, and the copy kernel that calibrated FETCH_SIZE); it no longer builds (ntt256.h was
// removed with the env-switched integer path in round 2).  Its results are quoted in DESIGN.md 4.1.
// NTT pass microbenchmark (dev tool): each N=2^16 pass kernel over 248 limbs, real vs
// load/store-only (NTT_NOCOMPUTE) builds, to separate memory time from arithmetic time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "../aes-fhe_amd/csrc/ntt256.h"
#include "../aes-fhe_amd/csrc/ntt256f.h"
#include "tabs_cw.h"
using namespace aesfhe;
#define CK(x) do { hipError_t e_ = (x); if (e_) { printf("%s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_copy(const u64* __restrict__ a, u64* __restrict__ b, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// Row-pass variants (timing only): TW = 0 production (16 B {w, w/q} per twiddle), 1 = 8 B
// twiddles (w/q only, w = rint(wq*q) recovered exactly), 2 = no twiddle loads (upper bound).
template <int TW>
__global__ __launch_bounds__(256) void k_rows_var(Span dst, Tabs T, const double* __restrict__ W8) {
    __shared__ u64 s[16 * 16 * kPad];
    int pid;
    u64* io = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, b = tid & 15, rl = tid >> 4;
    const int row = blockIdx.x * 16 + rl;
    const u64 q = T.q[pid], q2 = 2 * q;
    const double qd = (double)q;
    const long toff = (long)pid << T.logN;
    const Tw* W = T.tw + toff;
    const double* Wq = W8 + toff;
    u64* rp = io + (long)row * 256;
    u64 x[16];
    auto tw = [&](int idx, u64& w, double& wq) {
        if (TW == 0) { const Tw t = W[idx]; w = t.w; wq = t.wq; }
        else if (TW == 1) { wq = Wq[idx]; w = rint_u(wq, qd); }
        else { w = (u64)idx * 7919u; wq = (double)w / qd; }
    };
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = rp[a * 16 + b];
#pragma unroll
    for (int st = 0; st < 4; st++) {
        const int ml = 1 << st, h = 8 >> st;
        const int base = ml * (256 + row);
#pragma unroll
        for (int a = 0; a < 16; a++) {
            if (a & h) continue;
            u64 w; double wq; tw(base + (a >> (4 - st)), w, wq);
            ct_lazy(x[a], x[a + h], w, wq, q, q2);
        }
    }
    u64* sr = s + rl * 16 * kPad;
#pragma unroll
    for (int a = 0; a < 16; a++) sr[a * kPad + b] = x[a];
    __syncthreads();
    const int ap = b;
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = sr[ap * kPad + bb];
#pragma unroll
    for (int st = 4; st < 8; st++) {
        const int ml = 1 << st, h = 128 >> st;
        const int base = ml * (256 + row) + ap * (ml >> 4);
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {
            if (bb & h) continue;
            u64 w; double wq; tw(base + (bb >> (8 - st)), w, wq);
            ct_lazy(x[bb], x[bb + h], w, wq, q, q2);
        }
    }
#pragma unroll
    for (int bb = 0; bb < 16; bb++) sr[ap * kPad + bb] = canon4(x[bb], q, q2);
    __syncthreads();
    u64* base = io + (long)blockIdx.x * 16 * 256;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int e = k * 256 + tid, r = e >> 8, cc = e & 255;
        base[e] = s[r * 16 * kPad + (cc >> 4) * kPad + (cc & 15)];
    }
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
    double* dw8; CK(hipMalloc(&dw8, N * 8));
    { std::vector<double> h8(N); for (int i = 0; i < N; i++) h8[i] = htw[i].wq; CK(hipMemcpy(dw8, h8.data(), N * 8, hipMemcpyHostToDevice)); }
    timeit("rows var0 (16B tw)", [&] { hipLaunchKernelGGL(k_rows_var<0>, dim3(16, L), dim3(256), 0, 0, s, T, dw8); });
    timeit("rows var1 (8B tw)", [&] { hipLaunchKernelGGL(k_rows_var<1>, dim3(16, L), dim3(256), 0, 0, s, T, dw8); });
    timeit("rows var2 (no tw load)", [&] { hipLaunchKernelGGL(k_rows_var<2>, dim3(16, L), dim3(256), 0, 0, s, T, dw8); });
    {   // fp64 passes need the w/q tables: reuse the 8 B table for both directions
        T.psif = dw8; T.ipsif = dw8;
        T.cw = T.icw = tools_make_cw(dw8, dq, 1, logN);
        std::vector<double> hf(1, 1.0 / q); double* dnf; CK(hipMalloc(&dnf, 8)); CK(hipMemcpy(dnf, hf.data(), 8, hipMemcpyHostToDevice));
        T.ninvf = dnf;
        timeit("f64 fwd_cols", [&] { hipLaunchKernelGGL(k_nttf_fwd_cols, dim3(16, L), dim3(256), 0, 0, s, s2, T); });
        timeit("f64 fwd_rows", [&] { hipLaunchKernelGGL(k_nttf_fwd_rows_t<false>, dim3(16, L), dim3(256), 0, 0, s2, T, RowFin{}); });
        timeit("f64 inv_rows", [&] { hipLaunchKernelGGL(k_nttf_inv_rows, dim3(16, L), dim3(256), 0, 0, s, s2, T); });
        timeit("f64 inv_cols", [&] { hipLaunchKernelGGL(k_nttf_inv_cols, dim3(16, L), dim3(256), 0, 0, s2, T); });
        // a 40-bit prime (no folding path)
        u64 q40 = 1099511480321ULL; CK(hipMemcpy(dq, &q40, 8, hipMemcpyHostToDevice)); double qi40 = 1.0 / q40; CK(hipMemcpy(dqi, &qi40, 8, hipMemcpyHostToDevice));
        timeit("f64 fwd_cols q40", [&] { hipLaunchKernelGGL(k_nttf_fwd_cols, dim3(16, L), dim3(256), 0, 0, s, s2, T); });
        timeit("f64 fwd_rows q40", [&] { hipLaunchKernelGGL(k_nttf_fwd_rows_t<false>, dim3(16, L), dim3(256), 0, 0, s2, T, RowFin{}); });
        timeit("f64 inv_rows q40", [&] { hipLaunchKernelGGL(k_nttf_inv_rows, dim3(16, L), dim3(256), 0, 0, s, s2, T); });
        timeit("f64 inv_cols q40", [&] { hipLaunchKernelGGL(k_nttf_inv_cols, dim3(16, L), dim3(256), 0, 0, s2, T); });
        timeit("int fwd_rows q40", [&] { hipLaunchKernelGGL(k_ntt256_fwd_rows, dim3(16, L), dim3(256), 0, 0, s, T); });
    }
    timeit("inv_rows", [&] { hipLaunchKernelGGL(k_ntt256_inv_rows, dim3(16, L), dim3(256), 0, 0, s, s2, T); });
    timeit("inv_cols", [&] { hipLaunchKernelGGL(k_ntt256_inv_cols, dim3(16, L), dim3(256), 0, 0, s, T); });
    return 0;
}
