// Dev tool: the forward N = 2^16 NTT as ONE persistent launch in which column-pass tasks hand
// their raw-double intermediate to row-pass tasks of the same limb (per-limb arrival counter,
// agent-scope release / acquire), against the two-launch form.  Tasks come from 8 queues (block
// b serves queue b % 8 = the workgroups sharing an XCD, so a limb's producer and consumer tasks
// normally share that XCD's L2); a queue lists the 16 column tasks of its limb k, then, `lag`
// limbs later, the 16 row tasks of limb k.  A task waits only on tasks dequeued before it, so
// the launch cannot deadlock whatever the residency; every spin is bounded (timeout word).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/ntt_fuse_bench tools/ntt_fuse_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../aes-fhe_amd/csrc/ntt256f.h"
#include "tabs_cw.h"
using namespace aesfhe;

__global__ __launch_bounds__(256) void k_fused_fwd(Span src, Span mid, Tabs T, unsigned* head, unsigned* cnt,
                                                   unsigned* tmo, int limbs, int lag) {
    __shared__ double s[256 * kPadF];
    __shared__ double twq[256];
    __shared__ unsigned task_s;
    const int q = blockIdx.x & 7;
    const int nk = (limbs - q + 7) / 8;
    const int L = lag < nk ? lag : nk;
    const unsigned ntasks = 32u * nk;
    for (;;) {
        __syncthreads();  // the previous task's LDS reads are done
        if (threadIdx.x == 0) task_s = atomicAdd(&head[q], 1u);
        __syncthreads();
        const unsigned i = task_s;
        if (i >= ntasks) break;
        bool prod;
        int k, blk;
        if (i < 16u * L) {
            prod = true, k = i / 16, blk = i % 16;
        } else {
            const unsigned j = i - 16u * L;
            if (j < 32u * (nk - L)) {
                const int st = L + j / 32, r = j % 32;
                prod = r < 16;
                k = prod ? st : st - L;
                blk = r & 15;
            } else {
                const unsigned j2 = j - 32u * (nk - L);
                prod = false, k = nk - L + j2 / 16, blk = j2 % 16;
            }
        }
        const int y = q + 8 * k;
        if (prod) {
            nttf_fwd_cols_body<256>(src, mid, T, blk, y, s, twq);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add(&cnt[y], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            if (threadIdx.x == 0) {
                unsigned spins = 0;
                while (__hip_atomic_load(&cnt[y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 16u) {
                    __builtin_amdgcn_s_sleep(2);
                    if (++spins > (1u << 24)) {
                        atomicOr(tmo, 1u);
                        break;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __syncthreads();
            nttf_fwd_rows_body<false, 256>(mid, T, RowFin{}, blk, y, s);
        }
    }
}

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_) {                                                             \
            printf("%s @%d\n", hipGetErrorString(e_), __LINE__);              \
            return 1;                                                         \
        }                                                                     \
    } while (0)

template <class T>
static T* up(const std::vector<T>& v) {
    T* d = nullptr;
    if (hipMalloc(&d, v.size() * sizeof(T)) != hipSuccess) abort();
    if (hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) abort();
    return d;
}
__global__ void k_copy16(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ b, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

int main(int argc, char** argv) {
    const int logN = 16, N = 1 << logN, L = 30, K = 8;
    const int limbs = argc > 1 ? atoi(argv[1]) : 468;  // 12 x 39
    Chain ch = make_chain(logN, L, K, 50, 50, 40);
    const int np = (int)ch.q.size();
    std::vector<u64> hq(ch.q);
    std::vector<double> hqi(np), hpsif((size_t)np * N), hr((size_t)np * 2048);
    for (int p = 0; p < np; p++) {
        u64 q = hq[p];
        hqi[p] = 1.0 / (double)q;
        u64 psi = min_primitive_root(q, N);
        std::vector<u64> pw(N);
        pw[0] = 1;
        for (int k = 1; k < N; k++) pw[k] = h_mulmod(pw[k - 1], psi, q);
        for (int k = 0; k < N; k++) hpsif[(size_t)p * N + k] = (double)pw[bit_reverse(k, logN)] / (double)q;
        for (int row = 0; row < 256; row++)
            for (int sh = 0; sh < 8; sh++) hr[(size_t)p * 2048 + row * 8 + sh] = hpsif[(size_t)p * N + (row << sh)];
    }
    Tabs T{};
    T.q = up(hq);
    T.qinv = up(hqi);
    T.psif = up(hpsif);
    T.rtwf = up(hr);
    T.logN = logN;
    T.cw = tools_make_cw(T.psif, T.q, np, logN);
    T.Lp1 = np;
    std::vector<u64> h((size_t)limbs * N);
    std::mt19937_64 rng(7);
    for (int y = 0; y < limbs; y++)
        for (int k = 0; k < N; k++) h[(size_t)y * N + k] = rng() % hq[y % np];
    u64 *src = up(h), *d1, *d2;
    const size_t bytes = (size_t)limbs * N * 8;
    CK(hipMalloc(&d1, bytes));
    CK(hipMalloc(&d2, bytes));
    unsigned* ctl;  // [0, 8): heads, [8]: timeout, [16, 16 + limbs): arrival counters
    const size_t ctl_bytes = ((16 + limbs) * 4 + 15) / 16 * 16;
    CK(hipMalloc(&ctl, ctl_bytes));
    Span ss{src, (long)np * N, np, np, 0, 0}, s1{d1, (long)np * N, np, np, 0, 0}, s2{d2, (long)np * N, np, np, 0, 0};
    auto two_pass = [&] {
        hipLaunchKernelGGL(k_nttf_fwd_cols<256>, dim3(16, limbs), dim3(256), 0, 0, ss, s1, T);
        hipLaunchKernelGGL((k_nttf_fwd_rows_t<false, 256>), dim3(16, limbs), dim3(256), 0, 0, s1, T, RowFin{});
    };
    int grid = 1024, lag = 2;
    auto fused = [&] {
        hipMemsetAsync(ctl, 0, ctl_bytes, 0);
        hipLaunchKernelGGL(k_fused_fwd, dim3(grid), dim3(256), 0, 0, ss, s2, T, ctl, ctl + 16, ctl + 8, limbs, lag);
    };
    two_pass();
    fused();
    CK(hipDeviceSynchronize());
    std::vector<u64> r1((size_t)limbs * N), r2((size_t)limbs * N);
    CK(hipMemcpy(r1.data(), d1, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r2.data(), d2, bytes, hipMemcpyDeviceToHost));
    unsigned tmo = 0;
    CK(hipMemcpy(&tmo, ctl + 8, 4, hipMemcpyDeviceToHost));
    long bad = 0;
    for (size_t i = 0; i < r1.size(); i++) bad += r1[i] != r2[i];
    printf("limbs %d: fused vs two-pass mismatches %ld, timeout %u\n", limbs, bad, tmo);
    if (bad || tmo) return 2;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, auto fn) {
        for (int w = 0; w < 3; w++) fn();
        hipEventRecord(a);
        const int it = 20;
        for (int i = 0; i < it; i++) fn();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1000 / it;
        printf("%-40s %8.1f us  alg %7.1f GB/s  frac %.3f\n", name, us, 16.0 * limbs * N / (us * 1e3),
               16.0 * limbs * N / (us * 1e3) / 8000.0);
    };
    timeit("copy 16 B / lane", [&] { hipLaunchKernelGGL(k_copy16, dim3((long)limbs * N / 512), dim3(256), 0, 0, (const ulonglong2*)src, (ulonglong2*)d2, (long)limbs * N / 2); });
    timeit("two-pass forward (cols + rows)", two_pass);
    for (int g : {512, 768, 1024})
        for (int lg : {1, 2, 4, 8}) {
            grid = g, lag = lg;
            char nm[64];
            snprintf(nm, sizeof nm, "fused grid %d lag %d", g, lg);
            timeit(nm, fused);
        }
    CK(hipMemcpy(&tmo, ctl + 8, 4, hipMemcpyDeviceToHost));
    printf("timeouts after timing: %u\n", tmo);
    return tmo ? 3 : 0;
}
