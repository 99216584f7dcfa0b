// Dev tool: issue cost of the quotient step of fmul_rem (kernels.h) on gfx950 -- rint(a * wq)
// (v_mul_f64 + v_rndne_f64) against the magic-number form fma(a, wq, 1.5 * 2^52) - 1.5 * 2^52
// (v_fma_f64 + v_add_f64, the correctly rounded quotient) -- and of v_rndne_f64 alone, on 8
// independent chains per lane.  Also counts, on the host, how often the two quotients differ.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/rint_bench tools/rint_bench.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>

constexpr double kM = 6755399441055744.0;  // 1.5 * 2^52

template <int V>
__device__ __forceinline__ double fmr(double a, double w, double wq, double q) {
    const double p = a * w;
    const double pl = __builtin_fma(a, w, -p);
    double qh;
    if (V == 0) qh = __builtin_rint(a * wq);
    else qh = __builtin_fma(a, wq, kM) - kM;
    const double u = __builtin_fma(-qh, q, p);
    return u + pl;
}

template <int V>
__global__ __launch_bounds__(256) void kern(double* out, double w, double wq, double q, int iters) {
    double x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = (double)(threadIdx.x * 8 + j + 1);
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (V <= 1) {
                double r = fmr<V>(x[j], w, wq, q);
                x[j] = r < 0.0 ? r + q : r;
            } else {
                x[j] = __builtin_rint(x[j] * 0.75 + 0.3);  // v_fma + v_rndne per step
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const double q = 1099511627689.0;  // ~2^40
    const double w = 123456789012.0, wq = w / q;
    double* out;
    hipMalloc(&out, 8 << 20);
    const int blocks = 256 * 16, threads = 256, iters = 2048;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = {"fmul_rem rint (mul + rndne)", "fmul_rem magic (fma + add)", "fma + rndne chain"};
    for (int v = 0; v < 3; v++) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(a);
            if (v == 0) kern<0><<<blocks, threads>>>(out, w, wq, q, iters);
            if (v == 1) kern<1><<<blocks, threads>>>(out, w, wq, q, iters);
            if (v == 2) kern<2><<<blocks, threads>>>(out, w, wq, q, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        const double ops = 8.0 * blocks * threads * iters;
        printf("%-30s %8.3f ms  %8.1f G ops/s\n", names[v], best, ops / (best * 1e6));
    }
    // host: how often do the two quotients differ (ties of a * wq near .5)
    std::mt19937_64 rng(3);
    long diff = 0, n = 20000000;
    for (long i = 0; i < n; i++) {
        const double qq = (double)((rng() >> 14) | 1ULL);  // ~2^50
        const double ww = (double)(rng() % (unsigned long long)qq), wwq = ww / qq;
        const double aa = (double)(rng() >> 13);            // < 2^51
        const double q1 = std::rint(aa * wwq), q2 = std::fma(aa, wwq, kM) - kM;
        diff += q1 != q2;
    }
    printf("quotients differ in %ld of %ld random cases\n", diff, n);
    return 0;
}
