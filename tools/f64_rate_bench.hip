// f64_rate_bench.hip -- issue rate of the fp64 instructions the exact-fp64 modular arithmetic
// uses (kernels.h fmul_rem / fred): v_fma_f64, v_mul_f64, v_add_f64, v_rndne_f64 (rint), and the
// two ways to get qh = round(a * wq): mul + rint vs fma with the 1.5 * 2^52 magic + add.
// 8 independent chains per thread, 1024 workgroups x 256 threads, timed with hipEvents.
// hipcc --offload-arch=gfx950 -O3 -o tools/f64_rate_bench tools/f64_rate_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define C 8
constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k_rate(double* out, double s) {
    double x[C];
    for (int c = 0; c < C; c++) x[c] = s * (threadIdx.x + 1 + c * 7) + blockIdx.x;
    const double w = 1.0000001, q = 1125899906842597.0, qi = 1.0 / q, mg = 6755399441055744.0;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < C; c++) {
            if (OP == 0) x[c] = __builtin_fma(x[c], w, s);            // 1 fma
            if (OP == 1) x[c] = __builtin_rint(x[c]) + s;              // rint + add
            if (OP == 2) x[c] = x[c] + s;                              // add
            if (OP == 3) {                                             // fmul_rem as shipped (6)
                const double p = x[c] * w, pl = __builtin_fma(x[c], w, -p);
                const double qh = __builtin_rint(x[c] * qi);
                x[c] = __builtin_fma(-qh, q, p) + pl;
            }
            if (OP == 4) {                                             // magic rounding (6)
                const double p = x[c] * w, pl = __builtin_fma(x[c], w, -p);
                const double qh = __builtin_fma(x[c], qi, mg) - mg;
                x[c] = __builtin_fma(-qh, q, p) + pl;
            }
        }
    }
    double r = 0;
    for (int c = 0; c < C; c++) r += x[c];
    if (r == 12345.0) out[0] = r;
}

template <int OP>
static float run(double* d, const char* name, int per_iter) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 1024 * 8;
    hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, d, 1e-3);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_rate<OP>, dim3(grid), dim3(256), 0, 0, d, 1e-3);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lane_ops = (double)grid * 256 * ITERS * C * per_iter;
    std::printf("%-28s %8.3f ms  %7.2f T lane-ops/s (%d ops/iter)\n", name, ms, lane_ops / ms / 1e9, per_iter);
    return ms;
}

int main() {
    double* d;
    hipMalloc(&d, 64);
    run<0>(d, "fma", 1);
    run<2>(d, "add", 1);
    run<1>(d, "rint + add", 2);
    run<3>(d, "fmul_rem (mul+rint)", 6);
    run<4>(d, "fmul_rem (fma magic)", 6);
    hipFree(d);
    return 0;
}
