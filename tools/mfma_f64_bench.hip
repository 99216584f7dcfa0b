// f64 MFMA on gfx950: operand / result layout check with exact integer data, and the issue rate
// of v_mfma_f64_16x16x4_f64 alone and beside independent fp64 VALU work (co-issue from two
// waves on one SIMD).  hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_bench.hip -o tools/mfma_f64_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// A [16][4], B [4][16] row-major; D [16][16]
__global__ void k_layout(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    double a = A[(l & 15) * 4 + (l >> 4)];
    double b = B[(l >> 4) * 16 + (l & 15)];
    d4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = c[r];
}

// NM independent accumulators, iters MFMAs each; VALU: nv dependent-free fp64 fma chains per MFMA
template <int NM, int NV>
__global__ void __launch_bounds__(256) k_rate(double* out, int iters, double s) {
    const int l = threadIdx.x;
    double a = 1.0 + l * s, b = 2.0 - l * s;
    d4 c[NM];
    for (int m = 0; m < NM; m++) c[m] = d4{0, 0, 0, 0};
    double v[NV > 0 ? NV : 1];
    for (int j = 0; j < (NV > 0 ? NV : 1); j++) v[j] = l * 0.5 + j;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int m = 0; m < NM; m++) c[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[m], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < NV; j++) v[j] = __builtin_fma(v[j], s, a);
    }
    double t = 0;
    for (int m = 0; m < NM; m++) t += c[m][0] + c[m][1] + c[m][2] + c[m][3];
    for (int j = 0; j < (NV > 0 ? NV : 1); j++) t += v[j];
    out[blockIdx.x * blockDim.x + l] = t;
}

// VALU only: NV independent fma chains
template <int NV>
__global__ void __launch_bounds__(256) k_valu(double* out, int iters, double s) {
    const int l = threadIdx.x;
    double a = 1.0 + l * s;
    double v[NV];
    for (int j = 0; j < NV; j++) v[j] = l * 0.5 + j;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int j = 0; j < NV; j++) v[j] = __builtin_fma(v[j], s, a);
    }
    double t = 0;
    for (int j = 0; j < NV; j++) t += v[j];
    out[blockIdx.x * blockDim.x + l] = t;
}

template <typename K>
float timeit(K kern, int blocks, int threads, double* out, int iters) {
    hipEvent_t a, b;
    HC(hipEventCreate(&a)); HC(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, 1e-9);
    HC(hipEventRecord(a));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, 1e-9);
    HC(hipEventRecord(b));
    HC(hipEventSynchronize(b));
    float ms;
    HC(hipEventElapsedTime(&ms, a, b));
    return ms / 5;
}

int main() {
    std::vector<double> A(64), B(64), D(256), R(256, 0);
    srand(3);
    for (auto& x : A) x = (double)((rand() % 17) - 8);
    for (int i = 0; i < 64; i++) B[i] = (double)((long)rand() * 7919 % (1L << 40)) - (double)(1L << 39);
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++)
            for (int k = 0; k < 4; k++) R[i * 16 + j] += A[i * 4 + k] * B[k * 16 + j];
    double *dA, *dB, *dD, *out;
    HC(hipMalloc(&dA, 512)); HC(hipMalloc(&dB, 512)); HC(hipMalloc(&dD, 2048));
    HC(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice));
    HC(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    HC(hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 256; i++) bad += D[i] != R[i];
    printf("layout: %d of 256 results differ from the exact integer product\n", bad);
    const int cus = 256, iters = 4096;
    HC(hipMalloc(&out, (size_t)cus * 8 * 256 * 8));
    // one wave per SIMD: 256 threads per block = 4 waves, one block per CU
    struct { const char* name; float ms; int mf; int nv; int waves; } rs[16];
    int n = 0;
#define RUN(NM, NV, WPS) { float ms = timeit(k_rate<NM, NV>, cus * WPS, 256, out, iters); rs[n++] = {#NM "x mfma + " #NV " valu, waves/SIMD " #WPS, ms, NM, NV, WPS}; }
    RUN(4, 0, 1) RUN(4, 0, 2) RUN(1, 0, 1) RUN(2, 0, 2) RUN(4, 4, 1) RUN(4, 8, 1) RUN(4, 16, 1) RUN(4, 8, 2) RUN(4, 16, 2) RUN(4, 32, 2)
    for (int i = 0; i < n; i++) {
        const double mf = (double)cus * 4 * rs[i].waves * iters * rs[i].mf;  // MFMAs issued
        const double cyc = rs[i].ms * 1e-3 * 2.4e9;                             // at 2.4 GHz
        printf("%-40s %8.3f ms  %6.1f cyc/MFMA/SIMD  valu/mfma %d\n", rs[i].name, rs[i].ms,
               cyc / (mf / (cus * 4)), rs[i].nv);
    }
    for (int wps = 1; wps <= 2; wps++) {
        float ms = timeit(k_valu<16>, cus * wps, 256, out, iters);
        const double fmas = (double)cus * 4 * wps * iters * 16;  // wave-instructions
        printf("valu only 16 chains, waves/SIMD %d: %8.3f ms  %5.2f cyc per wave-fma per SIMD\n", wps, ms,
               ms * 1e-3 * 2.4e9 / (fmas / (cus * 4)));
    }
    return 0;
}
