// Probe of gfx950's v_mfma_f64_16x16x4_f64 for the S-box kernel's inner sums (dev tool):
//  1. layout: lane l holds A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15]; D register r of lane l
//     is D[row][l & 15] with row = (l >> 4) + 4 r (MI355X_MICROARCH.md) -- or 4 (l >> 4) + r;
//  2. exactness: small integer weights times 45-bit integers summed over K = 16 (four chained
//     MFMAs) against the int64 sums (every partial sum an integer below 2^53);
//  3. rates: cycles per MFMA back to back; v_fma_f64 alone; both in one wave (do the matrix and
//     vector pipes overlap?).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_f64_probe tools/mfma_f64_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// A: [16][16] (row, k), B: [16][16] (k, col); D = A B over K = 16 in four MFMAs of K = 4
__global__ void k_layout(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    v4d c = {0.0, 0.0, 0.0, 0.0};
    for (int s = 0; s < 4; s++)
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 16 + 4 * s + (l >> 4)], B[(4 * s + (l >> 4)) * 16 + (l & 15)], c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[l * 4 + r] = c[r];
}

template <int MODE>  // 0: MFMA only, 1: VALU FMA only, 2: both (independent chains)
__global__ void k_rate(int iters, double* out) {
    const double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    v4d c0 = {}, c1 = {}, c2 = {}, c3 = {};
    double f[16];
    for (int j = 0; j < 16; j++) f[j] = j * 1e-3 + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        if (MODE != 1) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
        }
        if (MODE != 0) {
#pragma unroll
            for (int r = 0; r < 4; r++)
#pragma unroll
                for (int j = 0; j < 16; j++) f[j] = __builtin_fma(f[j], a, b);
        }
    }
    double s = 0.0;
    for (int r = 0; r < 4; r++) s += c0[r] + c1[r] + c2[r] + c3[r];
    for (int j = 0; j < 16; j++) s += f[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    // 1 + 2: layout and exactness
    std::vector<double> A(256), B(256), D(256);
    srand(7);
    auto rnd = [] { return ((uint64_t)rand() << 31) ^ (uint64_t)rand(); };
    for (int i = 0; i < 256; i++) {
        A[i] = (double)((int)(rnd() % 33) - 16);
        B[i] = (double)((int64_t)(rnd() & ((1ull << 45) - 1)) - (1ll << 44));
    }
    double *dA, *dB, *dD;
    HC(hipMalloc(&dA, 2048));
    HC(hipMalloc(&dB, 2048));
    HC(hipMalloc(&dD, 2048));
    HC(hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice));
    HC(hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    HC(hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost));
    int bad1 = 0, bad2 = 0;
    for (int l = 0; l < 64; l++)
        for (int r = 0; r < 4; r++) {
            const int col = l & 15, row1 = (l >> 4) + 4 * r, row2 = 4 * (l >> 4) + r;
            int64_t s1 = 0, s2 = 0;
            for (int k = 0; k < 16; k++) {
                s1 += (int64_t)A[row1 * 16 + k] * (int64_t)B[k * 16 + col];
                s2 += (int64_t)A[row2 * 16 + k] * (int64_t)B[k * 16 + col];
            }
            bad1 += (double)s1 != D[l * 4 + r] || (int64_t)D[l * 4 + r] != s1;
            bad2 += (int64_t)D[l * 4 + r] != s2;
        }
    printf("mfma_f64_16x16x4 D row = (l>>4) + 4r, col = l&15, exact integer sums (K = 16, |A| <= 16, |B| < 2^44): %d of 256 wrong\n", bad1);
    printf("  alternative row = 4 (l>>4) + r: %d of 256 wrong\n", bad2);
    // 3: rates, 1024 blocks x 256 threads
    double* out;
    HC(hipMalloc(&out, 1024 * 256 * 8));
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    const int iters = 2000;
    auto run = [&](const char* name, auto kern, double mfma_per_iter, double fma_per_iter) {
        hipLaunchKernelGGL(kern, dim3(1024), dim3(256), 0, 0, iters, out);
        HC(hipDeviceSynchronize());
        HC(hipEventRecord(e0));
        hipLaunchKernelGGL(kern, dim3(1024), dim3(256), 0, 0, iters, out);
        HC(hipEventRecord(e1));
        HC(hipEventSynchronize(e1));
        float ms;
        HC(hipEventElapsedTime(&ms, e0, e1));
        const double waves = 1024.0 * 4, s = ms * 1e-3;
        const double mf = waves * iters * mfma_per_iter * 1024.0 * 2, vf = waves * iters * fma_per_iter * 64.0 * 2;
        printf("%-28s %8.3f ms  MFMA %6.1f TF  VALU %6.1f TF  total %6.1f TF\n", name, ms, mf / s / 1e12, vf / s / 1e12, (mf + vf) / s / 1e12);
    };
    run("MFMA f64 16x16x4 only", k_rate<0>, 4, 0);
    run("v_fma_f64 only", k_rate<1>, 0, 64);
    run("both in one wave", k_rate<2>, 4, 64);
    return 0;
}
