// Probe of gfx950's v_mfma_f64_16x16x4_f64 layout and rate against VALU fp64 FMAs (dev tool for
// the matrix-core S-box inner sums).
// Layout per cdna_hip_programming.md: lane l holds A[row l&15][k l>>4] and B[k l>>4][col l&15];
// D[row][col] sits in lane col + 16 (row & 3), register row >> 2.  Exactness: integer operands
// whose products and sums stay below 2^53 must come out exact (checked with 40-bit values).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_f64_probe tools/mfma_f64_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void k_probe(const double* A, const double* B, double* D) {
    const int l = threadIdx.x;
    v4d c = {};
    for (int s = 0; s < 4; s++)  // K = 16 in four steps
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(A[s * 64 + l], B[s * 64 + l], c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[l * 4 + r] = c[r];
}

__global__ void k_rate_mfma(int iters, double* out) {
    const double a = threadIdx.x, b = 3.0;
    v4d c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    double s = 0;
    for (int r = 0; r < 4; r++) s += c0[r] + c1[r] + c2[r] + c3[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_rate_valu(int iters, double* out) {
    double a[8];
    for (int u = 0; u < 8; u++) a[u] = threadIdx.x + u;
    const double m = 1.0000001, d = 0.5;
    for (int i = 0; i < iters; i++)
#pragma unroll
        for (int u = 0; u < 8; u++) a[u] = __builtin_fma(a[u], m, d);
    double s = 0;
    for (int u = 0; u < 8; u++) s += a[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    std::vector<double> A(256), B(256);
    srand(11);
    // A: small signed integers (S-box weights), B: 40-bit residues; sums of 16 stay < 2^48
    for (auto& x : A) x = (double)((rand() % 17) - 8);
    for (auto& x : B) x = (double)(((uint64_t)rand() << 20 ^ (uint64_t)rand()) & ((1ULL << 40) - 1));
    double Am[16][16], Bm[16][16];
    for (int s = 0; s < 4; s++)
        for (int l = 0; l < 64; l++) {
            Am[l & 15][4 * s + (l >> 4)] = A[s * 64 + l];
            Bm[4 * s + (l >> 4)][l & 15] = B[s * 64 + l];
        }
    double *dA, *dB, *dD;
    hipMalloc(&dA, 256 * 8);
    hipMalloc(&dB, 256 * 8);
    hipMalloc(&dD, 256 * 8);
    hipMemcpy(dA, A.data(), 256 * 8, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 256 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    std::vector<double> D(256);
    hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int row = 0; row < 16; row++)
        for (int col = 0; col < 16; col++) {
            long double want = 0;
            for (int k = 0; k < 16; k++) want += (long double)Am[row][k] * Bm[k][col];
            const int lane = col + 16 * (row & 3), reg = row >> 2;
            if (D[lane * 4 + reg] != (double)want) bad++;
        }
    printf("mfma_f64_16x16x4 layout (D: lane col + 16 (row & 3), reg row >> 2) + exact integer sums: %s (%d of 256 wrong)\n",
           bad ? "WRONG" : "confirmed", bad);
    if (bad) {  // try the other plausible map
        int bad2 = 0;
        for (int row = 0; row < 16; row++)
            for (int col = 0; col < 16; col++) {
                long double want = 0;
                for (int k = 0; k < 16; k++) want += (long double)Am[row][k] * Bm[k][col];
                const int lane = col + 16 * (row >> 2), reg = row & 3;
                if (D[lane * 4 + reg] != (double)want) bad2++;
            }
        printf("  alternative (lane col + 16 (row >> 2), reg row & 3): %d of 256 wrong\n", bad2);
    }
    double* dO;
    const int blocks = 256 * 8, iters = 2048;
    hipMalloc(&dO, blocks * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms = 0;
    hipLaunchKernelGGL(k_rate_mfma, dim3(blocks), dim3(256), 0, 0, 16, dO);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate_mfma, dim3(blocks), dim3(256), 0, 0, iters, dO);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("mfma f64 rate: %.1f TFLOP/s (%.3f ms)\n", 2.0 * 1024 * 4 * iters * (blocks * 4.0) / ms / 1e9, ms);
    hipLaunchKernelGGL(k_rate_valu, dim3(blocks), dim3(256), 0, 0, 16, dO);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate_valu, dim3(blocks), dim3(256), 0, 0, iters * 8, dO);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("valu f64 fma rate: %.1f TFLOP/s (%.3f ms)\n", 2.0 * 8 * iters * 8.0 * blocks * 256 / ms / 1e9, ms);
    return bad ? 1 : 0;
}
