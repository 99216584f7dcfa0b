// Probe of gfx950's v_mfma_i32_32x32x32_i8 operand and result layout (dev tool).
// Hypothesis: lane l holds A[row l&31][k = 16 (l>>5) + j] and B[k = 16 (l>>5) + j][col l&31] in byte
// j = 0..15 of its 4-dword fragment, and D[row][col] sits in lane (col + 32 (row>>2 & 1)), register
// (row & 3) + 4 (row >> 3) (the dtype-independent 32x32 C/D map of cdna_hip_programming.md 3).
// Any k order that A and B share gives the same D, so random signed bytes checked against a CPU
// product prove the row / column / D maps and that the k map is common to both operands.
// Also times back-to-back MFMAs (cycles per instruction, one wave per SIMD).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_i8_probe tools/mfma_i8_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k_probe(const int8_t* A, const int8_t* B, int* D) {
    const int l = threadIdx.x;
    v4i a, b;
    for (int w = 0; w < 4; w++) {
        int x = 0, y = 0;
        for (int j = 0; j < 4; j++) {
            x |= (int)(uint8_t)A[l * 16 + 4 * w + j] << (8 * j);
            y |= (int)(uint8_t)B[l * 16 + 4 * w + j] << (8 * j);
        }
        a[w] = x;
        b[w] = y;
    }
    v16i c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; r++) D[l * 16 + r] = c[r];
}

// v_permlane32_swap semantics used by bconv_mfma.h swap_halves: (x, y) -> (x with lanes 32..63
// from y's lanes 0..31, y with lanes 0..31 from x's lanes 32..63)
__global__ void k_swap(unsigned* out) {
    const unsigned l = threadIdx.x;
    const auto r = __builtin_amdgcn_permlane32_swap(1000u + l, 2000u + l, false, false);
    out[l] = r[0];
    out[64 + l] = r[1];
}

__global__ void k_rate(int iters, int* out) {
    v4i a = {(int)threadIdx.x, 1, 2, 3}, b = {3, 2, 1, (int)threadIdx.x};
    v16i c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c3, 0, 0, 0);
    }
    int s = 0;
    for (int r = 0; r < 16; r++) s += c0[r] + c1[r] + c2[r] + c3[r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    std::vector<int8_t> A(64 * 16), B(64 * 16);
    srand(7);
    for (auto& x : A) x = (int8_t)(rand() & 255);
    for (auto& x : B) x = (int8_t)(rand() & 255);
    // logical matrices under the hypothesis
    int Am[32][32], Bm[32][32];
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
            Am[l & 31][16 * (l >> 5) + j] = A[l * 16 + j];
            Bm[16 * (l >> 5) + j][l & 31] = B[l * 16 + j];
        }
    int8_t *dA, *dB;
    int* dD;
    hipMalloc(&dA, 1024);
    hipMalloc(&dB, 1024);
    hipMalloc(&dD, 64 * 16 * 4);
    hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    std::vector<int> D(64 * 16);
    hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int row = 0; row < 32; row++)
        for (int col = 0; col < 32; col++) {
            long want = 0;
            for (int k = 0; k < 32; k++) want += (long)Am[row][k] * Bm[k][col];
            const int lane = col + 32 * ((row >> 2) & 1), reg = (row & 3) + 4 * (row >> 3);
            if (D[lane * 16 + reg] != want) bad++;
        }
    printf("mfma_i32_32x32x32_i8 layout hypothesis: %s (%d of 1024 wrong)\n", bad ? "WRONG" : "confirmed", bad);
    {
        unsigned* dS;
        hipMalloc(&dS, 128 * 4);
        hipLaunchKernelGGL(k_swap, dim3(1), dim3(64), 0, 0, dS);
        std::vector<unsigned> S(128);
        hipMemcpy(S.data(), dS, 128 * 4, hipMemcpyDeviceToHost);
        int sb = 0;
        for (unsigned l = 0; l < 64; l++) {
            const unsigned want0 = l < 32 ? 1000 + l : 2000 + (l - 32), want1 = l < 32 ? 1000 + l + 32 : 2000 + l;
            sb += (S[l] != want0) + (S[64 + l] != want1);
        }
        printf("permlane32_swap (x, y) -> (x[0..31] | y[0..31], x[32..63] | y[32..63]): %s (%d wrong; lane 0/32: %u %u / %u %u)\n",
               sb ? "WRONG" : "confirmed", sb, S[0], S[32], S[64], S[96]);
        bad += sb;
    }
    // rate: 1 wave per SIMD on every CU, 4 independent accumulators
    int* dO;
    const int blocks = 256 * 4, iters = 4096;
    hipMalloc(&dO, blocks * 64 * 4);
    hipLaunchKernelGGL(k_rate, dim3(blocks), dim3(64), 0, 0, 16, dO);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate, dim3(blocks), dim3(64), 0, 0, iters, dO);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = 2.0 * 32 * 32 * 32 * 4.0 * iters * blocks;
    printf("rate: %.1f TOPS i8 (%d waves x %d x 4 MFMA in %.3f ms)\n", ops / ms / 1e9, blocks, iters, ms);
    return bad ? 1 : 0;
}
