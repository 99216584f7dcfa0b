// Memory skeleton of the NTT column pass (dev tool): k_nttf_fwd_cols's access
// pattern -- a workgroup reads a tile of columns x 256 rows (row stride 2 KB) and writes it back
// to another buffer -- without the butterflies, with 8-byte lanes (the kernel: 16 columns, lane
// (column, row group)) against 16-byte lanes (two adjacent columns per lane: 32 columns per
// 256-thread workgroup, or 16 columns per 128 threads).  468 limbs, N = 2^16, as tools/ntt_q_bench.
//   hipcc --offload-arch=gfx950 -O3 -o tools/cols_skel_bench tools/cols_skel_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64;
typedef u64 v2u __attribute__((ext_vector_type(2)));
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int N = 1 << 16;

// 8 B lanes: 16 columns x 256 rows per workgroup of 256 (lane: column tid & 15, rows a 16 + (tid >> 4))
__global__ __launch_bounds__(256) void k_s8(const u64* __restrict__ in, u64* __restrict__ out) {
    const int cl = threadIdx.x & 15, b = threadIdx.x >> 4, c = blockIdx.x * 16 + cl;
    const u64* src = in + (long)blockIdx.y * N;
    u64* dst = out + (long)blockIdx.y * N;
    u64 x[16];
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = src[(a * 16 + b) * 256 + c];
#pragma unroll
    for (int a = 0; a < 16; a++) __builtin_nontemporal_store(x[a] + 1, dst + (a * 16 + b) * 256 + c);
}
// 16 B lanes, 32 columns x 256 rows per 256 threads (lane: columns 2 (tid & 15) + {0, 1})
__global__ __launch_bounds__(256) void k_s16(const u64* __restrict__ in, u64* __restrict__ out) {
    const int cp = threadIdx.x & 15, b = threadIdx.x >> 4, c = blockIdx.x * 32 + 2 * cp;
    const u64* src = in + (long)blockIdx.y * N;
    u64* dst = out + (long)blockIdx.y * N;
    v2u x[16];
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = *(const v2u*)(src + (a * 16 + b) * 256 + c);
#pragma unroll
    for (int a = 0; a < 16; a++) __builtin_nontemporal_store(x[a] + 1, (v2u*)(dst + (a * 16 + b) * 256 + c));
}
// 16 B lanes, 16 columns x 256 rows per 128 threads (lane: columns 2 (tid & 7) + {0, 1}, 32 values)
__global__ __launch_bounds__(128) void k_s16h(const u64* __restrict__ in, u64* __restrict__ out) {
    const int cp = threadIdx.x & 7, b = threadIdx.x >> 3, c = blockIdx.x * 16 + 2 * cp;
    const u64* src = in + (long)blockIdx.y * N;
    u64* dst = out + (long)blockIdx.y * N;
    v2u x[16];
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = *(const v2u*)(src + (a * 16 + b) * 256 + c);
#pragma unroll
    for (int a = 0; a < 16; a++) __builtin_nontemporal_store(x[a] + 1, (v2u*)(dst + (a * 16 + b) * 256 + c));
}

int main() {
    const int limbs = 468;
    const size_t bytes = (size_t)limbs * N * 8;
    u64 *a, *b;
    HC(hipMalloc(&a, bytes));
    HC(hipMalloc(&b, bytes));
    HC(hipMemset(a, 1, bytes));
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) {
        launch();
        HC(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 5; r++) {
            HC(hipEventRecord(e0));
            for (int k = 0; k < 10; k++) launch();
            HC(hipEventRecord(e1));
            HC(hipEventSynchronize(e1));
            float ms;
            HC(hipEventElapsedTime(&ms, e0, e1));
            best = ms / 10 < best ? ms / 10 : best;
        }
        printf("%-40s %7.1f us  %5.2f TB/s\n", name, best * 1e3, 2.0 * bytes / (best * 1e-3) / 1e12);
    };
    timeit("8 B lanes, 16 cols / 256 thr (the pass)", [&] { hipLaunchKernelGGL(k_s8, dim3(16, limbs), dim3(256), 0, 0, a, b); });
    timeit("16 B lanes, 32 cols / 256 thr", [&] { hipLaunchKernelGGL(k_s16, dim3(8, limbs), dim3(256), 0, 0, a, b); });
    timeit("16 B lanes, 16 cols / 128 thr", [&] { hipLaunchKernelGGL(k_s16h, dim3(16, limbs), dim3(128), 0, 0, a, b); });
    timeit("8 B lanes, 16 cols / 256 thr (again)", [&] { hipLaunchKernelGGL(k_s8, dim3(16, limbs), dim3(256), 0, 0, a, b); });
    return 0;
}
