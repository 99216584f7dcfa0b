// Memory skeleton of the ModUp base conversion (dev tool): the access pattern of
// k_bconv_mfma without its arithmetic, to separate the pattern's own rate from the kernel's.
// ns = 12 source limbs -> nt = 24 target limbs per batch element, N = 2^16, B = 32 (the round's
// ModUp of one 12-limb digit).  Variants:
//   cur   the kernel's pattern: workgroup = 256 coefficients (4 waves x 64), every lane reads its
//         12 slots x 2 column groups (256 B per half-wave), then writes 24 targets x 64 coeffs
//         (512 B per wave-store), nontemporal
//   plain the same with plain stores
//   wide  each wave owns 128 coefficients (two 64-coefficient passes over the same targets)
//   copy  a plain streaming copy of the same byte count (reads 1/3, writes 2/3 of it)
//   mfma  k_bconv_mfma<3, false> itself, then split over 1-3 target groups (blockIdx.y)
// Round-5 record (profiles/r05/ab/bconv_mem/variants.log): skeleton 86-90 us (6.7-7.0 TB/s), the
// kernel 107-120 us; variants of it measured there and dropped: one tile in flight at 68 VGPRs /
// 7 waves (107-111 us), the next coefficient block's source words prefetched across blocks
// (120-142 us), 5 waves forced (46 VGPRs spilled, 319 us), 2-3 target groups (125 / 145 us).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bconv_mem_bench tools/bconv_mem_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#include "../aes-fhe_amd/csrc/bconv_mfma.h"
using namespace aesfhe;
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

#ifndef BC_NT
#define BC_NT 24
#endif
#ifndef BC_SL
#define BC_SL BC_NS_DEFAULT
#endif
// BC_NT targets; BC_SL / BC_DL: limbs per batch element of the source / destination buffers, and
// BC_SKIP the digit's own limbs skipped in the destination (the round's digit 0 at l = 30:
// -DBC_NT=29 -DBC_SL=31 -DBC_DL=41 -DBC_SKIP=12)
#define BC_NS_DEFAULT 12
constexpr int LOGN = 16, N = 1 << LOGN, NS = 12, NT = BC_NT, B = 32;
#ifdef BC_DL
constexpr int SL = BC_SL, DL = BC_DL, SKIP = BC_SKIP;
#else
constexpr int SL = NS, DL = NT, SKIP = 0;
#endif

template <bool NTS, int PASSES>
__global__ __launch_bounds__(256) void k_skel(const u64* __restrict__ src, u64* __restrict__ dst) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
    const int z = blockIdx.z;
    for (int p = 0; p < PASSES; p++) {
        const long kb = ((long)blockIdx.x * PASSES + p) * 256 + w * 64;
        const u64* s = src + (long)z * NS * N;
        u64 acc[2] = {0, 0};
#pragma unroll
        for (int sl = 0; sl < NS / 2; sl++)
#pragma unroll
            for (int g = 0; g < 2; g++) acc[g] ^= s[((long)(2 * sl + h) << LOGN) + kb + 32 * g + c];
        const u64 v = acc[0] ^ (acc[1] << 1);
        u64* d = dst + (long)z * NT * N + kb + lane;
#pragma unroll 4
        for (int t = 0; t < NT; t++) {
            if (NTS)
                __builtin_nontemporal_store(v + t, d + ((long)t << LOGN));
            else
                d[(long)t << LOGN] = v + t;
        }
    }
}

typedef u64 v2u __attribute__((ext_vector_type(2)));
__global__ void k_copy(const v2u* __restrict__ a, v2u* __restrict__ b, long n, long nr) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const v2u v = a[i < nr ? i : i - nr];  // n = 2 nr
        __builtin_nontemporal_store(v, b + i);
    }
}

int main() {
    u64 *src, *dst;
    const size_t sb = (size_t)B * SL * N * 8, db = (size_t)B * DL * N * 8;
    HC(hipMalloc(&src, sb));
    HC(hipMalloc(&dst, db));
    HC(hipMemset(src, 1, sb));
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
        printf("%-8s %8.1f us  %6.2f TB/s (%zu MB read + %zu MB written)\n", name, best * 1e3, (sb + db) / (best * 1e-3) / 1e12,
               sb >> 20, db >> 20);
    };
    timeit("cur", [&] { hipLaunchKernelGGL((k_skel<true, 1>), dim3(N / 256, 1, B), dim3(256), 0, 0, src, dst); });
    timeit("plain", [&] { hipLaunchKernelGGL((k_skel<false, 1>), dim3(N / 256, 1, B), dim3(256), 0, 0, src, dst); });
    timeit("wide", [&] { hipLaunchKernelGGL((k_skel<true, 2>), dim3(N / 512, 1, B), dim3(256), 0, 0, src, dst); });
    timeit("wide4", [&] { hipLaunchKernelGGL((k_skel<true, 4>), dim3(N / 1024, 1, B), dim3(256), 0, 0, src, dst); });
    {  // the real kernel on the same shape (constants arbitrary: timing only)
        const int np = 64;
        std::vector<int8_t> tab((size_t)np * 8 * kBconvKT);
        for (auto& x : tab) x = (int8_t)(rand() & 255);
        std::vector<double> corr(np), pc(4 * np), qinv(np), sinvf(NS);
        std::vector<u64> q(np);
        for (int i = 0; i < np; i++) {
            q[i] = (1ULL << 40) - 87 - 2 * i;
            corr[i] = 12345.0;
            qinv[i] = 1.0 / (double)q[i];
            pc[4 * i] = (double)q[i], pc[4 * i + 1] = qinv[i], pc[4 * i + 2] = (double)((1ULL << 32) % q[i]);
            pc[4 * i + 3] = pc[4 * i + 2] / (double)q[i];
        }
        for (int i = 0; i < NS; i++) sinvf[i] = 0.3;
        int8_t* dtab;
        double *dcorr, *dpc, *dqinv, *dsinvf;
        u64* dq;
        HC(hipMalloc(&dtab, tab.size()));
        HC(hipMalloc(&dcorr, np * 8));
        HC(hipMalloc(&dpc, 4 * np * 8));
        HC(hipMalloc(&dqinv, np * 8));
        HC(hipMalloc(&dsinvf, NS * 8));
        HC(hipMalloc(&dq, np * 8));
        HC(hipMemcpy(dtab, tab.data(), tab.size(), hipMemcpyHostToDevice));
        HC(hipMemcpy(dcorr, corr.data(), np * 8, hipMemcpyHostToDevice));
        HC(hipMemcpy(dpc, pc.data(), 4 * np * 8, hipMemcpyHostToDevice));
        HC(hipMemcpy(dqinv, qinv.data(), np * 8, hipMemcpyHostToDevice));
        HC(hipMemcpy(dsinvf, sinvf.data(), NS * 8, hipMemcpyHostToDevice));
        HC(hipMemcpy(dq, q.data(), np * 8, hipMemcpyHostToDevice));
        HC(hipMemset(src, 0, sb));  // canonical inputs
        BconvArgs a{};
        a.src = src, a.sbs = (long)SL * N, a.scs = 0, a.dst = dst, a.dbs = (long)DL * N, a.dcs = 0, a.nc = 1, a.ns = NS;
        a.s_nq = NS, a.s_q0 = 30, a.s_p0 = 0, a.sinvf = dsinvf, a.einv = dsinvf, a.nt = NT, a.skip0 = SKIP ? 0 : NT, a.skipn = SKIP;
        a.tl_l = 1000, a.Lp1 = 0, a.tab = dtab, a.corr = dcorr, a.pc = dpc, a.qall = dq, a.qinvall = dqinv;
        a.tiles_per_group = (NT + 3) / 4;
        timeit("mfma", [&] { hipLaunchKernelGGL((k_bconv_mfma<3, false>), dim3(N / 256, 1, B), dim3(256), 0, 0, a, LOGN); });
        {  // the same on random canonical words (< 2^40, every q above): the kernel's power draw, and so
           // the clock it holds, depends on its data (MI355X_MICROARCH.md 'DVFS give-back')
            std::vector<u64> h((size_t)B * SL * N);
            uint64_t x = 88172645463325252ULL;
            for (auto& v : h) {
                x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                v = x & ((1ULL << 40) - 1);
                if (v >= (1ULL << 40) - 256) v -= 256;
            }
            HC(hipMemcpy(src, h.data(), sb, hipMemcpyHostToDevice));
            timeit("mfma_rnd", [&] { hipLaunchKernelGGL((k_bconv_mfma<3, false>), dim3(N / 256, 1, B), dim3(256), 0, 0, a, LOGN); });
            timeit("cur_rnd", [&] { hipLaunchKernelGGL((k_skel<true, 1>), dim3(N / 256, 1, B), dim3(256), 0, 0, src, dst); });
            HC(hipMemset(src, 0, sb));
            timeit("mfma_0", [&] { hipLaunchKernelGGL((k_bconv_mfma<3, false>), dim3(N / 256, 1, B), dim3(256), 0, 0, a, LOGN); });
        }
        for (int tg = 1; tg <= 3; tg++) {  // target groups split over blockIdx.y (more, shorter workgroups)
            a.tiles_per_group = (NT / 4 + tg - 1) / tg;
            char nm[32];
            snprintf(nm, sizeof nm, "groups%d", tg);
            timeit(nm, [&] { hipLaunchKernelGGL((k_bconv_mfma<3, false>), dim3(N / 256, tg, B), dim3(256), 0, 0, a, LOGN); });
        }
    }
    timeit("copy", [&] {
        hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (const v2u*)src, (v2u*)dst, (long)(db / 16), (long)(sb / 16));
    });
    return 0;
}
