// Dev tool: k_bsgs_terms (the fused BSGS term sums, kernels_ops.h) on a synthetic CoeffToSlot map
// at the bench's shape -- N = 2^16, level 25 (ne = 36 limbs of Q u P), alpha = 12 (beta = 3),
// B ciphertexts, nb babies g_1^i (rotation stride 1), 2 giants -- timing variants: the k-block
// walk (orbit order vs 0, 1, 2, ...), the batch block BB and the wave target.  Values are
// arbitrary residues (timing only; parity is the GPU tests' job).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/bsgs_bench tools/bsgs_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../aes-fhe_amd/csrc/kernels_ops.h"
using namespace aesfhe;
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int LOGN = 16, N = 1 << LOGN, L = 25, K = 10, LP1 = 31, A = 12, NE = L + 1 + K, NP = LP1 + K;
constexpr int BETA = (L + 1 + A - 1) / A;

__global__ void k_fill(u64* p, long n, u64 seed) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        p[i] = ((u64)i * 0x9E3779B97F4A7C15ULL + seed) >> 25;  // < 2^39
}

static u64* dev(long words, u64 seed) {
    u64* p;
    HC(hipMalloc(&p, words * 8));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, p, words, seed);
    return p;
}

static std::vector<unsigned short> order(int nb, u64 g1, bool orbit) {
    const int nblk = N / 256;
    const u64 M = 2ULL * N;
    std::vector<unsigned short> o(nblk);
    for (int i = 0; i < nblk; i++) o[i] = i;
    if (!orbit) return o;
    auto brv = [&](u64 x) { return (u64)(__builtin_bitreverse32((unsigned)x) >> (32 - LOGN)); };
    auto pi = [&](int kb) {
        const u64 k = (u64)kb << 8, ek = 2 * brv(k) + 1;
        return (int)(brv((((g1 * ek) & (M - 1)) - 1) >> 1) >> 8);
    };
    std::vector<char> seen(nblk, 0);
    int n = 0;
    for (int s = 0; s < nblk; s++)
        for (int kb = s; !seen[kb]; kb = pi(kb)) seen[kb] = 1, o[n++] = kb;
    return o;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 32, nb = argc > 2 ? atoi(argv[2]) : 8, stride = argc > 3 ? atoi(argv[3]) : 1;
    const int gn = argc > 4 ? atoi(argv[4]) : 2;
    const long neN = (long)NE * N;
    std::vector<u64> q(NP);
    std::vector<double> qinv(NP), pmodf(LP1);
    for (int i = 0; i < NP; i++) q[i] = (1ULL << 40) - 87 - 2 * i, qinv[i] = 1.0 / (double)q[i];
    for (int i = 0; i < LP1; i++) pmodf[i] = 0.37;
    u64 *dq;
    double *dqinv, *dpm;
    HC(hipMalloc(&dq, NP * 8));
    HC(hipMalloc(&dqinv, NP * 8));
    HC(hipMalloc(&dpm, LP1 * 8));
    HC(hipMemcpy(dq, q.data(), NP * 8, hipMemcpyHostToDevice));
    HC(hipMemcpy(dqinv, qinv.data(), NP * 8, hipMemcpyHostToDevice));
    HC(hipMemcpy(dpm, pmodf.data(), LP1 * 8, hipMemcpyHostToDevice));
    u64* c = dev((long)B * 2 * (L + 1) * N, 1);
    u64* ext = dev((long)BETA * B * neN, 2);
    const long kdig = 2L * NP * N, kcomp = (long)NP * N;
    std::vector<const u64*> keys(nb, nullptr);
    std::vector<u64> gal(nb, 0);
    const u64 M = 2ULL * N;
    u64 g1 = 1;
    for (int s = 0; s < stride; s++) g1 = (g1 * 5) & (M - 1);
    u64 gp = 1;
    for (int i = 1; i < nb; i++) {
        keys[i] = dev((long)BETA * kdig, 10 + i);
        gp = (gp * g1) & (M - 1);
        gal[i] = gp;
    }
    std::vector<const u64*> pt((size_t)gn * nb);
    for (auto& p : pt) p = dev(neN, 99);
    std::vector<u64*> outs(gn);
    for (auto& p : outs) HC(hipMalloc(&p, (long)B * 2 * neN * 8));
    const u64 **dkeys, **dpt;
    u64 **douts, *dgal;
    HC(hipMalloc(&dkeys, nb * 8));
    HC(hipMalloc(&dpt, pt.size() * 8));
    HC(hipMalloc(&douts, gn * 8));
    HC(hipMalloc(&dgal, nb * 8));
    HC(hipMemcpy(dkeys, keys.data(), nb * 8, hipMemcpyHostToDevice));
    HC(hipMemcpy(dpt, pt.data(), pt.size() * 8, hipMemcpyHostToDevice));
    HC(hipMemcpy(douts, outs.data(), gn * 8, hipMemcpyHostToDevice));
    HC(hipMemcpy(dgal, gal.data(), nb * 8, hipMemcpyHostToDevice));
    unsigned short* dord[2];
    for (int o = 0; o < 2; o++) {
        auto v = order(nb, g1, o == 1);
        HC(hipMalloc(&dord[o], v.size() * 2));
        HC(hipMemcpy(dord[o], v.data(), v.size() * 2, hipMemcpyHostToDevice));
    }
    HC(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    // algorithmic bytes: ext + c once, keys and plaintexts once, outputs written
    const double alg = 8.0 * N * ((double)B * NE * BETA + (double)B * 2 * (L + 1) + (nb - 1) * 2.0 * BETA * NE + gn * nb * NE +
                                  gn * (double)B * 2 * NE);
    auto run = [&](const char* name, auto kern, int bb, int o) {
        auto launch = [&] {
            hipLaunchKernelGGL(kern, dim3((NE * (N / 256) + 7) / 8 * 8 * ((B + bb - 1) / bb)), dim3(256), 0, 0, (const u64*)c,
                               2L * (L + 1) * N, (const u64*)(c + (long)(L + 1) * N), 2L * (L + 1) * N, (const u64*)ext, neN,
                               (long)B * neN, (const u64* const*)dkeys, (const u64*)dgal, kdig, kcomp, (const u64* const*)dpt, nb,
                               gn, (u64* const*)douts, L, NE, BETA, A, (const u64*)dq, (const double*)dqinv, (const double*)dpm,
                               LP1, LOGN, B, (const unsigned short*)dord[o]);
        };
        launch();
        HC(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 3; r++) {
            HC(hipEventRecord(e0));
            for (int k = 0; k < 3; k++) launch();
            HC(hipEventRecord(e1));
            HC(hipEventSynchronize(e1));
            float ms;
            HC(hipEventElapsedTime(&ms, e0, e1));
            best = ms / 3 < best ? ms / 3 : best;
        }
        printf("%-14s %9.1f us  alg %.2f GB -> %6.2f TB/s\n", name, best * 1e3, alg / 1e9, alg / (best * 1e-3) / 1e12);
    };
    printf("B %d, nb %d babies (stride %d), beta %d, ne %d\n", B, nb, stride, BETA, NE);
    if (gn <= 2) {
        run("m4_b4_p1", (k_bsgs_terms<2, 4, 4, 1>), 4, 1);
        run("m3_b4_p1", (k_bsgs_terms<2, 3, 4, 1>), 4, 1);
        run("m3_b4_p2", (k_bsgs_terms<2, 3, 4, 2>), 4, 1);
        run("m3_b4_p2_lin", (k_bsgs_terms<2, 3, 4, 2>), 4, 0);
        run("m3_b4_p3", (k_bsgs_terms<2, 3, 4, 3>), 4, 1);
        run("m3_b8_p1", (k_bsgs_terms<2, 3, 8, 1>), 8, 1);
        run("m3_b3_p2", (k_bsgs_terms<2, 3, 3, 2>), 3, 1);
    } else {
        run("g4_m3_b4_p1", (k_bsgs_terms<4, 3, 4, 1>), 4, 1);
        run("g4_m3_b4_p2", (k_bsgs_terms<4, 3, 4, 2>), 4, 1);
        run("g4_m3_b2_p2", (k_bsgs_terms<4, 3, 2, 2>), 2, 1);
        run("g4_m3_b2_p1", (k_bsgs_terms<4, 3, 2, 1>), 2, 1);
    }
    return 0;
}
