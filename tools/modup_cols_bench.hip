// Dev tool (A/B for DESIGN.md §4.7): the key switch's ModUp of one digit followed by the
// extension limbs' NTT column pass, as the production pair (k_modup<A, 2> writing every
// extension limb, then k_nttf_fwd_cols<256> reading it back) against an LDS-resident fusion:
// one workgroup stages a 4-column x 256-row tile of the digit's A limbs (already times
// hatinv, 8 B each: A * 32 KB / 4 = 80 KB at A = 10) in LDS ONCE and loops over every target
// limb, each wave forming x_t = sum_i yhat_i hat_i,t for its 4 columns (the k_modup arithmetic)
// and running the 8 column stages in registers (16 lanes x 16 values per column, the
// k_nttf_fwd_cols arithmetic; the 16 x 16 transpose through the wave's own 8.5 KB of LDS).  The
// extension limb never reaches HBM; the y words are read from HBM once per tile instead of
// being written + read back once per target.  Outputs (raw-double intermediates) are compared
// word for word.  Synthetic chain: A source limbs + T targets (T - 10 of ~2^40 like the Q limbs
// at scale 40, 10 special of ~2^50), random residues and constants (the arithmetic is the same
// for any odd q < 2^51; NTT-friendliness does not change a single operation).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/modup_cols_bench tools/modup_cols_bench.hip
//   tools/modup_cols_bench [B] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../aes-fhe_amd/csrc/kernels_ops.h"
#include "../aes-fhe_amd/csrc/ntt256f.h"
#include "tabs_cw.h"
using namespace aesfhe;

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

constexpr int A = 10;       // digit width (alpha)
constexpr int TC = 4;       // columns per fused tile
constexpr int PADR = 4;     // transpose tile: (row * 4 + col) + 4 * (row >> 4) doubles

// grid (256 / TC tiles, B); 256 threads = 4 waves; targets t = w, w + 4, ... per wave.
// dc: [B][l+1][N] canonical coefficients (digit = limbs lo .. lo + A - 1); out: the extension
// span's layout [B][ne][N] (limb t of ct b at out + b * exs + t * N), targets t outside the digit.
__global__ __launch_bounds__(256) void k_modup_cols_lds(const u64* __restrict__ dc, long dcs, u64* __restrict__ out,
                                                        long exs, int lo, int l, int ne,
                                                        const double* __restrict__ hatinvf, const TwD* __restrict__ hat,
                                                        int hs, Tabs T) {
    extern __shared__ double lds[];
    double* sy = lds;                                        // [A][256][TC]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* sw = lds + A * 256 * TC + wave * (256 * PADR + 64);  // per-wave transpose tile
    double* twq = lds + A * 256 * TC + 4 * (256 * PADR + 64) + wave * 256;
    const int c0 = blockIdx.x * TC, bb = blockIdx.y;
    // 1. the digit's tile, times hatinv (k_modup's first step), into LDS
    for (int i = 0; i < A; i++) {
        const int pi = lo + i;
        const double qp = (double)T.q[pi];
        const double f = hatinvf[i], w = tw_w(f, qp);
        const u64* src = dc + (long)bb * dcs + ((long)pi << T.logN);
        for (int e = threadIdx.x; e < 256 * TC; e += 256) {
            const int r = e / TC, cc = e % TC;
            const double v = fmul_rem(u2d(src[r * 256 + c0 + cc]), w, f, qp);
            sy[(i * 256 + r) * TC + cc] = v < 0.0 ? v + qp : v;
        }
    }
    __syncthreads();
    const int cl = lane & 3, b = lane >> 2;
    const int c = c0 + cl;
    for (int t = wave; t < ne; t += 4) {
        if (t >= lo && t < lo + A) continue;  // wave-uniform
        const int pid = t <= l ? t : T.Lp1 + (t - l - 1);
        const double q = (double)T.q[pid], qi = T.qinv[pid];
        const bool big = q >= kBigPrime;
        const double* tg = T.psif + ((long)pid << T.logN);
        for (int e = lane; e < 256; e += 64) twq[e] = tg[e];
        TwD f[A];
#pragma unroll
        for (int i = 0; i < A; i++) f[i] = hat[pid * hs + i];
        // 2. x_t for rows a * 16 + b of column c (k_modup's second step, canonical)
        double x[16];
#pragma unroll
        for (int a = 0; a < 16; a++) {
            double acc = 0.0;
#pragma unroll
            for (int i = 0; i < A; i++) {
                acc += fmul_rem_r(sy[(i * 256 + a * 16 + b) * TC + cl], f[i].w, f[i].wq, q);
                if (big && (i & 3) == 3) acc = fred(acc, q, qi);
            }
            x[a] = u2d(fcanon(acc, q, qi));
        }
        // 3. the column pass (nttf_fwd_cols_body<256> with 4 columns per wave)
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const int m = 1 << st, hh = 8 >> st;
            if (big && st == 2) {
#pragma unroll
                for (int a = 0; a < 16; a++) x[a] = fred(x[a], q, qi);
            }
#pragma unroll
            for (int a = 0; a < 16; a++) {
                if (a & hh) continue;
                ct_f(x[a], x[a + hh], tg[m + (a >> (4 - st))], q);
            }
        }
        wave_sync_lds();  // the previous target's transpose reads (and twq writes) are done
#pragma unroll
        for (int a = 0; a < 16; a++) {
            const int row = a * 16 + b;
            sw[row * PADR + cl + 4 * (row >> 4)] = x[a];
        }
        wave_sync_lds();
        const int ap = b;
#pragma unroll
        for (int q2 = 0; q2 < 16; q2++) {
            const int row = ap * 16 + q2;
            x[q2] = sw[row * PADR + cl + 4 * (row >> 4)];
        }
#pragma unroll
        for (int st = 4; st < 8; st++) {
            const int m = 1 << st, hh = 128 >> st;
            if (big && (st & 1) == 0) {
#pragma unroll
                for (int q2 = 0; q2 < 16; q2++) x[q2] = fred(x[q2], q, qi);
            }
#pragma unroll
            for (int q2 = 0; q2 < 16; q2++) {
                if (q2 & hh) continue;
                ct_f(x[q2], x[q2 + hh], twq[m + ap * (m >> 4) + (q2 >> (8 - st))], q);
            }
        }
        u64* o = out + (long)bb * exs + ((long)t << T.logN);
#pragma unroll
        for (int q2 = 0; q2 < 16; q2++) st_d(&o[(ap * 16 + q2) * 256 + c], x[q2]);
        wave_sync_lds();
    }
}

template <int AA, typename... Args>
static void launch_modup(dim3 g, hipStream_t s, Args... args) {
    g.x /= 2;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_modup<AA, 2>), g, dim3(256), 0, s, args...);
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 16;
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    const int logN = 16, N = 1 << logN;
    const int K = 10, l = 30, Lp1 = l + 1, ne = l + 1 + K, np = Lp1 + K, lo = 0;
    std::mt19937_64 rng(7);
    std::vector<u64> q(np);
    std::vector<double> qinv(np);
    for (int i = 0; i < np; i++) {
        const int bits = i < Lp1 ? 40 : 50;
        q[i] = ((rng() >> (64 - bits)) | (1ULL << (bits - 1))) | 1ULL;
        qinv[i] = 1.0 / (double)q[i];
    }
    std::vector<double> psif((size_t)np * N);
    for (int i = 0; i < np; i++)
        for (int k = 0; k < N; k++) psif[(size_t)i * N + k] = (double)(rng() % q[i]) / (double)q[i];
    std::vector<double> hatinvf(A);
    for (int i = 0; i < A; i++) hatinvf[i] = (double)(rng() % q[lo + i]) / (double)q[lo + i];
    std::vector<TwD> hat((size_t)np * K);
    for (int t = 0; t < np; t++)
        for (int i = 0; i < K; i++) {
            const double w = (double)(rng() % q[t]);
            hat[(size_t)t * K + i] = TwD{w, w / (double)q[t]};
        }
    const long lN = (long)(l + 1) * N, neN = (long)ne * N;
    std::vector<u64> dch((size_t)B * lN);
    for (int b = 0; b < B; b++)
        for (int i = 0; i <= l; i++)
            for (int k = 0; k < N; k++) dch[(size_t)b * lN + (size_t)i * N + k] = rng() % q[i];
    u64 *dq, *dc, *ext1, *ext2;
    double *dqinv, *dpsif, *dhinv;
    TwD* dhat;
    CK(hipMalloc(&dq, np * 8));
    CK(hipMalloc(&dqinv, np * 8));
    CK(hipMalloc(&dpsif, psif.size() * 8));
    CK(hipMalloc(&dhinv, A * 8));
    CK(hipMalloc(&dhat, hat.size() * sizeof(TwD)));
    CK(hipMalloc(&dc, dch.size() * 8));
    CK(hipMalloc(&ext1, (size_t)B * neN * 8));
    CK(hipMalloc(&ext2, (size_t)B * neN * 8));
    CK(hipMemcpy(dq, q.data(), np * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dqinv, qinv.data(), np * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpsif, psif.data(), psif.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dhinv, hatinvf.data(), A * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dhat, hat.data(), hat.size() * sizeof(TwD), hipMemcpyHostToDevice));
    CK(hipMemcpy(dc, dch.data(), dch.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(ext1, 0, (size_t)B * neN * 8));
    CK(hipMemset(ext2, 0, (size_t)B * neN * 8));
    Tabs T{};
    T.q = dq;
    T.qinv = dqinv;
    T.psif = dpsif;
    T.logN = logN;
    T.cw = tools_make_cw(dpsif, dq, np, logN);
    T.Lp1 = Lp1;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const int nt = ne - A;  // targets: limbs A .. ne - 1 (digit 0)
    Span sp{ext1 + (long)A * N, neN, nt, (l + 1) - A, A, Lp1};
    const size_t lds = ((size_t)A * 256 * TC + 4 * (256 * PADR + 64) + 4 * 256) * 8;
    CK(hipFuncSetAttribute((const void*)k_modup_cols_lds, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    auto base = [&]() {
        launch_modup<A>(dim3(N / 256, 1, B), s, (const u64*)dc, lN, ext1, neN, lo, l, ne, (const double*)dhinv,
                        (const TwD*)dhat, K, (const u64*)dq, (const double*)dqinv, Lp1, logN);
        hipLaunchKernelGGL(k_nttf_fwd_cols<256>, dim3(16, B * nt), dim3(256), 0, s, sp, sp, T);
    };
    auto fused = [&]() {
        hipLaunchKernelGGL(k_modup_cols_lds, dim3(256 / TC, B), dim3(256), lds, s, (const u64*)dc, lN, ext2, neN, lo,
                           l, ne, (const double*)dhinv, (const TwD*)dhat, K, T);
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto fn) {
        fn();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; r++) fn();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return 1e3 * ms / reps;
    };
    // the column pass alone: in place (the engine's form) and out of place (into ext2's layout)
    Span sp2{ext2 + (long)A * N, neN, nt, (l + 1) - A, A, Lp1};
    auto cols_in = [&]() { hipLaunchKernelGGL(k_nttf_fwd_cols<256>, dim3(16, B * nt), dim3(256), 0, s, sp, sp, T); };
    auto cols_out = [&]() { hipLaunchKernelGGL(k_nttf_fwd_cols<256>, dim3(16, B * nt), dim3(256), 0, s, sp, sp2, T); };
    auto modup = [&]() {
        launch_modup<A>(dim3(N / 256, 1, B), s, (const u64*)dc, lN, ext1, neN, lo, l, ne, (const double*)dhinv,
                        (const TwD*)dhat, K, (const u64*)dq, (const double*)dqinv, Lp1, logN);
    };
    const double tci = timeit(cols_in), tco = timeit(cols_out), tm = timeit(modup), tci2 = timeit(cols_in), tco2 = timeit(cols_out);
    fprintf(stderr, "{\"cols_inplace_us\": [%.1f, %.1f], \"cols_outofplace_us\": [%.1f, %.1f], \"modup_us\": %.1f, "
            "\"cols_bytes\": %.0f}\n", tci, tci2, tco, tco2, tm, 16.0 * N * B * nt);
    const double tb = timeit(base), tf = timeit(fused), tb2 = timeit(base), tf2 = timeit(fused);
    CK(hipGetLastError());
    std::vector<u64> h1((size_t)B * neN), h2((size_t)B * neN);
    CK(hipMemcpy(h1.data(), ext1, h1.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), ext2, h2.size() * 8, hipMemcpyDeviceToHost));
    long diff = 0;
    for (int b = 0; b < B; b++)
        for (int t = A; t < ne; t++)
            for (int k = 0; k < N; k++) {
                const size_t o = (size_t)b * neN + (size_t)t * N + k;
                diff += h1[o] != h2[o];
            }
    // algorithmic bytes of the pair per call: y read (A limbs), extension limbs written (nt)
    const double alg = 8.0 * N * B * (A + nt);
    printf("{\"B\": %d, \"alpha\": %d, \"targets\": %d, \"lds_bytes\": %zu, \"modup_plus_cols_us\": [%.1f, %.1f], "
           "\"fused_lds_us\": [%.1f, %.1f], \"differing_words\": %ld, \"alg_bytes\": %.0f}\n",
           B, A, nt, lds, tb, tb2, tf, tf2, diff, alg);
    return diff != 0;
}
