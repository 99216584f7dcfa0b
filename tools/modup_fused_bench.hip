// ModUp base conversion fused with the forward column pass (dev tool).
// The round's key-switch digit shapes at N = 2^16, l = 30, K = 10, alpha = 12 (digit j = 0, 1, 2:
// 12 / 12 / 7 sources -> 29 / 29 / 34 targets), B = 32 elements: the engine's pair
// (k_bconv_mfma into a buffer, k_nttf_fwd_cols out of place into ext) against k_bconv_cols
// (bconv_cols.h) writing ext directly.  Every output word of the fused kernel is checked against
// the pair mod q (the raw-double intermediates differ in representation, not in residue).
// Constants are arbitrary but in range (random w < q twiddles, random signed-byte tables).
//   hipcc --offload-arch=gfx950 -O3 -o tools/modup_fused_bench tools/modup_fused_bench.hip
//   tools/modup_fused_bench [digit] [B]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../aes-fhe_amd/csrc/bconv_cols.h"
#include "tabs_cw.h"
using namespace aesfhe;
#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static bool is_prime(u64 n) {
    if (n < 2) return false;
    for (u64 p : {2ULL, 3ULL, 5ULL, 7ULL, 11ULL, 13ULL, 17ULL, 19ULL, 23ULL, 29ULL, 31ULL, 37ULL}) {
        if (n % p == 0) return n == p;
    }
    u64 d = n - 1;
    int r = 0;
    while (!(d & 1)) d >>= 1, r++;
    auto mulm = [&](u64 a, u64 b) { return (u64)((unsigned __int128)a * b % n); };
    auto powm = [&](u64 a, u64 e) { u64 x = 1; while (e) { if (e & 1) x = mulm(x, a); a = mulm(a, a); e >>= 1; } return x; };
    for (u64 a : {2ULL, 3ULL, 5ULL, 7ULL, 11ULL, 13ULL, 17ULL, 19ULL, 23ULL, 29ULL, 31ULL, 37ULL}) {
        u64 x = powm(a, d);
        if (x == 1 || x == n - 1) continue;
        bool ok = false;
        for (int i = 1; i < r; i++) {
            x = mulm(x, x);
            if (x == n - 1) { ok = true; break; }
        }
        if (!ok) return false;
    }
    return true;
}

int main(int argc, char** argv) {
    constexpr int LOGN = 16, N = 1 << LOGN;
    // digit -1: ModDown's shape instead (the product's combined ModDown + rescale at l = 30:
    // sources q_30 + the 10 special primes and the v slot -> the 30 kept limbs, 2 components)
    const int digit = argc > 1 ? atoi(argv[1]) : 0;
    const int B = argc > 2 ? atoi(argv[2]) : 32;
    const bool only_cold = argc > 3 && !strcmp(argv[3], "cold");  // PMC runs: the cold launches only
    const bool md = digit < 0;
    const int L = 30, K = 10, A = 12, l = 30, Lp1 = L + 1, np = Lp1 + K, ne = l + 1 + K;
    const int lo = md ? 0 : digit * A, hi = md ? 0 : std::min(lo + A, l + 1);
    const int alpha = md ? K + 1 : hi - lo, nt = md ? l : ne - alpha, nc = md ? 2 : 1;
    const int nstep = (alpha + (md ? 1 : 0) + 3) / 4;
    printf("%s: %d sources -> %d targets, B = %d x %d, %d MFMA steps\n", md ? "moddown" : "modup", alpha, nt, B, nc, nstep);
    // primes: q_0 ~ 2^50, q_1..q_30 ~ 2^40, p_0..p_9 ~ 2^50, all = 1 mod 2N
    std::vector<u64> q(np);
    {
        u64 c = (1ULL << 50) + 1;
        while (!is_prime(c)) c -= 2 * N;
        q[0] = c;
        c = (1ULL << 40) + 1;
        for (int i = 1; i < Lp1; i++) {
            do c -= 2 * N; while (!is_prime(c));
            q[i] = c;
        }
        c = q[0];
        for (int i = Lp1; i < np; i++) {
            do c -= 2 * N; while (!is_prime(c));
            q[i] = c;
        }
    }
    uint64_t rs = 88172645463325252ULL;
    auto rnd = [&]() { rs ^= rs << 13, rs ^= rs >> 7, rs ^= rs << 17; return rs; };
    std::vector<double> qinv(np), psif((size_t)np * N), pc(4 * np), corr(np), sinvf(np);
    for (int i = 0; i < np; i++) {
        qinv[i] = 1.0 / (double)q[i];
        for (int k = 0; k < N; k++) psif[(size_t)i * N + k] = (double)(rnd() % q[i]) / (double)q[i];
        const u64 w32 = (1ULL << 32) % q[i];
        pc[4 * i] = (double)q[i], pc[4 * i + 1] = qinv[i], pc[4 * i + 2] = (double)w32, pc[4 * i + 3] = (double)w32 / (double)q[i];
        corr[i] = (double)(rnd() % q[i]);
        sinvf[i] = 1.0 / (double)q[i];  // y = x (the YIN fused kernel reads y directly)
    }
    std::vector<int8_t> tab((size_t)np * 8 * kBconvKT);
    for (auto& x : tab) x = (int8_t)(rnd() & 255);
    {  // as the engine's tables (bconv_row): zero bytes for the dead slots past the sources (and the
       // v slot's bytes 1..7), which the fused kernel does not zero in B
        const int live = alpha;  // ModDown: the 11 sources; the v slot (slot 11) keeps its byte 0
        for (size_t r = 0; r < tab.size() / kBconvKT; r++)
            for (int k = 8 * live; k < kBconvKT; k++)
                if (!(md && k == 8 * live)) tab[r * kBconvKT + k] = 0;
    }
    // sources: canonical words of the digit's primes, B elements of l + 1 limbs
    const long lN = (long)(l + 1) * N, neN = (long)ne * N;
    // ModDown: two components per element, words below every prime (canonical for any source)
    std::vector<u64> hsrc((size_t)(md ? 2 : 1) * B * lN);
    for (size_t r = 0; r < hsrc.size() / lN; r++)
        for (int i = 0; i <= l; i++)
            for (int k = 0; k < N; k++) hsrc[r * lN + (size_t)i * N + k] = md ? rnd() % (1ULL << 39) : rnd() % q[i];
    auto up = [&](const void* h, size_t n) { void* d; HC(hipMalloc(&d, n)); HC(hipMemcpy(d, h, n, hipMemcpyHostToDevice)); return d; };
    u64* dq = (u64*)up(q.data(), np * 8);
    double* dqinv = (double*)up(qinv.data(), np * 8);
    double* dpsif = (double*)up(psif.data(), psif.size() * 8);
    double* dpc = (double*)up(pc.data(), pc.size() * 8);
    double* dcorr = (double*)up(corr.data(), np * 8);
    double* dsinvf = (double*)up(sinvf.data(), np * 8);
    int8_t* dtab = (int8_t*)up(tab.data(), tab.size());
    u64* dsrc = (u64*)up(hsrc.data(), hsrc.size() * 8);
    u64 *dmu, *dext, *dext2;
    const size_t ow = (size_t)B * (md ? 2 * (size_t)l * N : (size_t)neN);  // output words
    HC(hipMalloc(&dmu, ow * 8));
    HC(hipMalloc(&dext, ow * 8));
    HC(hipMalloc(&dext2, ow * 8));
    HC(hipMemset(dext, 0, ow * 8));
    HC(hipMemset(dext2, 0, ow * 8));
    Tabs T{};
    T.q = dq, T.qinv = dqinv, T.psif = dpsif, T.logN = LOGN, T.Lp1 = Lp1;
    T.cw = tools_make_cw(dpsif, dq, np, LOGN);
    std::vector<double> einv(16, 0.0), sinvmd(16, 0.0);  // ModDown: 1 / e_j of the sources q_30, p_0 .. p_9
    for (int j = 0; j < K + 1; j++) einv[j] = sinvmd[j] = 1.0 / (double)q[j == 0 ? l : Lp1 + j - 1];
    double* deinv = (double*)up(einv.data(), einv.size() * 8);
    double* dsinvmd = (double*)up(sinvmd.data(), sinvmd.size() * 8);  // the pair's y = x (w = 1 per source prime)
    BconvArgs a{};
    const long kN = (long)l * N;  // ModDown: conv of the kept limbs 0 .. 29
    if (!md) {
        a.src = dsrc + (long)lo * N, a.sbs = lN, a.scs = 0, a.dst = dmu, a.dbs = neN, a.dcs = 0, a.nc = 1, a.ns = alpha;
        a.s_nq = alpha, a.s_q0 = lo, a.s_p0 = Lp1, a.sinvf = dsinvf + lo, a.nt = nt, a.skip0 = lo, a.skipn = alpha, a.tl_l = l;
    } else {  // the sources: limb 30 and the special limbs of dsrc's elements, as [B][2][11][N] rows of lN
        a.src = dsrc + (long)(l + 1 - alpha) * N, a.sbs = 2 * lN, a.scs = lN, a.dst = dmu, a.dbs = 2 * kN, a.dcs = kN;
        a.nc = 2, a.ns = alpha, a.s_nq = 1, a.s_q0 = l, a.s_p0 = Lp1, a.sinvf = dsinvmd, a.einv = deinv;
        a.nt = nt, a.skip0 = nt, a.skipn = 0, a.tl_l = l - 1;
    }
    a.Lp1 = Lp1, a.tab = dtab, a.corr = dcorr, a.pc = dpc, a.qall = dq, a.qinvall = dqinv;
    const int ntile = (nt + 3) / 4;
    a.tiles_per_group = ntile;
    auto pair = [&](bool conv, bool cols) {
        if (conv) {
            const dim3 g(N / 256, 1, B * nc);
            if (md) hipLaunchKernelGGL((k_bconv_mfma<3, true>), g, dim3(256), 0, 0, a, LOGN);
            else switch (nstep) {
                case 1: hipLaunchKernelGGL((k_bconv_mfma<1, false>), g, dim3(256), 0, 0, a, LOGN); break;
                case 2: hipLaunchKernelGGL((k_bconv_mfma<2, false>), g, dim3(256), 0, 0, a, LOGN); break;
                default: hipLaunchKernelGGL((k_bconv_mfma<3, false>), g, dim3(256), 0, 0, a, LOGN); break;
            }
        }
        if (cols) {
            if (md) {
                Span s1{dmu, kN, nt, nt, 0, Lp1}, s2{dext, kN, nt, nt, 0, Lp1};
                hipLaunchKernelGGL(k_nttf_fwd_cols<256>, dim3(16, B * 2 * nt), dim3(256), 0, 0, s1, s2, T);
                return;
            }
            auto fwd = [&](long off, int n, int nq, int p0) {
                Span s1{dmu + off, neN, n, nq, p0, Lp1}, s2{dext + off, neN, n, nq, p0, Lp1};
                hipLaunchKernelGGL(k_nttf_fwd_cols<256>, dim3(16, B * n), dim3(256), 0, 0, s1, s2, T);
            };
            if (lo > 0) fwd(0, lo, lo, 0);
            fwd((long)hi * N, ne - hi, (l + 1) - hi, hi);
        }
    };
    BconvArgs af = a;
    af.dst = dext2;
    int pf = 1;
    // pf: 0, 1, 2 = prefetch depth with 4 targets per workgroup; 3 = PF 1, 2 targets, 2 LDS tiles;
    // 4 = PF 1, 2 targets, 1 LDS tile
    auto fused = [&]() {
        const int tt = pf >= 3 ? 2 : 4, nti = (nt + tt - 1) / tt;
        const dim3 g(16 * B * nc * nti);
#define FV(S, P, TT_, LT_) do { if (md) hipLaunchKernelGGL((k_bconv_cols<S, true, true, P, TT_, LT_>), g, dim3(256), 0, 0, af, T, nti); \
                      else hipLaunchKernelGGL((k_bconv_cols<S, true, false, P, TT_, LT_>), g, dim3(256), 0, 0, af, T, nti); } while (0)
#define FM(S, MD) do { if (md) hipLaunchKernelGGL((k_bconv_cols<S, true, true, 1, 4, 2, MD>), g, dim3(256), 0, 0, af, T, nti); \
                      else hipLaunchKernelGGL((k_bconv_cols<S, true, false, 1, 4, 2, MD>), g, dim3(256), 0, 0, af, T, nti); } while (0)
#define FZ(S, P) do { if (P == 1 && pf == 3) FV(S, 1, 2, 2); else if (P == 1 && pf == 4) FV(S, 1, 2, 1); \
                      else if (P == 1 && pf == 5) FM(S, 1); else if (P == 1 && pf == 6) FM(S, 2); \
                      else FV(S, P, 4, 2); } while (0)
#define FS(S) do { if (pf == 0) FZ(S, 0); else if (pf == 2) FZ(S, 2); else FZ(S, 1); } while (0)  // 3..6: PF 1
        switch (nstep) {
            case 1: FS(1); break;
            case 2: FS(2); break;
            default: FS(3); break;
        }
#undef FS
#undef FZ
#undef FM
#undef FV
    };
    pair(true, true);
    for (int chk = 0; chk <= 4 && !only_cold; chk++) {
    pf = chk;
    HC(hipMemset(dext2, 0, ow * 8));
    fused();
    HC(hipDeviceSynchronize());
    {  // check: every target limb, residue equality
        std::vector<u64> r1(ow), r2(ow);
        HC(hipMemcpy(r1.data(), dext, r1.size() * 8, hipMemcpyDeviceToHost));
        HC(hipMemcpy(r2.data(), dext2, r2.size() * 8, hipMemcpyDeviceToHost));
        long bad = 0, tot = 0;
        double maxr = 0;
        const int nlimb = md ? l : ne;
        for (int bb = 0; bb < B * nc; bb++)
            for (int tl = 0; tl < nlimb; tl++) {
                if (!md && tl >= lo && tl < hi) continue;
                const int pid = tl <= l ? tl : Lp1 + tl - l - 1;
                const long long Q = (long long)q[pid];
                for (int k = 0; k < N; k++) {
                    const size_t o = (size_t)bb * nlimb * N + (size_t)tl * N + k;
                    double d1, d2;
                    memcpy(&d1, &r1[o], 8), memcpy(&d2, &r2[o], 8);
                    const long long i1 = (long long)d1, i2 = (long long)d2;
                    maxr = std::max(maxr, std::fabs(d2) / (double)Q);
                    if ((double)i1 != d1 || (double)i2 != d2 || ((i1 - i2) % Q) != 0) {
                        if (bad < 5) printf("  mismatch b %d limb %d k %d: %.1f vs %.1f\n", bb, tl, k, d1, d2);
                        bad++;
                    }
                    tot++;
                }
            }
        printf("check V%d: %ld / %ld words differ mod q (max |fused| = %.2f q)\n", pf, bad, tot, maxr);
        if (bad) return 1;
    }
    }
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
        const double by = 8.0 * N * B * nc * (alpha + nt);
        printf("%-28s %8.1f us  (%.2f TB/s of the fused kernel's read + write)\n", name, best * 1e3, by / (best * 1e-3) / 1e12);
        return best;
    };
    // cold: the 256 MiB Infinity Cache flushed (a 1 GiB memset) before every launch, so the sources
    // come from HBM as in the engine, where the INTT wrote them with streaming stores; per-launch events
    void* flush;
    HC(hipMalloc(&flush, 1ULL << 30));
    auto cold = [&](const char* name, auto launch) {
        launch();
        HC(hipDeviceSynchronize());
        float tot = 0;
        for (int r = 0; r < 10; r++) {
            HC(hipMemsetAsync(flush, r, 1ULL << 30));
            HC(hipEventRecord(e0));
            launch();
            HC(hipEventRecord(e1));
            HC(hipEventSynchronize(e1));
            float ms;
            HC(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        printf("%-28s %8.1f us  (cold: Infinity Cache flushed before each launch)\n", name, tot / 10 * 1e3);
    };
    cold("cold bconv_mfma", [&] { pair(true, false); });
    cold("cold cols", [&] { pair(false, true); });
    if (only_cold) {  // PMC passes: one fused variant alone (argv[4], default 1)
        pf = argc > 4 ? atoi(argv[4]) : 1;
        char nm[32];
        snprintf(nm, sizeof nm, "cold fused V%d", pf);
        cold(nm, fused);
        return 0;
    }
    for (pf = 0; pf <= 6; pf++) {  // 5 / 6: the conversion alone / the column stages alone (MODE 1 / 2)
        char nm[32];
        snprintf(nm, sizeof nm, "cold fused V%d", pf);
        cold(nm, fused);
    }
    for (int rep = 0; rep < 2; rep++) {
        timeit("bconv_mfma", [&] { pair(true, false); });
        timeit("cols", [&] { pair(false, true); });
        timeit("pair", [&] { pair(true, true); });
        for (pf = 0; pf <= 6; pf++) {
            char nm[32];
            snprintf(nm, sizeof nm, "fused V%d", pf);
            timeit(nm, fused);
        }
    }
    return 0;
}
