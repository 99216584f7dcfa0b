// Dev tool: experimental one-launch forward NTTs (k_nttf_fwd_q / _q2, below) against the two-pass
// kernels on the bench's prime chain (N = 2^16, L = 30, K = 8: 39 primes, limbs cycle over
// them like a ciphertext batch), bit-exact check + timing.  Also checks the FIN epilogue.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/ntt_q_bench tools/ntt_q_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../aes-fhe_amd/csrc/ntt256f.h"
#include "tabs_cw.h"
using namespace aesfhe;

// ===== experimental one-launch forward NTT kernels (not in the engine: measured slower than
// the two-pass form) =====
namespace aesfhe {
// ---------------------------------------------------------------------------------------------
// Forward NTT in ONE launch (N = 2^16): the first two CT stages (m = 1, 2) split the transform
// into four independent 2^14-point sub-transforms, one per output quarter (bit-reversed output
// order keeps each quarter contiguous).  Workgroup (limb, quarter s) of 1024 threads reads the
// four input quarters at k, k + N/4, k + N/2, k + 3N/4, forms its radix-4 output
// (s = 0: (a0 + w1 a2) + w2 (a1 + w1 a3), s = 1: ... - w2 (...), s = 2/3: (a0 - w1 a2) +- w3
// (a1 - w1 a3)), then runs the remaining 14 stages (m' = m / 4 = 1 .. 2^13, twiddle
// psi^{brv(4 m' + s m' + i')}) with the whole 128 KB sub-transform resident in LDS: 16
// registers per thread, four register groups (distances 2^13..2^10 | 2^9..2^6 | 2^5..2^2 |
// 2, 1) with an LDS exchange between groups.  Each limb is read once from HBM and written
// once -- the intermediate of the two-pass form never leaves the CU.  The four quarter
// workgroups of a limb are blocks b, b + 8, b + 16, b + 24 (dealt round-robin over the 8
// XCDs, so they normally share an XCD's L2 and the 4x re-read of the input is an L2 hit;
// placement only affects speed, never correctness).  NOT in place: src and dst must not
// overlap (the quarters of a limb are read by all four workgroups).
// Ranges: c in (-2q, 3q) after the head, +q per stage (table twiddles): primes < 2^42 reach
// 17q; larger primes fold c and then before every second stage (as the two-pass kernels).
constexpr int kQPad = 16384 + 2 * (16384 >> 6);  // LDS words: index k -> k + 2 (k >> 6)
__device__ __forceinline__ int qp(int k) { return k + 2 * (k >> 6); }

// MODE: timing knobs for tools/ntt_q_bench.hip only (wrong results; 0 in the engine):
// 1 = head reads its own quarter only, 2 = no butterflies, 4 = no LDS exchanges.
template <bool FIN, int MODE = 0>
__global__ __launch_bounds__(1024) void k_nttf_fwd_q(Span src, Span dst, Tabs T, RowFin fin, int total) {
    __shared__ double lds[kQPad];
    const int b = blockIdx.x, g = b & 7, r = b >> 3, qs = r & 3;
    const int limb = (r >> 2) * 8 + g;
    if (limb >= total) return;
    int pid;
    const u64* in = span_ptr(src, limb, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, limb, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* W = T.psif + ((long)pid << 16);
    double x[16];
    // ---- head: stages m = 1, 2 restricted to quarter qs; k = tid + 1024 j
    {
        const double w1q = W[1], w1 = tw_w(w1q, q);
        const double wsq = W[2 + (qs >> 1)], ws = tw_w(wsq, q);
        const double s1 = qs >= 2 ? -1.0 : 1.0, s2 = (qs & 1) ? -1.0 : 1.0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int k = tid + 1024 * j;
            double a0, a1, a2, a3;
            if (MODE & 1) {
                a0 = u2d(in[k + qs * 16384]);
                a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
            } else {
                a0 = u2d(in[k]), a1 = u2d(in[k + 16384]);
                a2 = u2d(in[k + 32768]), a3 = u2d(in[k + 49152]);
            }
            const double u = a0 + s1 * fmul_rem(a2, w1, w1q, q);
            const double v = a1 + s1 * fmul_rem(a3, w1, w1q, q);
            x[j] = u + s2 * fmul_rem(v, ws, wsq, q);
        }
    }
    auto ctq = [&](double& xa, double& xb, double wq, double qq) {
        if (!(MODE & 2)) ct_f(xa, xb, wq, qq);
        else xa += wq;
    };
    const double* Wq = W;  // twiddle of (m', i') at 4 m' + qs m' + i' = m' (4 + qs) + i'
    const int q4 = 4 + qs;
    // ---- group 0: m' = 1, 2, 4, 8 (distances 2^13 .. 2^10), k = tid + 1024 j
#pragma unroll
    for (int st = 0; st < 4; st++) {
        const int ml = 1 << st, h = 8 >> st;
        if (big && (st & 1) == 0) {
#pragma unroll
            for (int j = 0; j < 16; j++) x[j] = fred(x[j], q, qi);
        }
#pragma unroll
        for (int jj = 0; jj < ml; jj++) {
            const double wq = Wq[ml * q4 + jj];  // uniform: scalar load
#pragma unroll
            for (int k = 0; k < h; k++) ctq(x[jj * 2 * h + k], x[jj * 2 * h + k + h], wq, q);
        }
    }
#pragma unroll
    for (int j = 0; j < 16; j++) if (!(MODE & 4)) lds[qp(tid + 1024 * j)] = x[j];
    __syncthreads();
    // ---- group 1: m' = 16 .. 128 (distances 2^9 .. 2^6); blk = wave id, k = blk*1024 + o + 64 j
    {
        const int blk = __builtin_amdgcn_readfirstlane(tid >> 6), o = tid & 63;
        const int base = blk * 1024 + o;
#pragma unroll
        for (int j = 0; j < 16; j++) if (!(MODE & 4)) x[j] = lds[qp(base + 64 * j)];
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const int ml = 16 << st, h = 8 >> st, nj = 1 << st;
            if (big && (st & 1) == 0) {
#pragma unroll
                for (int j = 0; j < 16; j++) x[j] = fred(x[j], q, qi);
            }
#pragma unroll
            for (int jj = 0; jj < nj; jj++) {
                const double wq = Wq[ml * q4 + blk * nj + jj];  // wave-uniform
#pragma unroll
                for (int k = 0; k < h; k++) ctq(x[jj * 2 * h + k], x[jj * 2 * h + k + h], wq, q);
            }
        }
#pragma unroll
        for (int j = 0; j < 16; j++) if (!(MODE & 4)) lds[qp(base + 64 * j)] = x[j];
    }
    __syncthreads();
    // ---- group 2: m' = 256 .. 2048 (distances 2^5 .. 2^2); blk = tid >> 2, k = 64 blk + o + 4 j
    {
        const int blk = tid >> 2, o = tid & 3;
        const int base = blk * 64 + o;
#pragma unroll
        for (int j = 0; j < 16; j++) if (!(MODE & 4)) x[j] = lds[qp(base + 4 * j)];
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const int ml = 256 << st, h = 8 >> st, nj = 1 << st;
            if (big && (st & 1) == 0) {
#pragma unroll
                for (int j = 0; j < 16; j++) x[j] = fred(x[j], q, qi);
            }
#pragma unroll
            for (int jj = 0; jj < nj; jj++) {
                const double wq = Wq[ml * q4 + blk * nj + jj];
#pragma unroll
                for (int k = 0; k < h; k++) ctq(x[jj * 2 * h + k], x[jj * 2 * h + k + h], wq, q);
            }
        }
#pragma unroll
        for (int j = 0; j < 16; j++) if (!(MODE & 4)) lds[qp(base + 4 * j)] = x[j];
    }
    __syncthreads();
    // ---- group 3: m' = 4096, 8192 (distances 2, 1); blocks of 4: blk_u = tid + 1024 u
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int blk = tid + 1024 * u, k0 = 4 * blk;
        double* xv = x + 4 * u;
#pragma unroll
        for (int e = 0; e < 4; e++) if (!(MODE & 4)) xv[e] = lds[qp(k0 + e)];
        if (big) {
#pragma unroll
            for (int e = 0; e < 4; e++) xv[e] = fred(xv[e], q, qi);
        }
        const double wa = Wq[4096 * q4 + blk];
        ctq(xv[0], xv[2], wa, q);
        ctq(xv[1], xv[3], wa, q);
        ctq(xv[0], xv[1], Wq[8192 * q4 + 2 * blk], q);
        ctq(xv[2], xv[3], Wq[8192 * q4 + 2 * blk + 1], q);
    }
    // ---- canonical residues out: quarter qs, 4 contiguous words per (thread, u)
    const long qoff = (long)qs * 16384;
    if (!FIN) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k0 = 4 * (tid + 1024 * u);
#pragma unroll
            for (int e = 0; e < 4; e++) out[qoff + k0 + e] = fcanon(x[4 * u + e], q, qi);
        }
    } else {
        const int y = limb, p = y / fin.nl, i = y - p * fin.nl, bb = p >> 1, c = p & 1;
        const long off = ((long)i << 16) + qoff;
        const u64* ap = fin.acc + (long)bb * fin.abs_ + (long)c * fin.acs + off;
        const u64* dp = fin.addend.ptr && c < fin.addend.np ? fin.addend.ptr + (long)bb * fin.addend.bs + (long)c * fin.addend.ps + off : nullptr;
        u64* op = fin.out + (long)bb * fin.obs + (long)c * fin.ops + off;
        const double f = fin.dinvf[i], w = tw_w(f, q);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k0 = 4 * (tid + 1024 * u);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const double conv = (double)fcanon(x[4 * u + e], q, qi);
                double v = fmul_rem(u2d(ap[k0 + e]) - conv, w, f, q);
                if (dp) v += u2d(dp[k0 + e]);
                op[k0 + e] = fcanon(v, q, qi);
            }
        }
    }
}


// ---- v2: 512 threads x 32 registers hold the 2^14-point quarter; LDS (70 KB) is only the
// transit buffer of the two layout exchanges, each done in two rounds of half the quarter, so
// two workgroups share a CU (one streams HBM while the other computes).
//   G0: distances 2^13..2^9  (m' = 1..16)      k = t + 512 j                     (regs: k bits 9..13)
//   G1: distances 2^8..2^4   (m' = 32..512)    k = (t & 15) + 16 j + 512 (t >> 4)  (regs: bits 4..8)
//   G2: distances 2^3..2^0   (m' = 1024..8192) k = (j & 15) + 8192 (j >> 4) + g2(t) (regs: 0..3, 13)
//       g2(t) = 16 (t & 127) + 4096 t7 + 2048 t8
// A round moves the elements with one k bit = rr; that bit is the SAME thread bit in both
// layouts of the exchange (k bit 3 = t bit 3 for G0 -> G1, k bit 12 = t bit 7 for G1 -> G2),
// so a thread writes all its registers and then reads all its registers in the same round and
// nothing is overwritten before it has been written out.  LDS index = the 13 remaining k bits
// (k'), padded: A(k') = k' + 8 (k' >> 8), B(k') = k' + (k' >> 4) + 16 (k' >> 9).
constexpr int kQ2Lds = 8191 + (8191 >> 4) + 16 * (8191 >> 9) + 1;
__device__ __forceinline__ int q2a(int k) {  // drop k bit 3
    const int kk = (k & 7) | ((k >> 4) << 3);
    return kk + 8 * (kk >> 8);
}
__device__ __forceinline__ int q2b(int k) {  // drop k bit 12
    const int kk = (k & 4095) | ((k >> 13) << 12);
    return kk + (kk >> 4) + 16 * (kk >> 9);
}
__device__ __forceinline__ int q2c(int k) {  // drop k bit 13 (output transpose)
    const int kk = k & 8191;
    return kk + (kk >> 4) + 16 * (kk >> 9);
}

template <bool FIN, int MODE = 0>
__global__ __launch_bounds__(512, 4) void k_nttf_fwd_q2(Span src, Span dst, Tabs T, RowFin fin, int total) {
    __shared__ double lds[kQ2Lds];
    const int b = blockIdx.x, g = b & 7, r = b >> 3, qs = r & 3;
    const int limb = (r >> 2) * 8 + g;
    if (limb >= total) return;
    int pid;
    const u64* in = span_ptr(src, limb, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, limb, T.logN, T.Lp1, pid);
    const int t = threadIdx.x;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* W = T.psif + ((long)pid << 16);
    const int q4 = 4 + qs;  // twiddle of (m', i') is psi^{brv(m' (4 + qs) + i')}
    double x[32];
    // ---- head (stages m = 1, 2 of the full transform, restricted to quarter qs)
    {
        const double w1q = (qs >= 2 ? -1.0 : 1.0) * W[1], w1 = tw_w(w1q, q);  // -w for s = 2, 3
        const double wsq = ((qs & 1) ? -1.0 : 1.0) * W[2 + (qs >> 1)], ws = tw_w(wsq, q);
#pragma unroll
        for (int j = 0; j < 32; j++) {
            const int k = t + 512 * j;
            double a0, a1, a2, a3;
            if (MODE & 1) {
                a0 = u2d(in[k + qs * 16384]);
                a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
            } else {
                a0 = u2d(in[k]), a1 = u2d(in[k + 16384]);
                a2 = u2d(in[k + 32768]), a3 = u2d(in[k + 49152]);
            }
            const double u = a0 + fmul_rem(a2, w1, w1q, q);
            const double v = a1 + fmul_rem(a3, w1, w1q, q);
            x[j] = u + fmul_rem(v, ws, wsq, q);
        }
    }
    auto ctq = [&](double& xa, double& xb, double wq) {
        if (!(MODE & 2)) ct_f(xa, xb, wq, q);
        else xa += wq;
    };
    auto fold = [&](int lo, int n) {
        if (big) {
#pragma unroll
            for (int j = 0; j < n; j++) x[lo + j] = fred(x[lo + j], q, qi);
        }
    };
    // ---- G0: global stages 0..4, folds (big primes) before 0, 2, 4
#pragma unroll
    for (int st = 0; st < 5; st++) {
        const int ml = 1 << st, h = 16 >> st;
        if ((st & 1) == 0) fold(0, 32);
#pragma unroll
        for (int jj = 0; jj < ml; jj++) {
            const double wq = W[ml * q4 + jj];  // uniform: scalar load
#pragma unroll
            for (int k = 0; k < h; k++) ctq(x[jj * 2 * h + k], x[jj * 2 * h + k + h], wq);
        }
    }
    // ---- exchange G0 -> G1: round rr = k bit 3 = t bit 3 (both layouts)
    const int g1base = (t & 15) + 512 * (t >> 4);
#pragma unroll
    for (int rr = 0; rr < 2; rr++) {
        if (((t >> 3) & 1) == rr && !(MODE & 4)) {
#pragma unroll
            for (int j = 0; j < 32; j++) lds[q2a(t + 512 * j)] = x[j];
        }
        __syncthreads();
        if (((t >> 3) & 1) == rr && !(MODE & 4)) {
#pragma unroll
            for (int j = 0; j < 32; j++) x[j] = lds[q2a(g1base + 16 * j)];
        }
        __syncthreads();
    }
    // ---- G1: global stages 5..9 (m' = 32 << st), folds before global 6, 8
    {
        const double* Wg = W + 32 * q4;
        const int tb = t >> 4;  // i' = tb * 2^st + (j >> (5 - st))
#pragma unroll
        for (int st = 0; st < 5; st++) {
            const int ml = 32 << st, h = 16 >> st, nj = 1 << st;
            if (st & 1) fold(0, 32);
#pragma unroll
            for (int jj = 0; jj < nj; jj++) {
                const double wq = Wg[(ml - 32) * q4 + tb * nj + jj];
#pragma unroll
                for (int k = 0; k < h; k++) ctq(x[jj * 2 * h + k], x[jj * 2 * h + k + h], wq);
            }
        }
    }
    // ---- exchange G1 -> G2: round rr = k bit 12 = t bit 7 (both layouts)
    const int g2 = 16 * (t & 127) + 4096 * ((t >> 7) & 1) + 2048 * ((t >> 8) & 1);
#pragma unroll
    for (int rr = 0; rr < 2; rr++) {
        if (((t >> 7) & 1) == rr && !(MODE & 4)) {
#pragma unroll
            for (int j = 0; j < 32; j++) lds[q2b(g1base + 16 * j)] = x[j];
        }
        __syncthreads();
        if (((t >> 7) & 1) == rr && !(MODE & 4)) {
#pragma unroll
            for (int j = 0; j < 32; j++) x[j] = lds[q2b(g2 + (j & 15) + 8192 * (j >> 4))];
        }
        if (rr == 0) __syncthreads();
    }
    // ---- G2: global stages 10..13 (m' = 1024 << st) on each 16-register half, folds before 10, 12
#pragma unroll
    for (int hf = 0; hf < 2; hf++) {
        double* xh = x + 16 * hf;
        const int kb = g2 + 8192 * hf;  // k of xh[0] (a multiple of 16); i' = k >> (4 - st)
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const int ml = 1024 << st, h = 8 >> st, nj = 1 << st;
            if ((st & 1) == 0) fold(16 * hf, 16);
#pragma unroll
            for (int jj = 0; jj < nj; jj++) {
                const double wq = W[ml * q4 + (kb >> (4 - st)) + jj];
#pragma unroll
                for (int k = 0; k < h; k++) ctq(xh[jj * 2 * h + k], xh[jj * 2 * h + k + h], wq);
            }
        }
    }
    // ---- canonical residues, transposed through LDS (two rounds on k bit 13, a register bit
    // in both layouts) so that each store instruction writes 1 KB contiguous: thread t stores
    // k = 2t + e + 1024 j (e = 0, 1 as one 16-B store), j = 0..15.
#pragma unroll
    for (int j = 0; j < 32; j++) x[j] = (double)fcanon(x[j], q, qi);  // exact: < 2^50
    const long qoff = (long)qs * 16384;
    const u64* ap = nullptr;
    const u64* dp = nullptr;
    u64* op = out + qoff;
    double fw = 0.0, fq = 0.0;
    if (FIN) {
        const int y = limb, p = y / fin.nl, i = y - p * fin.nl, bb = p >> 1, c = p & 1;
        const long off = ((long)i << 16) + qoff;
        ap = fin.acc + (long)bb * fin.abs_ + (long)c * fin.acs + off;
        dp = fin.addend.ptr && c < fin.addend.np ? fin.addend.ptr + (long)bb * fin.addend.bs + (long)c * fin.addend.ps + off : nullptr;
        op = fin.out + (long)bb * fin.obs + (long)c * fin.ops + off;
        fq = fin.dinvf[i];
        fw = tw_w(fq, q);
    }
#pragma unroll
    for (int rr = 0; rr < 2; rr++) {
        __syncthreads();  // rr = 0: the G2 reads of the last exchange are done
        if (!(MODE & 4)) {
#pragma unroll
            for (int e = 0; e < 16; e++) lds[q2c(g2 + e)] = x[16 * rr + e];
        }
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < 8; jj++) {
            const int k = 2 * t + 1024 * jj;  // + 8192 rr
            double v0 = x[16 * rr + 2 * jj], v1 = x[16 * rr + 2 * jj + 1];
            if (!(MODE & 4)) {
                v0 = lds[q2c(k)];
                v1 = lds[q2c(k + 1)];
            }
            const int kg = k + 8192 * rr;
            ulonglong2 o;
            if (!FIN) {
                o.x = (u64)__double_as_longlong(v0 + 4503599627370496.0) & 0xFFFFFFFFFFFFFULL;
                o.y = (u64)__double_as_longlong(v1 + 4503599627370496.0) & 0xFFFFFFFFFFFFFULL;
            } else {
                const ulonglong2 av = *(const ulonglong2*)(ap + kg);
                double r0 = fmul_rem(u2d(av.x) - v0, fw, fq, q), r1 = fmul_rem(u2d(av.y) - v1, fw, fq, q);
                if (dp) {
                    const ulonglong2 dv = *(const ulonglong2*)(dp + kg);
                    r0 += u2d(dv.x);
                    r1 += u2d(dv.y);
                }
                o.x = fcanon(r0, q, qi);
                o.y = fcanon(r1, q, qi);
            }
            *(ulonglong2*)(op + kg) = o;
        }
    }
}

}  // namespace aesfhe

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_) {                                                             \
            printf("%s @%d\n", hipGetErrorString(e_), __LINE__);              \
            return 1;                                                         \
        }                                                                     \
    } while (0)

template <class T>
static T* up(const std::vector<T>& v) {
    T* d = nullptr;
    if (hipMalloc(&d, v.size() * sizeof(T)) != hipSuccess) abort();
    if (hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) abort();
    return d;
}

__global__ void k_copy(const u64* __restrict__ a, u64* __restrict__ b, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}
__global__ void k_copy16(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ b, long n) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}
__global__ void k_copy16x4(const ulonglong2* __restrict__ a, ulonglong2* __restrict__ b, long n) {
    long i = ((long)blockIdx.x * blockDim.x) * 4 + threadIdx.x;
    ulonglong2 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) v[u] = a[i + u * blockDim.x];
#pragma unroll
    for (int u = 0; u < 4; u++) b[i + u * blockDim.x] = v[u];
}

// Infinity-Cache experiment: one workgroup moves a whole limb src -> mid -> dst with a barrier in
// between (the data movement of a one-workgroup-per-limb NTT whose transpose goes through
// memory).  MODE 0: mid = a per-workgroup slot (reused, stays on-die if anything does); 1: mid =
// a separate buffer per limb; 2: mid = dst itself (in place).
template <int MODE>
__global__ __launch_bounds__(1024) void k_copy_mid(const ulonglong2* __restrict__ a, ulonglong2* mid,
                                                   ulonglong2* b, int limbs, int half) {
    for (int y = blockIdx.x; y < limbs; y += gridDim.x) {
        const ulonglong2* s = a + (long)y * half;
        ulonglong2* d = b + (long)y * half;
        ulonglong2* m = MODE == 0 ? mid + (long)blockIdx.x * half : MODE == 1 ? mid + (long)y * half : d;
        for (int e = threadIdx.x; e < half; e += 4096) {
            ulonglong2 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = s[e + u * 1024];
#pragma unroll
            for (int u = 0; u < 4; u++) m[e + u * 1024] = v[u];
        }
        __syncthreads();
        for (int e = threadIdx.x; e < half; e += 4096) {
            ulonglong2 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = m[(e + u * 1024) ^ 2048];  // another lane's words
#pragma unroll
            for (int u = 0; u < 4; u++) d[e + u * 1024] = v[u];
        }
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    const int logN = 16, N = 1 << logN, L = 30, K = 8;
    const int limbs = argc > 1 ? atoi(argv[1]) : 468;  // 12 x 39
    Chain ch = make_chain(logN, L, K, 50, 50, 40);
    const int np = (int)ch.q.size();
    std::vector<u64> hq(ch.q);
    std::vector<double> hqi(np), hpsif((size_t)np * N), hr((size_t)np * 2048), hz(np, 0.0);
    for (int p = 0; p < np; p++) {
        u64 q = hq[p];
        hqi[p] = 1.0 / (double)q;
        u64 psi = min_primitive_root(q, N);
        std::vector<u64> pw(N);
        pw[0] = 1;
        for (int k = 1; k < N; k++) pw[k] = h_mulmod(pw[k - 1], psi, q);
        for (int k = 0; k < N; k++) hpsif[(size_t)p * N + k] = (double)pw[bit_reverse(k, logN)] / (double)q;
        for (int row = 0; row < 256; row++)
            for (int sh = 0; sh < 8; sh++) hr[(size_t)p * 2048 + row * 8 + sh] = hpsif[(size_t)p * N + (row << sh)];
    }
    Tabs T{};
    T.q = up(hq);
    T.qinv = up(hqi);
    T.psif = up(hpsif);
    T.rtwf = up(hr);
    T.logN = logN;
    T.cw = tools_make_cw(T.psif, T.q, np, logN);
    T.Lp1 = np;
    // limb y uses prime y % np: one "poly" per np limbs
    std::vector<u64> h((size_t)limbs * N);
    std::mt19937_64 rng(7);
    for (int y = 0; y < limbs; y++)
        for (int k = 0; k < N; k++) {
            u64 q = hq[y % np];
            h[(size_t)y * N + k] = (y % 3 == 0 && k < N / 2) ? q - 1 : rng() % q;
        }
    u64 *src = up(h), *d1, *d2, *acc, *o1, *o2;
    const size_t bytes = (size_t)limbs * N * 8;
    CK(hipMalloc(&d1, bytes));
    CK(hipMalloc(&d2, bytes));
    CK(hipMalloc(&acc, bytes));
    CK(hipMalloc(&o1, bytes));
    CK(hipMalloc(&o2, bytes));
    CK(hipMemcpy(acc, src, bytes, hipMemcpyDeviceToDevice));
    const int polys = limbs / np;
    Span ss{src, (long)np * N, np, np, 0, 0}, s1{d1, (long)np * N, np, np, 0, 0}, s2{d2, (long)np * N, np, np, 0, 0};
    const int qgrid = (limbs + 7) / 8 * 32;
    auto two_pass = [&] {
        hipLaunchKernelGGL(k_nttf_fwd_cols, dim3(16, limbs), dim3(256), 0, 0, ss, s1, T);
        hipLaunchKernelGGL(k_nttf_fwd_rows_t<false>, dim3(16, limbs), dim3(256), 0, 0, s1, T, RowFin{});
    };
    auto one_pass = [&] { hipLaunchKernelGGL(k_nttf_fwd_q2<false>, dim3(qgrid), dim3(512), 0, 0, ss, s2, T, RowFin{}, limbs); };
    auto one_pass_v1 = [&] { hipLaunchKernelGGL(k_nttf_fwd_q<false>, dim3(qgrid), dim3(1024), 0, 0, ss, s2, T, RowFin{}, limbs); };
    two_pass();
    one_pass();
    CK(hipDeviceSynchronize());
    std::vector<u64> r1((size_t)limbs * N), r2((size_t)limbs * N);
    CK(hipMemcpy(r1.data(), d1, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r2.data(), d2, bytes, hipMemcpyDeviceToHost));
    long bad = 0;
    for (size_t i = 0; i < r1.size(); i++) bad += r1[i] != r2[i];
    printf("limbs %d (%d polys x %d primes): one-pass vs two-pass mismatches %ld\n", limbs, polys, np, bad);
    // FIN epilogue: out = (acc - ntt(src)) * D^{-1}, layout (b, c, i) with nl = np, 2 comps
    {
        std::vector<double> hd(np);
        for (int p = 0; p < np; p++) hd[p] = (double)(hq[p] / 3) / (double)hq[p];
        RowFin f{};
        f.acc = acc;
        f.abs_ = 2L * np * N;
        f.acs = (long)np * N;
        f.addend = Opnd2{nullptr, 0, 0, 0};
        f.dinvf = up(hd);
        f.nl = np;
        f.obs = 2L * np * N;
        f.ops = (long)np * N;
        const int lf = polys / 2 * 2 * np;
        if (lf > 0) {
            CK(hipMemcpy(d1, src, bytes, hipMemcpyDeviceToDevice));
            hipLaunchKernelGGL(k_nttf_fwd_cols, dim3(16, lf), dim3(256), 0, 0, ss, s1, T);
            f.out = o1;
            hipLaunchKernelGGL(k_nttf_fwd_rows_t<true>, dim3(16, lf), dim3(256), 0, 0, s1, T, f);
            f.out = o2;
            hipLaunchKernelGGL(k_nttf_fwd_q2<true>, dim3((lf + 7) / 8 * 32), dim3(512), 0, 0, ss, s2, T, f, lf);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(r1.data(), o1, (size_t)lf * N * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(r2.data(), o2, (size_t)lf * N * 8, hipMemcpyDeviceToHost));
            long bf = 0;
            for (size_t i = 0; i < (size_t)lf * N; i++) bf += r1[i] != r2[i];
            printf("FIN epilogue (%d limbs): mismatches %ld\n", lf, bf);
            bad += bf;
        }
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto timeit = [&](const char* name, auto fn) {
        for (int w = 0; w < 3; w++) fn();
        hipEventRecord(a);
        const int it = 20;
        for (int i = 0; i < it; i++) fn();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1000 / it;
        printf("%-34s %8.1f us  alg %7.1f GB/s (16 B/coef)  frac %.3f\n", name, us, 16.0 * limbs * N / (us * 1e3),
               16.0 * limbs * N / (us * 1e3) / 8000.0);
    };
    timeit("copy (r+w = 16 B/coef)", [&] { hipLaunchKernelGGL(k_copy, dim3((long)limbs * N / 256), dim3(256), 0, 0, src, d2, (long)limbs * N); });
    timeit("copy 16 B / lane", [&] { hipLaunchKernelGGL(k_copy16, dim3((long)limbs * N / 512), dim3(256), 0, 0, (const ulonglong2*)src, (ulonglong2*)d2, (long)limbs * N / 2); });
    timeit("copy 16 B x4 / lane", [&] { hipLaunchKernelGGL(k_copy16x4, dim3((long)limbs * N / 2048), dim3(256), 0, 0, (const ulonglong2*)src, (ulonglong2*)d2, (long)limbs * N / 2); });
    {
        ulonglong2* mid;
        CK(hipMalloc(&mid, bytes));
        const int half = N / 2;
        for (int g : {256, 512}) {
            char nm[64];
            snprintf(nm, sizeof nm, "copy via WG slot, grid %d", g);
            timeit(nm, [&] { hipLaunchKernelGGL(k_copy_mid<0>, dim3(g), dim3(1024), 0, 0, (const ulonglong2*)src, mid, (ulonglong2*)d2, limbs, half); });
            snprintf(nm, sizeof nm, "copy via per-limb mid, grid %d", g);
            timeit(nm, [&] { hipLaunchKernelGGL(k_copy_mid<1>, dim3(g), dim3(1024), 0, 0, (const ulonglong2*)src, mid, (ulonglong2*)d2, limbs, half); });
            snprintf(nm, sizeof nm, "copy via dst in place, grid %d", g);
            timeit(nm, [&] { hipLaunchKernelGGL(k_copy_mid<2>, dim3(g), dim3(1024), 0, 0, (const ulonglong2*)src, mid, (ulonglong2*)d2, limbs, half); });
        }
        CK(hipFree(mid));
    }
    timeit("two-pass forward (cols + rows)", two_pass);
    timeit("one-pass forward (k_nttf_fwd_q2)", one_pass);
    timeit("one-pass v1 (k_nttf_fwd_q)", one_pass_v1);
    timeit("  cols pass alone", [&] { hipLaunchKernelGGL(k_nttf_fwd_cols, dim3(16, limbs), dim3(256), 0, 0, ss, s1, T); });
    timeit("  rows pass alone", [&] { hipLaunchKernelGGL(k_nttf_fwd_rows_t<false>, dim3(16, limbs), dim3(256), 0, 0, s1, T, RowFin{}); });
#define QMODE(M, name) timeit(name, [&] { hipLaunchKernelGGL((k_nttf_fwd_q2<false, M>), dim3(qgrid), dim3(512), 0, 0, ss, s2, T, RowFin{}, limbs); })
    QMODE(1, "  q: own quarter only (1)");
    QMODE(2, "  q: no butterflies (2)");
    QMODE(4, "  q: no LDS (4)");
    QMODE(3, "  q: own quarter, no bfly (3)");
    QMODE(6, "  q: no bfly, no LDS (6)");
    QMODE(7, "  q: memory only (7)");
    return bad ? 2 : 0;
}
