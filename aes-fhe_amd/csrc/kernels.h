// kernels.h -- device code of the MI355X CKKS engine (gfx950, wave64).
//
// Arithmetic: residues are u64 canonical in [0, q) with every prime q < 2^51.  A modular
// product uses an fp64 quotient estimate (a*b*(1/q), |error| < 1) and two wrapping 64-bit
// multiplies; the exact remainder then lies in [-q, 2q) and one signed correction makes it
// canonical.  Fixed multiplicands (twiddles, base-conversion constants) carry w/q in fp64 so
// the estimate is a single multiply.  This path is integer/HBM work: no MFMA.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#define AESFHE_HD __host__ __device__
#include "ckks_host.h"

namespace aesfhe {

constexpr int kMaxPrimes = 96;
constexpr double kBigPrime = 4398046511104.0;  // 2^42: primes at or above it fold lazily more often

__device__ __forceinline__ u64 add_m(u64 a, u64 b, u64 q) {
    u64 s = a + b;
    return s >= q ? s - q : s;
}
__device__ __forceinline__ u64 sub_m(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }

__device__ __forceinline__ u64 fix_m(u64 r, u64 q) {  // r = true value in [-q, 2q) mod 2^64
    int64_t s = (int64_t)r;
    s = s < 0 ? s + (int64_t)q : s;
    s = s >= (int64_t)q ? s - (int64_t)q : s;
    return (u64)s;
}

// fp64 view of an integer a < 2^52 (exact): the 2^52 magic-number trick, two instructions
__device__ __forceinline__ double u2d(u64 a) {
    return __longlong_as_double((long long)(a | 0x4330000000000000ULL)) - 4503599627370496.0;
}
// nearest integer of a non-negative x < 2^52 (one fma against 2^52, then the mantissa bits)
__device__ __forceinline__ u64 rint_u(double x_times, double scale) {
    return (u64)__double_as_longlong(__builtin_fma(x_times, scale, 4503599627370496.0)) & 0xFFFFFFFFFFFFFULL;
}

// a * b mod q, a,b < q < 2^51: quotient a*b/q rounded to nearest in fp64 (|error| <= 1), exact
// remainder from two wrapping 64-bit products, one two-sided correction.
__device__ __forceinline__ u64 mul_m(u64 a, u64 b, u64 q, double qinv) {
    const u64 qh = rint_u(u2d(a) * u2d(b), qinv);
    return fix_m(a * b - qh * q, q);
}
// a * w mod q for a < 2^52, w < q < 2^51, wq = w / q: remainder in (-q, q), one correction
__device__ __forceinline__ u64 mul_w(u64 a, u64 w, double wq, u64 q) {
    const u64 qh = rint_u(u2d(a), wq);
    int64_t r = (int64_t)(a * w - qh * q);
    r += (r >> 63) & (int64_t)q;
    return (u64)r;
}

// ---- all-fp64 modular arithmetic on exact integers carried in doubles (|x| < 2^52) ----------
// r = a*w - qh*q with qh = rint(a*w/q) (quotient from w/q rounded: |a*w/q - qh| <= 1):
// p + pl = a*w exactly (fma split); u = fma(-qh, q, p) is exact because p - qh*q is an integer
// of magnitude <= q + |pl| < 2^53 (one rounding of an exactly representable value); r = u + pl is
// exact for the same reason.  Six full-rate fp64 ops, |r| <= q for a constant w with wq = w/q,
// <= 1.5q with an on-the-fly quotient wq = w * (1/q); signed a allowed (|a| < 2^52).
// tools/mulmod_bench.hip; verified on 1.6e8 random/edge operands per prime size (CPU, same ops).
constexpr double kMagic52 = 6755399441055744.0;  // 1.5 * 2^52: rint(v) = (v + M) - M, |v| < 2^51
__device__ __forceinline__ double fmul_rem(double a, double w, double wq, double q) {
    const double p = a * w;
    const double pl = __builtin_fma(a, w, -p);
    const double qh = __builtin_rint(a * wq);
    const double u = __builtin_fma(-qh, q, p);
    return u + pl;
}
__device__ __forceinline__ double fmul_rem_r(double a, double w, double wq, double q) {
    return fmul_rem(a, w, wq, q);
}
// x - rint(x/q)*q for |x| < 2^53: result in [-q/2 - 1, q/2 + 1] (exact: qh*q < 2^53)
__device__ __forceinline__ double fred(double x, double q, double qinv) {
    const double qh = __builtin_rint(x * qinv);
    return __builtin_fma(-qh, q, x);
}
// canonical residue in [0, q) of |x| < 2^53, as u64: fred lands in [-q/2 - 1, q/2 + 1], so one
// conditional +q suffices; the exact integer r < 2^52 is converted by the 2^52 magic number
// (one add + the mantissa bits) instead of the multi-instruction f64 -> u64 conversion.
__device__ __forceinline__ u64 fcanon(double x, double q, double qinv) {
    double r = fred(x, q, qinv);
    r = r < 0.0 ? r + q : r;
    return (u64)__double_as_longlong(r + 4503599627370496.0) & 0xFFFFFFFFFFFFFULL;
}
// w from its table entry wq = w/q (w < q < 2^52): rint(wq * q) is exact, |wq*q - w| < 2^-4
__device__ __forceinline__ double tw_w(double wq, double q) {
    return __builtin_rint(wq * q);
}
// an optional operand (ptr == nullptr or component >= np reads as zero), for fused epilogues
struct Opnd2 {
    const u64* ptr;
    long bs, ps;
    int np;
};
struct alignas(16) TwD {
    double w;   // constant as an exact double (< 2^52)
    double wq;  // w / q
};

// A set of limbs: poly p (0..npoly-1), limb l (0..nl-1) at base + p*pstride + l*N.
// Prime of limb l: l < nq ? qpid0 + l : spid0 + (l - nq)  (Q limbs then special limbs).
struct Span {
    u64* base;
    long pstride;
    int nl;
    int nq;
    int qpid0;
    int spid0;
    int pmask = -1;  // polynomial index cycled through (an operand in aesfhe_mul's cyclic broadcast)
};

__device__ __forceinline__ u64* span_ptr(const Span& s, int y, int logN, int Lp1, int& pid) {
    (void)Lp1;
    int p = y / s.nl, l = y - p * s.nl;
    pid = l < s.nq ? s.qpid0 + l : s.spid0 + (l - s.nq);
    return s.base + (long)(p & s.pmask) * s.pstride + ((long)l << logN);
}

constexpr int kColW = 64;  // Tabs::cw / icw entries per prime (R = 512 reads up to index 47)

struct Tabs {
    const u64* q;
    const double* qinv;
    const u64* psi;      // [np][N] psi^{brv(k)}
    const double* psif;  // psi/q
    const u64* ipsi;     // [np][N] psi^{-brv(k)}
    const double* ipsif;
    const double* rtwf;   // N = 2^16 only: [np][256][8] psi^{brv(row << s)} / q (ntt256f.h)
    const double* irtwf;  // the same for psi^{-1}
    const u64* ninv;
    const double* ninvf;
    const struct Tw* tw;   // [np][N] {psi^{brv(k)}, psi^{brv(k)}/q} interleaved (16 B)
    const struct Tw* itw;  // [np][N] inverse
    // [np][kColW] psi^{brv(k)} (cw) / psi^{-brv(k)} (icw) as exact doubles, k < kColW: the column
    // passes' wave-uniform stages read w by scalar load beside w/q instead of recomputing
    // w = rint(wq q) on the VALU (2 instructions per twiddle per wave; round 6)
    const double* cw;
    const double* icw;
    int logN;
    int Lp1;
};

struct alignas(16) Tw {
    u64 w;
    double wq;
};

// ---------------------------------------------------------------------------------------------
// NTT pass kernels.  N = R1 x 256; pass "cols" covers the first log2(R1)
// stages (column sub-NTTs of stride 256), pass "rows" the last 8 stages (contiguous rows).
constexpr int kTile = 4096;  // u64 elements staged in LDS per workgroup (32 KiB)
constexpr int kC2 = 256;

template <int R1>
__global__ __launch_bounds__(256) void k_ntt_fwd_cols(Span src, Span dst, Tabs T) {
    constexpr int CW = (kTile / R1) < kC2 ? (kTile / R1) : kC2;
    __shared__ u64 s[R1 * CW];
    int pid;
    const u64* in = span_ptr(src, blockIdx.y, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int c0 = blockIdx.x * CW;
    const u64 q = T.q[pid];
    const u64* W = T.psi + ((long)pid << T.logN);
    const double* Wf = T.psif + ((long)pid << T.logN);
    for (int e = threadIdx.x; e < R1 * CW; e += 256) {
        int r = e / CW, c = e - r * CW;
        s[e] = in[r * kC2 + c0 + c];
    }
    __syncthreads();
    for (int m = 1, t = R1 / 2; m < R1; m <<= 1, t >>= 1) {
        for (int bf = threadIdx.x; bf < (R1 / 2) * CW; bf += 256) {
            int c = bf % CW, g = bf / CW;
            int i = g / t, r1 = i * 2 * t + (g - i * t), r2 = r1 + t;
            u64 w = W[m + i];
            double wf = Wf[m + i];
            u64 U = s[r1 * CW + c];
            u64 V = mul_w(s[r2 * CW + c], w, wf, q);
            s[r1 * CW + c] = add_m(U, V, q);
            s[r2 * CW + c] = sub_m(U, V, q);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < R1 * CW; e += 256) {
        int r = e / CW, c = e - r * CW;
        out[r * kC2 + c0 + c] = s[e];
    }
}

template <int R1>
__global__ __launch_bounds__(256) void k_ntt_fwd_rows(Span dst, Tabs T) {
    constexpr int RW = (kTile / kC2) < R1 ? (kTile / kC2) : R1;
    __shared__ u64 s[RW * kC2];
    int pid;
    u64* io = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int row0 = blockIdx.x * RW;
    const u64 q = T.q[pid];
    const u64* W = T.psi + ((long)pid << T.logN);
    const double* Wf = T.psif + ((long)pid << T.logN);
    u64* base = io + (long)row0 * kC2;
    for (int e = threadIdx.x; e < RW * kC2; e += 256) s[e] = base[e];
    __syncthreads();
    for (int ml = 1, t = kC2 / 2; ml < kC2; ml <<= 1, t >>= 1) {
        for (int bf = threadIdx.x; bf < RW * (kC2 / 2); bf += 256) {
            int rl = bf / (kC2 / 2), g = bf - rl * (kC2 / 2);
            int i = g / t, c1 = i * 2 * t + (g - i * t), c2 = c1 + t;
            int widx = R1 * ml + (row0 + rl) * ml + i;
            u64 w = W[widx];
            double wf = Wf[widx];
            u64* rowp = s + rl * kC2;
            u64 U = rowp[c1];
            u64 V = mul_w(rowp[c2], w, wf, q);
            rowp[c1] = add_m(U, V, q);
            rowp[c2] = sub_m(U, V, q);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < RW * kC2; e += 256) base[e] = s[e];
}

template <int R1>
__global__ __launch_bounds__(256) void k_ntt_inv_rows(Span src, Span dst, Tabs T) {
    constexpr int RW = (kTile / kC2) < R1 ? (kTile / kC2) : R1;
    __shared__ u64 s[RW * kC2];
    int pid;
    const u64* in = span_ptr(src, blockIdx.y, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int row0 = blockIdx.x * RW;
    const u64 q = T.q[pid];
    const u64* W = T.ipsi + ((long)pid << T.logN);
    const double* Wf = T.ipsif + ((long)pid << T.logN);
    const int N = 1 << T.logN;
    for (int e = threadIdx.x; e < RW * kC2; e += 256) s[e] = in[(long)row0 * kC2 + e];
    __syncthreads();
    for (int t = 1; t < kC2; t <<= 1) {
        int hg = N / (2 * t);
        for (int bf = threadIdx.x; bf < RW * (kC2 / 2); bf += 256) {
            int rl = bf / (kC2 / 2), g = bf - rl * (kC2 / 2);
            int i = g / t, c1 = i * 2 * t + (g - i * t), c2 = c1 + t;
            int widx = hg + (row0 + rl) * (kC2 / (2 * t)) + i;
            u64* rowp = s + rl * kC2;
            u64 U = rowp[c1], V = rowp[c2];
            rowp[c1] = add_m(U, V, q);
            rowp[c2] = mul_w(sub_m(U, V, q), W[widx], Wf[widx], q);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < RW * kC2; e += 256) out[(long)row0 * kC2 + e] = s[e];
}

template <int R1>
__global__ __launch_bounds__(256) void k_ntt_inv_cols(Span dst, Tabs T) {
    constexpr int CW = (kTile / R1) < kC2 ? (kTile / R1) : kC2;
    __shared__ u64 s[R1 * CW];
    int pid;
    u64* io = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int c0 = blockIdx.x * CW;
    const u64 q = T.q[pid];
    const u64* W = T.ipsi + ((long)pid << T.logN);
    const double* Wf = T.ipsif + ((long)pid << T.logN);
    for (int e = threadIdx.x; e < R1 * CW; e += 256) {
        int r = e / CW, c = e - r * CW;
        s[e] = io[r * kC2 + c0 + c];
    }
    __syncthreads();
    for (int tr = 1; tr < R1; tr <<= 1) {
        int hg = R1 / (2 * tr);
        for (int bf = threadIdx.x; bf < (R1 / 2) * CW; bf += 256) {
            int c = bf % CW, g = bf / CW;
            int i = g / tr, r1 = i * 2 * tr + (g - i * tr), r2 = r1 + tr;
            u64 U = s[r1 * CW + c], V = s[r2 * CW + c];
            s[r1 * CW + c] = add_m(U, V, q);
            s[r2 * CW + c] = mul_w(sub_m(U, V, q), W[hg + i], Wf[hg + i], q);
        }
        __syncthreads();
    }
    const u64 ni = T.ninv[pid];
    const double nif = T.ninvf[pid];
    for (int e = threadIdx.x; e < R1 * CW; e += 256) {
        int r = e / CW, c = e - r * CW;
        io[r * kC2 + c0 + c] = mul_w(s[e], ni, nif, q);
    }
}

}  // namespace aesfhe
