// kernels_ops.h -- elementwise, base-conversion, key-switching, sampling and automorphism
// kernels of the MI355X CKKS engine.  Specification: DESIGN.md section 3 (shared with the CPU
// oracle, oracle/ckks_oracle.c, which these kernels must match residue for residue).
#pragma once
#include "kernels.h"

namespace aesfhe {

// fp64-quotient reduction of x < 2^52
// reduction of x < 2^63 (lazy sums): fp64 quotient estimate, two-sided correction
__device__ __forceinline__ u64 red_m(u64 x, u64 q, double qinv) {
    u64 qh = (u64)((double)x * qinv);
    return fix_m(x - qh * q, q);
}

// An operand for elementwise kernels: element (b, p, l, k) at ptr + (b & bmask)*bs + p*ps + l*N + k.
// ptr == nullptr or p >= np reads as zero.  bmask: batch elements cycled through (B_op - 1 for a
// power-of-two B_op below the output's batch, the cyclic broadcast of aesfhe_mul; -1 otherwise;
// a B = 1 broadcast keeps bs = 0).
struct Opnd {
    const u64* ptr;
    long bs;
    long ps;
    int np;
    int bmask = -1;
};

// Absent operands read this zero word: the address is selected, not the load, so a kernel's
// operand loads carry no branch and issue together (a branch per opnd_get put every load
// behind its own wait).
__device__ const u64 kZeroWord = 0;
__device__ __forceinline__ u64 opnd_get(const Opnd& o, int b, int p, int l, int k, int logN) {
    const bool has = o.ptr && p < o.np;
    return *(has ? o.ptr + (long)(b & o.bmask) * o.bs + (long)p * o.ps + ((long)l << logN) + k : &kZeroWord);
}

struct Out {
    u64* ptr;
    long bs;
    long ps;
};

// out = a +- b ; grid (N/256, nl, B*np)
__global__ void k_addsub(Opnd a, Opnd b, Out o, int np, const u64* __restrict__ qs, int sub,
                         int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    const u64 q = qs[l];
    u64 va = opnd_get(a, bb, p, l, k, logN), vb = opnd_get(b, bb, p, l, k, logN);
    o.ptr[(long)bb * o.bs + (long)p * o.ps + ((long)l << logN) + k] = sub ? sub_m(va, vb, q) : add_m(va, vb, q);
}

// Batch gather (aesfhe_ct_gather): element b of dst = element idx[b] of src, `per` words each
// (a multiple of 2 * 256).  grid (x, n): 16 B per lane per step, grid-stride over the element.
__global__ void k_gather_batch(const u64* __restrict__ src, u64* __restrict__ dst,
                               const int* __restrict__ idx, long per) {
    const int b = blockIdx.y;
    const ulonglong2* s = (const ulonglong2*)(src + (long)idx[b] * per);
    ulonglong2* o = (ulonglong2*)(dst + (long)b * per);
    const long nv = per >> 1;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long)gridDim.x * blockDim.x)
        o[i] = s[i];
}

// Constant factors for x * (A + B X^{N/2}): f[2*l] for k < N/2, f[2*l+1] for k >= N/2.
// out (+)= in * f ; grid (N/256, nl, B*np)
__global__ void k_mul_const(Opnd in, Out o, int np, const u64* __restrict__ f,
                            const double* __restrict__ ff, const u64* __restrict__ qs, int acc,
                            int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    const u64 q = qs[l];
    const int h = k >> (logN - 1);
    u64 v = mul_w(opnd_get(in, bb, p, l, k, logN), f[2 * l + h], ff[2 * l + h], q);
    u64* dst = o.ptr + (long)bb * o.bs + (long)p * o.ps + ((long)l << logN) + k;
    *dst = acc ? add_m(*dst, v, q) : v;
}

// out = in * pt (pt limbs [l][N]) ; grid (N/256, nl, B*np)
__global__ void k_mul_pt(Opnd in, const u64* __restrict__ pt, Out o, int np,
                         const u64* __restrict__ qs, const double* __restrict__ qinv, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    u64 v = mul_m(opnd_get(in, bb, p, l, k, logN), pt[((long)l << logN) + k], qs[l], qinv[l]);
    o.ptr[(long)bb * o.bs + (long)p * o.ps + ((long)l << logN) + k] = v;
}

// out = in (+ pt on poly 0) ; grid (N/256, nl, B*np)
__global__ void k_add_pt(Opnd in, const u64* __restrict__ pt, Out o, int np,
                         const u64* __restrict__ qs, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    u64 v = opnd_get(in, bb, p, l, k, logN);
    if (p == 0) v = add_m(v, pt[((long)l << logN) + k], qs[l]);
    o.ptr[(long)bb * o.bs + (long)p * o.ps + ((long)l << logN) + k] = v;
}

// out = in + (f[2l] for k < N/2, f[2l+1] otherwise) on poly 0 ; grid (N/256, nl, B*np)
__global__ void k_add_const(Opnd in, Out o, int np, const u64* __restrict__ f,
                            const u64* __restrict__ qs, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    u64 v = opnd_get(in, bb, p, l, k, logN);
    if (p == 0) v = add_m(v, f[2 * l + (k >> (logN - 1))], qs[l]);
    o.ptr[(long)bb * o.bs + (long)p * o.ps + ((long)l << logN) + k] = v;
}

// (d0,d1,d2) (+)= (a0 b0, a0 b1 + a1 b0, a1 b1) ; grid (N/256, nl, B)
__global__ void k_tensor(Opnd a, Opnd b, Out o, const u64* __restrict__ qs,
                         const double* __restrict__ qinv, int acc, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z;
    const u64 q = qs[l];
    const double qi = qinv[l];
    u64 a0 = opnd_get(a, bb, 0, l, k, logN), a1 = opnd_get(a, bb, 1, l, k, logN);
    u64 b0 = opnd_get(b, bb, 0, l, k, logN), b1 = opnd_get(b, bb, 1, l, k, logN);
    u64 d0 = mul_m(a0, b0, q, qi);
    u64 d1 = add_m(mul_m(a0, b1, q, qi), mul_m(a1, b0, q, qi), q);
    u64 d2 = mul_m(a1, b1, q, qi);
    u64* base = o.ptr + (long)bb * o.bs + ((long)l << logN) + k;
    if (acc) {
        base[0] = add_m(base[0], d0, q);
        base[o.ps] = add_m(base[o.ps], d1, q);
        base[2 * o.ps] = add_m(base[2 * o.ps], d2, q);
    } else {  // streaming stores: the 3-component product is read back only by the key switch
        __builtin_nontemporal_store(d0, &base[0]);
        __builtin_nontemporal_store(d1, &base[o.ps]);
        __builtin_nontemporal_store(d2, &base[2 * o.ps]);
    }
}

// Fused multiply-add tensor (aesfhe_mul_fma): (d0, d1, d2) = alpha (a (x) b) + C (c0, c1, 0)
// + (K, 0, 0), fac[l] = {alpha, C, K} mod q_l; absent operands read as zero.  grid (N/256, nl, B)
__global__ void k_tensor_fma(Opnd a, Opnd b, Opnd c, Out o, const u64* __restrict__ fac,
                             const u64* __restrict__ qs, const double* __restrict__ qinv, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z;
    const u64 q = qs[l];
    const double qi = qinv[l];
    const u64 am = fac[3 * l], cm = fac[3 * l + 1], km = fac[3 * l + 2];
    const u64 a0 = opnd_get(a, bb, 0, l, k, logN), a1 = opnd_get(a, bb, 1, l, k, logN);
    const u64 b0 = opnd_get(b, bb, 0, l, k, logN), b1 = opnd_get(b, bb, 1, l, k, logN);
    u64 d0 = mul_m(mul_m(a0, b0, q, qi), am, q, qi);
    u64 d1 = mul_m(add_m(mul_m(a0, b1, q, qi), mul_m(a1, b0, q, qi), q), am, q, qi);
    const u64 d2 = mul_m(mul_m(a1, b1, q, qi), am, q, qi);
    d0 = add_m(d0, mul_m(opnd_get(c, bb, 0, l, k, logN), cm, q, qi), q);
    d1 = add_m(d1, mul_m(opnd_get(c, bb, 1, l, k, logN), cm, q, qi), q);
    d0 = add_m(d0, km, q);
    u64* base = o.ptr + (long)bb * o.bs + ((long)l << logN) + k;
    base[0] = d0;
    base[o.ps] = d1;
    base[2 * o.ps] = d2;
}

// Fused linear combination: out[b][p][l] = sum_i in_i[b][p][l] * f_i(l, half) (one pass, lazy
// sum in u64: n <= 64 terms of < 2^51 each).  ptrs/bstr: [n]; f/ff: [n][nl][2].  Inputs with
// fewer polynomials than np contribute zero to the missing ones (npi[i]).
// grid (N/256, nl, B*np)
__global__ void k_lincomb(const u64* const* __restrict__ ptrs, const long* __restrict__ bstr,
                          const int* __restrict__ npi, int n, const long* __restrict__ pss,
                          const u64* __restrict__ f,
                          const double* __restrict__ ff, Out o, int np, int nl,
                          const u64* __restrict__ qs, const double* __restrict__ qinv, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    const u64 q = qs[l];
    const int h = k >> (logN - 1);
    const long off = ((long)l << logN) + k;
    u64 acc = 0;
    // chunks of 8 inputs: the 8 loads are issued before the first product consumes one
    for (int i0 = 0; i0 < n; i0 += 8) {
        u64 v[8];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const int i = i0 + c;
            v[c] = (i < n && p < npi[i]) ? ptrs[i][(long)bb * bstr[i] + (long)p * pss[i] + off] : 0;
        }
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const int i = i0 + c;
            if (i < n) {
                const int fi = (i * nl + l) * 2 + h;
                acc += mul_w(v[c], f[fi], ff[fi], q);
            }
        }
    }
    o.ptr[(long)bb * o.bs + (long)p * o.ps + ((long)l << logN) + k] = red_m(acc, q, qinv[l]);
}

// m linear combinations of the same n <= 16 aligned inputs in one pass.  F/FF: [m][n][nl][2]
// (row-uniform factors -> scalar loads).  out: [m][B][np][nl][N].  grid (N/256, nl, B*np)
constexpr int kManyMax = 16;
__global__ void k_lincomb_many(const u64* const* __restrict__ ptrs, const long* __restrict__ bstr,
                               const int* __restrict__ npi, int n, const long* __restrict__ pss,
                               const u64* __restrict__ F, const double* __restrict__ FF, int m,
                               u64* __restrict__ out, long orow, long obs, int np, int nl,
                               const u64* __restrict__ qs, const double* __restrict__ qinv,
                               int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    const u64 q = qs[l];
    const int h = k >> (logN - 1);
    const long off = ((long)l << logN) + k;
    u64 v[kManyMax];
#pragma unroll
    for (int j = 0; j < kManyMax; j++)
        v[j] = (j < n && p < npi[j]) ? ptrs[j][(long)bb * bstr[j] + (long)p * pss[j] + off] : 0;
    u64* o = out + (long)bb * obs + ((long)p * nl << logN) + off;
    for (int i = 0; i < m; i++) {
        u64 acc = 0;
#pragma unroll
        for (int j = 0; j < kManyMax; j++) {
            if (j < n) {
                const int fi = ((i * n + j) * nl + l) * 2 + h;
                acc += mul_w(v[j], F[fi], FF[fi], q);
            }
        }
        o[(long)i * orow] = red_m(acc, q, qinv[l]);
    }
}

// Fused dot product: (d0,d1,d2) = sum_i a_i (x) b_i (one pass).  a/b pointer + batch-stride
// arrays [n]; inputs compact 2-poly ciphertexts at the same level (poly stride ps).
// grid (N/256, nl, B)
__global__ void k_dot(const u64* const* __restrict__ ap, const long* __restrict__ abs_,
                      const u64* const* __restrict__ bp, const long* __restrict__ bbs, int n,
                      long ps, Out o, const u64* __restrict__ qs, const double* __restrict__ qinv,
                      int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z;
    const u64 q = qs[l];
    const double qi = qinv[l];
    const long off = ((long)l << logN) + k;
    u64 d0 = 0, d1 = 0, d2 = 0;
    for (int i = 0; i < n; i++) {
        const u64* a = ap[i] + (long)bb * abs_[i] + off;
        const u64* b = bp[i] + (long)bb * bbs[i] + off;
        const u64 a0 = a[0], a1 = a[ps], b0 = b[0], b1 = b[ps];
        d0 += mul_m(a0, b0, q, qi);
        d1 += mul_m(a0, b1, q, qi) + mul_m(a1, b0, q, qi);
        d2 += mul_m(a1, b1, q, qi);
        if ((i & 15) == 15) {  // keep the lazy sums below 2^52 for red_m
            d0 = red_m(d0, q, qi);
            d1 = red_m(d1, q, qi);
            d2 = red_m(d2, q, qi);
        }
    }
    u64* base = o.ptr + (long)bb * o.bs + off;
    base[0] = red_m(d0, q, qi);
    base[o.ps] = red_m(d1, q, qi);
    base[2 * o.ps] = red_m(d2, q, qi);
}

// aesfhe_dot_fma's tensor: the k_dot sum of n pairs (n may be 0) plus the addends on d0 / d1,
// d0 += sum_j c_j0 C_j + K, d1 += sum_j c_j1 C_j (C_j = cf[j * nl + l], K = km[l]; addend j read
// at limb l of its own layout: batch stride cbs[j], 0 = broadcast, poly stride cps[j]), one pass.
// grid (N/256, nl, B)
__global__ void k_dot_fma(const u64* const* __restrict__ ap, const long* __restrict__ abs_,
                          const u64* const* __restrict__ bp, const long* __restrict__ bbs, int n,
                          long ps, const u64* const* __restrict__ cp, const long* __restrict__ cbs,
                          const long* __restrict__ cps, int nc, const u64* __restrict__ cf,
                          const u64* __restrict__ km, int nl, Out o, const u64* __restrict__ qs,
                          const double* __restrict__ qinv, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z;
    const u64 q = qs[l];
    const double qi = qinv[l];
    const long off = ((long)l << logN) + k;
    u64 d0 = 0, d1 = 0, d2 = 0;
    for (int i = 0; i < n; i++) {
        const u64* a = ap[i] + (long)bb * abs_[i] + off;
        const u64* b = bp[i] + (long)bb * bbs[i] + off;
        const u64 a0 = a[0], a1 = a[ps], b0 = b[0], b1 = b[ps];
        d0 += mul_m(a0, b0, q, qi);
        d1 += mul_m(a0, b1, q, qi) + mul_m(a1, b0, q, qi);
        d2 += mul_m(a1, b1, q, qi);
        if ((i & 15) == 15) {  // keep the lazy sums below 2^52 for red_m
            d0 = red_m(d0, q, qi);
            d1 = red_m(d1, q, qi);
            d2 = red_m(d2, q, qi);
        }
    }
    d0 = red_m(d0, q, qi);
    d1 = red_m(d1, q, qi);
    for (int j = 0; j < nc; j++) {
        const u64* c = cp[j] + (long)bb * cbs[j] + off;
        const u64 f = cf[(long)j * nl + l];
        d0 = add_m(d0, mul_m(c[0], f, q, qi), q);
        d1 = add_m(d1, mul_m(c[cps[j]], f, q, qi), q);
    }
    u64* base = o.ptr + (long)bb * o.bs + off;
    base[0] = add_m(d0, km[l], q);
    base[o.ps] = d1;
    base[2 * o.ps] = red_m(d2, q, qi);
}

// ---------------------------------------------------------------------------------------------
// rescale
// t[P][i][k] = centered(x[P][k]) mod q_i for i < l ; grid (N/256, l, P)
// SC (level-down fused into the rescale, level_down_view): the top limb is first multiplied by
// the level-down constant sc = C mod q_l ({sc, scf = sc / q_l})
template <bool SC = false>
__global__ void k_rescale_spread(const u64* __restrict__ x, u64* __restrict__ t, u64 ql,
                                 const u64* __restrict__ qs, const double* __restrict__ qinv,
                                 const u64* __restrict__ qlmod, int l, int logN, u64 sc, double scf) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y, P = blockIdx.z;
    const u64 q = qs[i];
    u64 v = x[((long)P << logN) + k];
    if (SC) v = mul_w(v, sc, scf, ql);
    u64 r = red_m(v, q, qinv[i]);
    if (v > (ql >> 1)) r = sub_m(r, qlmod[i], q);
    t[(((long)P * l + i) << logN) + k] = r;
}

// out[P][i] = (c[P][i] - t[P][i]) * q_l^{-1} ; grid (N/256, l, P) with P = b*np + p
// SC: c is first multiplied by the level-down constant (f / ff: [2 i] = C mod q_i, w/q), the
// residues k_mul_const would have written
template <bool SC = false>
__global__ void k_rescale_finish(Opnd c, const u64* __restrict__ t, Out o, int np, int l,
                                 const u64* __restrict__ qs, const u64* __restrict__ inv,
                                 const double* __restrict__ invf, int logN, const u64* __restrict__ f,
                                 const double* __restrict__ ff) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y, P = blockIdx.z, bb = P / np, p = P - bb * np;
    const u64 q = qs[i];
    u64 cv = opnd_get(c, bb, p, i, k, logN);
    if (SC) cv = mul_w(cv, f[2 * i], ff[2 * i], q);
    u64 tv = t[(((long)P * l + i) << logN) + k];
    o.ptr[(long)bb * o.bs + (long)p * o.ps + ((long)i << logN) + k] = mul_w(sub_m(cv, tv, q), inv[i], invf[i], q);
}

// rescale finish writing to per-group output ciphertexts: P = (g*Bg + b)*np + p
__global__ void k_rescale_finish_g(const u64* __restrict__ c, long cps, const u64* __restrict__ t,
                                   u64* const* __restrict__ outs, long ops, int np, int Bg, int l,
                                   const u64* __restrict__ qs, const u64* __restrict__ inv,
                                   const double* __restrict__ invf, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y, P = blockIdx.z;
    const int g = P / (Bg * np), rem = P - g * Bg * np;
    const u64 q = qs[i];
    u64 cv = c[(long)P * cps + ((long)i << logN) + k];
    u64 tv = t[(((long)P * l + i) << logN) + k];
    outs[g][(long)rem * ops + ((long)i << logN) + k] = mul_w(sub_m(cv, tv, q), inv[i], invf[i], q);
}

// ModUp base conversion of digit [lo, lo+alpha) (INTT'ed limbs of dc) to the other limbs t of
// the extended basis (Q_l then P), exact fp64 arithmetic (kernels.h fmul_rem):
//   y_i = [x_i * qhat_i^{-1}]_{q_i} in [0, q_i) (canonical, so the multiple of Q that the fast
//   conversion adds is the oracle's), ext[t] = sum_i y_i * (qhat_i mod p_t) mod p_t.
// Constants: hatinv as w/q (w = rint(wq * q) is exact), hat as {w, w/q}, [target pid][i] with
// row stride hs.  grid (N/256,
// ceil(ne/16), B): each thread converts one coefficient into up to 16 target limbs.
// A = alpha (digit width) as a template parameter: the per-target constant loads are then
// unconditional and the compiler issues all A of them before the first use (with a runtime
// alpha every term was a branch, and each scalar load was waited for on its own).
template <int A, int C>  // C coefficients per thread (k + 256 c): every constant fetched serves C
__global__ void k_modup(const u64* __restrict__ dc, long dcs, u64* __restrict__ ext, long exs,
                        int lo, int l, int ne, const double* __restrict__ hatinvf,
                        const TwD* __restrict__ hat, int hs, const u64* __restrict__ qall,
                        const double* __restrict__ qinvall, int Lp1, int logN) {
    const int k = blockIdx.x * (256 * C) + threadIdx.x;
    const int bb = blockIdx.z;
    double y[C][A];
#pragma unroll
    for (int i = 0; i < A; i++) {
        const int pi = lo + i;
        const double qp = (double)qall[pi];
        const double f = hatinvf[i], w = tw_w(f, qp);
        const u64* src = dc + (long)bb * dcs + ((long)pi << logN) + k;
#pragma unroll
        for (int c = 0; c < C; c++) {
            const double r = fmul_rem(u2d(src[256 * c]), w, f, qp);
            y[c][i] = r < 0.0 ? r + qp : r;
        }
    }
    const int tg = (ne + gridDim.y - 1) / gridDim.y, t0 = blockIdx.y * tg;  // targets per thread
    for (int t = t0; t < t0 + tg && t < ne; t++) {
        if (t >= lo && t < lo + A) continue;
        const int pid = t <= l ? t : Lp1 + (t - l - 1);
        const double qt = (double)qall[pid], qti = qinvall[pid];
        TwD f[A];
#pragma unroll
        for (int i = 0; i < A; i++) f[i] = hat[pid * hs + i];  // [target][source]: contiguous
        double acc[C];
#pragma unroll
        for (int c = 0; c < C; c++) acc[c] = 0.0;
        // terms lie in (-1.5 qt, 1.5 qt): below 2^42 the A <= 16 of them sum exactly without
        // folding; 50-bit targets fold every 4 (uniform branch)
        const bool fold = qt >= kBigPrime;
#pragma unroll
        for (int i = 0; i < A; i++) {
#pragma unroll
            for (int c = 0; c < C; c++) acc[c] += fmul_rem_r(y[c][i], f[i].w, f[i].wq, qt);
            if (fold && (i & 3) == 3) {
#pragma unroll
                for (int c = 0; c < C; c++) acc[c] = fred(acc[c], qt, qti);
            }
        }
        u64* o = ext + (long)bb * exs + ((long)t << logN) + k;
        // streaming stores: ext of one digit (B ne limbs) is far larger than the caches
#pragma unroll
        for (int c = 0; c < C; c++) __builtin_nontemporal_store(fcanon(acc[c], qt, qti), &o[256 * c]);
    }
}

// All digits at once: acc[b][c][t] = sum_j e_j[b][t] * key_j,c[pid(t)], e_j = d (limbs of digit
// j, NTT) or ext_j (other limbs).  key layout [dnum][2][np][N]; ext layout [beta][B][ne][N].
// grid (N/256, ne, 1); loops over the batch so each key word is read once per batch.
// With pmodf != nullptr (combined ModDown + rescale) the Q limbs also get P * addend_c
// (pmodf = (P mod q_i) / q_i), so that the later division by P * q_l... keeps the addend.
template <int BM>  // digits held in registers (beta <= BM)
__global__ void k_ks_inner_all(const u64* __restrict__ d, long dbs, const u64* __restrict__ ext,
                               long exs, long exj, const u64* __restrict__ key, long kdig,
                               long kcomp, u64* __restrict__ acc, long abs_, long acs, int B,
                               int beta, int K, int l, const u64* __restrict__ qall,
                               const double* __restrict__ qinvall, int Lp1, Opnd addend,
                               const double* __restrict__ pmodf, int logN, int accum) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int t = blockIdx.y;
    const int pid = t <= l ? t : Lp1 + (t - l - 1);
    const double q = (double)qall[pid];
    const double qi = qinvall[pid];
    const int own = t <= l ? t / K : -1;  // the digit whose limbs include t (Q limbs only)
    double kb[BM], ka[BM], kbq[BM], kaq[BM];
#pragma unroll
    for (int j = 0; j < BM; j++) {
        kb[j] = ka[j] = kbq[j] = kaq[j] = 0.0;
        if (j < beta) {
            const long ko = (long)j * kdig + ((long)pid << logN) + k;
            kb[j] = u2d(key[ko]);
            ka[j] = u2d(key[ko + kcomp]);
            kbq[j] = kb[j] * qi;
            kaq[j] = ka[j] * qi;
        }
    }
#pragma unroll 4
    for (int bb = 0; bb < B; bb++) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int j = 0; j < BM; j++) {
            if (j < beta) {
                const double e = u2d((j == own) ? d[(long)bb * dbs + ((long)t << logN) + k]
                                                : ext[(long)j * exj + (long)bb * exs + ((long)t << logN) + k]);
                s0 += fmul_rem(e, kb[j], kbq[j], q);
                s1 += fmul_rem(e, ka[j], kaq[j], q);
                if ((j & 3) == 3) {
                    s0 = fred(s0, q, qi);
                    s1 = fred(s1, q, qi);
                }
            }
        }
        if (pmodf && t <= l) {
            const double f = pmodf[t], w = tw_w(f, q);
            s0 = fred(s0, q, qi) + fmul_rem(u2d(opnd_get(addend, bb, 0, t, k, logN)), w, f, q);
            s1 = fred(s1, q, qi) + fmul_rem(u2d(opnd_get(addend, bb, 1, t, k, logN)), w, f, q);
        }
        u64* a0 = acc + (long)bb * abs_ + ((long)t << logN) + k;
        if (accum) {  // the lazy-ModDown sums of aesfhe_linear_bsgs
            s0 += u2d(a0[0]);
            s1 += u2d(a0[acs]);
        }
        a0[0] = fcanon(s0, q, qi);
        a0[acs] = fcanon(s1, q, qi);
    }
}

// Hoisted baby steps (aesfhe_linear_bsgs): the inner products of one extension with nk keys in
// one launch -- accs[i] = sum_j ext_j (x) keys[i]_j (+ P * addend on the Q limbs, as
// k_ks_inner_all with pmodf).  Keys are taken KC at a time into registers and the batch loop
// runs inside, so the extension slice of a workgroup (beta * B words per lane, 256 KB at B = 32:
// far beyond what L2 keeps per workgroup) is read ceil(nk / KC) times instead of nk times (it
// came from HBM every time: 7 ms per CtS call at 15 keys).  grid (N/256, ne, 1)
template <int BM, int KC>
__global__ void k_ks_inner_multi(const u64* __restrict__ d, long dbs, const u64* __restrict__ ext,
                                 long exs, long exj, const u64* const* __restrict__ keys, int nk, long kdig,
                                 long kcomp, u64* const* __restrict__ accs, long abs_, long acs, int B,
                                 int beta, int K, int l, const u64* __restrict__ qall,
                                 const double* __restrict__ qinvall, int Lp1, Opnd addend,
                                 const double* __restrict__ pmodf, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int t = blockIdx.y;
    const int pid = t <= l ? t : Lp1 + (t - l - 1);
    const double q = (double)qall[pid];
    const double qi = qinvall[pid];
    const int own = t <= l ? t / K : -1;
    const bool pm = pmodf && t <= l;
    const double f = pm ? pmodf[t] : 0.0, fw = pm ? tw_w(f, q) : 0.0;
    for (int i0 = 0; i0 < nk; i0 += KC) {
        double kb[KC][BM], ka[KC][BM];
#pragma unroll
        for (int ii = 0; ii < KC; ii++) {
#pragma unroll
            for (int j = 0; j < BM; j++) {
                // absent keys / digits read the zero word (address select, no branch per load)
                const bool ok = i0 + ii < nk && j < beta;
                const u64* kp = keys[ok ? i0 + ii : 0] + (long)j * kdig + ((long)pid << logN) + k;
                kb[ii][j] = u2d(*(ok ? kp : &kZeroWord));
                ka[ii][j] = u2d(*(ok ? kp + kcomp : &kZeroWord));
            }
        }
#pragma unroll 1
        for (int bb = 0; bb < B; bb++) {
            double e[BM];
#pragma unroll
            for (int j = 0; j < BM; j++)
                e[j] = u2d(*(j >= beta ? &kZeroWord
                             : (j == own) ? d + (long)bb * dbs + ((long)t << logN) + k
                                          : ext + (long)j * exj + (long)bb * exs + ((long)t << logN) + k));
            double ad0 = 0.0, ad1 = 0.0;
            if (pm) {
                ad0 = fmul_rem(u2d(opnd_get(addend, bb, 0, t, k, logN)), fw, f, q);
                ad1 = fmul_rem(u2d(opnd_get(addend, bb, 1, t, k, logN)), fw, f, q);
            }
#pragma unroll
            for (int ii = 0; ii < KC; ii++) {
                if (i0 + ii >= nk) break;
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int j = 0; j < BM; j++) {
                    if (j < beta) {
                        s0 += fmul_rem(e[j], kb[ii][j], kb[ii][j] * qi, q);
                        s1 += fmul_rem(e[j], ka[ii][j], ka[ii][j] * qi, q);
                        if ((j & 3) == 3) {
                            s0 = fred(s0, q, qi);
                            s1 = fred(s1, q, qi);
                        }
                    }
                }
                if (pm) {
                    s0 = fred(s0, q, qi) + ad0;
                    s1 = fred(s1, q, qi) + ad1;
                }
                u64* a0 = accs[i0 + ii] + (long)bb * abs_ + ((long)t << logN) + k;
                a0[0] = fcanon(s0, q, qi);
                a0[acs] = fcanon(s1, q, qi);
            }
        }
    }
}

// ModDown base conversion from the dropped limbs E = {q_{l-r+1}..q_l, p_0..p_{K-1}} (acc limbs
// l-r+1 .. l+K, already in coefficient form) to the kept limbs q_0..q_{l-r}; r = 0 is the plain
// ModDown by P, r >= 1 the combined ModDown + rescale by D = P q_l ... q_{l-r+1}:
//   y_j = [x_j * (D/e_j)^{-1}]_{e_j} in [0, e_j),  conv[i] = sum_j y_j * ((D/e_j) mod q_i) mod q_i.
// r >= 1 makes the conversion exact: v = rint(sum_j y_j * (1/e_j)) (fp64, j in order) counts the
// multiples of D in sum_j y_j (D/e_j), and conv[i] -= v * (D mod q_i), so the division rounds to
// nearest like a plain rescale (einv[j] = 1/e_j, dmodf[i] = (D mod q_i)/q_i).
// invf[j]: w/q table, hat[i * hs + j]: {w, w/q}.  grid (N/256, ceil((l-r+1)/16), B*2)
// NE = K + r (dropped limbs) as a template parameter, for the same reason as k_modup's A.
template <int NE>
__global__ void k_moddown(const u64* __restrict__ acc, long abs_, long acs, int l, int r,
                          u64* __restrict__ conv, long cbs, long ccs,
                          const double* __restrict__ invf, const TwD* __restrict__ hat,
                          const double* __restrict__ einv, const double* __restrict__ dmodf,
                          int Lp1, const u64* __restrict__ qall, const double* __restrict__ qinvall,
                          int logN, int hs) {
    // two coefficients per thread (k, k + 256), as k_modup
    const int k = blockIdx.x * 512 + threadIdx.x;
    const int bb = blockIdx.z >> 1, c = blockIdx.z & 1;
    const u64* src = acc + (long)bb * abs_ + (long)c * acs;
    const int t0 = l - r + 1;
    double y[NE], z[NE];
#pragma unroll
    for (int j = 0; j < NE; j++) {
        const int pid = j < r ? t0 + j : Lp1 + (j - r);
        const double pp = (double)qall[pid];
        const double f = invf[j], w = tw_w(f, pp);
        const u64* sp = src + ((long)(t0 + j) << logN) + k;
        const double v = fmul_rem(u2d(sp[0]), w, f, pp), v2 = fmul_rem(u2d(sp[256]), w, f, pp);
        y[j] = v < 0.0 ? v + pp : v;  // canonical: the oracle's conversion
        z[j] = v2 < 0.0 ? v2 + pp : v2;
    }
    double v = 0.0, v2 = 0.0;
    {  // exact conversion (every r): v multiples of D, round-to-nearest division
        double u = 0.0, u2 = 0.0;
#pragma unroll
        for (int j = 0; j < NE; j++) {
            u = u + y[j] * einv[j];
            u2 = u2 + z[j] * einv[j];
        }
        v = __builtin_rint(u);
        v2 = __builtin_rint(u2);
    }
    const int ig = (l - r + 1 + gridDim.y - 1) / gridDim.y, i0 = blockIdx.y * ig;  // outputs per thread
    for (int i = i0; i < i0 + ig && i <= l - r; i++) {
        const double q = (double)qall[i], qi = qinvall[i];
        const double fd = dmodf[i], wd = tw_w(fd, q);
        TwD f[NE];
#pragma unroll
        for (int j = 0; j < NE; j++) f[j] = hat[i * hs + j];  // [target][source]: contiguous
        double sum = fmul_rem(-v, wd, fd, q), sum2 = fmul_rem(-v2, wd, fd, q);
        const bool fold = q >= kBigPrime;  // as k_modup: small targets sum NE + 1 terms unfolded
#pragma unroll
        for (int j = 0; j < NE; j++) {
            sum += fmul_rem_r(y[j], f[j].w, f[j].wq, q);
            sum2 += fmul_rem_r(z[j], f[j].w, f[j].wq, q);
            if (fold && (j & 3) == 3) {
                sum = fred(sum, q, qi);
                sum2 = fred(sum2, q, qi);
            }
        }
        u64* o = conv + (long)bb * cbs + (long)c * ccs + ((long)i << logN) + k;
        __builtin_nontemporal_store(fcanon(sum, q, qi), &o[0]);  // streaming, as k_modup
        __builtin_nontemporal_store(fcanon(sum2, q, qi), &o[256]);
    }
}

// launch helper: F<n> for a runtime n in 1..16
#define AESFHE_DISPATCH16(n, F, ...)                                                     \
    switch (n) {                                                                         \
        case 1: F<1>(__VA_ARGS__); break;   case 2: F<2>(__VA_ARGS__); break;             \
        case 3: F<3>(__VA_ARGS__); break;   case 4: F<4>(__VA_ARGS__); break;             \
        case 5: F<5>(__VA_ARGS__); break;   case 6: F<6>(__VA_ARGS__); break;             \
        case 7: F<7>(__VA_ARGS__); break;   case 8: F<8>(__VA_ARGS__); break;             \
        case 9: F<9>(__VA_ARGS__); break;   case 10: F<10>(__VA_ARGS__); break;           \
        case 11: F<11>(__VA_ARGS__); break; case 12: F<12>(__VA_ARGS__); break;           \
        case 13: F<13>(__VA_ARGS__); break; case 14: F<14>(__VA_ARGS__); break;           \
        case 15: F<15>(__VA_ARGS__); break; case 16: F<16>(__VA_ARGS__); break;           \
        default: break;                                                                  \
    }

// out[b][c][i] = addend_c + (acc[b][c][i] - conv[b][c][i]) * D^{-1}  (addend absent: r >= 1) ; grid (N/256, l+1, B*2)
__global__ void k_moddown_finish(const u64* __restrict__ acc, long abs_, long acs,
                                 const u64* __restrict__ conv, long cbs, long ccs, Opnd addend,
                                 Out o, const u64* __restrict__ qs, const u64* __restrict__ pinv,
                                 const double* __restrict__ pinvf, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y, bb = blockIdx.z >> 1, c = blockIdx.z & 1;
    const u64 q = qs[i];
    u64 a = acc[(long)bb * abs_ + (long)c * acs + ((long)i << logN) + k];
    u64 v = conv[(long)bb * cbs + (long)c * ccs + ((long)i << logN) + k];
    u64 r = mul_w(sub_m(a, v, q), pinv[i], pinvf[i], q);
    r = add_m(r, opnd_get(addend, bb, c, i, k, logN), q);
    o.ptr[(long)bb * o.bs + (long)c * o.ps + ((long)i << logN) + k] = r;
}

// ---------------------------------------------------------------------------------------------
// automorphism X -> X^g in the NTT domain: out[k] = in[brv((g e(k) mod 2N - 1)/2)],
// e(k) = 2 brv(k) + 1.  grid (N/256, total limbs); src/dst Spans share the limb indexing.
__global__ void k_galois(Span src, Span dst, u64 g, int logN, int Lp1) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    int pid;
    const u64* in = span_ptr(src, blockIdx.y, logN, Lp1, pid);
    u64* out = span_ptr(dst, blockIdx.y, logN, Lp1, pid);
    const u64 M = 2ULL << logN;
    const unsigned rk = __brev((unsigned)k) >> (32 - logN);
    const u64 e = 2 * (u64)rk + 1;
    const u64 t = (g * e) & (M - 1);
    const unsigned idx = __brev((unsigned)((t - 1) >> 1)) >> (32 - logN);
    out[k] = in[idx];
}

// ---------------------------------------------------------------------------------------------
// sampling.  Uniform residues directly in the NTT domain, index pid*N + k.  A
// thread draws one ChaCha20 block = the 8 words of k = 8t .. 8t + 7.  grid (ceil(N / 2048), limbs)
__global__ void k_sample_uniform(Span dst, ChaKey K, u64 key, const u64* __restrict__ qall, int logN,
                                 int Lp1) {
    const int k0 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (k0 >= (1 << logN)) return;
    int pid;
    u64* out = span_ptr(dst, blockIdx.y, logN, Lp1, pid);
    uint32_t o[16];
    chacha20_block(K, key, (((u64)pid << logN) + k0) >> 3, o);
    const u64 q = qall[pid];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
        ulonglong2 v;
        v.x = __umul64hi((u64)o[2 * e] | ((u64)o[2 * e + 1] << 32), q);
        v.y = __umul64hi((u64)o[2 * e + 2] | ((u64)o[2 * e + 3] << 32), q);
        *(ulonglong2*)&out[k0 + e] = v;
    }
}

// small coefficient polynomial (kind 0 ternary, 1 CBD-21) -> residues of the span's limbs 0..nlim-1
// (coefficient form): one ChaCha20 block per thread (8 coefficients), written to every limb.
// grid ceil(N / 2048)
__global__ void k_sample_small(Span dst, ChaKey K, u64 key, int kind, const u64* __restrict__ qall,
                               int logN, int Lp1, int nlim) {
    const int k0 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (k0 >= (1 << logN)) return;
    uint32_t o[16];
    chacha20_block(K, key, (u64)k0 >> 3, o);
    i64 v[8];
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const u64 r = (u64)o[2 * e] | ((u64)o[2 * e + 1] << 32);
        v[e] = kind == 0 ? ternary(r) : cbd21(r);
    }
    for (int y = 0; y < nlim; y++) {
        int pid;
        u64* out = span_ptr(dst, y, logN, Lp1, pid);
        const u64 q = qall[pid];
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            ulonglong2 w;
            w.x = v[e] >= 0 ? (u64)v[e] : q - (u64)(-v[e]);
            w.y = v[e + 1] >= 0 ? (u64)v[e + 1] : q - (u64)(-v[e + 1]);
            *(ulonglong2*)&out[k0 + e] = w;
        }
    }
}

// signed 64-bit coefficients (device copy of host input) -> residues ; grid (N/256, nl, B)
__global__ void k_coeffs_res(const i64* __restrict__ co, u64* __restrict__ out, int nl,
                             const u64* __restrict__ qs, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z;
    const i64 v = co[((long)bb << logN) + k];
    const u64 q = qs[l];
    u64 r;
    if (v >= 0) r = (u64)v % q;
    else r = q - 1 - ((u64)(-(v + 1)) % q);
    out[(((long)bb * nl + l) << logN) + k] = r;
}

// key material: out = -a*s + e (+ pmod[pid] * sp) over the limbs of a Span-indexed set
// a, e, sp, out share the Span limb indexing (pid-major tables with row stride N)
__global__ void k_key_combine(const u64* __restrict__ a, const u64* __restrict__ s,
                              const u64* __restrict__ e, const u64* __restrict__ sp,
                              const u64* __restrict__ pmod, int lo, int hi, u64* __restrict__ out,
                              const u64* __restrict__ qall, const double* __restrict__ qinvall,
                              int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int pid = blockIdx.y;
    const long off = ((long)pid << logN) + k;
    const u64 q = qall[pid];
    const double qi = qinvall[pid];
    u64 v = add_m(sub_m(0, mul_m(a[off], s[off], q, qi), q), e[off], q);
    if (sp && pid >= lo && pid < hi) v = add_m(v, mul_m(pmod[pid], sp[off], q, qi), q);
    out[off] = v;
}

// public-key encryption: c0 = v pk0 + e0 + m, c1 = v pk1 + e1 (all NTT, limbs 0..l)
// vem: [B][4][l+1][N] = (v, e0, e1, m) ; grid (N/256, l+1, B)
__global__ void k_enc_pk(const u64* __restrict__ vem, const u64* __restrict__ pk0,
                         const u64* __restrict__ pk1, u64* __restrict__ ct, int nl,
                         const u64* __restrict__ qs, const double* __restrict__ qinv, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z;
    const u64 q = qs[l];
    const double qi = qinv[l];
    const long lo = ((long)l << logN) + k;
    const long step = (long)nl << logN;
    const u64* base = vem + (long)bb * 4 * step + lo;
    u64 v = base[0], e0 = base[step], e1 = base[2 * step], m = base[3 * step];
    u64* c = ct + (long)bb * 2 * step + lo;
    c[0] = add_m(add_m(mul_m(v, pk0[lo], q, qi), e0, q), m, q);
    c[step] = add_m(mul_m(v, pk1[lo], q, qi), e1, q);
}

// secret-key encryption: c1 = a (uniform, NTT), c0 = -a s + e0 + m ; vem as above with v unused.
// A thread takes 8 consecutive k (one ChaCha20 block of a).  grid (ceil(N / 2048), l+1, B)
__global__ void k_enc_sk(const u64* __restrict__ vem, const u64* __restrict__ s,
                         u64* __restrict__ ct, int nl, const u64* __restrict__ qs,
                         const double* __restrict__ qinv, ChaKey K, const u64* __restrict__ keys, int logN) {
    const int k0 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (k0 >= (1 << logN)) return;
    const int l = blockIdx.y, bb = blockIdx.z;
    const u64 q = qs[l];
    const double qi = qinv[l];
    const long step = (long)nl << logN;
    uint32_t o[16];
    chacha20_block(K, keys[bb], (((u64)l << logN) + k0) >> 3, o);
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const long lo = ((long)l << logN) + k0 + e;
        const u64* base = vem + (long)bb * 4 * step + lo;
        const u64 e0 = base[step], m = base[3 * step];
        const u64 a = __umul64hi((u64)o[2 * e] | ((u64)o[2 * e + 1] << 32), q);
        u64* c = ct + (long)bb * 2 * step + lo;
        c[step] = a;
        c[0] = add_m(add_m(sub_m(0, mul_m(a, s[lo], q, qi), q), e0, q), m, q);
    }
}

// limb-0 decryption combine: t[b][k] = c0 + c1 s (+ c2 s^2) ; grid (N/256, 1, B)
__global__ void k_dec_limb0(const u64* __restrict__ ct, long bs, long ps, int np,
                            const u64* __restrict__ s, u64* __restrict__ t, u64 q, double qinv,
                            int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int bb = blockIdx.z;
    const u64* c = ct + (long)bb * bs + k;
    u64 sv = s[k];
    u64 v = c[0];
    if (np >= 2) v = add_m(v, mul_m(c[ps], sv, q, qinv), q);
    if (np == 3) v = add_m(v, mul_m(c[2 * ps], mul_m(sv, sv, q, qinv), q, qinv), q);
    t[((long)bb << logN) + k] = v;
}

// elementwise square (s^2 for the relinearisation key) over np pid-major limbs
__global__ void k_square(const u64* __restrict__ s, u64* __restrict__ o,
                         const u64* __restrict__ qall, const double* __restrict__ qinvall,
                         int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const long off = ((long)blockIdx.y << logN) + k;
    o[off] = mul_m(s[off], s[off], qall[blockIdx.y], qinvall[blockIdx.y]);
}

// Bivariate polynomial evaluation with shared power bases (aesfhe_poly2).  For outputs
// t0 <= t < t0 + mc (mc <= kPoly2Out) and element (batch bb, limb l, coefficient k):
//   a_{t,i} = F[t,i,0] + sum_{j>=1} F[t,i,j] * y^j       (inner sums, never rescaled)
//   d_t     = (a_{t,0}, a'_{t,0}, 0) + sum_{i>=1} x^i (x) a_{t,i}
// F: TwD table [nl][half][mtot][nx][ny]; the j = 0 entries are additive constants, the i = 0
// row already carries the factor R = round(Delta_l) of the implicit x^0 ciphertext.
// All arithmetic is exact integer arithmetic in fp64 (fmul_rem / fred): signed residues in
// [-q, q], sums folded back below 2^53 every 4 terms.  The y basis lives in registers (as
// doubles), x^i is loaded once per i (outer loop), the mc output accumulators stay in
// registers.  x/y: pointer, batch-stride and poly-stride arrays of 2-poly ciphertexts at level
// >= nl-1 (only limbs 0..nl-1 are read: truncation).  out: [mtot][B][3][nl][N] (output t at
// out + t*oos).  grid (N/256, nl, B)
constexpr int kPoly2Max = 16, kPoly2Out = 4, kPoly2OutMax = 8;
__global__ void __launch_bounds__(256) k_poly2(const u64* const* __restrict__ xp, const long* __restrict__ xbs,
                        const long* __restrict__ xps, int nx, const u64* const* __restrict__ yp,
                        const long* __restrict__ ybs, const long* __restrict__ yps, int ny,
                        const TwD* __restrict__ F, int mtot, int t0, int mc,
                        u64* __restrict__ out, long oos, long obs, const u64* __restrict__ qs,
                        const double* __restrict__ qinv, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z, nl = gridDim.y;
    const int h = (int)((blockIdx.x * blockDim.x) >> (logN - 1));  // block-uniform half
    const double q = (double)qs[l];
    const double qi = qinv[l];
    const long off = ((long)l << logN) + k;
    double y0[kPoly2Max - 1], y1[kPoly2Max - 1];
#pragma unroll
    for (int j = 0; j < kPoly2Max - 1; j++) {
        y0[j] = y1[j] = 0.0;
        if (j < ny - 1) {
            const u64* p = yp[j] + (long)bb * ybs[j] + off;
            y0[j] = u2d(p[0]);
            y1[j] = u2d(p[yps[j]]);
        }
    }
    double d0[kPoly2Out], d1[kPoly2Out], d2[kPoly2Out];
#pragma unroll
    for (int t = 0; t < kPoly2Out; t++) d0[t] = d1[t] = d2[t] = 0.0;
    const TwD* Fl = F + ((size_t)(l * 2 + h) * mtot + t0) * nx * ny;
#pragma unroll 1
    for (int i = 0; i < nx; i++) {
        double xa = 0.0, xb = 0.0;
        if (i > 0) {
            const u64* p = xp[i - 1] + (long)bb * xbs[i - 1] + off;
            xa = u2d(p[0]);
            xb = u2d(p[xps[i - 1]]);
        }
#pragma unroll
        for (int t = 0; t < kPoly2Out; t++) {
            if (t < mc) {
                const TwD* Fi = Fl + ((size_t)t * nx + i) * ny;
                double a0 = Fi[0].w, a1 = 0.0;
#pragma unroll
                for (int j = 1; j < kPoly2Max; j++) {
                    if (j < ny) {
                        const TwD f = Fi[j];
                        a0 += fmul_rem_r(y0[j - 1], f.w, f.wq, q);
                        a1 += fmul_rem_r(y1[j - 1], f.w, f.wq, q);
                        if ((j & 3) == 0) {  // keep |sum| <= q/2 + 4q + q < 2^53
                            a0 = fred(a0, q, qi);
                            a1 = fred(a1, q, qi);
                        }
                    }
                }
                a0 = fred(a0, q, qi);
                a1 = fred(a1, q, qi);
                if (i == 0) {
                    d0[t] += a0;
                    d1[t] += a1;
                } else {
                    const double a0q = a0 * qi, a1q = a1 * qi;
                    d0[t] += fmul_rem(xa, a0, a0q, q);
                    d1[t] += fmul_rem(xa, a1, a1q, q) + fmul_rem(xb, a0, a0q, q);
                    d2[t] += fmul_rem(xb, a1, a1q, q);
                }
                d0[t] = fred(d0[t], q, qi);
                d1[t] = fred(d1[t], q, qi);
                d2[t] = fred(d2[t], q, qi);
            }
        }
    }
    u64* o = out + (long)bb * obs + off;
    const long pstr = (long)nl << logN;
#pragma unroll
    for (int t = 0; t < kPoly2Out; t++) {
        if (t < mc) {
            u64* ot = o + (long)(t0 + t) * oos;
            ot[0] = fcanon(d0[t], q, qi);
            ot[pstr] = fcanon(d1[t], q, qi);
            ot[2 * pstr] = fcanon(d2[t], q, qi);
        }
    }
}

// Integer-weight bivariate polynomial (aesfhe_poly2_int): out_t = sum (w_tij / den) x^i y^j.
// Constants factor as F_ij = w_ij * H(cx(i), cy(j)) (classes: x^0 / y^0 and one per basis level).
// The H factor lives on the y basis: y'_j = H(c, cy(j)) * y_j for the current x class c (x is
// sorted by class; entering class c multiplies y' by Rt[c][cy(j)] = H(c,cy) H(c-1,cy)^{-1}, or
// H(0,cy) for c = 0), so every inner sum is a_i = c0 * w_i0 + sum_j w_ij y'_j with small integer
// weights: exact fp64 FMAs with no folding where |a| <= (|w_0| + sum_j |w_j| / 2) q < 2^52 (the host
// picks the kernel per limb from the actual weights: every limb of a 40-44-bit chain for the AES
// S-box's |64 W| <= 8), the tensor accumulators staying below 2^53.  Other limbs (the 50-bit q_0)
// use remainder products and fold.  Wt: [mtot][nx][ny] doubles (scalar loads), Rt: [nl][cxn][cyn]
// {w, w/q}, C0: [nl][cxn] = H(c, 0) as doubles, xstart[c]..xstart[c+1]: the i of class c.  BIG: the q >= 2^42 path; the host launches
// each run of limbs of one size class (limbs l0 .. l0 + gridDim.y - 1 of nl).  grid (N/256, run, B)
// NY > 0: ny fixed at compile time (the weight loads are then unconditional and issued together;
// with a runtime ny each scalar load sat behind its own branch and was waited for alone).
template <bool BIG, int NY, int MO>  // MO: outputs per launch (<= MOMax)
__global__ void __launch_bounds__(256, MO > 4 ? 2 : 3) k_poly2_int(const u64* const* __restrict__ xp, const long* __restrict__ xbs,
                        const long* __restrict__ xps, int nx, const u64* const* __restrict__ yp,
                        const long* __restrict__ ybs, const long* __restrict__ yps, int ny,
                        const int* __restrict__ xstart, const int* __restrict__ ycls, int cxn,
                        int cyn, const double* __restrict__ Wt, const TwD* __restrict__ Rt,
                        const double* __restrict__ C0, int mtot, int t0, int mc,
                        u64* __restrict__ out, long oos, long obs, const u64* __restrict__ qs,
                        const double* __restrict__ qinv, int l0, int nl, int logN, int orot) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = l0 + blockIdx.y, bb = blockIdx.z;
    const double q = (double)qs[l];
    const double qi = qinv[l];
    constexpr bool big = BIG;
    const int nyv = NY > 0 ? NY : ny;
    const long off = ((long)l << logN) + k;
    double d0[MO], d1[MO], d2[MO];
#pragma unroll
    for (int t = 0; t < MO; t++) d0[t] = d1[t] = d2[t] = 0.0;
    const TwD* Rl = Rt + (size_t)l * cxn * cyn;
#pragma unroll 1
    for (int c = 0; c < cxn; c++) {  // x classes in order: y' = H(c, cy(j)) * y_j, reloaded
        const TwD* Rc = Rl + c * cyn;
        double y0[kPoly2Max - 1], y1[kPoly2Max - 1];
#pragma unroll
        for (int j = 0; j < kPoly2Max - 1; j++) {
            y0[j] = y1[j] = 0.0;
            if (j < nyv - 1) {
                const u64* p = yp[j] + (long)bb * ybs[j] + off;
                const TwD r = Rc[ycls[j + 1]];
                y0[j] = fred(fmul_rem_r(u2d(p[0]), r.w, r.wq, q), q, qi);
                y1[j] = fred(fmul_rem_r(u2d(p[yps[j]]), r.w, r.wq, q), q, qi);
            }
        }
        const double c0 = C0[(size_t)l * cxn + c];
#pragma unroll 1
    for (int i = xstart[c]; i < xstart[c + 1]; i++) {
        double xa = 0.0, xb = 0.0;
        if (i > 0) {
            const u64* p = xp[i - 1] + (long)bb * xbs[i - 1] + off;
            xa = u2d(p[0]);
            xb = u2d(p[xps[i - 1]]);
        }
#pragma unroll
        for (int t = 0; t < MO; t++) {
            if (t < mc) {
                const double* w = Wt + ((size_t)(t0 + t) * nx + i) * ny;
                double a0, a1;
                if constexpr (!big) {
                    a0 = w[0] * c0;  // exact: |w0| <= 1024, c0 < 2^42
                    a1 = 0.0;
#pragma unroll
                    for (int j = 1; j < kPoly2Max; j++) {
                        if (j < nyv) {
                            a0 = __builtin_fma(w[j], y0[j - 1], a0);
                            a1 = __builtin_fma(w[j], y1[j - 1], a1);
                        }
                    }
                } else {
                    const double w0 = w[0];
                    a0 = fmul_rem(c0, w0, w0 * qi, q);
                    a1 = 0.0;
#pragma unroll
                    for (int j = 1; j < kPoly2Max; j++) {
                        if (j < nyv) {
                            const double wj = w[j], wjq = wj * qi;
                            a0 = fred(a0 + fmul_rem(y0[j - 1], wj, wjq, q), q, qi);
                            a1 = fred(a1 + fmul_rem(y1[j - 1], wj, wjq, q), q, qi);
                        }
                    }
                }
                if (i == 0) {
                    d0[t] += a0;
                    d1[t] += a1;
                } else {
                    const double a0q = a0 * qi, a1q = a1 * qi;
                    d0[t] += fmul_rem(xa, a0, a0q, q);
                    d1[t] += fmul_rem(xa, a1, a1q, q) + fmul_rem(xb, a0, a0q, q);
                    d2[t] += fmul_rem(xb, a1, a1q, q);
                }
                if constexpr (big) {
                    d0[t] = fred(d0[t], q, qi);
                    d1[t] = fred(d1[t], q, qi);
                    d2[t] = fred(d2[t], q, qi);
                }
            }
        }
    }
    }
    // orot (aesfhe_poly2_int_rot): element 4 s + c of each output takes input element
    // 4 s + ((c + orot) & 3) -- the output written rotated within its slab of 4
    const int ob = (bb & ~3) | ((bb - orot) & 3);
    u64* o = out + (long)ob * obs + off;
    const long pstr = (long)nl << logN;
#pragma unroll
    for (int t = 0; t < MO; t++) {
        if (t < mc) {
            u64* ot = o + (long)(t0 + t) * oos;
            ot[0] = fcanon(d0[t], q, qi);
            ot[pstr] = fcanon(d1[t], q, qi);
            ot[2 * pstr] = fcanon(d2[t], q, qi);
        }
    }
}

// a = w_0 c0 + sum_j w_j y'_j (polynomial 0) and a' = sum_j w_j y''_j (polynomial 1): exact FMAs
// (the sums stay below 2^52), or for BIG limbs remainder products folded as they are added
template <int NY, bool BIG>
__device__ __forceinline__ void inner_sums(const double* __restrict__ w, double c0, const double (&y0)[NY - 1],
                                           const double (&y1)[NY - 1], double q, double qi, double& a0, double& a1) {
    if constexpr (!BIG) {
        a0 = w[0] * c0;  // exact: |w0| <= 1024, c0 < 2^45
        a1 = 0.0;
#pragma unroll
        for (int j = 1; j < NY; j++) {
            a0 = __builtin_fma(w[j], y0[j - 1], a0);
            a1 = __builtin_fma(w[j], y1[j - 1], a1);
        }
    } else {
        const double w0 = w[0];
        a0 = fmul_rem(c0, w0, w0 * qi, q);
        a1 = 0.0;
#pragma unroll
        for (int j = 1; j < NY; j++) {
            const double wj = w[j], wjq = wj * qi;
            a0 = fred(a0 + fmul_rem(y0[j - 1], wj, wjq, q), q, qi);
            a1 = fred(a1 + fmul_rem(y1[j - 1], wj, wjq, q), q, qi);
        }
    }
}

// k_poly2_int's exact path (BIG = false) for the S-box shape: the full 16-term y basis, whole
// blocks of MO outputs (no per-output guards), the x^0 term peeled out of the monomial loop (no
// per-monomial branches), and LAZY: y' = H y left unreduced (|y'| <= q instead of q/2 + 1: the
// fred of every y' word -- 3 fp64 ops x 30 per class -- dropped; the host takes LAZY where the
// doubled bound still keeps |a| <= (|w_0| + sum_j |w_j|) q < 2^51 and the tensor sums < 2^52).
// The inner sums and the tensor accumulators are exact integers congruent to k_poly2_int's, so
// the canonical outputs are the same words.
// Both output blocks (t0 .. t0 + MO - 1 and t0 + MO .. t0 + 2 MO - 1) in one launch: workgroups b
// and b + 8 -- dealt to the same XCD -- take the same 256 coefficients, one block each, so the
// second one's x / y reads hit that XCD's L2 instead of HBM.  grid (2 N/256, run, B).
// BIG (q_0 and other limbs past the exact-FMA bound): every inner-sum term a remainder product,
// folded as it is added, and the tensor accumulators folded per monomial (k_poly2_int<true>'s
// arithmetic), so the whole 8-output block of those limbs is one launch as well.
template <int MO, bool LAZY, bool BIG = false>
__global__ void __launch_bounds__(256, 3) k_poly2_int_s(const u64* const* __restrict__ xp, const long* __restrict__ xbs,
                        const long* __restrict__ xps, int nx, const u64* const* __restrict__ yp,
                        const long* __restrict__ ybs, const long* __restrict__ yps,
                        const int* __restrict__ xstart, const int* __restrict__ ycls, int cxn,
                        int cyn, const double* __restrict__ Wt, const TwD* __restrict__ Rt,
                        const double* __restrict__ C0, int t0, u64* __restrict__ out, long oos, long obs,
                        const u64* __restrict__ qs, const double* __restrict__ qinv, int l0, int nl,
                        int logN, int orot) {
    constexpr int NY = kPoly2Max;
    static_assert(!(BIG && LAZY), "the folding path needs reduced y'");
    const int bx = blockIdx.x, half = (bx >> 3) & 1;            // blocks b, b + 8: one XCD
    const int k = (((bx >> 4) << 3) | (bx & 7)) * blockDim.x + threadIdx.x;
    const int l = l0 + blockIdx.y, bb = blockIdx.z;
    t0 += half * MO;
    const double q = (double)qs[l];
    const double qi = qinv[l];
    const long off = ((long)l << logN) + k;
    const TwD* Rl = Rt + (size_t)l * cxn * cyn;
    double y0[NY - 1], y1[NY - 1];
    auto load_y = [&](int c) {  // y' = H(c, cy(j)) y_j
        const TwD* Rc = Rl + c * cyn;
#pragma unroll
        for (int j = 0; j < NY - 1; j++) {
            const u64* p = yp[j] + (long)bb * ybs[j] + off;
            const TwD r = Rc[ycls[j + 1]];
            const double v0 = fmul_rem_r(u2d(p[0]), r.w, r.wq, q), v1 = fmul_rem_r(u2d(p[yps[j]]), r.w, r.wq, q);
            y0[j] = LAZY ? v0 : fred(v0, q, qi);
            y1[j] = LAZY ? v1 : fred(v1, q, qi);
        }
    };
    double d0[MO], d1[MO], d2[MO];
    // class 0 = the x^0 term: d = (a_0, a_0', 0)
    load_y(0);
    {
        const double c0 = C0[(size_t)l * cxn];
#pragma unroll
        for (int t = 0; t < MO; t++) {
            const double* w = Wt + (size_t)(t0 + t) * nx * NY;
            double a0, a1;
            inner_sums<NY, BIG>(w, c0, y0, y1, q, qi, a0, a1);
            d0[t] = a0;
            d1[t] = a1;
            d2[t] = 0.0;
        }
    }
#pragma unroll 1
    for (int c = 1; c < cxn; c++) {
        load_y(c);
        const double c0 = C0[(size_t)l * cxn + c];
#pragma unroll 1
        for (int i = xstart[c]; i < xstart[c + 1]; i++) {
            const u64* p = xp[i - 1] + (long)bb * xbs[i - 1] + off;
            const double xa = u2d(p[0]), xb = u2d(p[xps[i - 1]]);
#pragma unroll
            for (int t = 0; t < MO; t++) {
                const double* w = Wt + ((size_t)(t0 + t) * nx + i) * NY;
                double a0, a1;
                inner_sums<NY, BIG>(w, c0, y0, y1, q, qi, a0, a1);
                const double a0q = a0 * qi, a1q = a1 * qi;
                d0[t] += fmul_rem(xa, a0, a0q, q);
                d1[t] += fmul_rem(xa, a1, a1q, q) + fmul_rem(xb, a0, a0q, q);
                d2[t] += fmul_rem(xb, a1, a1q, q);
                if constexpr (BIG) {
                    d0[t] = fred(d0[t], q, qi);
                    d1[t] = fred(d1[t], q, qi);
                    d2[t] = fred(d2[t], q, qi);
                }
            }
        }
    }
    const int ob = (bb & ~3) | ((bb - orot) & 3);  // aesfhe_poly2_int_rot
    u64* o = out + (long)ob * obs + off;
    const long pstr = (long)nl << logN;
#pragma unroll
    for (int t = 0; t < MO; t++) {
        u64* ot = o + (long)(t0 + t) * oos;
        ot[0] = fcanon(d0[t], q, qi);
        ot[pstr] = fcanon(d1[t], q, qi);
        ot[2 * pstr] = fcanon(d2[t], q, qi);
    }
}

// k_poly2_int_s for the limbs past the exact-FMA bound (the 50-bit q_0), the inner sums split
// instead of folded: y' = yh 2^24 + yl (|yl| <= 2^23, |yh| <= 2^26: exact), so sum_j w_j yh_j and
// sum_j w_j yl_j are exact fp64 FMA chains (row sums <= 512: below 2^35) and a = fmul_rem(ah, 2^24)
// + al (|a| <= 1.5 q + 2^32 < 2^51).  16 + 16 FMAs and one remainder product per (output,
// monomial, polynomial) instead of 16 remainder products with folds.  The two y polynomials run in
// two passes over the monomials (one split y basis live: 60 VGPRs, not 120): pass 0 adds x_a a0
// into d0 and x_b a0 into d1, pass 1 x_a a1 into d1 and x_b a1 into d2.  Same residues as the
// folding kernel (every step exact mod q, canonical outputs).  grid (2 N/256, run, B) as
// k_poly2_int_s (blocks b, b + 8: the two output blocks on one XCD).
template <int MO>
__global__ void __launch_bounds__(256, 3) k_poly2_int_split(const u64* const* __restrict__ xp, const long* __restrict__ xbs,
                        const long* __restrict__ xps, int nx, const u64* const* __restrict__ yp,
                        const long* __restrict__ ybs, const long* __restrict__ yps,
                        const int* __restrict__ xstart, const int* __restrict__ ycls, int cxn,
                        int cyn, const double* __restrict__ Wt, const TwD* __restrict__ Rt,
                        const double* __restrict__ C0, int t0, u64* __restrict__ out, long oos, long obs,
                        const u64* __restrict__ qs, const double* __restrict__ qinv, int l0, int nl,
                        int logN, int orot) {
    constexpr int NY = kPoly2Max;
    constexpr double S = 16777216.0, Si = 1.0 / 16777216.0;  // 2^24
    const int bx = blockIdx.x, half = (bx >> 3) & 1;
    const int k = (((bx >> 4) << 3) | (bx & 7)) * blockDim.x + threadIdx.x;
    const int l = l0 + blockIdx.y, bb = blockIdx.z;
    t0 += half * MO;
    const double q = (double)qs[l], qi = qinv[l], sq = S * qi;
    const long off = ((long)l << logN) + k;
    const TwD* Rl = Rt + (size_t)l * cxn * cyn;
    double d0[MO], d1[MO], d2[MO];
#pragma unroll
    for (int t = 0; t < MO; t++) d0[t] = d1[t] = d2[t] = 0.0;
#pragma unroll 1
    for (int p = 0; p < 2; p++) {
        double yh[NY - 1], yl[NY - 1];
#pragma unroll 1
        for (int c = 0; c < cxn; c++) {
            const TwD* Rc = Rl + c * cyn;
#pragma unroll
            for (int j = 0; j < NY - 1; j++) {  // y' = H(c, cy(j)) y_j, reduced, split at 2^24
                const u64* yq = yp[j] + (long)bb * ybs[j] + off + (p ? yps[j] : 0);
                const TwD r = Rc[ycls[j + 1]];
                const double v = fred(fmul_rem_r(u2d(*yq), r.w, r.wq, q), q, qi);
                yh[j] = __builtin_rint(v * Si);
                yl[j] = __builtin_fma(-yh[j], S, v);
            }
            const double c0 = p ? 0.0 : C0[(size_t)l * cxn + c];  // the x^0 term: polynomial 0 only
            const double c0h = __builtin_rint(c0 * Si), c0l = __builtin_fma(-c0h, S, c0);
#pragma unroll 1
            for (int i = xstart[c]; i < xstart[c + 1]; i++) {  // class 0: i = 0, the x^0 term
                double xa = 1.0, xb = 0.0;  // x^0: (1, 0)
                if (i > 0) {
                    const u64* xq = xp[i - 1] + (long)bb * xbs[i - 1] + off;
                    xa = u2d(xq[0]);
                    xb = u2d(xq[xps[i - 1]]);
                }
#pragma unroll
                for (int t = 0; t < MO; t++) {
                    const double* w = Wt + ((size_t)(t0 + t) * nx + i) * NY;
                    double ah = w[0] * c0h, al = w[0] * c0l;
#pragma unroll
                    for (int j = 1; j < NY; j++) {
                        ah = __builtin_fma(w[j], yh[j - 1], ah);
                        al = __builtin_fma(w[j], yl[j - 1], al);
                    }
                    const double a = fmul_rem(ah, S, sq, q) + al, aq = a * qi;
                    if (i == 0) {  // x^0: a itself
                        if (p == 0) d0[t] += a;
                        else d1[t] += a;
                    } else if (p == 0) {
                        d0[t] += fmul_rem(xa, a, aq, q);
                        d1[t] += fmul_rem(xb, a, aq, q);
                    } else {
                        d1[t] += fmul_rem(xa, a, aq, q);
                        d2[t] += fmul_rem(xb, a, aq, q);
                    }
                    d0[t] = fred(d0[t], q, qi);
                    d1[t] = fred(d1[t], q, qi);
                    d2[t] = fred(d2[t], q, qi);
                }
            }
        }
    }
    const int ob = (bb & ~3) | ((bb - orot) & 3);  // aesfhe_poly2_int_rot
    u64* o = out + (long)ob * obs + off;
    const long pstr = (long)nl << logN;
#pragma unroll
    for (int t = 0; t < MO; t++) {
        u64* ot = o + (long)(t0 + t) * oos;
        ot[0] = fcanon(d0[t], q, qi);
        ot[pstr] = fcanon(d1[t], q, qi);
        ot[2 * pstr] = fcanon(d2[t], q, qi);
    }
}

// ModRaise: x = limb 0 of every polynomial in coefficient form (mod q_0); out limb i =
// centred x mod q_i for i < nl.  x: [P][N] (P = B * npoly), out: [P][nl][N].  grid (N/256, nl, P)
__global__ void k_lift0(const u64* __restrict__ x, u64* __restrict__ out, int nl, u64 q0,
                        const u64* __restrict__ qs, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y, p = blockIdx.z;
    const u64 v = x[((long)p << logN) + k], q = qs[i];
    u64 r;
    if (v > (q0 >> 1)) {  // negative: v - q0
        const u64 m = (q0 - v) % q;
        r = m ? q - m : 0;
    } else {
        r = v % q;
    }
    out[(((long)p * nl + i) << logN) + k] = r;
}

// Sum of ciphertext x plaintext products: out[b][p][l] = sum_i ct_i[b][p][l] * pt_i[l] (lazy
// fp64 sums folded every 4 terms).  grid (N/256, nl, B*np)
__global__ void k_dot_pt(const u64* const* __restrict__ cp, const long* __restrict__ cbs, long cps,
                         const u64* const* __restrict__ pp, int n, Out o, int np,
                         const u64* __restrict__ qs, const double* __restrict__ qinv, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int l = blockIdx.y, bb = blockIdx.z / np, p = blockIdx.z - bb * np;
    const double q = (double)qs[l], qi = qinv[l];
    const long off = ((long)l << logN) + k;
    double acc = 0.0;
    int i = 0;
    for (; i + 8 <= n; i += 8) {  // chunks of 8 loads in flight: one HBM round trip per chunk
        double cv[8], wv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            cv[u] = u2d(cp[i + u][(long)bb * cbs[i + u] + (long)p * cps + off]);
            wv[u] = u2d(pp[i + u][off]);
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            acc += fmul_rem(cv[u], wv[u], wv[u] * qi, q);
            if ((u & 3) == 3) acc = fred(acc, q, qi);
        }
    }
    for (; i < n; i++) {
        const double c = u2d(cp[i][(long)bb * cbs[i] + (long)p * cps + off]);
        const double w = u2d(pp[i][off]);
        acc += fmul_rem(c, w, w * qi, q);
        if ((i & 3) == 3) acc = fred(acc, q, qi);
    }
    o.ptr[(long)bb * o.bs + (long)p * o.ps + off] = fcanon(acc, q, qi);
}

// ---- lazy-ModDown linear transforms (aesfhe_linear_bsgs) over Q_l u P limbs ---------------------
// limb t of an extended polynomial (t <= l: q_t, else p_{t-l-1}) has prime index ext_pid
__device__ __forceinline__ int ext_pid(int t, int l, int Lp1) { return t <= l ? t : Lp1 + (t - l - 1); }

// out[b][c][t] = (P mod q_t) * in[b][c][t] on the Q limbs, 0 on the P limbs (P * x in Q_l u P);
// in: Opnd (level-l ciphertext), out: [B][2][ne][N].  grid (N/256, ne, B*2)
__global__ void k_scale_p_ext(Opnd in, u64* __restrict__ out, int l, int ne, const u64* __restrict__ qall,
                              const double* __restrict__ qinvall, const double* __restrict__ pmodf, int Lp1, int logN) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int t = blockIdx.y, bb = blockIdx.z >> 1, c = blockIdx.z & 1;
    u64 v = 0;
    if (t <= l) {
        const double q = (double)qall[t], qi = qinvall[t], f = pmodf[t];
        v = fcanon(fmul_rem(u2d(opnd_get(in, bb, c, t, k, logN)), tw_w(f, q), f, q), q, qi);
    }
    out[((((long)bb * 2 + c) * ne + t) << logN) + k] = v;
}

// All giants of a BSGS map in one pass over the babies: outs[j][b][c][t] = sum_i pt[j][i][t] *
// E_i[b][c][t] (pt[j * nb + i] == nullptr: no term), so each baby is read once instead of once
// per giant (the QP-domain term sums were 18 % of a bootstrap, memory-bound on the re-reads).
// GM: accumulators held in registers (ng <= GM).  grid (N/256, ne, B*2)
// gal[i] > 1: baby i is stored unpermuted and sigma_{gal[i]} is applied by the read (the NTT-slot
// gather of k_galois), so the permuted copy of each baby is never written.
template <int GM, int BCT>
__global__ void k_dot_pt_ext_multi(const u64* const* __restrict__ ep, const u64* __restrict__ gal,
                                   const u64* const* __restrict__ pt, int nb,
                                   int ng, u64* const* __restrict__ outs, int l, int ne,
                                   const u64* __restrict__ qall, const double* __restrict__ qinvall, int Lp1,
                                   int logN, int nbc) {
    // 1-D grid, XCD-local plaintext rows: block id -> (x = id & 7, w = id >> 3); pair (limb t,
    // 256-word k-block) = (w / ng_) * 8 + x, bc group = w % ng_ (ng_ = nbc / BCT groups of BCT
    // (b, c) polynomials) -- the workgroups that share one pair's plaintext words (nb * ng rows of
    // 2 KB) run back to back on one XCD, so the plaintexts come from HBM once instead of once per
    // ciphertext (dealt over XCDs by limb, the 1.3 GB of CtS plaintexts were re-read from HBM by
    // every bc), and each plaintext word loaded serves BCT polynomials (the L2 -> CU load count per
    // baby word drops from 1 + ng to 1 + ng / BCT).  The automorphism gather of a k-block reads
    // exactly one 2 KB row of the baby (its high index byte is fixed by the block).
    const int kbits = logN - 8, ngrp = nbc / BCT;
    const int x8 = blockIdx.x & 7, w = blockIdx.x >> 3;
    const int pair = (w / ngrp) * 8 + x8, bc0 = (w % ngrp) * BCT;
    if (pair >= (ne << kbits)) return;
    const int t = pair >> kbits, k = ((pair & ((1 << kbits) - 1)) << 8) + threadIdx.x;
    const int pid = ext_pid(t, l, Lp1);
    const double q = (double)qall[pid], qi = qinvall[pid];
    const long po = ((long)t << logN) + k;
    long base[BCT];
#pragma unroll
    for (int u = 0; u < BCT; u++) base[u] = ((long)(bc0 + u) * ne + t) << logN;  // bc = 2 b + c
    const u64 M = 2ULL << logN;
    const u64 ek = 2 * (u64)(__brev((unsigned)k) >> (32 - logN)) + 1;
    double acc[BCT][GM];
#pragma unroll
    for (int u = 0; u < BCT; u++)
#pragma unroll
        for (int j = 0; j < GM; j++) acc[u][j] = 0.0;
    for (int i = 0; i < nb; i++) {
        const u64 g = gal[i];
        long src = k;
        if (g > 1) src = __brev((unsigned)((((g * ek) & (M - 1)) - 1) >> 1)) >> (32 - logN);
        double e[BCT];
#pragma unroll
        for (int u = 0; u < BCT; u++) e[u] = u2d(ep[i][base[u] + src]);
        // every giant's plaintext word is requested before the first product (a load behind
        // each pointer test serialised the GM loads)
        const u64* pj[GM];
        double wv[GM];
#pragma unroll
        for (int j = 0; j < GM; j++) pj[j] = j < ng ? pt[j * nb + i] : nullptr;
#pragma unroll
        for (int j = 0; j < GM; j++) wv[j] = pj[j] ? u2d(pj[j][po]) : 0.0;
#pragma unroll
        for (int j = 0; j < GM; j++) {
            if (pj[j]) {
                const double wq = wv[j] * qi;
#pragma unroll
                for (int u = 0; u < BCT; u++) acc[u][j] += fmul_rem(e[u], wv[j], wq, q);
            }
        }
        if ((i & 3) == 3) {
#pragma unroll
            for (int u = 0; u < BCT; u++)
#pragma unroll
                for (int j = 0; j < GM; j++) acc[u][j] = fred(acc[u][j], q, qi);
        }
    }
#pragma unroll
    for (int j = 0; j < GM; j++)
        if (j < ng) {
#pragma unroll
            for (int u = 0; u < BCT; u++) outs[j][base[u] + k] = fcanon(acc[u][j], q, qi);
        }
}

// The babies of a lazy-ModDown BSGS map formed on the fly inside its term sums (round 5; replaces
// k_scale_p_ext + k_ks_inner_multi + k_dot_pt_ext_multi): baby i in Q_l u P at NTT slot src = the
// slot sigma_i reads (the k_galois gather; identity: src = k) is
//   keyed:    E_c = sum_d x_d[src] key_{i,d,c}[src] (+ P c0[src] for c = 0 on the Q limbs), x_d = the
//             extension of digit d (ext) or, on the digit's own limbs, c1 itself;
//   identity: E_c = P c_c[src] on the Q limbs, 0 on the special limbs,
// and every giant's sum takes outs[j][b][c][t][k] = sum_i pt[j][i][t][k] E_{i,c}: the same
// residues as the three kernels (each step exact mod q, outputs canonical), but the babies -- nb
// full Q u P batches, written and read back -- never reach HBM: per (b, t, k) the HBM words drop
// from ~4 nb + beta ceil(nk / KC) to the beta extension words (their permuted re-reads for the
// other babies hit the 2 KB row already cached) and the sums written.  Keys (2 beta words per baby)
// and plaintexts are shared by the batch through L2 (the XCD-local grid of k_dot_pt_ext_multi).
// The 256-slot k-blocks are walked in the order kord (host, bsgs_block_order): a block's slots
// all read ONE source block per baby (sigma_g maps the top 8 bits of k by the top 8 bits alone),
// and with babies g_i = g_1^i the blocks block k reads are the orbit window pi^i(kb), i < nb, of
// the block map pi of g_1 -- so walking kb along pi's orbits, each XCD taking one contiguous
// eighth of the walk, gives consecutive workgroups nb - 1 of nb source blocks in common (ext, c0,
// c1 and keys reused from the XCD's L2).  Identity order when the babies are not powers of one
// element.  grid: 1-D, block id -> (x = id & 7, w = id >> 3): r = w / ceil(B / BB) runs over
// (limb t, position in x's eighth of the walk), batch block w % ceil(B / BB) fastest (the keys
// of one k-block shared by the whole batch from L2).  GM >= ng accumulator pairs; BM >= beta.
// PB: babies whose loads are issued together; OCC: launch-bounds wave target (tools/bsgs_bench.hip)
template <int GM, int BM, int BB, int PB = 1, int OCC = 1>
__global__ __launch_bounds__(256, OCC) void k_bsgs_terms(const u64* __restrict__ c0p, long c0bs, const u64* __restrict__ c1p, long c1bs,
                             const u64* __restrict__ ext, long exs, long exj,
                             const u64* const* __restrict__ keys, const u64* __restrict__ gal, long kdig, long kcomp,
                             const u64* const* __restrict__ pt, int nb, int ng, u64* const* __restrict__ outs,
                             int l, int ne, int beta, int A, const u64* __restrict__ qall,
                             const double* __restrict__ qinvall, const double* __restrict__ pmodf, int Lp1, int logN,
                             int B, const unsigned short* __restrict__ kord) {
    // BB batch elements per thread: every key and plaintext word loaded serves BB of them (the
    // first form, one element per thread, re-read each baby's 2 beta key words per element from
    // L2 and lost to the unfused kernels)
    const int nblk = 1 << (logN - 8), nbb = (B + BB - 1) / BB;
    const int x8 = blockIdx.x & 7, w = blockIdx.x >> 3;
    const int r = w / nbb, b0 = (w % nbb) * BB;
    int t, m;
    if (nblk >= 8) {  // XCD x8 walks positions [x8 seg, x8 seg + seg) of every limb
        const int seg = nblk >> 3;
        t = r / seg;
        m = x8 * seg + r - t * seg;
    } else {  // fewer blocks than XCDs (N < 2^11): positions dealt round robin
        const int pos = r * 8 + x8;
        t = pos / nblk;
        m = pos - t * nblk;
    }
    if (t >= ne) return;
    const int k = ((int)kord[m] << 8) + threadIdx.x;
    const int pid = ext_pid(t, l, Lp1);
    const bool isq = t <= l;
    const int own = isq ? t / A : -1;
    const double q = (double)qall[pid], qi = qinvall[pid];
    const double pf = isq ? pmodf[t] : 0.0, pw = isq ? tw_w(pf, q) : 0.0;
    const long po = ((long)t << logN) + k;
    const u64 M = 2ULL << logN;
    const u64 ek = 2 * (u64)(__brev((unsigned)k) >> (32 - logN)) + 1;
    const u64* c0r[BB];
    const u64* c1r[BB];
    const u64* er[BB];
#pragma unroll
    for (int u = 0; u < BB; u++) {  // elements past B alias the last one (computed, not stored)
        const int b = min(b0 + u, B - 1);
        c0r[u] = c0p + (long)b * c0bs + ((long)t << logN);
        c1r[u] = c1p + (long)b * c1bs + ((long)t << logN);
        er[u] = ext + (long)b * exs + ((long)t << logN);
    }
    double acc0[BB][GM], acc1[BB][GM];
#pragma unroll
    for (int u = 0; u < BB; u++)
#pragma unroll
        for (int j = 0; j < GM; j++) acc0[u][j] = acc1[u][j] = 0.0;
    // absent plaintexts (a giant without a term on this baby) read the zero word: w = 0 adds 0
    auto pt_word = [&](int j, int i) {
        const u64* pp = j < ng ? pt[j * nb + i] : nullptr;
        return u2d(*(pp ? pp + po : &kZeroWord));
    };
    auto add_terms = [&](const double (&e0)[BB], const double (&e1)[BB], const double (&wv)[GM]) {
#pragma unroll
        for (int u = 0; u < BB; u++) {
            const double f0 = fred(e0[u], q, qi), f1 = fred(e1[u], q, qi);  // |e| <= q/2 + 1
#pragma unroll
            for (int j = 0; j < GM; j++) {
                const double wq = wv[j] * qi;
                acc0[u][j] += fmul_rem(f0, wv[j], wq, q);
                acc1[u][j] += fmul_rem(f1, wv[j], wq, q);
            }
        }
    };
    int i = 0;
    if (!keys[0]) {  // the identity baby (rotation 0, the host puts it first): (P c0, P c1) on the Q limbs
        double wv[GM], e0[BB], e1[BB];
#pragma unroll
        for (int j = 0; j < GM; j++) wv[j] = pt_word(j, 0);
#pragma unroll
        for (int u = 0; u < BB; u++) {
            e0[u] = isq ? fmul_rem(u2d(*(isq ? c0r[u] + k : &kZeroWord)), pw, pf, q) : 0.0;
            e1[u] = isq ? fmul_rem(u2d(*(isq ? c1r[u] + k : &kZeroWord)), pw, pf, q) : 0.0;
        }
        add_terms(e0, e1, wv);
        i = 1;
    }
    // keyed babies, PB per iteration with every load of the PB issued before any arithmetic (a
    // past-the-end slot of the last iteration re-reads baby nb - 1 and adds nothing)
    int nsum = 1;
#pragma unroll 1
    for (; i < nb; i += PB) {
        double kb[PB][BM], ka[PB][BM], x[PB][BB][BM], c0v[PB][BB], wv[PB][GM];
#pragma unroll
        for (int p = 0; p < PB; p++) {
            const int ii = min(i + p, nb - 1);
            const bool live = i + p < nb;
            const u64 g = gal[ii];
            const long src = __brev((unsigned)((((g * ek) & (M - 1)) - 1) >> 1)) >> (32 - logN);
            const u64* kp = keys[ii];
#pragma unroll
            for (int d = 0; d < BM; d++) {  // the baby's key words: once for the BB elements
                const u64* kk = kp + (long)min(d, beta - 1) * kdig + ((long)pid << logN) + src;
                kb[p][d] = u2d(kk[0]);
                ka[p][d] = u2d(kk[kcomp]);
            }
#pragma unroll
            for (int j = 0; j < GM; j++) wv[p][j] = live ? pt_word(j, ii) : 0.0;
#pragma unroll
            for (int u = 0; u < BB; u++) {
#pragma unroll
                for (int d = 0; d < BM; d++)  // the own digit's word is c1 itself (Q limbs only: own = -1 on P)
                    x[p][u][d] = u2d(*(d == own ? c1r[u] + src : er[u] + (long)min(d, beta - 1) * exj + src));
                c0v[p][u] = u2d(*(isq ? c0r[u] + src : &kZeroWord));  // c has the Q limbs only
            }
        }
#pragma unroll
        for (int p = 0; p < PB; p++) {
            double e0[BB], e1[BB];
#pragma unroll
            for (int u = 0; u < BB; u++) {
                double a0 = isq ? fmul_rem(c0v[p][u], pw, pf, q) : 0.0, a1 = 0.0;
#pragma unroll
                for (int d = 0; d < BM; d++) {
                    if (d < beta) {
                        a0 += fmul_rem(x[p][u][d], kb[p][d], kb[p][d] * qi, q);
                        a1 += fmul_rem(x[p][u][d], ka[p][d], ka[p][d] * qi, q);
                        if ((d & 3) == 3) {
                            a0 = fred(a0, q, qi);
                            a1 = fred(a1, q, qi);
                        }
                    }
                }
                e0[u] = a0;
                e1[u] = a1;
            }
            add_terms(e0, e1, wv[p]);
        }
        nsum += PB;
        if (nsum >= 4) {  // accumulators: <= 4 + PB - 1 terms of < 1.5 q between folds
            nsum = 0;
#pragma unroll
            for (int u = 0; u < BB; u++)
#pragma unroll
                for (int j = 0; j < GM; j++) {
                    acc0[u][j] = fred(acc0[u][j], q, qi);
                    acc1[u][j] = fred(acc1[u][j], q, qi);
                }
        }
    }
#pragma unroll
    for (int u = 0; u < BB; u++) {
        if (b0 + u >= B) break;
#pragma unroll
        for (int j = 0; j < GM; j++)
            if (j < ng) {
                u64* o = outs[j] + (((long)(2 * (b0 + u)) * ne + t) << logN) + k;
                o[0] = fcanon(acc0[u][j], q, qi);
                o[(long)ne << logN] = fcanon(acc1[u][j], q, qi);
            }
    }
}

}  // namespace aesfhe
