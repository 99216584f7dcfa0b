// ks_fused.h -- key-switch inner product fused into the row pass of the ext NTT (N = 2^16, 2^17).
//
// The unfused key switch (engine.hip ks_modup / ks_apply) writes every extended limb ext[j][b][t]
// in canonical NTT form (row pass) and reads it straight back in k_ks_inner_all:
// 2 * beta * B * (l + 1 + K) limbs of HBM traffic per call, the largest single item of a key
// switch.  Here ks_modup stops after the column pass (the raw-double intermediate stays in the
// ext buffer) and one workgroup per (target limb t, 8-row block, batch element b) runs the row
// pass of ext[j][b][t] for every digit j in registers, multiplies by the key digit and
// accumulates, writing only the two accumulators acc[b][0/1][t] (accum: added to what acc holds)
// -- the same canonical values k_ks_inner_all produces (the arithmetic is exact mod q; only the lazy ranges differ).
//
// Ranges: the row NTT (table twiddles) leaves |x| <= 17q for q < 2^42 (folded to q/2 + 1 for larger primes
// before the product); fmul_rem(x, key) lies in (-1.5q, 1.5q) (on-the-fly key quotient), so the
// beta <= 12 products plus the folded initial term (<= q/2 + 1) sum below 19q < 2^47 for small
// primes; big primes fold every 4 digits (< 6.5q < 2^53).
#pragma once
#include "kernels_ops.h"
#include "ntt256f.h"

namespace aesfhe {

// Row NTT with 8 elements per lane (32 lanes per 256-point row), so that the two accumulators of
// the inner product fit beside it at 4+ waves per SIMD (16 elements per lane held 232 VGPRs:
// 2 waves per SIMD, latency-bound).  Layouts of row element e (0..255), lane L (0..31), register r:
//   A: e = L + 32 r          stages ml = 1, 2, 4     (distances 128, 64, 32)
//   B: e = 32 (L >> 2) + (L & 3) + 4 r   ml = 8, 16, 32   (16, 8, 4)
//   C: e = 8 L + r           ml = 64, 128     (2, 1)
// then back to A for the coalesced inner product.  Twiddle of stage ml, element e:
// psi^{brv(ml rt + (e >> (8 - log2 ml)))}.  LDS per row: e -> e + (e >> 3) (288 words),
// conflict-free for the A / B / C patterns.
__device__ __forceinline__ int r8p(int e) { return e + (e >> 3); }

// A row (and its LDS region) belongs to 32 lanes of ONE wave, so the layout exchanges need only
// wave-level ordering, not a workgroup barrier: LDS instructions of a wave complete in issue
// order, and the fence + wave barrier stop the compiler from moving the accesses across.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// rt: 256 + row when W is the limb's global psi table, 1 when W is the row's own LDS copy
// (entry ml + j = the table's ml rt + j, stages ml = 1 .. 128).
__device__ __forceinline__ void row_ntt8_stages(double (&x)[8], double* sr, int L, int rt, const double* W, double q,
                                                double qi, bool big);
__device__ __forceinline__ void row_ntt8_fwd(double (&x)[8], const u64* rp, double* sr, int L, int rt,
                                             const double* W, double q, double qi, bool big) {
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = ld_d(&rp[L + 32 * r]);
    row_ntt8_stages(x, sr, L, rt, W, q, qi, big);
}
__device__ __forceinline__ void row_ntt8_stages(double (&x)[8], double* sr, int L, int rt, const double* W, double q,
                                                double qi, bool big) {
    // A: ml = 1, 2, 4 (global stages 0..2 of the pass); twiddle j = r >> (3 - st)
#pragma unroll
    for (int st = 0; st < 3; st++) {
        const int ml = 1 << st, h = 4 >> st;
        if (big && (st & 1) == 0) {
#pragma unroll
            for (int r = 0; r < 8; r++) x[r] = fred(x[r], q, qi);
        }
        const int base = ml * rt;
#pragma unroll
        for (int j = 0; j < ml; j++) {
            const double wq = W[base + j];
#pragma unroll
            for (int k = 0; k < h; k++) ct_f(x[j * 2 * h + k], x[j * 2 * h + k + h], wq, q);
        }
    }
#pragma unroll
    for (int r = 0; r < 8; r++) sr[r8p(L + 32 * r)] = x[r];
    wave_lds_sync();
    const int eb = 32 * (L >> 2) + (L & 3);
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = sr[r8p(eb + 4 * r)];
    // B: ml = 8, 16, 32 (stages 3..5); twiddle j = e >> (8 - st) = (L >> 2) * ml / 8 + (r >> (6 - st))
#pragma unroll
    for (int st = 3; st < 6; st++) {
        const int ml = 1 << st, h = 4 >> (st - 3), nj = ml >> 3;
        if (big && (st & 1) == 0) {
#pragma unroll
            for (int r = 0; r < 8; r++) x[r] = fred(x[r], q, qi);
        }
        const int base = ml * rt + (L >> 2) * nj;
#pragma unroll
        for (int j = 0; j < nj; j++) {
            const double wq = W[base + j];
#pragma unroll
            for (int k = 0; k < h; k++) ct_f(x[j * 2 * h + k], x[j * 2 * h + k + h], wq, q);
        }
    }
    wave_lds_sync();  // every lane has read its B elements
#pragma unroll
    for (int r = 0; r < 8; r++) sr[r8p(eb + 4 * r)] = x[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = sr[r8p(8 * L + r)];
    // C: ml = 64 (distance 2, j = 2L + (r >> 2)), ml = 128 (distance 1, j = 4L + (r >> 1))
    if (big) {
#pragma unroll
        for (int r = 0; r < 8; r++) x[r] = fred(x[r], q, qi);
    }
    {
        const int base = 64 * rt + 2 * L;
        const double w0 = W[base], w1 = W[base + 1];
        ct_f(x[0], x[2], w0, q);
        ct_f(x[1], x[3], w0, q);
        ct_f(x[4], x[6], w1, q);
        ct_f(x[5], x[7], w1, q);
    }
    {
        const int base = 128 * rt + 4 * L;
#pragma unroll
        for (int j = 0; j < 4; j++) ct_f(x[2 * j], x[2 * j + 1], W[base + j], q);
    }
    wave_lds_sync();  // every lane has read its C elements
#pragma unroll
    for (int r = 0; r < 8; r++) sr[r8p(8 * L + r)] = big ? fred(x[r], q, qi) : x[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = sr[r8p(L + 32 * r)];  // back to A
    wave_lds_sync();  // the next digit rewrites sr
}

// Inverse (Gentleman-Sande) row pass in the same layouts, mirrored: C (distances 1, 2), B (4, 8,
// 16), A (32, 64, 128); x in and out in layout A.  W: the row's inverse twiddles staged like the
// forward ones (entry ml + g = ipsi^brv(ml (R + row) + g), ml = 128 / distance groups per row).
// Raw doubles out, as k_nttf_inv_rows: inputs folded to |x| <= q/2 + 1, so below 2^42 the sums
// reach 2^8 (q/2 + 1) < 2^50; larger primes fold every sum (the inverse column pass folds its
// input first either way).
__device__ __forceinline__ void row_intt8(double (&x)[8], double* sr, int L, const double* W, double q, double qi,
                                          bool big) {
    auto gs = [&](double& a, double& b, double wq) {
        if (big) gs_f<true>(a, b, wq, q, qi);
        else gs_f<false>(a, b, wq, q, qi);
    };
#pragma unroll
    for (int r = 0; r < 8; r++) sr[r8p(L + 32 * r)] = x[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = sr[r8p(8 * L + r)];
    // C: distance 1 (ml = 128, group 4L + j), distance 2 (ml = 64, group 2L + (r >> 2))
#pragma unroll
    for (int j = 0; j < 4; j++) gs(x[2 * j], x[2 * j + 1], W[128 + 4 * L + j]);
    {
        const double w0 = W[64 + 2 * L], w1 = W[64 + 2 * L + 1];
        gs(x[0], x[2], w0);
        gs(x[1], x[3], w0);
        gs(x[4], x[6], w1);
        gs(x[5], x[7], w1);
    }
    wave_lds_sync();  // every lane has read its C elements
#pragma unroll
    for (int r = 0; r < 8; r++) sr[r8p(8 * L + r)] = x[r];
    wave_lds_sync();
    const int eb = 32 * (L >> 2) + (L & 3);
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = sr[r8p(eb + 4 * r)];
    // B: distances 4, 8, 16 = ml 32, 16, 8 (register distance h = 1, 2, 4; nj = ml / 8 groups)
#pragma unroll
    for (int st = 5; st >= 3; st--) {
        const int ml = 1 << st, h = 4 >> (st - 3), nj = ml >> 3;
        const int base = ml + (L >> 2) * nj;
#pragma unroll
        for (int j = 0; j < nj; j++) {
            const double wq = W[base + j];
#pragma unroll
            for (int k = 0; k < h; k++) gs(x[j * 2 * h + k], x[j * 2 * h + k + h], wq);
        }
    }
    wave_lds_sync();  // every lane has read its B elements
#pragma unroll
    for (int r = 0; r < 8; r++) sr[r8p(eb + 4 * r)] = x[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = sr[r8p(L + 32 * r)];
    // A: distances 32, 64, 128 = ml 4, 2, 1 (h = 1, 2, 4)
#pragma unroll
    for (int st = 2; st >= 0; st--) {
        const int ml = 1 << st, h = 4 >> st;
#pragma unroll
        for (int j = 0; j < ml; j++) {
            const double wq = W[ml + j];
#pragma unroll
            for (int k = 0; k < h; k++) gs(x[j * 2 * h + k], x[j * 2 * h + k + h], wq);
        }
    }
    wave_lds_sync();  // sr is free again
}

// grid: 8 * ceil(B / G) * (ne * (R / 8) / 8) blocks of 256 (8 rows x 32 lanes; R = N / 256 rows:
// 256 or 512); block id -> (xcd group
// x = id & 7, batch group, pair), pair = (t, 8-row block): all batch groups of one (t, row block)
// are dealt to one XCD (blocks x, x + 8, ...) so the key rows they share are L2 hits.  G batch
// elements per workgroup share each key word loaded (G = 2 halves the key reads, the largest
// load stream of the kernel, at the price of a second pair of accumulators).
//
// PROD (relinearisation of a ciphertext product a (x) b, combined ModDown + rescale): no tensor
// ciphertext exists.  On the Q limbs the prologue reads a0, a1, b0, b1 and forms d0 = a0 b0,
// d1 = a0 b1 + a1 b0 (the addend, times P) and d2 = a1 b1 (the own digit's limb, times its key
// words), so the own digit is skipped in the loop; addend = a, d = unused, pb = b.  Products
// by fmul_rem with the on-the-fly quotient, as the key products: congruent, not canonical,
// |x| < 3q before the P / key product.  fac (optional; aesfhe_mul_fma): per-prime {alpha, C, K};
// the product becomes alpha (a (x) b) + C (c0, c1, 0) + (K, 0, 0) (pc = c, absent: no C term),
// |x| < 4.5q + K before the P / key product.
//
// Target limbs t0 .. t0 + nt - 1 only (the grid covers nt limbs).  EPI selects the epilogue:
// 0 the canonical accumulators into acc; 2 (INV) their inverse row pass instead, raw doubles into
// acc (ModDown's INTT then runs only its column pass: the dropped limbs of ks_finish_fused);
// 1 (FIN, G = 1): the
// ModDown finish of the key switch in the epilogue, for Q limbs t <= lk (engine.hip
// ks_finish_fused): the limb's two accumulators never reach HBM.  The conv limbs (column pass
// done, raw doubles, fin.conv[b][c][t]) get their row pass here -- same prime, same row, so the
// staged twiddles serve them -- and out[b][c][t] = (acc_c - conv_c) D^{-1} (+ fin.add_c) is
// written canonical; the dropped limbs (t > lk) ran through the non-FIN launch first, into acc.
// The PROD prologue (see k_nttf_rows_ks below): d0 = a0 b0, d1 = a0 b1 + a1 b0 times P and the own
// digit's d2 = a1 b1 times its key words, for the lane's 8 elements of (limb t, row).  FMA (the
// multiply-add of aesfhe_mul_fma, fac != nullptr) is a template argument: with a runtime `if (fac)`
// inside the element loop every element's 6 operand loads sat behind their own branch and wait
// (the ISA showed vmcnt(5)..(0) per element), so the prologue's 48 loads were serialised 8 times.
template <bool FMA>
__device__ __forceinline__ void ks_prod_prologue(double (&a0)[8], double (&a1)[8], const u64* kp, long kcomp,
                                                 const u64* xa, long aps, const u64* xb, long bps, const u64* xc,
                                                 long cps, bool has_c, double wv, double f, double fal, double fC,
                                                 double fK, double q, double qi, bool big) {
    double x0[8], x1[8], y0[8], y1[8], kb[8], ka[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {  // every operand word requested before the first product
        x0[r] = u2d(xa[32 * r]);
        x1[r] = u2d(xa[aps + 32 * r]);
        y0[r] = u2d(xb[32 * r]);
        y1[r] = u2d(xb[bps + 32 * r]);
        kb[r] = u2d(kp[32 * r]);
        ka[r] = u2d(kp[32 * r + kcomp]);
    }
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const double y0q = y0[r] * qi, y1q = y1[r] * qi;
        double p0 = fmul_rem(x0[r], y0[r], y0q, q);
        double p1 = fmul_rem(x0[r], y1[r], y1q, q) + fmul_rem(x1[r], y0[r], y0q, q);
        double p2 = fmul_rem(x1[r], y1[r], y1q, q);
        if constexpr (FMA) {  // multiply-add: alpha (a (x) b) + C (c0, c1, 0) + (K, 0, 0)
            p0 = fmul_rem(p0, fal, fal * qi, q) + fK;
            p1 = fmul_rem(p1, fal, fal * qi, q);
            p2 = fmul_rem(p2, fal, fal * qi, q);
            if (has_c) {
                p0 += fmul_rem(u2d(xc[32 * r]), fC, fC * qi, q);
                p1 += fmul_rem(u2d(xc[cps + 32 * r]), fC, fC * qi, q);
            }
        }
        a0[r] = fmul_rem(p0, wv, f, q) + fmul_rem(p2, kb[r], kb[r] * qi, q);
        a1[r] = fmul_rem(p1, wv, f, q) + fmul_rem(p2, ka[r], ka[r] * qi, q);
        if (big) {
            a0[r] = fred(a0[r], q, qi);
            a1[r] = fred(a1[r], q, qi);
        }
    }
}

struct KsFin {
    const u64* conv;
    long cbs, cps;
    u64* out;
    long obs, ops;
    const double* dinvf;  // D^{-1} mod q_t as w / q
    Opnd2 add;            // plain ModDown (r = 0): the addend joins here, not in the accumulators
};
template <int G, int R = 256, bool PROD = false, int EPI = 0>
__global__ __launch_bounds__(256, G == 1 ? 4 : 2) void k_nttf_rows_ks(const u64* __restrict__ d, long dbs,
                                                      const u64* __restrict__ ext, long exs, long exj,
                                                      const u64* __restrict__ key, long kdig, long kcomp,
                                                      u64* __restrict__ acc, long abs_, long acs, int B,
                                                      int beta, int K, int l, int ne, Tabs T, Opnd addend,
                                                      const double* __restrict__ pmodf, int accum, Opnd pb,
                                                      const u64* __restrict__ fac, Opnd pc, int t0, int nt,
                                                      KsFin fin) {
    constexpr bool FIN = EPI == 1, INV = EPI == 2;
    static_assert(!FIN || G == 1, "the fused finish runs one batch element per workgroup");
    // one LDS array (row transposes, then the 8 rows' twiddles -- see row_ntt8_fwd's rt)
    __shared__ double s[8 * 288 + 8 * 256];
    const int nbg = (B + G - 1) / G;
    const int id = blockIdx.x, x8 = id & 7, rest = id >> 3;
    const int b0 = (rest % nbg) * G, pair = (rest / nbg) * 8 + x8;
    constexpr int RB = R / 8;  // 8-row blocks per limb
    constexpr int LOGN = R == 256 ? 16 : 17;
    const int tq = pair / RB, rb = pair - tq * RB;
    if (tq >= nt) return;
    const int t = t0 + tq;
    const int pid = t <= l ? t : T.Lp1 + (t - l - 1);
    const int own = t <= l ? t / K : -1;  // the digit whose limbs include t (Q limbs only)
    const int tid = threadIdx.x, L = tid & 31, rl = tid >> 5;
    const int row = rb * 8 + rl;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* W = T.psif + ((long)pid << LOGN);
    double* sr = s + rl * 288;
    // the row's 255 twiddles are the same for every digit: staged in LDS once per workgroup
    double* tw = s + 8 * 288 + rl * 256;
#pragma unroll
    for (int m = 0; m < 8; m++) {
        const int e = L + 32 * m;
        if (e > 0) {
            const int ml = 1 << (31 - __clz(e));
            tw[e] = W[(long)ml * (R + row) + (e - ml)];
        }
    }
    wave_lds_sync();  // the row's twiddles: written and read by its own 32 lanes
    const long roff = ((long)t << LOGN) + (long)row * 256 + L;  // element (row, L + 32 r) at roff + 32 r
    // the accumulators start from the epilogue terms (P * addend, the previous acc), so their
    // loads are issued first and land while the digits compute; folded to |x| <= q/2 + 1
    double a0[G][8], a1[G][8];
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int bb = b0 + g;
#pragma unroll
        for (int r = 0; r < 8; r++) a0[g][r] = a1[g][r] = 0.0;
        if (bb >= B) continue;
        // operand words at (limb t, row, L + 32 r): base pointers formed once (block-uniform
        // checks), so the 8 loads of each stream issue together (an opnd_get per element put
        // every load behind its own branch and serialised the prologue)
        if (PROD && t <= l) {
            const double f = pmodf[t], w = tw_w(f, q);
            const u64* kp = key + (long)own * kdig + ((long)pid << LOGN) + (long)row * 256 + L;
            const u64* xa = addend.ptr + (long)(bb & addend.bmask) * addend.bs + roff;
            const u64* xb = pb.ptr + (long)(bb & pb.bmask) * pb.bs + roff;
            const u64* xc = pc.ptr ? pc.ptr + (long)(bb & pc.bmask) * pc.bs + roff : xb;
            const double fal = fac ? (double)fac[3 * t] : 0.0, fC = fac ? (double)fac[3 * t + 1] : 0.0,
                         fK = fac ? (double)fac[3 * t + 2] : 0.0;
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const double x0 = u2d(xa[32 * r]), x1 = u2d(xa[addend.ps + 32 * r]);
                const double y0 = u2d(xb[32 * r]), y1 = u2d(xb[pb.ps + 32 * r]);
                const double kb = u2d(kp[32 * r]), ka = u2d(kp[32 * r + kcomp]);
                const double y0q = y0 * qi, y1q = y1 * qi;
                double p0 = fmul_rem(x0, y0, y0q, q);
                double p1 = fmul_rem(x0, y1, y1q, q) + fmul_rem(x1, y0, y0q, q);
                double p2 = fmul_rem(x1, y1, y1q, q);
                if (fac) {  // multiply-add: alpha (a (x) b) + C (c0, c1, 0) + (K, 0, 0)
                    p0 = fmul_rem(p0, fal, fal * qi, q) + fK;
                    p1 = fmul_rem(p1, fal, fal * qi, q);
                    p2 = fmul_rem(p2, fal, fal * qi, q);
                    if (pc.ptr) {
                        p0 += fmul_rem(u2d(xc[32 * r]), fC, fC * qi, q);
                        p1 += fmul_rem(u2d(xc[pc.ps + 32 * r]), fC, fC * qi, q);
                    }
                }
                a0[g][r] = fmul_rem(p0, w, f, q) + fmul_rem(p2, kb, kb * qi, q);
                a1[g][r] = fmul_rem(p1, w, f, q) + fmul_rem(p2, ka, ka * qi, q);
                if (big) {
                    a0[g][r] = fred(a0[g][r], q, qi);
                    a1[g][r] = fred(a1[g][r], q, qi);
                }
            }
        } else if (!PROD && pmodf && t <= l && addend.ptr) {
            const double f = pmodf[t], w = tw_w(f, q);
            const u64* xa = addend.ptr + (long)bb * addend.bs + roff;
            if (addend.np > 0) {
#pragma unroll
                for (int r = 0; r < 8; r++) a0[g][r] = fmul_rem(u2d(xa[32 * r]), w, f, q);
            }
            if (addend.np > 1) {
#pragma unroll
                for (int r = 0; r < 8; r++) a1[g][r] = fmul_rem(u2d(xa[addend.ps + 32 * r]), w, f, q);
            }
        }
        if (accum) {
            const u64* o0 = acc + (long)bb * abs_ + roff;
#pragma unroll
            for (int r = 0; r < 8; r++) {
                a0[g][r] = fred(a0[g][r] + u2d(o0[32 * r]), q, qi);
                a1[g][r] = fred(a1[g][r] + u2d(o0[acs + 32 * r]), q, qi);
            }
        }
    }
    int nsum = 0;  // digits summed since the last fold (big primes fold every 4)
#pragma unroll 1
    for (int j = 0; j < beta; j++) {
        if (PROD && j == own) continue;  // in the prologue (block-uniform)
        // the key digit's words are loaded first: they arrive while the row NTT computes
        const u64* kp = key + (long)j * kdig + ((long)pid << LOGN) + (long)row * 256 + L;
        u64 kbw[8], kaw[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            kbw[r] = kp[32 * r];
            kaw[r] = kp[32 * r + kcomp];
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int bb = b0 + g;
            if (bb >= B) break;  // block-uniform
            double v[8];
            if (j == own) {  // the digit's own limbs: d itself, already in NTT form
                const u64* dp = d + (long)bb * dbs + roff;
#pragma unroll
                for (int r = 0; r < 8; r++) v[r] = u2d(dp[32 * r]);
            } else {
                row_ntt8_fwd(v, ext + (long)j * exj + (long)bb * exs + ((long)t << LOGN) + (long)row * 256, sr, L, 1,
                             tw, q, qi, big);
            }
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const double kb = u2d(kbw[r]), ka = u2d(kaw[r]);
                a0[g][r] += fmul_rem(v[r], kb, kb * qi, q);
                a1[g][r] += fmul_rem(v[r], ka, ka * qi, q);
            }
        }
        if (big && (++nsum & 3) == 0) {
#pragma unroll
            for (int g = 0; g < G; g++)
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    a0[g][r] = fred(a0[g][r], q, qi);
                    a1[g][r] = fred(a1[g][r], q, qi);
                }
        }
    }
    if constexpr (FIN) {
        // ranges: |acc| < 19q and |conv| <= 17q below 2^42 (file header), so |acc - conv| < 2^48;
        // big primes fold both to q/2 + 1 first -- fmul_rem's input bound either way
        const int bb = b0;
        if (bb >= B) return;
        const double f = fin.dinvf[t], w = tw_w(f, q);
        const long coff = ((long)t << LOGN) + (long)row * 256;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            double cv[8];
            row_ntt8_fwd(cv, fin.conv + (long)bb * fin.cbs + (long)c * fin.cps + coff, sr, L, 1, tw, q, qi, big);
            const u64* ap = fin.add.ptr && c < fin.add.np ? fin.add.ptr + (long)bb * fin.add.bs + (long)c * fin.add.ps + roff
                                                          : nullptr;
            u64* op = fin.out + (long)bb * fin.obs + (long)c * fin.ops + roff;
#pragma unroll
            for (int r = 0; r < 8; r++) {
                double a = c ? a1[0][r] : a0[0][r];
                if (big) a = fred(a, q, qi);
                double v = fmul_rem(a - cv[r], w, f, q);
                if (ap) v += u2d(ap[32 * r]);
                __builtin_nontemporal_store(fcanon(v, q, qi), &op[32 * r]);  // streaming
            }
        }
        return;
    }
    if constexpr (INV) {
        // the row's inverse twiddles replace its forward ones in LDS (the row's own 32 lanes;
        // row_ntt8_stages ended with a wave barrier, so every forward read is done)
        const double* IW = T.ipsif + ((long)pid << LOGN);
#pragma unroll
        for (int m = 0; m < 8; m++) {
            const int e = L + 32 * m;
            if (e > 0) {
                const int ml = 1 << (31 - __clz(e));
                tw[e] = IW[(long)ml * (R + row) + (e - ml)];
            }
        }
        wave_lds_sync();
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int bb = b0 + g;
            if (bb >= B) break;
            u64* o0 = acc + (long)bb * abs_ + roff;
#pragma unroll
            for (int c = 0; c < 2; c++) {
                double x[8];
#pragma unroll
                for (int r = 0; r < 8; r++) x[r] = fred(c ? a1[g][r] : a0[g][r], q, qi);
                row_intt8(x, sr, L, tw, q, qi, big);
#pragma unroll
                for (int r = 0; r < 8; r++) st_d(&o0[(long)c * acs + 32 * r], x[r]);
            }
        }
        return;
    }
#pragma unroll
    for (int g = 0; g < G; g++) {
        const int bb = b0 + g;
        if (bb >= B) break;
        u64* o0 = acc + (long)bb * abs_ + roff;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            __builtin_nontemporal_store(fcanon(a0[g][r], q, qi), &o0[32 * r]);  // streaming
            __builtin_nontemporal_store(fcanon(a1[g][r], q, qi), &o0[acs + 32 * r]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Pipelined variant (G = 1): the extension row of the NEXT digit (and, in
// the FIN epilogue, the next conv row) is fetched by LDS-DMA (global_load_lds_dwordx4: no VGPR
// destination) into a per-wave staging buffer while the current digit's row NTT runs, so the ext
// latency that k_nttf_rows_ks exposes once per digit (the load is issued, then waited for by the
// NTT's first butterflies) overlaps the NTT instead.  The own digit of a plain key switch (d rows,
// already NTT form) joins the prologue.  16 KB more LDS (51.2 KB: 3 workgroups per CU) and no
// more registers for the staging.  A row pair of a wave is 4 KB contiguous in HBM and lands
// linearly in the wave's 4 KB of the buffer (4 x 1 KB wave-instructions); the wave that issues a
// DMA is the one that reads it (after its own vmcnt), so no workgroup barrier is needed.
typedef __attribute__((address_space(3))) void ks_lds_void;
__device__ __forceinline__ void ks_dma_rows(const u64* g, double* lds_wave, int lane) {
#pragma unroll
    for (int k = 0; k < 4; k++)
        __builtin_amdgcn_global_load_lds((const void*)(g + 128 * k + 2 * lane), (ks_lds_void*)(lds_wave + 128 * k), 16, 0, 0);
}
// every DMA of this wave landed (and, being the issuing wave, its LDS reads see the bytes)
__device__ __forceinline__ void ks_dma_wait() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
// this wave's LDS reads are complete before a new DMA may overwrite the buffer
__device__ __forceinline__ void ks_lds_reads_done() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

template <int R = 256, bool PROD = false, int EPI = 0>
__global__ __launch_bounds__(256, 3) void k_nttf_rows_ks_p(const u64* __restrict__ d, long dbs,
                                                      const u64* __restrict__ ext, long exs, long exj,
                                                      const u64* __restrict__ key, long kdig, long kcomp,
                                                      u64* __restrict__ acc, long abs_, long acs, int B,
                                                      int beta, int K, int l, int ne, Tabs T, Opnd addend,
                                                      const double* __restrict__ pmodf, int accum, Opnd pb,
                                                      const u64* __restrict__ fac, Opnd pc, int t0, int nt,
                                                      KsFin fin) {
    constexpr bool FIN = EPI == 1, INV = EPI == 2;
    // sr (row transposes) | tw (the 8 rows' twiddles) | eb (DMA staging, 2 rows per wave)
    __shared__ double s[8 * 288 + 8 * 256 + 8 * 256];
    const int id = blockIdx.x, x8 = id & 7, rest = id >> 3;
    const int bb = rest % B, pair = (rest / B) * 8 + x8;
    constexpr int RB = R / 8;
    constexpr int LOGN = R == 256 ? 16 : 17;
    const int tq = pair / RB, rb = pair - tq * RB;
    if (tq >= nt) return;
    const int t = t0 + tq;
    const int pid = t <= l ? t : T.Lp1 + (t - l - 1);
    const int own = t <= l ? t / K : -1;
    const int tid = threadIdx.x, L = tid & 31, rl = tid >> 5, lane = tid & 63, w = tid >> 6;
    const int row = rb * 8 + rl;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* W = T.psif + ((long)pid << LOGN);
    double* sr = s + rl * 288;
    double* tw = s + 8 * 288 + rl * 256;
    double* ebw = s + 8 * 288 + 8 * 256 + w * 512;  // the wave's 2 rows
    const double* er = ebw + (rl & 1) * 256;         // this lane's row in it
    const long woff = ((long)t << LOGN) + (long)(rb * 8 + 2 * w) * 256;  // the wave's first row
    // the first ext digit is requested before anything else: it lands while the prologue works
    auto next_digit = [&](int j) {
        for (j++; j < beta && j == own; j++) {
        }
        return j;
    };
    int jn = next_digit(-1);
    if (jn < beta) ks_dma_rows(ext + (long)jn * exj + (long)bb * exs + woff, ebw, lane);
#pragma unroll
    for (int m = 0; m < 8; m++) {
        const int e = L + 32 * m;
        if (e > 0) {
            const int ml = 1 << (31 - __clz(e));
            tw[e] = W[(long)ml * (R + row) + (e - ml)];
        }
    }
    const long roff = ((long)t << LOGN) + (long)row * 256 + L;
    double a0[8], a1[8];
#pragma unroll
    for (int r = 0; r < 8; r++) a0[r] = a1[r] = 0.0;
    if (PROD && t <= l) {
        const double f = pmodf[t], wv = tw_w(f, q);
        const u64* kp = key + (long)own * kdig + ((long)pid << LOGN) + (long)row * 256 + L;
        const u64* xa = addend.ptr + (long)(bb & addend.bmask) * addend.bs + roff;
        const u64* xb = pb.ptr + (long)(bb & pb.bmask) * pb.bs + roff;
        const u64* xc = pc.ptr ? pc.ptr + (long)(bb & pc.bmask) * pc.bs + roff : xb;
        if (fac)
            ks_prod_prologue<true>(a0, a1, kp, kcomp, xa, addend.ps, xb, pb.ps, xc, pc.ps, pc.ptr != nullptr, wv, f,
                                   (double)fac[3 * t], (double)fac[3 * t + 1], (double)fac[3 * t + 2], q, qi, big);
        else
            ks_prod_prologue<false>(a0, a1, kp, kcomp, xa, addend.ps, xb, pb.ps, xc, pc.ps, false, wv, f, 0.0, 0.0, 0.0,
                                    q, qi, big);
    } else if (!PROD) {
        if (pmodf && t <= l && addend.ptr) {
            const double f = pmodf[t], wv = tw_w(f, q);
            const u64* xa = addend.ptr + (long)bb * addend.bs + roff;
            if (addend.np > 0) {
#pragma unroll
                for (int r = 0; r < 8; r++) a0[r] = fmul_rem(u2d(xa[32 * r]), wv, f, q);
            }
            if (addend.np > 1) {
#pragma unroll
                for (int r = 0; r < 8; r++) a1[r] = fmul_rem(u2d(xa[addend.ps + 32 * r]), wv, f, q);
            }
        }
        if (own >= 0 && own < beta) {  // the own digit's limbs: d itself, already in NTT form
            const u64* kp = key + (long)own * kdig + ((long)pid << LOGN) + (long)row * 256 + L;
            const u64* dp = d + (long)bb * dbs + roff;
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const double v = u2d(dp[32 * r]), kb = u2d(kp[32 * r]), ka = u2d(kp[32 * r + kcomp]);
                a0[r] += fmul_rem(v, kb, kb * qi, q);
                a1[r] += fmul_rem(v, ka, ka * qi, q);
            }
        }
    }
    if (accum) {
        const u64* o0 = acc + (long)bb * abs_ + roff;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            a0[r] = fred(a0[r] + u2d(o0[32 * r]), q, qi);
            a1[r] = fred(a1[r] + u2d(o0[acs + 32 * r]), q, qi);
        }
    } else if (big) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
            a0[r] = fred(a0[r], q, qi);
            a1[r] = fred(a1[r], q, qi);
        }
    }
    wave_lds_sync();  // the row's twiddles (written by its own 32 lanes) before use
    int nsum = 0;
    const long coff = ((long)t << LOGN) + (long)(rb * 8 + 2 * w) * 256;
#pragma unroll 1
    while (jn < beta) {
        const int j = jn;
        ks_dma_wait();  // ext_j is in this wave's staging rows
        double v[8];
#pragma unroll
        for (int r = 0; r < 8; r++) v[r] = er[L + 32 * r];
        ks_lds_reads_done();
        jn = next_digit(j);
        // the next digit's row (or the FIN epilogue's first conv row) streams in during this NTT
        if (jn < beta) ks_dma_rows(ext + (long)jn * exj + (long)bb * exs + woff, ebw, lane);
        else if (FIN) ks_dma_rows(fin.conv + (long)bb * fin.cbs + coff, ebw, lane);
        const u64* kp = key + (long)j * kdig + ((long)pid << LOGN) + (long)row * 256 + L;
        u64 kbw[8], kaw[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            kbw[r] = kp[32 * r];
            kaw[r] = kp[32 * r + kcomp];
        }
        row_ntt8_stages(v, sr, L, 1, tw, q, qi, big);
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const double kb = u2d(kbw[r]), ka = u2d(kaw[r]);
            a0[r] += fmul_rem(v[r], kb, kb * qi, q);
            a1[r] += fmul_rem(v[r], ka, ka * qi, q);
        }
        if (big && (++nsum & 3) == 0) {
#pragma unroll
            for (int r = 0; r < 8; r++) {
                a0[r] = fred(a0[r], q, qi);
                a1[r] = fred(a1[r], q, qi);
            }
        }
    }
    if constexpr (FIN) {
        const double f = fin.dinvf[t], wv = tw_w(f, q);
        if (beta == 0 || next_digit(-1) >= beta)  // no ext digit: conv row 0 not requested yet
            ks_dma_rows(fin.conv + (long)bb * fin.cbs + coff, ebw, lane);
#pragma unroll 1
        for (int c = 0; c < 2; c++) {
            ks_dma_wait();
            double cv[8];
#pragma unroll
            for (int r = 0; r < 8; r++) cv[r] = er[L + 32 * r];
            ks_lds_reads_done();
            if (c == 0) ks_dma_rows(fin.conv + (long)bb * fin.cbs + fin.cps + coff, ebw, lane);
            row_ntt8_stages(cv, sr, L, 1, tw, q, qi, big);
            const u64* ap = fin.add.ptr && c < fin.add.np ? fin.add.ptr + (long)bb * fin.add.bs + (long)c * fin.add.ps + roff
                                                          : nullptr;
            u64* op = fin.out + (long)bb * fin.obs + (long)c * fin.ops + roff;
#pragma unroll
            for (int r = 0; r < 8; r++) {
                double a = c ? a1[r] : a0[r];
                if (big) a = fred(a, q, qi);
                double v = fmul_rem(a - cv[r], wv, f, q);
                if (ap) v += u2d(ap[32 * r]);
                __builtin_nontemporal_store(fcanon(v, q, qi), &op[32 * r]);
            }
        }
        return;
    }
    if constexpr (INV) {
        const double* IW = T.ipsif + ((long)pid << LOGN);
#pragma unroll
        for (int m = 0; m < 8; m++) {
            const int e = L + 32 * m;
            if (e > 0) {
                const int ml = 1 << (31 - __clz(e));
                tw[e] = IW[(long)ml * (R + row) + (e - ml)];
            }
        }
        wave_lds_sync();
        u64* o0 = acc + (long)bb * abs_ + roff;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            double x[8];
#pragma unroll
            for (int r = 0; r < 8; r++) x[r] = fred(c ? a1[r] : a0[r], q, qi);
            row_intt8(x, sr, L, tw, q, qi, big);
#pragma unroll
            for (int r = 0; r < 8; r++) st_d(&o0[(long)c * acs + 32 * r], x[r]);
        }
        return;
    }
    u64* o0 = acc + (long)bb * abs_ + roff;
#pragma unroll
    for (int r = 0; r < 8; r++) {
        __builtin_nontemporal_store(fcanon(a0[r], q, qi), &o0[32 * r]);
        __builtin_nontemporal_store(fcanon(a1[r], q, qi), &o0[acs + 32 * r]);
    }
}

}  // namespace aesfhe
