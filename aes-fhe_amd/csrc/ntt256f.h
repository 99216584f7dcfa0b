// ntt256f.h -- fp64-arithmetic NTT passes for N = 2^16 (= 256 x 256), the BASELINE.json ring.
//
// Same data movement as ntt256.h (register-resident 256-point sub-transforms, 16 lanes x 16
// registers, one LDS transpose per pass), but every residue is carried as an exact integer in
// a double and every butterfly is full-rate fp64 (fmul_rem, kernels.h): ~11 VALU ops instead of
// ~30 mixed integer ops with six quarter-rate 32-bit multiplies.  Twiddles are read as w/q only
// (8 B, Tabs::psif / ipsif) and w = rint(wq * q) is recovered exactly (|wq*q - w| < 2^-4).
//
// Ranges (fmul_rem needs |input| < 2^51, fred needs |x| < 2^53):
//   forward CT   x' = x + v, y' = x - v with v in (-q, q) (table twiddles: column passes, the
//                fused key-switch pass) or (-1.5q, 1.5q) (generated twiddles, tw_row: the
//                standalone row passes): primes < 2^42 grow to at most 9q + 8 * 1.5q = 21q over
//                both passes; larger primes are folded (fred, |x| <= q/2+1) before every second
//                stage (fmul_rem inputs <= 2q).
//   inverse GS   x' = x + y doubles per stage, y' = (x - y) w in (-1.5q, 1.5q): primes < 2^42
//                reach at most 2^8 q per pass (the column pass starts folded); for larger primes
//                the sum output is folded in every butterfly (inputs <= q, differences <= 2.5q).
// The branch on the prime size is block-uniform (one prime per block).  Between the two passes
// of a transform the intermediate is stored as raw doubles; final outputs are canonical u64
// residues in [0, q), so results are identical to ntt256.h and to the oracle residue for residue.
#pragma once
#include <type_traits>

#include "kernels.h"

namespace aesfhe {

// kBigPrime (2^42): defined in kernels.h

__device__ __forceinline__ void ct_f(double& x, double& y, double wq, double q) {
    const double v = fmul_rem(y, tw_w(wq, q), wq, q);
    const double t = x;
    x = t + v;
    y = t - v;
}
template <bool FOLD>
__device__ __forceinline__ void gs_f(double& x, double& y, double wq, double q, double qi) {
    const double s = x + y, d = x - y;
    x = FOLD ? fred(s, q, qi) : s;
    y = fmul_rem(d, tw_w(wq, q), wq, q);
}
// CT / GS butterflies with an on-the-fly twiddle (w exact, |w| < q; wq = w * (1/q) rounded
// twice, so fmul_rem's remainder is within 1.5q instead of q)
__device__ __forceinline__ void ct_fw(double& x, double& y, double w, double wq, double q) {
    const double v = fmul_rem(y, w, wq, q);
    const double t = x;
    x = t + v;
    y = t - v;
}
template <bool FOLD>
__device__ __forceinline__ void gs_fw(double& x, double& y, double w, double wq, double q, double qi) {
    const double s = x + y, d = x - y;
    x = FOLD ? fred(s, q, qi) : s;
    y = fmul_rem(d, w, wq, q);
}
// Row-pass twiddles without the N-entry table walk.  The row pass's stage with group size
// ml = 2^s (m = 256 ml) uses psi^{brv(m + i)}, i = ml * row + j (j < ml); the three bit fields
// of m + i are disjoint, so brv is additive and
//     psi^{brv(256 ml + ml row + j)} = psi^{brv(256 ml + j)} * psi^{brv(row << s)}
// = (a table entry shared by every row: 255 per prime, cache-resident) x (a per-row factor,
// Tabs::rtwf[pid][row][s]).  Walking the N-entry table instead reads as many bytes as the limb
// (the row passes' reads are 1.5-1.9x their writes): the standalone row passes run 5-16 %
// faster generated (tools/ntt_q_bench.hip: 87.6 vs 104 us over 468 limbs), at +1 modular
// product per twiddle.
__device__ __forceinline__ void tw_row(const double* W, int idx, double rq, double q, double qi,
                                       double& w, double& wq) {
    w = fmul_rem(tw_w(W[idx], q), tw_w(rq, q), rq, q);
    wq = w * qi;
}
__device__ __forceinline__ double ld_d(const u64* p) { return __longlong_as_double((long long)*p); }
// raw-double intermediates between NTT passes are streamed (nontemporal): one pass writes far more
// than the caches hold before the next pass reads it back
__device__ __forceinline__ void st_d(u64* p, double v) { __builtin_nontemporal_store((u64)__double_as_longlong(v), p); }

constexpr int kPadF = 17;  // LDS row stride (8 B words) of the 16 x 16 transpose tiles

// Row passes: a row and its LDS tile belong to 16 lanes of one wave (lane (b, rl) = (tid & 15,
// tid >> 4): wave w holds rows 4w .. 4w + 3), and the coalesced copy-in / copy-out below move
// only the wave's own 4 rows, so the exchanges need wave-level ordering, not a workgroup barrier
// (LDS instructions of a wave complete in issue order; the fences and the wave barrier keep the
// compiler from moving accesses across).
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Forward, column pass: the first log2(R) stages on columns of stride 256 (R = N / 256 rows:
// 256 for N = 2^16, 512 for N = 2^17); canonical u64 in, raw doubles out.  Workgroup = 16
// columns [c0, c0+16); lane (cl, b) = (tid & 15, tid >> 4).  R = 512: the first stage (distance
// 256 rows) pairs the two 256-row halves in registers; each half is then an independent
// 256-point column transform whose stage-m twiddles sit at m (2 + h) + group (half h, group
// within the half), so the R = 256 code runs on each half with the index multiplier 2 + h.
// (the body takes the 16-column block bx of span limb by and LDS s[256 * kPadF], twq[R]; a
// caller that loops over blocks separates them with a workgroup barrier)
// SPREAD (the rescale's spread in the copy-in, engine.hip rescale_view): limb y = (p, i) of dst
// is not read from a span but formed from poly p's dropped top limb x[p] (canonical mod q_l, INTT
// form): centered(x) mod q_i, canonical -- the residues k_rescale_spread wrote, so the pass's
// output is unchanged while the spread's l-limb write + read-back is gone (x[p] is read once per
// target limb, the same 16-column strip by the same XCD each time: bx's XCD is fixed).  SPREAD 2:
// x is first multiplied by the level-down constant sc mod q_l (scf = sc / q_l).  SPREAD 3: x mod
// q_i without centring -- the ModUp of a one-limb key-switch digit (k_modup<1>: hat = hatinv = 1).
// x of poly p at x + p * xs.
struct SpreadSrc {
    const u64* x;
    long xs;
    u64 ql, sc;
    double scf;
};
template <int R, int SPREAD = 0>
__device__ __forceinline__ void nttf_fwd_cols_body(const Span& src, const Span& dst, const Tabs& T, int bx, int by,
                                                   double* s, double* twq, const SpreadSrc& ss = SpreadSrc{}) {
    static_assert(R == 256 || R == 512, "rows of 256: N = 2^16 or 2^17");
    constexpr int H = R / 256;
    int pid;
    const u64* in = SPREAD ? ss.x + (long)(by / dst.nl) * ss.xs : span_ptr(src, by, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, by, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, cl = tid & 15, b = tid >> 4;
    const int c = bx * 16 + cl;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* tg = T.psif + ((long)pid << T.logN);
    const double* cw = T.cw + (long)pid * kColW;
#pragma unroll
    for (int h = 0; h < H; h++) twq[tid + 256 * h] = tg[tid + 256 * h];
    double x[16 * H];
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
        for (int a = 0; a < 16; a++) {
            const u64 v = in[(h * 256 + a * 16 + b) * 256 + c];
            if constexpr (SPREAD == 0) {
                x[16 * h + a] = u2d(v);
            } else {
                const u64 w = SPREAD == 2 ? mul_w(v, ss.sc, ss.scf, ss.ql) : v;
                double d = u2d(w) - (SPREAD != 3 && w > (ss.ql >> 1) ? (double)ss.ql : 0.0);  // centered, exact
                d = fred(d, q, qi);
                x[16 * h + a] = d < 0.0 ? d + q : d;
            }
        }
    __syncthreads();
    if (H == 2) {  // stage m = 1 across the halves: canonical in, (-q, 2q) out
        const double w = cw[1], wq = tg[1];
#pragma unroll
        for (int a = 0; a < 16; a++) ct_fw(x[a], x[16 + a], w, wq, q);
    }
#pragma unroll
    for (int h = 0; h < H; h++) {
        double* xh = x + 16 * h;
        const int mul = H == 1 ? 1 : 2 + h;
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const int m = 1 << st, hh = 8 >> st;
            if (big && (H == 1 ? st == 2 : (st & 1) == 0)) {
#pragma unroll
                for (int a = 0; a < 16; a++) xh[a] = fred(xh[a], q, qi);
            }
#pragma unroll
            for (int a = 0; a < 16; a++) {
                if (a & hh) continue;
                const int ti = m * mul + (a >> (4 - st));  // uniform: scalar loads of w and w/q
                ct_fw(xh[a], xh[a + hh], cw[ti], tg[ti], q);
            }
        }
        if (h > 0) __syncthreads();  // the previous half's LDS reads are done
#pragma unroll
        for (int a = 0; a < 16; a++) s[(a * 16 + b) * kPadF + cl] = xh[a];
        __syncthreads();
        const int ap = b;
#pragma unroll
        for (int bb = 0; bb < 16; bb++) xh[bb] = s[(ap * 16 + bb) * kPadF + cl];
#pragma unroll
        for (int st = 4; st < 8; st++) {
            const int m = 1 << st, hh = 128 >> st;
            if (big && (st & 1) == 0) {
#pragma unroll
                for (int bb = 0; bb < 16; bb++) xh[bb] = fred(xh[bb], q, qi);
            }
#pragma unroll
            for (int bb = 0; bb < 16; bb++) {
                if (bb & hh) continue;
                ct_f(xh[bb], xh[bb + hh], twq[m * mul + ap * (m >> 4) + (bb >> (8 - st))], q);
            }
        }
#pragma unroll
        for (int bb = 0; bb < 16; bb++) st_d(&out[(h * 256 + ap * 16 + bb) * 256 + c], xh[bb]);
    }
}
template <int R = 256>
__global__ __launch_bounds__(256) void k_nttf_fwd_cols(Span src, Span dst, Tabs T) {
    __shared__ double s[256 * kPadF];
    __shared__ double twq[R];
    nttf_fwd_cols_body<R>(src, dst, T, blockIdx.x, blockIdx.y, s, twq);
}
template <int R, int SPREAD>
__global__ __launch_bounds__(256) void k_nttf_fwd_cols_spread(SpreadSrc ss, Span dst, Tabs T) {
    __shared__ double s[256 * kPadF];
    __shared__ double twq[R];
    nttf_fwd_cols_body<R, SPREAD>(dst, dst, T, blockIdx.x, blockIdx.y, s, twq, ss);
}

// ModDown finish fused into the row pass of the conv NTT (key switch): limb y of
// the span is (batch b, component c, limb i) = (y / nl / 2, y / nl % 2, y % nl) and the pass
// writes out[b][c][i] = (acc[b][c][i] - conv) * D^{-1} (+ addend) instead of conv itself.
struct RowFin {
    const u64* acc;
    long abs_, acs;
    Opnd2 addend;
    u64* out;
    long obs, ops;
    const double* dinvf;
    int nl;
    // optional per-limb constant on acc (w/q): out = (C_i acc - conv) D^{-1} -- the exact-scale
    // level-down folded into a rescale (engine.hip rescale_view)
    const double* cf;
};

// The forward row pass's 8 stages on the 16 rows of one workgroup: lane (b, rl) loads row
// row = r0 + rl from rp (raw doubles, stride-16 gather), 4 stages in registers, LDS transpose
// through sr = s + rl * 16 * kPadF, 4 stages.  On return lane ap = b holds elements
// ap * 16 + bb (bb = 0..15) of its row, lazily reduced (ranges: file header).
__device__ __forceinline__ void row_ntt_load(double (&x)[16], const u64* rp, int b) {
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = ld_d(&rp[a * 16 + b]);
}
// the 8 stages on x as loaded by row_ntt_load (the split lets a caller issue its own epilogue
// loads between the two, behind the row's loads)
template <int RR>
__device__ __forceinline__ void row_ntt_fwd_stages(double (&x)[16], double* sr, int b, int row,
                                                   const double* W, const double* R, double q, double qi,
                                                   bool big) {
#pragma unroll
    for (int st = 0; st < 4; st++) {
        const int ml = 1 << st, h = 8 >> st;
        if (big && (st & 1) == 0) {
#pragma unroll
            for (int a = 0; a < 16; a++) x[a] = fred(x[a], q, qi);
        }
        const double rq = R[st];
#pragma unroll
        for (int j = 0; j < ml; j++) {  // butterflies of twiddle j: a = j * 2h + k, k < h
            double w, wq;
            tw_row(W, RR * ml + j, rq, q, qi, w, wq);
#pragma unroll
            for (int k = 0; k < h; k++) ct_fw(x[j * 2 * h + k], x[j * 2 * h + k + h], w, wq, q);
        }
    }
#pragma unroll
    for (int a = 0; a < 16; a++) sr[a * kPadF + b] = x[a];
    wave_sync_lds();
    const int ap = b;
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = sr[ap * kPadF + bb];
#pragma unroll
    for (int st = 4; st < 8; st++) {
        const int ml = 1 << st, h = 128 >> st, nj = ml >> 4;
        if (big && (st & 1) == 0) {
#pragma unroll
            for (int bb = 0; bb < 16; bb++) x[bb] = fred(x[bb], q, qi);
        }
        const double rq = R[st];
#pragma unroll
        for (int j = 0; j < nj; j++) {  // bb = j * 2h + k, k < h
            double w, wq;
            tw_row(W, RR * ml + ap * nj + j, rq, q, qi, w, wq);
#pragma unroll
            for (int k = 0; k < h; k++) ct_fw(x[j * 2 * h + k], x[j * 2 * h + k + h], w, wq, q);
        }
    }
}
template <int RR>
__device__ __forceinline__ void row_ntt_fwd(double (&x)[16], const u64* rp, double* sr, int b, int row,
                                            const double* W, const double* R, double q, double qi,
                                            bool big) {
    row_ntt_load(x, rp, b);
    row_ntt_fwd_stages<RR>(x, sr, b, row, W, R, q, qi, big);
}
// element e = k * 256 + tid (k = 0..15) of the workgroup's 16 x 256 tile, as stored by lane
// (ap, rl) at sr[ap * kPadF + bb]: the coalesced read-out order of the row passes
__device__ __forceinline__ int row_tile_idx(int e) {
    const int r = e >> 8, cc = e & 255;
    return r * 16 * kPadF + (cc >> 4) * kPadF + (cc & 15);
}

// Forward, row pass: stages m = 256..32768 within rows of 256 contiguous elements; raw doubles
// in, canonical u64 out (FIN: the ModDown finish above).  Workgroup = 16 rows [r0, r0+16);
// lane (b, rl) = (tid & 15, tid >> 4).
// (body: the 16-row block bx of span limb by, LDS s[16 * 16 * kPadF])
template <bool FIN, int R>
__device__ __forceinline__ void nttf_fwd_rows_body(const Span& dst, const Tabs& T, const RowFin& fin, int bx, int by,
                                                   double* s) {
    int pid;
    u64* io = span_ptr(dst, by, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, b = tid & 15, rl = tid >> 4;
    const int row = bx * 16 + rl;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* W = T.psif + ((long)pid << T.logN);
    const double* Rf = T.rtwf + (long)pid * R * 8 + row * 8;
    double x[16];
    double* sr = s + rl * 16 * kPadF;
    const int ap = b;
    // wave w stores its rows 4w .. 4w + 3: element e = 1024 w + 64 k + lane of the 16 x 256 tile
    const int e0 = (tid >> 6) * 1024 + (tid & 63);
    row_ntt_load(x, io + (long)row * 256, b);
    // FIN: the accumulator words of this lane's output elements are requested right behind the
    // row's loads, so they arrive while the row transform computes
    u64 accw[FIN ? 16 : 1];
    if (FIN) {
        const int p = by / fin.nl, i = by - p * fin.nl;
        const u64* apf = fin.acc + (long)(p >> 1) * fin.abs_ + (long)(p & 1) * fin.acs + ((long)i << T.logN) +
                         (long)bx * 16 * 256;
#pragma unroll
        for (int k = 0; k < (FIN ? 16 : 1); k++) accw[k] = apf[e0 + 64 * k];
    }
    row_ntt_fwd_stages<R>(x, sr, b, row, W, Rf, q, qi, big);
    // coalesced store through LDS: canonical residues, then row-major copy-out
#pragma unroll
    for (int bb = 0; bb < 16; bb++) sr[ap * kPadF + bb] = __longlong_as_double((long long)fcanon(x[bb], q, qi));
    wave_sync_lds();
    if (!FIN) {
        u64* base = io + (long)bx * 16 * 256;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int e = e0 + 64 * k;
            __builtin_nontemporal_store((u64)__double_as_longlong(s[row_tile_idx(e)]), &base[e]);
        }
    } else {
        const int y = by, p = y / fin.nl, i = y - p * fin.nl, bb = p >> 1, c = p & 1;
        const long off = ((long)i << T.logN) + (long)bx * 16 * 256;
        const u64* dp = fin.addend.ptr && c < fin.addend.np ? fin.addend.ptr + (long)bb * fin.addend.bs + (long)c * fin.addend.ps + off : nullptr;
        u64* op = fin.out + (long)bb * fin.obs + (long)c * fin.ops + off;
        const double f = fin.dinvf[i], w = tw_w(f, q);
        const double cf = fin.cf ? fin.cf[i] : 0.0, cw = fin.cf ? tw_w(cf, q) : 0.0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int e = e0 + 64 * k;
            const double conv = u2d((u64)__double_as_longlong(s[row_tile_idx(e)]));
            double a = u2d(accw[FIN ? k : 0]);
            if (fin.cf) a = fmul_rem(a, cw, cf, q);  // block-uniform
            double v = fmul_rem(a - conv, w, f, q);
            if (dp) v += u2d(dp[e]);
            __builtin_nontemporal_store(fcanon(v, q, qi), &op[e]);  // streaming
        }
    }
}
template <bool FIN, int R = 256>
__global__ __launch_bounds__(256) void k_nttf_fwd_rows_t(Span dst, Tabs T, RowFin fin) {
    __shared__ double s[16 * 16 * kPadF];
    nttf_fwd_rows_body<FIN, R>(dst, T, fin, blockIdx.x, blockIdx.y, s);
}

// Inverse, row pass (Gentleman-Sande, distances 1..128 within rows): canonical u64 in (src),
// raw doubles out (dst).  PROD: the input is the product src (x) src2 mod q of two canonical
// operands (the d2 = a1 b1 term of a ciphertext product, computed here instead of being written
// by a tensor kernel and read back; src2 has src's shape).
// FMA (with PROD): fac holds the per-prime {alpha, C, K} of a fused multiply-add (aesfhe_mul_fma)
// and the product is alpha (src (x) src2).
template <int RR = 256, bool PROD = false, bool FMA = false>
__global__ __launch_bounds__(256, 4) void k_nttf_inv_rows(Span src, Span dst, Tabs T, Span src2,
                                                          const u64* __restrict__ fac) {
    __shared__ double s[16 * 16 * kPadF];
    int pid;
    const u64* in = span_ptr(src, blockIdx.y, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, b = tid & 15, rl = tid >> 4;
    const int row = blockIdx.x * 16 + rl;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* W = T.ipsif + ((long)pid << T.logN);
    const u64* gb = in + (long)blockIdx.x * 16 * 256;
    {  // wave w loads its rows 4w .. 4w + 3 (coalesced), element e = 1024 w + 64 k + lane
        const int e0 = (tid >> 6) * 1024 + (tid & 63);
        if (PROD) {
            int pid2;
            const u64* gb2 = span_ptr(src2, blockIdx.y, T.logN, T.Lp1, pid2) + (long)blockIdx.x * 16 * 256;
            const double al = FMA ? (double)fac[3 * pid] : 0.0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int e = e0 + 64 * k;
                const double y = u2d(gb2[e]);
                double v = fmul_rem(u2d(gb[e]), y, y * qi, q);
                if (FMA) v = fmul_rem(v, al, al * qi, q);
                s[row_tile_idx(e)] = u2d(fcanon(v, q, qi));
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int e = e0 + 64 * k;
                s[row_tile_idx(e)] = u2d(gb[e]);
            }
        }
    }
    wave_sync_lds();
    double* sr = s + rl * 16 * kPadF;
    const int ap = b;
    double x[16];
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = sr[ap * kPadF + bb];
    const double* R = T.irtwf + (long)pid * RR * 8 + row * 8;
    auto stages_lo = [&](auto fold) {
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const int t = 1 << st, ml = 128 / t, nj = 8 / t;  // group size ml = 2^(7 - st)
            const double rq = R[7 - st];
#pragma unroll
            for (int j = 0; j < nj; j++) {  // butterflies of twiddle j: bb = j * 2t + k, k < t
                double w, wq;
                tw_row(W, RR * ml + ap * nj + j, rq, q, qi, w, wq);
#pragma unroll
                for (int k = 0; k < t; k++)
                    gs_fw<decltype(fold)::value>(x[j * 2 * t + k], x[j * 2 * t + k + t], w, wq, q, qi);
            }
        }
    };
    if (big) stages_lo(std::true_type{});
    else stages_lo(std::false_type{});
#pragma unroll
    for (int bb = 0; bb < 16; bb++) sr[ap * kPadF + bb] = x[bb];
    wave_sync_lds();
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = sr[a * kPadF + b];
    auto stages_hi = [&](auto fold) {
#pragma unroll
        for (int st = 4; st < 8; st++) {
            const int t = 1 << st, ta = t >> 4, ml = 128 / t;
            const double rq = R[7 - st];
#pragma unroll
            for (int j = 0; j < ml; j++) {  // a = j * 2ta + k, k < ta
                double w, wq;
                tw_row(W, RR * ml + j, rq, q, qi, w, wq);
#pragma unroll
                for (int k = 0; k < ta; k++)
                    gs_fw<decltype(fold)::value>(x[j * 2 * ta + k], x[j * 2 * ta + k + ta], w, wq, q, qi);
            }
        }
    };
    if (big) stages_hi(std::true_type{});
    else stages_hi(std::false_type{});
    u64* op = out + (long)row * 256;
#pragma unroll
    for (int a = 0; a < 16; a++) st_d(&op[a * 16 + b], x[a]);
}

// Inverse, column pass (distances 256..32768 = rows 1..128 of each 256-row half) and the N^{-1}
// scaling: raw doubles in, canonical u64 out.  R = 512 (N = 2^17): both halves run the R = 256
// stages (twiddle index multiplier 2 + h, as in the forward pass), stay in registers, and the
// last stage (distance 256 rows) pairs them before the scaling.
// LF (round 6): the final N^{-1} scaling is a per-limb factor lf[limb index within the span] (w/q)
// instead -- the key switch's INTT folds the digit's qhat^{-1} into it (engine.hip ks_modup), so
// the fused ModUp (bconv_cols.h YIN) reads y directly
template <int R = 256, bool LF = false>
__global__ __launch_bounds__(256) void k_nttf_inv_cols(Span dst, Tabs T, const double* __restrict__ lf) {
    static_assert(R == 256 || R == 512, "rows of 256: N = 2^16 or 2^17");
    constexpr int H = R / 256;
    __shared__ double s[256 * kPadF];
    __shared__ double twq[R];
    int pid;
    u64* io = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, cl = tid & 15, b = tid >> 4;
    const int c = blockIdx.x * 16 + cl;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* tg = T.ipsif + ((long)pid << T.logN);
    const double* icw = T.icw + (long)pid * kColW;
#pragma unroll
    for (int h = 0; h < H; h++) twq[tid + 256 * h] = tg[tid + 256 * h];
    const int ap = b;
    double x[16 * H];
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
        for (int bb = 0; bb < 16; bb++) x[16 * h + bb] = fred(ld_d(&io[(h * 256 + ap * 16 + bb) * 256 + c]), q, qi);
    __syncthreads();
#pragma unroll
    for (int h = 0; h < H; h++) {
        double* xh = x + 16 * h;
        const int mul = H == 1 ? 1 : 2 + h;
        auto stages_lo = [&](auto fold) {
#pragma unroll
            for (int st = 0; st < 4; st++) {
                const int tr = 1 << st;
                const int base = (128 / tr) * mul + ap * (8 / tr);
#pragma unroll
                for (int bb = 0; bb < 16; bb++) {
                    if (bb & tr) continue;
                    gs_f<decltype(fold)::value>(xh[bb], xh[bb + tr], twq[base + (bb >> (st + 1))], q, qi);
                }
            }
        };
        if (big) stages_lo(std::true_type{});
        else stages_lo(std::false_type{});
        if (h > 0) __syncthreads();  // the previous half's LDS reads are done
#pragma unroll
        for (int bb = 0; bb < 16; bb++) s[(ap * 16 + bb) * kPadF + cl] = xh[bb];
        __syncthreads();
#pragma unroll
        for (int a = 0; a < 16; a++) xh[a] = s[(a * 16 + b) * kPadF + cl];
        auto stages_hi = [&](auto fold) {
#pragma unroll
            for (int st = 4; st < 8; st++) {
                const int tr = 1 << st, ta = tr >> 4;
                const int base = (128 / tr) * mul;
#pragma unroll
                for (int a = 0; a < 16; a++) {
                    if (a & ta) continue;
                    const int ti = base + (a >> (st - 3));  // uniform: scalar loads of w and w/q
                    gs_fw<decltype(fold)::value>(xh[a], xh[a + ta], icw[ti], tg[ti], q, qi);
                }
            }
        };
        if (big) stages_hi(std::true_type{});
        else stages_hi(std::false_type{});
    }
    if (H == 2) {  // stage m = 1 across the halves (inputs folded to |x| <= q/2 + 1)
        const double w = icw[1], wq = tg[1];
#pragma unroll
        for (int a = 0; a < 16; a++) {
            x[a] = fred(x[a], q, qi);
            x[16 + a] = fred(x[16 + a], q, qi);
            gs_fw<false>(x[a], x[16 + a], w, wq, q, qi);
        }
    }
    const double nif = LF ? lf[blockIdx.y % dst.nl] : T.ninvf[pid];
    const double ni = LF ? tw_w(nif, q) : (double)T.ninv[pid];
#pragma unroll
    for (int h = 0; h < H; h++)
#pragma unroll
        for (int a = 0; a < 16; a++) {
            const double r = fred(x[16 * h + a], q, qi);
            __builtin_nontemporal_store(fcanon(fmul_rem(r, ni, nif, q), q, qi), &io[(h * 256 + a * 16 + b) * 256 + c]);
        }
}


}  // namespace aesfhe
