// ks_fused.h -- key-switch inner product fused into the row pass of the ext NTT (N = 2^16).
//
// The unfused key switch (engine.hip ks_modup / ks_apply) writes every extended limb ext[j][b][t]
// in canonical NTT form (row pass) and reads it straight back in k_ks_inner_all:
// 2 * beta * B * (l + 1 + K) limbs of HBM traffic per call, the largest single item of a key
// switch.  Here ks_modup stops after the column pass (the raw-double intermediate stays in the
// ext buffer) and one workgroup per (target limb t, 16-row block, batch element b) runs the row
// pass of ext[j][b][t] for every digit j in registers, multiplies by the key digit and
// accumulates, writing only the two accumulators acc[b][0/1][t] (accum: added to what acc holds)
// -- the same canonical values k_ks_inner_all produces (the arithmetic is exact mod q; only the lazy ranges differ).
//
// Ranges: row_ntt_fwd leaves |x| <= 17q for q < 2^42 (folded to q/2 + 1 for larger primes
// before the product); fmul_rem(x, key) lies in (-1.5q, 1.5q) (on-the-fly key quotient), so the
// beta <= 12 products sum below 18q < 2^47 for small primes; big primes fold every 4 digits.
#pragma once
#include "kernels_ops.h"
#include "ntt256f.h"

namespace aesfhe {

// grid: 8 * B * (ne * 16 / 8) blocks of 256; block id -> (xcd group x = id & 7, b, pair), pair =
// (t, row block): all B batch elements of one (t, row block) are dealt to one XCD (blocks
// x, x + 8, ...) so the key rows they share are L2 hits.
__global__ __launch_bounds__(256) void k_nttf_rows_ks(const u64* __restrict__ d, long dbs,
                                                      const u64* __restrict__ ext, long exs, long exj,
                                                      const u64* __restrict__ key, long kdig, long kcomp,
                                                      u64* __restrict__ acc, long abs_, long acs, int B,
                                                      int beta, int K, int l, int ne, Tabs T, Opnd addend,
                                                      const double* __restrict__ pmodf, int accum) {
    __shared__ double s[16 * 16 * kPadF];
    const int id = blockIdx.x, x8 = id & 7, rest = id >> 3;
    const int bb = rest % B, pair = (rest / B) * 8 + x8;
    const int t = pair >> 4, rb = pair & 15;
    if (t >= ne) return;
    const int pid = t <= l ? t : T.Lp1 + (t - l - 1);
    const int own = t <= l ? t / K : -1;  // the digit whose limbs include t (Q limbs only)
    const int tid = threadIdx.x, b = tid & 15, rl = tid >> 4;
    const int row = rb * 16 + rl;
    const double q = (double)T.q[pid], qi = T.qinv[pid];
    const bool big = q >= kBigPrime;
    const double* W = T.psif + ((long)pid << 16);
    double* sr = s + rl * 16 * kPadF;
    const long toff = ((long)t << 16) + (long)rb * 4096;  // this block's tile within a limb
    double a0[16], a1[16];
#pragma unroll
    for (int k = 0; k < 16; k++) a0[k] = a1[k] = 0.0;
#pragma unroll 1
    for (int j = 0; j < beta; j++) {
        double v[16];
        if (j == own) {  // the digit's own limbs: d itself, already in NTT form
            const u64* dp = d + (long)bb * dbs + toff;
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = u2d(dp[k * 256 + tid]);
        } else {
            double x[16];
            row_ntt_fwd(x, ext + (long)j * exj + (long)bb * exs + ((long)t << 16) + (long)row * 256, sr, b, row,
                        W, q, qi, big);
            __syncthreads();  // every lane has read its transposed column out of s
#pragma unroll
            for (int k = 0; k < 16; k++) sr[b * kPadF + k] = big ? fred(x[k], q, qi) : x[k];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 16; k++) v[k] = s[row_tile_idx(k * 256 + tid)];
            __syncthreads();  // s is rewritten by the next digit's transpose
        }
        const u64* kp = key + (long)j * kdig + ((long)pid << 16) + (long)rb * 4096;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int e = k * 256 + tid;
            const double kb = u2d(kp[e]), ka = u2d(kp[e + kcomp]);
            a0[k] += fmul_rem(v[k], kb, kb * qi, q);
            a1[k] += fmul_rem(v[k], ka, ka * qi, q);
        }
        if (big && (j & 3) == 3) {
#pragma unroll
            for (int k = 0; k < 16; k++) {
                a0[k] = fred(a0[k], q, qi);
                a1[k] = fred(a1[k], q, qi);
            }
        }
    }
    u64* o0 = acc + (long)bb * abs_ + toff;
    if (pmodf && t <= l) {
        const double f = pmodf[t], w = tw_w(f, q);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int e = k * 256 + tid, kk = rb * 4096 + e;
            a0[k] = fred(a0[k], q, qi) + fmul_rem(u2d(opnd_get(addend, bb, 0, t, kk, 16)), w, f, q);
            a1[k] = fred(a1[k], q, qi) + fmul_rem(u2d(opnd_get(addend, bb, 1, t, kk, 16)), w, f, q);
        }
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int e = k * 256 + tid;
        const double p0 = accum ? u2d(o0[e]) : 0.0, p1 = accum ? u2d(o0[acs + e]) : 0.0;
        o0[e] = fcanon(a0[k] + p0, q, qi);
        o0[acs + e] = fcanon(a1[k] + p1, q, qi);
    }
}

}  // namespace aesfhe
