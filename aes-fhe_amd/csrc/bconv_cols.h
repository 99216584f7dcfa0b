// bconv_cols.h -- base conversion on the matrix cores fused with the forward NTT column pass
// (N = 2^16).  VERDICT r5 item 1: k_bconv_mfma wrote every extension limb and k_nttf_fwd_cols read
// it back one launch later (together ~34 % of the round); here the extension limb never reaches
// HBM in coefficient form.
//
// A workgroup owns one 16-column strip (16 columns x 256 rows = 4096 coefficients) of one batch
// element and one tile of 4 targets.  For each of the 16 row groups a (rows 16 a + b, b = tid >> 4)
// every wave converts its 64 coefficients -- exactly the coefficients its lanes hold in the column
// pass's register layout (lane (cl, b) = (tid & 15, tid >> 4) holds rows 16 a + b of column
// 16 bx + cl) -- with the k_bconv_mfma arithmetic (i8 byte planes, v_mfma_i32_32x32x32_i8, one
// permlane32_swap per target pair: bconv_mfma.h), so after the 16 row groups each lane holds its
// column tile of all 4 targets in registers (xv[4][16], 128 VGPRs) and runs the column pass's 8
// stages on each (ntt256f.h nttf_fwd_cols_body, R = 256) with one LDS transpose per target (two
// LDS tiles alternate: one workgroup barrier per target).  Output: the column pass's raw-double
// intermediate, as k_nttf_fwd_cols writes it; the key-switch row kernels read it unchanged.
//
// The conversion output enters the butterflies folded (fred: |x| <= q/2 + 1) instead of canonical:
// the column stages' growth bound (ntt256f.h header: 9q from canonical inputs) holds with margin,
// and the final canonical residues of the row pass are unchanged (every step is exact mod q).
//
// YIN: the sources are already y_i = [x_i qhat_i^{-1}]_{q_i} (the INTT that produced them folded
// qhat^{-1} into its N^{-1} scaling, engine.hip ks_modup), so the B operand is the loaded word.
// VC (ModDown's exact conversion): v = rint(sum_j y_j (1/e_j)), j in order (fp64,
// the oracle's sum), rides in slot ns as in k_bconv_mfma.  One permlane32_swap per slot pair gives
// every lane all slots of its own coefficient (group h of lane half h), so each lane forms one v;
// one more swap hands the other group's v to the lane half that holds slot ns.
// Source words: the ntile workgroups of one (strip, element) unit are dealt to one XCD back to back
// (block id = ((u / 8) ntile + tile) 8 + u % 8), so the unit's 4096 x ns source words come from HBM
// once and from that XCD's L2 for the other tiles.
#pragma once
#include "bconv_mfma.h"
#include "ntt256f.h"

namespace aesfhe {

// the 8 forward column stages (R = 256) of the register tile x (x[a] = row 16 a + b of column c),
// transposed through the LDS tile s (all 256 threads of the workgroup; s must not be read by any
// thread from an earlier use -- the caller's barrier discipline), twiddles: stages 0-3 from the
// prime's tables tg (w / q) and cw (w, Tabs::cw) -- uniform: scalar loads, no w = rint(wq q) on the
// VALU --, 4-7 from the LDS copy twq of w / q; raw doubles stored to out
__device__ __forceinline__ void cols256_stages_store(double (&x)[16], double q, double qi, bool big, const double* tg,
                                                     const double* cw, const double* twq, double* s, u64* out, int b,
                                                     int cl, int c) {
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
            const int ti = m + (a >> (4 - st));
            ct_fw(x[a], x[a + hh], cw[ti], tg[ti], q);
        }
    }
#pragma unroll
    for (int a = 0; a < 16; a++) s[(a * 16 + b) * kPadF + cl] = x[a];
    __syncthreads();
    const int ap = b;
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = s[(ap * 16 + bb) * kPadF + cl];
#pragma unroll
    for (int st = 4; st < 8; st++) {
        const int m = 1 << st, hh = 128 >> st;
        if (big && (st & 1) == 0) {
#pragma unroll
            for (int bb = 0; bb < 16; bb++) x[bb] = fred(x[bb], q, qi);
        }
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {
            if (bb & hh) continue;
            ct_f(x[bb], x[bb + hh], twq[m + ap * (m >> 4) + (bb >> (8 - st))], q);
        }
    }
#pragma unroll
    for (int bb = 0; bb < 16; bb++) st_d(&out[(ap * 16 + bb) * 256 + c], x[bb]);
}

// grid: 16 * nz * ntile workgroups (1-D, XCD-aware order above), 256 threads; nz = batch * nc
// (a.nc components per element), ntile = ceil(nt / 4); 16 * nz must be a multiple of 8.
// PF: row groups of source words in flight ahead of the one being converted (register prefetch;
// 0 = load at use).  TT: targets per workgroup (4, or 2: the MFMA's other two target rows are
// dummies -- half the registers for the column tiles, twice the workgroups and source reads);
// LT: LDS transpose tiles (2 alternate with one barrier per target; 1 needs a second barrier
// before each reuse, for a smaller LDS footprint).  (Two targets' column stages interleaved -- PAIR,
// round 6 -- measured slower and were removed: DESIGN 4.8.)
// MODE (dev decomposition, tools/modup_fused_bench.hip; the engine runs 0): 1 = the conversion
// alone (the column stages skipped, xv stored as is), 2 = the column stages alone (loads kept, the
// MFMAs and their epilogue skipped)
template <int NSTEP, bool YIN, bool VC = false, int PF = 1, int TT = 4, int LT = 2, int MODE = 0>
__global__ __launch_bounds__(256, TT == 4 ? 2 : 3) void k_bconv_cols(BconvArgs a, Tabs T, int ntile) {
    static_assert(TT == 4 || TT == 2, "4 or 2 targets per workgroup");
    static_assert(LT == 1 || LT == 2, "1 or 2 LDS tiles");
    __shared__ double s[LT][256 * kPadF];
    __shared__ double twq[TT][256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
    const int cl = tid & 15, b = tid >> 4;
    const int id = blockIdx.x, x8 = id & 7, j = id >> 3;
    const int tile = j % ntile, u = (j / ntile) * 8 + x8;
    const int bx = u & 15, z = u >> 4, zb = z / a.nc, zc = z - zb * a.nc;
    const int logN = T.logN;
    const u64* src = a.src + (long)zb * a.sbs + (long)zc * a.scs;
    u64* dst = a.dst + (long)zb * a.dbs + (long)zc * a.dcs;
    auto limb_of = [&](int tau) { return tau < a.skip0 ? tau : tau + a.skipn; };
    auto pid_of = [&](int tl) { return tl <= a.tl_l ? tl : a.Lp1 + tl - a.tl_l - 1; };
    const int tau0 = TT * tile;
    const int nlive = min(TT, a.nt - tau0);
    // the tile's stage 4-7 twiddles into LDS (read after the first barrier of the column stages)
#pragma unroll
    for (int m = 0; m < TT; m++)
        if (m < nlive) twq[m][tid] = T.psif[((long)pid_of(limb_of(tau0 + m)) << logN) + tid];
    // A fragments of the tile (row r = (target r >> 3, byte plane (r & 3) + 4 ((r >> 2) & 1))),
    // fixed for the whole workgroup
    bc_v4i af[NSTEP];
    {
        const int row = lane & 31, ta = row >> 3, pb = (row & 3) + 4 * ((row >> 2) & 1);
        const int tau = tau0 + ta;  // TT = 2: rows of ta >= 2 are dummies (pid 0), never stored
        const bc_v4i* ap =
            (const bc_v4i*)(a.tab + ((long)(ta < TT && tau < a.nt ? pid_of(limb_of(tau)) : 0) * 8 + pb) * kBconvKT + 16 * h);
#pragma unroll
        for (int st = 0; st < NSTEP; st++) af[st] = ap[2 * st];
    }
    // this lane's source slots (lane half h of step st: 4 st + 2 h + {0, 1}); a dead slot reads
    // slot 0's word and is zeroed
    const u64* sp[NSTEP][2];
    double sq[NSTEP][2], sf[NSTEP][2];
#pragma unroll
    for (int st = 0; st < NSTEP; st++)
#pragma unroll
        for (int uu = 0; uu < 2; uu++) {
            const int sl = 4 * st + 2 * h + uu;
            const int i = sl < a.ns ? sl : 0;
            sp[st][uu] = src + ((long)i << logN) + bx * 16 + (c & 15);
            if (!YIN) {
                const int pid = i < a.s_nq ? a.s_q0 + i : a.s_p0 + i - a.s_nq;
                sq[st][uu] = (double)a.qall[pid];
                sf[st][uu] = a.sinvf[i];
            }
        }
    double xv[TT][16];
    // the epilogue's per-target constants, loaded once (unguarded: a target past nt reads pid 0's),
    // not per row group behind the live-target check (a scalar-cache round trip each)
    double eq[TT], eqi[TT], ew32[TT], ef32[TT], ecr[TT];
#pragma unroll
    for (int m = 0; m < TT; m++) {
        const int pid = tau0 + m < a.nt ? pid_of(limb_of(tau0 + m)) : 0;
        const double* pc = a.pc + 4 * pid;
        eq[m] = pc[0], eqi[m] = pc[1], ew32[m] = pc[2], ef32[m] = pc[3], ecr[m] = a.corr[pid];
    }
    double ev[VC ? 4 * NSTEP : 1];  // VC: 1 / e_j per slot (0 past the sources), uniform
#pragma unroll
    for (int sl = 0; sl < (VC ? 4 * NSTEP : 0); sl++) ev[sl] = a.einv[sl];
    // the source words of row group ar (group g's column c is coefficient
    // (16 ar + 4 w + 2 g + (c >> 4), 16 bx + (c & 15))), PF row groups ahead of their use
    u64 raw[PF + 1][NSTEP][2][2];
    auto load = [&](u64 (&r)[NSTEP][2][2], int ar) {
#pragma unroll
        for (int st = 0; st < NSTEP; st++)
#pragma unroll
            for (int uu = 0; uu < 2; uu++)
#pragma unroll
                for (int g = 0; g < 2; g++) r[st][uu][g] = sp[st][uu][(16 * ar + 4 * w + 2 * g + (c >> 4)) * 256];
    };
#pragma unroll
    for (int p = 0; p < PF; p++) load(raw[p], p);
#pragma unroll
    for (int ar = 0; ar < 16; ar++) {
        if (ar + PF < 16) load(raw[(ar + PF) % (PF + 1)], ar + PF);
        bc_v4i bf[2][NSTEP];
        double ys[2][NSTEP][2];  // VC: the slots' y values (a dead slot's 1/e is 0)
#pragma unroll
        for (int st = 0; st < NSTEP; st++)
#pragma unroll
            for (int uu = 0; uu < 2; uu++)
#pragma unroll
                for (int g = 0; g < 2; g++) {
                    u64 yb = PF ? raw[ar % (PF + 1)][st][uu][g] : sp[st][uu][(16 * ar + 4 * w + 2 * g + (c >> 4)) * 256];
                    if (!YIN) {
                        const double q = sq[st][uu], f = sf[st][uu];
                        double y = fmul_rem(u2d(yb), tw_w(f, q), f, q);
                        y = y < 0.0 ? y + q : y;
                        yb = (u64)__double_as_longlong(y + 4503599627370496.0) & 0xFFFFFFFFFFFFFULL;
                    }
                    // (a dead slot holds slot 0's word: its A bytes are zero -- bconv_row places
                    // only live slots, and only their residue bytes -- so it adds nothing)
                    if (VC) ys[g][st][uu] = u2d(yb);
                    bf[g][st][2 * uu] = (int)(unsigned)yb ^ (int)0x80808080;
                    bf[g][st][2 * uu + 1] = (int)(unsigned)(yb >> 32) ^ (int)0x80808080;
                }
        if constexpr (VC) {
            // lane (c, h): group h's slots from both halves (yl[st][uu][half])
            double yl[NSTEP][2][2];
#pragma unroll
            for (int st = 0; st < NSTEP; st++)
#pragma unroll
                for (int uu = 0; uu < 2; uu++) swap_halves(ys[0][st][uu], ys[1][st][uu], yl[st][uu][0], yl[st][uu][1]);
            double sum = 0.0;
#pragma unroll
            for (int st = 0; st < NSTEP; st++)
#pragma unroll
                for (int hh = 0; hh < 2; hh++)
#pragma unroll
                    for (int uu = 0; uu < 2; uu++) {
                        // unconditional: a dead slot's 1/e is 0 in the tables (+0 leaves the sum
                        // unchanged), and a runtime-guarded scalar load per term cost a scalar-cache
                        // round trip each (DESIGN 4.5's lesson)
                        const int sl = 4 * st + 2 * hh + uu;
                        sum = sum + yl[st][uu][hh] * ev[sl];
                    }
            const int vown = (int)__builtin_rint(sum);  // group h's v
            const auto pr = __builtin_amdgcn_permlane32_swap((unsigned)vown, (unsigned)vown, false, false);
            const int voth = (int)(h ? pr[0] : pr[1]);  // group 1 - h's v (the other half's)
            // slot ns = 4 st + 2 hh + uu lives in lane half hh: byte 0 = v, bytes 1..7 zero
#pragma unroll
            for (int st = 0; st < NSTEP; st++)
#pragma unroll
                for (int uu = 0; uu < 2; uu++)
                    if (4 * st + 2 * h + uu == a.ns) {
#pragma unroll
                        for (int g = 0; g < 2; g++) {
                            bf[g][st][2 * uu] = ((g == h ? vown : voth) & 0xff) ^ (int)0x80808080;
                            bf[g][st][2 * uu + 1] = (int)0x80808080;
                        }
                    }
        }
        if constexpr (MODE == 2) {
#pragma unroll
            for (int m = 0; m < TT; m++) xv[m][ar] = (double)(bf[0][0][0] & 0xffffff) + (double)(bf[1][NSTEP - 1][3] & 0xff);
            continue;
        }
        bc_v16i acc[2];
#pragma unroll
        for (int g = 0; g < 2; g++) {
            acc[g] = bc_v16i{};
#pragma unroll
            for (int st = 0; st < NSTEP; st++) acc[g] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[st], bf[g][st], acc[g], 0, 0, 0);
        }
        // epilogue (bconv_mfma.h): this half's 4 planes of target m, group g, as one exact double;
        // the swap gives lane (c, h) group h's column c = its own coefficient of the column layout
#pragma unroll
        for (int m = 0; m < TT; m++) {
            if (m >= nlive) break;  // block-uniform
            double part[2];
#pragma unroll
            for (int g = 0; g < 2; g++) {
                const int p01 = acc[g][4 * m] + acc[g][4 * m + 1] * 256, p23 = acc[g][4 * m + 2] + acc[g][4 * m + 3] * 256;
                part[g] = __builtin_fma((double)p23, 65536.0, (double)p01);
            }
            double lo, hi;
            swap_halves(part[0], part[1], lo, hi);
            xv[m][ar] = fred(lo + fmul_rem(hi, ew32[m], ef32[m], eq[m]) + ecr[m], eq[m], eqi[m]);
        }
    }
    // the column stages of each live target; LDS tile m % LT (LT = 2: the barrier inside the
    // stages of target m + 1 orders every read of tile m & 1 for target m before its reuse by
    // target m + 2; LT = 1: one more barrier before each reuse)
    __syncthreads();  // twq
    if constexpr (MODE == 1) {
#pragma unroll
        for (int m = 0; m < TT; m++) {
            if (m >= nlive) break;
            u64* o = dst + ((long)limb_of(tau0 + m) << logN);
#pragma unroll
            for (int ar = 0; ar < 16; ar++) st_d(&o[(ar * 16 + b) * 256 + bx * 16 + cl], xv[m][ar]);
        }
        return;
    }
#pragma unroll
    for (int m = 0; m < TT; m++) {
        if (m >= nlive) break;
        if (LT == 1 && m > 0) __syncthreads();
        const int tl = limb_of(tau0 + m), pid = pid_of(tl);
        const double q = (double)T.q[pid], qi = T.qinv[pid];
        cols256_stages_store(xv[m], q, qi, q >= kBigPrime, T.psif + ((long)pid << logN), T.cw + (long)pid * kColW,
                             twq[m], s[m % LT], dst + ((long)tl << logN), b, cl, bx * 16 + cl);
    }
}

}  // namespace aesfhe
