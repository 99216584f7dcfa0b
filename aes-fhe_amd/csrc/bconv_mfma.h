// bconv_mfma.h -- RNS base conversion (ModUp, ModDown) on the gfx950 matrix cores.
//
// A base conversion is a matrix product: out_t[k] = sum_i y_i[k] * H[i][t] mod p_t over the
// source limbs i (y_i = [x_i * s_i]_{q_i}, canonical) and the targets t.  The exact-fp64 VALU
// form (k_modup / k_moddown, kernels_ops.h) spends six fp64 ops per term and was issue-bound
// (SQ WAIT_INST 0.69 / 0.74, fp64 at 0.34 / 0.38 of peak).  Here the sum runs exactly on
// v_mfma_i32_32x32x32_i8 over byte planes:
//   y_i = sum_a u_{i,a} 256^a (u the 8 bytes of the canonical u64), so
//   sum_i y_i H[i][t] = sum_{(i,a)} u_{i,a} H'[(i,a)][t]  (mod p_t),  H' = 256^a H[i][t] mod p_t,
//   H' = sum_b c_b 256^b with signed balanced bytes c_b (b = 0..6, host tables), so
//   sum_{(i,a)} u_{i,a} H' = sum_b 256^b S_b,  S_b = sum_{(i,a)} u_{i,a} c_b[(i,a)][t]  (exact i32).
// The MFMA takes signed bytes: u XOR 0x80 = u - 128, and the host folds 128 sum_{(i,a)} H' mod p_t
// into a per-target correction.  A (32 x K, the constants) has the rows (target, byte plane b);
// B (K x 32) the columns = coefficients, one u64 y per 8 bytes of K (no packing: the u64 IS the
// operand).  The 32 x 32 i32 result (D row r: lane half (r >> 2) & 1, register (r & 3) + 4 (r >> 3))
// holds half of the byte planes of 4 targets per lane; V = sum_b 256^b S_b, out = (lo + (2^32 mod p)
// hi + corr) mod p (tools/mfma_i8_probe.hip pins the operand / result maps).
// ModDown's exact conversion: v = rint(sum_j y_j (1/e_j)) (fp64, j in order, as the
// oracle) rides in one more byte slot of K whose constant column is -D mod q_i.
#pragma once
#include "kernels.h"

namespace aesfhe {

typedef int bc_v4i __attribute__((ext_vector_type(4)));
typedef int bc_v16i __attribute__((ext_vector_type(16)));

// One base conversion launch.  z = blockIdx.z indexes (batch element, component): element z / nc,
// component z % nc.  Sources are consecutive limbs from src; targets tau = 0 .. nt - 1 map to the
// output limb tl = tau < skip0 ? tau : tau + skipn (ModUp skips the digit's own limbs) whose
// prime is pid = tl <= tl_l ? tl : Lp1 + tl - tl_l - 1 (Q limbs, then the special primes).
struct BconvArgs {
    const u64* src;
    long sbs, scs;     // source strides: batch element, component (limb i at + i N)
    u64* dst;
    long dbs, dcs;     // output strides: batch element, component (limb tl at + tl N)
    int nc;            // components per batch element (ModUp 1, ModDown 2)
    int ns;            // source limbs
    int s_nq, s_q0, s_p0;  // source i's prime: i < s_nq ? s_q0 + i : s_p0 + i - s_nq
    const double* sinvf;   // y_i = [x_i * w_i]_{q_i}, w_i / q_i per source
    const double* einv;    // VC: 1 / e_i
    int nt, skip0, skipn, tl_l, Lp1;
    const int8_t* tab;     // [pid][8 planes][128 bytes of K]: signed bytes of H' per (slot, byte)
    const double* corr;    // [pid] 128 sum H' mod p (exact double)
    const double* pc;      // [pid][4] {p, 1/p, 2^32 mod p, (2^32 mod p) / p} as doubles (epilogue constants)
    const u64* qall;
    const double* qinvall;
    int tiles_per_group;   // target tiles (4 targets) per blockIdx.y
};
constexpr int kBconvKT = 128;  // K bytes per table row (up to 4 MFMA steps of 32)

// (x, y) -> (x with lanes 32..63 taken from y's lanes 0..31, y with lanes 0..31 taken from x's
// lanes 32..63): v_permlane32_swap on both dwords of the doubles
__device__ __forceinline__ void swap_halves(double x, double y, double& xo, double& yo) {
    const u64 a = (u64)__double_as_longlong(x), b = (u64)__double_as_longlong(y);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)a, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(a >> 32), (unsigned)(b >> 32), false, false);
    xo = __longlong_as_double((long long)(((u64)(unsigned)hi[0] << 32) | (unsigned)lo[0]));
    yo = __longlong_as_double((long long)(((u64)(unsigned)hi[1] << 32) | (unsigned)lo[1]));
}

// grid (N / 256, target groups, batch * nc), 256 threads: each wave converts 64 coefficients (two
// 32-column groups) into every target of its group.  NSTEP MFMA K-steps of 32 bytes = 4 u64
// slots: lane half h of step s holds slots 4 s + 2 h, 4 s + 2 h + 1.  VC: slot ns carries v.
template <int NSTEP, bool VC>
__global__ __launch_bounds__(256, 3) void k_bconv_mfma(BconvArgs a, int logN) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int z = blockIdx.z, zb = z / a.nc, zc = z - zb * a.nc;
    const long kb = (long)blockIdx.x * 256 + w * 64;  // the wave's 64 coefficients
    const u64* src = a.src + (long)zb * a.sbs + (long)zc * a.scs;
    // ---- y slots of this lane (both column groups), as the B operand --------------------------
    bc_v4i bf[2][NSTEP];
    double ys[2][2 * NSTEP];  // VC: this lane's y values (slot order), for the in-order v sum
#pragma unroll
    for (int s = 0; s < NSTEP; s++) {
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int sl = 4 * s + 2 * h + u;
            const bool live = sl < a.ns;
            const int i = live ? sl : 0;
            const int pid = i < a.s_nq ? a.s_q0 + i : a.s_p0 + i - a.s_nq;
            const double q = (double)a.qall[pid];
            const double f = a.sinvf[i], wv = tw_w(f, q);
            const u64* sp = src + ((long)i << logN) + kb + c;
#pragma unroll
            for (int g = 0; g < 2; g++) {
                double y = fmul_rem(u2d(sp[32 * g]), wv, f, q);
                y = y < 0.0 ? y + q : y;  // canonical: the oracle's y
                ys[g][2 * s + u] = live ? y : 0.0;
                const u64 yb = live ? ((u64)__double_as_longlong(y + 4503599627370496.0) & 0xFFFFFFFFFFFFFULL) : 0;
                bf[g][s][2 * u] = (int)(unsigned)yb ^ (int)0x80808080;
                bf[g][s][2 * u + 1] = (int)(unsigned)(yb >> 32) ^ (int)0x80808080;
            }
        }
    }
    if constexpr (VC) {
        // v = rint(sum_j y_j * (1/e_j)), j = 0 .. ns - 1 in order (the oracle's fp64 sum): the
        // partner lane (other half, same column) holds the other slots
#pragma unroll
        for (int g = 0; g < 2; g++) {
            double other[2 * NSTEP];
#pragma unroll
            for (int m = 0; m < 2 * NSTEP; m++) other[m] = __shfl_xor(ys[g][m], 32);
            double uu = 0.0;
#pragma unroll
            for (int s = 0; s < NSTEP; s++)
#pragma unroll
                for (int hh = 0; hh < 2; hh++)
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        const int sl = 4 * s + 2 * hh + u;
                        const double yv = hh == h ? ys[g][2 * s + u] : other[2 * s + u];
                        if (sl < a.ns) uu = uu + yv * a.einv[sl];
                    }
            const int v = (int)__builtin_rint(uu);
            // slot ns (in this lane when 4 s + 2 h + u == ns): byte 0 = v, bytes 1..7 zero
#pragma unroll
            for (int s = 0; s < NSTEP; s++)
#pragma unroll
                for (int u = 0; u < 2; u++)
                    if (4 * s + 2 * h + u == a.ns) {
                        bf[g][s][2 * u] = (v & 0xff) ^ (int)0x80808080;
                        bf[g][s][2 * u + 1] = (int)0x80808080;
                    }
        }
    }
    // ---- target tiles ------------------------------------------------------------------------
    // A rows: row r = (target r >> 3 of the tile, byte plane (r & 3) + 4 ((r >> 2) & 1)), so that
    // lane half h holds, in registers 4 m .. 4 m + 3, planes 4 h .. 4 h + 3 of the tile's target m
    // (all four targets, both column groups).  Each half folds its 4 planes into one exact double
    // (lo for h = 0, hi for h = 1); one cross-half exchange of 4 doubles then gives half 0 the whole
    // of column group 0 and half 1 the whole of group 1, so every lane finishes the tile's 4
    // targets for one coefficient: the targets -- and their constants -- are wave-uniform (scalar
    // loads), and each store writes 64 consecutive coefficients of one limb (512 B).
    // Two tiles in flight: tile + 1's MFMAs are issued before tile's epilogue (the matrix pipe
    // runs beside the VALU epilogue) and tile + 2's A fragments are requested before it (ping-pong
    // register sets, the loop unrolled by two).  A target past nt reads pid 0's row: its D rows --
    // which depend on that A row only -- are computed and never stored.
    const int row = lane & 31;
    const int ta = row >> 3, pb = (row & 3) + 4 * ((row >> 2) & 1);
    u64* dst = a.dst + (long)zb * a.dbs + (long)zc * a.dcs + kb + 32 * h + c;
    const int tile0 = blockIdx.y * a.tiles_per_group;
    const int ntile = (a.nt + 3) >> 2;
    const int tile1 = min(tile0 + a.tiles_per_group, ntile);
    auto limb_of = [&](int tau) { return tau < a.skip0 ? tau : tau + a.skipn; };
    auto pid_of = [&](int tl) { return tl <= a.tl_l ? tl : a.Lp1 + tl - a.tl_l - 1; };
    auto fetch = [&](bc_v4i (&af)[NSTEP], int tile) {
        const int tau = 4 * tile + ta;
        const bc_v4i* ap =
            (const bc_v4i*)(a.tab + ((long)(tau < a.nt ? pid_of(limb_of(tau)) : 0) * 8 + pb) * kBconvKT + 16 * h);
#pragma unroll
        for (int s = 0; s < NSTEP; s++) af[s] = ap[2 * s];  // bytes 32 s + 16 h .. + 15 of the row
    };
    auto mma = [&](bc_v16i (&acc)[2], const bc_v4i (&af)[NSTEP]) {
#pragma unroll
        for (int g = 0; g < 2; g++) {
            acc[g] = bc_v16i{};
#pragma unroll
            for (int s = 0; s < NSTEP; s++) acc[g] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bf[g][s], acc[g], 0, 0, 0);
        }
    };
    auto epilogue = [&](const bc_v16i (&acc)[2], int tile) {
        // this half's 4 planes of target m, group g: |S| < 2^21, byte pairs exact in i32 (< 2^30),
        // then |part| < 2^46 in fp64
        double part[2][4];
#pragma unroll
        for (int g = 0; g < 2; g++)
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const int p01 = acc[g][4 * m] + acc[g][4 * m + 1] * 256, p23 = acc[g][4 * m + 2] + acc[g][4 * m + 3] * 256;
                part[g][m] = __builtin_fma((double)p23, 65536.0, (double)p01);
            }
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int tau = 4 * tile + m;  // wave-uniform
            if (tau >= a.nt) break;
            // v_permlane32_swap: lanes 32..63 of the first operand <-> lanes 0..31 of the second
            // (tools/mfma_i8_probe.hip checks it): (part[0], part[1]) become (lo of group h, hi of
            // group h) in every lane, no select
            double lo, hi;
            swap_halves(part[0][m], part[1][m], lo, hi);
            const int tl = limb_of(tau), pid = pid_of(tl);
            const double* pc = a.pc + 4 * pid;
            const double q = pc[0], qi = pc[1], w32 = pc[2], f32 = pc[3], cr = a.corr[pid];
            // (2^32 hi mod p) in (-p, p); + corr < p: below 2^52
            const double v = lo + fmul_rem(hi, w32, f32, q) + cr;
            __builtin_nontemporal_store(fcanon(v, q, qi), dst + ((long)tl << logN));  // streaming
        }
    };
    if (tile0 < tile1) {
        bc_v4i af0[NSTEP], af1[NSTEP];
        bc_v16i acc0[2], acc1[2];
        fetch(af0, tile0);
        mma(acc0, af0);
        if (tile0 + 1 < tile1) fetch(af1, tile0 + 1);
#pragma unroll 1
        for (int tile = tile0; tile < tile1; tile += 2) {
            // acc0 = tile (issued), af1 = tile + 1 (requested)
            if (tile + 1 < tile1) {
                mma(acc1, af1);
                if (tile + 2 < tile1) fetch(af0, tile + 2);
            }
            epilogue(acc0, tile);
            if (tile + 1 >= tile1) break;
            // acc1 = tile + 1 (issued), af0 = tile + 2 (requested)
            if (tile + 2 < tile1) {
                mma(acc0, af0);
                if (tile + 3 < tile1) fetch(af1, tile + 3);
            }
            epilogue(acc1, tile + 1);
        }
    }
}

}  // namespace aesfhe
