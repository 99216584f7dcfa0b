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
// operand).  The 32 x 32 i32 result puts, in each lane, the 8 planes of 2 targets of one
// coefficient (D row r: lane half (r >> 2) & 1, register (r & 3) + 4 (r >> 3)), so the epilogue
// is per lane: V = sum_b 256^b S_b, out = (lo + (2^32 mod p) hi + corr) mod p, ~28 VALU ops per
// output against ~78 (tools/mfma_i8_probe.hip pins the operand / result maps).
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
    // Two tiles in flight: tile + 1's MFMAs are issued before tile's epilogue, so the matrix
    // pipe runs beside the VALU epilogue, and tile + 2's A fragments and constants are requested
    // before it as well (ping-pong register sets, the loop unrolled by two; every load
    // branch-free: a target past nt reads pid 0's row, its D rows -- which depend on that A row
    // only -- are computed and never stored).
    const int row = lane & 31;  // this lane's A row: target 2 ((row >> 2) & 1) + (row >> 4), plane b
    const int ta = 2 * ((row >> 2) & 1) + (row >> 4), pb = 4 * ((row >> 3) & 1) + (row & 3);
    u64* dst = a.dst + (long)zb * a.dbs + (long)zc * a.dcs + kb + c;
    const int tile0 = blockIdx.y * a.tiles_per_group;
    const int ntile = (a.nt + 3) >> 2;
    const int tile1 = min(tile0 + a.tiles_per_group, ntile);
    auto limb_of = [&](int tau) { return tau < a.skip0 ? tau : tau + a.skipn; };
    auto pid_of = [&](int tl) { return tl <= a.tl_l ? tl : a.Lp1 + tl - a.tl_l - 1; };
    // A fragments of a tile (the epilogue constants are requested after the tile's successor's
    // MFMAs are issued: their L1 round trip overlaps the matrix pipe)
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
    // this lane holds targets 4 tile + 2 h + t2 (t2 = 0, 1), plane b of t2 in register
    // 8 t2 + 4 (b >> 2) + (b & 3), of coefficients kb + 32 g + c
    auto epilogue = [&](const bc_v16i (&acc)[2], int tile) {
        double qv[2], qiv[2], crv[2], wv[2], fv[2];
#pragma unroll
        for (int t2 = 0; t2 < 2; t2++) {
            const int tt = 4 * tile + 2 * h + t2;
            const int pid = tt < a.nt ? pid_of(limb_of(tt)) : 0;
            const double* pc = a.pc + 4 * pid;
            qv[t2] = pc[0];
            qiv[t2] = pc[1];
            wv[t2] = pc[2];
            fv[t2] = pc[3];
            crv[t2] = a.corr[pid];
        }
#pragma unroll
        for (int t2 = 0; t2 < 2; t2++) {
            const int tau = 4 * tile + 2 * h + t2;
            const double q = qv[t2], qi = qiv[t2], cr = crv[t2], w32 = wv[t2], f32 = fv[t2];
            u64* op = dst + ((long)limb_of(tau) << logN);
#pragma unroll
            for (int g = 0; g < 2; g++) {
                const int r0 = 8 * t2;
                // |S_b| <= 128 * 128 * (7 * 16 + 1) < 2^21: byte pairs combine exactly in i32
                // (|S + 256 S'| < 2^30), then |lo|, |hi| < 2^46 in fp64
                const int p01 = acc[g][r0 + 0] + acc[g][r0 + 1] * 256, p23 = acc[g][r0 + 2] + acc[g][r0 + 3] * 256;
                const int p45 = acc[g][r0 + 4] + acc[g][r0 + 5] * 256, p67 = acc[g][r0 + 6] + acc[g][r0 + 7] * 256;
                const double lo = __builtin_fma((double)p23, 65536.0, (double)p01);
                const double hi = __builtin_fma((double)p67, 65536.0, (double)p45);
                // (2^32 hi mod p) in (-p, p); + corr < p: below 2^52
                const double v = lo + fmul_rem(hi, w32, f32, q) + cr;
                if (tau < a.nt) __builtin_nontemporal_store(fcanon(v, q, qi), &op[32 * g]);  // streaming
            }
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
