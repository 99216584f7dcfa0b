// ntt256.h -- register-resident NTT passes for N = 2^16 (= 256 x 256), the BASELINE.json ring.
//
// Each pass runs 256-point sub-transforms.  A sub-transform lives in 16 lanes x 16 registers:
// the first four butterfly stages (distances 128..16) run in registers on x[a*16 + b] for the
// lane's fixed b, one LDS transpose regroups the data so each lane holds x[a*16 + b] for a fixed
// a, the last four stages (distances 8..1) run in registers again.  Stage twiddles come from the
// same bit-reversed psi tables as the generic kernels, so results are identical
// residue for residue.  A 256-thread workgroup processes 16 sub-transforms (one wave = 4).
#pragma once
#include "kernels.h"

namespace aesfhe {

__device__ __forceinline__ u64 mulw(u64 a, u64 w, double wq, u64 q) { return mul_w(a, w, wq, q); }

__device__ __forceinline__ void ct_bfly(u64& x, u64& y, u64 w, double wq, u64 q) {
    u64 v = mulw(y, w, wq, q);
    u64 s = x + v;
    s = s >= q ? s - q : s;
    u64 d = x >= v ? x - v : x + q - v;
    x = s;
    y = d;
}

__device__ __forceinline__ void gs_bfly(u64& x, u64& y, u64 w, double wq, u64 q) {
    u64 s = x + y;
    s = s >= q ? s - q : s;
    u64 d = x >= y ? x - y : x + q - y;
    x = s;
    y = mulw(d, w, wq, q);
}

// Lazy (Harvey) butterflies: every prime < 2^50 so values up to 4q stay below 2^52, the exact
// range of the fp64 quotient trick.  CT: inputs [0, 4q) -> outputs [0, 4q); GS: [0, 2q) ->
// [0, 2q).  Passes reduce to canonical [0, q) only where a transform ends.
__device__ __forceinline__ void ct_lazy(u64& x, u64& y, u64 w, double wq, u64 q, u64 q2) {
#ifdef NTT_NOCOMPUTE  // timing-only build (tools/ntt_bench.hip): keep the data flow, drop the math
    x ^= w;
    y ^= x;
    return;
#endif
    const u64 qh = rint_u(u2d(y), wq);
    const u64 v = y * w - qh * q + q;  // (0, 2q)
    const u64 xr = x >= q2 ? x - q2 : x;  // [0, 2q)
    x = xr + v;
    y = xr - v + q2;
}

__device__ __forceinline__ void gs_lazy(u64& x, u64& y, u64 w, double wq, u64 q, u64 q2) {
#ifdef NTT_NOCOMPUTE
    x ^= w;
    y ^= x;
    return;
#endif
    u64 s = x + y;
    s = s >= q2 ? s - q2 : s;         // [0, 2q)
    const u64 d = x - y + q2;         // (0, 4q)
    const u64 qh = rint_u(u2d(d), wq);
    y = d * w - qh * q + q;           // (0, 2q)
    x = s;
}

__device__ __forceinline__ u64 canon4(u64 x, u64 q, u64 q2) {  // [0, 4q) -> [0, q)
    x = x >= q2 ? x - q2 : x;
    return x >= q ? x - q : x;
}

constexpr int kPad = 17;  // LDS row stride (u64) of the 16 x 16 transpose tiles: kills conflicts

// Forward, column pass: stages m = 1..128 on columns of stride 256.
// Workgroup = 16 columns [c0, c0+16); lane (cl, b) = (tid & 15, tid >> 4).
__global__ __launch_bounds__(256) void k_ntt256_fwd_cols(Span src, Span dst, Tabs T) {
    __shared__ u64 s[256 * kPad];
    __shared__ Tw tws[256];
    int pid;
    const u64* in = span_ptr(src, blockIdx.y, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, cl = tid & 15, b = tid >> 4;
    const int c = blockIdx.x * 16 + cl;
    const u64 q = T.q[pid], q2 = 2 * q;
    const long toff = (long)pid << T.logN;
    const Tw* tg = T.tw + toff;
    tws[tid] = tg[tid];
    u64 x[16];
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = in[(a * 16 + b) * 256 + c];
    __syncthreads();
    // stages 0..3: pairs (a, a + h), twiddle W[m + (a >> (4 - s))]
#pragma unroll
    for (int st = 0; st < 4; st++) {
        const int m = 1 << st, h = 8 >> st;
#pragma unroll
        for (int a = 0; a < 16; a++) {
            if (a & h) continue;
            const Tw t = tg[m + (a >> (4 - st))];  // uniform address: scalar load
            ct_lazy(x[a], x[a + h], t.w, t.wq, q, q2);
        }
    }
    // transpose: row r = a*16 + b, column cl
#pragma unroll
    for (int a = 0; a < 16; a++) s[(a * 16 + b) * kPad + cl] = x[a];
    __syncthreads();
    const int ap = b;  // now lane holds rows ap*16 + bb, bb = 0..15
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = s[(ap * 16 + bb) * kPad + cl];
    // stages 4..7: m = 16 << (st-4), pairs (bb, bb + h), group i = ap*(m/16) + (bb >> (8 - st))
#pragma unroll
    for (int st = 4; st < 8; st++) {
        const int m = 1 << st, h = 128 >> st;
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {
            if (bb & h) continue;
            const Tw t = tws[m + ap * (m >> 4) + (bb >> (8 - st))];
            ct_lazy(x[bb], x[bb + h], t.w, t.wq, q, q2);
        }
    }
#pragma unroll
    for (int bb = 0; bb < 16; bb++) out[(ap * 16 + bb) * 256 + c] = x[bb];
}

// Forward, row pass: stages m = 256..32768 within rows of 256 contiguous elements.
// Workgroup = 16 rows [r0, r0+16); lane (b, rl) = (tid & 15, tid >> 4).
__global__ __launch_bounds__(256) void k_ntt256_fwd_rows(Span dst, Tabs T) {
    __shared__ u64 s[16 * 16 * kPad];
    int pid;
    u64* io = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, b = tid & 15, rl = tid >> 4;
    const int row = blockIdx.x * 16 + rl;
    const u64 q = T.q[pid], q2 = 2 * q;
    const long toff = (long)pid << T.logN;
    const Tw* W = T.tw + toff;
    u64* rp = io + (long)row * 256;
    u64 x[16];
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = rp[a * 16 + b];
    // local stages ml = 1..8: twiddle index ml*(256 + row) + (a >> (4 - st))
#pragma unroll
    for (int st = 0; st < 4; st++) {
        const int ml = 1 << st, h = 8 >> st;
        const int base = ml * (256 + row);
#pragma unroll
        for (int a = 0; a < 16; a++) {
            if (a & h) continue;
            const Tw t = W[base + (a >> (4 - st))];
            ct_lazy(x[a], x[a + h], t.w, t.wq, q, q2);
        }
    }
    u64* sr = s + rl * 16 * kPad;
#pragma unroll
    for (int a = 0; a < 16; a++) sr[a * kPad + b] = x[a];
    __syncthreads();
    const int ap = b;
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = sr[ap * kPad + bb];
#pragma unroll
    for (int st = 4; st < 8; st++) {
        const int ml = 1 << st, h = 128 >> st;
        const int base = ml * (256 + row) + ap * (ml >> 4);
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {
            if (bb & h) continue;
            const Tw t = W[base + (bb >> (8 - st))];
            ct_lazy(x[bb], x[bb + h], t.w, t.wq, q, q2);
        }
    }
    // coalesced store through LDS: lane writes back its 16 elements, then row-major copy-out
#pragma unroll
    for (int bb = 0; bb < 16; bb++) sr[ap * kPad + bb] = canon4(x[bb], q, q2);
    __syncthreads();
    u64* base = io + (long)blockIdx.x * 16 * 256;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int e = k * 256 + tid, r = e >> 8, cc = e & 255;
        base[e] = s[r * 16 * kPad + (cc >> 4) * kPad + (cc & 15)];
    }
}

// Inverse, row pass (Gentleman-Sande, distances 1..128 within rows), reads src, writes dst.
__global__ __launch_bounds__(256) void k_ntt256_inv_rows(Span src, Span dst, Tabs T) {
    __shared__ u64 s[16 * 16 * kPad];
    int pid;
    const u64* in = span_ptr(src, blockIdx.y, T.logN, T.Lp1, pid);
    u64* out = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, b = tid & 15, rl = tid >> 4;
    const int row = blockIdx.x * 16 + rl;
    const u64 q = T.q[pid], q2 = 2 * q;
    const long toff = (long)pid << T.logN;
    const Tw* W = T.itw + toff;
    const int N = 1 << T.logN;
    // coalesced load through LDS, then lane (b, rl) takes elements ap*16 + bb (ap = b)
    const u64* gb = in + (long)blockIdx.x * 16 * 256;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int e = k * 256 + tid, r = e >> 8, cc = e & 255;
        s[r * 16 * kPad + (cc >> 4) * kPad + (cc & 15)] = gb[e];
    }
    __syncthreads();
    u64* sr = s + rl * 16 * kPad;
    const int ap = b;
    u64 x[16];
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = sr[ap * kPad + bb];
    // t = 1, 2, 4, 8: pairs (bb, bb + t); index N/(2t) + row*(128/t) + (ap*16 + bb)/(2t)
#pragma unroll
    for (int st = 0; st < 4; st++) {
        const int t = 1 << st;
        const int base = N / (2 * t) + row * (128 / t) + ap * (8 / t);
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {
            if (bb & t) continue;
            const Tw w = W[base + (bb >> (st + 1))];
            gs_lazy(x[bb], x[bb + t], w.w, w.wq, q, q2);
        }
    }
#pragma unroll
    for (int bb = 0; bb < 16; bb++) sr[ap * kPad + bb] = x[bb];
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = sr[a * kPad + b];
    // t = 16..128: pairs (a, a + t/16); index N/(2t) + row*(128/t) + a/(2t/16)
#pragma unroll
    for (int st = 4; st < 8; st++) {
        const int t = 1 << st, ta = t >> 4;
        const int base = N / (2 * t) + row * (128 / t);
#pragma unroll
        for (int a = 0; a < 16; a++) {
            if (a & ta) continue;
            const Tw w = W[base + (a >> (st - 3))];
            gs_lazy(x[a], x[a + ta], w.w, w.wq, q, q2);
        }
    }
    u64* op = out + (long)row * 256;
#pragma unroll
    for (int a = 0; a < 16; a++) op[a * 16 + b] = x[a];
}

// Inverse, column pass (distances 256..32768 = rows 1..128), then the N^{-1} scaling.
__global__ __launch_bounds__(256) void k_ntt256_inv_cols(Span dst, Tabs T) {
    __shared__ u64 s[256 * kPad];
    __shared__ Tw tws[256];
    int pid;
    u64* io = span_ptr(dst, blockIdx.y, T.logN, T.Lp1, pid);
    const int tid = threadIdx.x, cl = tid & 15, b = tid >> 4;
    const int c = blockIdx.x * 16 + cl;
    const u64 q = T.q[pid], q2 = 2 * q;
    const long toff = (long)pid << T.logN;
    const Tw* tg = T.itw + toff;
    tws[tid] = tg[tid];
    const int ap = b;
    u64 x[16];
    // lane (cl, ap) holds rows ap*16 + bb
#pragma unroll
    for (int bb = 0; bb < 16; bb++) x[bb] = io[(ap * 16 + bb) * 256 + c];
    __syncthreads();
    // row distance tr = 1..8: index 128/tr + r/(2tr), r = ap*16 + bb
#pragma unroll
    for (int st = 0; st < 4; st++) {
        const int tr = 1 << st;
        const int base = 128 / tr + ap * (8 / tr);
#pragma unroll
        for (int bb = 0; bb < 16; bb++) {
            if (bb & tr) continue;
            const Tw w = tws[base + (bb >> (st + 1))];
            gs_lazy(x[bb], x[bb + tr], w.w, w.wq, q, q2);
        }
    }
#pragma unroll
    for (int bb = 0; bb < 16; bb++) s[(ap * 16 + bb) * kPad + cl] = x[bb];
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 16; a++) x[a] = s[(a * 16 + b) * kPad + cl];
    // row distance tr = 16..128 (a-distance tr/16): index 128/tr + a/(2 tr/16)
#pragma unroll
    for (int st = 4; st < 8; st++) {
        const int tr = 1 << st, ta = tr >> 4;
        const int base = 128 / tr;
#pragma unroll
        for (int a = 0; a < 16; a++) {
            if (a & ta) continue;
            const Tw w = tg[base + (a >> (st - 3))];  // uniform: scalar load
            gs_lazy(x[a], x[a + ta], w.w, w.wq, q, q2);
        }
    }
    const u64 ni = T.ninv[pid];
    const double nif = T.ninvf[pid];
#pragma unroll
    for (int a = 0; a < 16; a++) io[(a * 16 + b) * 256 + c] = mulw(x[a], ni, nif, q);
}

}  // namespace aesfhe
