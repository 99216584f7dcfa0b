// codec_dev.h -- the canonical-embedding codec on the device: HEAAN's special FFT
// and its inverse, stage by stage, bit-identical to the host Codec (ckks_host.h) and the oracle.
//
// Bit-identity: every butterfly performs the host's operations in the host's order with
// explicitly rounded fp64 intrinsics (__dadd_rn / __dsub_rn / __dmul_rn / __ddiv_rn: no
// contraction into FMAs, whatever the compiler flags), on twiddles the host computed (libm
// cos / sin, uploaded once per engine).  Butterflies of one stage are independent, so the order
// in which the device runs them does not change any result.  Rounding to integers uses round()
// (half away from zero), which is llround's rule for every finite value below 2^63.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace aesfhe {

struct CodecTabs {
    const double* kre;  // cos(2 pi j / M), j = 0..M
    const double* kim;  // sin(2 pi j / M)
    const long* rot;    // 5^j mod M, j < n
    long M;             // 2N
    int n, logn;        // slots N/2, log2(n)
};

// One stage of the inverse special FFT (Codec::special_inv, stage `len`) over B vectors of n
// slots (vector b at re + b * n): one thread per butterfly.
__global__ void k_sfft_inv_stage(double* __restrict__ re, double* __restrict__ im, CodecTabs T, int len, int B) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int half = T.n >> 1;
    if (t >= (long)B * half) return;
    const int b = (int)(t / half), u = (int)(t % half);
    const int lenh = len >> 1;
    const int i = (u / lenh) * len, j = u % lenh;
    const long lenq = (long)len << 2;
    const long idx = (lenq - (T.rot[j] % lenq)) * T.M / lenq;
    double* r = re + (long)b * T.n;
    double* m = im + (long)b * T.n;
    const double ar = r[i + j], ai = m[i + j], br = r[i + j + lenh], bi = m[i + j + lenh];
    const double ur = __dadd_rn(ar, br), ui = __dadd_rn(ai, bi);
    const double vr = __dsub_rn(ar, br), vi = __dsub_rn(ai, bi);
    const double wr = T.kre[idx], wi = T.kim[idx];
    const double tr = __dsub_rn(__dmul_rn(vr, wr), __dmul_rn(vi, wi));
    const double ti = __dadd_rn(__dmul_rn(vr, wi), __dmul_rn(vi, wr));
    r[i + j] = ur;
    m[i + j] = ui;
    r[i + j + lenh] = tr;
    m[i + j + lenh] = ti;
}

// One stage of the forward special FFT (Codec::special, stage `len`).
__global__ void k_sfft_fwd_stage(double* __restrict__ re, double* __restrict__ im, CodecTabs T, int len, int B) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int half = T.n >> 1;
    if (t >= (long)B * half) return;
    const int b = (int)(t / half), u = (int)(t % half);
    const int lenh = len >> 1;
    const int i = (u / lenh) * len, j = u % lenh;
    const long lenq = (long)len << 2;
    const long idx = (T.rot[j] % lenq) * T.M / lenq;
    double* r = re + (long)b * T.n;
    double* m = im + (long)b * T.n;
    const double ur = r[i + j], ui = m[i + j], xr = r[i + j + lenh], xi = m[i + j + lenh];
    const double wr = T.kre[idx], wi = T.kim[idx];
    const double vr = __dsub_rn(__dmul_rn(xr, wr), __dmul_rn(xi, wi));
    const double vi = __dadd_rn(__dmul_rn(xr, wi), __dmul_rn(xi, wr));
    r[i + j] = __dadd_rn(ur, vr);
    m[i + j] = __dadd_rn(ui, vi);
    r[i + j + lenh] = __dsub_rn(ur, vr);
    m[i + j + lenh] = __dsub_rn(ui, vi);
}

// Bit-reversal permutation of each vector (Codec::bitrev), out of place: dst[brv(k)] = src[k].
__global__ void k_sfft_bitrev(const double* __restrict__ sre, const double* __restrict__ sim,
                              double* __restrict__ dre, double* __restrict__ dim_, int n, int logn, int B) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B * n) return;
    const int b = (int)(t / n), k = (int)(t % n);
    const int r = (int)(__brev((unsigned)k) >> (32 - logn));
    dre[(long)b * n + r] = sre[t];
    dim_[(long)b * n + r] = sim[t];
}

// Encoder input: B slot vectors of n_slots values (row stride `stride`) zero-padded to n.
__global__ void k_sfft_load(const double* __restrict__ re, const double* __restrict__ im, long stride,
                            long n_slots, double* __restrict__ dre, double* __restrict__ dim_, int n, int B) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B * n) return;
    const long b = t / n, k = t % n;
    const bool in = k < n_slots;
    dre[t] = in && re ? re[b * stride + k] : 0.0;
    dim_[t] = in && im ? im[b * stride + k] : 0.0;
}

// Encoder output (aesfhe_encode): after the inverse FFT and the bit reversal, coefficient
// k = round(re[k] / n * scale), k + n = round(im[k] / n * scale); flags[block] = 1 if any value
// of the block overflows int64 (plain vector stores, one word per workgroup).
__global__ void k_sfft_round(const double* __restrict__ re, const double* __restrict__ im, int n, int B,
                             double scale, int64_t* __restrict__ co, int* __restrict__ flags) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (t < (long)B * n) {
        const long b = t / n, k = t % n;
        const double dn = (double)n;
        const double a = __dmul_rn(__ddiv_rn(re[t], dn), scale), c = __dmul_rn(__ddiv_rn(im[t], dn), scale);
        bad = !(fabs(a) < 9.0e18) || !(fabs(c) < 9.0e18);
        co[b * 2 * n + k] = bad ? 0 : (int64_t)round(a);
        co[b * 2 * n + k + n] = bad ? 0 : (int64_t)round(c);
    }
    const int any = __syncthreads_or(bad ? 1 : 0);
    if (threadIdx.x == 0) flags[blockIdx.x] = any;
}

// Decoder input (aesfhe_decode): re[k] = co[k] / scale, im[k] = co[k + n] / scale, written
// bit-reversed (the forward FFT starts with the permutation).
__global__ void k_sfft_unround(const int64_t* __restrict__ co, int n, int logn, int B, double scale,
                               double* __restrict__ re, double* __restrict__ im) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (long)B * n) return;
    const long b = t / n;
    const int k = (int)(t % n);
    const int r = (int)(__brev((unsigned)k) >> (32 - logn));
    re[b * n + r] = __ddiv_rn((double)co[b * 2 * n + k], scale);
    im[b * n + r] = __ddiv_rn((double)co[b * 2 * n + k + n], scale);
}

// Decryption to coefficients on the device: residues r0 (mod q0) and, for level >= 1, r1 (mod q1)
// of B x N coefficients -> the centred CRT value mod q0 q1 (or mod q0), saturated to +-(2^63-1):
// the host arithmetic of aesfhe_decrypt in 128-bit integers.
__global__ void k_dec_crt(const uint64_t* __restrict__ t0, const uint64_t* __restrict__ t1, long cnt, uint64_t q0,
                          uint64_t q1, uint64_t q0inv_mod_q1, int64_t* __restrict__ out) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cnt) return;
    const uint64_t r0 = t0[i];
    if (!t1) {
        out[i] = r0 > q0 / 2 ? (int64_t)r0 - (int64_t)q0 : (int64_t)r0;
        return;
    }
    typedef unsigned __int128 u128;
    const uint64_t r1 = t1[i];
    const uint64_t r0m = r0 % q1;
    const uint64_t diff = r1 >= r0m ? r1 - r0m : r1 + q1 - r0m;
    const uint64_t d = (uint64_t)(((u128)diff * q0inv_mod_q1) % q1);
    const u128 Q = (u128)q0 * q1;
    const u128 x = (u128)r0 + (u128)q0 * d;
    const u128 imax = (u128)INT64_MAX;
    if (x > Q / 2) {
        const u128 m = Q - x;
        out[i] = m > imax ? -INT64_MAX : -(int64_t)m;
    } else {
        out[i] = x > imax ? INT64_MAX : (int64_t)x;
    }
}

}  // namespace aesfhe
