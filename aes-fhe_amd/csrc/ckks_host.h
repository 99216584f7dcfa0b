// ckks_host.h -- host-side pieces of the MI355X CKKS engine: 64-bit modular helpers, the
// deterministic prime chain, root selection, the counter-based PRNG (also used on device)
// and the canonical-embedding codec.  Every integer / floating-point choice here follows the
// specification in DESIGN.md section 3, which the CPU oracle (oracle/ckks_oracle.c) restates
// independently; tests/test_abi.py checks the two agree bit for bit.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#ifndef AESFHE_HD
#define AESFHE_HD
#endif

namespace aesfhe {

using u64 = uint64_t;
using i64 = int64_t;
using u128 = unsigned __int128;

// ---------------------------------------------------------------------------------------------
// host modular arithmetic (setup only; the device uses the fp64-quotient form in kernels.h)
inline u64 h_mulmod(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
inline u64 h_addmod(u64 a, u64 b, u64 q) { u64 s = a + b; return s >= q ? s - q : s; }
inline u64 h_submod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }
inline u64 h_powmod(u64 a, u64 e, u64 q) {
    u64 r = 1 % q;
    a %= q;
    while (e) {
        if (e & 1) r = h_mulmod(r, a, q);
        a = h_mulmod(a, a, q);
        e >>= 1;
    }
    return r;
}
inline u64 h_invmod(u64 a, u64 q) { return h_powmod(a, q - 2, q); }
inline u64 h_smod(i64 a, u64 q) {
    if (a >= 0) return (u64)a % q;
    u64 r = (u64)(-(a + 1)) % q;
    return q - 1 - r;
}

inline bool is_prime_u64(u64 n) {
    if (n < 2) return false;
    static const u64 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (u64 p : small) {
        if (n == p) return true;
        if (n % p == 0) return false;
    }
    u64 d = n - 1;
    int s = 0;
    while (!(d & 1)) { d >>= 1; s++; }
    for (u64 a : small) {
        u64 x = h_powmod(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool comp = true;
        for (int r = 1; r < s; r++) {
            x = h_mulmod(x, x, n);
            if (x == n - 1) { comp = false; break; }
        }
        if (comp) return false;
    }
    return true;
}

inline unsigned bit_reverse(unsigned x, int bits) {
    unsigned r = 0;
    for (int i = 0; i < bits; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

// ---------------------------------------------------------------------------------------------
// counter-based PRNG.  rnd(K, label, idx) = 64-bit word idx mod 8 of the
// ChaCha20 block (RFC 7539 rounds; the original 64-bit counter / 64-bit nonce layout) keyed by the
// engine's 256-bit key K, nonce = the stream label, block counter = idx / 8.  Labels are public
// domain separators (derive: SplitMix64 mixing of key seeds, purposes and nonces); every secret and
// every error / mask sample comes from ChaCha20 under K, so its strength rests on K's entropy
// (256 bits from the OS for an unseeded engine; an explicit 64-bit seed is for reproducible tests).
struct ChaKey {
    uint32_t k[8];
};
AESFHE_HD inline uint32_t cc_rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define AESFHE_QR(a, b, c, d)                 \
    a += b, d ^= a, d = cc_rotl(d, 16);       \
    c += d, b ^= c, b = cc_rotl(b, 12);       \
    a += b, d ^= a, d = cc_rotl(d, 8);        \
    c += d, b ^= c, b = cc_rotl(b, 7)
AESFHE_HD inline void chacha20_block(const ChaKey& K, u64 label, u64 ctr, uint32_t out[16]) {
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                      K.k[0], K.k[1], K.k[2], K.k[3], K.k[4], K.k[5], K.k[6], K.k[7],
                      (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)label, (uint32_t)(label >> 32)};
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = x[i];
    for (int r = 0; r < 10; r++) {
        AESFHE_QR(w[0], w[4], w[8], w[12]);
        AESFHE_QR(w[1], w[5], w[9], w[13]);
        AESFHE_QR(w[2], w[6], w[10], w[14]);
        AESFHE_QR(w[3], w[7], w[11], w[15]);
        AESFHE_QR(w[0], w[5], w[10], w[15]);
        AESFHE_QR(w[1], w[6], w[11], w[12]);
        AESFHE_QR(w[2], w[7], w[8], w[13]);
        AESFHE_QR(w[3], w[4], w[9], w[14]);
    }
    for (int i = 0; i < 16; i++) out[i] = w[i] + x[i];
}
#undef AESFHE_QR
AESFHE_HD inline u64 rnd(const ChaKey& K, u64 label, u64 idx) {
    uint32_t o[16];
    chacha20_block(K, label, idx >> 3, o);
    const int w = (int)(idx & 7);
    return (u64)o[2 * w] | ((u64)o[2 * w + 1] << 32);
}
// engine key from the engine seed words (seed, ext[0..2]) as little-endian 32-bit halves
inline ChaKey chacha_key(u64 seed, const u64* ext) {
    ChaKey K;
    const u64 w[4] = {seed, ext ? ext[0] : 0, ext ? ext[1] : 0, ext ? ext[2] : 0};
    for (int i = 0; i < 4; i++) {
        K.k[2 * i] = (uint32_t)w[i];
        K.k[2 * i + 1] = (uint32_t)(w[i] >> 32);
    }
    return K;
}
AESFHE_HD inline u64 mix64(u64 z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
AESFHE_HD inline u64 derive(u64 a, u64 b) { return mix64(a ^ mix64(b)); }
AESFHE_HD inline i64 ternary(u64 r) {
    u64 t = r % 3;
    return t == 0 ? 0 : (t == 1 ? 1 : -1);
}
AESFHE_HD inline i64 cbd21(u64 r) {
    return (i64)__builtin_popcountll(r & 0x1FFFFFULL) - (i64)__builtin_popcountll((r >> 21) & 0x1FFFFFULL);
}

// ---------------------------------------------------------------------------------------------
// prime chain: q_0 = largest prime < 2^base_bits, specials = largest primes
// < 2^special_bits, q_L..q_1 picked greedily closest to the running canonical scale Delta_l,
// Delta_{l-1} = Delta_l^2 / q_l.  All primes == 1 mod 2N.
struct Chain {
    std::vector<u64> q;       // q_0..q_L, p_0..p_{K-1}
    std::vector<double> scale;  // Delta_0..Delta_L
};

// Hybrid key switching keeps its error small only while every digit's modulus Q_j stays below
// P (the ModDown divides the digit's inner-product error by P): digits of A primes of q (chain q_0
// .. q_{Lp1-1}, then the K special primes) checked by their bit sizes.  Applied to digits wider
// than K (aesfhe_params.digit_primes > K); the default digits of K primes are accepted as before.
// The oracle applies the same rule (ckks_oracle.c digits_below_p).
inline bool digits_below_p(const std::vector<uint64_t>& q, int Lp1, int K, int A) {
    double logp = 0.0;
    for (int k = 0; k < K; k++) logp += std::log2((double)q[Lp1 + k]);
    for (int lo = 0; lo < Lp1; lo += A) {
        double lq = 0.0;
        for (int i = lo; i < lo + A && i < Lp1; i++) lq += std::log2((double)q[i]);
        if (lq > logp) return false;
    }
    return true;
}

inline Chain make_chain(int logN, int L, int K, int base_bits, int special_bits, int scale_bits) {
    const u64 M = 2ULL << logN;
    Chain c;
    c.q.assign(L + 1 + K, 0);
    c.scale.assign(L + 1, 0.0);
    std::vector<u64> used;
    auto dup = [&](u64 x) { for (u64 u : used) if (u == x) return true; return false; };
    {
        u64 k = ((1ULL << base_bits) - 2) / M;
        for (;; k--) {
            u64 cand = k * M + 1;
            if (is_prime_u64(cand)) { c.q[0] = cand; used.push_back(cand); break; }
            if (k == 1) throw std::runtime_error("no base prime");
        }
    }
    {
        u64 k = ((1ULL << special_bits) - 2) / M;
        int got = 0;
        for (; got < K; k--) {
            u64 cand = k * M + 1;
            if (!dup(cand) && is_prime_u64(cand)) { c.q[L + 1 + got] = cand; used.push_back(cand); got++; }
            if (k == 1) throw std::runtime_error("no special prime");
        }
    }
    c.scale[L] = std::ldexp(1.0, scale_bits);
    for (int l = L; l >= 1; l--) {
        double target = c.scale[l];
        u64 k0 = (u64)std::floor((target - 1.0) / (double)M);
        u64 up = 0, dn = 0;
        for (u64 k = k0 + 1;; k++) {
            u64 cand = k * M + 1;
            if (!dup(cand) && is_prime_u64(cand)) { up = cand; break; }
        }
        for (u64 k = k0; k >= 1; k--) {
            u64 cand = k * M + 1;
            if (!dup(cand) && is_prime_u64(cand)) { dn = cand; break; }
        }
        u64 pick;
        if (!dn) pick = up;
        else {
            double du = (double)up - target, dd = target - (double)dn;
            pick = (du < dd) ? up : dn;
        }
        c.q[l] = pick;
        used.push_back(pick);
        c.scale[l - 1] = c.scale[l] * c.scale[l] / (double)pick;
    }
    return c;
}

inline std::vector<double> scales_from_primes(const std::vector<u64>& q, int L, int scale_bits) {
    std::vector<double> s(L + 1);
    s[L] = std::ldexp(1.0, scale_bits);
    for (int l = L; l >= 1; l--) s[l - 1] = s[l] * s[l] / (double)q[l];
    return s;
}

// minimal primitive 2N-th root of unity modulo q
inline u64 min_primitive_root(u64 q, int N) {
    const u64 M = 2 * (u64)N;
    u64 psi0 = 0;
    for (u64 g = 2;; g++) {
        psi0 = h_powmod(g, (q - 1) / M, q);
        if (h_powmod(psi0, (u64)N, q) == q - 1) break;
    }
    u64 best = psi0, cur = psi0, sq = h_mulmod(psi0, psi0, q);
    for (int i = 0; i < N; i++) {
        if (cur < best) best = cur;
        cur = h_mulmod(cur, sq, q);
    }
    return best;
}

// ---------------------------------------------------------------------------------------------
// canonical-embedding codec: HEAAN special FFT.  Explicit real arithmetic in a
// fixed order; compiled with -ffp-contract=off so it matches the oracle bit for bit.
struct Codec {
    int logN = 0, n = 0;
    long M = 0;
    std::vector<double> kre, kim;
    std::vector<long> rot;

    explicit Codec(int logN_) : logN(logN_) {
        long N = 1L << logN;
        n = (int)(N / 2);
        M = 2 * N;
        kre.resize(M + 1);
        kim.resize(M + 1);
        // libm cos/sin through volatile pointers: never fused into sincos() (its last bit can
        // differ), so the table matches the oracle's bit for bit
        double (*volatile fcos)(double) = ::cos;
        double (*volatile fsin)(double) = ::sin;
        for (long j = 0; j <= M; j++) {
            double ang = 2.0 * M_PI * (double)j / (double)M;
            kre[j] = fcos(ang);
            kim[j] = fsin(ang);
        }
        rot.resize(n);
        long g = 1;
        for (int j = 0; j < n; j++) { rot[j] = g; g = (g * 5) % M; }
    }

    static void bitrev(double* re, double* im, int n) {
        for (int i = 1, j = 0; i < n; ++i) {
            int bit = n >> 1;
            for (; j >= bit; bit >>= 1) j -= bit;
            j += bit;
            if (i < j) {
                double t = re[i]; re[i] = re[j]; re[j] = t;
                t = im[i]; im[i] = im[j]; im[j] = t;
            }
        }
    }

    void special_inv(double* re, double* im) const {
        for (int len = n; len >= 1; len >>= 1) {
            for (int i = 0; i < n; i += len) {
                int lenh = len >> 1;
                long lenq = (long)len << 2;
                for (int j = 0; j < lenh; ++j) {
                    long idx = (lenq - (rot[j] % lenq)) * M / lenq;
                    double ur = re[i + j] + re[i + j + lenh], ui = im[i + j] + im[i + j + lenh];
                    double vr = re[i + j] - re[i + j + lenh], vi = im[i + j] - im[i + j + lenh];
                    double wr = kre[idx], wi = kim[idx];
                    double tr = vr * wr - vi * wi, ti = vr * wi + vi * wr;
                    re[i + j] = ur; im[i + j] = ui;
                    re[i + j + lenh] = tr; im[i + j + lenh] = ti;
                }
            }
        }
        bitrev(re, im, n);
        for (int i = 0; i < n; i++) { re[i] /= (double)n; im[i] /= (double)n; }
    }

    void special(double* re, double* im) const {
        bitrev(re, im, n);
        for (int len = 2; len <= n; len <<= 1) {
            for (int i = 0; i < n; i += len) {
                int lenh = len >> 1;
                long lenq = (long)len << 2;
                for (int j = 0; j < lenh; ++j) {
                    long idx = (rot[j] % lenq) * M / lenq;
                    double ur = re[i + j], ui = im[i + j];
                    double xr = re[i + j + lenh], xi = im[i + j + lenh];
                    double wr = kre[idx], wi = kim[idx];
                    double vr = xr * wr - xi * wi, vi = xr * wi + xi * wr;
                    re[i + j] = ur + vr; im[i + j] = ui + vi;
                    re[i + j + lenh] = ur - vr; im[i + j + lenh] = ui - vi;
                }
            }
        }
    }
};

}  // namespace aesfhe
