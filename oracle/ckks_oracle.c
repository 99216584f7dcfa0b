/*
 * ckks_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the RNS-CKKS engine that the
 * reference (songhayeong/aes-fhe) reaches through `desilofhe.Engine`.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline -- never as the product path (the product is
 * aes-fhe_amd/csrc, HIP for gfx950, which fails loudly when its extension is missing).
 *
 * What it restates.  desilofhe is a closed, unpinned third-party binary that is absent from
 * /root/reference (imported at engine_context.py:6, xor_service.py:12,69, new.py:6,
 * gf_service.py:7) and cannot be fetched here.  Its published algorithm is RNS-CKKS
 * (Cheon-Kim-Kim-Song 2017; full-RNS variant Cheon-Han-Kim-Kim-Song 2018) with hybrid key
 * switching (Han-Ki 2020).  This file restates exactly that algorithm, with every integer
 * choice (prime chain, roots, NTT ordering, PRNG streams, fast base conversion, rounding in
 * rescale) fixed by the specification in DESIGN.md section 3 so that the HIP engine must
 * reproduce it residue-for-residue.
 *
 * How it is pinned (parity is NOT unpinned):
 *   - the reference's own engine-contract tests: enc/dec identity atol 1e-6
 *     (test/test_engine_rot.py:21-29), rotate(ct,k) == np.roll(v,k) (:32-40), relinearize
 *     no-op on 2-poly (:43-50), square after relin atol 1e-5 (:53-61) -> tests/test_oracle_ckks.py;
 *   - NTT known answers against big-integer schoolbook negacyclic convolution;
 *   - the reference services' decoded outputs (xor_service.py:271-286, sbox_service.py:116-138,
 *     new.py:186-227) captured as golden fixtures in tests/golden/ from the reference's Python
 *     run over an exact-arithmetic stand-in of desilofhe (tests/golden/make_golden.py).
 *
 * Plain C11, 64-bit words, unsigned __int128 products.  OpenMP over limbs.
 */
#include "../include/aesfhe.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef uint64_t u64;
typedef int64_t i64;
typedef unsigned __int128 u128;

#define MAXP 96

/* ------------------------------------------------------------------------------------------ */
/* errors                                                                                      */
static __thread char g_err[512];

static int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

const char *aesfhe_last_error(void) { return g_err; }
const char *aesfhe_backend_name(void) { return "oracle-cpu"; }
int32_t aesfhe_abi_version(void) { return AESFHE_ABI_VERSION; }

/* ------------------------------------------------------------------------------------------ */
/* modular arithmetic                                                                          */
static inline u64 add_mod(u64 a, u64 b, u64 q) {
    u64 s = a + b;
    return s >= q ? s - q : s;
}
static inline u64 sub_mod(u64 a, u64 b, u64 q) { return a >= b ? a - b : a + q - b; }
static inline u64 mul_mod_slow(u64 a, u64 b, u64 q) { return (u64)(((u128)a * b) % q); }
static u64 pow_mod(u64 a, u64 e, u64 q) {
    u64 r = 1 % q;
    a %= q;
    while (e) {
        if (e & 1) r = mul_mod_slow(r, a, q);
        a = mul_mod_slow(a, a, q);
        e >>= 1;
    }
    return r;
}
static u64 inv_mod(u64 a, u64 q) { return pow_mod(a, q - 2, q); }

/* Montgomery multiplication (R = 2^64) for data x data products */
typedef struct {
    u64 q, qinv_neg, r2; /* qinv_neg = -q^{-1} mod 2^64, r2 = 2^128 mod q */
} mont_t;

static inline u64 mont_redc(u128 t, const mont_t *m) {
    u64 lo = (u64)t;
    u64 k = lo * m->qinv_neg;
    u128 s = t + (u128)k * m->q;
    u64 r = (u64)(s >> 64);
    /* t < q*2^64 and k*q < q*2^64 -> s>>64 < 2q */
    return r >= m->q ? r - m->q : r;
}
static inline u64 mul_mod(u64 a, u64 b, const mont_t *m) {
    u64 t = mont_redc((u128)a * b, m);     /* a b R^-1 */
    return mont_redc((u128)t * m->r2, m);  /* a b */
}
static void mont_init(mont_t *m, u64 q) {
    m->q = q;
    u64 inv = 1; /* Newton iteration for q^{-1} mod 2^64 */
    for (int i = 0; i < 7; i++) inv *= 2 - q * inv;
    m->qinv_neg = (u64)0 - inv;
    u64 r1 = (u64)(((u128)1 << 64) % q);
    m->r2 = mul_mod_slow(r1, r1, q);
}

/* Shoup multiplication by a fixed operand w (wp = floor(w 2^64 / q)) */
static inline u64 shoup_pre(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
static inline u64 mul_shoup(u64 a, u64 w, u64 wp, u64 q) {
    u64 qh = (u64)(((u128)a * wp) >> 64);
    u64 r = a * w - qh * q;
    return r >= q ? r - q : r;
}

static u64 smod(i64 a, u64 q) {
    if (a >= 0) return (u64)a % q;
    u64 r = (u64)(-(a + 1)) % q; /* avoids overflow at INT64_MIN */
    r = q - 1 - r;
    return r;
}

/* deterministic Miller-Rabin for 64-bit */
static int is_prime(u64 n) {
    if (n < 2) return 0;
    static const u64 small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (int i = 0; i < 12; i++) {
        if (n == small[i]) return 1;
        if (n % small[i] == 0) return 0;
    }
    u64 d = n - 1;
    int s = 0;
    while (!(d & 1)) {
        d >>= 1;
        s++;
    }
    for (int i = 0; i < 12; i++) {
        u64 x = pow_mod(small[i], d, n);
        if (x == 1 || x == n - 1) continue;
        int comp = 1;
        for (int r = 1; r < s; r++) {
            x = mul_mod_slow(x, x, n);
            if (x == n - 1) {
                comp = 0;
                break;
            }
        }
        if (comp) return 0;
    }
    return 1;
}

static unsigned brv(unsigned x, int bits) {
    unsigned r = 0;
    for (int i = 0; i < bits; i++) {
        r = (r << 1) | (x & 1);
        x >>= 1;
    }
    return r;
}

/* ------------------------------------------------------------------------------------------ */
/* PRNG: counter-based, shared bit-for-bit with the HIP engine: rnd(K, label, idx)
 * = 64-bit word idx mod 8 of the ChaCha20 block (20 rounds, RFC 7539 quarter round; the original
 * 64-bit counter / 64-bit nonce layout) under the engine's 256-bit key K, nonce = label, counter =
 * idx / 8.  A one-block cache per thread serves the sequential loops (7 of 8 words).             */
#define CC_ROTL(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
#define CC_QR(a, b, c, d)                                   \
    do {                                                    \
        a += b; d ^= a; d = CC_ROTL(d, 16);                 \
        c += d; b ^= c; b = CC_ROTL(b, 12);                 \
        a += b; d ^= a; d = CC_ROTL(d, 8);                  \
        c += d; b ^= c; b = CC_ROTL(b, 7);                  \
    } while (0)
static void chacha20_block(const uint32_t k[8], u64 label, u64 ctr, uint32_t out[16]) {
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                      k[4], k[5], k[6], k[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)label,
                      (uint32_t)(label >> 32)};
    uint32_t w[16];
    for (int i = 0; i < 16; i++) w[i] = x[i];
    for (int r = 0; r < 10; r++) {
        CC_QR(w[0], w[4], w[8], w[12]);
        CC_QR(w[1], w[5], w[9], w[13]);
        CC_QR(w[2], w[6], w[10], w[14]);
        CC_QR(w[3], w[7], w[11], w[15]);
        CC_QR(w[0], w[5], w[10], w[15]);
        CC_QR(w[1], w[6], w[11], w[12]);
        CC_QR(w[2], w[7], w[8], w[13]);
        CC_QR(w[3], w[4], w[9], w[14]);
    }
    for (int i = 0; i < 16; i++) out[i] = w[i] + x[i];
}
/* one cached block per thread, keyed by the key's words (not its address: a freed engine's key
 * storage can be reused by a new engine with another key) */
static __thread struct {
    uint32_t k[8];
    u64 label, ctr;
    int valid;
    uint32_t w[16];
} cc_cache;
static u64 rnd(const uint32_t k[8], u64 label, u64 idx) {
    const u64 ctr = idx >> 3;
    if (!cc_cache.valid || cc_cache.label != label || cc_cache.ctr != ctr || memcmp(cc_cache.k, k, sizeof cc_cache.k)) {
        chacha20_block(k, label, ctr, cc_cache.w);
        memcpy(cc_cache.k, k, sizeof cc_cache.k);
        cc_cache.label = label;
        cc_cache.ctr = ctr;
        cc_cache.valid = 1;
    }
    const int j = (int)(idx & 7);
    return (u64)cc_cache.w[2 * j] | ((u64)cc_cache.w[2 * j + 1] << 32);
}
/* stream labels: SplitMix64 mixing of key seeds, purposes and nonces (public domain separators) */
static inline u64 mix64(u64 z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static inline u64 derive(u64 a, u64 b) { return mix64(a ^ mix64(b)); }
static inline i64 ternary(u64 r) {
    u64 t = r % 3;
    return t == 0 ? 0 : (t == 1 ? 1 : -1);
}
static inline i64 cbd21(u64 r) {
    return (i64)__builtin_popcountll(r & 0x1FFFFFULL) -
           (i64)__builtin_popcountll((r >> 21) & 0x1FFFFFULL);
}
static inline u64 uniform_mod(u64 r, u64 q) { return (u64)(((u128)r * q) >> 64); }

/* ------------------------------------------------------------------------------------------ */
/* engine                                                                                      */
struct aesfhe_engine {
    int logN, N, L, K, A, dnum, np; /* np = L+1+K; A = key-switch digit width (alpha) */
    u64 q[MAXP];
    double scales[MAXP];
    mont_t mont[MAXP];
    u64 *psi[MAXP], *psip[MAXP];   /* psi^{brv(k)} and Shoup companions */
    u64 *ipsi[MAXP], *ipsip[MAXP]; /* psi^{-brv(k)} */
    u64 ninv[MAXP], ninvp[MAXP];
    u64 iroot[MAXP]; /* psi^{N/2}: a square root of -1 */
    u64 seed;
    uint32_t ck[8]; /* ChaCha20 key of every random stream */
    int threads;
    int profiling;
    double prof_ms[3];
    int64_t prof_n[3];
};

struct aesfhe_key {
    int kind; /* 0 sk 1 pk 2 relin 3 galois */
    u64 galois;
    u64 keyseed;
    u64 *data;
    int ndig; /* switching keys: digits stored (dnum, or fewer after aesfhe_key_trim) */
};

struct aesfhe_ct {
    int B, npoly, level, is_zero;
    u64 *data; /* [B][npoly][level+1][N] */
};

struct aesfhe_pt {
    int level;
    int ext;   /* 1: K special limbs follow (aesfhe_pt_create_ext) */
    u64 *data; /* [level+1 (+K)][N] */
};

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* prime chain generation -- DESIGN.md 3.1 (must match the HIP engine bit for bit) */
static int gen_primes(aesfhe_engine *e, int base_bits, int special_bits, int scale_bits) {
    const u64 M = 2 * (u64)e->N;
    int used = 0;
    u64 list[MAXP];
    /* q_0: largest prime < 2^base_bits, == 1 mod 2N */
    {
        u64 k = (((u64)1 << base_bits) - 2) / M;
        for (;; k--) {
            u64 c = k * M + 1;
            if (is_prime(c)) {
                e->q[0] = c;
                list[used++] = c;
                break;
            }
            if (k == 1) return fail(AESFHE_EARG, "no base prime");
        }
    }
    /* special primes: largest primes < 2^special_bits, distinct */
    {
        u64 k = (((u64)1 << special_bits) - 2) / M;
        int got = 0;
        for (; got < e->K; k--) {
            u64 c = k * M + 1;
            int dup = 0;
            for (int j = 0; j < used; j++) dup |= list[j] == c;
            if (!dup && is_prime(c)) {
                e->q[e->L + 1 + got] = c;
                list[used++] = c;
                got++;
            }
            if (k == 1) return fail(AESFHE_EARG, "no special prime");
        }
    }
    /* scaling primes q_L..q_1 chosen greedily to track Delta_l */
    e->scales[e->L] = ldexp(1.0, scale_bits);
    for (int l = e->L; l >= 1; l--) {
        double target = e->scales[l];
        u64 k0 = (u64)floor((target - 1.0) / (double)M);
        u64 up = 0, dn = 0;
        for (u64 k = k0 + 1;; k++) {
            u64 c = k * M + 1;
            int dup = 0;
            for (int j = 0; j < used; j++) dup |= list[j] == c;
            if (!dup && is_prime(c)) {
                up = c;
                break;
            }
        }
        for (u64 k = k0; k >= 1; k--) {
            u64 c = k * M + 1;
            int dup = 0;
            for (int j = 0; j < used; j++) dup |= list[j] == c;
            if (!dup && is_prime(c)) {
                dn = c;
                break;
            }
        }
        u64 pick;
        if (!dn) pick = up;
        else {
            double du = (double)up - target, dd = target - (double)dn;
            pick = (du < dd) ? up : dn;
        }
        e->q[l] = pick;
        list[used++] = pick;
        e->scales[l - 1] = e->scales[l] * e->scales[l] / (double)pick;
    }
    return 0;
}

static void derive_scales(aesfhe_engine *e, int scale_bits) {
    e->scales[e->L] = ldexp(1.0, scale_bits);
    for (int l = e->L; l >= 1; l--) e->scales[l - 1] = e->scales[l] * e->scales[l] / (double)e->q[l];
}

/* minimal primitive 2N-th root of unity -- DESIGN.md 3.2 */
static u64 min_root(u64 q, int N) {
    u64 M = 2 * (u64)N, psi0 = 0;
    for (u64 g = 2;; g++) {
        psi0 = pow_mod(g, (q - 1) / M, q);
        if (pow_mod(psi0, (u64)N, q) == q - 1) break;
    }
    u64 best = psi0, cur = psi0, sq = mul_mod_slow(psi0, psi0, q);
    for (int i = 0; i < N; i++) {
        if (cur < best) best = cur;
        cur = mul_mod_slow(cur, sq, q);
    }
    return best;
}

static void build_tables(aesfhe_engine *e) {
    const int N = e->N;
    for (int p = 0; p < e->np; p++) {
        u64 q = e->q[p];
        mont_init(&e->mont[p], q);
        u64 psi = min_root(q, N), ip = inv_mod(psi, q);
        e->psi[p] = malloc(sizeof(u64) * N);
        e->psip[p] = malloc(sizeof(u64) * N);
        e->ipsi[p] = malloc(sizeof(u64) * N);
        e->ipsip[p] = malloc(sizeof(u64) * N);
        u64 *pw = malloc(sizeof(u64) * N), *ipw = malloc(sizeof(u64) * N);
        pw[0] = 1;
        ipw[0] = 1;
        for (int k = 1; k < N; k++) {
            pw[k] = mul_mod_slow(pw[k - 1], psi, q);
            ipw[k] = mul_mod_slow(ipw[k - 1], ip, q);
        }
        for (int k = 0; k < N; k++) {
            unsigned r = brv((unsigned)k, e->logN);
            e->psi[p][k] = pw[r];
            e->ipsi[p][k] = ipw[r];
            e->psip[p][k] = shoup_pre(pw[r], q);
            e->ipsip[p][k] = shoup_pre(ipw[r], q);
        }
        e->iroot[p] = pw[N / 2];
        free(pw);
        free(ipw);
        e->ninv[p] = inv_mod((u64)N, q);
        e->ninvp[p] = shoup_pre(e->ninv[p], q);
    }
}

/* forward negacyclic NTT, natural -> bit-reversed (Cooley-Tukey, merged psi) */
static void ntt_fwd(const aesfhe_engine *e, u64 *a, int p) {
    const int N = e->N;
    const u64 q = e->q[p];
    const u64 *w = e->psi[p], *wp = e->psip[p];
    int t = N;
    for (int m = 1; m < N; m <<= 1) {
        t >>= 1;
        for (int i = 0; i < m; i++) {
            int j1 = 2 * i * t;
            u64 S = w[m + i], Sp = wp[m + i];
            for (int j = j1; j < j1 + t; j++) {
                u64 U = a[j], V = mul_shoup(a[j + t], S, Sp, q);
                a[j] = add_mod(U, V, q);
                a[j + t] = sub_mod(U, V, q);
            }
        }
    }
}

/* inverse, bit-reversed -> natural (Gentleman-Sande), includes N^{-1} */
static void ntt_inv(const aesfhe_engine *e, u64 *a, int p) {
    const int N = e->N;
    const u64 q = e->q[p];
    const u64 *w = e->ipsi[p], *wp = e->ipsip[p];
    int t = 1;
    for (int m = N; m > 1; m >>= 1) {
        int h = m >> 1, j1 = 0;
        for (int i = 0; i < h; i++) {
            u64 S = w[h + i], Sp = wp[h + i];
            for (int j = j1; j < j1 + t; j++) {
                u64 U = a[j], V = a[j + t];
                a[j] = add_mod(U, V, q);
                a[j + t] = mul_shoup(sub_mod(U, V, q), S, Sp, q);
            }
            j1 += 2 * t;
        }
        t <<= 1;
    }
    for (int j = 0; j < N; j++) a[j] = mul_shoup(a[j], e->ninv[p], e->ninvp[p], q);
}

static void prof_add(aesfhe_engine *e, int fam, double ms) {
    if (!((e->profiling >> fam) & 1)) return;
    e->prof_ms[fam] += ms;
    e->prof_n[fam] += 1;
}

/* Hybrid key switching keeps its error small only while every digit's modulus Q_j (A primes of
 * the chain) stays below P, the product of the K special primes (engine: ckks_host.h
 * digits_below_p, the same rule on the same bit sizes); checked for digits wider than K. */
static int digits_below_p(const aesfhe_engine *e) {
    const int Lp1 = e->L + 1;
    double logp = 0.0;
    for (int k = 0; k < e->K; k++) logp += log2((double)e->q[Lp1 + k]);
    for (int lo = 0; lo < Lp1; lo += e->A) {
        double lq = 0.0;
        for (int i = lo; i < lo + e->A && i < Lp1; i++) lq += log2((double)e->q[i]);
        if (lq > logp) return 0;
    }
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
int aesfhe_engine_create(const aesfhe_params *pp, aesfhe_engine **out) {
    if (!pp || !out) return fail(AESFHE_EARG, "null argument");
    if (pp->log_n < 4 || pp->log_n > 17) return fail(AESFHE_EARG, "log_n out of range");
    if (pp->max_level < 1 || pp->special_primes < 1 || pp->max_level + 1 + pp->special_primes > MAXP)
        return fail(AESFHE_EARG, "bad level / special prime count");
    if (pp->scale_bits < 20 || pp->scale_bits > 60 || pp->base_bits > 61 || pp->special_bits > 61)
        return fail(AESFHE_EARG, "bad bit sizes");
    aesfhe_engine *e = calloc(1, sizeof *e);
    e->logN = pp->log_n;
    e->N = 1 << pp->log_n;
    e->L = pp->max_level;
    e->K = pp->special_primes;
    e->np = e->L + 1 + e->K;
    e->A = pp->digit_primes > 0 ? pp->digit_primes : e->K;
    if (e->A > 16) {
        free(e);
        return fail(AESFHE_EARG, "key-switch digit width %d outside 1..16", pp->digit_primes);
    }
    e->dnum = (e->L + 1 + e->A - 1) / e->A;
    e->seed = pp->seed;
    {
        const u64 w[4] = {pp->seed, pp->seed_ext[0], pp->seed_ext[1], pp->seed_ext[2]};
        for (int i = 0; i < 4; i++) {
            e->ck[2 * i] = (uint32_t)w[i];
            e->ck[2 * i + 1] = (uint32_t)(w[i] >> 32);
        }
    }
    e->threads = pp->threads;
#ifdef _OPENMP
    /* per-engine thread count (num_threads on every parallel loop): never the process-wide
     * omp_set_num_threads, which would leak one engine's setting into every other engine */
    if (e->threads <= 0) e->threads = omp_get_max_threads();
#endif
    if (pp->primes) {
        for (int i = 0; i < e->np; i++) e->q[i] = pp->primes[i];
        derive_scales(e, pp->scale_bits);
    } else {
        int rc = gen_primes(e, pp->base_bits, pp->special_bits, pp->scale_bits);
        if (rc) {
            free(e);
            return rc;
        }
    }
    if (e->A > e->K && !digits_below_p(e)) {
        int A = e->A, K = e->K;
        free(e);
        return fail(AESFHE_EARG, "a key-switch digit of %d primes exceeds P (%d special primes)", A, K);
    }
    build_tables(e);
    *out = e;
    return 0;
}

int aesfhe_chain(const aesfhe_params *pp, uint64_t *primes, double *scales) {
    aesfhe_engine tmp;
    memset(&tmp, 0, sizeof tmp);
    tmp.logN = pp->log_n;
    tmp.N = 1 << pp->log_n;
    tmp.L = pp->max_level;
    tmp.K = pp->special_primes;
    tmp.np = tmp.L + 1 + tmp.K;
    if (tmp.np > MAXP) return fail(AESFHE_EARG, "too many primes");
    int rc = gen_primes(&tmp, pp->base_bits, pp->special_bits, pp->scale_bits);
    if (rc) return rc;
    memcpy(primes, tmp.q, sizeof(u64) * tmp.np);
    memcpy(scales, tmp.scales, sizeof(double) * (tmp.L + 1));
    return 0;
}

void aesfhe_engine_destroy(aesfhe_engine *e) {
    if (!e) return;
    for (int p = 0; p < e->np; p++) {
        free(e->psi[p]);
        free(e->psip[p]);
        free(e->ipsi[p]);
        free(e->ipsip[p]);
    }
    free(e);
}

int aesfhe_engine_dims(const aesfhe_engine *e, int32_t d[4]) {
    d[0] = e->logN;
    d[1] = e->L;
    d[2] = e->K;
    d[3] = e->dnum;
    return 0;
}
int aesfhe_engine_primes(const aesfhe_engine *e, uint64_t *o) {
    memcpy(o, e->q, sizeof(u64) * e->np);
    return 0;
}
int aesfhe_engine_scales(const aesfhe_engine *e, double *o) {
    memcpy(o, e->scales, sizeof(double) * (e->L + 1));
    return 0;
}
double aesfhe_engine_mul_scale(const aesfhe_engine *e, int32_t l) {
    if (l < 1 || l > e->L) return 0.0;
    return e->scales[l - 1] * (double)e->q[l] / e->scales[l];
}
int aesfhe_engine_sync(aesfhe_engine *e) {
    (void)e;
    return 0;
}
int aesfhe_engine_profile(aesfhe_engine *e, int32_t en) {
    e->profiling = en == -1 ? 7 : (en & 7);
    if (en) {
        memset(e->prof_ms, 0, sizeof e->prof_ms);
        memset(e->prof_n, 0, sizeof e->prof_n);
    }
    return 0;
}
int aesfhe_engine_profile_read(aesfhe_engine *e, const char *fam, int64_t *n, double *ms,
                               double *bytes) {
    int f = !strcmp(fam, "ntt") ? 0 : !strcmp(fam, "keyswitch") ? 1 : 2;
    *n = e->prof_n[f];
    *ms = e->prof_ms[f];
    if (bytes) *bytes = 0;
    return 0;
}
int aesfhe_engine_profile_kernels(aesfhe_engine *e, char *buf, int64_t cap, int64_t *need) {
    (void)e;
    if (need) *need = 3;
    if (buf && cap >= 3) memcpy(buf, "{}", 3);
    return 0;
}
int64_t aesfhe_engine_device_bytes(const aesfhe_engine *e) {
    (void)e;
    return 0;
}
int aesfhe_engine_pool_trim(aesfhe_engine *e) { return e ? 0 : fail(AESFHE_EARG, "null engine"); }
int aesfhe_engine_pool_stats(const aesfhe_engine *e, int64_t *out) {
    (void)e;
    if (!out) return AESFHE_EARG;
    for (int i = 0; i < 7; i++) out[i] = 0;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* host codec: HEAAN special FFT.  Explicit re/im arithmetic, no FMA.          */
typedef struct {
    int logN;
    int n;
    long M;
    double *kre, *kim;
    long *rot;
} codec_t;

static void codec_init(codec_t *c, int logN) {
    c->logN = logN;
    long N = 1L << logN;
    c->n = (int)(N / 2);
    c->M = 2 * N;
    c->kre = malloc(sizeof(double) * (c->M + 1));
    c->kim = malloc(sizeof(double) * (c->M + 1));
    /* called through volatile pointers so no compiler fuses them into sincos(), whose last
       bit can differ: the HIP engine's host codec must produce the same table */
    double (*volatile fcos)(double) = cos;
    double (*volatile fsin)(double) = sin;
    for (long j = 0; j <= c->M; j++) {
        double ang = 2.0 * M_PI * (double)j / (double)c->M;
        c->kre[j] = fcos(ang);
        c->kim[j] = fsin(ang);
    }
    c->rot = malloc(sizeof(long) * c->n);
    long g = 1;
    for (int j = 0; j < c->n; j++) {
        c->rot[j] = g;
        g = (g * 5) % c->M;
    }
}
static void codec_free(codec_t *c) {
    free(c->kre);
    free(c->kim);
    free(c->rot);
}
static void bitrev_cplx(double *re, double *im, int n) {
    for (int i = 1, j = 0; i < n; ++i) {
        int bit = n >> 1;
        for (; j >= bit; bit >>= 1) j -= bit;
        j += bit;
        if (i < j) {
            double t = re[i];
            re[i] = re[j];
            re[j] = t;
            t = im[i];
            im[i] = im[j];
            im[j] = t;
        }
    }
}
static void fft_special_inv(const codec_t *c, double *re, double *im) {
    const int n = c->n;
    for (int len = n; len >= 1; len >>= 1) {
        for (int i = 0; i < n; i += len) {
            int lenh = len >> 1;
            long lenq = (long)len << 2;
            for (int j = 0; j < lenh; ++j) {
                long idx = (lenq - (c->rot[j] % lenq)) * c->M / lenq;
                double ur = re[i + j] + re[i + j + lenh], ui = im[i + j] + im[i + j + lenh];
                double vr = re[i + j] - re[i + j + lenh], vi = im[i + j] - im[i + j + lenh];
                double wr = c->kre[idx], wi = c->kim[idx];
                double tr = vr * wr - vi * wi, ti = vr * wi + vi * wr;
                re[i + j] = ur;
                im[i + j] = ui;
                re[i + j + lenh] = tr;
                im[i + j + lenh] = ti;
            }
        }
    }
    bitrev_cplx(re, im, n);
    for (int i = 0; i < n; i++) {
        re[i] /= (double)n;
        im[i] /= (double)n;
    }
}
static void fft_special(const codec_t *c, double *re, double *im) {
    const int n = c->n;
    bitrev_cplx(re, im, n);
    for (int len = 2; len <= n; len <<= 1) {
        for (int i = 0; i < n; i += len) {
            int lenh = len >> 1;
            long lenq = (long)len << 2;
            for (int j = 0; j < lenh; ++j) {
                long idx = (c->rot[j] % lenq) * c->M / lenq;
                double ur = re[i + j], ui = im[i + j];
                double xr = re[i + j + lenh], xi = im[i + j + lenh];
                double wr = c->kre[idx], wi = c->kim[idx];
                double vr = xr * wr - xi * wi, vi = xr * wi + xi * wr;
                re[i + j] = ur + vr;
                im[i + j] = ui + vi;
                re[i + j + lenh] = ur - vr;
                im[i + j + lenh] = ui - vi;
            }
        }
    }
}

int aesfhe_encode(int32_t logN, const double *re, const double *im, int64_t n_slots,
                  double scale, int64_t *co) {
    if (logN < 2 || logN > 17) return fail(AESFHE_EARG, "log_n out of range");
    codec_t c;
    codec_init(&c, logN);
    if (n_slots < 0 || n_slots > c.n) {
        codec_free(&c);
        return fail(AESFHE_EARG, "too many slots: %lld > %d", (long long)n_slots, c.n);
    }
    double *vr = calloc(c.n, sizeof(double)), *vi = calloc(c.n, sizeof(double));
    for (int64_t i = 0; i < n_slots; i++) {
        vr[i] = re ? re[i] : 0.0;
        vi[i] = im ? im[i] : 0.0;
    }
    fft_special_inv(&c, vr, vi);
    int rc = 0;
    for (int i = 0; i < c.n; i++) {
        double a = vr[i] * scale, b = vi[i] * scale;
        if (!(fabs(a) < 9.0e18) || !(fabs(b) < 9.0e18)) {
            rc = fail(AESFHE_EARG, "encoded coefficient overflows int64 (scale too large?)");
            break;
        }
        co[i] = llround(a);
        co[i + c.n] = llround(b);
    }
    free(vr);
    free(vi);
    codec_free(&c);
    return rc;
}

int aesfhe_decode(int32_t logN, const int64_t *co, double scale, double *re, double *im) {
    if (logN < 2 || logN > 17) return fail(AESFHE_EARG, "log_n out of range");
    codec_t c;
    codec_init(&c, logN);
    for (int i = 0; i < c.n; i++) {
        re[i] = (double)co[i] / scale;
        im[i] = (double)co[i + c.n] / scale;
    }
    fft_special(&c, re, im);
    codec_free(&c);
    return 0;
}

/* The client-path entry points (include/aesfhe.h "device-resident client path"): the oracle's
 * "device" is host memory, so they are the host codec / encryption over B rows. */
int aesfhe_encode_device(aesfhe_engine *e, const double *re, const double *im, int32_t B, int64_t n_slots,
                         int64_t stride, double scale, int64_t *co) {
    if (B < 1 || n_slots < 0 || stride < n_slots || !co) return fail(AESFHE_EARG, "bad encode shape");
    for (int b = 0; b < B; b++) {
        int rc = aesfhe_encode(e->logN, re ? re + (size_t)b * stride : NULL, im ? im + (size_t)b * stride : NULL,
                               n_slots, scale, co + (size_t)b * e->N);
        if (rc) return rc;
    }
    return 0;
}
int aesfhe_decode_device(aesfhe_engine *e, const int64_t *co, int32_t B, double scale, double *re, double *im) {
    if (B < 1 || !co || !re || !im) return fail(AESFHE_EARG, "bad decode arguments");
    const size_t n = (size_t)e->N / 2;
    for (int b = 0; b < B; b++) {
        int rc = aesfhe_decode(e->logN, co + (size_t)b * e->N, scale, re + b * n, im + b * n);
        if (rc) return rc;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* small helpers                                                                               */
static aesfhe_ct *ct_new(const aesfhe_engine *e, int B, int npoly, int level) {
    aesfhe_ct *c = calloc(1, sizeof *c);
    c->B = B;
    c->npoly = npoly;
    c->level = level;
    c->data = calloc((size_t)B * npoly * (level + 1) * e->N, sizeof(u64));
    return c;
}
static inline u64 *limb(const aesfhe_engine *e, const aesfhe_ct *c, int b, int p, int i) {
    return c->data + (((size_t)b * c->npoly + p) * (c->level + 1) + i) * e->N;
}
void aesfhe_ct_free(aesfhe_ct *c) {
    if (!c) return;
    free(c->data);
    free(c);
}
int aesfhe_ct_info(const aesfhe_ct *c, int32_t info[4]) {
    info[0] = c->B;
    info[1] = c->npoly;
    info[2] = c->level;
    info[3] = c->is_zero;
    return 0;
}

/* galois permutation in NTT domain: out[k] = in[idx(k)] with e(idx) = g e(k) mod 2N */
static void galois_perm(const aesfhe_engine *e, const u64 *in, u64 *out, u64 g) {
    const u64 M = 2 * (u64)e->N;
    for (int k = 0; k < e->N; k++) {
        u64 ek = 2 * (u64)brv((unsigned)k, e->logN) + 1;
        u64 t = (g * ek) % M;
        out[k] = in[brv((unsigned)((t - 1) / 2), e->logN)];
    }
}

/* residues of a signed coefficient vector into NTT form for prime p */
static void coeffs_to_ntt(const aesfhe_engine *e, const i64 *co, u64 *dst, int p) {
    for (int k = 0; k < e->N; k++) dst[k] = smod(co[k], e->q[p]);
    ntt_fwd(e, dst, p);
}

/* ------------------------------------------------------------------------------------------ */
/* keys                                                                    */
void aesfhe_key_free(aesfhe_key *k) {
    if (!k) return;
    free(k->data);
    free(k);
}
int aesfhe_key_info(const aesfhe_key *k, int32_t *kind, uint64_t *g) {
    *kind = k->kind;
    *g = k->galois;
    return 0;
}

uint64_t aesfhe_galois_elt(int32_t logN, int64_t rot, int32_t conj) {
    u64 M = 2ULL << logN, n = 1ULL << (logN - 1);
    if (conj) return M - 1;
    i64 r = rot % (i64)n;
    if (r < 0) r += (i64)n;
    u64 ex = (n - (u64)r) % n; /* np.roll(v, k) == left-rotation by -k */
    u64 g = 1;
    for (u64 i = 0; i < ex; i++) g = (g * 5) % M;
    return g;
}

int aesfhe_key_secret(aesfhe_engine *e, uint64_t seed, aesfhe_key **out) {
    aesfhe_key *k = calloc(1, sizeof *k);
    k->kind = 0;
    k->keyseed = derive(e->seed, seed);
    k->data = malloc(sizeof(u64) * (size_t)e->np * e->N);
    i64 *s = malloc(sizeof(i64) * e->N);
    u64 key = derive(k->keyseed, 1);
    for (int i = 0; i < e->N; i++) s[i] = ternary(rnd(e->ck, key, (u64)i));
#pragma omp parallel for schedule(static) num_threads(e->threads)
    for (int p = 0; p < e->np; p++) coeffs_to_ntt(e, s, k->data + (size_t)p * e->N, p);
    free(s);
    *out = k;
    return 0;
}

int aesfhe_key_public(aesfhe_engine *e, const aesfhe_key *sk, aesfhe_key **out) {
    if (!sk || sk->kind != 0) return fail(AESFHE_EARG, "public key needs a secret key");
    const int N = e->N, nq = e->L + 1;
    aesfhe_key *k = calloc(1, sizeof *k);
    k->kind = 1;
    k->keyseed = sk->keyseed;
    k->data = malloc(sizeof(u64) * 2 * (size_t)nq * N);
    u64 ka = derive(sk->keyseed, 2), ke = derive(sk->keyseed, 3);
    i64 *ee = malloc(sizeof(i64) * N);
    for (int i = 0; i < N; i++) ee[i] = cbd21(rnd(e->ck, ke, (u64)i));
#pragma omp parallel for schedule(static) num_threads(e->threads)
    for (int p = 0; p < nq; p++) {
        u64 *b = k->data + (size_t)p * N, *a = k->data + ((size_t)nq + p) * N;
        const u64 *s = sk->data + (size_t)p * N;
        const u64 q = e->q[p];
        u64 *et = malloc(sizeof(u64) * N);
        coeffs_to_ntt(e, ee, et, p);
        for (int j = 0; j < N; j++) {
            a[j] = uniform_mod(rnd(e->ck, ka, (u64)p * N + j), q);
            b[j] = add_mod(sub_mod(0, mul_mod(a[j], s[j], &e->mont[p]), q), et[j], q);
        }
        free(et);
    }
    free(ee);
    *out = k;
    return 0;
}

/* switching key from s' (NTT, all np primes) to s: [dnum][2][np][N] (b, a) */
static aesfhe_key *make_ksk_salt(aesfhe_engine *e, const aesfhe_key *sk, const u64 *sprime, int kind,
                                 u64 g, u64 salt);
static aesfhe_key *make_ksk(aesfhe_engine *e, const aesfhe_key *sk, const u64 *sprime, int kind,
                            u64 g) {
    return make_ksk_salt(e, sk, sprime, kind, g, 0);
}
static aesfhe_key *make_ksk_t(aesfhe_engine *e, const u64 *starget, u64 keyseed, const u64 *sprime,
                              int kind, u64 g, u64 salt);
static aesfhe_key *make_ksk_salt(aesfhe_engine *e, const aesfhe_key *sk, const u64 *sprime, int kind,
                                 u64 g, u64 salt) {
    return make_ksk_t(e, sk->data, sk->keyseed, sprime, kind, g, salt);
}
/* switching key s' -> s: s = `starget` (all limbs of Q u P), stream from keyseed */
static aesfhe_key *make_ksk_t(aesfhe_engine *e, const u64 *starget, u64 keyseed, const u64 *sprime,
                              int kind, u64 g, u64 salt) {
    const int N = e->N, np = e->np, nq = e->L + 1;
    aesfhe_key *k = calloc(1, sizeof *k);
    k->kind = kind;
    k->galois = g;
    k->keyseed = keyseed;
    k->data = malloc(sizeof(u64) * (size_t)e->dnum * 2 * np * N);
    k->ndig = e->dnum;
    u64 base = derive(derive(keyseed, 4 + (u64)kind), g);
    if (salt) base = derive(base, salt);
    /* P mod q_i */
    u64 Pmod[MAXP];
    for (int p = 0; p < nq; p++) {
        u64 acc = 1;
        for (int j = 0; j < e->K; j++) acc = mul_mod_slow(acc, e->q[nq + j] % e->q[p], e->q[p]);
        Pmod[p] = acc;
    }
    for (int d = 0; d < e->dnum; d++) {
        u64 ka = derive(base, 2 * (u64)d), ke = derive(base, 2 * (u64)d + 1);
        i64 *ee = malloc(sizeof(i64) * N);
        for (int i = 0; i < N; i++) ee[i] = cbd21(rnd(e->ck, ke, (u64)i));
        int lo = d * e->A, hi = lo + e->A; /* digit primes [lo, hi) intersect [0, nq) */
#pragma omp parallel for schedule(static) num_threads(e->threads)
        for (int p = 0; p < np; p++) {
            u64 *b = k->data + (((size_t)d * 2 + 0) * np + p) * N;
            u64 *a = k->data + (((size_t)d * 2 + 1) * np + p) * N;
            const u64 *s = starget + (size_t)p * N;
            const u64 q = e->q[p];
            u64 *et = malloc(sizeof(u64) * N);
            coeffs_to_ntt(e, ee, et, p);
            int indigit = (p < nq) && p >= lo && p < hi;
            for (int j = 0; j < N; j++) {
                a[j] = uniform_mod(rnd(e->ck, ka, (u64)p * N + j), q);
                u64 v = add_mod(sub_mod(0, mul_mod(a[j], s[j], &e->mont[p]), q), et[j], q);
                if (indigit)
                    v = add_mod(v, mul_mod(Pmod[p], sprime[(size_t)p * N + j], &e->mont[p]), q);
                b[j] = v;
            }
            free(et);
        }
        free(ee);
    }
    return k;
}

int aesfhe_key_relin(aesfhe_engine *e, const aesfhe_key *sk, aesfhe_key **out) {
    if (!sk || sk->kind != 0) return fail(AESFHE_EARG, "relinearization key needs a secret key");
    const int N = e->N;
    u64 *s2 = malloc(sizeof(u64) * (size_t)e->np * N);
    for (int p = 0; p < e->np; p++)
        for (int j = 0; j < N; j++) {
            u64 v = sk->data[(size_t)p * N + j];
            s2[(size_t)p * N + j] = mul_mod(v, v, &e->mont[p]);
        }
    *out = make_ksk(e, sk, s2, 2, 0);
    free(s2);
    return 0;
}

/* sparse ternary secret (include/aesfhe.h aesfhe_key_secret_sparse) */
int aesfhe_key_secret_sparse(aesfhe_engine *e, uint64_t seed, int32_t hw, aesfhe_key **out) {
    const int N = e->N;
    if (hw < 1 || hw > N) return fail(AESFHE_EARG, "sparse secret weight must be in [1, N]");
    aesfhe_key *k = calloc(1, sizeof *k);
    k->kind = 0;
    k->keyseed = derive(e->seed, seed);
    k->data = malloc(sizeof(u64) * (size_t)e->np * N);
    i64 *s = calloc(N, sizeof(i64));
    int *idx = malloc(sizeof(int) * N);
    for (int i = 0; i < N; i++) idx[i] = i;
    const u64 key = derive(k->keyseed, 9);
    for (int i = 0; i < hw; i++) {
        const int j = i + (int)(rnd(e->ck, key, (u64)i) % (u64)(N - i));
        const int t = idx[i];
        idx[i] = idx[j];
        idx[j] = t;
        s[idx[i]] = (rnd(e->ck, key, (u64)N + i) & 1) ? -1 : 1;
    }
#pragma omp parallel for schedule(static) num_threads(e->threads)
    for (int p = 0; p < e->np; p++) coeffs_to_ntt(e, s, k->data + (size_t)p * N, p);
    free(s);
    free(idx);
    *out = k;
    return 0;
}

/* switching key sk_from -> sk_to: galois kind with element 1 */
int aesfhe_key_switch(aesfhe_engine *e, const aesfhe_key *sk_from, const aesfhe_key *sk_to, aesfhe_key **out) {
    if (!sk_from || !sk_to || sk_from->kind != 0 || sk_to->kind != 0)
        return fail(AESFHE_EARG, "switching key needs two secret keys");
    *out = make_ksk_salt(e, sk_to, sk_from->data, 3, 1, sk_from->keyseed | 1);
    return 0;
}

/* hoisted rotation key for g (kind 5): switches s -> sigma_g^{-1}(s); aesfhe_rotate_hoisted
 * applies it as rotate = sigma_g o keyswitch (the HIP engine shares the ModUp of c1) */
int aesfhe_key_galois_hoisted(aesfhe_engine *e, const aesfhe_key *sk, uint64_t g, aesfhe_key **out) {
    if (!sk || sk->kind != 0) return fail(AESFHE_EARG, "galois key needs a secret key");
    if (!(g & 1) || g >= 2ULL * e->N) return fail(AESFHE_EARG, "bad galois element");
    const int N = e->N;
    const u64 M = 2ULL * (u64)N;
    u64 ginv = 1;
    for (u64 x = 1;; x = x * g % M)
        if (x * g % M == 1) { ginv = x; break; }
    u64 *st = malloc(sizeof(u64) * (size_t)e->np * N);
    for (int p = 0; p < e->np; p++) galois_perm(e, sk->data + (size_t)p * N, st + (size_t)p * N, ginv);
    *out = make_ksk_t(e, st, sk->keyseed, sk->data, 5, g, 0x4015);
    free(st);
    return 0;
}

int aesfhe_key_galois(aesfhe_engine *e, const aesfhe_key *sk, uint64_t g, aesfhe_key **out) {
    if (!sk || sk->kind != 0) return fail(AESFHE_EARG, "galois key needs a secret key");
    if (!(g & 1) || g >= 2ULL * e->N) return fail(AESFHE_EARG, "bad galois element");
    const int N = e->N;
    u64 *sg = malloc(sizeof(u64) * (size_t)e->np * N);
    for (int p = 0; p < e->np; p++) galois_perm(e, sk->data + (size_t)p * N, sg + (size_t)p * N, g);
    *out = make_ksk(e, sk, sg, 3, g);
    free(sg);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* encryption / decryption                                                     */
int aesfhe_encrypt(aesfhe_engine *e, const aesfhe_key *key, const int64_t *co, int32_t B,
                   int32_t level, uint64_t nonce, aesfhe_ct **out) {
    if (!key || (key->kind != 0 && key->kind != 1)) return fail(AESFHE_EARG, "encryption key must be pk or sk");
    if (level < 0 || level > e->L || B < 1) return fail(AESFHE_EARG, "bad level/batch");
    const int N = e->N;
    aesfhe_ct *c = ct_new(e, B, 2, level);
    u64 base = derive(derive(e->seed, 0xE0CULL), nonce);
    for (int b = 0; b < B; b++) {
        u64 k0 = derive(base, 3 * (u64)b), k1 = derive(base, 3 * (u64)b + 1),
            k2 = derive(base, 3 * (u64)b + 2);
        i64 *v = malloc(sizeof(i64) * N), *e0 = malloc(sizeof(i64) * N), *e1 = malloc(sizeof(i64) * N);
        for (int i = 0; i < N; i++) v[i] = ternary(rnd(e->ck, k0, (u64)i));  /* one stream per loop: */
        for (int i = 0; i < N; i++) e0[i] = cbd21(rnd(e->ck, k1, (u64)i));   /* the block cache     */
        for (int i = 0; i < N; i++) e1[i] = cbd21(rnd(e->ck, k2, (u64)i));   /* serves 7 of 8 words */
        const i64 *m = co + (size_t)b * N;
#pragma omp parallel for schedule(static) num_threads(e->threads)
        for (int p = 0; p <= level; p++) {
            const u64 q = e->q[p];
            u64 *c0 = limb(e, c, b, 0, p), *c1 = limb(e, c, b, 1, p);
            u64 *tm = malloc(sizeof(u64) * N), *te = malloc(sizeof(u64) * N);
            coeffs_to_ntt(e, m, tm, p);
            coeffs_to_ntt(e, e0, te, p);
            if (key->kind == 1) {
                u64 *tv = malloc(sizeof(u64) * N), *te1 = malloc(sizeof(u64) * N);
                coeffs_to_ntt(e, v, tv, p);
                coeffs_to_ntt(e, e1, te1, p);
                const u64 *pk0 = key->data + (size_t)p * N, *pk1 = key->data + ((size_t)(e->L + 1) + p) * N;
                for (int j = 0; j < N; j++) {
                    c0[j] = add_mod(add_mod(mul_mod(tv[j], pk0[j], &e->mont[p]), te[j], q), tm[j], q);
                    c1[j] = add_mod(mul_mod(tv[j], pk1[j], &e->mont[p]), te1[j], q);
                }
                free(tv);
                free(te1);
            } else {
                const u64 *s = key->data + (size_t)p * N;
                for (int j = 0; j < N; j++) {
                    u64 a = uniform_mod(rnd(e->ck, k0, (u64)p * N + j), q);
                    c1[j] = a;
                    c0[j] = add_mod(add_mod(sub_mod(0, mul_mod(a, s[j], &e->mont[p]), q), te[j], q), tm[j], q);
                }
            }
            free(tm);
            free(te);
        }
        free(v);
        free(e0);
        free(e1);
    }
    *out = c;
    return 0;
}

/* limb 0, and limb 1 when present, CRT-combined and centred mod q0 q1 (level 0:
 * mod q0); coefficients beyond +-(2^63 - 1) saturate. */
static void dec_limb(aesfhe_engine *e, const aesfhe_key *sk, const aesfhe_ct *c, int b, int p, u64 *t) {
    const int N = e->N;
    const u64 q = e->q[p];
    const u64 *s = sk->data + (size_t)p * N;
    const u64 *c0 = limb(e, c, b, 0, p);
    for (int j = 0; j < N; j++) t[j] = c0[j];
    if (c->npoly >= 2) {
        const u64 *c1 = limb(e, c, b, 1, p);
        for (int j = 0; j < N; j++) t[j] = add_mod(t[j], mul_mod(c1[j], s[j], &e->mont[p]), q);
    }
    if (c->npoly == 3) {
        const u64 *c2 = limb(e, c, b, 2, p);
        for (int j = 0; j < N; j++) {
            u64 s2 = mul_mod(s[j], s[j], &e->mont[p]);
            t[j] = add_mod(t[j], mul_mod(c2[j], s2, &e->mont[p]), q);
        }
    }
    ntt_inv(e, t, p);
}

int aesfhe_decrypt(aesfhe_engine *e, const aesfhe_key *sk, const aesfhe_ct *c, int64_t *out) {
    if (!sk || sk->kind != 0) return fail(AESFHE_EARG, "decryption needs the secret key");
    const int N = e->N;
    const u64 q0 = e->q[0];
    u64 *t0 = malloc(sizeof(u64) * N), *t1 = malloc(sizeof(u64) * N);
    for (int b = 0; b < c->B; b++) {
        dec_limb(e, sk, c, b, 0, t0);
        int64_t *o = out + (size_t)b * N;
        if (c->level < 1) {
            for (int j = 0; j < N; j++) o[j] = t0[j] > q0 / 2 ? (i64)t0[j] - (i64)q0 : (i64)t0[j];
            continue;
        }
        dec_limb(e, sk, c, b, 1, t1);
        const u64 q1 = e->q[1], q0inv = pow_mod(q0 % q1, q1 - 2, q1);
        const u128 Q = (u128)q0 * q1;
        for (int j = 0; j < N; j++) {
            u64 r1 = t1[j], r0m = t0[j] % q1;
            u64 d = (u64)((u128)(r1 >= r0m ? r1 - r0m : r1 + q1 - r0m) * q0inv % q1);
            u128 x = (u128)t0[j] + (u128)q0 * d;
            if (x > Q / 2) {
                u128 m = Q - x;
                o[j] = m > (u128)INT64_MAX ? -INT64_MAX : -(i64)m;
            } else {
                o[j] = x > (u128)INT64_MAX ? INT64_MAX : (i64)x;
            }
        }
    }
    free(t0);
    free(t1);
    return 0;
}

int aesfhe_encrypt_device(aesfhe_engine *e, const aesfhe_key *key, const int64_t *co, int32_t B,
                          int32_t level, uint64_t nonce, aesfhe_ct **out) {
    if (!co) return fail(AESFHE_EARG, "null coefficient buffer");
    return aesfhe_encrypt(e, key, co, B, level, nonce, out);
}
int aesfhe_decrypt_device(aesfhe_engine *e, const aesfhe_key *sk, const aesfhe_ct *c, int64_t *out) {
    if (!out) return fail(AESFHE_EARG, "null coefficient buffer");
    return aesfhe_decrypt(e, sk, c, out);
}

int aesfhe_ct_export(aesfhe_engine *e, const aesfhe_ct *c, uint64_t *out) {
    memcpy(out, c->data, sizeof(u64) * (size_t)c->B * c->npoly * (c->level + 1) * e->N);
    return 0;
}
int aesfhe_ct_import(aesfhe_engine *e, const uint64_t *in, int32_t B, int32_t np, int32_t level,
                     aesfhe_ct **out) {
    if (B < 1 || np < 1 || np > 3 || level < 0 || level > e->L) return fail(AESFHE_EARG, "bad shape");
    aesfhe_ct *c = ct_new(e, B, np, level);
    memcpy(c->data, in, sizeof(u64) * (size_t)B * np * (level + 1) * e->N);
    *out = c;
    return 0;
}
/* "Device" transfer: the oracle's memory is host memory, so these are the host copies the
 * CPU (gloo) path of parallel.py hands to torch.distributed. */
int aesfhe_ct_export_device(aesfhe_engine *e, const aesfhe_ct *c, int32_t start, int32_t count, void *dst) {
    if (!c || !dst || start < 0 || count < 1 || start + count > c->B) return fail(AESFHE_EARG, "bad export range");
    size_t per = (size_t)c->npoly * (c->level + 1) * e->N;
    memcpy(dst, c->data + per * start, sizeof(u64) * per * count);
    return 0;
}
int aesfhe_ct_import_device(aesfhe_engine *e, const void *src, int32_t B, int32_t np, int32_t level,
                            aesfhe_ct **out) {
    if (!src) return fail(AESFHE_EARG, "null source");
    return aesfhe_ct_import(e, (const uint64_t *)src, B, np, level, out);
}

static size_t key_words(const aesfhe_engine *e, int kind) {
    switch (kind) {
        case 0: return (size_t)e->np * e->N;
        case 1: return (size_t)2 * (e->L + 1) * e->N;
        case 2: case 3: case 5: return (size_t)e->dnum * 2 * e->np * e->N;
        default: return 0;
    }
}
int aesfhe_key_export(aesfhe_engine *e, const aesfhe_key *k, int32_t *kind, uint64_t *galois,
                      uint64_t *keyseed, int64_t *words, uint64_t *out) {
    if (!k) return fail(AESFHE_EARG, "null key");
    *kind = k->kind;
    *galois = k->galois;
    *keyseed = k->keyseed;
    *words = (int64_t)(k->ndig > 0 ? (size_t)k->ndig * 2 * e->np * e->N : key_words(e, k->kind));
    if (out) memcpy(out, k->data, sizeof(u64) * (size_t)*words);
    return 0;
}
/* aesfhe_key_trim (include/aesfhe.h): the first beta(max_level) digits, word for word */
int aesfhe_key_trim(aesfhe_engine *e, aesfhe_key *k, int32_t max_level) {
    if (!k || k->ndig < 1) return fail(AESFHE_EARG, "only switching keys (relinearization, galois, hoisted rotation) can be trimmed");
    if (max_level < 0 || max_level > e->L) return fail(AESFHE_EARG, "bad level %d", max_level);
    const int nd = (max_level + 1 + e->A - 1) / e->A;
    if (nd < k->ndig) {
        u64 *d = malloc(sizeof(u64) * (size_t)nd * 2 * e->np * e->N);
        memcpy(d, k->data, sizeof(u64) * (size_t)nd * 2 * e->np * e->N);
        free(k->data);
        k->data = d;
        k->ndig = nd;
    }
    return 0;
}
int aesfhe_key_import(aesfhe_engine *e, int32_t kind, uint64_t galois, uint64_t keyseed,
                      const uint64_t *in, int64_t words, aesfhe_key **out) {
    size_t want = key_words(e, kind);
    if (!in || !want) return fail(AESFHE_EARG, "unknown key kind %d", kind);
    int ndig = 0;
    if (kind == 2 || kind == 3 || kind == 5) { /* switching keys: dnum digits or a trimmed key's first ones */
        const size_t dw = (size_t)2 * e->np * e->N;
        if (words > 0 && (size_t)words % dw == 0 && (size_t)words / dw <= (size_t)e->dnum)
            want = (size_t)words, ndig = (int)((size_t)words / dw);
    }
    if ((size_t)words != want) return fail(AESFHE_EARG, "key of kind %d needs %zu words, got %lld", kind, want, (long long)words);
    aesfhe_key *k = calloc(1, sizeof *k);
    k->kind = kind;
    k->galois = galois;
    k->keyseed = keyseed;
    k->ndig = ndig;
    k->data = malloc(sizeof(u64) * want);
    memcpy(k->data, in, sizeof(u64) * want);
    *out = k;
    return 0;
}
int aesfhe_ct_copy(aesfhe_engine *e, const aesfhe_ct *c, aesfhe_ct **out) {
    aesfhe_ct *r = ct_new(e, c->B, c->npoly, c->level);
    memcpy(r->data, c->data, sizeof(u64) * (size_t)c->B * c->npoly * (c->level + 1) * e->N);
    r->is_zero = c->is_zero;
    *out = r;
    return 0;
}
int aesfhe_ct_slice(aesfhe_engine *e, const aesfhe_ct *c, int32_t start, int32_t count, aesfhe_ct **out) {
    if (start < 0 || count < 1 || start + count > c->B) return fail(AESFHE_EARG, "bad slice");
    aesfhe_ct *r = ct_new(e, count, c->npoly, c->level);
    size_t per = (size_t)c->npoly * (c->level + 1) * e->N;
    memcpy(r->data, c->data + per * start, sizeof(u64) * per * count);
    r->is_zero = c->is_zero;
    *out = r;
    return 0;
}
int aesfhe_ct_concat(aesfhe_engine *e, const aesfhe_ct *const *parts, int32_t n, aesfhe_ct **out) {
    if (n < 1) return fail(AESFHE_EARG, "empty concat");
    int B = 0;
    for (int i = 0; i < n; i++) {
        if (parts[i]->level != parts[0]->level || parts[i]->npoly != parts[0]->npoly)
            return fail(AESFHE_EARG, "concat parts differ in level/npoly");
        B += parts[i]->B;
    }
    aesfhe_ct *r = ct_new(e, B, parts[0]->npoly, parts[0]->level);
    size_t per = (size_t)r->npoly * (r->level + 1) * e->N, off = 0;
    int allz = 1;
    for (int i = 0; i < n; i++) {
        memcpy(r->data + off, parts[i]->data, sizeof(u64) * per * parts[i]->B);
        off += per * parts[i]->B;
        allz &= parts[i]->is_zero;
    }
    r->is_zero = allz;
    *out = r;
    return 0;
}
int aesfhe_ct_gather(aesfhe_engine *e, const aesfhe_ct *c, const int32_t *idx, int32_t n, aesfhe_ct **out) {
    if (n < 1 || !idx) return fail(AESFHE_EARG, "empty gather");
    for (int b = 0; b < n; b++)
        if (idx[b] < 0 || idx[b] >= c->B) return fail(AESFHE_EARG, "gather index %d out of [0, %d)", idx[b], c->B);
    aesfhe_ct *r = ct_new(e, n, c->npoly, c->level);
    size_t per = (size_t)c->npoly * (c->level + 1) * e->N;
    for (int b = 0; b < n; b++) memcpy(r->data + per * b, c->data + per * idx[b], sizeof(u64) * per);
    r->is_zero = c->is_zero;
    *out = r;
    return 0;
}
int aesfhe_ct_zero(aesfhe_engine *e, int32_t B, int32_t level, aesfhe_ct **out) {
    if (B < 1 || level < 0 || level > e->L) return fail(AESFHE_EARG, "bad zero shape");
    aesfhe_ct *r = ct_new(e, B, 2, level);
    r->is_zero = 1;
    *out = r;
    return 0;
}

int aesfhe_pt_create(aesfhe_engine *e, const int64_t *co, int32_t level, aesfhe_pt **out) {
    if (level < 0 || level > e->L) return fail(AESFHE_EARG, "bad plaintext level");
    aesfhe_pt *p = calloc(1, sizeof *p);
    p->level = level;
    p->data = malloc(sizeof(u64) * (size_t)(level + 1) * e->N);
#pragma omp parallel for schedule(static) num_threads(e->threads)
    for (int i = 0; i <= level; i++) coeffs_to_ntt(e, co, p->data + (size_t)i * e->N, i);
    *out = p;
    return 0;
}
/* the same over Q_level u P (level+1+K limbs) */
int aesfhe_pt_create_ext(aesfhe_engine *e, const int64_t *co, int32_t level, aesfhe_pt **out) {
    if (level < 0 || level > e->L) return fail(AESFHE_EARG, "bad plaintext level");
    const int nl = level + 1, ne = nl + e->K;
    aesfhe_pt *p = calloc(1, sizeof *p);
    p->level = level;
    p->ext = 1;
    p->data = malloc(sizeof(u64) * (size_t)ne * e->N);
#pragma omp parallel for schedule(static) num_threads(e->threads)
    for (int t = 0; t < ne; t++) coeffs_to_ntt(e, co, p->data + (size_t)t * e->N, t < nl ? t : e->L + 1 + (t - nl));
    *out = p;
    return 0;
}
void aesfhe_pt_free(aesfhe_pt *p) {
    if (!p) return;
    free(p->data);
    free(p);
}

/* ------------------------------------------------------------------------------------------ */
/* rescale: drop q_l with rounding; operates on every polynomial               */
static aesfhe_ct *rescale_raw(aesfhe_engine *e, const aesfhe_ct *c) {
    const int N = e->N, l = c->level;
    double t0 = now_ms();
    aesfhe_ct *r = ct_new(e, c->B, c->npoly, l - 1);
    const u64 ql = e->q[l];
    for (int b = 0; b < c->B; b++)
        for (int pp = 0; pp < c->npoly; pp++) {
            u64 *x = malloc(sizeof(u64) * N);
            memcpy(x, limb(e, c, b, pp, l), sizeof(u64) * N);
            ntt_inv(e, x, l);
#pragma omp parallel for schedule(static) num_threads(e->threads)
            for (int i = 0; i < l; i++) {
                const u64 q = e->q[i];
                u64 *t = malloc(sizeof(u64) * N);
                u64 qlmod = ql % q;
                for (int j = 0; j < N; j++) {
                    u64 v = x[j] % q;
                    t[j] = x[j] > (ql >> 1) ? sub_mod(v, qlmod, q) : v;
                }
                ntt_fwd(e, t, i);
                u64 inv = inv_mod(ql % q, q), invp = shoup_pre(inv, q);
                const u64 *ci = limb(e, c, b, pp, i);
                u64 *ri = limb(e, r, b, pp, i);
                for (int j = 0; j < N; j++) ri[j] = mul_shoup(sub_mod(ci[j], t[j], q), inv, invp, q);
                free(t);
            }
            free(x);
        }
    prof_add(e, 2, now_ms() - t0);
    return r;
}

int aesfhe_rescale(aesfhe_engine *e, const aesfhe_ct *c, aesfhe_ct **out) {
    if (c->level < 1) return fail(AESFHE_ELEVEL, "cannot rescale a level-0 ciphertext");
    if (c->is_zero) {
        aesfhe_ct *r = ct_new(e, c->B, c->npoly, c->level - 1);
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    *out = rescale_raw(e, c);
    return 0;
}

/* multiply every residue by the constant A + B*X^{N/2} */
static void mul_int_const_inplace(aesfhe_engine *e, aesfhe_ct *c, i64 A, i64 Bc) {
    const int N = e->N;
    for (int i = 0; i <= c->level; i++) {
        const u64 q = e->q[i];
        u64 a = smod(A, q), bb = smod(Bc, q);
        u64 bi = mul_mod_slow(bb, e->iroot[i], q);
        u64 f0 = add_mod(a, bi, q), f1 = sub_mod(a, bi, q);
        u64 f0p = shoup_pre(f0, q), f1p = shoup_pre(f1, q);
        for (int b = 0; b < c->B; b++)
            for (int pp = 0; pp < c->npoly; pp++) {
                u64 *x = limb(e, c, b, pp, i);
                for (int j = 0; j < N / 2; j++) x[j] = mul_shoup(x[j], f0, f0p, q);
                for (int j = N / 2; j < N; j++) x[j] = mul_shoup(x[j], f1, f1p, q);
            }
    }
}

static aesfhe_ct *truncate_ct(aesfhe_engine *e, const aesfhe_ct *c, int level) {
    aesfhe_ct *r = ct_new(e, c->B, c->npoly, level);
    for (int b = 0; b < c->B; b++)
        for (int pp = 0; pp < c->npoly; pp++)
            memcpy(limb(e, r, b, pp, 0), limb(e, c, b, pp, 0), sizeof(u64) * (size_t)(level + 1) * e->N);
    r->is_zero = c->is_zero;
    return r;
}

static aesfhe_ct *level_down_raw(aesfhe_engine *e, const aesfhe_ct *c, int lt) {
    if (lt == c->level) {
        aesfhe_ct *r;
        aesfhe_ct_copy(e, c, &r);
        return r;
    }
    if (c->is_zero) {
        aesfhe_ct *r = ct_new(e, c->B, c->npoly, lt);
        r->is_zero = 1;
        return r;
    }
    aesfhe_ct *t = truncate_ct(e, c, lt + 1);
    i64 C = llround(e->scales[lt] * (double)e->q[lt + 1] / e->scales[c->level]);
    mul_int_const_inplace(e, t, C, 0);
    aesfhe_ct *r = rescale_raw(e, t);
    aesfhe_ct_free(t);
    return r;
}

int aesfhe_level_down(aesfhe_engine *e, const aesfhe_ct *c, int32_t lt, aesfhe_ct **out) {
    if (lt < 0 || lt > c->level) return fail(AESFHE_EARG, "level_down target %d not in [0,%d]", lt, c->level);
    *out = level_down_raw(e, c, lt);
    return 0;
}

int aesfhe_mul_const(aesfhe_engine *e, const aesfhe_ct *c, double re, double im, aesfhe_ct **out) {
    if (c->level < 1) return fail(AESFHE_ELEVEL, "no level left for a constant multiplication");
    double s = aesfhe_engine_mul_scale(e, c->level);
    i64 A = llround(re * s), Bc = llround(im * s);
    if (c->is_zero || (A == 0 && Bc == 0)) {
        aesfhe_ct *r = ct_new(e, c->B, c->npoly, c->level - 1);
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    aesfhe_ct *t;
    aesfhe_ct_copy(e, c, &t);
    mul_int_const_inplace(e, t, A, Bc);
    *out = rescale_raw(e, t);
    aesfhe_ct_free(t);
    return 0;
}

/* align two operands to the lower level; returns owned copies */
static void align2(aesfhe_engine *e, const aesfhe_ct *a, const aesfhe_ct *b, aesfhe_ct **ao, aesfhe_ct **bo) {
    int l = a->level < b->level ? a->level : b->level;
    *ao = level_down_raw(e, a, l);
    *bo = level_down_raw(e, b, l);
}

static int bcast_ok(const aesfhe_ct *a, const aesfhe_ct *b) {
    return a->B == b->B || a->B == 1 || b->B == 1;
}

static int addsub(aesfhe_engine *e, const aesfhe_ct *a0, const aesfhe_ct *b0, int sub, aesfhe_ct **out) {
    if (!bcast_ok(a0, b0)) return fail(AESFHE_EARG, "batch mismatch %d vs %d", a0->B, b0->B);
    aesfhe_ct *a, *b;
    align2(e, a0, b0, &a, &b);
    int B = a->B > b->B ? a->B : b->B, np = a->npoly > b->npoly ? a->npoly : b->npoly;
    aesfhe_ct *r = ct_new(e, B, np, a->level);
    r->is_zero = a->is_zero && b->is_zero;
    const int N = e->N;
    for (int bb = 0; bb < B; bb++)
        for (int pp = 0; pp < np; pp++)
            for (int i = 0; i <= a->level; i++) {
                const u64 q = e->q[i];
                u64 *x = limb(e, r, bb, pp, i);
                const u64 *xa = (pp < a->npoly && !a->is_zero) ? limb(e, a, a->B == 1 ? 0 : bb, pp, i) : NULL;
                const u64 *xb = (pp < b->npoly && !b->is_zero) ? limb(e, b, b->B == 1 ? 0 : bb, pp, i) : NULL;
                for (int j = 0; j < N; j++) {
                    u64 va = xa ? xa[j] : 0, vb = xb ? xb[j] : 0;
                    x[j] = sub ? sub_mod(va, vb, q) : add_mod(va, vb, q);
                }
            }
    aesfhe_ct_free(a);
    aesfhe_ct_free(b);
    *out = r;
    return 0;
}
int aesfhe_add(aesfhe_engine *e, const aesfhe_ct *a, const aesfhe_ct *b, aesfhe_ct **out) { return addsub(e, a, b, 0, out); }
int aesfhe_sub(aesfhe_engine *e, const aesfhe_ct *a, const aesfhe_ct *b, aesfhe_ct **out) { return addsub(e, a, b, 1, out); }
int aesfhe_negate(aesfhe_engine *e, const aesfhe_ct *a, aesfhe_ct **out) {
    aesfhe_ct *z = ct_new(e, a->B, a->npoly, a->level);
    z->is_zero = 1;
    int rc = addsub(e, z, a, 1, out);
    aesfhe_ct_free(z);
    return rc;
}

int aesfhe_add_pt(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_pt *pt, aesfhe_ct **out) {
    if (pt->level < c->level) return fail(AESFHE_EARG, "plaintext level %d below ciphertext level %d", pt->level, c->level);
    aesfhe_ct *r;
    aesfhe_ct_copy(e, c, &r);
    r->is_zero = 0;
    for (int b = 0; b < c->B; b++)
        for (int i = 0; i <= c->level; i++) {
            const u64 q = e->q[i];
            u64 *x = limb(e, r, b, 0, i);
            const u64 *y = pt->data + (size_t)i * e->N;
            for (int j = 0; j < e->N; j++) x[j] = add_mod(x[j], y[j], q);
        }
    *out = r;
    return 0;
}

int aesfhe_add_const(aesfhe_engine *e, const aesfhe_ct *c, double re, double im, aesfhe_ct **out) {
    double s = e->scales[c->level];
    i64 A = llround(re * s), Bc = llround(im * s);
    aesfhe_ct *r;
    aesfhe_ct_copy(e, c, &r);
    r->is_zero = c->is_zero && A == 0 && Bc == 0;
    for (int i = 0; i <= c->level; i++) {
        const u64 q = e->q[i];
        u64 a = smod(A, q), bi = mul_mod_slow(smod(Bc, q), e->iroot[i], q);
        u64 f0 = add_mod(a, bi, q), f1 = sub_mod(a, bi, q);
        for (int b = 0; b < c->B; b++) {
            u64 *x = limb(e, r, b, 0, i);
            for (int j = 0; j < e->N / 2; j++) x[j] = add_mod(x[j], f0, q);
            for (int j = e->N / 2; j < e->N; j++) x[j] = add_mod(x[j], f1, q);
        }
    }
    *out = r;
    return 0;
}

int aesfhe_mul_pt(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_pt *pt, aesfhe_ct **out) {
    if (c->level < 1) return fail(AESFHE_ELEVEL, "no level left for a plaintext multiplication");
    if (pt->level < c->level) return fail(AESFHE_EARG, "plaintext level %d below ciphertext level %d", pt->level, c->level);
    if (c->is_zero) {
        aesfhe_ct *r = ct_new(e, c->B, c->npoly, c->level - 1);
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    aesfhe_ct *t;
    aesfhe_ct_copy(e, c, &t);
    for (int b = 0; b < c->B; b++)
        for (int pp = 0; pp < c->npoly; pp++)
            for (int i = 0; i <= c->level; i++) {
                u64 *x = limb(e, t, b, pp, i);
                const u64 *y = pt->data + (size_t)i * e->N;
                for (int j = 0; j < e->N; j++) x[j] = mul_mod(x[j], y[j], &e->mont[i]);
            }
    *out = rescale_raw(e, t);
    aesfhe_ct_free(t);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* tensor                                                                     */
static void tensor_acc(aesfhe_engine *e, const aesfhe_ct *a, const aesfhe_ct *b, aesfhe_ct *r) {
    const int N = e->N;
    for (int bb = 0; bb < r->B; bb++)
        for (int i = 0; i <= r->level; i++) {
            const mont_t *m = &e->mont[i];
            const u64 q = e->q[i];
            int ia = bb % a->B, ib = bb % b->B; /* cyclic broadcast (cyclic_ok; B = 1 included) */
            const u64 *a0 = limb(e, a, ia, 0, i), *a1 = limb(e, a, ia, 1, i);
            const u64 *b0 = limb(e, b, ib, 0, i), *b1 = limb(e, b, ib, 1, i);
            u64 *d0 = limb(e, r, bb, 0, i), *d1 = limb(e, r, bb, 1, i), *d2 = limb(e, r, bb, 2, i);
            for (int j = 0; j < N; j++) {
                d0[j] = add_mod(d0[j], mul_mod(a0[j], b0[j], m), q);
                d1[j] = add_mod(d1[j], add_mod(mul_mod(a0[j], b1[j], m), mul_mod(a1[j], b0[j], m), q), q);
                d2[j] = add_mod(d2[j], mul_mod(a1[j], b1[j], m), q);
            }
        }
}

/* aesfhe_mul / aesfhe_tensor: the smaller batch may be any power of two dividing the larger;
 * element i of the result takes element i mod B_small of that operand */
static int cyclic_ok(const aesfhe_ct *a, const aesfhe_ct *b) {
    const int lo = a->B < b->B ? a->B : b->B, hi = a->B < b->B ? b->B : a->B;
    return a->B == b->B || (lo >= 1 && (lo & (lo - 1)) == 0 && hi % lo == 0);
}

int aesfhe_tensor(aesfhe_engine *e, const aesfhe_ct *a0, const aesfhe_ct *b0, aesfhe_ct **out) {
    if (a0->npoly != 2 || b0->npoly != 2) return fail(AESFHE_EDEGREE, "tensor inputs should have 2 polynomials");
    if (!cyclic_ok(a0, b0)) return fail(AESFHE_EARG, "batch mismatch");
    aesfhe_ct *a, *b;
    align2(e, a0, b0, &a, &b);
    int B = a->B > b->B ? a->B : b->B;
    aesfhe_ct *r = ct_new(e, B, 3, a->level);
    if (a->is_zero || b->is_zero) r->is_zero = 1;
    else tensor_acc(e, a, b, r);
    aesfhe_ct_free(a);
    aesfhe_ct_free(b);
    *out = r;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* hybrid key switching.  d: one polynomial, level l, NTT domain.             */
/* out0/out1: (l+1) limbs each.                                                                */
/* a trimmed key (aesfhe_key_trim) keeps its first digits only: it serves a key switch at level l
 * iff it stores the beta(l) digits the switch reads -- the HIP engine's check_key_digits, checked
 * at every entry point before any work (a misused trimmed key returns AESFHE_ELEVEL
 * instead of aborting the process) */
static int key_level_ok(const aesfhe_engine *e, const aesfhe_key *k, int l) {
    if (!k || k->ndig <= 0) return 0;
    const int beta = (l + 1 + e->A - 1) / e->A;
    if (beta > k->ndig)
        return fail(AESFHE_ELEVEL, "key trimmed to %d digits cannot switch at level %d (%d digits)", k->ndig, l, beta);
    return 0;
}
#define KEY_LEVEL_OK(k, l)                         \
    do {                                           \
        const int kl_rc_ = key_level_ok(e, (k), (l)); \
        if (kl_rc_) return kl_rc_;                 \
    } while (0)

/* inner product of the ModUp digits with the key: acc = 2 x (l+1+K) limbs over Q_l and P */
static u64 *ks_acc(aesfhe_engine *e, const u64 *d, int l, const aesfhe_key *k) {
    const int N = e->N, K = e->K, nq = e->L + 1, ne = l + 1 + K;
    int pid[MAXP];
    for (int t = 0; t < ne; t++) pid[t] = t <= l ? t : nq + (t - l - 1);
    u64 *dc = malloc(sizeof(u64) * (size_t)(l + 1) * N);
    memcpy(dc, d, sizeof(u64) * (size_t)(l + 1) * N);
#pragma omp parallel for schedule(static) num_threads(e->threads)
    for (int i = 0; i <= l; i++) ntt_inv(e, dc + (size_t)i * N, i);
    u64 *acc = calloc((size_t)2 * ne * N, sizeof(u64));
    const int A = e->A;
    int beta = (l + 1 + A - 1) / A;
    if (k->ndig > 0 && beta > k->ndig) {  /* unreachable: every entry point runs key_level_ok first */
        fprintf(stderr, "ckks_oracle: key trimmed to %d digits switched at level %d (%d digits)\n", k->ndig, l, beta);
        abort();
    }
    for (int j = 0; j < beta; j++) {
        int lo = j * A, hi = lo + A < l + 1 ? lo + A : l + 1, na = hi - lo;
        u64 hatinv[MAXP], hat[MAXP][MAXP];
        for (int i = lo; i < hi; i++) {
            u64 prod = 1;
            for (int i2 = lo; i2 < hi; i2++)
                if (i2 != i) prod = mul_mod_slow(prod, e->q[i2] % e->q[i], e->q[i]);
            hatinv[i - lo] = inv_mod(prod, e->q[i]);
            for (int t = 0; t < ne; t++) {
                u64 qt = e->q[pid[t]], h = 1;
                for (int i2 = lo; i2 < hi; i2++)
                    if (i2 != i) h = mul_mod_slow(h, e->q[i2] % qt, qt);
                hat[i - lo][t] = h;
            }
        }
        const u64 *kb = k->data + ((size_t)j * 2 + 0) * e->np * N;
        const u64 *ka = k->data + ((size_t)j * 2 + 1) * e->np * N;
#pragma omp parallel for schedule(static) num_threads(e->threads)
        for (int t = 0; t < ne; t++) {
            const u64 qt = e->q[pid[t]];
            u64 *ext = malloc(sizeof(u64) * N);
            if (t >= lo && t < hi) {
                memcpy(ext, d + (size_t)t * N, sizeof(u64) * N);
            } else {
                for (int c = 0; c < N; c++) {
                    u64 s = 0;
                    for (int i = lo; i < hi; i++) {
                        u64 y = mul_mod_slow(dc[(size_t)i * N + c], hatinv[i - lo], e->q[i]);
                        s = add_mod(s, mul_mod_slow(y % qt, hat[i - lo][t], qt), qt);
                    }
                    ext[c] = s;
                }
                ntt_fwd(e, ext, pid[t]);
            }
            const u64 *kbt = kb + (size_t)pid[t] * N, *kat = ka + (size_t)pid[t] * N;
            u64 *a0 = acc + (size_t)t * N, *a1 = acc + ((size_t)ne + t) * N;
            for (int c = 0; c < N; c++) {
                a0[c] = add_mod(a0[c], mul_mod(ext[c], kbt[c], &e->mont[pid[t]]), qt);
                a1[c] = add_mod(a1[c], mul_mod(ext[c], kat[c], &e->mont[pid[t]]), qt);
            }
            free(ext);
        }
        (void)na;
    }
    free(dc);
    return acc;
}

/* ModDown of the accumulators by D = P * q_l ... q_{l-r+1} (r = 0: plain
 * ModDown by P, r >= 1: combined with r rescales).  Dropped limbs E = {q_{l-r+1}..q_l, p_0..}:
 * y_j = [INTT(acc_j) * (D/e_j)^{-1}]_{e_j}, conv_i = sum_j y_j (D/e_j mod q_i), out_i =
 * (acc_i - conv_i) D^{-1} for i <= l - r.  The conversion is exact (every r): v = rint(sum_j
 * y_j * (1/e_j)) (fp64, in j order) multiples of D are removed from conv (round-to-nearest
 * division, as a plain rescale).  Output limbs: (l-r+1) per component. */
static void moddown_r(aesfhe_engine *e, const u64 *acc, int l, int r, u64 *out0, u64 *out1) {
    const int N = e->N, K = e->K, nq = e->L + 1, ne = l + 1 + K, nE = K + r, lk = l - r;
    int Ep[MAXP];
    for (int j = 0; j < nE; j++) Ep[j] = j < r ? lk + 1 + j : nq + (j - r);
    u64 inv[MAXP], hat[MAXP][MAXP], Dinv[MAXP], Dmod[MAXP];
    double einv[MAXP];
    for (int j = 0; j < nE; j++) {
        const u64 ej = e->q[Ep[j]];
        u64 prod = 1;
        for (int j2 = 0; j2 < nE; j2++)
            if (j2 != j) prod = mul_mod_slow(prod, e->q[Ep[j2]] % ej, ej);
        inv[j] = inv_mod(prod, ej);
        einv[j] = 1.0 / (double)ej;
        for (int i = 0; i <= lk; i++) {
            const u64 qi = e->q[i];
            u64 h = 1;
            for (int j2 = 0; j2 < nE; j2++)
                if (j2 != j) h = mul_mod_slow(h, e->q[Ep[j2]] % qi, qi);
            hat[j][i] = h;
        }
    }
    for (int i = 0; i <= lk; i++) {
        const u64 qi = e->q[i];
        u64 D = 1;
        for (int j = 0; j < nE; j++) D = mul_mod_slow(D, e->q[Ep[j]] % qi, qi);
        Dinv[i] = inv_mod(D, qi);
        Dmod[i] = D;
    }
    for (int c = 0; c < 2; c++) {
        const u64 *a = acc + (size_t)c * ne * N;
        u64 *outc = c == 0 ? out0 : out1;
        u64 *y = malloc(sizeof(u64) * (size_t)nE * N);
#pragma omp parallel for schedule(static) num_threads(e->threads)
        for (int j = 0; j < nE; j++) {
            const int p = Ep[j];
            u64 *z = y + (size_t)j * N;
            memcpy(z, a + (size_t)(lk + 1 + j) * N, sizeof(u64) * N);
            ntt_inv(e, z, p);
            for (int x = 0; x < N; x++) z[x] = mul_mod_slow(z[x], inv[j], e->q[p]);
        }
#pragma omp parallel for schedule(static) num_threads(e->threads)
        for (int i = 0; i <= lk; i++) {
            const u64 qi = e->q[i];
            u64 *conv = malloc(sizeof(u64) * N);
            for (int x = 0; x < N; x++) {
                u64 sum = 0;
                for (int j = 0; j < nE; j++)
                    sum = add_mod(sum, mul_mod_slow(y[(size_t)j * N + x] % qi, hat[j][i], qi), qi);
                {  /* exact conversion: remove the v multiples of D (v = rint(sum y_j / e_j)) */
                    double u = 0.0;
                    for (int j = 0; j < nE; j++) u = u + (double)y[(size_t)j * N + x] * einv[j];
                    const u64 v = (u64)rint(u);
                    sum = sub_mod(sum, mul_mod_slow(v % qi, Dmod[i], qi), qi);
                }
                conv[x] = sum;
            }
            ntt_fwd(e, conv, i);
            const u64 dp = shoup_pre(Dinv[i], qi);
            for (int x = 0; x < N; x++)
                outc[(size_t)i * N + x] = mul_shoup(sub_mod(a[(size_t)i * N + x], conv[x], qi), Dinv[i], dp, qi);
            free(conv);
        }
        free(y);
    }
}

/* hybrid key switching of one polynomial, ModDown by P: out0/out1 (l+1 limbs each) */
static void keyswitch(aesfhe_engine *e, const u64 *d, int l, const aesfhe_key *k, u64 *out0, u64 *out1) {
    double t0 = now_ms();
    u64 *acc = ks_acc(e, d, l, k);
    moddown_r(e, acc, l, 0, out0, out1);
    free(acc);
    prof_add(e, 1, now_ms() - t0);
}

static int relin_raw(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_key *rlk, aesfhe_ct **out);

/* relinearisation fused with r rescales: acc_c += P * d_c on the Q limbs,
 * then ModDown by P q_l ... q_{l-r+1}; the result is at level l - r. */
static aesfhe_ct *relin_rescale_raw(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_key *rlk, int r) {
    const int N = e->N, l = c->level, K = e->K, ne = l + 1 + K;
    if (K + r > 16) {  /* the HIP engine's table limit: separate relinearisation and rescales */
        aesfhe_ct *x;
        relin_raw(e, c, rlk, &x);
        for (int i = 0; i < r; i++) {
            aesfhe_ct *y = rescale_raw(e, x);
            aesfhe_ct_free(x);
            x = y;
        }
        return x;
    }
    double t0 = now_ms();
    aesfhe_ct *out = ct_new(e, c->B, 2, l - r);
    for (int b = 0; b < c->B; b++) {
        u64 *acc = ks_acc(e, limb(e, c, b, 2, 0), l, rlk);
        for (int cc = 0; cc < 2; cc++)
#pragma omp parallel for schedule(static) num_threads(e->threads)
            for (int i = 0; i <= l; i++) {
                const u64 qi = e->q[i];
                u64 P = 1;
                for (int kk = 0; kk < K; kk++) P = mul_mod_slow(P, e->q[e->L + 1 + kk] % qi, qi);
                const u64 *dci = limb(e, c, b, cc, i);
                u64 *ai = acc + ((size_t)cc * ne + i) * N;
                for (int x = 0; x < N; x++) ai[x] = add_mod(ai[x], mul_mod_slow(dci[x], P, qi), qi);
            }
        moddown_r(e, acc, l, r, limb(e, out, b, 0, 0), limb(e, out, b, 1, 0));
        free(acc);
    }
    prof_add(e, 1, now_ms() - t0);
    return out;
}

static int relin_raw(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_key *rlk, aesfhe_ct **out) {
    const int N = e->N, l = c->level;
    aesfhe_ct *r = ct_new(e, c->B, 2, l);
    u64 *k0 = malloc(sizeof(u64) * (size_t)(l + 1) * N), *k1 = malloc(sizeof(u64) * (size_t)(l + 1) * N);
    for (int b = 0; b < c->B; b++) {
        keyswitch(e, limb(e, c, b, 2, 0), l, rlk, k0, k1);
        for (int i = 0; i <= l; i++) {
            const u64 q = e->q[i];
            const u64 *d0 = limb(e, c, b, 0, i), *d1 = limb(e, c, b, 1, i);
            u64 *r0 = limb(e, r, b, 0, i), *r1 = limb(e, r, b, 1, i);
            for (int j = 0; j < N; j++) {
                r0[j] = add_mod(d0[j], k0[(size_t)i * N + j], q);
                r1[j] = add_mod(d1[j], k1[(size_t)i * N + j], q);
            }
        }
    }
    free(k0);
    free(k1);
    *out = r;
    return 0;
}

int aesfhe_relinearize(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_key *rlk, aesfhe_ct **out) {
    if (c->npoly != 3) return fail(AESFHE_EDEGREE, "Input ciphertext should have 3 polynomials");
    if (!rlk || rlk->kind != 2) return fail(AESFHE_EARG, "relinearize needs a relinearization key");
    KEY_LEVEL_OK(rlk, c->level);
    if (c->is_zero) {
        aesfhe_ct *r = ct_new(e, c->B, 2, c->level);
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    return relin_raw(e, c, rlk, out);
}

int aesfhe_mul(aesfhe_engine *e, const aesfhe_ct *a, const aesfhe_ct *b, const aesfhe_key *rlk, aesfhe_ct **out) {
    if (!rlk || rlk->kind != 2) return fail(AESFHE_EARG, "multiply needs a relinearization key");
    int l = a->level < b->level ? a->level : b->level;
    if (l < 1) return fail(AESFHE_ELEVEL, "no level left for a ciphertext multiplication");
    aesfhe_ct *t, *rl;
    KEY_LEVEL_OK(rlk, l);
    int rc = aesfhe_tensor(e, a, b, &t);
    if (rc) return rc;
    if (t->is_zero) {
        aesfhe_ct *r = ct_new(e, t->B, 2, l - 1);
        r->is_zero = 1;
        aesfhe_ct_free(t);
        *out = r;
        return 0;
    }
    (void)rl;
    *out = relin_rescale_raw(e, t, rlk, 1);
    aesfhe_ct_free(t);
    return 0;
}

int aesfhe_galois(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_key *gk, aesfhe_ct **out) {
    if (!gk || gk->kind != 3) return fail(AESFHE_EARG, "galois needs a rotation/conjugation key");
    if (c->npoly != 2) return fail(AESFHE_EDEGREE, "Input ciphertext should have 2 polynomials");
    KEY_LEVEL_OK(gk, c->level);
    const int N = e->N, l = c->level;
    aesfhe_ct *r = ct_new(e, c->B, 2, l);
    if (c->is_zero) {
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    u64 *p1 = malloc(sizeof(u64) * (size_t)(l + 1) * N);
    u64 *k0 = malloc(sizeof(u64) * (size_t)(l + 1) * N), *k1 = malloc(sizeof(u64) * (size_t)(l + 1) * N);
    for (int b = 0; b < c->B; b++) {
        for (int i = 0; i <= l; i++) galois_perm(e, limb(e, c, b, 1, i), p1 + (size_t)i * N, gk->galois);
        keyswitch(e, p1, l, gk, k0, k1);
        for (int i = 0; i <= l; i++) {
            const u64 q = e->q[i];
            u64 *r0 = limb(e, r, b, 0, i), *r1 = limb(e, r, b, 1, i);
            galois_perm(e, limb(e, c, b, 0, i), r0, gk->galois);
            for (int j = 0; j < N; j++) {
                r0[j] = add_mod(r0[j], k0[(size_t)i * N + j], q);
                r1[j] = k1[(size_t)i * N + j];
            }
        }
    }
    free(p1);
    free(k0);
    free(k1);
    *out = r;
    return 0;
}

/* n rotations with hoisted keys: out_i = sigma_g((c0 + KS_0, KS_1)), KS = keyswitch of c1 (not
 * permuted) with key i; the ModUp of c1 is the same for every key (the HIP engine computes it once) */
int aesfhe_rotate_hoisted(aesfhe_engine *e, const aesfhe_ct *c, const aesfhe_key *const *keys, int32_t n,
                          aesfhe_ct **outs) {
    if (n < 1) return fail(AESFHE_EARG, "rotate_hoisted needs at least one key");
    for (int i = 0; i < n; i++)
        if (!keys[i] || keys[i]->kind != 5) return fail(AESFHE_EARG, "rotate_hoisted needs hoisted rotation keys");
    for (int i = 0; i < n; i++) KEY_LEVEL_OK(keys[i], c->level);
    if (c->npoly != 2) return fail(AESFHE_EDEGREE, "Input ciphertext should have 2 polynomials");
    const int N = e->N, l = c->level;
    u64 *k0 = malloc(sizeof(u64) * (size_t)(l + 1) * N), *k1 = malloc(sizeof(u64) * (size_t)(l + 1) * N);
    u64 *t = malloc(sizeof(u64) * (size_t)N);
    for (int i = 0; i < n; i++) {
        aesfhe_ct *r = ct_new(e, c->B, 2, l);
        outs[i] = r;
        if (c->is_zero) {
            r->is_zero = 1;
            continue;
        }
        for (int b = 0; b < c->B; b++) {
            u64 *c1 = malloc(sizeof(u64) * (size_t)(l + 1) * N);
            for (int p = 0; p <= l; p++) memcpy(c1 + (size_t)p * N, limb(e, c, b, 1, p), sizeof(u64) * N);
            keyswitch(e, c1, l, keys[i], k0, k1);
            free(c1);
            for (int p = 0; p <= l; p++) {
                const u64 q = e->q[p];
                const u64 *c0 = limb(e, c, b, 0, p);
                for (int j = 0; j < N; j++) t[j] = add_mod(c0[j], k0[(size_t)p * N + j], q);
                galois_perm(e, t, limb(e, r, b, 0, p), keys[i]->galois);
                galois_perm(e, k1 + (size_t)p * N, limb(e, r, b, 1, p), keys[i]->galois);
            }
        }
    }
    free(k0);
    free(k1);
    free(t);
    return 0;
}

/* P mod q_i for the Q primes */
static u64 p_mod(const aesfhe_engine *e, int i) {
    const u64 qi = e->q[i];
    u64 P = 1;
    for (int kk = 0; kk < e->K; kk++) P = mul_mod_slow(P, e->q[e->L + 1 + kk] % qi, qi);
    return P;
}

/* Baby-step giant-step linear map with lazy ModDown (include/aesfhe.h).  Per batch
 * element: E_i = sigma_i(P c0 + acc0_i, acc1_i) over Q_l u P (acc_i = ks_acc(c1, bkey_i); NULL
 * key: E = (P c0, P c1), zero special limbs); S_j = sum_t pts_t * E_{tbaby_t} over Q_l u P;
 * part_j = moddown_r(S_j, l, 1); giants: G = sum_{j keyed} [ks_acc(sigma_j(part_j1)) with P
 * sigma_j(part_j0) added to acc0]; out = moddown_r(G, l-1, 0) + sum_{j unkeyed} part_j. */
int aesfhe_linear_bsgs(aesfhe_engine *e, const aesfhe_ct *c, int32_t nb, const aesfhe_key *const *bkeys,
                       int32_t ng, const aesfhe_key *const *gkeys, const int32_t *nterm, const int32_t *tbaby,
                       const aesfhe_pt *const *pts, aesfhe_ct **out) {
    if (nb < 1 || ng < 1) return fail(AESFHE_EARG, "linear_bsgs needs baby and giant steps");
    if (c->npoly != 2) return fail(AESFHE_EDEGREE, "Input ciphertext should have 2 polynomials");
    const int N = e->N, K = e->K, l = c->level, ne = l + 1 + K, nq = e->L + 1;
    if (l < 1) return fail(AESFHE_ELEVEL, "no level left for a linear map");
    int tot = 0;
    for (int j = 0; j < ng; j++) {
        if (nterm[j] < 1 || nterm[j] > 256) return fail(AESFHE_EARG, "giant step with %d terms", nterm[j]);
        if (gkeys[j] && gkeys[j]->kind != 3) return fail(AESFHE_EARG, "giant steps need galois keys");
        tot += nterm[j];
    }
    for (int i = 0; i < nb; i++)
        if (bkeys[i] && bkeys[i]->kind != 5) return fail(AESFHE_EARG, "baby steps need hoisted rotation keys");
    for (int i = 0; i < nb; i++) KEY_LEVEL_OK(bkeys[i], l);
    for (int j = 0; j < ng; j++) KEY_LEVEL_OK(gkeys[j], l - 1);
    for (int t = 0; t < tot; t++) {
        if (tbaby[t] < 0 || tbaby[t] >= nb) return fail(AESFHE_EARG, "bad baby index");
        if (!pts[t] || !pts[t]->ext || pts[t]->level != l) return fail(AESFHE_EARG, "linear_bsgs needs Q u P plaintexts at the input level");
    }
    for (int j = 0, t0 = 0; j < ng; t0 += nterm[j], j++)
        for (int t = t0; t < t0 + nterm[j]; t++)
            for (int t2 = t0; t2 < t; t2++)
                if (tbaby[t2] == tbaby[t]) return fail(AESFHE_EARG, "two terms of one giant on the same baby");
    aesfhe_ct *r = ct_new(e, c->B, 2, l - 1);
    if (c->is_zero) {
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    int pid[MAXP];
    for (int t = 0; t < ne; t++) pid[t] = t <= l ? t : nq + (t - l - 1);
    u64 Pm[MAXP];
    for (int i = 0; i < nq; i++) Pm[i] = p_mod(e, i);
    const size_t eN = (size_t)2 * ne * N;
    u64 *E = malloc(sizeof(u64) * eN * nb), *S = malloc(sizeof(u64) * eN);
    u64 *c1 = malloc(sizeof(u64) * (size_t)(l + 1) * N);
    const int l2 = l - 1, ne2 = l2 + 1 + K;
    aesfhe_ct **parts = calloc((size_t)ng, sizeof *parts);
    for (int j = 0; j < ng; j++) parts[j] = ct_new(e, 1, 2, l2);
    for (int b = 0; b < c->B; b++) {
        /* 1. babies */
        for (int p = 0; p <= l; p++) memcpy(c1 + (size_t)p * N, limb(e, c, b, 1, p), sizeof(u64) * N);
        for (int i = 0; i < nb; i++) {
            u64 *Ei = E + eN * i;
            if (!bkeys[i]) {
                memset(Ei, 0, sizeof(u64) * eN);
                for (int cc = 0; cc < 2; cc++)
                    for (int t = 0; t <= l; t++) {
                        const u64 *src = limb(e, c, b, cc, t);
                        u64 *dst = Ei + ((size_t)cc * ne + t) * N;
                        for (int x = 0; x < N; x++) dst[x] = mul_mod_slow(src[x], Pm[t], e->q[t]);
                    }
                continue;
            }
            u64 *acc = ks_acc(e, c1, l, bkeys[i]);
            for (int t = 0; t <= l; t++) {
                const u64 *c0 = limb(e, c, b, 0, t);
                u64 *a0 = acc + (size_t)t * N;
                for (int x = 0; x < N; x++) a0[x] = add_mod(a0[x], mul_mod_slow(c0[x], Pm[t], e->q[t]), e->q[t]);
            }
            for (size_t y = 0; y < (size_t)2 * ne; y++) galois_perm(e, acc + y * N, Ei + y * N, bkeys[i]->galois);
            free(acc);
        }
        /* 2. giant parts */
        int t0 = 0;
        for (int j = 0; j < ng; j++) {
            memset(S, 0, sizeof(u64) * eN);
            for (int t = t0; t < t0 + nterm[j]; t++) {
                const u64 *Ei = E + eN * tbaby[t];
#pragma omp parallel for schedule(static) num_threads(e->threads)
                for (int y = 0; y < 2 * ne; y++) {
                    const int lt = y % ne, p = pid[lt];
                    const u64 *pv = pts[t]->data + (size_t)lt * N;
                    for (int x = 0; x < N; x++)
                        S[(size_t)y * N + x] = add_mod(S[(size_t)y * N + x], mul_mod(Ei[(size_t)y * N + x], pv[x], &e->mont[p]), e->q[p]);
                }
            }
            t0 += nterm[j];
            moddown_r(e, S, l, 1, limb(e, parts[j], 0, 0, 0), limb(e, parts[j], 0, 1, 0));
        }
        /* 3. giants, one ModDown */
        u64 *G = NULL, *p1 = malloc(sizeof(u64) * (size_t)(l2 + 1) * N), *p0 = malloc(sizeof(u64) * (size_t)(l2 + 1) * N);
        for (int j = 0; j < ng; j++) {
            if (!gkeys[j]) continue;
            for (int t = 0; t <= l2; t++) {
                galois_perm(e, limb(e, parts[j], 0, 1, t), p1 + (size_t)t * N, gkeys[j]->galois);
                galois_perm(e, limb(e, parts[j], 0, 0, t), p0 + (size_t)t * N, gkeys[j]->galois);
            }
            u64 *acc = ks_acc(e, p1, l2, gkeys[j]);
            for (int t = 0; t <= l2; t++) {
                u64 *a0 = acc + (size_t)t * N;
                for (int x = 0; x < N; x++) a0[x] = add_mod(a0[x], mul_mod_slow(p0[(size_t)t * N + x], Pm[t], e->q[t]), e->q[t]);
            }
            if (!G) {
                G = acc;
            } else {
                for (int y = 0; y < 2 * ne2; y++) {
                    const u64 q = e->q[y % ne2 <= l2 ? y % ne2 : nq + (y % ne2 - l2 - 1)];
                    for (int x = 0; x < N; x++) G[(size_t)y * N + x] = add_mod(G[(size_t)y * N + x], acc[(size_t)y * N + x], q);
                }
                free(acc);
            }
        }
        free(p0);
        free(p1);
        u64 *o0 = limb(e, r, b, 0, 0), *o1 = limb(e, r, b, 1, 0);
        if (G) moddown_r(e, G, l2, 0, o0, o1);
        else {
            memset(o0, 0, sizeof(u64) * (size_t)(l2 + 1) * N);
            memset(o1, 0, sizeof(u64) * (size_t)(l2 + 1) * N);
        }
        free(G);
        for (int j = 0; j < ng; j++) {
            if (gkeys[j]) continue;
            for (int cc = 0; cc < 2; cc++)
                for (int t = 0; t <= l2; t++) {
                    u64 *o = limb(e, r, b, cc, t);
                    const u64 *pv = limb(e, parts[j], 0, cc, t);
                    for (int x = 0; x < N; x++) o[x] = add_mod(o[x], pv[x], e->q[t]);
                }
        }
    }
    for (int j = 0; j < ng; j++) aesfhe_ct_free(parts[j]);
    free(parts);
    free(E);
    free(S);
    free(c1);
    *out = r;
    return 0;
}

int aesfhe_power_basis(aesfhe_engine *e, const aesfhe_ct *c, int32_t d, const aesfhe_key *rlk, aesfhe_ct **outs) {
    if (d < 1) return fail(AESFHE_EARG, "degree must be >= 1");
    int need = 0;
    while ((1 << need) < d) need++;
    if (c->level < need) return fail(AESFHE_ELEVEL, "power basis of degree %d needs %d levels, have %d", d, need, c->level);
    if (d > 1) KEY_LEVEL_OK(rlk, c->level);
    aesfhe_ct_copy(e, c, &outs[0]);
    for (int k = 2; k <= d; k++) {
        int hi = 1;
        while (hi * 2 <= k) hi *= 2;
        int rc;
        if (hi == k) rc = aesfhe_mul(e, outs[k / 2 - 1], outs[k / 2 - 1], rlk, &outs[k - 1]);
        else rc = aesfhe_mul(e, outs[hi - 1], outs[k - hi - 1], rlk, &outs[k - 1]);
        if (rc) return rc;
    }
    return 0;
}

int aesfhe_lincomb(aesfhe_engine *e, const aesfhe_ct *const *cts, int32_t n, const double *re,
                   const double *im, aesfhe_ct **out) {
    if (n < 1) return fail(AESFHE_EARG, "empty linear combination");
    int l = cts[0]->level, B = 1, np = 2;
    for (int i = 0; i < n; i++) {
        if (cts[i]->level < l) l = cts[i]->level;
        if (cts[i]->B > B) B = cts[i]->B;
        if (cts[i]->npoly > np) np = cts[i]->npoly;
    }
    for (int i = 0; i < n; i++)
        if (cts[i]->B != B && cts[i]->B != 1) return fail(AESFHE_EARG, "batch mismatch");
    if (l < 1) return fail(AESFHE_ELEVEL, "no level left for a linear combination");
    double s = aesfhe_engine_mul_scale(e, l);
    aesfhe_ct *acc = ct_new(e, B, np, l);
    int any = 0;
    for (int i = 0; i < n; i++) {
        /* inputs above level l are truncated to its limbs (no rescale) and their scale
         * D_level is compensated in the constant: si = s * (D_l / D_level) */
        const double si = s * (e->scales[l] / e->scales[cts[i]->level]);
        i64 A = llround(re[i] * si), Bc = llround(im[i] * si);
        if (cts[i]->is_zero || (A == 0 && Bc == 0)) continue;
        any = 1;
        aesfhe_ct *t = truncate_ct(e, cts[i], l);
        mul_int_const_inplace(e, t, A, Bc);
        for (int b = 0; b < B; b++)
            for (int pp = 0; pp < t->npoly; pp++)
                for (int x = 0; x <= l; x++) {
                    const u64 q = e->q[x];
                    u64 *dst = limb(e, acc, b, pp, x);
                    const u64 *src = limb(e, t, t->B == 1 ? 0 : b, pp, x);
                    for (int j = 0; j < e->N; j++) dst[j] = add_mod(dst[j], src[j], q);
                }
        aesfhe_ct_free(t);
    }
    if (!any) {
        aesfhe_ct_free(acc);
        aesfhe_ct *r = ct_new(e, B, np, l - 1);
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    *out = rescale_raw(e, acc);
    aesfhe_ct_free(acc);
    return 0;
}

/* out = alpha * a * b + gamma * c + beta, one relinearisation + rescale (include/aesfhe.h):
 * (d0, d1, d2) = alpha * tensor(a, b) at l = min(level a, level b) (a, b level-downed to l),
 * plus C * c truncated to l (C = llround(gamma * (D_l * (D_l / D_c)))), plus the constant
 * K = (llround(beta * D_l) mod q) * (llround(D_l) mod q) on d0; then relin + rescale -> l - 1 */
int aesfhe_mul_fma(aesfhe_engine *e, const aesfhe_ct *a, const aesfhe_ct *b, const aesfhe_key *rlk,
                   int64_t alpha, const aesfhe_ct *c, double gamma, double beta, aesfhe_ct **out) {
    if (!rlk || rlk->kind != 2) return fail(AESFHE_EARG, "multiply needs a relinearization key");
    if (a->npoly != 2 || b->npoly != 2) return fail(AESFHE_EDEGREE, "multiply inputs should have 2 polynomials");
    const int l = a->level < b->level ? a->level : b->level;
    if (l < 1) return fail(AESFHE_ELEVEL, "no level left for a ciphertext multiplication");
    int B = a->B > b->B ? a->B : b->B;
    if (c) {
        if (c->npoly != 2) return fail(AESFHE_EDEGREE, "fma addend should have 2 polynomials");
        if (c->level < l) return fail(AESFHE_ELEVEL, "fma addend level %d below the product level %d", c->level, l);
        if (c->B > B) B = c->B;
    }
    if ((a->B != B && a->B != 1) || (b->B != B && b->B != 1) || (c && c->B != B && c->B != 1))
        return fail(AESFHE_EARG, "batch mismatch");
    KEY_LEVEL_OK(rlk, l);
    const int N = e->N;
    aesfhe_ct *t = ct_new(e, B, 3, l);
    if (!a->is_zero && !b->is_zero) {
        aesfhe_ct *x = level_down_raw(e, a, l), *y = level_down_raw(e, b, l);
        tensor_acc(e, x, y, t);
        aesfhe_ct_free(x);
        aesfhe_ct_free(y);
    }
    const i64 Cc = c ? llround(gamma * (e->scales[l] * (e->scales[l] / e->scales[c->level]))) : 0;
    const i64 Rb = llround(beta * e->scales[l]), R = llround(e->scales[l]);
    for (int bb = 0; bb < B; bb++)
        for (int i = 0; i <= l; i++) {
            const u64 q = e->q[i];
            const u64 am = smod(alpha, q), cm = smod(Cc, q);
            const u64 km = mul_mod_slow(smod(Rb, q), smod(R, q), q);
            u64 *d0 = limb(e, t, bb, 0, i), *d1 = limb(e, t, bb, 1, i), *d2 = limb(e, t, bb, 2, i);
            const int cz = !c || c->is_zero;
            const u64 *c0 = cz ? NULL : limb(e, c, c->B == 1 ? 0 : bb, 0, i);
            const u64 *c1 = cz ? NULL : limb(e, c, c->B == 1 ? 0 : bb, 1, i);
            for (int j = 0; j < N; j++) {
                u64 v0 = mul_mod_slow(d0[j], am, q), v1 = mul_mod_slow(d1[j], am, q);
                if (c0) {
                    v0 = add_mod(v0, mul_mod_slow(c0[j], cm, q), q);
                    v1 = add_mod(v1, mul_mod_slow(c1[j], cm, q), q);
                }
                d0[j] = add_mod(v0, km, q);
                d1[j] = v1;
                d2[j] = mul_mod_slow(d2[j], am, q);
            }
        }
    *out = relin_rescale_raw(e, t, rlk, 1);
    aesfhe_ct_free(t);
    return 0;
}

int aesfhe_lincomb_many(aesfhe_engine *e, const aesfhe_ct *const *cts, int32_t n, const double *re,
                        const double *im, int32_t m, aesfhe_ct **outs) {
    for (int r = 0; r < m; r++) {
        int rc = aesfhe_lincomb(e, cts, n, re + (size_t)r * n, im + (size_t)r * n, &outs[r]);
        if (rc) return rc;
    }
    return 0;
}

int aesfhe_dot(aesfhe_engine *e, const aesfhe_ct *const *a, const aesfhe_ct *const *b, int32_t n,
               const aesfhe_key *rlk, aesfhe_ct **out) {
    if (n < 1) return fail(AESFHE_EARG, "empty dot product");
    if (!rlk || rlk->kind != 2) return fail(AESFHE_EARG, "dot needs a relinearization key");
    int l = a[0]->level, B = 1;
    for (int i = 0; i < n; i++) {
        if (a[i]->npoly != 2 || b[i]->npoly != 2) return fail(AESFHE_EDEGREE, "dot inputs should have 2 polynomials");
        if (a[i]->level < l) l = a[i]->level;
        if (b[i]->level < l) l = b[i]->level;
        if (a[i]->B > B) B = a[i]->B;
        if (b[i]->B > B) B = b[i]->B;
    }
    for (int i = 0; i < n; i++)
        if ((a[i]->B != B && a[i]->B != 1) || (b[i]->B != B && b[i]->B != 1)) return fail(AESFHE_EARG, "batch mismatch");
    if (l < 1) return fail(AESFHE_ELEVEL, "no level left for a dot product");
    KEY_LEVEL_OK(rlk, l);
    aesfhe_ct *acc = ct_new(e, B, 3, l);
    int any = 0;
    for (int i = 0; i < n; i++) {
        if (a[i]->is_zero || b[i]->is_zero) continue;
        any = 1;
        aesfhe_ct *x = level_down_raw(e, a[i], l), *y = level_down_raw(e, b[i], l);
        tensor_acc(e, x, y, acc);
        aesfhe_ct_free(x);
        aesfhe_ct_free(y);
    }
    if (!any) {
        aesfhe_ct_free(acc);
        aesfhe_ct *r = ct_new(e, B, 2, l - 1);
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    *out = relin_rescale_raw(e, acc, rlk, 1);
    aesfhe_ct_free(acc);
    return 0;
}

/* sum_i a_i (x) b_i + sum_j gamma_j c_j + beta, one relinearisation + rescale (include/aesfhe.h
 * aesfhe_dot_fma): the aesfhe_dot tensor sum, then every addend truncated to l times
 * C_j = llround(gamma_j * D_l * (D_l / D_cj)) on d0 / d1 and K = llround(beta D_l) llround(D_l)
 * on d0 (the aesfhe_mul_fma constants). */
int aesfhe_dot_fma(aesfhe_engine *e, const aesfhe_ct *const *a, const aesfhe_ct *const *b, int32_t n,
                   const aesfhe_ct *const *c, const double *gamma, int32_t nc, double beta,
                   const aesfhe_key *rlk, aesfhe_ct **out) {
    if (n < 1) return fail(AESFHE_EARG, "empty dot product");
    if (nc < 0) return fail(AESFHE_EARG, "negative addend count");
    if (!rlk || rlk->kind != 2) return fail(AESFHE_EARG, "dot needs a relinearization key");
    int l = a[0]->level, B = 1;
    for (int i = 0; i < n; i++) {
        if (a[i]->npoly != 2 || b[i]->npoly != 2) return fail(AESFHE_EDEGREE, "dot inputs should have 2 polynomials");
        if (a[i]->level < l) l = a[i]->level;
        if (b[i]->level < l) l = b[i]->level;
        if (a[i]->B > B) B = a[i]->B;
        if (b[i]->B > B) B = b[i]->B;
    }
    for (int j = 0; j < nc; j++) {
        if (c[j]->npoly != 2) return fail(AESFHE_EDEGREE, "dot_fma addends should have 2 polynomials");
        if (c[j]->B > B) B = c[j]->B;
    }
    for (int j = 0; j < nc; j++)
        if (c[j]->level < l) return fail(AESFHE_ELEVEL, "dot_fma addend level %d below the product level %d", c[j]->level, l);
    for (int i = 0; i < n; i++)
        if ((a[i]->B != B && a[i]->B != 1) || (b[i]->B != B && b[i]->B != 1)) return fail(AESFHE_EARG, "batch mismatch");
    for (int j = 0; j < nc; j++)
        if (c[j]->B != B && c[j]->B != 1) return fail(AESFHE_EARG, "batch mismatch");
    if (l < 1) return fail(AESFHE_ELEVEL, "no level left for a dot product");
    KEY_LEVEL_OK(rlk, l);
    const int N = e->N;
    aesfhe_ct *acc = ct_new(e, B, 3, l);
    for (int i = 0; i < n; i++) {
        if (a[i]->is_zero || b[i]->is_zero) continue;
        aesfhe_ct *x = level_down_raw(e, a[i], l), *y = level_down_raw(e, b[i], l);
        tensor_acc(e, x, y, acc);
        aesfhe_ct_free(x);
        aesfhe_ct_free(y);
    }
    const i64 Rb = llround(beta * e->scales[l]), R = llround(e->scales[l]);
    for (int j = 0; j < nc; j++) {
        const i64 Cc = llround(gamma[j] * (e->scales[l] * (e->scales[l] / e->scales[c[j]->level])));
        if (c[j]->is_zero || Cc == 0) continue;
        for (int bb = 0; bb < B; bb++)
            for (int i = 0; i <= l; i++) {
                const u64 q = e->q[i], cm = smod(Cc, q);
                u64 *d0 = limb(e, acc, bb, 0, i), *d1 = limb(e, acc, bb, 1, i);
                const u64 *c0 = limb(e, c[j], c[j]->B == 1 ? 0 : bb, 0, i);
                const u64 *c1 = limb(e, c[j], c[j]->B == 1 ? 0 : bb, 1, i);
                for (int k = 0; k < N; k++) {
                    d0[k] = add_mod(d0[k], mul_mod_slow(c0[k], cm, q), q);
                    d1[k] = add_mod(d1[k], mul_mod_slow(c1[k], cm, q), q);
                }
            }
    }
    if (Rb != 0)
        for (int bb = 0; bb < B; bb++)
            for (int i = 0; i <= l; i++) {
                const u64 q = e->q[i], km = mul_mod_slow(smod(Rb, q), smod(R, q), q);
                u64 *d0 = limb(e, acc, bb, 0, i);
                for (int k = 0; k < N; k++) d0[k] = add_mod(d0[k], km, q);
            }
    *out = relin_rescale_raw(e, acc, rlk, 1);
    aesfhe_ct_free(acc);
    return 0;
}

/* Bivariate polynomial over shared power bases (include/aesfhe.h aesfhe_poly2), evaluated
 * term by term: per output, inner sums a_i = F_i0 + sum_{j>=1} F_ij y^j (F = llround(c*S1*
 * rx_i*ry_j), times R = llround(D_l) for an x^0 or y^0 factor, R^2 for both), tensor
 * d = sum_{i>=1} x^i (x) a_i + (a_0, a_0', 0), then relinearisation and two rescales.  Inputs
 * above level l are truncated to l; rx_i = D_l / D_level(x_i) (1 for x^0), ry_j likewise. */
int aesfhe_poly2(aesfhe_engine *e, const aesfhe_ct *const *xb, int32_t nx, const aesfhe_ct *const *yb,
                 int32_t ny, const double *re, const double *im, int32_t m, const aesfhe_key *rlk,
                 aesfhe_ct **outs) {
    if (nx < 1 || ny < 1 || nx > 16 || ny > 16 || m < 1)
        return fail(AESFHE_EARG, "poly2 needs 1 <= nx, ny <= %d and m >= 1", 16);
    if (nx + ny < 3) return fail(AESFHE_EARG, "poly2 needs at least one basis ciphertext");
    if (!rlk || rlk->kind != 2) return fail(AESFHE_EARG, "poly2 needs a relinearization key");
    const aesfhe_ct *all[32] = {0};
    int na = 0;
    for (int i = 0; i < nx - 1; i++) all[na++] = xb[i];
    for (int j = 0; j < ny - 1; j++) all[na++] = yb[j];
    int l = all[0]->level, B = 1;
    for (int a = 0; a < na; a++) {
        if (all[a]->npoly != 2) return fail(AESFHE_EDEGREE, "poly2 inputs should have 2 polynomials");
        if (all[a]->is_zero) return fail(AESFHE_EARG, "poly2 basis ciphertext is zero");
        if (all[a]->level < l) l = all[a]->level;
        if (all[a]->B > B) B = all[a]->B;
    }
    for (int a = 0; a < na; a++)
        if (all[a]->B != B && all[a]->B != 1) return fail(AESFHE_EARG, "batch mismatch");
    if (l < 2) return fail(AESFHE_ELEVEL, "no level left for a bivariate polynomial");
    KEY_LEVEL_OK(rlk, l);
    const double *D = e->scales;
    const double S1 = D[l - 2] / D[l] * ((double)e->q[l] / D[l]) * (double)e->q[l - 1];
    const i64 R = llround(D[l]);
    const int per = nx * ny, N = e->N;
    double rx[16], ry[16];
    rx[0] = ry[0] = 1.0;
    for (int i = 1; i < nx; i++) rx[i] = D[l] / D[xb[i - 1]->level];
    for (int j = 1; j < ny; j++) ry[j] = D[l] / D[yb[j - 1]->level];
    aesfhe_ct *al[32];
    for (int a = 0; a < na; a++) al[a] = truncate_ct(e, all[a], l);
    aesfhe_ct **X = al, **Y = al + (nx - 1);
    i64 *A = malloc(sizeof(i64) * per), *Bc = malloc(sizeof(i64) * per);
    for (int t = 0; t < m; t++) {
        int any = 0;
        for (int c = 0; c < per; c++) {
            A[c] = llround(re[(size_t)t * per + c] * S1 * rx[c / ny] * ry[c % ny]);
            Bc[c] = llround(im[(size_t)t * per + c] * S1 * rx[c / ny] * ry[c % ny]);
            if (A[c] || Bc[c]) any = 1;
        }
        if (!any) {
            outs[t] = ct_new(e, B, 2, l - 2);
            outs[t]->is_zero = 1;
            continue;
        }
        aesfhe_ct *acc = ct_new(e, B, 3, l);
#pragma omp parallel for schedule(static) num_threads(e->threads)
        for (int li = 0; li <= l; li++) {
            const u64 q = e->q[li];
            const mont_t *mt = &e->mont[li];
            const u64 r1 = smod(R, q), r2 = mul_mod_slow(r1, r1, q), I = e->iroot[li];
            u64 f[2][256], fp[2][256];
            for (int c = 0; c < per; c++) {
                const int j = c % ny, i = c / ny;
                const u64 sc = (i == 0 && j == 0) ? r2 : (i == 0 || j == 0) ? r1 : 1;
                const u64 a = mul_mod_slow(smod(A[c], q), sc, q), b = mul_mod_slow(smod(Bc[c], q), sc, q);
                const u64 bi = mul_mod_slow(b, I, q);
                f[0][c] = add_mod(a, bi, q);
                f[1][c] = sub_mod(a, bi, q);
                fp[0][c] = shoup_pre(f[0][c], q);
                fp[1][c] = shoup_pre(f[1][c], q);
            }
            for (int b = 0; b < B; b++) {
                u64 *d0 = limb(e, acc, b, 0, li), *d1 = limb(e, acc, b, 1, li), *d2 = limb(e, acc, b, 2, li);
                for (int k = 0; k < N; k++) {
                    const int hh = k >= N / 2;
                    u64 s0 = 0, s1 = 0, s2 = 0;
                    for (int i = 0; i < nx; i++) {
                        u64 a0 = f[hh][i * ny], a1 = 0;
                        for (int j = 1; j < ny; j++) {
                            const aesfhe_ct *y = Y[j - 1];
                            const int yb_ = y->B == 1 ? 0 : b;
                            const int c = i * ny + j;
                            a0 = add_mod(a0, mul_shoup(limb(e, y, yb_, 0, li)[k], f[hh][c], fp[hh][c], q), q);
                            a1 = add_mod(a1, mul_shoup(limb(e, y, yb_, 1, li)[k], f[hh][c], fp[hh][c], q), q);
                        }
                        if (i == 0) {
                            s0 = add_mod(s0, a0, q);
                            s1 = add_mod(s1, a1, q);
                        } else {
                            const aesfhe_ct *x = X[i - 1];
                            const int xb_ = x->B == 1 ? 0 : b;
                            const u64 x0 = limb(e, x, xb_, 0, li)[k], x1 = limb(e, x, xb_, 1, li)[k];
                            s0 = add_mod(s0, mul_mod(x0, a0, mt), q);
                            s1 = add_mod(s1, add_mod(mul_mod(x0, a1, mt), mul_mod(x1, a0, mt), q), q);
                            s2 = add_mod(s2, mul_mod(x1, a1, mt), q);
                        }
                    }
                    d0[k] = s0;
                    d1[k] = s1;
                    d2[k] = s2;
                }
            }
        }
        outs[t] = relin_rescale_raw(e, acc, rlk, 2);
        aesfhe_ct_free(acc);
    }
    free(A);
    free(Bc);
    for (int a = 0; a < na; a++) aesfhe_ct_free(al[a]);
    return 0;
}

/* Integer-weight bivariate polynomial (include/aesfhe.h aesfhe_poly2_int): term by term with
 * F_ij = w_ij * H(cx(i), cy(j)) mod q; classes cx = 0 for x^0, else 1 + rank of the basis level
 * among the distinct levels (highest first); H = llround(S1 * r_x * r_y / den) mod q (times R
 * per x^0 / y^0 factor).  Tensor, relinearisation and two rescales as aesfhe_poly2. */
static int level_class(const aesfhe_ct *const *b, int n, int i, int *lev, int *nlev) {
    if (i == 0) return 0;
    (void)n;
    int L = b[i - 1]->level, rank = 0;
    for (int k = 0; k < *nlev; k++)
        if (lev[k] > L) rank++;
    return 1 + rank;
}

int aesfhe_poly2_int(aesfhe_engine *e, const aesfhe_ct *const *xb, int32_t nx, const aesfhe_ct *const *yb,
                     int32_t ny, const int32_t *w, int32_t den, int32_t m, const aesfhe_key *rlk,
                     aesfhe_ct **outs) {
    if (nx < 1 || ny < 1 || nx > 16 || ny > 16 || m < 1)
        return fail(AESFHE_EARG, "poly2 needs 1 <= nx, ny <= %d and m >= 1", 16);
    if (nx + ny < 3) return fail(AESFHE_EARG, "poly2 needs at least one basis ciphertext");
    if (den < 1) return fail(AESFHE_EARG, "poly2_int needs den >= 1");
    if (!rlk || rlk->kind != 2) return fail(AESFHE_EARG, "poly2 needs a relinearization key");
    const aesfhe_ct *all[32] = {0};
    int na = 0;
    for (int i = 0; i < nx - 1; i++) all[na++] = xb[i];
    for (int j = 0; j < ny - 1; j++) all[na++] = yb[j];
    int l = all[0]->level, B = 1;
    for (int a = 0; a < na; a++) {
        if (all[a]->npoly != 2) return fail(AESFHE_EDEGREE, "poly2 inputs should have 2 polynomials");
        if (all[a]->is_zero) return fail(AESFHE_EARG, "poly2 basis ciphertext is zero");
        if (all[a]->level < l) l = all[a]->level;
        if (all[a]->B > B) B = all[a]->B;
    }
    for (int a = 0; a < na; a++)
        if (all[a]->B != B && all[a]->B != 1) return fail(AESFHE_EARG, "batch mismatch");
    if (l < 2) return fail(AESFHE_ELEVEL, "no level left for a bivariate polynomial");
    KEY_LEVEL_OK(rlk, l);
    for (int t = 0; t < m; t++)
        for (int i = 0; i < nx; i++) {
            long sum = 0;
            for (int j = 0; j < ny; j++) sum += labs((long)w[((size_t)t * nx + i) * ny + j]);
            if (sum > 512) return fail(AESFHE_EARG, "poly2_int: sum of |w| over a row exceeds 512");
        }
    const double *D = e->scales;
    const double S1 = D[l - 2] / D[l] * ((double)e->q[l] / D[l]) * (double)e->q[l - 1];
    const i64 R = llround(D[l]);
    int levx[16], nlx = 0, levy[16], nly = 0;  /* distinct basis levels */
    for (int i = 0; i < nx - 1; i++) {
        int f = 0;
        for (int k = 0; k < nlx; k++) f |= levx[k] == xb[i]->level;
        if (!f) levx[nlx++] = xb[i]->level;
    }
    for (int j = 0; j < ny - 1; j++) {
        int f = 0;
        for (int k = 0; k < nly; k++) f |= levy[k] == yb[j]->level;
        if (!f) levy[nly++] = yb[j]->level;
    }
    int cx[16], cy[16];
    for (int i = 0; i < nx; i++) cx[i] = level_class(xb, nx, i, levx, &nlx);
    for (int j = 0; j < ny; j++) cy[j] = level_class(yb, ny, j, levy, &nly);
    /* level of each class (index 1..): the class rank order */
    double rxc[17], ryc[17];
    rxc[0] = ryc[0] = 1.0;
    for (int i = 1; i < nx; i++) rxc[cx[i]] = D[l] / D[xb[i - 1]->level];
    for (int j = 1; j < ny; j++) ryc[cy[j]] = D[l] / D[yb[j - 1]->level];
    const int N = e->N;
    aesfhe_ct *al[32];
    for (int a = 0; a < na; a++) al[a] = truncate_ct(e, all[a], l);
    aesfhe_ct **X = al, **Y = al + (nx - 1);
    for (int t = 0; t < m; t++) {
        int any = 0;
        for (int c = 0; c < nx * ny; c++) any |= w[(size_t)t * nx * ny + c] != 0;
        if (!any) {
            outs[t] = ct_new(e, B, 2, l - 2);
            outs[t]->is_zero = 1;
            continue;
        }
        aesfhe_ct *acc = ct_new(e, B, 3, l);
#pragma omp parallel for schedule(static) num_threads(e->threads)
        for (int li = 0; li <= l; li++) {
            const u64 q = e->q[li];
            const mont_t *mt = &e->mont[li];
            const u64 r1 = smod(R, q);
            u64 F[16][16], Fp[16][16];
            for (int i = 0; i < nx; i++)
                for (int j = 0; j < ny; j++) {
                    u64 h = smod(llround(S1 * rxc[cx[i]] * ryc[cy[j]] / (double)den), q);
                    if (cx[i] == 0) h = mul_mod_slow(h, r1, q);
                    if (cy[j] == 0) h = mul_mod_slow(h, r1, q);
                    F[i][j] = mul_mod_slow(smod(w[((size_t)t * nx + i) * ny + j], q), h, q);
                    Fp[i][j] = shoup_pre(F[i][j], q);
                }
            for (int b = 0; b < B; b++) {
                u64 *d0 = limb(e, acc, b, 0, li), *d1 = limb(e, acc, b, 1, li), *d2 = limb(e, acc, b, 2, li);
                for (int k = 0; k < N; k++) {
                    u64 s0 = 0, s1 = 0, s2 = 0;
                    for (int i = 0; i < nx; i++) {
                        u64 a0 = F[i][0], a1 = 0;
                        for (int j = 1; j < ny; j++) {
                            const aesfhe_ct *y = Y[j - 1];
                            const int yb_ = y->B == 1 ? 0 : b;
                            a0 = add_mod(a0, mul_shoup(limb(e, y, yb_, 0, li)[k], F[i][j], Fp[i][j], q), q);
                            a1 = add_mod(a1, mul_shoup(limb(e, y, yb_, 1, li)[k], F[i][j], Fp[i][j], q), q);
                        }
                        if (i == 0) {
                            s0 = add_mod(s0, a0, q);
                            s1 = add_mod(s1, a1, q);
                        } else {
                            const aesfhe_ct *x = X[i - 1];
                            const int xb_ = x->B == 1 ? 0 : b;
                            const u64 x0 = limb(e, x, xb_, 0, li)[k], x1 = limb(e, x, xb_, 1, li)[k];
                            s0 = add_mod(s0, mul_mod(x0, a0, mt), q);
                            s1 = add_mod(s1, add_mod(mul_mod(x0, a1, mt), mul_mod(x1, a0, mt), q), q);
                            s2 = add_mod(s2, mul_mod(x1, a1, mt), q);
                        }
                    }
                    d0[k] = s0;
                    d1[k] = s1;
                    d2[k] = s2;
                }
            }
        }
        outs[t] = relin_rescale_raw(e, acc, rlk, 2);
        aesfhe_ct_free(acc);
    }
    for (int a = 0; a < na; a++) aesfhe_ct_free(al[a]);
    return 0;
}

/* aesfhe_poly2_int, then each output's batch rotated within slabs of 4 (include/aesfhe.h) */
int aesfhe_poly2_int_rot(aesfhe_engine *e, const aesfhe_ct *const *xb, int32_t nx, const aesfhe_ct *const *yb,
                         int32_t ny, const int32_t *w, int32_t den, int32_t m, const aesfhe_key *rlk,
                         int32_t slab_rot, aesfhe_ct **outs) {
    if (slab_rot < 0 || slab_rot > 3) return fail(AESFHE_EARG, "slab rotation %d outside 0..3", slab_rot);
    int B = 1;
    for (int i = 0; i < nx - 1; i++) B = xb[i]->B > B ? xb[i]->B : B;
    for (int j = 0; j < ny - 1; j++) B = yb[j]->B > B ? yb[j]->B : B;
    if (slab_rot && B % 4) return fail(AESFHE_EARG, "slab rotation needs a batch of whole slabs (4 s), got %d", B);
    int rc = aesfhe_poly2_int(e, xb, nx, yb, ny, w, den, m, rlk, outs);
    if (rc || !slab_rot) return rc;
    for (int t = 0; t < m; t++) {
        aesfhe_ct *c = outs[t];
        const size_t per = (size_t)c->npoly * (c->level + 1) * e->N;
        u64 *tmp = malloc(sizeof(u64) * per * c->B);
        for (int b = 0; b < c->B; b++) {
            const int src = (b & ~3) | ((b + slab_rot) & 3);
            memcpy(tmp + per * b, c->data + per * src, sizeof(u64) * per);
        }
        memcpy(c->data, tmp, sizeof(u64) * per * c->B);
        free(tmp);
    }
    return 0;
}

/* ModRaise (include/aesfhe.h aesfhe_mod_raise) */
int aesfhe_mod_raise(aesfhe_engine *e, const aesfhe_ct *c, int32_t level, aesfhe_ct **out) {
    if (level < 0 || level > e->L) return fail(AESFHE_EARG, "bad mod-raise level");
    const int N = e->N;
    aesfhe_ct *r = ct_new(e, c->B, c->npoly, level);
    if (c->is_zero) {
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    const u64 q0 = e->q[0];
    for (int b = 0; b < c->B; b++)
        for (int pp = 0; pp < c->npoly; pp++) {
            i64 *x = malloc(sizeof(i64) * N);
            u64 *t = malloc(sizeof(u64) * N);
            memcpy(t, limb(e, c, b, pp, 0), sizeof(u64) * N);
            ntt_inv(e, t, 0);
            for (int k = 0; k < N; k++) x[k] = t[k] > (q0 >> 1) ? (i64)t[k] - (i64)q0 : (i64)t[k];
#pragma omp parallel for schedule(static) num_threads(e->threads)
            for (int i = 0; i <= level; i++) coeffs_to_ntt(e, x, limb(e, r, b, pp, i), i);
            free(x);
            free(t);
        }
    *out = r;
    return 0;
}

/* multiplication by +-X^{N/2} (every slot times +-i), exact */
int aesfhe_mul_i(aesfhe_engine *e, const aesfhe_ct *c, int32_t sign, aesfhe_ct **out) {
    aesfhe_ct *r;
    aesfhe_ct_copy(e, c, &r);
    if (!c->is_zero) mul_int_const_inplace(e, r, 0, sign >= 0 ? 1 : -1);
    *out = r;
    return 0;
}

/* sum_i ct_i * pt_i, one rescale (include/aesfhe.h aesfhe_dot_pt) */
int aesfhe_dot_pt(aesfhe_engine *e, const aesfhe_ct *const *cts, const aesfhe_pt *const *pts, int32_t n,
                  aesfhe_ct **out) {
    if (n < 1 || n > 256) return fail(AESFHE_EARG, "dot_pt needs 1..256 terms");
    int l = cts[0]->level, B = 1, np = cts[0]->npoly;
    for (int i = 0; i < n; i++) {
        if (cts[i]->level < l) l = cts[i]->level;
        if (cts[i]->B > B) B = cts[i]->B;
        if (cts[i]->npoly != np) return fail(AESFHE_EDEGREE, "dot_pt inputs should have the same number of polynomials");
    }
    for (int i = 0; i < n; i++) {
        if (cts[i]->B != B && cts[i]->B != 1) return fail(AESFHE_EARG, "batch mismatch");
        if (pts[i]->level < l) return fail(AESFHE_EARG, "plaintext level %d below ciphertext level %d", pts[i]->level, l);
    }
    if (l < 1) return fail(AESFHE_ELEVEL, "no level left for a plaintext dot product");
    aesfhe_ct *acc = ct_new(e, B, np, l);
    int any = 0;
    for (int i = 0; i < n; i++) {
        if (cts[i]->is_zero) continue;
        any = 1;
        aesfhe_ct *t = level_down_raw(e, cts[i], l);
        for (int b = 0; b < B; b++)
            for (int pp = 0; pp < np; pp++)
#pragma omp parallel for schedule(static) num_threads(e->threads)
                for (int x = 0; x <= l; x++) {
                    const u64 q = e->q[x];
                    const u64 *src = limb(e, t, t->B == 1 ? 0 : b, pp, x);
                    const u64 *pv = pts[i]->data + (size_t)x * e->N;
                    u64 *dst = limb(e, acc, b, pp, x);
                    for (int j = 0; j < e->N; j++) dst[j] = add_mod(dst[j], mul_mod(src[j], pv[j], &e->mont[x]), q);
                }
        aesfhe_ct_free(t);
    }
    if (!any) {
        aesfhe_ct_free(acc);
        aesfhe_ct *r = ct_new(e, B, np, l - 1);
        r->is_zero = 1;
        *out = r;
        return 0;
    }
    *out = rescale_raw(e, acc);
    aesfhe_ct_free(acc);
    return 0;
}

int aesfhe_ntt_host(aesfhe_engine *e, uint64_t *limbs, int32_t nlimb, const int32_t *pids, int32_t inv) {
    for (int i = 0; i < nlimb; i++)
        if (pids[i] < 0 || pids[i] >= e->np) return fail(AESFHE_EARG, "bad prime index");
#pragma omp parallel for schedule(static) num_threads(e->threads)
    for (int i = 0; i < nlimb; i++) {
        if (inv) ntt_inv(e, limbs + (size_t)i * e->N, pids[i]);
        else ntt_fwd(e, limbs + (size_t)i * e->N, pids[i]);
    }
    return 0;
}

int aesfhe_bench_ntt(aesfhe_engine *e, int32_t nlimb, int32_t iters, double *fwd_ms, double *inv_ms) {
    u64 *buf = malloc(sizeof(u64) * (size_t)nlimb * e->N);
    for (size_t i = 0; i < (size_t)nlimb * e->N; i++) buf[i] = i % e->q[0];
    double t0 = now_ms();
    for (int it = 0; it < iters; it++)
        for (int i = 0; i < nlimb; i++) ntt_fwd(e, buf + (size_t)i * e->N, i % (e->L + 1));
    double t1 = now_ms();
    for (int it = 0; it < iters; it++)
        for (int i = 0; i < nlimb; i++) ntt_inv(e, buf + (size_t)i * e->N, i % (e->L + 1));
    double t2 = now_ms();
    *fwd_ms = (t1 - t0) / iters;
    *inv_ms = (t2 - t1) / iters;
    free(buf);
    return 0;
}
