/* asan_check.c -- host-memory sanitizer run of the CPU oracle (test infrastructure only).
 *
 * Built with -fsanitize=address,undefined together with ckks_oracle.c (oracle/Makefile target
 * `asan`) and run by tests/test_asan.py: every ABI entry point family the tests use is driven
 * once at a small ring (N = 2^10) -- engine, keys of every kind, encrypt / decrypt, the codec,
 * add / mul / rescale / rotate / conjugate, power basis, lincomb, dot, poly2_int, hoisted
 * rotations, linear_bsgs, mod_raise, key and ciphertext export / import -- and every object is
 * freed, the engine first (the teardown order the GPU engine's refcount exists for).  Exit 0
 * and no sanitizer report = pass. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/aesfhe.h"

#define CK(x)                                                                      \
    do {                                                                           \
        int rc_ = (x);                                                             \
        if (rc_) {                                                                 \
            fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,  \
                    aesfhe_last_error());                                          \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(void) {
    const int logn = 10, N = 1 << logn, n = N / 2, L = 8, K = 3;
    aesfhe_params p = {logn, L, K, 40, 50, 50, 0, 2, 12345, NULL};
    aesfhe_engine *e;
    CK(aesfhe_engine_create(&p, &e));
    aesfhe_key *sk, *pk, *rlk, *cjk, *rot, *hk[2], *sparse, *swk;
    CK(aesfhe_key_secret(e, 1, &sk));
    CK(aesfhe_key_public(e, sk, &pk));
    CK(aesfhe_key_relin(e, sk, &rlk));
    CK(aesfhe_key_galois(e, sk, aesfhe_galois_elt(logn, 0, 1), &cjk));
    CK(aesfhe_key_galois(e, sk, aesfhe_galois_elt(logn, -3, 0), &rot));
    CK(aesfhe_key_galois_hoisted(e, sk, aesfhe_galois_elt(logn, -1, 0), &hk[0]));
    CK(aesfhe_key_galois_hoisted(e, sk, aesfhe_galois_elt(logn, 5, 0), &hk[1]));
    CK(aesfhe_key_secret_sparse(e, 2, 32, &sparse));
    CK(aesfhe_key_switch(e, sk, sparse, &swk));

    double *re = calloc(n, sizeof(double)), *im = calloc(n, sizeof(double));
    int64_t *co = calloc(2 * (size_t)N, sizeof(int64_t));
    double sc[64];
    uint64_t primes[64];
    CK(aesfhe_engine_scales(e, sc));
    CK(aesfhe_engine_primes(e, primes));
    for (int i = 0; i < n; i++) { re[i] = (i % 7) / 7.0; im[i] = -(i % 3) / 5.0; }
    CK(aesfhe_encode(logn, re, im, n, sc[L], co));
    CK(aesfhe_encode(logn, re, im, n, sc[L], co + N));
    aesfhe_ct *a, *b, *m, *r, *c, *pb[4], *lc, *dt, *hr[2], *lb, *mr, *sw, *imp, *sl, *cat;
    CK(aesfhe_encrypt(e, pk, co, 2, L, 0, &a));
    CK(aesfhe_encrypt(e, sk, co, 1, L, 1, &b));
    CK(aesfhe_mul(e, a, b, rlk, &m));
    CK(aesfhe_galois(e, m, rot, &r));
    CK(aesfhe_galois(e, r, cjk, &c));
    CK(aesfhe_power_basis(e, b, 4, rlk, pb));
    double lre[3] = {0.5, -1.0, 0.25}, lim[3] = {0.0, 0.5, 0.0};
    CK(aesfhe_lincomb(e, (const aesfhe_ct *const *)pb, 3, lre, lim, &lc));
    CK(aesfhe_dot(e, (const aesfhe_ct *const *)pb, (const aesfhe_ct *const *)pb + 1, 2, rlk, &dt));
    CK(aesfhe_rotate_hoisted(e, a, (const aesfhe_key *const *)hk, 2, hr));
    aesfhe_pt *pt;
    CK(aesfhe_pt_create_ext(e, co, L, &pt));
    const aesfhe_key *bk[2] = {NULL, hk[0]}, *gk[1] = {rot};
    int32_t nterm[1] = {2}, tb[2] = {0, 1};
    const aesfhe_pt *pts[2] = {pt, pt};
    CK(aesfhe_linear_bsgs(e, a, 2, bk, 1, gk, nterm, tb, pts, &lb));
    aesfhe_ct *low;
    CK(aesfhe_level_down(e, a, 0, &low));
    CK(aesfhe_mod_raise(e, low, L, &mr));
    CK(aesfhe_galois(e, low, swk, &sw));
    int32_t w[2 * 2 * 2] = {1, -2, 3, 0, 4, 1, -1, 2};
    aesfhe_ct *xb[1] = {pb[1]}, *yb[1] = {pb[0]}, *p2[2];
    CK(aesfhe_poly2_int(e, (const aesfhe_ct *const *)xb, 2, (const aesfhe_ct *const *)yb, 2, w, 64, 2, rlk, p2));
    /* export / import */
    int32_t info[4];
    CK(aesfhe_ct_info(m, info));
    size_t words = (size_t)info[0] * info[1] * (info[2] + 1) * N;
    uint64_t *buf = malloc(words * 8);
    CK(aesfhe_ct_export(e, m, buf));
    CK(aesfhe_ct_import(e, buf, info[0], info[1], info[2], &imp));
    CK(aesfhe_ct_export_device(e, m, 1, 1, buf));
    CK(aesfhe_ct_slice(e, m, 1, 1, &sl));
    const aesfhe_ct *parts[2] = {sl, imp};
    CK(aesfhe_ct_concat(e, parts, 2, &cat));
    int32_t kind; uint64_t g, ks; int64_t kw;
    CK(aesfhe_key_export(e, rlk, &kind, &g, &ks, &kw, NULL));
    uint64_t *kb = malloc((size_t)kw * 8);
    CK(aesfhe_key_export(e, rlk, &kind, &g, &ks, &kw, kb));
    aesfhe_key *rlk2;
    CK(aesfhe_key_import(e, kind, g, ks, kb, kw, &rlk2));
    int64_t *dec = malloc(sizeof(int64_t) * 3 * (size_t)N);
    CK(aesfhe_decrypt(e, sk, c, dec));
    CK(aesfhe_ct_info(c, info));
    CK(aesfhe_decode(logn, dec, sc[info[2]], re, im));
    /* errors are reported, not crashed on */
    aesfhe_ct *bad;
    if (aesfhe_relinearize(e, a, rlk, &bad) != AESFHE_EDEGREE) return 2;
    if (aesfhe_ct_slice(e, a, 1, 5, &bad) != AESFHE_EARG) return 3;
    /* engine first, then its objects */
    aesfhe_engine_destroy(e);
    aesfhe_ct *cts[] = {a, b, m, r, c, pb[0], pb[1], pb[2], pb[3], lc, dt, hr[0], hr[1], lb, low, mr, sw,
                        p2[0], p2[1], imp, sl, cat};
    for (size_t i = 0; i < sizeof cts / sizeof cts[0]; i++) aesfhe_ct_free(cts[i]);
    aesfhe_key *keys[] = {sk, pk, rlk, cjk, rot, hk[0], hk[1], sparse, swk, rlk2};
    for (size_t i = 0; i < sizeof keys / sizeof keys[0]; i++) aesfhe_key_free(keys[i]);
    aesfhe_pt_free(pt);
    free(re); free(im); free(co); free(buf); free(kb); free(dec);
    printf("asan_check ok\n");
    return 0;
}
