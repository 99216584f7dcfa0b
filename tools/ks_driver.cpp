// Product-multiply driver over the C ABI only (dev tool for PMC collection without Python):
// B ciphertexts at N = 2^16, L = 30, `iters` ct x ct multiplies (tensor + fused relinearise /
// rescale) at levels 30 -> 30-iters, so NTT, ModUp, inner product and ModDown kernels all run.
//   ./tools/ks_driver [B] [iters]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../include/aesfhe.h"
#define CK(x) do { int rc_ = (x); if (rc_) { printf("%s -> %d: %s\n", #x, rc_, aesfhe_last_error()); return 1; } } while (0)

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 16, iters = argc > 2 ? atoi(argv[2]) : 8;
    aesfhe_params p = {16, 30, 8, 40, 50, 50, 0, 0, 1, nullptr};
    aesfhe_engine* e;
    CK(aesfhe_engine_create(&p, &e));
    aesfhe_key *sk, *rlk;
    CK(aesfhe_key_secret(e, 3, &sk));
    CK(aesfhe_key_relin(e, sk, &rlk));
    const int N = 1 << 16;
    std::vector<int64_t> co((size_t)B * N);
    for (size_t i = 0; i < co.size(); i++) co[i] = (int64_t)((i * 2654435761u) % 1000) - 500;
    aesfhe_ct *a, *b;
    CK(aesfhe_encrypt(e, sk, co.data(), B, 30, 1, &a));
    CK(aesfhe_encrypt(e, sk, co.data(), B, 30, 2, &b));
    for (int it = 0; it < iters; it++) {
        aesfhe_ct *c, *d;
        CK(aesfhe_mul(e, a, b, rlk, &c));
        CK(aesfhe_mul(e, b, b, rlk, &d));
        aesfhe_ct_free(a);
        aesfhe_ct_free(b);
        a = c;
        b = d;
    }
    CK(aesfhe_engine_sync(e));
    printf("ks_driver ok: B=%d, %d multiply pairs\n", B, iters);
    aesfhe_ct_free(a);
    aesfhe_ct_free(b);
    aesfhe_key_free(rlk);
    aesfhe_key_free(sk);
    aesfhe_engine_destroy(e);
    return 0;
}
