// host_asan.cpp -- sanitizer run of the HIP engine's host-side code (aes-fhe_amd/csrc/ckks_host.h:
// prime chain, roots, PRNG, canonical-embedding codec), built with g++ -fsanitize=address,undefined
// by tests/test_asan.py.  The device code cannot be sanitized on this pool; the host pieces that
// index tables and buffers are exercised here at every supported ring size.
#include <cstdio>
#include <vector>

#include "../../aes-fhe_amd/csrc/ckks_host.h"

using namespace aesfhe;

int main() {
    for (int logN = 10; logN <= 17; logN++) {
        const int N = 1 << logN, L = logN >= 16 ? 30 : 8, K = logN >= 16 ? 10 : 3;
        Chain c = make_chain(logN, L, K, 50, 50, 40);
        if ((int)c.q.size() != L + 1 + K || (int)c.scale.size() != L + 1) return 1;
        for (u64 q : c.q) {
            if (!is_prime_u64(q) || q % (2ULL * N) != 1) return 2;
            u64 psi = min_primitive_root(q, N);
            if (h_powmod(psi, (u64)N, q) != q - 1) return 3;
        }
        std::vector<double> sc = scales_from_primes(c.q, L, 40);
        if (sc.size() != (size_t)L + 1) return 4;
        Codec cd(logN);
        std::vector<double> re(N / 2), im(N / 2), r0(N / 2), i0(N / 2);
        for (int i = 0; i < N / 2; i++) {
            re[i] = r0[i] = (double)(mix64(i) % 1000) / 500.0 - 1.0;
            im[i] = i0[i] = (double)(mix64(i + N) % 1000) / 500.0 - 1.0;
        }
        cd.special_inv(re.data(), im.data());
        cd.special(re.data(), im.data());
        for (int i = 0; i < N / 2; i++)
            if (std::fabs(re[i] - r0[i]) > 1e-9 || std::fabs(im[i] - i0[i]) > 1e-9) return 5;
        long t = 0;
        for (int i = 0; i < 4096; i++) t += ternary(mix64(i)) + cbd21(mix64(i + 7));
        (void)t;
    }
    std::printf("host_asan ok\n");
    return 0;
}
