// host_asan.cpp -- sanitizer run of the HIP engine's host-side code (aes-fhe_amd/csrc/ckks_host.h:
// prime chain, roots, PRNG, canonical-embedding codec), built with g++ -fsanitize=address,undefined
// by tests/test_asan.py.  The device code cannot be sanitized on this pool; the host pieces that
// index tables and buffers are exercised here at every supported ring size.
#include <cstdio>
#include <vector>

#include "../../aes-fhe_amd/csrc/ckks_host.h"

using namespace aesfhe;

// RFC 7539 section 2.3.2 block-function vector: key 00..1f, block count 1, nonce 00 00 00 09 00 00
// 00 4a 00 00 00 00 -- in this 64-bit counter / 64-bit nonce layout: ctr = 1 | 0x09000000 << 32,
// label = 0x4a000000.
static int chacha_kat() {
    ChaKey K;
    for (int i = 0; i < 8; i++)
        K.k[i] = (uint32_t)(4 * i) | (uint32_t)(4 * i + 1) << 8 | (uint32_t)(4 * i + 2) << 16 | (uint32_t)(4 * i + 3) << 24;
    const uint32_t want[16] = {0xe4e7f110, 0x15593bd1, 0x1fdd0f50, 0xc47120a3, 0xc7f4d1c7, 0x0368c033,
                               0x9aaa2204, 0x4e6cd4c3, 0x466482d2, 0x09aa9f07, 0x05d7c214, 0xa2028bd9,
                               0xd19c12b5, 0xb94e16de, 0xe883d0cb, 0x4e3c50a2};
    uint32_t o[16];
    chacha20_block(K, 0x4a000000ULL, 1ULL | (0x09000000ULL << 32), o);
    for (int i = 0; i < 16; i++)
        if (o[i] != want[i]) return 1;
    // rnd: word idx mod 8 of block idx / 8
    const u64 r = rnd(K, 0x4a000000ULL, ((1ULL | (0x09000000ULL << 32)) << 3) + 2);
    return r == ((u64)want[4] | (u64)want[5] << 32) ? 0 : 2;
}

int main() {
    if (int rc = chacha_kat()) {
        std::printf("chacha20 KAT failed (%d)\n", rc);
        return 10 + rc;
    }
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
