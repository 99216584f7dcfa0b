/* oracle_chacha_kat.c -- the CPU oracle's ChaCha20 (oracle/ckks_oracle.c, included whole so that its
 * static PRNG is reachable) against the RFC 7539 section 2.3.2 block-function vector, and its
 * one-block cache against uncached blocks (tests/test_asan.py builds and runs it). */
#include "../../oracle/ckks_oracle.c"

int main(void) {
    uint32_t k[8];
    for (int i = 0; i < 8; i++)
        k[i] = (uint32_t)(4 * i) | (uint32_t)(4 * i + 1) << 8 | (uint32_t)(4 * i + 2) << 16 | (uint32_t)(4 * i + 3) << 24;
    const uint32_t want[16] = {0xe4e7f110, 0x15593bd1, 0x1fdd0f50, 0xc47120a3, 0xc7f4d1c7, 0x0368c033,
                               0x9aaa2204, 0x4e6cd4c3, 0x466482d2, 0x09aa9f07, 0x05d7c214, 0xa2028bd9,
                               0xd19c12b5, 0xb94e16de, 0xe883d0cb, 0x4e3c50a2};
    const u64 ctr = 1ULL | (0x09000000ULL << 32), label = 0x4a000000ULL;
    uint32_t o[16];
    chacha20_block(k, label, ctr, o);
    for (int i = 0; i < 16; i++)
        if (o[i] != want[i]) return 1;
    for (int j = 7; j >= 0; j--) /* cached and uncached words agree, any order */
        if (rnd(k, label, (ctr << 3) + j) != ((u64)want[2 * j] | (u64)want[2 * j + 1] << 32)) return 2;
    printf("oracle chacha ok\n");
    return 0;
}
