// bsgs_plan_asan.cpp -- sanitizer run of aesfhe_linear_bsgs's host planning
// (aes-fhe_amd/csrc/bsgs_plan.h), built with g++ -fsanitize=address,undefined by tests/test_asan.py.
// Random term lists (every chunk size, uneven last chunk, 1..256 terms per giant) are checked
// against a direct model; invalid lists (duplicate baby, baby out of range, 0 / 257 terms) must
// be refused; the k-block orders at N = 2^8 .. 2^17 must be permutations, following pi along each
// orbit for the BSGS babies g, g^2, ... and the identity order otherwise.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../aes-fhe_amd/csrc/bsgs_plan.h"

using namespace aesfhe;

static int check_plans(std::mt19937_64& rng) {
    static const char dummy[4096] = {0};
    for (int it = 0; it < 3000; it++) {
        const int nb = 1 + (int)(rng() % 40), ng = 1 + (int)(rng() % 20), gmax = 1 + (int)(rng() % 9);
        std::vector<int32_t> nterm(ng), tbaby;
        std::vector<const void*> pts;
        for (int j = 0; j < ng; j++) {
            std::vector<int> bs(nb);
            for (int b = 0; b < nb; b++) bs[b] = b;
            std::shuffle(bs.begin(), bs.end(), rng);
            nterm[j] = 1 + (int)(rng() % nb);
            for (int t = 0; t < nterm[j]; t++) {
                tbaby.push_back(bs[t]);
                pts.push_back(dummy + (rng() % sizeof dummy));
            }
        }
        std::vector<BsgsChunk> plan;
        const std::string err = bsgs_plan_terms(nb, ng, nterm.data(), tbaby.data(), pts.data(), gmax, plan);
        if (!err.empty()) return 1;
        if ((int)plan.size() != (ng + gmax - 1) / gmax) return 2;
        int t0 = 0, j = 0;
        for (const BsgsChunk& c : plan) {
            if (c.j0 != j || c.gn < 1 || c.gn > gmax || c.pt.size() != (size_t)c.gn * nb) return 3;
            int terms = 0;
            for (int jj = 0; jj < c.gn; jj++, j++) {
                for (int t = t0; t < t0 + nterm[j]; t++) {
                    if (c.pt[(size_t)jj * nb + tbaby[t]] != pts[t]) return 4;
                    terms++;
                }
                t0 += nterm[j];
            }
            int live = 0;
            for (const void* p : c.pt) live += p != nullptr;
            if (live != terms || c.terms != terms) return 5;
        }
        if (j != ng) return 6;
        // invalid variants of the same list
        if (nterm[0] >= 2) {
            std::vector<int32_t> tb = tbaby;
            tb[1] = tb[0];  // giant 0's first two terms on one baby
            if (bsgs_plan_terms(nb, ng, nterm.data(), tb.data(), pts.data(), gmax, plan).find("same baby") == std::string::npos)
                return 7;
        }
        {
            std::vector<int32_t> tb = tbaby;
            tb[rng() % tb.size()] = (rng() & 1) ? nb : -1;
            if (bsgs_plan_terms(nb, ng, nterm.data(), tb.data(), pts.data(), gmax, plan) != "bad baby index") return 8;
        }
        for (int bad : {0, 257}) {
            std::vector<int32_t> nt = nterm;
            nt[rng() % ng] = bad;
            if (bsgs_plan_terms(nb, ng, nt.data(), tbaby.data(), pts.data(), gmax, plan).find("terms") == std::string::npos)
                return 9;
        }
    }
    std::vector<BsgsChunk> plan;
    if (bsgs_plan_terms(0, 1, nullptr, nullptr, nullptr, 8, plan).empty()) return 10;
    return 0;
}

static uint64_t powmod2n(uint64_t g, uint64_t e, uint64_t M) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r = (r * g) & (M - 1);
        g = (g * g) & (M - 1);
        e >>= 1;
    }
    return r;
}

static int check_orders(std::mt19937_64& rng) {
    for (int logN = 8; logN <= 17; logN++) {
        const uint64_t M = 2ULL << logN, n = 1ULL << (logN - 1);
        const int nblk = 1 << (logN - 8);
        for (int it = 0; it < 40; it++) {
            std::vector<uint64_t> gal;
            const int nb = 1 + (int)(rng() % 16);
            const bool orbit = it % 2 == 0;
            const uint64_t g = orbit ? powmod2n(5, rng() % n, M) | 1 : 0;
            for (int i = 0; i < nb; i++) {
                if (orbit) gal.push_back(i == 0 ? 0 : powmod2n(g, i, M));
                else gal.push_back(i == 0 ? 0 : (2 * (rng() % n) + 1) & (M - 1));
            }
            std::vector<unsigned short> ord;
            if (!bsgs_block_order(logN, gal, ord)) return 20;
            if ((int)ord.size() != nblk) return 21;
            std::vector<char> seen(nblk, 0);
            for (unsigned short b : ord) {
                if (b >= nblk || seen[b]) return 22;
                seen[b] = 1;
            }
        }
    }
    return 0;
}

int main() {
    std::mt19937_64 rng(7);
    if (int rc = check_plans(rng)) {
        std::printf("plan check failed (%d)\n", rc);
        return rc;
    }
    if (int rc = check_orders(rng)) {
        std::printf("order check failed (%d)\n", rc);
        return rc;
    }
    std::printf("bsgs_plan_asan ok\n");
    return 0;
}
