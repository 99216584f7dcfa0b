// bsgs_plan.h -- host-side planning of aesfhe_linear_bsgs (engine.hip), kept
// free of HIP so that tests/native/bsgs_plan_asan.cpp runs it under AddressSanitizer + UBSan
// (the host code around the BSGS term-sum launches is where round 5's
// unexplained host faults sat).  Everything a launch reads from these tables is sized here:
//   * the term lists: nterm[j] terms of giant j, tbaby[t] its baby, validated (1..256 terms per
//     giant, baby indices in range, one term per (giant, baby));
//   * the giants in chunks of at most gmax (the term-sum kernels' accumulator count), each with
//     its gn x nb table of plaintext pointers (nullptr = no term) and its term count;
//   * the k-block order k_bsgs_terms walks a limb in (bsgs_block_order, below).
#pragma once
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace aesfhe {

struct BsgsChunk {
    int j0 = 0, gn = 0;              // giants j0 .. j0 + gn - 1
    std::vector<const void*> pt;     // [gn][nb] plaintext of (giant, baby), nullptr when absent
    int terms = 0;
};

// "" when the plan is valid, else the error (the engine raises AESFHE_EARG with it)
inline std::string bsgs_plan_terms(int nb, int ng, const int32_t* nterm, const int32_t* tbaby,
                                   const void* const* pts, int gmax, std::vector<BsgsChunk>& out) {
    char msg[160];
    out.clear();
    if (nb < 1 || ng < 1) return "linear_bsgs needs baby and giant steps";
    if (gmax < 1) return "bad giant chunk size";
    std::vector<int> first(ng + 1, 0);
    for (int j = 0; j < ng; j++) {
        if (nterm[j] < 1 || nterm[j] > 256) {
            std::snprintf(msg, sizeof msg, "giant step with %d terms", nterm[j]);
            return msg;
        }
        first[j + 1] = first[j] + nterm[j];
    }
    for (int t = 0; t < first[ng]; t++)
        if (tbaby[t] < 0 || tbaby[t] >= nb) return "bad baby index";
    for (int j0 = 0; j0 < ng; j0 += gmax) {
        BsgsChunk c;
        c.j0 = j0;
        c.gn = ng - j0 < gmax ? ng - j0 : gmax;
        c.pt.assign((size_t)c.gn * nb, nullptr);
        for (int j = 0; j < c.gn; j++)
            for (int t = first[j0 + j]; t < first[j0 + j + 1]; t++) {
                const void*& slot = c.pt[(size_t)j * nb + tbaby[t]];
                if (slot) return "two terms of one giant on the same baby";
                slot = pts[t];
                c.terms++;
            }
        out.push_back(std::move(c));
    }
    return "";
}

// The order k_bsgs_terms walks the 256-slot k-blocks of a limb in: along the orbits of pi, the
// block map of the first keyed baby's Galois element g (slot k = 256 kb + j reads slot
// sigma_g(k) = brv(((g (2 brv(k) + 1)) mod 2N - 1) / 2), whose block depends on kb alone), when
// every keyed baby i is g^(i - i1 + 1) (the BSGS babies: rotations by i x stride); otherwise
// 0, 1, 2, ...  Either order is a permutation of the blocks, so results do not depend on it.
// false if the walk does not cover every block once (never for a Galois element: pi is a
// bijection; the engine raises).
inline bool bsgs_block_order(int logN, const std::vector<uint64_t>& gal, std::vector<unsigned short>& ord) {
    const int nblk = logN >= 8 ? 1 << (logN - 8) : 1;
    const uint64_t M = 2ULL << logN;
    ord.assign(nblk, 0);
    for (int i = 0; i < nblk; i++) ord[i] = (unsigned short)i;
    uint64_t g1 = 0;
    int i1 = -1;
    for (int i = 0; i < (int)gal.size(); i++)
        if (gal[i] > 1) {
            g1 = gal[i], i1 = i;
            break;
        }
    if (!g1 || logN < 8) return true;
    uint64_t gp = 1;  // keyed babies must be g1^(i - i1 + 1), identity babies anywhere
    for (int i = i1; i < (int)gal.size(); i++) {
        gp = (gp * g1) & (M - 1);
        if (gal[i] != 0 && gal[i] != gp) return true;
    }
    auto brv = [&](uint64_t x) {
        uint32_t v = (uint32_t)x, r = 0;
        for (int b = 0; b < logN; b++) r |= ((v >> b) & 1u) << (logN - 1 - b);
        return (uint64_t)r;
    };
    auto pi = [&](int kb) {
        const uint64_t k = (uint64_t)kb << 8, ek = 2 * brv(k) + 1;
        return (int)(brv((((g1 * ek) & (M - 1)) - 1) >> 1) >> 8);
    };
    std::vector<char> seen(nblk, 0);
    int n = 0;
    for (int s = 0; s < nblk; s++)
        for (int kb = s; !seen[kb]; kb = pi(kb)) {
            if (n >= nblk) return false;
            seen[kb] = 1;
            ord[n++] = (unsigned short)kb;
        }
    return n == nblk;
}

}  // namespace aesfhe
