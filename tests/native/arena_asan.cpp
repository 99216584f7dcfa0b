// arena_asan.cpp -- the engine's device arena (aes-fhe_amd/csrc/arena.h) over malloc / free,
// built with g++ -fsanitize=address,undefined by tests/test_asan.py.  Random get / put / split /
// trim sequences with a shadow model: live blocks never overlap and stay inside one chunk, the
// byte counters match the model, peak_live is the running maximum, both ends of every block are
// writable (ASan catches an overrun), and once everything is freed each chunk is one free block
// again (a trim returns all of them: held == 0, and LeakSanitizer sees no chunk left behind).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <random>
#include <vector>

#include "../../aes-fhe_amd/csrc/arena.h"

using namespace aesfhe;

struct Counts {
    long allocs = 0, frees = 0, syncs = 0;
    size_t fail_above = (size_t)-1;  // simulated device-memory limit per allocation
};

static int fail(const char* what, long step) {
    std::printf("arena check failed at step %ld: %s\n", step, what);
    return 1;
}

int main(int argc, char** argv) {
    Counts cnt;
    Arena a;
    a.first_fit = argc > 1 && std::strcmp(argv[1], "first_fit") == 0;  // the placement the engine takes at N = 2^16
    a.A.alloc = [](size_t n, void* c) -> void* {
        auto* k = (Counts*)c;
        if (n > k->fail_above) return nullptr;
        k->allocs++;
        return std::malloc(n);
    };
    a.A.release = [](void* p, void* c) {
        ((Counts*)c)->frees++;
        std::free(p);
    };
    a.A.sync = [](void* c) { ((Counts*)c)->syncs++; };
    a.A.ctx = &cnt;
    a.chunk_bytes = 1 << 20;

    std::mt19937_64 rng(12345);
    std::map<char*, size_t> live;  // shadow: block -> rounded size
    size_t live_bytes = 0, peak = 0;
    const long steps = 100000;
    for (long s = 0; s < steps; s++) {
        const int op = (int)(rng() % 100);
        if (op < 48 || live.empty()) {
            // sizes from a few bytes to 1.5 chunks (a larger request gets a chunk of its own)
            const size_t n = rng() % 8 == 0 ? (size_t)(rng() % (3u << 19)) + 1 : (size_t)(rng() % 40000) + 1;
            char* p = (char*)a.get(n);
            if (!p) return fail("get returned null", s);
            const size_t r = Arena::round_up(n);
            if ((uintptr_t)p % 16) return fail("misaligned block", s);
            std::memset(p, (int)(s & 0xff), std::min<size_t>(r, 64));  // both ends of the rounded block are ours
            std::memset(p + r - std::min<size_t>(r, 64), (int)(s & 0xff), std::min<size_t>(r, 64));
            auto nx = live.lower_bound(p);
            if (nx != live.end() && p + r > nx->first) return fail("overlaps the next live block", s);
            if (nx != live.begin() && std::prev(nx)->first + std::prev(nx)->second > p) return fail("overlaps the previous live block", s);
            char* ch = a.chunk_of(p);
            if (!ch || p + r > ch + a.chunks_.at(ch)) return fail("block leaves its chunk", s);
            live[p] = r;
            live_bytes += r;
            peak = std::max(peak, live_bytes);
        } else if (op < 90) {
            auto it = live.begin();
            std::advance(it, (long)(rng() % live.size()));
            live_bytes -= it->second;
            a.put(it->first);
            live.erase(it);
        } else if (op < 97) {
            // zero-copy split of a block made of `parts` aligned parts, then free some parts
            const int parts = 2 + (int)(rng() % 6);
            const size_t part = Arena::kAlign * (1 + rng() % 40);
            char* p = (char*)a.get(parts * part);
            if (!p) return fail("get for split returned null", s);
            if (!a.split(p, parts, part)) return fail("split refused a whole block", s);
            if (a.split(p, parts, part)) return fail("split accepted a block of the wrong size", s);
            for (int t = 0; t < parts; t++) {
                live[p + t * part] = part;
                live_bytes += part;
            }
            peak = std::max(peak, live_bytes);
            for (int t = 0; t < parts; t += 2) {
                a.put(p + t * part);
                live.erase(p + t * part);
                live_bytes -= part;
            }
        } else {
            a.trim();
        }
        a.put(nullptr);           // ignored
        a.put((char*)&cnt);       // unknown pointer: ignored
        if (a.live != live_bytes) return fail("live bytes differ from the model", s);
        if (a.peak_live != peak) return fail("peak_live is not the running maximum", s);
        if (a.live > a.held) return fail("live above held", s);
        if (s % 5000 == 0 && a.fragmentation() > a.held) return fail("fragmentation above held", s);
    }
    // allocator failure: a request beyond the simulated limit returns null, state unchanged
    cnt.fail_above = 1 << 22;
    const size_t held0 = a.held;
    if (a.get((size_t)1 << 23) != nullptr) return fail("oversized get did not fail", steps);
    if (a.live != live_bytes) return fail("failed get changed live bytes", steps);
    if (a.held > held0) return fail("failed get grew held", steps);
    cnt.fail_above = (size_t)-1;
    for (auto& kv : live) a.put(kv.first);
    live.clear();
    if (a.live != 0) return fail("live bytes after freeing everything", steps);
    if (a.fragmentation() != 0) return fail("fragmentation with nothing live", steps);
    for (auto& kv : a.chunks_) {
        auto f = a.free_addr_.find(kv.first);
        if (f == a.free_addr_.end() || f->second != kv.second) return fail("a chunk did not merge back to one free block", steps);
    }
    a.trim();
    if (a.held != 0 || !a.chunks_.empty() || !a.free_addr_.empty() || !a.free_size_.empty())
        return fail("trim left chunks behind", steps);
    if (cnt.allocs != cnt.frees) return fail("allocator calls unbalanced", steps);
    // growth cap: an arena holding more than grow_cap x its peak live set grows by the request alone
    {
        Arena b;
        b.A = a.A;
        b.chunk_bytes = 1 << 20;
        void* x = b.get(600000);  // peak 600 000 in one 1 MiB chunk
        b.put(x);
        void* lo = b.get(400000);
        void* mid = b.get(100000);
        b.put(lo);                // free: 400 128 at the start, 548 352 at the end; held 1.75 x peak
        const size_t held0 = b.held;
        void* big = b.get(560000);  // fits no free block (548 352 and 400 128 free)
        if (!big || b.exact_chunks != 1 || b.held != held0 + Arena::round_up(560000))
            return fail("cap: fragmented growth took a whole chunk", steps);
        b.grow_cap = 0;             // disabled: a whole chunk again
        void* big2 = b.get(560000);
        if (!big2 || b.held != held0 + Arena::round_up(560000) + ((size_t)1 << 20))
            return fail("cap disabled: chunk size", steps);
        b.put(big);
        b.put(big2);
        b.put(mid);
        b.trim();
        if (b.held != 0) return fail("cap: trim", steps);
    }
    if (cnt.allocs != cnt.frees) return fail("allocator calls unbalanced (cap)", steps);
    std::printf("arena_asan ok (%s): %ld steps, %ld chunk allocations, peak live %zu bytes\n", a.first_fit ? "first fit" : "best fit",
                steps, cnt.allocs, peak);
    return 0;
}
