// Replays an AESFHE_ARENA_TRACE event file (engine.hip Pool) through arena.h under other
// policies, on the CPU (fake addresses, no memory): held / peak live / hipMalloc count per
// policy, at the end of the trace and at its largest.  Dev tool for VERDICT r4 item 7.
//   g++ -O2 -std=c++17 -o tools/arena_replay tools/arena_replay.cpp
//   tools/arena_replay TRACE [TRACE ...]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../aes-fhe_amd/csrc/arena.h"

using namespace aesfhe;

struct Ev {
    char op, tag;
    unsigned long long p;
    size_t n;
    int parts;
};

static std::vector<Ev> load(const char* path) {
    std::vector<Ev> ev;
    FILE* f = fopen(path, "r");
    if (!f) {
        perror(path);
        exit(1);
    }
    char line[256];
    while (fgets(line, sizeof line, f)) {
        Ev e{};
        char op, tag;
        void* p;
        if (sscanf(line, "%c %c %p", &op, &tag, &p) < 3) continue;
        e.op = op, e.tag = tag, e.p = (unsigned long long)p;
        if (op == 'g') sscanf(line, "%*c %*c %*p %zu", &e.n);
        if (op == 's') sscanf(line, "%*c %*c %*p %d %zu", &e.parts, &e.n);
        ev.push_back(e);
    }
    fclose(f);
    return ev;
}

struct Policy {
    const char* name;
    size_t chunk;
    double cap;
    size_t exact_round;  // exact chunks rounded up to this (0: the request)
    bool two;            // two arenas (ciphertexts / temporaries) or one
    int fit = 0;         // 0 best fit (arena.h), 1 address-ordered first fit, 2 best fit from the top of a chunk
    size_t big = 0;      // blocks >= big: exact-size cache (reused only by the same size), 0 off
    bool clamp = false;  // new chunks clamped to cap x peak_live - held (never below the request)
    int buckets = 0;     // > 0: one arena per size class (0.25 / 1 / 4 GB boundaries, up to 4 classes)
    size_t thr = 0;      // fit 6 / 7: blocks >= thr placed from the top of a free block
};

// arena.h with another placement rule (replay only)
struct ArenaX : Arena {
    int fit = 0;
    bool clamp = false;
    size_t thr = 0;
    void* getx(size_t bytes) {
        const size_t n = round_up(bytes);
        if (clamp && free_size_.lower_bound(n) == free_size_.end() && peak_live > 0) {
            const double room = grow_cap * (double)std::max(peak_live, live + n) - (double)held;
            const size_t want = std::max(n, (size_t)std::max(0.0, std::min((double)chunk_bytes, room)));
            const size_t cb = chunk_bytes;
            const double cap = grow_cap;
            chunk_bytes = (want + kAlign - 1) & ~(kAlign - 1);
            grow_cap = 0;
            new_chunk(n);
            chunk_bytes = cb;
            grow_cap = cap;
        }
        if (fit == 6 || fit == 7) {  // two-ended first fit (creation order): blocks >= thr from the top
            first_fit = true;
            const bool big = n >= thr;
            std::map<std::pair<uint64_t, char*>, size_t>::iterator f = free_ff_.end();
            auto find = [&] {
                f = free_ff_.end();
                if (big && fit == 7) {  // big ones: the newest chunk first
                    for (auto r = free_ff_.rbegin(); r != free_ff_.rend(); ++r)
                        if (r->second >= n) {
                            f = std::prev(r.base());
                            break;
                        }
                } else {
                    for (auto g = free_ff_.begin(); g != free_ff_.end(); ++g)
                        if (g->second >= n) {
                            f = g;
                            break;
                        }
                }
            };
            find();
            if (f == free_ff_.end()) {
                if (!new_chunk(n)) return nullptr;
                find();
            }
            char* b = f->first.second;
            const size_t have = f->second;
            del_free(b, have);
            char* p = b;
            if (big) {
                p = b + (have - n);
                if (have > n) add_free(b, have - n);
            } else if (have > n) {
                add_free(b + n, have - n);
            }
            live_[p] = n;
            live += n;
            peak_live = std::max(peak_live, live);
            return p;
        }
        if (fit == 0) return get(bytes);
        if (fit == 5) {  // arena.h's own first-fit mode
            first_fit = true;
            return get(bytes);
        }
        if (fit == 4) {  // best fit, but a chunk made for one big request (> chunk_bytes) only serves requests >= half its size
            for (auto f = free_size_.lower_bound(n); f != free_size_.end(); ++f) {
                char* ch = chunk_of(f->second);
                const size_t cs = chunks_[ch];
                if (cs > chunk_bytes && 2 * n < cs) continue;
                char* p = f->second;
                const size_t have = f->first;
                free_size_.erase(f);
                free_addr_.erase(p);
                if (have > n) add_free(p + n, have - n);
                live_[p] = n;
                live += n;
                peak_live = std::max(peak_live, live);
                return p;
            }
            // none: a new chunk (whole chunk_bytes, or the request alone when larger / capped)
            if (!new_chunk(n)) return nullptr;
            return getx(bytes);
        }
        std::map<char*, size_t>::iterator it = free_addr_.end();
        if (fit == 1) {
            for (auto f = free_addr_.begin(); f != free_addr_.end(); ++f)
                if (f->second >= n) {
                    it = f;
                    break;
                }
        }
        if (it == free_addr_.end()) {
            if (fit == 2) return get(bytes);
            if (!new_chunk(n)) return nullptr;
            for (auto f = free_addr_.begin(); f != free_addr_.end(); ++f)
                if (f->second >= n) {
                    it = f;
                    break;
                }
        }
        char* p = it->first;
        const size_t have = it->second;
        del_free(p, have);
        if (have > n) add_free(p + n, have - n);
        live_[p] = n;
        live += n;
        peak_live = std::max(peak_live, live);
        return p;
    }
};

struct Fake {
    unsigned long long next = 1ULL << 46;
};

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: arena_replay TRACE [TRACE ...]\n");
        return 2;
    }
    const size_t G = 1ULL << 30;
    const Policy pols[] = {
        {"now: 8G chunks, cap 1.2, two arenas", 8 * G, 1.2, 0, true},
        {"engine N=2^16: first fit (arena.h), 4G, cap 1.2", 4 * G, 1.2, 0, false, 5},
        {"two-ended ff, big >= 256M, 4G cap 1.2", 4 * G, 1.2, 0, false, 6, 0, false, 0, G / 4},
        {"two-ended ff, big >= 1G, 4G cap 1.2", 4 * G, 1.2, 0, false, 6, 0, false, 0, G},
        {"two-ended ff, big >= 64M, 4G cap 1.2", 4 * G, 1.2, 0, false, 6, 0, false, 0, G / 16},
        {"two-ended ff, big >= 256M, 8G cap 1.2", 8 * G, 1.2, 0, false, 6, 0, false, 0, G / 4},
        {"two-ended ff, big >= 256M, 4G cap 1.1", 4 * G, 1.1, 0, false, 6, 0, false, 0, G / 4},
        {"two-ended, big newest-first >= 256M, 4G", 4 * G, 1.2, 0, false, 7, 0, false, 0, G / 4},
        {"two-ended, big newest-first >= 1G, 4G", 4 * G, 1.2, 0, false, 7, 0, false, 0, G},
        {"two-ended ff, big >= 4G, 16G cap 1.1", 16 * G, 1.1, 0, false, 6, 0, false, 0, 4 * G},
        {"two-ended ff, big >= 8G, 16G cap 1.1", 16 * G, 1.1, 0, false, 6, 0, false, 0, 8 * G},
        {"two-ended ff, big >= 2G, 32G cap 1.1", 32 * G, 1.1, 0, false, 6, 0, false, 0, 2 * G},
        {"two-ended ff, big >= 8G, 32G cap 1.1", 32 * G, 1.1, 0, false, 6, 0, false, 0, 8 * G},
        {"ff(seq) 32G cap 1.1", 32 * G, 1.1, 0, false, 5},
        {"ff(seq) 64G cap 1.1", 64 * G, 1.1, 0, false, 5},
        {"ff(seq) 32G cap 1.05", 32 * G, 1.05, 0, false, 5},
        {"ff(seq) 2G cap 1.2", 2 * G, 1.2, 0, false, 5},
        {"ff(seq) 3G cap 1.2", 3 * G, 1.2, 0, false, 5},
        {"ff(seq) 6G cap 1.2", 6 * G, 1.2, 0, false, 5},
        {"ff(seq) 4G cap 1.1", 4 * G, 1.1, 0, false, 5},
        {"ff(seq) 4G cap 1.3", 4 * G, 1.3, 0, false, 5},
        {"ff(seq) 4G no cap", 4 * G, 0.0, 0, false, 5},
        {"ff(seq) 8G cap 1.2", 8 * G, 1.2, 0, false, 5},
        {"ff(seq) 16G cap 1.1", 16 * G, 1.1, 0, false, 5},
        {"cap 1.1", 8 * G, 1.1, 0, true},
        {"cap 1.05", 8 * G, 1.05, 0, true},
        {"cap 1.0", 8 * G, 1.0, 0, true},
        {"4G chunks, cap 1.2", 4 * G, 1.2, 0, true},
        {"2G chunks, cap 1.2", 2 * G, 1.2, 0, true},
        {"2G chunks, cap 1.05", 2 * G, 1.05, 0, true},
        {"1G chunks, cap 1.05", G, 1.05, 0, true},
        {"8G chunks, cap 1.05, exact to 1G", 8 * G, 1.05, G, true},
        {"one arena, 8G, cap 1.2", 8 * G, 1.2, 0, false},
        {"two, first fit", 8 * G, 1.2, 0, true, 1},
        {"two, clamp 1.15", 8 * G, 1.15, 0, true, 0, 0, true},
        {"two, clamp 1.1", 8 * G, 1.1, 0, true, 0, 0, true},
        {"one, clamp 1.15", 8 * G, 1.15, 0, false, 0, 0, true},
        {"one, clamp 1.1", 8 * G, 1.1, 0, false, 0, 0, true},
        {"one, clamp 1.05", 8 * G, 1.05, 0, false, 0, 0, true},
        {"one, clamp 1.02", 8 * G, 1.02, 0, false, 0, 0, true},
        {"one, clamp 1.1, 16G", 16 * G, 1.1, 0, false, 0, 0, true},
        {"one, clamp 1.1, first fit", 8 * G, 1.1, 0, false, 1, 0, true},
        {"one, clamp 1.05, first fit", 8 * G, 1.05, 0, false, 1, 0, true},
        {"one, first fit", 8 * G, 1.2, 0, false, 1},
        {"one, first fit, 4G", 4 * G, 1.2, 0, false, 1},
        {"one, first fit, 16G", 16 * G, 1.2, 0, false, 1},
        {"one, first fit, cap 1.1", 8 * G, 1.1, 0, false, 1},
        {"one, first fit, 16G, cap 1.1", 16 * G, 1.1, 0, false, 1},
        {"two, big >= 2G exact cache", 8 * G, 1.2, 0, true, 0, 2 * G},
        {"one, big >= 2G exact cache", 8 * G, 1.2, 0, false, 0, 2 * G},
        {"one, first fit, big >= 2G cache", 8 * G, 1.2, 0, false, 1, 2 * G},
        {"one, first fit, big >= 4G cache", 8 * G, 1.2, 0, false, 1, 4 * G},
        {"one, big chunks reserved, cap 1.1", 8 * G, 1.1, 0, false, 4},
        {"one, big chunks reserved, cap 1.2", 8 * G, 1.2, 0, false, 4},
        {"one, big chunks reserved, 4G, cap 1.1", 4 * G, 1.1, 0, false, 4},
        {"size classes, 8G, clamp 1.1", 8 * G, 1.1, 0, false, 0, 0, true, 4},
        {"size classes, 8G, cap 1.2", 8 * G, 1.2, 0, false, 0, 0, false, 4},
        {"size classes, 4G, clamp 1.1", 4 * G, 1.1, 0, false, 0, 0, true, 4},
        {"size classes, first fit, 8G", 8 * G, 1.1, 0, false, 1, 0, true, 4},
    };
    for (int a = 1; a < argc; a++) {
        const auto ev = load(argv[a]);
        printf("%s: %zu events\n", argv[a], ev.size());
        for (const auto& pol : pols) {
            Fake fk;
            // REPLAY_ADDR=down: each new chunk below the previous ones (device addresses need not rise)
            static const bool down = getenv("REPLAY_ADDR") && !strcmp(getenv("REPLAY_ADDR"), "down");
            ArenaAllocator al{[](size_t n, void* ctx) -> void* {
                                  auto* f = (Fake*)ctx;
                                  const size_t r = (n + 4095) & ~(size_t)4095;
                                  if (down) {
                                      f->next -= r;
                                      return (void*)f->next;
                                  }
                                  void* p = (void*)f->next;
                                  f->next += r;
                                  return p;
                              },
                              [](void*, void*) {}, [](void*) {}, &fk};
            ArenaX ar[4];
            for (auto& x : ar) x.A = al, x.chunk_bytes = pol.chunk, x.grow_cap = pol.cap, x.fit = pol.fit, x.clamp = pol.clamp, x.thr = pol.thr;
            // exact-size cache for big blocks: free blocks by size; held = every block ever made
            std::multimap<size_t, char*> bigfree;
            std::unordered_map<char*, size_t> biglive;
            size_t bigheld = 0, biglivesz = 0;
            std::unordered_map<unsigned long long, std::pair<int, char*>> map;
            size_t peak_total = 0, max_held = 0;
            // host time of the allocator's get / put (first fit scans the free list)
            double get_ns = 0, put_ns = 0, get_max_ns = 0;
            long ngets = 0, nputs = 0;
            using clk = std::chrono::steady_clock;
            for (const auto& e : ev) {
                int k = pol.two && e.tag == 't' ? 1 : 0;
                if (pol.buckets && e.op == 'g')
                    k = e.n < (G >> 2) ? 0 : e.n < G ? 1 : e.n < 4 * G ? 2 : 3;
                if (e.op == 'g') {
                    if (pol.exact_round) {  // emulate rounding of exact chunks: pre-grow by the rounded need
                        Arena& A = ar[k];
                        const size_t n = Arena::round_up(e.n);
                        if (A.free_size_.lower_bound(n) == A.free_size_.end() && A.peak_live > 0 &&
                            (double)A.held > A.grow_cap * (double)A.peak_live) {
                            const size_t r = (n + pol.exact_round - 1) / pol.exact_round * pol.exact_round;
                            const double cap = A.grow_cap;
                            A.grow_cap = 0;
                            const size_t cb = A.chunk_bytes;
                            A.chunk_bytes = r;
                            A.new_chunk(n);
                            A.chunk_bytes = cb;
                            A.grow_cap = cap;
                        }
                    }
                    if (pol.big && e.n >= pol.big) {
                        auto f = bigfree.find(e.n);
                        char* p;
                        if (f != bigfree.end()) {
                            p = f->second;
                            bigfree.erase(f);
                        } else {
                            p = (char*)fk.next;
                            fk.next += (e.n + 4095) & ~(size_t)4095;
                            bigheld += e.n;
                        }
                        biglive[p] = e.n;
                        biglivesz += e.n;
                        map[e.p] = {9, p};
                    } else {
                        const auto t0 = clk::now();
                        char* p = (char*)ar[k].getx(e.n);
                        const double dt = std::chrono::duration<double, std::nano>(clk::now() - t0).count();
                        get_ns += dt, get_max_ns = std::max(get_max_ns, dt), ngets++;
                        map[e.p] = {k, p};
                    }
                } else if (e.op == 'p') {
                    auto it = map.find(e.p);
                    if (it == map.end()) continue;
                    if (it->second.first == 9) {
                        const size_t n = biglive[it->second.second];
                        biglive.erase(it->second.second);
                        biglivesz -= n;
                        bigfree.insert({n, it->second.second});
                    } else {
                        const auto t0 = clk::now();
                        ar[it->second.first].put(it->second.second);
                        put_ns += std::chrono::duration<double, std::nano>(clk::now() - t0).count(), nputs++;
                    }
                    map.erase(it);
                } else if (e.op == 's') {
                    auto it = map.find(e.p);
                    if (it == map.end()) continue;
                    const int kk = it->second.first;
                    char* base = it->second.second;
                    if (kk == 9) continue;  // (big blocks are never split in the traces)
                    ar[kk].split(base, e.parts, e.n);
                    for (int t = 0; t < e.parts; t++) map[e.p + (unsigned long long)t * e.n] = {kk, base + (size_t)t * e.n};
                }
                peak_total = std::max(peak_total, ar[0].live + ar[1].live + ar[2].live + ar[3].live + biglivesz);
                max_held = std::max(max_held, ar[0].held + ar[1].held + ar[2].held + ar[3].held + bigheld);
            }
            const size_t held = ar[0].held + ar[1].held + ar[2].held + ar[3].held + bigheld;
            printf("  %-36s held %6.1f GB (max %6.1f)  peak live %6.1f GB  held/peak %.3f  mallocs %lld"
                   "  get %.2f us avg (max %.1f) / put %.2f us over %ld / %ld\n", pol.name, held / 1e9,
                   max_held / 1e9, peak_total / 1e9, (double)held / (double)std::max<size_t>(1, peak_total),
                   (long long)(ar[0].mallocs + ar[1].mallocs + ar[2].mallocs + ar[3].mallocs),
                   get_ns / 1e3 / std::max(1L, ngets), get_max_ns / 1e3, put_ns / 1e3 / std::max(1L, nputs), ngets, nputs);
        }
    }
    return 0;
}
