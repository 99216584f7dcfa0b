// engine.hip -- MI355X (gfx950) RNS-CKKS engine implementing include/aesfhe.h.
//
// Replaces the closed desilofhe.Engine the reference calls (engine_context.py:6,32-85;
// xor_service.py:36-129).  One HIP stream per engine; every operation is enqueued
// asynchronously and host reads (decrypt / export) synchronise.  Device memory comes from a
// chunked best-fit arena (arena.h), so steady-state operations never call hipMalloc.
// Specification of every integer step: DESIGN.md section 3 (restated by oracle/ckks_oracle.c).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <unordered_map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/aesfhe.h"
#include "kernels_ops.h"
#include "ntt256f.h"
#include "ks_fused.h"
#include "bconv_mfma.h"
#include "bconv_cols.h"
#include "bsgs_plan.h"
#include "arena.h"
#include "codec_dev.h"

using namespace aesfhe;

// -----------------------------------------------------------------------------------------------
// errors
static thread_local char g_err[512];

static int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

struct ApiError {
    int code;
    std::string msg;
};

[[noreturn]] static void throw_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw ApiError{code, buf};
}

#define HIPC(x)                                                                              \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) throw_err(AESFHE_EDEVICE, "%s: %s (engine.hip:%d)", #x, hipGetErrorString(e_), __LINE__); \
    } while (0)

#define API_BEGIN try {
#define API_END                                                   \
    }                                                             \
    catch (const ApiError& e) {                                   \
        return set_err(e.code, "%s", e.msg.c_str());              \
    }                                                             \
    catch (const std::bad_alloc&) {                               \
        return set_err(AESFHE_ENOMEM, "host allocation failed");  \
    }                                                             \
    catch (const std::exception& e) {                             \
        return set_err(AESFHE_EARG, "%s", e.what());              \
    }                                                             \
    return AESFHE_OK;

extern "C" const char* aesfhe_last_error(void) { return g_err; }
extern "C" const char* aesfhe_backend_name(void) { return "hip-gfx950"; }
extern "C" int32_t aesfhe_abi_version(void) { return AESFHE_ABI_VERSION; }

// -----------------------------------------------------------------------------------------------
// engine state
// Device memory: the chunked best-fit arena of arena.h over hipMalloc / hipFree (its host logic
// is unit-tested on the CPU under AddressSanitizer, tests/native/arena_asan.cpp).
// AESFHE_ARENA_TRACE=path (diagnostic): every engine writes its two arenas' block events to
// path.<engine number> ("g tag ptr bytes", "p tag ptr", "s tag ptr parts part"), which
// tools/arena_replay.cpp replays under other arena policies on the CPU.
struct Pool : Arena {
    FILE* trace = nullptr;
    char tag = 'c';
    Pool() {
        A.alloc = [](size_t n, void*) -> void* {
            void* p = nullptr;
            if (hipMalloc(&p, n) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
            }
            return p;
        };
        A.release = [](void* p, void*) { hipFree(p); };
        A.sync = [](void*) { hipDeviceSynchronize(); };
        A.ctx = nullptr;
    }
    void* get(size_t bytes) {
        void* p = Arena::get(bytes);
        if (!p) throw_err(AESFHE_ENOMEM, "device allocation of %zu bytes failed (%zu held, %zu live)", round_up(bytes), held, live);
        if (trace) fprintf(trace, "g %c %p %zu\n", tag, p, round_up(bytes));
        return p;
    }
    void put(void* p, size_t) {
        if (trace && p) fprintf(trace, "p %c %p\n", tag, p);
        Arena::put(p);
    }
    void split(void* p, int parts, size_t part) {
        if (!Arena::split(p, parts, part))
            throw_err(AESFHE_EARG, "pool split of a block that is not %d x %zu bytes", parts, part);
        if (trace) fprintf(trace, "s %c %p %d %zu\n", tag, p, parts, part);
    }
};

struct ProfRec {
    int fam;
    hipEvent_t a, b;
    double bytes;
    const char* label;  // kernel class (static string) or nullptr
    int disp;           // kernel dispatches recorded inside the scope
};

struct KernStat {  // per kernel class (aesfhe_engine_profile_kernels)
    int64_t n = 0, d = 0;  // scopes (calls) and kernel dispatches
    double ms = 0, bytes = 0;
};

struct aesfhe_engine {
    // one reference for the engine handle plus one per live ct / pt / key: the tables, pool and
    // stream outlive aesfhe_engine_destroy until the last object is freed (Python's cycle
    // collector finalises an engine and its ciphertexts in arbitrary order)
    std::atomic<int> refs{1};
    int logN, N, L, K, A, dnum, np, Lp1;  // A: key-switch digit width (alpha)
    int device;
    u64 seed;
    ChaKey ck;  // ChaCha20 key of every random stream
    Chain chain;
    hipStream_t stream;
    // one arena for every block (`tpool` is unused): a second arena for the per-call temporaries
    // (tried in round 5 against the holes short-lived blocks leave between long-lived ones) held
    // more in the replay of the bench's block events (tools/arena_replay.cpp: bench round 1.28 vs
    // 1.26 x its peak live set, config 5 249 vs 236 GB)
    Pool pool, tpool;
    size_t peak_total = 0;  // largest pool.live + tpool.live seen
    // device tables
    u64 *q, *psi, *ipsi, *ninv;
    double *qinv, *psif, *ipsif, *ninvf;
    double *rtwf = nullptr, *irtwf = nullptr;  // N = 2^16 row-pass twiddle factors [np][256][8] (ntt256f.h)
    Tw *tw, *itw;
    double *cw = nullptr, *icw = nullptr;  // [np][kColW] uniform column-stage twiddles w (kernels.h)
    u64* iroot;  // host copy only needed
    std::vector<u64> h_iroot;
    // base conversion tables
    u64 *mu_hatinv, *mu_hat, *md_phatinv, *md_phat, *md_pinv, *rs_inv, *rs_mod, *pmod;
    // combined ModDown + rescale (drop r = 1, 2 top Q primes with P), see build_tables
    double *mdr_invf = nullptr, *mdr_dinvf = nullptr, *pmodf = nullptr;
    TwD* mdr_hatf = nullptr;  // {w, w/q}
    double *mdr_einv = nullptr, *mdr_dmodf = nullptr, *md_einv = nullptr;
    u64* mdr_dinv = nullptr;
    double *mu_hatinvf, *md_phatinvf, *md_pinvf, *rs_invf;
    double* mu_nhatf = nullptr;  // [level l][limb i] N^{-1} hatinv_{l,i} / q_i: the INTT before a fused ModUp
    // the same for a fused ModDown's sources: N^{-1} (D/e_j)^{-1} / e_j, plain ([kMdrMaxE]) and
    // combined with r rescales ([cell][kMdrMaxE], as mdr_invf)
    double *md_ninvf = nullptr, *mdr_ninvf = nullptr;
    TwD *mu_hatf, *md_phatf;  // base-conversion constants {w, w/q}
    // matrix-core base conversions (bconv_mfma.h): [set / cell][pid][8 planes][kBconvKT] signed
    // bytes, the XOR-0x80 corrections [set / cell][pid] and (2^32 mod p) / p per prime
    int8_t *bc_mu_tab = nullptr, *bc_md_tab = nullptr, *bc_mdr_tab = nullptr;
    double *bc_mu_corr = nullptr, *bc_md_corr = nullptr, *bc_mdr_corr = nullptr, *bc_pc = nullptr;
    // small-argument upload ring (device) + pinned staging
    char* ring_d = nullptr;
    char* ring_h = nullptr;
    size_t ring_size = 8u << 20, ring_off = 0;
    // device codec (codec_dev.h): twiddles / rotation table built on first use, overflow flags
    double *ckre = nullptr, *ckim = nullptr;
    long* crot = nullptr;
    int* cflags = nullptr;
    size_t cflags_n = 0;
    // aesfhe_poly2 constant tables, keyed by (level, shape, coefficients)
    std::map<std::string, TwD*> poly2_tabs;
    // profiling
    int prof = 0;  // bitmask of recorded families (1 << FAM_*)
    std::vector<ProfRec> recs;
    std::vector<hipEvent_t> spare;
    double prof_ms[4] = {0, 0, 0, 0};
    double prof_bytes[4] = {0, 0, 0, 0};
    int64_t prof_n[4] = {0, 0, 0, 0};
    std::map<std::string, KernStat> prof_k;

    Tabs tabs() const {
        Tabs t;
        t.q = q;
        t.qinv = qinv;
        t.psi = psi;
        t.psif = psif;
        t.ipsi = ipsi;
        t.ipsif = ipsif;
        t.rtwf = rtwf;
        t.irtwf = irtwf;
        t.ninv = ninv;
        t.ninvf = ninvf;
        t.tw = tw;
        t.itw = itw;
        t.cw = cw;
        t.icw = icw;
        t.logN = logN;
        t.Lp1 = Lp1;
        return t;
    }
};

struct aesfhe_key {
    aesfhe_engine* eng;
    int kind;
    u64 galois;
    u64 keyseed;
    u64* d;
    size_t bytes;
    int ndig = 0;  // switching keys: digits stored (dnum, or fewer after aesfhe_key_trim)
};

struct aesfhe_ct {
    aesfhe_engine* eng;
    int B, np, level, is_zero;
    u64* d;
    size_t bytes;
};

struct aesfhe_pt {
    aesfhe_engine* eng;
    int level;
    int ext = 0;  // 1: limbs 0..level then the K special limbs (aesfhe_pt_create_ext)
    u64* d;
    size_t bytes;
};

// -----------------------------------------------------------------------------------------------
// helpers
static const int FAM_NTT = 0, FAM_KS = 1, FAM_EW = 2;
static const int kMdrMaxR = 2, kMdrMaxE = 16;  // combined ModDown + rescale: r <= 2, K + r <= 16

struct ProfScope {
    aesfhe_engine* e;
    int fam;
    double bytes;
    hipEvent_t a = nullptr, b = nullptr;
    hipStream_t s;
    bool on;
    const char* label;
    int disp = 1;  // kernel dispatches inside the scope (the PMC record counts dispatches)
    ProfScope(aesfhe_engine* e_, int f, double by, const char* lab = nullptr, hipStream_t s_ = nullptr)
        : e(e_), fam(f), bytes(by), s(s_ ? s_ : e_->stream), on((e_->prof >> f) & 1), label(lab) {
        if (!on) return;
        a = take();
        b = take();
        hipEventRecord(a, s);
    }
    hipEvent_t take() {
        if (!e->spare.empty()) {
            hipEvent_t x = e->spare.back();
            e->spare.pop_back();
            return x;
        }
        hipEvent_t x;
        hipEventCreate(&x);
        return x;
    }
    ~ProfScope() {
        if (!on) return;
        hipEventRecord(b, s);
        e->recs.push_back({fam, a, b, bytes, label, disp});
    }
};

static void prof_flush(aesfhe_engine* e) {
    if (e->recs.empty()) return;
    hipStreamSynchronize(e->stream);
    for (auto& r : e->recs) {
        float ms = 0;
        hipEventElapsedTime(&ms, r.a, r.b);
        e->prof_ms[r.fam] += ms;
        e->prof_bytes[r.fam] += r.bytes;
        e->prof_n[r.fam] += 1;
        if (r.label) {
            KernStat& k = e->prof_k[r.label];
            k.n++;
            k.d += r.disp;
            k.ms += ms;
            k.bytes += r.bytes;
        }
        e->spare.push_back(r.a);
        e->spare.push_back(r.b);
    }
    e->recs.clear();
}

template <typename T>
static T* upload_small(aesfhe_engine* e, const T* src, size_t count) {
    size_t bytes = (count * sizeof(T) + 255) & ~(size_t)255;
    if (bytes > e->ring_size) throw_err(AESFHE_EARG, "argument upload too large");
    if (e->ring_off + bytes > e->ring_size) {
        HIPC(hipStreamSynchronize(e->stream));
        e->ring_off = 0;
    }
    memcpy(e->ring_h + e->ring_off, src, count * sizeof(T));
    T* dst = (T*)(e->ring_d + e->ring_off);
    HIPC(hipMemcpyAsync(dst, e->ring_h + e->ring_off, count * sizeof(T), hipMemcpyHostToDevice, e->stream));
    e->ring_off += bytes;
    return dst;
}

// AESFHE_POOL_POISON=1 (diagnostic): every pool block handed out is first filled with 0xA5 bytes on
// the engine stream, so a read of words nobody wrote is deterministic (and loud) instead of
// whatever the block held before
static void* pool_get(aesfhe_engine* e, size_t bytes, bool tmp = false) {
    static const bool poison = getenv("AESFHE_POOL_POISON") && atoi(getenv("AESFHE_POOL_POISON"));
    (void)tmp;  // one arena (round 5 replay: two arenas held more); tpool stays empty
    void* p = e->pool.get(bytes);
    e->peak_total = std::max(e->peak_total, e->pool.live + e->tpool.live);
    if (poison && p) HIPC(hipMemsetAsync(p, 0xA5, bytes, e->stream));
    return p;
}
static u64* dalloc(aesfhe_engine* e, size_t words) { return (u64*)pool_get(e, words * 8, true); }
static void dfree(aesfhe_engine* e, u64* p, size_t words) { e->pool.put(p, words * 8); }

struct Tmp {  // RAII temporary device buffer from the pool
    aesfhe_engine* e;
    u64* p;
    size_t w;
    Tmp(aesfhe_engine* e_, size_t words) : e(e_), p(dalloc(e_, words)), w(words) {}
    ~Tmp() { dfree(e, p, w); }
};

static aesfhe_ct* ct_new(aesfhe_engine* e, int B, int np, int level) {
    auto* c = new aesfhe_ct;
    c->eng = e;
    e->refs++;
    c->B = B;
    c->np = np;
    c->level = level;
    c->is_zero = 0;
    c->bytes = (size_t)B * np * (level + 1) * e->N * 8;
    c->d = (u64*)pool_get(e, c->bytes);
    return c;
}

// The m outputs of a batched result r (batch m * B, output t = elements t*B .. t*B + B - 1) as m
// ciphertexts of batch B sharing r's device block (split in the pool, no copy); r is consumed.
static std::vector<aesfhe_ct*> ct_split_batch(aesfhe_engine* e, aesfhe_ct* r, int m) {
    const int B = r->B / m;
    const size_t part = (size_t)B * r->np * (r->level + 1) * e->N * 8;
    e->pool.split(r->d, m, part);
    std::vector<aesfhe_ct*> out(m);
    for (int t = 0; t < m; t++) {
        auto* c = new aesfhe_ct;
        c->eng = e;
        e->refs++;
        c->B = B;
        c->np = r->np;
        c->level = r->level;
        c->is_zero = 0;
        c->bytes = part;
        c->d = (u64*)((char*)r->d + (size_t)t * part);
        out[t] = c;
    }
    r->d = nullptr;  // the blocks now belong to the parts
    aesfhe_ct_free(r);
    return out;
}

static aesfhe_ct* ct_zero_new(aesfhe_engine* e, int B, int np, int level) {
    aesfhe_ct* c = ct_new(e, B, np, level);
    HIPC(hipMemsetAsync(c->d, 0, c->bytes, e->stream));
    c->is_zero = 1;
    return c;
}

// A (possibly strided / truncated / broadcast) view of ciphertext data.
struct View {
    const u64* d;
    int B, np, level;
    long ps, bs;  // poly stride, batch stride (0 = broadcast)
    bool zero;
};

static View view_of(const aesfhe_ct* c) {
    View v;
    v.d = c->d;
    v.B = c->B;
    v.np = c->np;
    v.level = c->level;
    v.ps = (long)(c->level + 1) * c->eng->N;
    v.bs = (long)c->np * v.ps;
    v.zero = c->is_zero;
    return v;
}

static Opnd opnd(const View& v, int outB) {
    Opnd o;
    o.ptr = v.zero ? nullptr : v.d;
    o.bs = (v.B == 1 && outB > 1) ? 0 : v.bs;
    o.ps = v.ps;
    o.np = v.np;
    o.bmask = (v.B > 1 && v.B < outB) ? v.B - 1 : -1;  // cyclic broadcast (check_cyclic)
    return o;
}

static Out out_of(aesfhe_ct* c) {
    Out o;
    o.ptr = c->d;
    o.ps = (long)(c->level + 1) * c->eng->N;
    o.bs = (long)c->np * o.ps;
    return o;
}

static dim3 ew_grid(aesfhe_engine* e, int y, int z) { return dim3(e->N / 256, y, z); }

// -----------------------------------------------------------------------------------------------
// NTT dispatch
// Each pass launch is profiled separately (family "ntt"): algorithmic bytes of one pass =
// 8 B * N * limbs, half of the NTT's read-once + write-once 16 B per coefficient.
template <int R1>
static void ntt_fwd_t(aesfhe_engine* e, Span src, Span dst, int total) {
    constexpr int CW = (kTile / R1) < kC2 ? (kTile / R1) : kC2;
    constexpr int RW = (kTile / kC2) < R1 ? (kTile / kC2) : R1;
    Tabs T = e->tabs();
    const double by = 8.0 * e->N * (double)total;
    {
        ProfScope ps(e, FAM_NTT, by, "ntt_generic");
        hipLaunchKernelGGL(k_ntt_fwd_cols<R1>, dim3(kC2 / CW, total), dim3(256), 0, e->stream, src, dst, T);
    }
    {
        ProfScope ps(e, FAM_NTT, by, "ntt_generic");
        hipLaunchKernelGGL(k_ntt_fwd_rows<R1>, dim3(R1 / RW, total), dim3(256), 0, e->stream, dst, T);
    }
}
template <int R1>
static void ntt_inv_t(aesfhe_engine* e, Span src, Span dst, int total) {
    constexpr int CW = (kTile / R1) < kC2 ? (kTile / R1) : kC2;
    constexpr int RW = (kTile / kC2) < R1 ? (kTile / kC2) : R1;
    Tabs T = e->tabs();
    const double by = 8.0 * e->N * (double)total;
    {
        ProfScope ps(e, FAM_NTT, by, "ntt_generic");
        hipLaunchKernelGGL(k_ntt_inv_rows<R1>, dim3(R1 / RW, total), dim3(256), 0, e->stream, src, dst, T);
    }
    {
        ProfScope ps(e, FAM_NTT, by, "ntt_generic");
        hipLaunchKernelGGL(k_ntt_inv_cols<R1>, dim3(kC2 / CW, total), dim3(256), 0, e->stream, dst, T);
    }
}

// N = 2^16 / 2^17: register-resident fp64-arithmetic passes over R = N / 256 rows of 256
// (ntt256f.h): a column pass (the first log2 R stages) and a row pass (the last 8)
template <int R>
static void ntt256(aesfhe_engine* e, Span src, Span dst, int total, bool inverse, const double* lf = nullptr) {
    Tabs T = e->tabs();
    // algorithmic bytes per pass: 8 B * N * limbs = half of the transform's read-once +
    // write-once 16 B per coefficient (the two-pass split itself is charged as overhead)
    const double by = 8.0 * e->N * (double)total;
    {
        ProfScope ps(e, FAM_NTT, by, inverse ? "ntt_inv_rows" : "ntt_fwd_cols");
        if (!inverse) hipLaunchKernelGGL(k_nttf_fwd_cols<R>, dim3(16, total), dim3(256), 0, e->stream, src, dst, T);
        else hipLaunchKernelGGL((k_nttf_inv_rows<R, false>), dim3(R / 16, total), dim3(256), 0, e->stream, src, dst, T, Span{}, (const u64*)nullptr);
    }
    ProfScope ps(e, FAM_NTT, by, inverse ? "ntt_inv_cols" : "ntt_fwd_rows");
    if (!inverse) hipLaunchKernelGGL((k_nttf_fwd_rows_t<false, R>), dim3(R / 16, total), dim3(256), 0, e->stream, dst, T, RowFin{});
    else if (lf) hipLaunchKernelGGL((k_nttf_inv_cols<R, true>), dim3(16, total), dim3(256), 0, e->stream, dst, T, lf);
    else hipLaunchKernelGGL((k_nttf_inv_cols<R, false>), dim3(16, total), dim3(256), 0, e->stream, dst, T, (const double*)nullptr);
}

// the N = 2^16 / 2^17 fp64 passes with fused epilogues (ModDown finish, key-switch inner product)
static bool fused_ntt(const aesfhe_engine* e) { return e->logN == 16 || e->logN == 17; }

// inverse NTT of the product a (x) b (two canonical operand spans of one shape) into dst, the
// product formed in the row pass's copy-in (fused_ntt engines)
// lf (N = 2^16): per-limb output factors replacing N^{-1} (k_nttf_inv_cols LF)
static void intt_prod(aesfhe_engine* e, Span a, Span b, Span dst, int total, const u64* fac, const double* lf = nullptr) {
    if (total <= 0) return;
    Tabs T = e->tabs();
    const double by = 8.0 * e->N * (double)total;
    {
        ProfScope ps(e, FAM_NTT, 2.0 * by, "ntt_inv_rows_prod");  // two operands read
        if (e->logN == 16) {
            if (fac) hipLaunchKernelGGL((k_nttf_inv_rows<256, true, true>), dim3(16, total), dim3(256), 0, e->stream, a, dst, T, b, fac);
            else hipLaunchKernelGGL((k_nttf_inv_rows<256, true, false>), dim3(16, total), dim3(256), 0, e->stream, a, dst, T, b, fac);
        } else {
            if (fac) hipLaunchKernelGGL((k_nttf_inv_rows<512, true, true>), dim3(32, total), dim3(256), 0, e->stream, a, dst, T, b, fac);
            else hipLaunchKernelGGL((k_nttf_inv_rows<512, true, false>), dim3(32, total), dim3(256), 0, e->stream, a, dst, T, b, fac);
        }
    }
    ProfScope ps(e, FAM_NTT, by, "ntt_inv_cols");
    if (e->logN == 16) {
        if (lf) hipLaunchKernelGGL((k_nttf_inv_cols<256, true>), dim3(16, total), dim3(256), 0, e->stream, dst, T, lf);
        else hipLaunchKernelGGL((k_nttf_inv_cols<256, false>), dim3(16, total), dim3(256), 0, e->stream, dst, T, lf);
    } else {
        if (lf) throw_err(AESFHE_EUNSUPPORTED, "per-limb INTT factors at N = 2^17");
        hipLaunchKernelGGL((k_nttf_inv_cols<512, false>), dim3(16, total), dim3(256), 0, e->stream, dst, T, lf);
    }
    HIPC(hipGetLastError());
}

// the fp64 column pass alone (the extension limbs and the conv of a ModDown, whose row passes run
// fused with their consumers)
static void ntt_fwd_cols(aesfhe_engine* e, Span src, Span dst, int total) {
    if (e->logN == 16) hipLaunchKernelGGL(k_nttf_fwd_cols<256>, dim3(16, total), dim3(256), 0, e->stream, src, dst, e->tabs());
    else hipLaunchKernelGGL(k_nttf_fwd_cols<512>, dim3(16, total), dim3(256), 0, e->stream, src, dst, e->tabs());
}
static void ntt_fwd_cols(aesfhe_engine* e, Span sp, int total) { ntt_fwd_cols(e, sp, sp, total); }

static void ntt(aesfhe_engine* e, Span src, Span dst, int total, bool inverse) {
    if (total <= 0) return;
    if (e->logN == 16 || e->logN == 17) {
        if (e->logN == 16) ntt256<256>(e, src, dst, total, inverse);
        else ntt256<512>(e, src, dst, total, inverse);
        HIPC(hipGetLastError());
        return;
    }
    switch (e->logN) {
#define CASE(LG, R)                                                        \
    case LG:                                                               \
        if (inverse) ntt_inv_t<R>(e, src, dst, total);                     \
        else ntt_fwd_t<R>(e, src, dst, total);                             \
        break;
        CASE(10, 4)
        CASE(11, 8)
        CASE(12, 16)
        CASE(13, 32)
        CASE(14, 64)
        CASE(15, 128)
        CASE(16, 256)
        CASE(17, 512)
#undef CASE
        default:
            throw_err(AESFHE_EUNSUPPORTED, "log_n %d not supported by the HIP NTT", e->logN);
    }
    HIPC(hipGetLastError());
}

static Span span_s(u64* base, long pstride, int nl, int nq, int qpid0, int spid0) {
    Span s;
    s.base = base;
    s.pstride = pstride;
    s.nl = nl;
    s.nq = nq;
    s.qpid0 = qpid0;
    s.spid0 = spid0;
    return s;
}

// -----------------------------------------------------------------------------------------------
// engine creation: tables

// bytes of a canonical residue of prime q (0 <= y < q)
static int res_bytes(u64 q) {
    int b = 0;
    for (u64 x = q - 1; x; x >>= 8) b++;
    return b;
}
// The constant rows of one target prime p for a matrix-core base conversion (bconv_mfma.h):
// tab = 8 planes x kBconvKT bytes; source slot sl's byte a (K byte 8 sl + a) holds the signed
// balanced base-256 digits of H' = 256^a H[sl] mod p over the planes b = 0..6 (plane 7 zero), for
// the bytes a < res_bytes(q_sl) a canonical y can have; with vc, K byte 8 ns holds those of G
// (ModDown's -D mod p, times the in-kernel v).  Returns 128 * (sum of every H' placed) mod p:
// the kernel feeds the bytes as u - 128 (XOR 0x80, signed MFMA operands).
static u64 bconv_row(int8_t* tab, u64 p, int ns, const u64* srcq, const u64* H, bool vc, u64 G) {
    u64 corr = 0;
    auto place = [&](int k, u64 hp) {
        int64_t x = (int64_t)hp;  // < 2^50: seven balanced digits reach 2^55
        for (int b = 0; b < 7; b++) {
            const int d = (int)((x + 128) & 255) - 128;
            tab[b * kBconvKT + k] = (int8_t)d;
            x = (x - d) / 256;
        }
        if (x != 0) throw_err(AESFHE_EUNSUPPORTED, "base-conversion constant beyond 7 bytes");
        corr = (corr + h_mulmod(128 % p, hp, p)) % p;
    };
    for (int sl = 0; sl < ns; sl++) {
        u64 r = 1 % p;  // 256^a mod p
        for (int a = 0; a < res_bytes(srcq[sl]); a++) {
            place(8 * sl + a, h_mulmod(r, H[sl] % p, p));
            r = h_mulmod(r, 256 % p, p);
        }
    }
    if (vc) place(8 * ns, G % p);
    return corr;
}

static void build_tables(aesfhe_engine* e) {
    const int N = e->N, np = e->np, L = e->L, K = e->K, Lp1 = e->Lp1;
    const auto& Q = e->chain.q;
    std::vector<u64> hq(Q), hpsi((size_t)np * N), hipsi((size_t)np * N), hninv(np);
    std::vector<double> hqinv(np), hpsif((size_t)np * N), hipsif((size_t)np * N), hninvf(np);
    e->h_iroot.resize(np);
    for (int p = 0; p < np; p++) {
        u64 qq = Q[p];
        hqinv[p] = 1.0 / (double)qq;
        u64 psi = min_primitive_root(qq, N), ip = h_invmod(psi, qq);
        std::vector<u64> pw(N), ipw(N);
        pw[0] = ipw[0] = 1;
        for (int k = 1; k < N; k++) {
            pw[k] = h_mulmod(pw[k - 1], psi, qq);
            ipw[k] = h_mulmod(ipw[k - 1], ip, qq);
        }
        for (int k = 0; k < N; k++) {
            unsigned r = bit_reverse((unsigned)k, e->logN);
            hpsi[(size_t)p * N + k] = pw[r];
            hipsi[(size_t)p * N + k] = ipw[r];
            hpsif[(size_t)p * N + k] = (double)pw[r] / (double)qq;
            hipsif[(size_t)p * N + k] = (double)ipw[r] / (double)qq;
        }
        e->h_iroot[p] = pw[N / 2];
        hninv[p] = h_invmod((u64)N, qq);
        hninvf[p] = (double)hninv[p] / (double)qq;
    }
    auto up = [&](auto& vec, auto** dst) {
        using T = typename std::remove_reference<decltype(vec)>::type::value_type;
        size_t bytes = vec.size() * sizeof(T);
        HIPC(hipMalloc((void**)dst, std::max<size_t>(bytes, 8)));
        HIPC(hipMemcpy(*dst, vec.data(), bytes, hipMemcpyHostToDevice));
    };
    up(hq, &e->q);
    up(hqinv, &e->qinv);
    up(hpsi, &e->psi);
    up(hpsif, &e->psif);
    up(hipsi, &e->ipsi);
    up(hipsif, &e->ipsif);
    up(hninv, &e->ninv);
    up(hninvf, &e->ninvf);
    if (fused_ntt(e)) {  // row factors psi^{+-brv(row << s)} / q, s = 0..7, [np][R][8] (ntt256f.h tw_row)
        const int R = N / 256;
        std::vector<double> hr((size_t)np * R * 8), hir((size_t)np * R * 8);
        for (int p = 0; p < np; p++)
            for (int row = 0; row < R; row++)
                for (int sh = 0; sh < 8; sh++) {
                    hr[((size_t)p * R + row) * 8 + sh] = hpsif[(size_t)p * N + (row << sh)];
                    hir[((size_t)p * R + row) * 8 + sh] = hipsif[(size_t)p * N + (row << sh)];
                }
        up(hr, &e->rtwf);
        up(hir, &e->irtwf);
    }
    {
        std::vector<Tw> htw((size_t)np * N), hitw((size_t)np * N);
        for (size_t i = 0; i < htw.size(); i++) {
            htw[i] = Tw{hpsi[i], hpsif[i]};
            hitw[i] = Tw{hipsi[i], hipsif[i]};
        }
        up(htw, &e->tw);
        up(hitw, &e->itw);
    }
    {
        std::vector<double> hcw((size_t)np * kColW), hicw((size_t)np * kColW);
        for (int p = 0; p < np; p++)
            for (int k = 0; k < kColW; k++) {
                hcw[(size_t)p * kColW + k] = (double)hpsi[(size_t)p * N + (k < N ? k : 0)];
                hicw[(size_t)p * kColW + k] = (double)hipsi[(size_t)p * N + (k < N ? k : 0)];
            }
        up(hcw, &e->cw);
        up(hicw, &e->icw);
    }

    // ModUp tables per (digit j, width a <= alpha): hatinv[i], hat[i][pid]; stride A = alpha
    const int A = e->A;
    const size_t mu_sets = (size_t)e->dnum * A;
    std::vector<u64> hhatinv(mu_sets * A, 0), hhat(mu_sets * A * np, 0);
    std::vector<double> hhatinvf(mu_sets * A, 0);
    std::vector<TwD> hhatf(mu_sets * A * np, TwD{0, 0});
    for (int j = 0; j < e->dnum; j++)
        for (int a = 1; a <= A; a++) {
            int lo = j * A, hi = lo + a;
            if (hi > Lp1) continue;
            size_t set = (size_t)j * A + (a - 1);
            for (int i = lo; i < hi; i++) {
                u64 prod = 1;
                for (int i2 = lo; i2 < hi; i2++)
                    if (i2 != i) prod = h_mulmod(prod, Q[i2] % Q[i], Q[i]);
                u64 hv = h_invmod(prod, Q[i]);
                hhatinv[set * A + (i - lo)] = hv;
                hhatinvf[set * A + (i - lo)] = (double)hv / (double)Q[i];
                for (int pid = 0; pid < np; pid++) {
                    u64 qt = Q[pid], h = 1;
                    for (int i2 = lo; i2 < hi; i2++)
                        if (i2 != i) h = h_mulmod(h, Q[i2] % qt, qt);
                    hhat[(set * A + (i - lo)) * np + pid] = h;
                    // [set][target pid][i]: a target's alpha constants are contiguous (one
                    // scalar base, immediate offsets in k_modup)
                    hhatf[(set * np + pid) * A + (i - lo)] = TwD{(double)h, (double)h / (double)qt};
                }
            }
        }
    up(hhatinv, &e->mu_hatinv);
    up(hhatinvf, &e->mu_hatinvf);
    {  // the INTT in front of a fused ModUp (bconv_cols.h YIN) scales limb i of a level-l input by
       // N^{-1} hatinv_{l,i} (its digit's width at level l) instead of N^{-1}: it emits y directly
        std::vector<double> nh((size_t)Lp1 * Lp1, 0.0);
        for (int l = 0; l < Lp1; l++)
            for (int i = 0; i <= l; i++) {
                const int lo = (i / A) * A, a = std::min(A, l + 1 - lo);
                const u64 hv = hhatinv[((size_t)(i / A) * A + (a - 1)) * A + (i - lo)];
                nh[(size_t)l * Lp1 + i] = (double)h_mulmod(hninv[i], hv, Q[i]) / (double)Q[i];
            }
        up(nh, &e->mu_nhatf);
    }
    up(hhat, &e->mu_hat);
    up(hhatf, &e->mu_hatf);
    {  // matrix-core ModUp rows: [set][pid] (the digit's own pids are never targets)
        const size_t row = 8 * (size_t)kBconvKT;
        std::vector<int8_t> tab(mu_sets * np * row, 0);
        std::vector<double> corr(mu_sets * np, 0.0), pc(4 * (size_t)np);
        for (int j = 0; j < e->dnum; j++)
            for (int a = 1; a <= A; a++) {
                const int lo = j * A;
                if (lo + a > Lp1 || a > 16) continue;
                const size_t set = (size_t)j * A + (a - 1);
                for (int pid = 0; pid < np; pid++) {
                    std::vector<u64> H(a);
                    for (int i = 0; i < a; i++) H[i] = hhat[(set * A + i) * np + pid];
                    corr[set * np + pid] = (double)bconv_row(&tab[(set * np + pid) * row], Q[pid], a, &Q[lo], H.data(), false, 0);
                }
            }
        for (int pid = 0; pid < np; pid++) {  // {p, 1/p, 2^32 mod p, (2^32 mod p) / p}
            const u64 p = Q[pid], w = (1ULL << 32) % p;
            pc[4 * pid] = (double)p;
            pc[4 * pid + 1] = 1.0 / (double)p;
            pc[4 * pid + 2] = (double)w;
            pc[4 * pid + 3] = (double)w / (double)p;
        }
        up(tab, &e->bc_mu_tab);
        up(corr, &e->bc_mu_corr);
        up(pc, &e->bc_pc);
    }

    // ModDown tables
    std::vector<u64> hphatinv(K), hphat((size_t)K * Lp1), hpinv(Lp1), hpmod(np, 0);
    std::vector<double> hphatinvf(K), hpinvf(Lp1);
    std::vector<TwD> hphatf((size_t)K * Lp1);
    for (int k = 0; k < K; k++) {
        u64 pk = Q[Lp1 + k], prod = 1;
        for (int k2 = 0; k2 < K; k2++)
            if (k2 != k) prod = h_mulmod(prod, Q[Lp1 + k2] % pk, pk);
        hphatinv[k] = h_invmod(prod, pk);
        hphatinvf[k] = (double)hphatinv[k] / (double)pk;
        for (int i = 0; i < Lp1; i++) {
            u64 qi = Q[i], h = 1;
            for (int k2 = 0; k2 < K; k2++)
                if (k2 != k) h = h_mulmod(h, Q[Lp1 + k2] % qi, qi);
            hphat[(size_t)k * Lp1 + i] = h;
            hphatf[(size_t)i * K + k] = TwD{(double)h, (double)h / (double)qi};  // [target i][source k]
        }
    }
    for (int i = 0; i < Lp1; i++) {
        u64 qi = Q[i], P = 1;
        for (int k = 0; k < K; k++) P = h_mulmod(P, Q[Lp1 + k] % qi, qi);
        hpmod[i] = P;
        hpinv[i] = h_invmod(P, qi);
        hpinvf[i] = (double)hpinv[i] / (double)qi;
    }
    {  // matrix-core ModDown rows, r = 0: sources p_0..p_{K-1}, targets q_i, v slot G = -P mod q_i
        const size_t row = 8 * (size_t)kBconvKT;
        std::vector<int8_t> tab((size_t)Lp1 * row, 0);
        std::vector<double> corr(Lp1, 0.0);
        if (K + 1 <= 16)
            for (int i = 0; i < Lp1; i++) {
                const u64 qi = Q[i];
                std::vector<u64> H(K);
                u64 P = 1;
                for (int k = 0; k < K; k++) {
                    H[k] = hphat[(size_t)k * Lp1 + i];
                    P = h_mulmod(P, Q[Lp1 + k] % qi, qi);
                }
                corr[i] = (double)bconv_row(&tab[(size_t)i * row], qi, K, &Q[Lp1], H.data(), true, (qi - P) % qi);
            }
        up(tab, &e->bc_md_tab);
        up(corr, &e->bc_md_corr);
    }
    up(hphatinv, &e->md_phatinv);
    up(hphatinvf, &e->md_phatinvf);
    up(hphat, &e->md_phat);
    up(hphatf, &e->md_phatf);
    up(hpinv, &e->md_pinv);
    up(hpinvf, &e->md_pinvf);
    up(hpmod, &e->pmod);
    {
        std::vector<double> hpmodf(Lp1);
        for (int i = 0; i < Lp1; i++) hpmodf[i] = (double)hpmod[i] / (double)Q[i];
        up(hpmodf, &e->pmodf);
        std::vector<double> heinv0(kMdrMaxE, 0.0);  // 1/p_k: the exact conversion of plain ModDown
        for (int k = 0; k < K; k++) heinv0[k] = 1.0 / (double)Q[Lp1 + k];
        up(heinv0, &e->md_einv);
        std::vector<double> hn0(kMdrMaxE, 0.0);  // fused ModDown: N^{-1} phatinv_k folded into the INTT
        for (int k = 0; k < K; k++) hn0[k] = (double)h_mulmod(hninv[Lp1 + k], hphatinv[k], Q[Lp1 + k]) / (double)Q[Lp1 + k];
        up(hn0, &e->md_ninvf);
    }
    // combined ModDown + rescale: E = {q_{l-r+1}..q_l, p_0..p_{K-1}} (acc limb order), D = prod E
    //   mdr_invf[(r-1, l)][j]       = (D/e_j)^{-1} mod e_j, as w/e_j
    //   mdr_hatf[(r-1, l)][i][j]    = (D/e_j) mod q_i, as {w, w/q_i}   (i <= l - r)
    //   mdr_dinv[(r-1, l)][i] (+f)  = D^{-1} mod q_i
    {
        const size_t cells = (size_t)kMdrMaxR * Lp1;
        std::vector<double> hinvf(cells * kMdrMaxE, 0.0), hdinvf(cells * Lp1, 0.0);
        std::vector<TwD> hhatf(cells * kMdrMaxE * Lp1, TwD{0, 0});
        std::vector<u64> hdinv(cells * Lp1, 0);
        std::vector<double> heinv(cells * kMdrMaxE, 0.0), hdmodf(cells * Lp1, 0.0), hninvf(cells * kMdrMaxE, 0.0);
        // matrix-core rows [cell][target i][8][kBconvKT] (bconv_mfma.h), v slot G = -D mod q_i
        const size_t brow = 8 * (size_t)kBconvKT;
        std::vector<int8_t> btab(cells * Lp1 * brow, 0);
        std::vector<double> bcorr(cells * Lp1, 0.0);
        for (int r = 1; r <= kMdrMaxR && K + r <= kMdrMaxE; r++)
            for (int l = r; l <= L; l++) {
                const size_t cell = (size_t)(r - 1) * Lp1 + l;
                std::vector<int> E;
                for (int j = 0; j < r; j++) E.push_back(l - r + 1 + j);
                for (int j = 0; j < K; j++) E.push_back(Lp1 + j);
                std::vector<u64> Hc((size_t)(l - r + 1) * E.size()), Eq(E.size());
                for (size_t j = 0; j < E.size(); j++) Eq[j] = Q[E[j]];
                for (size_t j = 0; j < E.size(); j++) {
                    const u64 ej = Q[E[j]];
                    u64 prod = 1;
                    for (size_t j2 = 0; j2 < E.size(); j2++)
                        if (j2 != j) prod = h_mulmod(prod, Q[E[j2]] % ej, ej);
                    hinvf[cell * kMdrMaxE + j] = (double)h_invmod(prod, ej) / (double)ej;
                    hninvf[cell * kMdrMaxE + j] = (double)h_mulmod(hninv[E[j]], h_invmod(prod, ej), ej) / (double)ej;
                    heinv[cell * kMdrMaxE + j] = 1.0 / (double)ej;
                    for (int i = 0; i <= l - r; i++) {
                        const u64 qi = Q[i];
                        u64 h = 1;
                        for (size_t j2 = 0; j2 < E.size(); j2++)
                            if (j2 != j) h = h_mulmod(h, Q[E[j2]] % qi, qi);
                        hhatf[(cell * Lp1 + i) * kMdrMaxE + j] = TwD{(double)h, (double)h / (double)qi};  // [cell][target i][source j]
                        Hc[(size_t)i * E.size() + j] = h;
                    }
                }
                for (int i = 0; i <= l - r; i++) {
                    const u64 qi = Q[i];
                    u64 D = 1;
                    for (int ei : E) D = h_mulmod(D, Q[ei] % qi, qi);
                    const u64 di = h_invmod(D, qi);
                    hdinv[cell * Lp1 + i] = di;
                    hdmodf[cell * Lp1 + i] = (double)D / (double)qi;
                    hdinvf[cell * Lp1 + i] = (double)di / (double)qi;
                    if ((int)E.size() + 1 <= 16)
                        bcorr[cell * Lp1 + i] = (double)bconv_row(&btab[(cell * Lp1 + i) * brow], qi, (int)E.size(), Eq.data(),
                                                                  &Hc[(size_t)i * E.size()], true, (qi - D) % qi);
                }
            }
        up(btab, &e->bc_mdr_tab);
        up(bcorr, &e->bc_mdr_corr);
        up(hinvf, &e->mdr_invf);
        up(hninvf, &e->mdr_ninvf);
        up(hhatf, &e->mdr_hatf);
        up(hdinv, &e->mdr_dinv);
        up(hdinvf, &e->mdr_dinvf);
        up(heinv, &e->mdr_einv);
        up(hdmodf, &e->mdr_dmodf);
    }

    // rescale tables rs_inv[l][i] = q_l^{-1} mod q_i, rs_mod[l][i] = q_l mod q_i
    std::vector<u64> hrinv((size_t)Lp1 * Lp1, 0), hrmod((size_t)Lp1 * Lp1, 0);
    std::vector<double> hrinvf((size_t)Lp1 * Lp1, 0);
    for (int l = 1; l <= L; l++)
        for (int i = 0; i < l; i++) {
            u64 qi = Q[i];
            hrmod[(size_t)l * Lp1 + i] = Q[l] % qi;
            hrinv[(size_t)l * Lp1 + i] = h_invmod(Q[l] % qi, qi);
            hrinvf[(size_t)l * Lp1 + i] = (double)hrinv[(size_t)l * Lp1 + i] / (double)qi;
        }
    up(hrinv, &e->rs_inv);
    up(hrinvf, &e->rs_invf);
    up(hrmod, &e->rs_mod);
}

extern "C" int aesfhe_engine_create(const aesfhe_params* pp, aesfhe_engine** out) {
    API_BEGIN
    if (!pp || !out) throw_err(AESFHE_EARG, "null argument");
    if (pp->log_n < 10 || pp->log_n > 17) throw_err(AESFHE_EARG, "log_n must be in [10, 17]");
    if (pp->max_level < 1 || pp->special_primes < 1 || pp->special_primes > 16 ||
        pp->max_level + 1 + pp->special_primes > kMaxPrimes)
        throw_err(AESFHE_EARG, "bad level / special prime count");
    if (pp->scale_bits < 20 || pp->scale_bits > 50 || pp->base_bits > 50 || pp->special_bits > 50)
        throw_err(AESFHE_EARG, "bit sizes must keep every prime below 2^50");
    std::unique_ptr<aesfhe_engine> e(new aesfhe_engine());
    e->logN = pp->log_n;
    e->N = 1 << pp->log_n;
    e->L = pp->max_level;
    e->K = pp->special_primes;
    e->Lp1 = e->L + 1;
    e->np = e->L + 1 + e->K;
    e->A = pp->digit_primes > 0 ? pp->digit_primes : e->K;
    if (e->A > 16) throw_err(AESFHE_EARG, "key-switch digit width %d outside 1..16", e->A);
    e->dnum = (e->L + 1 + e->A - 1) / e->A;
    e->device = pp->device;
    e->seed = pp->seed;
    e->ck = chacha_key(pp->seed, pp->seed_ext);
    if (pp->primes) {
        e->chain.q.assign(pp->primes, pp->primes + e->np);
        e->chain.scale = scales_from_primes(e->chain.q, e->L, pp->scale_bits);
    } else {
        e->chain = make_chain(e->logN, e->L, e->K, pp->base_bits, pp->special_bits, pp->scale_bits);
    }
    for (u64 x : e->chain.q)  // lazy NTT keeps values < 4q, which must stay below 2^52
        if (x >> 50) throw_err(AESFHE_EARG, "prime %llu exceeds 2^50", (unsigned long long)x);
    if (e->A > e->K && !digits_below_p(e->chain.q, e->Lp1, e->K, e->A))
        throw_err(AESFHE_EARG, "a key-switch digit of %d primes exceeds P (%d special primes)", e->A, e->K);
    HIPC(hipSetDevice(e->device));
    HIPC(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    build_tables(e.get());
    // arena chunks of 16384 limbs (8 GiB at N = 2^16), at least 256 MiB; AESFHE_ARENA_CHUNK_MB
    // overrides it (several engines sharing one GPU, small batches)
    e->pool.chunk_bytes = std::max((size_t)1 << 28, ((size_t)16384 * 8) << e->logN);
    if (e->logN == 16) {  // the bench ring: first fit in 4 GiB chunks, cap 1.2 (arena.h)
        e->pool.chunk_bytes = (size_t)8192 * 8 << e->logN;
        e->pool.first_fit = true;
        e->pool.grow_cap = 1.2;
    }
    if (const char* cm = getenv("AESFHE_ARENA_CHUNK_MB")) {
        const long mb = atol(cm);
        if (mb > 0) e->pool.chunk_bytes = (size_t)mb << 20;
    }
    e->tpool.chunk_bytes = e->pool.chunk_bytes;
    e->tpool.tag = 't';
    if (const char* tp = getenv("AESFHE_ARENA_TRACE")) {
        static std::atomic<int> engines{0};
        const std::string path = std::string(tp) + "." + std::to_string(engines++);
        e->pool.trace = e->tpool.trace = fopen(path.c_str(), "w");
    }
    HIPC(hipMalloc(&e->ring_d, e->ring_size));
    HIPC(hipHostMalloc((void**)&e->ring_h, e->ring_size, hipHostMallocDefault));
    *out = e.release();
    API_END
}

extern "C" int aesfhe_chain(const aesfhe_params* pp, uint64_t* primes, double* scales) {
    API_BEGIN
    Chain c = make_chain(pp->log_n, pp->max_level, pp->special_primes, pp->base_bits, pp->special_bits, pp->scale_bits);
    std::copy(c.q.begin(), c.q.end(), primes);
    std::copy(c.scale.begin(), c.scale.end(), scales);
    API_END
}

static void engine_teardown(aesfhe_engine* e);
static void engine_unref(aesfhe_engine* e) {
    if (--e->refs == 0) engine_teardown(e);
}
extern "C" void aesfhe_engine_destroy(aesfhe_engine* e) {
    if (e) engine_unref(e);
}
static void engine_teardown(aesfhe_engine* e) {
    hipSetDevice(e->device);
    hipStreamSynchronize(e->stream);
    for (auto& r : e->recs) {
        hipEventDestroy(r.a);
        hipEventDestroy(r.b);
    }
    for (auto ev : e->spare) hipEventDestroy(ev);
    e->pool.release_all();
    e->tpool.release_all();
    if (e->pool.trace) fclose(e->pool.trace);
    void* ptrs[] = {e->q, e->psi, e->ipsi, e->ninv, e->qinv, e->psif, e->ipsif, e->ninvf, e->rtwf, e->irtwf,
                    e->mu_hatinv, e->mu_hat, e->md_phatinv, e->md_phat, e->md_pinv, e->rs_inv,
                    e->rs_mod, e->pmod, e->mu_hatinvf, e->mu_hatf, e->md_phatinvf, e->md_phatf,
                    e->md_pinvf, e->rs_invf, e->ring_d, e->tw, e->itw, e->mdr_invf, e->mdr_hatf,
                    e->mdr_dinv, e->mdr_dinvf, e->pmodf, e->mdr_einv, e->mdr_dmodf, e->md_einv,
                    e->bc_mu_tab, e->bc_md_tab, e->bc_mdr_tab, e->bc_mu_corr, e->bc_md_corr, e->bc_mdr_corr,
                    e->bc_pc, e->mu_nhatf, e->md_ninvf, e->mdr_ninvf, e->cw, e->icw};
    for (void* p : ptrs)
        if (p) hipFree(p);
    for (auto& kv : e->poly2_tabs) hipFree(kv.second);
    for (void* p : {(void*)e->ckre, (void*)e->ckim, (void*)e->crot, (void*)e->cflags})
        if (p) hipFree(p);
    if (e->ring_h) hipHostFree(e->ring_h);
    hipStreamDestroy(e->stream);
    delete e;
}

extern "C" int aesfhe_engine_dims(const aesfhe_engine* e, int32_t d[4]) {
    d[0] = e->logN;
    d[1] = e->L;
    d[2] = e->K;
    d[3] = e->dnum;
    return 0;
}
extern "C" int aesfhe_engine_primes(const aesfhe_engine* e, uint64_t* o) {
    std::copy(e->chain.q.begin(), e->chain.q.end(), o);
    return 0;
}
extern "C" int aesfhe_engine_scales(const aesfhe_engine* e, double* o) {
    std::copy(e->chain.scale.begin(), e->chain.scale.end(), o);
    return 0;
}
extern "C" double aesfhe_engine_mul_scale(const aesfhe_engine* e, int32_t l) {
    if (l < 1 || l > e->L) return 0.0;
    return e->chain.scale[l - 1] * (double)e->chain.q[l] / e->chain.scale[l];
}
extern "C" int aesfhe_engine_sync(aesfhe_engine* e) {
    API_BEGIN
    HIPC(hipStreamSynchronize(e->stream));
    API_END
}
extern "C" int aesfhe_engine_profile(aesfhe_engine* e, int32_t en) {
    API_BEGIN
    prof_flush(e);
    e->prof = en == -1 ? 7 : (en & 7);
    if (e->prof) {
        for (int i = 0; i < 4; i++) e->prof_ms[i] = e->prof_bytes[i] = 0, e->prof_n[i] = 0;
        e->prof_k.clear();
        // pre-create events so that none is created inside a measured region
        while (e->spare.size() < 65536) {
            hipEvent_t x;
            HIPC(hipEventCreate(&x));
            e->spare.push_back(x);
        }
    }
    API_END
}
extern "C" int aesfhe_engine_profile_read(aesfhe_engine* e, const char* fam, int64_t* n,
                                          double* ms, double* bytes) {
    API_BEGIN
    prof_flush(e);
    int f = !strcmp(fam, "ntt") ? FAM_NTT : !strcmp(fam, "keyswitch") ? FAM_KS : !strcmp(fam, "elementwise") ? FAM_EW : 3;
    if (f == 3) {
        *n = e->prof_n[0] + e->prof_n[1] + e->prof_n[2];
        *ms = e->prof_ms[0] + e->prof_ms[1] + e->prof_ms[2];
        if (bytes) *bytes = e->prof_bytes[0] + e->prof_bytes[1] + e->prof_bytes[2];
    } else {
        *n = e->prof_n[f];
        *ms = e->prof_ms[f];
        if (bytes) *bytes = e->prof_bytes[f];
    }
    API_END
}
extern "C" int aesfhe_engine_profile_kernels(aesfhe_engine* e, char* buf, int64_t cap, int64_t* need) {
    API_BEGIN
    prof_flush(e);
    std::string js = "{";
    char tmp[256];
    for (auto& kv : e->prof_k) {
        snprintf(tmp, sizeof tmp, "%s\"%s\": [%lld, %.6f, %.1f, %lld]", js.size() > 1 ? ", " : "", kv.first.c_str(),
                 (long long)kv.second.n, kv.second.ms, kv.second.bytes, (long long)kv.second.d);
        js += tmp;
    }
    js += "}";
    if (need) *need = (int64_t)js.size() + 1;
    if (buf && cap > 0) {
        const size_t m = std::min((size_t)cap - 1, js.size());
        memcpy(buf, js.data(), m);
        buf[m] = 0;
    }
    API_END
}
extern "C" int64_t aesfhe_engine_device_bytes(const aesfhe_engine* e) { return (int64_t)(e->pool.held + e->tpool.held); }
extern "C" int aesfhe_engine_pool_trim(aesfhe_engine* e) {
    API_BEGIN
    HIPC(hipSetDevice(e->device));
    HIPC(hipStreamSynchronize(e->stream));
    e->pool.trim();
    e->tpool.trim();
    API_END
}
// both arenas together: held, live, hipMallocs, trims, larger-block reuses, the largest combined
// live set, fragmentation
extern "C" int aesfhe_engine_pool_stats(const aesfhe_engine* e, int64_t* out) {
    if (!e || !out) return set_err(AESFHE_EARG, "null argument");
    out[0] = (int64_t)(e->pool.held + e->tpool.held);
    out[1] = (int64_t)(e->pool.live + e->tpool.live);
    out[2] = e->pool.mallocs + e->tpool.mallocs;
    out[3] = e->pool.trims + e->tpool.trims;
    out[4] = e->pool.reuse_larger + e->tpool.reuse_larger;
    out[5] = (int64_t)e->peak_total;
    out[6] = (int64_t)(e->pool.fragmentation() + e->tpool.fragmentation());
    return AESFHE_OK;
}

// -----------------------------------------------------------------------------------------------
// host codec
extern "C" int aesfhe_encode(int32_t logN, const double* re, const double* im, int64_t n_slots,
                             double scale, int64_t* co) {
    API_BEGIN
    if (logN < 2 || logN > 17) throw_err(AESFHE_EARG, "log_n out of range");
    Codec c(logN);
    if (n_slots < 0 || n_slots > c.n) throw_err(AESFHE_EARG, "too many slots: %lld > %d", (long long)n_slots, c.n);
    std::vector<double> vr(c.n, 0.0), vi(c.n, 0.0);
    for (int64_t i = 0; i < n_slots; i++) {
        vr[i] = re ? re[i] : 0.0;
        vi[i] = im ? im[i] : 0.0;
    }
    c.special_inv(vr.data(), vi.data());
    for (int i = 0; i < c.n; i++) {
        double a = vr[i] * scale, b = vi[i] * scale;
        if (!(std::fabs(a) < 9.0e18) || !(std::fabs(b) < 9.0e18))
            throw_err(AESFHE_EARG, "encoded coefficient overflows int64 (scale too large?)");
        co[i] = llround(a);
        co[i + c.n] = llround(b);
    }
    API_END
}

extern "C" int aesfhe_decode(int32_t logN, const int64_t* co, double scale, double* re, double* im) {
    API_BEGIN
    if (logN < 2 || logN > 17) throw_err(AESFHE_EARG, "log_n out of range");
    Codec c(logN);
    for (int i = 0; i < c.n; i++) {
        re[i] = (double)co[i] / scale;
        im[i] = (double)co[i + c.n] / scale;
    }
    c.special(re, im);
    API_END
}

// -----------------------------------------------------------------------------------------------
// keys
extern "C" void aesfhe_key_free(aesfhe_key* k) {
    if (!k) return;
    aesfhe_engine* e = k->eng;
    e->pool.put(k->d, k->bytes);
    delete k;
    engine_unref(e);
}
extern "C" int aesfhe_key_info(const aesfhe_key* k, int32_t* kind, uint64_t* g) {
    *kind = k->kind;
    *g = k->galois;
    return 0;
}
extern "C" uint64_t aesfhe_galois_elt(int32_t logN, int64_t rot, int32_t conj) {
    u64 M = 2ULL << logN, n = 1ULL << (logN - 1);
    if (conj) return M - 1;
    int64_t r = rot % (int64_t)n;
    if (r < 0) r += (int64_t)n;
    u64 ex = (n - (u64)r) % n;
    return h_powmod(5, ex, M);
}

static aesfhe_key* key_new(aesfhe_engine* e, int kind, size_t words) {
    auto* k = new aesfhe_key;
    k->eng = e;
    e->refs++;
    k->kind = kind;
    k->galois = 0;
    k->keyseed = 0;
    k->bytes = words * 8;
    k->d = (u64*)pool_get(e, k->bytes);
    return k;
}

// residues of a small sampled polynomial for every prime (pid-major [np][N]) in NTT form
static void sample_small_ntt(aesfhe_engine* e, u64* dst, int nprimes, u64 key, int kind) {
    Span s = span_s(dst, 0, nprimes, std::min(nprimes, e->Lp1), 0, e->Lp1);
    s.pstride = (long)nprimes * e->N;
    hipLaunchKernelGGL(k_sample_small, dim3((e->N / 8 + 255) / 256), dim3(256), 0, e->stream, s, e->ck, key, kind, e->q, e->logN, e->Lp1, nprimes);
    ntt(e, s, s, nprimes, false);
}

extern "C" int aesfhe_key_secret(aesfhe_engine* e, uint64_t seed, aesfhe_key** out) {
    API_BEGIN
    aesfhe_key* k = key_new(e, 0, (size_t)e->np * e->N);
    k->keyseed = derive(e->seed, seed);
    sample_small_ntt(e, k->d, e->np, derive(k->keyseed, 1), 0);
    *out = k;
    API_END
}

extern "C" int aesfhe_key_public(aesfhe_engine* e, const aesfhe_key* sk, aesfhe_key** out) {
    API_BEGIN
    if (!sk || sk->kind != 0) throw_err(AESFHE_EARG, "public key needs a secret key");
    const int N = e->N, nq = e->Lp1;
    aesfhe_key* k = key_new(e, 1, (size_t)2 * nq * N);
    k->keyseed = sk->keyseed;
    u64* b = k->d;
    u64* a = k->d + (size_t)nq * N;
    Span sa = span_s(a, 0, nq, nq, 0, e->Lp1);
    hipLaunchKernelGGL(k_sample_uniform, dim3((N / 8 + 255) / 256, nq), dim3(256), 0, e->stream, sa, e->ck, derive(sk->keyseed, 2), e->q, e->logN, e->Lp1);
    Tmp et(e, (size_t)nq * N);
    sample_small_ntt(e, et.p, nq, derive(sk->keyseed, 3), 1);
    hipLaunchKernelGGL(k_key_combine, dim3(N / 256, nq), dim3(256), 0, e->stream, a, sk->d, et.p, (const u64*)nullptr, (const u64*)nullptr, 0, 0, b, e->q, e->qinv, e->logN);
    HIPC(hipGetLastError());
    *out = k;
    API_END
}

// Switching key s' -> s: s = the target secret's residues `starget` (every limb
// of Q u P), randomness from `keyseed`.
static aesfhe_key* make_ksk_t(aesfhe_engine* e, const u64* starget, u64 keyseed, const u64* sprime, int kind,
                              u64 g, u64 salt) {
    const int N = e->N, np = e->np;
    aesfhe_key* k = key_new(e, kind, (size_t)e->dnum * 2 * np * N);
    k->galois = g;
    k->keyseed = keyseed;
    k->ndig = e->dnum;
    u64 base = derive(derive(keyseed, 4 + (u64)kind), g);
    if (salt) base = derive(base, salt);
    Tmp et(e, (size_t)np * N);
    for (int d = 0; d < e->dnum; d++) {
        u64* kb = k->d + ((size_t)d * 2 + 0) * np * N;
        u64* ka = k->d + ((size_t)d * 2 + 1) * np * N;
        Span sa = span_s(ka, 0, np, e->Lp1, 0, e->Lp1);
        hipLaunchKernelGGL(k_sample_uniform, dim3((N / 8 + 255) / 256, np), dim3(256), 0, e->stream, sa, e->ck, derive(base, 2 * (u64)d), e->q, e->logN, e->Lp1);
        sample_small_ntt(e, et.p, np, derive(base, 2 * (u64)d + 1), 1);
        int lo = d * e->A, hi = std::min(lo + e->A, e->Lp1);
        hipLaunchKernelGGL(k_key_combine, dim3(N / 256, np), dim3(256), 0, e->stream, (const u64*)ka, starget, et.p, sprime, e->pmod, lo, hi, kb, e->q, e->qinv, e->logN);
    }
    HIPC(hipGetLastError());
    return k;
}
static aesfhe_key* make_ksk(aesfhe_engine* e, const aesfhe_key* sk, const u64* sprime, int kind, u64 g,
                            u64 salt = 0) {
    return make_ksk_t(e, sk->d, sk->keyseed, sprime, kind, g, salt);
}

extern "C" int aesfhe_key_relin(aesfhe_engine* e, const aesfhe_key* sk, aesfhe_key** out) {
    API_BEGIN
    if (!sk || sk->kind != 0) throw_err(AESFHE_EARG, "relinearization key needs a secret key");
    Tmp s2(e, (size_t)e->np * e->N);
    hipLaunchKernelGGL(k_square, dim3(e->N / 256, e->np), dim3(256), 0, e->stream, sk->d, s2.p, e->q, e->qinv, e->logN);
    *out = make_ksk(e, sk, s2.p, 2, 0);
    API_END
}

extern "C" int aesfhe_key_galois(aesfhe_engine* e, const aesfhe_key* sk, uint64_t g, aesfhe_key** out) {
    API_BEGIN
    if (!sk || sk->kind != 0) throw_err(AESFHE_EARG, "galois key needs a secret key");
    if (!(g & 1) || g >= 2ULL * e->N) throw_err(AESFHE_EARG, "bad galois element");
    Tmp sg(e, (size_t)e->np * e->N);
    Span src = span_s(sk->d, 0, e->np, e->Lp1, 0, e->Lp1), dst = span_s(sg.p, 0, e->np, e->Lp1, 0, e->Lp1);
    hipLaunchKernelGGL(k_galois, dim3(e->N / 256, e->np), dim3(256), 0, e->stream, src, dst, (u64)g, e->logN, e->Lp1);
    *out = make_ksk(e, sk, sg.p, 3, g);
    API_END
}

// Hoisted rotation key for galois element g (kind 5): switches s -> sigma_g^{-1}(s), so that
// rotate = sigma_g o keyswitch and the ModUp of c1 is shared by every key of one input
// (aesfhe_rotate_hoisted).
extern "C" int aesfhe_key_galois_hoisted(aesfhe_engine* e, const aesfhe_key* sk, uint64_t g, aesfhe_key** out) {
    API_BEGIN
    if (!sk || sk->kind != 0) throw_err(AESFHE_EARG, "galois key needs a secret key");
    if (!(g & 1) || g >= 2ULL * e->N) throw_err(AESFHE_EARG, "bad galois element");
    const u64 M = 2ULL * e->N;
    u64 ginv = 1;  // g^{-1} mod 2N = g^(ord(g) - 1): walk the powers of g
    for (u64 x = 1;; x = x * g % M)
        if (x * g % M == 1) { ginv = x; break; }
    Tmp st(e, (size_t)e->np * e->N);
    Span src = span_s(sk->d, 0, e->np, e->Lp1, 0, e->Lp1), dst = span_s(st.p, 0, e->np, e->Lp1, 0, e->Lp1);
    hipLaunchKernelGGL(k_galois, dim3(e->N / 256, e->np), dim3(256), 0, e->stream, src, dst, ginv, e->logN, e->Lp1);
    *out = make_ksk_t(e, st.p, sk->keyseed, sk->d, 5, g, 0x4015);
    API_END
}

// Sparse ternary secret with exactly hw nonzero coefficients (bootstrapping's ephemeral secret):
// key = derive(derive(seed_e, seed), 9); partial Fisher-Yates over 0..N-1: position i swaps with
// i + rnd(K, key, i) mod (N - i), the coefficient there is -1 if rnd(K, key, N + i) is odd else +1.
extern "C" int aesfhe_key_secret_sparse(aesfhe_engine* e, uint64_t seed, int32_t hw, aesfhe_key** out) {
    API_BEGIN
    const int N = e->N;
    if (hw < 1 || hw > N) throw_err(AESFHE_EARG, "sparse secret weight must be in [1, N]");
    aesfhe_key* k = key_new(e, 0, (size_t)e->np * N);
    k->keyseed = derive(e->seed, seed);
    const u64 key = derive(k->keyseed, 9);
    std::vector<int> idx(N);
    for (int i = 0; i < N; i++) idx[i] = i;
    std::vector<int64_t> co(N, 0);
    for (int i = 0; i < hw; i++) {
        const int j = i + (int)(rnd(e->ck, key, (u64)i) % (u64)(N - i));
        std::swap(idx[i], idx[j]);
        co[idx[i]] = (rnd(e->ck, key, (u64)N + i) & 1) ? -1 : 1;
    }
    Tmp dco(e, N);
    HIPC(hipMemcpyAsync(dco.p, co.data(), (size_t)N * 8, hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_coeffs_res, dim3(N / 256, e->np, 1), dim3(256), 0, e->stream, (const i64*)dco.p, k->d, e->np, e->q, e->logN);
    Span s = span_s(k->d, 0, e->np, e->Lp1, 0, e->Lp1);
    s.pstride = (long)e->np * N;
    ntt(e, s, s, e->np, false);
    HIPC(hipStreamSynchronize(e->stream));
    *out = k;
    API_END
}

// Switching key from secret sk_from to sk_to (a galois-kind key with element 1: aesfhe_galois
// applies it as a plain key switch).
extern "C" int aesfhe_key_switch(aesfhe_engine* e, const aesfhe_key* sk_from, const aesfhe_key* sk_to, aesfhe_key** out) {
    API_BEGIN
    if (!sk_from || !sk_to || sk_from->kind != 0 || sk_to->kind != 0) throw_err(AESFHE_EARG, "switching key needs two secret keys");
    *out = make_ksk(e, sk_to, sk_from->d, 3, 1, sk_from->keyseed | 1);
    API_END
}

// -----------------------------------------------------------------------------------------------
// ciphertext management
extern "C" void aesfhe_ct_free(aesfhe_ct* c) {
    if (!c) return;
    aesfhe_engine* e = c->eng;
    e->pool.put(c->d, c->bytes);
    delete c;
    engine_unref(e);
}
extern "C" int aesfhe_ct_info(const aesfhe_ct* c, int32_t info[4]) {
    info[0] = c->B;
    info[1] = c->np;
    info[2] = c->level;
    info[3] = c->is_zero;
    return 0;
}
extern "C" int aesfhe_ct_export(aesfhe_engine* e, const aesfhe_ct* c, uint64_t* out) {
    API_BEGIN
    HIPC(hipMemcpyAsync(out, c->d, c->bytes, hipMemcpyDeviceToHost, e->stream));
    HIPC(hipStreamSynchronize(e->stream));
    API_END
}
extern "C" int aesfhe_ct_import(aesfhe_engine* e, const uint64_t* in, int32_t B, int32_t np,
                                int32_t level, aesfhe_ct** out) {
    API_BEGIN
    if (B < 1 || np < 1 || np > 3 || level < 0 || level > e->L) throw_err(AESFHE_EARG, "bad shape");
    aesfhe_ct* c = ct_new(e, B, np, level);
    HIPC(hipMemcpyAsync(c->d, in, c->bytes, hipMemcpyHostToDevice, e->stream));
    HIPC(hipStreamSynchronize(e->stream));
    *out = c;
    API_END
}
// Device-resident transfer (the multi-GPU scatter/gather, parallel.py): residues of batch
// elements [start, start + count) to / from a caller-owned device buffer of this engine's device
// (a torch tensor that torch.distributed hands to RCCL), no host staging.  Both synchronise the
// engine stream, so the buffer is complete (export) / reusable (import) on return.
extern "C" int aesfhe_ct_export_device(aesfhe_engine* e, const aesfhe_ct* c, int32_t start, int32_t count, void* dst) {
    API_BEGIN
    if (!c || !dst || start < 0 || count < 1 || start + count > c->B) throw_err(AESFHE_EARG, "bad export range");
    const size_t per = c->bytes / c->B;
    HIPC(hipMemcpyAsync(dst, (const char*)c->d + per * start, per * count, hipMemcpyDeviceToDevice, e->stream));
    HIPC(hipStreamSynchronize(e->stream));
    API_END
}
extern "C" int aesfhe_ct_import_device(aesfhe_engine* e, const void* src, int32_t B, int32_t np, int32_t level,
                                       aesfhe_ct** out) {
    API_BEGIN
    if (!src || B < 1 || np < 1 || np > 3 || level < 0 || level > e->L) throw_err(AESFHE_EARG, "bad shape");
    aesfhe_ct* c = ct_new(e, B, np, level);
    HIPC(hipMemcpyAsync(c->d, src, c->bytes, hipMemcpyDeviceToDevice, e->stream));
    HIPC(hipStreamSynchronize(e->stream));
    *out = c;
    API_END
}

// Key serialisation (keyio.py): words of each kind -- 0 secret np*N, 1 public 2(L+1)N,
// 2/3/5 switching keys dnum*2*np*N.
static size_t key_words(const aesfhe_engine* e, int kind) {
    switch (kind) {
        case 0: return (size_t)e->np * e->N;
        case 1: return (size_t)2 * e->Lp1 * e->N;
        case 2: case 3: case 5: return (size_t)e->dnum * 2 * e->np * e->N;
        default: return 0;
    }
}
extern "C" int aesfhe_key_export(aesfhe_engine* e, const aesfhe_key* k, int32_t* kind, uint64_t* galois,
                                 uint64_t* keyseed, int64_t* words, uint64_t* out) {
    API_BEGIN
    if (!k) throw_err(AESFHE_EARG, "null key");
    *kind = k->kind;
    *galois = k->galois;
    *keyseed = k->keyseed;
    *words = (int64_t)(k->bytes / 8);
    if (out) {
        HIPC(hipMemcpyAsync(out, k->d, k->bytes, hipMemcpyDeviceToHost, e->stream));
        HIPC(hipStreamSynchronize(e->stream));
    }
    API_END
}
extern "C" int aesfhe_key_import(aesfhe_engine* e, int32_t kind, uint64_t galois, uint64_t keyseed,
                                 const uint64_t* in, int64_t words, aesfhe_key** out) {
    API_BEGIN
    size_t want = key_words(e, kind);
    if (!in || !want) throw_err(AESFHE_EARG, "unknown key kind %d", kind);
    int ndig = 0;
    if (kind == 2 || kind == 3 || kind == 5) {  // switching keys: dnum digits, or a trimmed key's first ones
        const size_t dw = (size_t)2 * e->np * e->N;
        if (words > 0 && (size_t)words % dw == 0 && (size_t)words / dw >= 1 && (size_t)words / dw <= (size_t)e->dnum)
            want = (size_t)words, ndig = (int)((size_t)words / dw);
    }
    if ((size_t)words != want) throw_err(AESFHE_EARG, "key of kind %d needs %zu words, got %lld", kind, want, (long long)words);
    aesfhe_key* k = key_new(e, kind, want);
    k->galois = galois;
    k->keyseed = keyseed;
    k->ndig = ndig;
    HIPC(hipMemcpyAsync(k->d, in, want * 8, hipMemcpyHostToDevice, e->stream));
    HIPC(hipStreamSynchronize(e->stream));
    *out = k;
    API_END
}
// Drop a switching key's digits beyond those a key switch at level <= max_level reads (include/
// aesfhe.h): digit d of a key is generated from its own random streams, so the first ones are
// word for word the full key's and every switch at those levels is unchanged.
extern "C" int aesfhe_key_trim(aesfhe_engine* e, aesfhe_key* k, int32_t max_level) {
    API_BEGIN
    if (!k || k->ndig < 1) throw_err(AESFHE_EARG, "only switching keys (relinearization, galois, hoisted rotation) can be trimmed");
    if (max_level < 0 || max_level > e->L) throw_err(AESFHE_EARG, "bad level %d", max_level);
    const int nd = (max_level + 1 + e->A - 1) / e->A;  // ks_beta(e, max_level)
    if (nd < k->ndig) {
        const size_t bytes = (size_t)nd * 2 * e->np * e->N * 8;
        u64* d = (u64*)pool_get(e, bytes);
        HIPC(hipMemcpyAsync(d, k->d, bytes, hipMemcpyDeviceToDevice, e->stream));
        e->pool.put(k->d, k->bytes);  // stream-ordered: reused only by later work
        k->d = d;
        k->bytes = bytes;
        k->ndig = nd;
    }
    API_END
}
extern "C" int aesfhe_ct_copy(aesfhe_engine* e, const aesfhe_ct* c, aesfhe_ct** out) {
    API_BEGIN
    aesfhe_ct* r = ct_new(e, c->B, c->np, c->level);
    HIPC(hipMemcpyAsync(r->d, c->d, c->bytes, hipMemcpyDeviceToDevice, e->stream));
    r->is_zero = c->is_zero;
    *out = r;
    API_END
}
extern "C" int aesfhe_ct_slice(aesfhe_engine* e, const aesfhe_ct* c, int32_t start, int32_t count, aesfhe_ct** out) {
    API_BEGIN
    if (start < 0 || count < 1 || start + count > c->B) throw_err(AESFHE_EARG, "bad slice");
    aesfhe_ct* r = ct_new(e, count, c->np, c->level);
    size_t per = c->bytes / c->B;
    HIPC(hipMemcpyAsync(r->d, (char*)c->d + per * start, per * count, hipMemcpyDeviceToDevice, e->stream));
    r->is_zero = c->is_zero;
    *out = r;
    API_END
}
extern "C" int aesfhe_ct_concat(aesfhe_engine* e, const aesfhe_ct* const* parts, int32_t n, aesfhe_ct** out) {
    API_BEGIN
    if (n < 1) throw_err(AESFHE_EARG, "empty concat");
    int B = 0, allz = 1;
    for (int i = 0; i < n; i++) {
        if (parts[i]->level != parts[0]->level || parts[i]->np != parts[0]->np)
            throw_err(AESFHE_EARG, "concat parts differ in level/npoly");
        B += parts[i]->B;
        allz &= parts[i]->is_zero;
    }
    aesfhe_ct* r = ct_new(e, B, parts[0]->np, parts[0]->level);
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        HIPC(hipMemcpyAsync((char*)r->d + off, parts[i]->d, parts[i]->bytes, hipMemcpyDeviceToDevice, e->stream));
        off += parts[i]->bytes;
    }
    r->is_zero = allz;
    *out = r;
    API_END
}
extern "C" int aesfhe_ct_gather(aesfhe_engine* e, const aesfhe_ct* c, const int32_t* idx, int32_t n, aesfhe_ct** out) {
    API_BEGIN
    if (n < 1 || !idx) throw_err(AESFHE_EARG, "empty gather");
    for (int b = 0; b < n; b++)
        if (idx[b] < 0 || idx[b] >= c->B) throw_err(AESFHE_EARG, "gather index out of range");
    aesfhe_ct* r = ct_new(e, n, c->np, c->level);
    const long per = (long)(c->bytes / c->B / 8);  // np * (level + 1) * N words
    const int* di = upload_small(e, (const int*)idx, (size_t)n);
    const long blocks = std::min<long>(per / 512, 256);
    {
        ProfScope ps(e, FAM_EW, 2.0 * 8.0 * per * n, "gather");
        hipLaunchKernelGGL(k_gather_batch, dim3((unsigned)std::max<long>(blocks, 1), n), dim3(256), 0, e->stream,
                           (const u64*)c->d, r->d, di, per);
    }
    r->is_zero = c->is_zero;
    *out = r;
    API_END
}
extern "C" int aesfhe_ct_zero(aesfhe_engine* e, int32_t B, int32_t level, aesfhe_ct** out) {
    API_BEGIN
    if (B < 1 || level < 0 || level > e->L) throw_err(AESFHE_EARG, "bad zero shape");
    *out = ct_zero_new(e, B, 2, level);
    API_END
}

extern "C" int aesfhe_pt_create(aesfhe_engine* e, const int64_t* co, int32_t level, aesfhe_pt** out) {
    API_BEGIN
    if (level < 0 || level > e->L) throw_err(AESFHE_EARG, "bad plaintext level");
    const int N = e->N, nl = level + 1;
    auto* p = new aesfhe_pt;
    p->eng = e;
    e->refs++;
    p->level = level;
    p->bytes = (size_t)nl * N * 8;
    p->d = (u64*)pool_get(e, p->bytes);
    Tmp dco(e, N);
    HIPC(hipMemcpyAsync(dco.p, co, (size_t)N * 8, hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_coeffs_res, dim3(N / 256, nl, 1), dim3(256), 0, e->stream, (const i64*)dco.p, p->d, nl, e->q, e->logN);
    Span s = span_s(p->d, 0, nl, nl, 0, e->Lp1);
    ntt(e, s, s, nl, false);
    // the host buffer `co` may be reused by the caller once we return
    HIPC(hipStreamSynchronize(e->stream));
    *out = p;
    API_END
}
extern "C" int aesfhe_pt_create_ext(aesfhe_engine* e, const int64_t* co, int32_t level, aesfhe_pt** out) {
    API_BEGIN
    if (level < 0 || level > e->L) throw_err(AESFHE_EARG, "bad plaintext level");
    const int N = e->N, nl = level + 1, ne = nl + e->K;
    auto* p = new aesfhe_pt;
    p->eng = e;
    e->refs++;
    p->level = level;
    p->ext = 1;
    p->bytes = (size_t)ne * N * 8;
    p->d = (u64*)pool_get(e, p->bytes);
    Tmp dco(e, N);
    HIPC(hipMemcpyAsync(dco.p, co, (size_t)N * 8, hipMemcpyHostToDevice, e->stream));
    hipLaunchKernelGGL(k_coeffs_res, dim3(N / 256, nl, 1), dim3(256), 0, e->stream, (const i64*)dco.p, p->d, nl, e->q, e->logN);
    hipLaunchKernelGGL(k_coeffs_res, dim3(N / 256, e->K, 1), dim3(256), 0, e->stream, (const i64*)dco.p, p->d + (long)nl * N, e->K, e->q + e->Lp1, e->logN);
    Span s = span_s(p->d, 0, ne, nl, 0, e->Lp1);
    ntt(e, s, s, ne, false);
    HIPC(hipStreamSynchronize(e->stream));
    *out = p;
    API_END
}
extern "C" void aesfhe_pt_free(aesfhe_pt* p) {
    if (!p) return;
    aesfhe_engine* e = p->eng;
    e->pool.put(p->d, p->bytes);
    delete p;
    engine_unref(e);
}

// -----------------------------------------------------------------------------------------------
// encryption / decryption
// encryption of B coefficient vectors (int64, B x N) held on the host (aesfhe_encrypt) or on the
// device (aesfhe_encrypt_device)
static aesfhe_ct* encrypt_coeffs(aesfhe_engine* e, const aesfhe_key* key, const int64_t* co, int B, int level,
                                 uint64_t nonce, bool host) {
    if (!key || (key->kind != 0 && key->kind != 1)) throw_err(AESFHE_EARG, "encryption key must be pk or sk");
    if (level < 0 || level > e->L || B < 1) throw_err(AESFHE_EARG, "bad level/batch");
    const int N = e->N, nl = level + 1;
    const long step = (long)nl * N;
    aesfhe_ct* c = ct_new(e, B, 2, level);
    Tmp vem(e, (size_t)B * 4 * step);
    std::unique_ptr<Tmp> hco;
    const u64* dcop = (const u64*)co;
    if (host) {
        hco.reset(new Tmp(e, (size_t)B * N));
        HIPC(hipMemcpyAsync(hco->p, co, (size_t)B * N * 8, hipMemcpyHostToDevice, e->stream));
        dcop = hco->p;
    }
    const u64 base = derive(derive(e->seed, 0xE0CULL), nonce);
    std::vector<u64> k0s(B);
    for (int b = 0; b < B; b++) {
        u64 k0 = derive(base, 3 * (u64)b), k1 = derive(base, 3 * (u64)b + 1), k2 = derive(base, 3 * (u64)b + 2);
        k0s[b] = k0;
        u64* vb = vem.p + (size_t)b * 4 * step;
        Span sv = span_s(vb, 0, nl, nl, 0, e->Lp1), se0 = span_s(vb + step, 0, nl, nl, 0, e->Lp1), se1 = span_s(vb + 2 * step, 0, nl, nl, 0, e->Lp1);
        if (key->kind == 1)
            hipLaunchKernelGGL(k_sample_small, dim3((N / 8 + 255) / 256), dim3(256), 0, e->stream, sv, e->ck, k0, 0, e->q, e->logN, e->Lp1, nl);
        hipLaunchKernelGGL(k_sample_small, dim3((N / 8 + 255) / 256), dim3(256), 0, e->stream, se0, e->ck, k1, 1, e->q, e->logN, e->Lp1, nl);
        if (key->kind == 1)
            hipLaunchKernelGGL(k_sample_small, dim3((N / 8 + 255) / 256), dim3(256), 0, e->stream, se1, e->ck, k2, 1, e->q, e->logN, e->Lp1, nl);
        hipLaunchKernelGGL(k_coeffs_res, dim3(N / 256, nl, 1), dim3(256), 0, e->stream, (const i64*)(dcop + (size_t)b * N), vb + 3 * step, nl, e->q, e->logN);
    }
    // NTT everything: B * 4 groups of nl limbs (pid = limb index)
    Span all = span_s(vem.p, step, nl, nl, 0, e->Lp1);
    ntt(e, all, all, B * 4 * nl, false);
    if (key->kind == 1) {
        const u64* pk0 = key->d;
        const u64* pk1 = key->d + (size_t)e->Lp1 * N;
        hipLaunchKernelGGL(k_enc_pk, dim3(N / 256, nl, B), dim3(256), 0, e->stream, (const u64*)vem.p, pk0, pk1, c->d, nl, e->q, e->qinv, e->logN);
    } else {
        u64* dk = upload_small(e, k0s.data(), k0s.size());
        hipLaunchKernelGGL(k_enc_sk, dim3((N / 8 + 255) / 256, nl, B), dim3(256), 0, e->stream, (const u64*)vem.p, (const u64*)key->d, c->d, nl, e->q, e->qinv, e->ck, (const u64*)dk, e->logN);
    }
    HIPC(hipGetLastError());
    if (host) HIPC(hipStreamSynchronize(e->stream));  // host coefficient buffer may be reused by caller
    return c;
}

extern "C" int aesfhe_encrypt(aesfhe_engine* e, const aesfhe_key* key, const int64_t* co, int32_t B,
                              int32_t level, uint64_t nonce, aesfhe_ct** out) {
    API_BEGIN
    *out = encrypt_coeffs(e, key, co, B, level, nonce, true);
    API_END
}

// Decrypt: m = c0 + c1 s (+ c2 s^2) on limb 0, and on limb 1 too when the
// ciphertext has it; the two residues are CRT-combined and centred mod q0 q1 (a level-0
// ciphertext: mod q0), so the plaintext capacity is q0 q1 / (2 Delta) instead of q0 / (2 Delta)
// (= 32 at a 44-bit scale).  Coefficients beyond +-(2^63 - 1) saturate.
static void decrypt_limbs(aesfhe_engine* e, const aesfhe_key* sk, const aesfhe_ct* c, u64* t, int nl);
extern "C" int aesfhe_decrypt(aesfhe_engine* e, const aesfhe_key* sk, const aesfhe_ct* c, int64_t* out) {
    API_BEGIN
    if (!sk || sk->kind != 0) throw_err(AESFHE_EARG, "decryption needs the secret key");
    const int N = e->N;
    const int nl = c->level >= 1 ? 2 : 1;
    Tmp t(e, (size_t)nl * c->B * N);
    decrypt_limbs(e, sk, c, t.p, nl);
    std::vector<u64> h((size_t)nl * c->B * N);
    HIPC(hipMemcpyAsync(h.data(), t.p, h.size() * 8, hipMemcpyDeviceToHost, e->stream));
    HIPC(hipStreamSynchronize(e->stream));
    const u64 q0 = e->chain.q[0];
    const size_t cnt = (size_t)c->B * N;
    if (nl == 1) {
        for (size_t i = 0; i < cnt; i++) out[i] = h[i] > q0 / 2 ? (int64_t)h[i] - (int64_t)q0 : (int64_t)h[i];
    } else {
        const u64 q1 = e->chain.q[1], q0inv = h_invmod(q0 % q1, q1);
        const u128 Q = (u128)q0 * q1;
        for (size_t i = 0; i < cnt; i++) {
            const u64 r0 = h[i], r1 = h[cnt + i];
            const u64 d = h_mulmod(h_submod(r1, r0 % q1, q1), q0inv, q1);
            const u128 x = (u128)r0 + (u128)q0 * d;  // in [0, q0 q1)
            if (x > Q / 2) {
                const u128 m = Q - x;
                out[i] = m > (u128)INT64_MAX ? -INT64_MAX : -(int64_t)m;
            } else {
                out[i] = x > (u128)INT64_MAX ? INT64_MAX : (int64_t)x;
            }
        }
    }
    API_END
}

// -----------------------------------------------------------------------------------------------
// device-resident client path: the codec of aesfhe_encode / aesfhe_decode and
// the encryption / decryption on device buffers, stream-ordered on the engine's stream.
static CodecTabs codec_tabs(aesfhe_engine* e) {
    const int n = e->N / 2;
    const long M = 2L * e->N;
    if (!e->ckre) {
        Codec c(e->logN);  // host twiddles (libm cos / sin): the device tables are the same doubles
        HIPC(hipMalloc(&e->ckre, (M + 1) * sizeof(double)));
        HIPC(hipMalloc(&e->ckim, (M + 1) * sizeof(double)));
        HIPC(hipMalloc(&e->crot, n * sizeof(long)));
        HIPC(hipMemcpy(e->ckre, c.kre.data(), (M + 1) * sizeof(double), hipMemcpyHostToDevice));
        HIPC(hipMemcpy(e->ckim, c.kim.data(), (M + 1) * sizeof(double), hipMemcpyHostToDevice));
        HIPC(hipMemcpy(e->crot, c.rot.data(), n * sizeof(long), hipMemcpyHostToDevice));
    }
    return CodecTabs{e->ckre, e->ckim, e->crot, M, n, e->logN - 1};
}

static unsigned blocks_for(long count) { return (unsigned)((count + 255) / 256); }

extern "C" int aesfhe_encode_device(aesfhe_engine* e, const double* re, const double* im, int32_t B, int64_t n_slots,
                                    int64_t stride, double scale, int64_t* co) {
    API_BEGIN
    const CodecTabs T = codec_tabs(e);
    const int n = T.n;
    if (B < 1 || n_slots < 0 || n_slots > n || stride < n_slots || !co) throw_err(AESFHE_EARG, "bad encode shape");
    Tmp a(e, (size_t)B * 2 * n), b(e, (size_t)B * 2 * n);
    double *ar = (double*)a.p, *ai = ar + (size_t)B * n, *br = (double*)b.p, *bi = br + (size_t)B * n;
    const long tot = (long)B * n, bfly = (long)B * (n / 2);
    hipLaunchKernelGGL(k_sfft_load, dim3(blocks_for(tot)), dim3(256), 0, e->stream, re, im, (long)stride, (long)n_slots, ar, ai, n, B);
    for (int len = n; len >= 2; len >>= 1)  // len = 1 butterflies are identities (lenh = 0)
        hipLaunchKernelGGL(k_sfft_inv_stage, dim3(blocks_for(bfly)), dim3(256), 0, e->stream, ar, ai, T, len, B);
    hipLaunchKernelGGL(k_sfft_bitrev, dim3(blocks_for(tot)), dim3(256), 0, e->stream, (const double*)ar, (const double*)ai, br, bi, n, T.logn, B);
    const unsigned nb = blocks_for(tot);
    if (e->cflags_n < nb) {
        if (e->cflags) HIPC(hipFree(e->cflags));
        HIPC(hipMalloc(&e->cflags, nb * sizeof(int)));
        e->cflags_n = nb;
    }
    hipLaunchKernelGGL(k_sfft_round, dim3(nb), dim3(256), 0, e->stream, (const double*)br, (const double*)bi, n, B, scale, co, e->cflags);
    HIPC(hipGetLastError());
    std::vector<int> fl(nb);
    HIPC(hipMemcpyAsync(fl.data(), e->cflags, nb * sizeof(int), hipMemcpyDeviceToHost, e->stream));
    HIPC(hipStreamSynchronize(e->stream));
    for (int f : fl)
        if (f) throw_err(AESFHE_EARG, "encoded coefficient overflows int64 (scale too large?)");
    API_END
}

extern "C" int aesfhe_decode_device(aesfhe_engine* e, const int64_t* co, int32_t B, double scale, double* re, double* im) {
    API_BEGIN
    const CodecTabs T = codec_tabs(e);
    const int n = T.n;
    if (B < 1 || !co || !re || !im) throw_err(AESFHE_EARG, "bad decode arguments");
    const long tot = (long)B * n, bfly = (long)B * (n / 2);
    hipLaunchKernelGGL(k_sfft_unround, dim3(blocks_for(tot)), dim3(256), 0, e->stream, co, n, T.logn, B, scale, re, im);
    for (int len = 2; len <= n; len <<= 1)
        hipLaunchKernelGGL(k_sfft_fwd_stage, dim3(blocks_for(bfly)), dim3(256), 0, e->stream, re, im, T, len, B);
    HIPC(hipGetLastError());
    API_END
}

extern "C" int aesfhe_encrypt_device(aesfhe_engine* e, const aesfhe_key* key, const int64_t* co, int32_t B,
                                     int32_t level, uint64_t nonce, aesfhe_ct** out) {
    API_BEGIN
    if (!co) throw_err(AESFHE_EARG, "null coefficient buffer");
    *out = encrypt_coeffs(e, key, co, B, level, nonce, false);
    API_END
}

// residues of limb 0 (and 1) of c + c1 s (+ c2 s^2), coefficient domain: t[i * B * N ...]
static void decrypt_limbs(aesfhe_engine* e, const aesfhe_key* sk, const aesfhe_ct* c, u64* t, int nl) {
    const int N = e->N;
    View v = view_of(c);
    for (int i = 0; i < nl; i++) {
        u64* ti = t + (size_t)i * c->B * N;
        hipLaunchKernelGGL(k_dec_limb0, dim3(N / 256, 1, c->B), dim3(256), 0, e->stream, v.d + (size_t)i * N, v.bs, v.ps, c->np,
                           (const u64*)sk->d + (size_t)i * N, ti, e->chain.q[i], 1.0 / (double)e->chain.q[i], e->logN);
        Span s = span_s(ti, N, 1, 1, i, e->Lp1);
        ntt(e, s, s, c->B, true);
    }
}

extern "C" int aesfhe_decrypt_device(aesfhe_engine* e, const aesfhe_key* sk, const aesfhe_ct* c, int64_t* co) {
    API_BEGIN
    if (!sk || sk->kind != 0) throw_err(AESFHE_EARG, "decryption needs the secret key");
    if (!co) throw_err(AESFHE_EARG, "null coefficient buffer");
    const int N = e->N, nl = c->level >= 1 ? 2 : 1;
    Tmp t(e, (size_t)nl * c->B * N);
    decrypt_limbs(e, sk, c, t.p, nl);
    const long cnt = (long)c->B * N;
    const u64 q0 = e->chain.q[0], q1 = nl == 2 ? e->chain.q[1] : 1;
    hipLaunchKernelGGL(k_dec_crt, dim3(blocks_for(cnt)), dim3(256), 0, e->stream, (const uint64_t*)t.p,
                       nl == 2 ? (const uint64_t*)t.p + cnt : (const uint64_t*)nullptr, cnt, q0, q1,
                       nl == 2 ? h_invmod(q0 % q1, q1) : 0, co);
    HIPC(hipGetLastError());
    API_END
}

// -----------------------------------------------------------------------------------------------
// core primitives
// rescale a view (level l >= 1) into a new ct at level l-1
// C != 1: rescale of C * in (the exact-scale level-down, level_down_view), the constant folded
// into the spread (top limb) and the finish (every kept limb) instead of a k_mul_const pass.
static void const_factors(aesfhe_engine* e, int64_t A, int64_t Bc, int nl, std::vector<u64>& f, std::vector<double>& ff);
// into: write the result into this caller-owned compact block (in.B x in.np polys at level l-1)
// instead of a new ciphertext (the return value is then nullptr).
static aesfhe_ct* rescale_view(aesfhe_engine* e, const View& in, int64_t C = 1, u64* into = nullptr) {
    const int N = e->N, l = in.level, P = in.B * in.np;
    const bool sc = C != 1;
    u64* df = nullptr;
    double* dff = nullptr;
    double* dff_c = nullptr;
    u64 ctop = 1;
    double ctopf = 0.0;
    if (sc) {
        std::vector<u64> f;
        std::vector<double> ff;
        const_factors(e, C, 0, l + 1, f, ff);
        ctop = f[2 * l];
        ctopf = ff[2 * l];
        df = upload_small(e, f.data(), f.size());
        dff = upload_small(e, ff.data(), ff.size());
        std::vector<double> fc(l);  // per-limb w/q of C (RowFin::cf)
        for (int i = 0; i < l; i++) fc[i] = ff[2 * i];
        dff_c = upload_small(e, fc.data(), fc.size());
    }
    aesfhe_ct* r = into ? nullptr : ct_new(e, in.B, in.np, l - 1);
    aesfhe_ct alias{e, in.B, in.np, l - 1, 0, into, 0};
    aesfhe_ct* o = into ? &alias : r;
    Tmp x(e, (size_t)P * N), t(e, (size_t)P * l * N);
    // INTT of limb l of every poly: source poly p of batch b at d + b*bs + p*ps + l*N
    // (expressed as a Span over the flattened polys; requires bs == np*ps, true for compact views)
    Span src = span_s((u64*)in.d + (long)l * N, in.ps, 1, 1, l, e->Lp1);
    Span dx = span_s(x.p, N, 1, 1, l, e->Lp1);
    if (in.bs != (long)in.np * in.ps && in.B > 1) throw_err(AESFHE_EARG, "rescale of non-compact view");
    ntt(e, src, dx, P, true);
    Span st = span_s(t.p, (long)l * N, l, l, 0, e->Lp1);
    if (fused_ntt(e) && in.np == 2 && !in.zero) {
        // the spread runs in the copy-in of t's column pass (k_nttf_fwd_cols_spread reads the
        // top limb x once per target limb: t is never written in coefficient form) and the finish
        // in the epilogue of t's row pass (the ModDown finish's RowFin with acc = the input,
        // D = q_l, optional level-down constant): t never reaches HBM in NTT form
        const int total = P * l;
        {
            ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_fwd_cols_spread");
            const SpreadSrc ss{(const u64*)x.p, (long)N, e->chain.q[l], ctop, ctopf};
            auto kern = N == 65536 ? (sc ? k_nttf_fwd_cols_spread<256, 2> : k_nttf_fwd_cols_spread<256, 1>)
                                   : (sc ? k_nttf_fwd_cols_spread<512, 2> : k_nttf_fwd_cols_spread<512, 1>);
            hipLaunchKernelGGL(kern, dim3(16, total), dim3(256), 0, e->stream, ss, st, e->tabs());
        }
        RowFin f{(const u64*)in.d, in.bs, in.ps, Opnd2{nullptr, 0, 0, 0}, o->d, 2L * l * N, (long)l * N,
                 e->rs_invf + (size_t)l * e->Lp1, l, sc ? (const double*)dff_c : nullptr};
        ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total * 3.0, "ntt_fwd_rows_fin");  // half an NTT + input read + output write
        if (N == 65536) hipLaunchKernelGGL((k_nttf_fwd_rows_t<true, 256>), dim3(16, total), dim3(256), 0, e->stream, st, e->tabs(), f);
        else hipLaunchKernelGGL((k_nttf_fwd_rows_t<true, 512>), dim3(32, total), dim3(256), 0, e->stream, st, e->tabs(), f);
        HIPC(hipGetLastError());
        return r;
    }
    if (sc) hipLaunchKernelGGL(k_rescale_spread<true>, dim3(N / 256, l, P), dim3(256), 0, e->stream, (const u64*)x.p, t.p, e->chain.q[l], e->q, e->qinv, e->rs_mod + (size_t)l * e->Lp1, l, e->logN, ctop, ctopf);
    else hipLaunchKernelGGL(k_rescale_spread<false>, dim3(N / 256, l, P), dim3(256), 0, e->stream, (const u64*)x.p, t.p, e->chain.q[l], e->q, e->qinv, e->rs_mod + (size_t)l * e->Lp1, l, e->logN, ctop, ctopf);
    ntt(e, st, st, P * l, false);
    Opnd c = opnd(in, in.B);
    if (sc) hipLaunchKernelGGL(k_rescale_finish<true>, dim3(N / 256, l, P), dim3(256), 0, e->stream, c, (const u64*)t.p, out_of(o), in.np, l, e->q, e->rs_inv + (size_t)l * e->Lp1, e->rs_invf + (size_t)l * e->Lp1, e->logN, (const u64*)df, (const double*)dff);
    else hipLaunchKernelGGL(k_rescale_finish<false>, dim3(N / 256, l, P), dim3(256), 0, e->stream, c, (const u64*)t.p, out_of(o), in.np, l, e->q, e->rs_inv + (size_t)l * e->Lp1, e->rs_invf + (size_t)l * e->Lp1, e->logN, (const u64*)nullptr, (const double*)nullptr);
    HIPC(hipGetLastError());
    return r;
}

// rescale of a compact buffer holding G groups of Bg batch elements (np polys, level l) into G
// new ciphertexts at level l-1 (one rescale pass for all groups)
static std::vector<aesfhe_ct*> rescale_groups(aesfhe_engine* e, const u64* d, int G, int Bg, int np, int l) {
    const int N = e->N, P = G * Bg * np;
    if (fused_ntt(e) && np == 2) {
        // the groups are one compact batch of G * Bg ciphertexts: the fused rescale (spread in the
        // column pass, finish in the row pass), then the output block split per group (no copies)
        const long ps = (long)(l + 1) * N;
        aesfhe_ct* r = rescale_view(e, View{d, G * Bg, np, l, ps, np * ps, false});
        return G == 1 ? std::vector<aesfhe_ct*>{r} : ct_split_batch(e, r, G);
    }
    std::vector<aesfhe_ct*> outs(G);
    for (int g = 0; g < G; g++) outs[g] = ct_new(e, Bg, np, l - 1);
    Tmp x(e, (size_t)P * N), t(e, (size_t)P * l * N);
    const long cps = (long)(l + 1) * N;
    Span src = span_s((u64*)d + (long)l * N, cps, 1, 1, l, e->Lp1);
    Span dx = span_s(x.p, N, 1, 1, l, e->Lp1);
    ntt(e, src, dx, P, true);
    hipLaunchKernelGGL(k_rescale_spread<false>, dim3(N / 256, l, P), dim3(256), 0, e->stream, (const u64*)x.p, t.p, e->chain.q[l], e->q, e->qinv, e->rs_mod + (size_t)l * e->Lp1, l, e->logN, (u64)1, 0.0);
    Span st = span_s(t.p, (long)l * N, l, l, 0, e->Lp1);
    ntt(e, st, st, P * l, false);
    std::vector<u64*> op(G);
    for (int g = 0; g < G; g++) op[g] = outs[g]->d;
    auto dop = upload_small(e, op.data(), op.size());
    hipLaunchKernelGGL(k_rescale_finish_g, dim3(N / 256, l, P), dim3(256), 0, e->stream, d, cps, (const u64*)t.p, (u64* const*)dop, (long)l * N, np, Bg, l, e->q, e->rs_inv + (size_t)l * e->Lp1, e->rs_invf + (size_t)l * e->Lp1, e->logN);
    HIPC(hipGetLastError());
    return outs;
}

// constant factor tables for A + B X^{N/2} over limbs 0..nl-1
static void const_factors(aesfhe_engine* e, int64_t A, int64_t Bc, int nl, std::vector<u64>& f, std::vector<double>& ff) {
    f.resize(2 * nl);
    ff.resize(2 * nl);
    for (int i = 0; i < nl; i++) {
        u64 q = e->chain.q[i];
        u64 a = h_smod(A, q), b = h_smod(Bc, q);
        u64 bi = h_mulmod(b, e->h_iroot[i], q);
        f[2 * i] = h_addmod(a, bi, q);
        f[2 * i + 1] = h_submod(a, bi, q);
        ff[2 * i] = (double)f[2 * i] / (double)q;
        ff[2 * i + 1] = (double)f[2 * i + 1] / (double)q;
    }
}

// out (compact ct at in.level) (+)= in * (A + B X^{N/2})
static void mul_const_into(aesfhe_engine* e, const View& in, int64_t A, int64_t Bc, aesfhe_ct* o, int acc) {
    const int nl = in.level + 1;
    std::vector<u64> f;
    std::vector<double> ff;
    const_factors(e, A, Bc, nl, f, ff);
    u64* df = upload_small(e, f.data(), f.size());
    double* dff = upload_small(e, ff.data(), ff.size());
    ProfScope ps(e, FAM_EW, 8.0 * e->N * nl * (double)o->B * in.np * (acc ? 3 : 2), "mul_const");
    hipLaunchKernelGGL(k_mul_const, ew_grid(e, nl, o->B * in.np), dim3(256), 0, e->stream, opnd(in, o->B), out_of(o), in.np, (const u64*)df, (const double*)dff, e->q, acc, e->logN);
    HIPC(hipGetLastError());
}

static View truncated(const View& v, int level) {
    View t = v;
    t.level = level;
    return t;
}

// exact-scale level-down constant from level `from` to `lt` < from
static int64_t level_down_const(const aesfhe_engine* e, int from, int lt) {
    return llround(e->chain.scale[lt] * (double)e->chain.q[lt + 1] / e->chain.scale[from]);
}

static aesfhe_ct* level_down_view(aesfhe_engine* e, const View& v, int lt) {
    if (lt == v.level) {
        aesfhe_ct* r = ct_new(e, v.B, v.np, v.level);
        if (v.zero) {
            HIPC(hipMemsetAsync(r->d, 0, r->bytes, e->stream));
            r->is_zero = 1;
        } else if (v.bs == (long)v.np * v.ps) {
            HIPC(hipMemcpyAsync(r->d, v.d, r->bytes, hipMemcpyDeviceToDevice, e->stream));
        } else {
            throw_err(AESFHE_EARG, "copy of non-compact view");
        }
        return r;
    }
    if (v.zero) return ct_zero_new(e, v.B, v.np, lt);
    View t = truncated(v, lt + 1);
    return rescale_view(e, t, level_down_const(e, v.level, lt));  // C folded into the rescale's spread + finish (no k_mul_const pass)
}

// owned-or-borrowed aligned operand
struct Aligned {
    aesfhe_ct* owned = nullptr;
    View v;
    ~Aligned() {
        if (owned) aesfhe_ct_free(owned);
    }
};

static void align_to(aesfhe_engine* e, const aesfhe_ct* c, int l, Aligned& a) {
    if (c->level == l) {
        a.v = view_of(c);
    } else {
        a.owned = level_down_view(e, view_of(c), l);
        a.v = view_of(a.owned);
    }
}

// c seen at level l <= c->level: its first l+1 limbs, no rescale (the scale stays D_level(c);
// callers compensate it in a constant)
static View trunc_view(const aesfhe_ct* c, int l) {
    View v = view_of(c);
    v.level = l;
    return v;
}

static void check_bcast(int a, int b) {
    if (a != b && a != 1 && b != 1) throw_err(AESFHE_EARG, "batch mismatch %d vs %d", a, b);
}
// aesfhe_mul / aesfhe_tensor: the smaller batch may be any power of two dividing the larger --
// element i of the result takes element i mod B_small of it (a B = 1 broadcast is the special
// case; the sliced AES state's batch-4 round keys against its 4 s + c batch order)
static void check_cyclic(int a, int b) {
    const int lo = std::min(a, b), hi = std::max(a, b);
    if (a != b && (lo < 1 || (lo & (lo - 1)) || hi % lo)) throw_err(AESFHE_EARG, "batch mismatch %d vs %d", a, b);
}

extern "C" int aesfhe_rescale(aesfhe_engine* e, const aesfhe_ct* c, aesfhe_ct** out) {
    API_BEGIN
    if (c->level < 1) throw_err(AESFHE_ELEVEL, "cannot rescale a level-0 ciphertext");
    if (c->is_zero) *out = ct_zero_new(e, c->B, c->np, c->level - 1);
    else *out = rescale_view(e, view_of(c));
    API_END
}

extern "C" int aesfhe_level_down(aesfhe_engine* e, const aesfhe_ct* c, int32_t lt, aesfhe_ct** out) {
    API_BEGIN
    if (lt < 0 || lt > c->level) throw_err(AESFHE_EARG, "level_down target %d not in [0,%d]", lt, c->level);
    *out = level_down_view(e, view_of(c), lt);
    API_END
}

static int addsub(aesfhe_engine* e, const aesfhe_ct* a, const aesfhe_ct* b, int sub, aesfhe_ct** out) {
    API_BEGIN
    check_bcast(a->B, b->B);
    int l = std::min(a->level, b->level);
    Aligned A, Bv;
    align_to(e, a, l, A);
    align_to(e, b, l, Bv);
    int B = std::max(a->B, b->B), np = std::max(a->np, b->np);
    aesfhe_ct* r = ct_new(e, B, np, l);
    ProfScope ps(e, FAM_EW, 24.0 * e->N * (l + 1) * (double)B * np, "add");
    hipLaunchKernelGGL(k_addsub, ew_grid(e, l + 1, B * np), dim3(256), 0, e->stream, opnd(A.v, B), opnd(Bv.v, B), out_of(r), np, e->q, sub, e->logN);
    HIPC(hipGetLastError());
    r->is_zero = a->is_zero && b->is_zero;
    *out = r;
    API_END
}
extern "C" int aesfhe_add(aesfhe_engine* e, const aesfhe_ct* a, const aesfhe_ct* b, aesfhe_ct** out) { return addsub(e, a, b, 0, out); }
extern "C" int aesfhe_sub(aesfhe_engine* e, const aesfhe_ct* a, const aesfhe_ct* b, aesfhe_ct** out) { return addsub(e, a, b, 1, out); }
extern "C" int aesfhe_negate(aesfhe_engine* e, const aesfhe_ct* a, aesfhe_ct** out) {
    API_BEGIN
    aesfhe_ct* r = ct_new(e, a->B, a->np, a->level);
    View z = view_of(a);
    z.zero = true;
    hipLaunchKernelGGL(k_addsub, ew_grid(e, a->level + 1, a->B * a->np), dim3(256), 0, e->stream, opnd(z, a->B), opnd(view_of(a), a->B), out_of(r), a->np, e->q, 1, e->logN);
    HIPC(hipGetLastError());
    r->is_zero = a->is_zero;
    *out = r;
    API_END
}

extern "C" int aesfhe_add_pt(aesfhe_engine* e, const aesfhe_ct* c, const aesfhe_pt* pt, aesfhe_ct** out) {
    API_BEGIN
    if (pt->level < c->level) throw_err(AESFHE_EARG, "plaintext level %d below ciphertext level %d", pt->level, c->level);
    aesfhe_ct* r = ct_new(e, c->B, c->np, c->level);
    hipLaunchKernelGGL(k_add_pt, ew_grid(e, c->level + 1, c->B * c->np), dim3(256), 0, e->stream, opnd(view_of(c), c->B), (const u64*)pt->d, out_of(r), c->np, e->q, e->logN);
    HIPC(hipGetLastError());
    *out = r;
    API_END
}

extern "C" int aesfhe_add_const(aesfhe_engine* e, const aesfhe_ct* c, double re, double im, aesfhe_ct** out) {
    API_BEGIN
    const double s = e->chain.scale[c->level];
    const int64_t A = llround(re * s), Bc = llround(im * s);
    std::vector<u64> f;
    std::vector<double> ff;
    const_factors(e, A, Bc, c->level + 1, f, ff);
    u64* df = upload_small(e, f.data(), f.size());
    aesfhe_ct* r = ct_new(e, c->B, c->np, c->level);
    hipLaunchKernelGGL(k_add_const, ew_grid(e, c->level + 1, c->B * c->np), dim3(256), 0, e->stream, opnd(view_of(c), c->B), out_of(r), c->np, (const u64*)df, e->q, e->logN);
    HIPC(hipGetLastError());
    r->is_zero = c->is_zero && A == 0 && Bc == 0;
    *out = r;
    API_END
}

extern "C" int aesfhe_mul_pt(aesfhe_engine* e, const aesfhe_ct* c, const aesfhe_pt* pt, aesfhe_ct** out) {
    API_BEGIN
    if (c->level < 1) throw_err(AESFHE_ELEVEL, "no level left for a plaintext multiplication");
    if (pt->level < c->level) throw_err(AESFHE_EARG, "plaintext level %d below ciphertext level %d", pt->level, c->level);
    if (c->is_zero) {
        *out = ct_zero_new(e, c->B, c->np, c->level - 1);
    } else {
        aesfhe_ct* t = ct_new(e, c->B, c->np, c->level);
        hipLaunchKernelGGL(k_mul_pt, ew_grid(e, c->level + 1, c->B * c->np), dim3(256), 0, e->stream, opnd(view_of(c), c->B), (const u64*)pt->d, out_of(t), c->np, e->q, e->qinv, e->logN);
        HIPC(hipGetLastError());
        *out = rescale_view(e, view_of(t));
        aesfhe_ct_free(t);
    }
    API_END
}

extern "C" int aesfhe_mul_const(aesfhe_engine* e, const aesfhe_ct* c, double re, double im, aesfhe_ct** out) {
    API_BEGIN
    if (c->level < 1) throw_err(AESFHE_ELEVEL, "no level left for a constant multiplication");
    double s = aesfhe_engine_mul_scale(e, c->level);
    int64_t A = llround(re * s), Bc = llround(im * s);
    if (c->is_zero || (A == 0 && Bc == 0)) {
        *out = ct_zero_new(e, c->B, c->np, c->level - 1);
    } else {
        aesfhe_ct* t = ct_new(e, c->B, c->np, c->level);
        mul_const_into(e, view_of(c), A, Bc, t, 0);
        *out = rescale_view(e, view_of(t));
        aesfhe_ct_free(t);
    }
    API_END
}

// ModRaise (bootstrapping): the level-0 content of ct (limb 0, mod q_0, centred) lifted to
// every limb of `level`.  The result encrypts t = m + q_0 I; its scale is the caller's business.
extern "C" int aesfhe_mod_raise(aesfhe_engine* e, const aesfhe_ct* c, int32_t level, aesfhe_ct** out) {
    API_BEGIN
    if (level < 0 || level > e->L) throw_err(AESFHE_EARG, "bad mod-raise level");
    const int N = e->N, P = c->B * c->np, nl = level + 1;
    aesfhe_ct* r = ct_new(e, c->B, c->np, level);
    if (c->is_zero) {
        HIPC(hipMemsetAsync(r->d, 0, r->bytes, e->stream));
        r->is_zero = 1;
    } else {
        Tmp x(e, (size_t)P * N);
        const View v = view_of(c);
        Span src = span_s((u64*)v.d, v.ps, 1, 1, 0, e->Lp1), dx = span_s(x.p, N, 1, 1, 0, e->Lp1);
        if (v.B > 1 && v.bs != (long)v.np * v.ps) throw_err(AESFHE_EARG, "mod-raise of non-compact view");
        ntt(e, src, dx, P, true);
        hipLaunchKernelGGL(k_lift0, dim3(N / 256, nl, P), dim3(256), 0, e->stream, (const u64*)x.p, r->d, nl, e->chain.q[0], e->q, e->logN);
        HIPC(hipGetLastError());
        Span so = span_s(r->d, (long)nl * N, nl, nl, 0, e->Lp1);
        ntt(e, so, so, P * nl, false);
    }
    *out = r;
    API_END
}

// Multiplication by X^{N/2} (sign +1) or -X^{N/2}: every slot times i / -i, exact, no level.
extern "C" int aesfhe_mul_i(aesfhe_engine* e, const aesfhe_ct* c, int32_t sign, aesfhe_ct** out) {
    API_BEGIN
    aesfhe_ct* r = ct_new(e, c->B, c->np, c->level);
    if (c->is_zero) {
        HIPC(hipMemsetAsync(r->d, 0, r->bytes, e->stream));
        r->is_zero = 1;
    } else {
        mul_const_into(e, view_of(c), 0, sign >= 0 ? 1 : -1, r, 0);
    }
    *out = r;
    API_END
}

// sum_i ct_i * pt_i, one rescale (the diagonal sums of homomorphic linear transforms); plaintexts
// must hold at least level l + 1 limbs, l = the lowest ciphertext level.
extern "C" int aesfhe_dot_pt(aesfhe_engine* e, const aesfhe_ct* const* cts, const aesfhe_pt* const* pts, int32_t n, aesfhe_ct** out) {
    API_BEGIN
    if (n < 1 || n > 256) throw_err(AESFHE_EARG, "dot_pt needs 1..256 terms");
    int l = cts[0]->level, B = 1, np = cts[0]->np;
    for (int i = 0; i < n; i++) {
        l = std::min(l, cts[i]->level);
        B = std::max(B, cts[i]->B);
        if (cts[i]->np != np) throw_err(AESFHE_EDEGREE, "dot_pt inputs should have the same number of polynomials");
    }
    for (int i = 0; i < n; i++) {
        if (cts[i]->B != B && cts[i]->B != 1) throw_err(AESFHE_EARG, "batch mismatch");
        if (pts[i]->level < l) throw_err(AESFHE_EARG, "plaintext level %d below ciphertext level %d", pts[i]->level, l);
    }
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a plaintext dot product");
    const int nl = l + 1;
    std::vector<std::unique_ptr<Aligned>> al;
    std::vector<const u64*> pc, pp;
    std::vector<long> sb;
    for (int i = 0; i < n; i++) {
        if (cts[i]->is_zero) continue;
        al.emplace_back(new Aligned());
        align_to(e, cts[i], l, *al.back());
        const View& v = al.back()->v;
        if (v.ps != (long)nl * e->N) throw_err(AESFHE_EARG, "dot_pt: non-compact view");
        pc.push_back(v.d);
        sb.push_back(v.B == 1 && B > 1 ? 0 : v.bs);
        pp.push_back(pts[i]->d);
    }
    if (pc.empty()) {
        *out = ct_zero_new(e, B, np, l - 1);
    } else {
        aesfhe_ct* acc = ct_new(e, B, np, l);
        auto dpc = upload_small(e, pc.data(), pc.size());
        auto dpp = upload_small(e, pp.data(), pp.size());
        auto dsb = upload_small(e, sb.data(), sb.size());
        {
            ProfScope ps_(e, FAM_EW, 8.0 * e->N * nl * (double)B * np * (pc.size() + 1), "dot_pt");
            hipLaunchKernelGGL(k_dot_pt, ew_grid(e, nl, B * np), dim3(256), 0, e->stream, (const u64* const*)dpc, (const long*)dsb, (long)nl * e->N, (const u64* const*)dpp, (int)pc.size(), out_of(acc), np, e->q, e->qinv, e->logN);
        }
        HIPC(hipGetLastError());
        *out = rescale_view(e, view_of(acc));
        aesfhe_ct_free(acc);
    }
    API_END
}

// -----------------------------------------------------------------------------------------------
// key switching of one polynomial per batch element.
// d: NTT-domain polynomial of batch element b at d + b*dbs (level l, limbs contiguous).
// Result: out poly 0/1 = addend_{0/1} + KS(d)_{0/1}, written into ct `o` (2 polys, level l - r).
// r = 0: plain ModDown by P.  Either way the base conversion is exact (round-to-nearest
// division: v = rint(sum_j y_j / e_j) multiples of D removed), so the rounding noise is
// |eps| <= 1/2 per coefficient instead of the fast conversion's 0..K overflow.  r >= 1: combined ModDown + rescale -- P * addend joins the
// accumulators in the inner product and one base conversion from E = {q_{l-r+1}..q_l, P} divides
// by D = P q_l ... q_{l-r+1} (oracle/ckks_oracle.c moddown_r states the same procedure).
// template launchers (a template argument list inside hipLaunchKernelGGL would split its macro args)
template <int A, typename... Args>
static void launch_modup(dim3 g, hipStream_t s, Args... args) {  // two coefficients per thread
    g.x /= 2;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_modup<A, 2>), g, dim3(256), 0, s, args...);
}
template <int NE, typename... Args>
static void launch_moddown(dim3 g, hipStream_t s, Args... args) {
    hipLaunchKernelGGL(k_moddown<NE>, g, dim3(256), 0, s, args...);
}

// target-limb groups (gridDim.y) of a base conversion over P polynomials: a thread converts its
// two coefficients into every target of its group, so small batches (the reference services'
// single ciphertexts) would leave most CUs idle with one group; >= 1024 workgroups of 256 threads
// (4 per CU) otherwise, 1 group at the batched workloads (P >= 8 at N = 2^16).  The outputs do
// not depend on the grouping (each target is computed the same way).
static unsigned bconv_groups(int N, int P, int ntarget) {
    const long wg = (long)(N / 512) * P;
    const long g = (1024 + wg - 1) / wg;
    return (unsigned)std::max(1L, std::min(g, (long)ntarget));
}

// Base conversions on the matrix cores (bconv_mfma.h), the default (round 5: ModUp 214 -> 190 us,
// ModDown 453 -> 403 us per call, round +3.2 %, profiles/r05/ab/bconv_mfma/); AESFHE_BCONV_VALU=1
// selects the exact-fp64 VALU kernels (k_modup / k_moddown) for A/B runs.  Same residues either way.
static bool bconv_mfma_on() {
    static const bool on = !(getenv("AESFHE_BCONV_VALU") && atoi(getenv("AESFHE_BCONV_VALU")));
    return on;
}
// nslots = source slots (+ 1 for ModDown's v): ceil(nslots / 4) K-steps of 32 bytes (<= 4)
static void launch_bconv(aesfhe_engine* e, BconvArgs a, int nz, int nslots, bool vc) {
    const int N = e->N, nstep = (nslots + 3) / 4, ntile = (a.nt + 3) / 4;
    if (nstep < 1 || nstep > 4 || ntile < 1) throw_err(AESFHE_EUNSUPPORTED, "matrix-core base conversion of %d slots", nslots);
    // target groups: >= ~1024 workgroups of 256 threads when the batch alone does not fill the chip
    const long wg = (long)(N / 256) * nz;
    const long groups0 = std::max(1L, std::min((long)ntile, (1024 + wg - 1) / wg));
    a.tiles_per_group = (int)((ntile + groups0 - 1) / groups0);
    const unsigned groups = (unsigned)((ntile + a.tiles_per_group - 1) / a.tiles_per_group);
    const dim3 g(N / 256, groups, nz);
#define BCV(S, V) hipLaunchKernelGGL((k_bconv_mfma<S, V>), g, dim3(256), 0, e->stream, a, e->logN)
    switch (nstep * 2 + (vc ? 1 : 0)) {
        case 2: BCV(1, false); break;
        case 3: BCV(1, true); break;
        case 4: BCV(2, false); break;
        case 5: BCV(2, true); break;
        case 6: BCV(3, false); break;
        case 7: BCV(3, true); break;
        case 8: BCV(4, false); break;
        default: BCV(4, true); break;
    }
#undef BCV
    HIPC(hipGetLastError());
}

// ModUp fused with the extension limbs' forward column pass (bconv_cols.h, N = 2^16; round 6,
// VERDICT r5 item 1): the sources are y (the INTT folded qhat^{-1}), the extension limbs leave as
// the column pass's raw-double intermediate.  AESFHE_MODUP_FUSED=0 selects k_bconv_mfma + the
// column pass for A/B runs.  Same residues either way.
static bool modup_fused_on() {
    static const bool on = !(getenv("AESFHE_MODUP_FUSED") && !atoi(getenv("AESFHE_MODUP_FUSED")));
    return on;
}
// source row groups prefetched ahead (bconv_cols.h PF; AESFHE_BCC_PF=0 for A/B runs; PF 2 measured
// slower and was dropped)
static int bcc_pf() {
    static const int pf = getenv("AESFHE_BCC_PF") ? std::max(0, std::min(1, atoi(getenv("AESFHE_BCC_PF")))) : 1;
    return pf;
}
template <bool VC>
static void launch_bconv_cols_t(aesfhe_engine* e, const BconvArgs& a, int nz, int nslots) {
    const int nstep = (nslots + 3) / 4, ntile = (a.nt + 3) / 4;
    if (e->logN != 16 || nstep < 1 || nstep > 4 || ntile < 1 || (16 * nz) % 8)
        throw_err(AESFHE_EUNSUPPORTED, "fused base conversion of %d slots to %d targets", nslots, a.nt);
    if (!a.src || !a.dst || !a.tab || !a.corr || !a.pc || (VC && !a.einv))
        throw_err(AESFHE_EUNSUPPORTED, "fused base conversion with a missing table");  // never launch on a null table
    const dim3 g((unsigned)(16 * nz * ntile));
    const Tabs T = e->tabs();
    const int pf = bcc_pf();
#define BCC(S, P) hipLaunchKernelGGL((k_bconv_cols<S, true, VC, P>), g, dim3(256), 0, e->stream, a, T, ntile)
#define BCS(S) do { if (pf == 0) BCC(S, 0); else BCC(S, 1); } while (0)
    switch (nstep) {
        case 1: BCS(1); break;
        case 2: BCS(2); break;
        case 3: BCS(3); break;
        default: BCS(4); break;
    }
#undef BCS
#undef BCC
    HIPC(hipGetLastError());
}
static void launch_bconv_cols(aesfhe_engine* e, const BconvArgs& a, int nz) { launch_bconv_cols_t<false>(e, a, nz, a.ns); }

// The lazy-ModDown BSGS map with its babies formed inside the term sums (k_bsgs_terms) instead
// of written (k_ks_inner_multi + k_dot_pt_ext_multi) is the default; AESFHE_BSGS_FUSED=0 selects
// the unfused pair for A/B runs.  Its first form (one batch element per thread, every element
// re-reading its babies' keys) lost: 3.63 against 3.27 ms per refreshed bit ciphertext.  With
// the key and plaintext words of each baby serving BB = 2..4 elements per thread it gains:
// 3.15 against 3.23 ms, ten rounds 17.99 k / 17.89 k against 17.63 k / 17.66 k blocks/s
// (A/B/A/B on one box, profiles/r05/ab/bsgs_fused/).
// The order k_bsgs_terms walks the 256-slot k-blocks of a limb in: along the orbits of pi, the
// block map of the first keyed baby's Galois element g (slot k = 256 kb + j reads slot
// sigma_g(k) = brv(((g (2 brv(k) + 1)) mod 2N - 1) / 2), whose block depends on kb alone), when
// every keyed baby i is g^i (the BSGS babies: rotations by i x stride); otherwise 0, 1, 2, ...
// Either order is a permutation of the blocks, so results do not depend on it.
static std::vector<unsigned short> bsgs_block_order(int logN, const std::vector<u64>& gal) {
    std::vector<unsigned short> ord;  // bsgs_plan.h: the orbit walk, or 0, 1, 2, ...
    if (!aesfhe::bsgs_block_order(logN, std::vector<uint64_t>(gal.begin(), gal.end()), ord))
        throw_err(AESFHE_EUNSUPPORTED, "bsgs block order is not a permutation");
    return ord;
}

static bool bsgs_fused_on() {
    static const bool on = !(getenv("AESFHE_BSGS_FUSED") && !atoi(getenv("AESFHE_BSGS_FUSED")));
    return on;
}
// The LDS-DMA pipelined key-switch row kernels (ks_fused.h k_nttf_rows_ks_p) are the default
// (round 5: round +1.0 %, A/B/A/B on one box, profiles/r05/ab/ks_pipe/); AESFHE_KS_PIPE=0 selects
// k_nttf_rows_ks for A/B runs
static bool ks_pipe_on() {
    static const bool on = !(getenv("AESFHE_KS_PIPE") && !atoi(getenv("AESFHE_KS_PIPE")));
    return on;
}

static int ks_beta(const aesfhe_engine* e, int l) {
    const int beta = (l + 1 + e->A - 1) / e->A;
    if (beta > 12) throw_err(AESFHE_EUNSUPPORTED, "more than 12 key-switch digits");
    return beta;
}
// a switching key serves a key switch at level l when it stores the beta(l) digits it reads
// (aesfhe_key_trim keeps the first digits only; their words are the full key's, digit by digit)
static void check_key_digits(aesfhe_engine* e, const aesfhe_key* k, int l) {
    if (k && k->ndig > 0 && ks_beta(e, l) > k->ndig)
        throw_err(AESFHE_ELEVEL, "key trimmed to %d digits cannot switch at level %d (%d digits)", k->ndig, l, ks_beta(e, l));
}

// Key switch, first half (ModUp): ext[j][b] = the NTT-domain extension of digit j of d to every
// limb of Q_l u P outside the digit (the digit's own limbs are read from d by the inner product).
// ext holds ks_beta(l) * B * (l+1+K) limbs.  Shared by every key in aesfhe_rotate_hoisted.
// cols_only (fused_ntt engines): the extension limbs get only the NTT column pass; the row pass
// runs inside k_nttf_rows_ks together with the inner product (ks_fused.h).
// pa, pb (fused_ntt engines): the input is poly 1 of each, multiplied (d2 = a1 b1 of a product)
static void ks_modup(aesfhe_engine* e, const u64* d, long dbs, int B, int l, u64* ext, bool cols_only = false,
                     const Opnd* pa = nullptr, const Opnd* pb = nullptr, const u64* fac = nullptr) {
    const int N = e->N, K = e->K, ne = l + 1 + K;
    const long lN = (long)(l + 1) * N, neN = (long)ne * N;
    const int beta = ks_beta(e, l);
    Tmp dc(e, (size_t)B * lN);
    // fused (N = 2^16): every digit wider than one limb converts and runs its extension limbs'
    // column pass in one kernel (k_bconv_cols) from y = [x qhat^{-1}], which the INTT emits
    // directly (its N^{-1} times the digit's qhat^{-1} per limb; a one-limb digit's qhat^{-1} is 1,
    // so the spread path below reads the same words as before)
    const bool fcols = e->logN == 16 && bconv_mfma_on() && modup_fused_on();
    const double* lf = fcols ? e->mu_nhatf + (size_t)l * e->Lp1 : nullptr;
    // 1. INTT copy of the input
    Span sdc = span_s(dc.p, lN, l + 1, l + 1, 0, e->Lp1);
    if (pa) {
        Span sa = span_s((u64*)pa->ptr + pa->ps, pa->bs, l + 1, l + 1, 0, e->Lp1);
        Span sb = span_s((u64*)pb->ptr + pb->ps, pb->bs, l + 1, l + 1, 0, e->Lp1);
        sa.pmask = pa->bmask;  // cyclic broadcast of a product operand (check_cyclic)
        sb.pmask = pb->bmask;
        intt_prod(e, sa, sb, sdc, B * (l + 1), fac, lf);
    } else {
        Span sd = span_s((u64*)d, dbs, l + 1, l + 1, 0, e->Lp1);
        if (lf) ntt256<256>(e, sd, sdc, B * (l + 1), true, lf);
        else ntt(e, sd, sdc, B * (l + 1), true);
    }
    // out of place (cols_only): ModUp writes a buffer recycled across the digits and the column
    // pass reads it into ext_j -- the in-place pass read and wrote the same lines; one digit's
    // extension of extra memory, not one per digit (with the ModDown conv pass out of place as
    // well: round +0.8 %, A/B/A/B/A on one box, profiles/r04/ab/oop/)
    const bool oop = cols_only;
    std::unique_ptr<Tmp> mu;  // only when some digit runs k_modup (alpha > 1)
    bool any_wide = false;
    for (int j = 0; j < beta; j++) any_wide |= std::min((j + 1) * e->A, l + 1) - j * e->A > 1;
    if (oop && any_wide && !fcols) mu.reset(new Tmp(e, (size_t)B * neN));
    for (int j = 0; j < beta; j++) {
        const int A = e->A, lo = j * A, hi = std::min(lo + A, l + 1), alpha = hi - lo;
        const size_t set = (size_t)j * A + (alpha - 1);
        u64* exj = ext + (size_t)j * B * neN;
        u64* muj = mu ? mu->p : exj;  // where ModUp writes (mu absent: every digit is one limb)
        if (cols_only && alpha == 1) {
            // one-limb digit: the conversion is x mod p_t (hat = hatinv = 1), formed in the column
            // pass's copy-in from the digit limb itself (no k_modup<1> write + read-back)
            const SpreadSrc ss{(const u64*)dc.p + (long)lo * N, lN, 0, 0, 0.0};
            auto kern = N == 65536 ? k_nttf_fwd_cols_spread<256, 3> : k_nttf_fwd_cols_spread<512, 3>;
            auto cols = [&](Span sp, int total) {
                ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_fwd_cols_spread");
                hipLaunchKernelGGL(kern, dim3(16, total), dim3(256), 0, e->stream, ss, sp, e->tabs());
            };
            if (lo > 0) cols(span_s(exj, neN, lo, lo, 0, e->Lp1), B * lo);
            cols(span_s(exj + (long)hi * N, neN, ne - hi, (l + 1) - hi, hi, e->Lp1), B * (ne - hi));
            HIPC(hipGetLastError());
            continue;
        }
        if (fcols) {  // 2'. conversion + column pass in one launch, straight into ext_j (+ the row pass
                      // for callers that read the extension in NTT form: hoisted rotations, BSGS babies)
            BconvArgs a{};
            a.src = (const u64*)dc.p + (long)lo * N;
            a.sbs = lN;
            a.dst = exj;
            a.dbs = neN;
            a.nc = 1;
            a.ns = alpha;
            a.s_nq = alpha;
            a.s_q0 = lo;
            a.nt = ne - alpha;
            a.skip0 = lo;
            a.skipn = alpha;
            a.tl_l = l;
            a.Lp1 = e->Lp1;
            a.tab = e->bc_mu_tab + set * e->np * 8 * kBconvKT;
            a.corr = e->bc_mu_corr + set * e->np;
            a.pc = e->bc_pc;
            a.qall = e->q;
            a.qinvall = e->qinv;
            // algorithmic bytes: the digit's sources read once, the extension limbs written once
            {
                ProfScope ps(e, FAM_KS, 8.0 * N * (double)B * ne, "modup_cols");
                launch_bconv_cols(e, a, B);
            }
            if (!cols_only) {
                auto rows = [&](long off, int n, int nq, int p0, int total) {
                    ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_fwd_rows");
                    hipLaunchKernelGGL((k_nttf_fwd_rows_t<false, 256>), dim3(16, total), dim3(256), 0, e->stream,
                                       span_s(exj + off, neN, n, nq, p0, e->Lp1), e->tabs(), RowFin{});
                    HIPC(hipGetLastError());
                };
                if (lo > 0) rows(0, lo, lo, 0, B * lo);
                rows((long)hi * N, ne - hi, (l + 1) - hi, hi, B * (ne - hi));
            }
            continue;
        }
        // 2. ModUp base conversion of digit j to every other limb, then NTT those limbs
        {
            ProfScope ps(e, FAM_KS, 8.0 * N * (double)B * ne, "modup");
            if (alpha < 1 || alpha > 16) throw_err(AESFHE_EUNSUPPORTED, "ModUp digit width outside 1..16");
            if (bconv_mfma_on()) {
                BconvArgs a{};
                a.src = (const u64*)dc.p + (long)lo * N;
                a.sbs = lN;
                a.dst = muj;
                a.dbs = neN;
                a.nc = 1;
                a.ns = alpha;
                a.s_nq = alpha;
                a.s_q0 = lo;
                a.sinvf = e->mu_hatinvf + set * A;
                a.nt = ne - alpha;
                a.skip0 = lo;
                a.skipn = alpha;
                a.tl_l = l;
                a.Lp1 = e->Lp1;
                a.tab = e->bc_mu_tab + set * e->np * 8 * kBconvKT;
                a.corr = e->bc_mu_corr + set * e->np;
                a.pc = e->bc_pc;
                a.qall = e->q;
                a.qinvall = e->qinv;
                launch_bconv(e, a, B, alpha, false);
            } else
            AESFHE_DISPATCH16(alpha, launch_modup, dim3(N / 256, bconv_groups(N, B, ne), B), e->stream, (const u64*)dc.p, lN, muj, neN, lo, l, ne,
                              (const double*)(e->mu_hatinvf + set * A), (const TwD*)(e->mu_hatf + set * A * e->np),
                              A, e->q, e->qinv, e->Lp1, e->logN);
        }
        HIPC(hipGetLastError());
        auto fwd = [&](long off, int n, int nq, int p0, int total) {
            Span sp = span_s(exj + off, neN, n, nq, p0, e->Lp1);
            if (!cols_only) return ntt(e, sp, sp, total, false);
            ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_fwd_cols");
            ntt_fwd_cols(e, span_s(muj + off, neN, n, nq, p0, e->Lp1), sp, total);
        };
        if (lo > 0) fwd(0, lo, lo, 0, B * lo);
        fwd((long)hi * N, ne - hi, (l + 1) - hi, hi, B * (ne - hi));
    }
}

// Key switch, second half: inner product of ext (ks_modup of d) with key k, ModDown (fused with
// r rescales) and the finish into o (+ addend).
// Key switch, second half, part 1: acc[b][c] (layout [B][2][l+1+K][N], NTT domain over Q_l u P)
// = sum_j ext_j (x) key_j,c; with pmod, P * addend_c joins the Q limbs (np of addend selects
// which components), so that a later ModDown by P (q_l ...) returns addend + KS.  accum: add into
// acc instead of overwriting it (the lazy-ModDown sums of aesfhe_linear_bsgs).  ext_cols: ext
// holds column-pass intermediates (ks_modup cols_only) and the inner product runs in the fused
// row pass k_nttf_rows_ks.
// pb (ext_cols, pmod, no accum): relinearisation of the product addend (x) pb (k_nttf_rows_ks
// PROD; d unused).
static void ks_inner_acc(aesfhe_engine* e, const u64* d, long dbs, const u64* ext, int B, int l,
                         const aesfhe_key* k, Opnd addend, bool pmod, u64* acc, bool ext_cols, bool accum = false,
                         const Opnd* pb = nullptr, const u64* fac = nullptr, const Opnd* pc = nullptr) {
    const int N = e->N, K = e->K, ne = l + 1 + K;
    const long neN = (long)ne * N;
    const int beta = ks_beta(e, l);
    check_key_digits(e, k, l);
    const double* pm = pmod ? (const double*)e->pmodf : (const double*)nullptr;
    if (pb && (!ext_cols || !pmod || accum)) throw_err(AESFHE_EARG, "product key switch needs the fused combined path");
    if (ext_cols) {
        // row pass of every extension limb (credited half an NTT per limb: 8 N B) + the inner product
        // (key read once per call, accumulators written; ext never leaves the chip) + the Q-limb
        // operands: the own digit's d limbs and the addend (PROD: a0, a1, b0, b1)
        const int nown = std::min(l + 1, beta * e->A);
        const double opw = pb ? (4.0 + (pc && pc->ptr ? 2.0 : 0.0)) * (l + 1)
                              : (double)nown + (pmod && addend.ptr ? (double)addend.np * (l + 1) : 0.0);
        ProfScope ps(e, FAM_KS, 8.0 * N * ((double)B * (beta * ne - nown + opw) + (double)ne * (2.0 * beta + 2.0 * B * (accum ? 2 : 1))), pb ? "ks_rows_acc.prod" : "ks_rows_acc.ks");
        const int R = N / 256, blocks = 8 * B * (ne * (R / 8) / 8);
        const Opnd none{nullptr, 0, 0, 0};
        auto kern = pb ? (R == 256 ? k_nttf_rows_ks<1, 256, true> : k_nttf_rows_ks<1, 512, true>)
                       : (R == 256 ? k_nttf_rows_ks<1, 256, false> : k_nttf_rows_ks<1, 512, false>);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, e->stream, d, dbs, ext, neN, (long)B * neN, (const u64*)k->d, 2L * e->np * N, (long)e->np * N, acc, 2 * neN, neN, B, beta, e->A, l, ne, e->tabs(), addend, pm, (int)accum, pb ? *pb : none, fac, pc ? *pc : none, 0, ne, KsFin{});
    } else {
        ProfScope ps(e, FAM_KS, 8.0 * N * (double)ne * (beta * B + 2.0 * beta + 2.0 * B * (accum ? 2 : 1)), "ks_inner");
        auto inner = beta <= 4 ? k_ks_inner_all<4> : beta <= 8 ? k_ks_inner_all<8> : k_ks_inner_all<12>;
        hipLaunchKernelGGL(inner, dim3(N / 256, ne, 1), dim3(256), 0, e->stream, d, dbs, ext, neN, (long)B * neN, (const u64*)k->d, 2L * e->np * N, (long)e->np * N, acc, 2 * neN, neN, B, beta, e->A, l, e->q, e->qinv, e->Lp1, addend, pm, e->logN, (int)accum);
    }
    HIPC(hipGetLastError());
}

// Key switch, second half, part 2: ModDown of acc (2 components, layout [B][2][l+1+K][N]; its
// dropped limbs are overwritten) by D = P q_l ... q_{l-r+1} (fused with r rescales, DESIGN.md
// 3.12) into o (level l - r) = (acc - conv) D^{-1} + fin_add.
// ModDown, first part: INTT of acc's dropped limbs (top r Q limbs + the special limbs, layout
// [B][2][l+1+K][N]) and their exact base conversion to the lk + 1 = l - r + 1 kept limbs, into conv
// ([B][2][lk+1][N], coefficient form).  Returns D^{-1} mod q_i (as w / q) for the finish.
// rows_done (fused_ntt engines): the dropped limbs already hold their inverse row pass (raw
// doubles, k_nttf_rows_ks EPI 2), so only the inverse column pass runs.
// abs_ / acs: acc's batch and component strides (default: the full [B][2][l+1+K][N] layout; a
// caller that holds only the dropped limbs passes its own, with acc offset so that limb t is at
// acc + t N as before).
static const double* moddown_conv(aesfhe_engine* e, u64* acc, int B, int l, int r, u64* conv, bool rows_done = false,
                                  long abs_ = 0, long acs = 0) {
    const int N = e->N, K = e->K, ne = l + 1 + K;
    const long neN = (long)ne * N;
    if (!acs) acs = neN, abs_ = 2 * neN;
    if (r < 0 || r > kMdrMaxR || K + r > kMdrMaxE || l - r < 0) throw_err(AESFHE_EARG, "bad combined rescale depth %d", r);
    const int lk = l - r;  // output level
    const long kN = (long)(lk + 1) * N;
    // 4. ModDown: INTT the dropped limbs (top r Q limbs + the special limbs) of both accumulators
    {
        Span ssp = span_s(acc + (long)(lk + 1) * N, acs, K + r, r, lk + 1, e->Lp1);
        const int total = B * 2 * (K + r);
        if (rows_done) {
            ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_inv_cols");
            if (N == 65536) hipLaunchKernelGGL((k_nttf_inv_cols<256, false>), dim3(16, total), dim3(256), 0, e->stream, ssp, e->tabs(), (const double*)nullptr);
            else hipLaunchKernelGGL((k_nttf_inv_cols<512, false>), dim3(16, total), dim3(256), 0, e->stream, ssp, e->tabs(), (const double*)nullptr);
            HIPC(hipGetLastError());
        } else {
            ntt(e, ssp, ssp, total, true);
        }
    }
    const size_t cell = r ? (size_t)(r - 1) * e->Lp1 + l : 0;
    const double* invf = r ? e->mdr_invf + cell * kMdrMaxE : e->md_phatinvf;
    const TwD* hatf = r ? e->mdr_hatf + cell * kMdrMaxE * e->Lp1 : e->md_phatf;
    const int hs = r ? kMdrMaxE : K;  // hatf row stride (sources of one target)
    {
        ProfScope ps(e, FAM_KS, 8.0 * N * (double)B * 2 * (K + r + lk + 1), "moddown");
        if (K + r < 1 || K + r > 16) throw_err(AESFHE_EUNSUPPORTED, "ModDown source width outside 1..16");
        if (bconv_mfma_on() && K + r + 1 <= 16) {
            BconvArgs a{};
            a.src = acc + (long)(lk + 1) * N;
            a.sbs = abs_;
            a.scs = acs;
            a.dst = conv;
            a.dbs = 2 * kN;
            a.dcs = kN;
            a.nc = 2;
            a.ns = K + r;
            a.s_nq = r;
            a.s_q0 = lk + 1;
            a.s_p0 = e->Lp1;
            a.sinvf = invf;
            a.einv = r ? e->mdr_einv + cell * kMdrMaxE : e->md_einv;
            a.nt = lk + 1;
            a.skip0 = lk + 1;
            a.skipn = 0;
            a.tl_l = lk;
            a.Lp1 = e->Lp1;
            a.tab = r ? e->bc_mdr_tab + cell * e->Lp1 * 8 * kBconvKT : e->bc_md_tab;
            a.corr = r ? e->bc_mdr_corr + cell * e->Lp1 : e->bc_md_corr;
            a.pc = e->bc_pc;
            a.qall = e->q;
            a.qinvall = e->qinv;
            launch_bconv(e, a, B * 2, K + r + 1, true);
        } else
        AESFHE_DISPATCH16(K + r, launch_moddown, dim3(N / 512, bconv_groups(N, B * 2, lk + 1), B * 2), e->stream, (const u64*)acc, abs_, acs, l, r, conv, 2 * kN, kN,
                           invf, hatf, r ? e->mdr_einv + cell * kMdrMaxE : e->md_einv,
                           r ? e->mdr_dmodf + cell * e->Lp1 : e->pmodf, e->Lp1, e->q, e->qinv, e->logN, hs);
    }
    HIPC(hipGetLastError());
    return r ? e->mdr_dinvf + cell * e->Lp1 : e->md_pinvf;
}

// ModDown's conversion fused with conv's forward column pass (N = 2^16, rows_done accumulators;
// bconv_cols.h VC): the inverse column pass of the dropped limbs scales them by N^{-1} (D/e_j)^{-1}
// (md_ninvf / mdr_ninvf), so they leave as y_j, and k_bconv_cols writes conv's column-pass
// intermediate straight into conv2 ([B][2][lk + 1][N], what the FIN row launch reads) -- conv's
// coefficient form never reaches HBM.  Returns D^{-1} mod q_i (w / q) for the finish, as
// moddown_conv.  Same residues as moddown_conv + ntt_fwd_cols.
static bool moddown_cols_ok(const aesfhe_engine* e, int r) {
    return e->logN == 16 && bconv_mfma_on() && modup_fused_on() && r >= 0 && r <= kMdrMaxR && e->K + r + 1 <= 16;
}
static const double* moddown_conv_cols(aesfhe_engine* e, u64* acc, int B, int l, int r, u64* conv2, long abs_, long acs,
                                       bool rows_done = true) {
    const int N = e->N, K = e->K;
    const int lk = l - r;
    const long kN = (long)(lk + 1) * N;
    if (!moddown_cols_ok(e, r) || lk < 0) throw_err(AESFHE_EARG, "fused ModDown of depth %d", r);
    const size_t cell = r ? (size_t)(r - 1) * e->Lp1 + l : 0;
    {
        Span ssp = span_s(acc + (long)(lk + 1) * N, acs, K + r, r, lk + 1, e->Lp1);
        const int total = B * 2 * (K + r);
        const double* lf = r ? e->mdr_ninvf + cell * kMdrMaxE : e->md_ninvf;
        if (!rows_done) {  // canonical NTT-domain accumulators: the inverse row pass first
            ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_inv_rows");
            hipLaunchKernelGGL((k_nttf_inv_rows<256, false>), dim3(16, total), dim3(256), 0, e->stream, ssp, ssp, e->tabs(),
                               Span{}, (const u64*)nullptr);
            HIPC(hipGetLastError());
        }
        ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_inv_cols");
        hipLaunchKernelGGL((k_nttf_inv_cols<256, true>), dim3(16, total), dim3(256), 0, e->stream, ssp, e->tabs(), lf);
        HIPC(hipGetLastError());
    }
    BconvArgs a{};
    a.src = acc + (long)(lk + 1) * N;
    a.sbs = abs_;
    a.scs = acs;
    a.dst = conv2;
    a.dbs = 2 * kN;
    a.dcs = kN;
    a.nc = 2;
    a.ns = K + r;
    a.s_nq = r;
    a.s_q0 = lk + 1;
    a.s_p0 = e->Lp1;
    a.einv = r ? e->mdr_einv + cell * kMdrMaxE : e->md_einv;
    a.nt = lk + 1;
    a.skip0 = lk + 1;
    a.skipn = 0;
    a.tl_l = lk;
    a.Lp1 = e->Lp1;
    a.tab = r ? e->bc_mdr_tab + cell * e->Lp1 * 8 * kBconvKT : e->bc_md_tab;
    a.corr = r ? e->bc_mdr_corr + cell * e->Lp1 : e->bc_md_corr;
    a.pc = e->bc_pc;
    a.qall = e->q;
    a.qinvall = e->qinv;
    {
        // algorithmic bytes: the dropped limbs read once, conv's intermediate written once
        ProfScope ps(e, FAM_KS, 8.0 * N * (double)B * 2 * (K + r + lk + 1), "moddown_cols");
        launch_bconv_cols_t<true>(e, a, 2 * B, K + r + 1);
    }
    return r ? e->mdr_dinvf + cell * e->Lp1 : e->md_pinvf;
}

static void moddown_acc(aesfhe_engine* e, u64* acc, int B, int l, int r, Opnd fin_add, aesfhe_ct* o) {
    const int N = e->N, K = e->K, ne = l + 1 + K;
    const long neN = (long)ne * N;
    const int lk = l - r;  // output level
    const long kN = (long)(lk + 1) * N;
    if (moddown_cols_ok(e, r)) {  // conversion + conv's column pass fused, then the finishing row pass
        Tmp conv2(e, (size_t)B * 2 * kN);
        const double* dinvf = moddown_conv_cols(e, acc, B, l, r, conv2.p, 2 * neN, neN, false);
        const int total = B * 2 * (lk + 1);
        RowFin f{(const u64*)acc, 2 * neN, neN, Opnd2{fin_add.ptr, fin_add.bs, fin_add.ps, fin_add.np}, o->d,
                 2L * (lk + 1) * N, (long)(lk + 1) * N, dinvf, lk + 1};
        ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total * (3.0 + (fin_add.ptr ? 1.0 : 0.0)), "ntt_fwd_rows_fin");
        hipLaunchKernelGGL((k_nttf_fwd_rows_t<true, 256>), dim3(16, total), dim3(256), 0, e->stream,
                           span_s(conv2.p, kN, lk + 1, lk + 1, 0, e->Lp1), e->tabs(), f);
        HIPC(hipGetLastError());
        return;
    }
    Tmp conv(e, (size_t)B * 2 * kN);
    const double* dinvf = moddown_conv(e, acc, B, l, r, conv.p);
    const size_t cell = r ? (size_t)(r - 1) * e->Lp1 + l : 0;
    const u64* dinv = r ? e->mdr_dinv + cell * e->Lp1 : e->md_pinv;
    Span sc = span_s(conv.p, kN, lk + 1, lk + 1, 0, e->Lp1);
    if (fused_ntt(e)) {
        // conv NTT with the finish in the row pass's epilogue: conv never reaches HBM; the column
        // pass out of place (as ks_modup's), into a second buffer the row pass reads
        Tabs T = e->tabs();
        const int total = B * 2 * (lk + 1);
        Tmp conv2(e, (size_t)B * 2 * kN);
        {
            Span s2 = span_s(conv2.p, kN, lk + 1, lk + 1, 0, e->Lp1);
            ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_fwd_cols");
            ntt_fwd_cols(e, sc, s2, total);
            sc = s2;
        }
        RowFin f{(const u64*)acc, 2 * neN, neN, Opnd2{fin_add.ptr, fin_add.bs, fin_add.ps, fin_add.np}, o->d,
                 2L * (lk + 1) * N, (long)(lk + 1) * N, dinvf, lk + 1};
        // the row pass (credited half an NTT) plus the finish: acc read, output written (+ addend)
        ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total * (3.0 + (fin_add.ptr ? 1.0 : 0.0)), "ntt_fwd_rows_fin");
        if (N == 65536) hipLaunchKernelGGL((k_nttf_fwd_rows_t<true, 256>), dim3(16, total), dim3(256), 0, e->stream, sc, T, f);
        else hipLaunchKernelGGL((k_nttf_fwd_rows_t<true, 512>), dim3(32, total), dim3(256), 0, e->stream, sc, T, f);
        HIPC(hipGetLastError());
        return;
    }
    ntt(e, sc, sc, B * 2 * (lk + 1), false);
    ProfScope psf(e, FAM_KS, 8.0 * N * (double)B * 2 * (lk + 1) * 4, "moddown_finish");
    hipLaunchKernelGGL(k_moddown_finish, dim3(N / 256, lk + 1, B * 2), dim3(256), 0, e->stream, (const u64*)acc, 2 * neN, neN, (const u64*)conv.p, 2 * kN, kN, fin_add, out_of(o), e->q, dinv, dinvf, e->logN);
    HIPC(hipGetLastError());
}


// Key switch, second half, for fused_ntt engines (ext holds column-pass intermediates), with the
// ModDown finish fused into the Q limbs' row pass: k_nttf_rows_ks runs twice --
//   1. the dropped limbs t = lk + 1 .. l + K (top r Q limbs + P) into acc, as ks_inner_acc;
//   2. ModDown's INTT of those, the base conversion (conv) and conv's column pass (conv2);
//   3. the kept limbs t = 0 .. lk (FIN): the inner product, conv's row pass and the finish
//      (acc - conv) D^{-1} (+ fin_add) written straight into o.
// The kept limbs' accumulators (2 B (lk + 1) limbs) are neither written nor read back, which is
// what the unfused order (ks_inner_acc over every limb, then moddown_acc's finishing row pass)
// spends on them.  Residues identical: every step is exact mod q, outputs canonical.
// pmod: P * addend joins the accumulators (combined ModDown + rescale, 3.12; the giants of
// aesfhe_linear_bsgs with r = 0).  pb / fac / pc: the product relinearisation of keyswitch_prod
// (k_nttf_rows_ks PROD).  acc_in / accum: add to the accumulators of earlier key switches in
// acc_in (layout [B][2][l+1+K][N]; the last giant of aesfhe_linear_bsgs) instead of a fresh sum.
static void ks_finish_fused(aesfhe_engine* e, const u64* d, long dbs, const u64* ext, int B, int l,
                            const aesfhe_key* k, Opnd addend, bool pmod, int r, Opnd fin_add, aesfhe_ct* o,
                            const Opnd* pb = nullptr, const u64* fac = nullptr, const Opnd* pc = nullptr,
                            u64* acc_in = nullptr, bool accum = false) {
    const int N = e->N, K = e->K, ne = l + 1 + K, R = N / 256;
    const long neN = (long)ne * N;
    const int beta = ks_beta(e, l), lk = l - r;
    check_key_digits(e, k, l);
    if (r < 0 || r > kMdrMaxR || K + r > kMdrMaxE || lk < 0) throw_err(AESFHE_EARG, "bad combined rescale depth %d", r);
    if (pb && r < 1) throw_err(AESFHE_EARG, "product key switch needs the fused combined path");
    const long kN = (long)(lk + 1) * N;
    const double* pm = pmod ? (const double*)e->pmodf : (const double*)nullptr;
    const Opnd none{nullptr, 0, 0, 0};
    if (accum && (!acc_in || pb)) throw_err(AESFHE_EARG, "accumulating key switch without accumulators");
    // bytes of a launch over limbs [t0, t0 + nt), nq of them Q limbs: ext rows (every digit but
    // the limb's own), the own digit's d rows and the addend (PROD: a0, a1, b0, b1 [, c0, c1]),
    // the key words, and the outputs (acc: 2 B nt limbs; FIN: conv read + out written, + fin_add)
    auto bytes = [&](int nt, int nq, bool fin) {
        const double opw = pb ? (4.0 + (pc && pc->ptr ? 2.0 : 0.0)) * nq
                              : (double)nq + (pm && addend.ptr ? (double)addend.np * nq : 0.0);
        const double outw = (fin ? 2.0 * 2 * nq + (fin_add.ptr ? (double)fin_add.np * nq : 0.0) : 2.0 * nt) +
                            (accum ? 2.0 * nt : 0.0);  // accum: the earlier sums read
        return 8.0 * N * ((double)B * ((double)beta * nt - nq + opw + outw) + 2.0 * beta * nt);
    };
    auto launch = [&](int t0, int nt, bool fin, u64* acc, long abs_, long acs, const KsFin& kf) {
        const int blocks = 8 * B * (nt * (R / 8) / 8 + ((nt * (R / 8)) % 8 ? 1 : 0));
        const int nq = std::max(0, std::min(t0 + nt, l + 1) - t0);
        // one label per kernel instantiation (PROD or not): a class average over launches of very
        // different sizes is not comparable with a rocprof per-symbol average
        ProfScope ps(e, FAM_KS, bytes(nt, nq, fin),
                     fin ? (pb ? "ks_rows_fin.prod" : "ks_rows_fin.ks") : (pb ? "ks_rows_inner.prod" : "ks_rows_inner.ks"));
        // the dropped limbs leave with their inverse row pass done (EPI 2), the kept ones finished (EPI 1)
        auto kern = R == 256 ? (pb ? (fin ? k_nttf_rows_ks<1, 256, true, 1> : k_nttf_rows_ks<1, 256, true, 2>)
                                   : (fin ? k_nttf_rows_ks<1, 256, false, 1> : k_nttf_rows_ks<1, 256, false, 2>))
                             : (pb ? (fin ? k_nttf_rows_ks<1, 512, true, 1> : k_nttf_rows_ks<1, 512, true, 2>)
                                   : (fin ? k_nttf_rows_ks<1, 512, false, 1> : k_nttf_rows_ks<1, 512, false, 2>));
        if (ks_pipe_on())
            kern = R == 256 ? (pb ? (fin ? k_nttf_rows_ks_p<256, true, 1> : k_nttf_rows_ks_p<256, true, 2>)
                                  : (fin ? k_nttf_rows_ks_p<256, false, 1> : k_nttf_rows_ks_p<256, false, 2>))
                            : (pb ? (fin ? k_nttf_rows_ks_p<512, true, 1> : k_nttf_rows_ks_p<512, true, 2>)
                                  : (fin ? k_nttf_rows_ks_p<512, false, 1> : k_nttf_rows_ks_p<512, false, 2>));
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, e->stream, d, dbs, ext, neN, (long)B * neN, (const u64*)k->d,
                           2L * e->np * N, (long)e->np * N, acc, abs_, acs, B, beta, e->A, l, ne, e->tabs(), addend, pm,
                           (int)accum, pb ? *pb : none, fac, pc ? *pc : none, t0, nt, kf);
        HIPC(hipGetLastError());
    };
    // only the dropped limbs lk + 1 .. ne - 1 are written: an own accumulator holds just those
    // ([B][2][nd][N], nd = ne - lk - 1; ADVICE r4: the full [B][2][ne][N] block was ~1 GB per key
    // switch at B = 32, l = 30 of memory never touched), addressed through a base pointer offset by
    // lk + 1 limbs so that limb t still sits at acc + t N; the FIN launch does not read acc then
    const int nd = ne - (lk + 1);
    std::unique_ptr<Tmp> own;
    if (!acc_in) own.reset(new Tmp(e, (size_t)B * 2 * nd * N));
    // (an address, not a C++ pointer into the block: only limbs >= lk + 1 are ever formed from it,
    // by the dropped limbs' launch and moddown_conv; the FIN launch gets no accumulators at all)
    u64* acc = acc_in ? acc_in : reinterpret_cast<u64*>(reinterpret_cast<uintptr_t>(own->p) - (uintptr_t)(lk + 1) * N * sizeof(u64));
    const long abs_ = acc_in ? 2 * neN : 2L * nd * N, acs = acc_in ? neN : (long)nd * N;
    launch(lk + 1, nd, false, acc, abs_, acs, KsFin{});
    const double* dinvf;
    std::unique_ptr<Tmp> conv2;
    if (moddown_cols_ok(e, r)) {  // conversion + conv's column pass in one launch (bconv_cols.h)
        conv2.reset(new Tmp(e, (size_t)B * 2 * kN));
        dinvf = moddown_conv_cols(e, acc, B, l, r, conv2->p, abs_, acs);
        if (own) own.reset();
    } else {
        std::unique_ptr<Tmp> conv(new Tmp(e, (size_t)B * 2 * kN));
        dinvf = moddown_conv(e, acc, B, l, r, conv->p, true, abs_, acs);
        if (own) own.reset();  // the dropped limbs are converted: stream-ordered reuse from here on
        conv2.reset(new Tmp(e, (size_t)B * 2 * kN));
        {
            const int total = B * 2 * (lk + 1);
            ProfScope ps(e, FAM_NTT, 8.0 * N * (double)total, "ntt_fwd_cols");
            ntt_fwd_cols(e, span_s(conv->p, kN, lk + 1, lk + 1, 0, e->Lp1), span_s(conv2->p, kN, lk + 1, lk + 1, 0, e->Lp1), total);
        }
        conv.reset();  // conv's coefficient form is read only by the column pass
    }
    HIPC(hipGetLastError());
    const KsFin kf{conv2->p, 2 * kN, kN, o->d, 2L * (lk + 1) * N, (long)(lk + 1) * N, dinvf,
                   Opnd2{fin_add.ptr, fin_add.bs, fin_add.ps, fin_add.np}};
    // the kept limbs' accumulators exist only in acc_in (accumulating giants); with an own block
    // FIN reads none: nullptr, so that no later change can read conv2's reuse of that memory
    if (own && accum) throw_err(AESFHE_EARG, "accumulating key switch without accumulators");
    launch(0, lk + 1, true, own ? nullptr : acc, abs_, acs, kf);
}

// Key switch, second half: inner product of ext (ks_modup of d) with key k, ModDown (fused with
// r rescales) and the finish into o (+ addend).  ext_cols: see ks_inner_acc.
static void ks_apply(aesfhe_engine* e, const u64* d, long dbs, const u64* ext, int B, int l,
                     const aesfhe_key* k, Opnd addend, aesfhe_ct* o, int r, bool ext_cols = false) {
    Opnd fin_add = addend;
    if (r) fin_add.ptr = nullptr;  // already inside the accumulators (times P)
    if (ext_cols) return ks_finish_fused(e, d, dbs, ext, B, l, k, addend, r != 0, r, fin_add, o);
    Tmp acc(e, (size_t)B * 2 * (l + 1 + e->K) * e->N);
    ks_inner_acc(e, d, dbs, ext, B, l, k, addend, r != 0, acc.p, ext_cols);
    moddown_acc(e, acc.p, B, l, r, fin_add, o);
}

static void keyswitch(aesfhe_engine* e, const u64* d, long dbs, int B, int l, const aesfhe_key* k,
                      Opnd addend, aesfhe_ct* o, int r = 0) {
    const long neN = (long)(l + 1 + e->K) * e->N;
    Tmp ext(e, (size_t)ks_beta(e, l) * B * neN);
    const bool fuse = fused_ntt(e);
    ks_modup(e, d, dbs, B, l, ext.p, fuse);
    ks_apply(e, d, dbs, ext.p, B, l, k, addend, o, r, fuse);
}

// relinearisation + r >= 1 rescales of the product a (x) b without a tensor ciphertext
// (fused_ntt engines, combined ModDown + rescale): d2 = a1 b1 is formed in the INTT's copy-in,
// d0, d1 and the own digit's d2 term in the prologue of k_nttf_rows_ks (PROD).  Same residues
// as tensor_ct + relin_rescale; the 3-polynomial tensor (3 limbs written, 3 read back, per
// Q limb) never reaches HBM.
// fac / pc (optional): the multiply-add of aesfhe_mul_fma, per-prime {alpha, C, K} (device) and
// the addend ciphertext c (truncated to level l).
static void keyswitch_prod(aesfhe_engine* e, const Opnd& pa, const Opnd& pb, int B, int l, const aesfhe_key* k,
                           aesfhe_ct* o, int r, const u64* fac = nullptr, const Opnd* pc = nullptr) {
    if (!fused_ntt(e) || r < 1 || pa.np != 2 || pb.np != 2 || !pa.ptr || !pb.ptr)
        throw_err(AESFHE_EARG, "product key switch outside the fused combined path");
    const long neN = (long)(l + 1 + e->K) * e->N;
    Tmp ext(e, (size_t)ks_beta(e, l) * B * neN);
    ks_modup(e, nullptr, 0, B, l, ext.p, true, &pa, &pb, fac);
    ks_finish_fused(e, nullptr, 0, ext.p, B, l, k, pa, true, r, Opnd{nullptr, 0, 0, 0}, o, &pb, fac, pc);
}

static aesfhe_ct* relin_ct(aesfhe_engine* e, const aesfhe_ct* c, const aesfhe_key* rlk) {
    const int l = c->level;
    aesfhe_ct* r = ct_new(e, c->B, 2, l);
    View v = view_of(c);
    Opnd add = opnd(v, c->B);
    add.np = 2;  // d0, d1 are the addends of outputs 0, 1
    keyswitch(e, c->d + 2 * v.ps, v.bs, c->B, l, rlk, add, r);
    return r;
}

// relinearisation of a 3-polynomial ciphertext fused with r rescales (r = 1, 2): level l - r
static aesfhe_ct* relin_rescale(aesfhe_engine* e, const aesfhe_ct* c, const aesfhe_key* rlk, int r) {
    const int l = c->level;
    if (r > 0 && e->K + r > kMdrMaxE) {  // no combined tables: separate steps
        aesfhe_ct* x = relin_ct(e, c, rlk);
        for (int i = 0; i < r; i++) {
            aesfhe_ct* y = rescale_view(e, view_of(x));
            aesfhe_ct_free(x);
            x = y;
        }
        return x;
    }
    aesfhe_ct* out = ct_new(e, c->B, 2, l - r);
    View v = view_of(c);
    Opnd add = opnd(v, c->B);
    add.np = 2;
    keyswitch(e, c->d + 2 * v.ps, v.bs, c->B, l, rlk, add, out, r);
    return out;
}

static aesfhe_ct* tensor_ct(aesfhe_engine* e, const View& a, const View& b, int B) {
    const int l = a.level;
    aesfhe_ct* t = ct_new(e, B, 3, l);
    ProfScope ps(e, FAM_EW, 56.0 * e->N * (l + 1) * (double)B, "tensor");
    hipLaunchKernelGGL(k_tensor, ew_grid(e, l + 1, B), dim3(256), 0, e->stream, opnd(a, B), opnd(b, B), out_of(t), e->q, e->qinv, 0, e->logN);
    HIPC(hipGetLastError());
    return t;
}

extern "C" int aesfhe_tensor(aesfhe_engine* e, const aesfhe_ct* a, const aesfhe_ct* b, aesfhe_ct** out) {
    API_BEGIN
    if (a->np != 2 || b->np != 2) throw_err(AESFHE_EDEGREE, "tensor inputs should have 2 polynomials");
    check_cyclic(a->B, b->B);
    int l = std::min(a->level, b->level), B = std::max(a->B, b->B);
    if (a->is_zero || b->is_zero) {
        *out = ct_zero_new(e, B, 3, l);
    } else {
        Aligned A, Bv;
        align_to(e, a, l, A);
        align_to(e, b, l, Bv);
        *out = tensor_ct(e, A.v, Bv.v, B);
    }
    API_END
}

extern "C" int aesfhe_relinearize(aesfhe_engine* e, const aesfhe_ct* c, const aesfhe_key* rlk, aesfhe_ct** out) {
    API_BEGIN
    if (c->np != 3) throw_err(AESFHE_EDEGREE, "Input ciphertext should have 3 polynomials");
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "relinearize needs a relinearization key");
    if (c->is_zero) *out = ct_zero_new(e, c->B, 2, c->level);
    else *out = relin_ct(e, c, rlk);
    API_END
}

static aesfhe_ct* mul_ct(aesfhe_engine* e, const aesfhe_ct* a, const aesfhe_ct* b, const aesfhe_key* rlk) {
    check_cyclic(a->B, b->B);
    int l = std::min(a->level, b->level), B = std::max(a->B, b->B);
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a ciphertext multiplication");
    if (a->is_zero || b->is_zero) return ct_zero_new(e, B, 2, l - 1);
    Aligned A, Bv;
    align_to(e, a, l, A);
    align_to(e, b, l, Bv);
    if (fused_ntt(e) && e->K + 1 <= kMdrMaxE) {
        aesfhe_ct* r = ct_new(e, B, 2, l - 1);
        try {
            keyswitch_prod(e, opnd(A.v, B), opnd(Bv.v, B), B, l, rlk, r, 1);
        } catch (...) {
            aesfhe_ct_free(r);
            throw;
        }
        return r;
    }
    aesfhe_ct* t = tensor_ct(e, A.v, Bv.v, B);
    aesfhe_ct* r = relin_rescale(e, t, rlk, 1);
    aesfhe_ct_free(t);
    return r;
}

extern "C" int aesfhe_mul(aesfhe_engine* e, const aesfhe_ct* a, const aesfhe_ct* b, const aesfhe_key* rlk, aesfhe_ct** out) {
    API_BEGIN
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "multiply needs a relinearization key");
    if (a->np != 2 || b->np != 2) throw_err(AESFHE_EDEGREE, "multiply inputs should have 2 polynomials");
    *out = mul_ct(e, a, b, rlk);
    API_END
}

// out = alpha * a * b + gamma * c + beta with one relinearisation + rescale (oracle:
// aesfhe_mul_fma states the same constants): c truncated to the product level l, its scale
// compensated in C = llround(gamma * (D_l * (D_l / D_c))); beta as K = llround(beta D_l) *
// llround(D_l) mod q on d0.
extern "C" int aesfhe_mul_fma(aesfhe_engine* e, const aesfhe_ct* a, const aesfhe_ct* b, const aesfhe_key* rlk,
                              int64_t alpha, const aesfhe_ct* c, double gamma, double beta, aesfhe_ct** out) {
    API_BEGIN
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "multiply needs a relinearization key");
    if (a->np != 2 || b->np != 2) throw_err(AESFHE_EDEGREE, "multiply inputs should have 2 polynomials");
    const int l = std::min(a->level, b->level);
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a ciphertext multiplication");
    int B = std::max(a->B, b->B);
    if (c) {
        if (c->np != 2) throw_err(AESFHE_EDEGREE, "fma addend should have 2 polynomials");
        if (c->level < l) throw_err(AESFHE_ELEVEL, "fma addend level %d below the product level %d", c->level, l);
        B = std::max(B, c->B);
    }
    if ((a->B != B && a->B != 1) || (b->B != B && b->B != 1) || (c && c->B != B && c->B != 1))
        throw_err(AESFHE_EARG, "batch mismatch");
    Aligned A, Bv;
    const bool prod = !a->is_zero && !b->is_zero;
    if (prod) {
        align_to(e, a, l, A);
        align_to(e, b, l, Bv);
    }
    const bool hasc = c && !c->is_zero;
    const double* D = e->chain.scale.data();
    const int64_t Cc = c ? llround(gamma * (D[l] * (D[l] / D[c->level]))) : 0;
    const int64_t Rb = llround(beta * D[l]), R = llround(D[l]);
    std::vector<u64> fac(3 * (size_t)(l + 1));
    for (int i = 0; i <= l; i++) {
        const u64 q = e->chain.q[i];
        fac[3 * i] = h_smod(alpha, q);
        fac[3 * i + 1] = h_smod(Cc, q);
        fac[3 * i + 2] = h_mulmod(h_smod(Rb, q), h_smod(R, q), q);
    }
    u64* dfac = upload_small(e, fac.data(), fac.size());
    const Opnd none{nullptr, 0, 0, 0};
    if (prod && fused_ntt(e) && e->K + 1 <= kMdrMaxE) {  // tensor-free (keyswitch_prod with the fma factors)
        aesfhe_ct* r = ct_new(e, B, 2, l - 1);
        try {
            const Opnd oc = hasc ? opnd(trunc_view(c, l), B) : none;
            keyswitch_prod(e, opnd(A.v, B), opnd(Bv.v, B), B, l, rlk, r, 1, dfac, &oc);
        } catch (...) {
            aesfhe_ct_free(r);
            throw;
        }
        *out = r;
        return AESFHE_OK;
    }
    aesfhe_ct* t = ct_new(e, B, 3, l);
    {
        ProfScope ps(e, FAM_EW, 72.0 * e->N * (l + 1) * (double)B, "tensor_fma");
        hipLaunchKernelGGL(k_tensor_fma, ew_grid(e, l + 1, B), dim3(256), 0, e->stream, prod ? opnd(A.v, B) : none, prod ? opnd(Bv.v, B) : none,
                           hasc ? opnd(trunc_view(c, l), B) : none, out_of(t), (const u64*)dfac, e->q, e->qinv, e->logN);
    }
    HIPC(hipGetLastError());
    try {
        *out = relin_rescale(e, t, rlk, 1);
    } catch (...) {
        aesfhe_ct_free(t);
        throw;
    }
    aesfhe_ct_free(t);
    API_END
}

extern "C" int aesfhe_galois(aesfhe_engine* e, const aesfhe_ct* c, const aesfhe_key* gk, aesfhe_ct** out) {
    API_BEGIN
    if (!gk || gk->kind != 3) throw_err(AESFHE_EARG, "galois needs a rotation/conjugation key");
    if (c->np != 2) throw_err(AESFHE_EDEGREE, "Input ciphertext should have 2 polynomials");
    const int N = e->N, l = c->level;
    if (c->is_zero) {
        *out = ct_zero_new(e, c->B, 2, l);
    } else {
        // permute both polynomials into a temporary ct, then key-switch poly 1
        aesfhe_ct* p = ct_new(e, c->B, 2, l);
        Span src = span_s(c->d, (long)(l + 1) * N, l + 1, l + 1, 0, e->Lp1), dst = span_s(p->d, (long)(l + 1) * N, l + 1, l + 1, 0, e->Lp1);
        hipLaunchKernelGGL(k_galois, dim3(N / 256, c->B * 2 * (l + 1)), dim3(256), 0, e->stream, src, dst, (u64)gk->galois, e->logN, e->Lp1);
        HIPC(hipGetLastError());
        aesfhe_ct* r = ct_new(e, c->B, 2, l);
        View pv = view_of(p);
        Opnd add = opnd(pv, c->B);
        add.np = 1;  // only output 0 gets sigma(c0)
        keyswitch(e, p->d + pv.ps, pv.bs, c->B, l, gk, add, r);
        aesfhe_ct_free(p);
        *out = r;
    }
    API_END
}

// n rotations of one ciphertext with hoisted keys (aesfhe_key_galois_hoisted): ModUp of c1 once,
// then per key the inner product + ModDown into (c0 + KS_0, KS_1) and sigma_g of both polys.
extern "C" int aesfhe_rotate_hoisted(aesfhe_engine* e, const aesfhe_ct* c, const aesfhe_key* const* keys, int32_t n,
                                     aesfhe_ct** outs) {
    API_BEGIN
    if (n < 1) throw_err(AESFHE_EARG, "rotate_hoisted needs at least one key");
    for (int i = 0; i < n; i++)
        if (!keys[i] || keys[i]->kind != 5) throw_err(AESFHE_EARG, "rotate_hoisted needs hoisted rotation keys");
    if (c->np != 2) throw_err(AESFHE_EDEGREE, "Input ciphertext should have 2 polynomials");
    const int N = e->N, l = c->level, B = c->B;
    for (int i = 0; i < n; i++) outs[i] = nullptr;
    try {
        if (c->is_zero) {
            for (int i = 0; i < n; i++) outs[i] = ct_zero_new(e, B, 2, l);
        } else {
            const long neN = (long)(l + 1 + e->K) * N;
            View cv = view_of(c);
            const u64* c1 = c->d + cv.ps;
            Tmp ext(e, (size_t)ks_beta(e, l) * B * neN);
            ks_modup(e, c1, cv.bs, B, l, ext.p);
            for (int i = 0; i < n; i++) {
                aesfhe_ct* r = ct_new(e, B, 2, l);
                Opnd add = opnd(cv, B);
                add.np = 1;  // output 0 gets c0
                ks_apply(e, c1, cv.bs, ext.p, B, l, keys[i], add, r, 0);
                aesfhe_ct* o = ct_new(e, B, 2, l);
                Span src = span_s(r->d, (long)(l + 1) * N, l + 1, l + 1, 0, e->Lp1), dst = span_s(o->d, (long)(l + 1) * N, l + 1, l + 1, 0, e->Lp1);
                hipLaunchKernelGGL(k_galois, dim3(N / 256, B * 2 * (l + 1)), dim3(256), 0, e->stream, src, dst, (u64)keys[i]->galois, e->logN, e->Lp1);
                HIPC(hipGetLastError());
                aesfhe_ct_free(r);
                outs[i] = o;
            }
        }
    } catch (...) {
        for (int i = 0; i < n; i++) aesfhe_ct_free(outs[i]), outs[i] = nullptr;
        throw;
    }
    API_END
}

// Baby-step giant-step linear map with lazy ModDown (include/aesfhe.h): babies E_i in Q_l u P,
// per giant one ModDown fused with the rescale, the giant key switches summed in Q_{l-1} u P and
// ModDown'd once.  Against aesfhe_rotate_hoisted + aesfhe_dot_pt + aesfhe_galois it saves one
// ModDown per baby step, one rescale per giant and all but one of the giants' ModDowns.
extern "C" int aesfhe_linear_bsgs(aesfhe_engine* e, const aesfhe_ct* c, int32_t nb, const aesfhe_key* const* bkeys,
                                  int32_t ng, const aesfhe_key* const* gkeys, const int32_t* nterm,
                                  const int32_t* tbaby, const aesfhe_pt* const* pts, aesfhe_ct** out) {
    API_BEGIN
    if (nb < 1 || ng < 1) throw_err(AESFHE_EARG, "linear_bsgs needs baby and giant steps");
    if (c->np != 2) throw_err(AESFHE_EDEGREE, "Input ciphertext should have 2 polynomials");
    const int N = e->N, K = e->K, l = c->level, B = c->B, ne = l + 1 + K;
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a linear map");
    const long neN = (long)ne * N;
    int tot = 0;
    for (int j = 0; j < ng; j++) {
        if (nterm[j] < 1 || nterm[j] > 256) throw_err(AESFHE_EARG, "giant step with %d terms", nterm[j]);
        if (gkeys[j] && gkeys[j]->kind != 3) throw_err(AESFHE_EARG, "giant steps need galois keys");
        tot += nterm[j];
    }
    for (int i = 0; i < nb; i++) {
        if (bkeys[i] && bkeys[i]->kind != 5) throw_err(AESFHE_EARG, "baby steps need hoisted rotation keys");
        check_key_digits(e, bkeys[i], l);
    }
    for (int t = 0; t < tot; t++) {
        if (tbaby[t] < 0 || tbaby[t] >= nb) throw_err(AESFHE_EARG, "bad baby index");
        if (!pts[t] || !pts[t]->ext || pts[t]->level != l) throw_err(AESFHE_EARG, "linear_bsgs needs Q u P plaintexts at the input level");
    }
    if (c->is_zero) {
        *out = ct_zero_new(e, B, 2, l - 1);
        return 0;
    }
    View cv = view_of(c);
    const u64* c1 = c->d + cv.ps;
    Opnd c0 = opnd(cv, B);
    c0.np = 1;  // P * c0 joins accumulator 0 only
    // 1. babies in Q_l u P
    std::vector<std::unique_ptr<Tmp>> E;
    bool any_key = false;
    for (int i = 0; i < nb; i++) any_key |= bkeys[i] != nullptr;
    // fused (AESFHE_BSGS_FUSED=1, bsgs_fused_on): the babies are formed inside the term sums
    // (k_bsgs_terms) from the extension and the keys, never written
    bool only_first_keyless = true;  // k_bsgs_terms peels a key-less (identity) baby at index 0 only
    for (int i = 1; i < nb; i++) only_first_keyless &= bkeys[i] != nullptr;
    const bool fused_terms = bsgs_fused_on() && only_first_keyless;
    std::unique_ptr<Tmp> ext_keep;
    if (fused_terms && any_key) {
        ext_keep.reset(new Tmp(e, (size_t)ks_beta(e, l) * B * neN));
        ks_modup(e, c1, cv.bs, B, l, ext_keep->p);
    }
    if (!fused_terms) {
        std::unique_ptr<Tmp> ext;
        if (any_key) {
            ext.reset(new Tmp(e, (size_t)ks_beta(e, l) * B * neN));
            ks_modup(e, c1, cv.bs, B, l, ext->p);
        }
        std::vector<const u64*> kd;
        std::vector<u64*> ko;
        for (int i = 0; i < nb; i++) {
            E.emplace_back(new Tmp(e, (size_t)B * 2 * neN));
            if (!bkeys[i]) {
                hipLaunchKernelGGL(k_scale_p_ext, dim3(N / 256, ne, B * 2), dim3(256), 0, e->stream, opnd(cv, B), E.back()->p, l, ne, e->q, e->qinv, (const double*)e->pmodf, e->Lp1, e->logN);
                HIPC(hipGetLastError());
                continue;
            }
            kd.push_back((const u64*)bkeys[i]->d);
            ko.push_back(E.back()->p);
        }
        if (!kd.empty()) {
            // every keyed baby's inner product in one launch (the extension read once from HBM);
            // stored unpermuted: the term kernel applies sigma_i as it reads (k_dot_pt_ext_multi)
            const int beta = ks_beta(e, l);
            auto dk = upload_small(e, kd.data(), kd.size());
            auto dko = upload_small(e, ko.data(), ko.size());
            ProfScope ps(e, FAM_KS, 8.0 * N * (double)ne * (beta * B + kd.size() * (2.0 * beta + 2.0 * B)), "ks_inner_multi");
            auto inner = beta <= 4 ? k_ks_inner_multi<4, 4> : beta <= 8 ? k_ks_inner_multi<8, 2> : k_ks_inner_multi<12, 1>;
            hipLaunchKernelGGL(inner, dim3(N / 256, ne, 1), dim3(256), 0, e->stream, c1, cv.bs, (const u64*)ext->p, neN, (long)B * neN, (const u64* const*)dk, (int)kd.size(), 2L * e->np * N, (long)e->np * N, (u64* const*)dko, 2 * neN, neN, B, beta, e->A, l, e->q, e->qinv, e->Lp1, c0, (const double*)e->pmodf, e->logN);
            HIPC(hipGetLastError());
        }
    }
    // 2. giant parts: sum of plaintext products in Q_l u P (every giant in one pass over the
    // babies, kGM at a time), ModDown fused with the rescale
    std::vector<aesfhe_ct*> parts(ng, nullptr);
    aesfhe_ct* sumq = nullptr;
    try {
        constexpr int kGM = 8;
        // the term tables, validated and sized on the host (bsgs_plan.h, ASan-tested)
        std::vector<BsgsChunk> plan;
        {
            std::vector<const void*> pd(tot);
            for (int t = 0; t < tot; t++) pd[t] = pts[t]->d;
            const std::string err = bsgs_plan_terms(nb, ng, nterm, tbaby, pd.data(), kGM, plan);
            if (!err.empty()) throw_err(AESFHE_EARG, "%s", err.c_str());
        }
        std::vector<const u64*> ep(nb);
        std::vector<u64> gal(nb, 0);
        for (int i = 0; i < nb; i++) {
            ep[i] = fused_terms ? (bkeys[i] ? (const u64*)bkeys[i]->d : nullptr) : E[i]->p;  // fused: the baby's key
            gal[i] = bkeys[i] ? bkeys[i]->galois : 0;
        }
        auto dep = upload_small(e, ep.data(), ep.size());
        auto dgal = upload_small(e, gal.data(), gal.size());
        const std::vector<unsigned short> kord = bsgs_block_order(e->logN, gal);
        auto dkord = upload_small(e, kord.data(), kord.size());
        for (const BsgsChunk& ch : plan) {
            const int j0 = ch.j0, gn = ch.gn;
            const double terms = ch.terms;
            std::vector<std::unique_ptr<Tmp>> S;
            std::vector<u64*> so;
            for (int j = 0; j < gn; j++) {
                S.emplace_back(new Tmp(e, (size_t)B * 2 * neN));
                so.push_back(S.back()->p);
            }
            auto dpt = upload_small(e, ch.pt.data(), ch.pt.size());
            auto dso = upload_small(e, so.data(), so.size());
            if (fused_terms) {
                // bytes: the extension (beta words per (b, t, k), read once; the permuted re-reads of
                // the other babies hit cache), c0 / c1, the keys (2 beta words per baby, once per
                // call: shared by the batch) and the plaintexts once, the sums written
                const int beta = ks_beta(e, l);
                ProfScope ps_(e, FAM_EW, 8.0 * N * ne * ((double)B * (beta + 2 + 2.0 * gn) + 2.0 * beta * nb + terms),
                              "bsgs_terms");
                const u64* ex = ext_keep ? (const u64*)ext_keep->p : (const u64*)c->d;  // no keyed baby: never read
                // accumulator pairs GM >= gn, digit words BM = beta exactly, batch block BB (registers
                // 2 BB GM doubles), PB babies' loads in flight together: tools/bsgs_bench.hip timed
                // <2, 3, 4, 2> at 3.07 ms against 3.75 (PB 1), 3.32 (BB 8), 4.00 (PB 3); <4, 3, 4, 2>
                // 4.95 ms against 5.08 (PB 1).  beta > 4 only above the bootstrap's levels.
                using KF = decltype(&k_bsgs_terms<2, 2, 4, 2>);
                auto pick = [&](auto gm) -> KF {
                    constexpr int G = decltype(gm)::value, BBc = G <= 4 ? 4 : 2, PBc = G <= 4 ? 2 : 1;
                    return beta <= 2 ? k_bsgs_terms<G, 2, BBc, PBc> : beta == 3 ? k_bsgs_terms<G, 3, BBc, PBc>
                         : beta == 4 ? k_bsgs_terms<G, 4, BBc, PBc> : k_bsgs_terms<G, 12, 1, 1>;
                };
                KF kern = gn <= 2 ? pick(std::integral_constant<int, 2>{}) : gn <= 4 ? pick(std::integral_constant<int, 4>{})
                                  : pick(std::integral_constant<int, 8>{});
                const int BBv = beta > 4 ? 1 : gn <= 4 ? 4 : 2;
                hipLaunchKernelGGL(kern, dim3((ne * (N / 256) + 7) / 8 * 8 * ((B + BBv - 1) / BBv)), dim3(256), 0, e->stream, (const u64*)c->d, cv.bs, c1,
                                   cv.bs, ex, neN, (long)B * neN, (const u64* const*)dep, (const u64*)dgal, 2L * e->np * N,
                                   (long)e->np * N, (const u64* const*)dpt, nb, gn, (u64* const*)dso, l, ne, beta, e->A, e->q,
                                   e->qinv, (const double*)e->pmodf, e->Lp1, e->logN, B, (const unsigned short*)dkord);
            } else {
                ProfScope ps_(e, FAM_EW, 8.0 * N * ne * ((double)B * 2 * (nb + gn) + terms), "dot_pt_ext_multi");
                // two (b, c) polynomials per workgroup (four measured the same: 153.7 vs 153.3 ms per
                // B = 16 bit bootstrap, 162.7 with one)
                hipLaunchKernelGGL((k_dot_pt_ext_multi<kGM, 2>), dim3((ne * (N / 256) + 7) / 8 * 8 * B), dim3(256), 0, e->stream, (const u64* const*)dep, (const u64*)dgal, (const u64* const*)dpt, nb, gn, (u64* const*)dso, l, ne, e->q, e->qinv, e->Lp1, e->logN, B * 2);
            }
            HIPC(hipGetLastError());
            for (int j = 0; j < gn; j++) {
                parts[j0 + j] = ct_new(e, B, 2, l - 1);
                moddown_acc(e, S[j]->p, B, l, 1, Opnd{nullptr, 0, 0, 0}, parts[j0 + j]);
            }
        }
        E.clear();
        ext_keep.reset();
        // 3. giants: key switches of sigma_j(part_j) summed in Q_{l-1} u P, one ModDown
        const int l2 = l - 1, ne2 = l2 + 1 + K;
        const long ne2N = (long)ne2 * N, l2N = (long)(l2 + 1) * N;
        std::unique_ptr<Tmp> accg;
        const bool fuse = fused_ntt(e);
        int last = -1;  // the last keyed giant: its key switch carries the ModDown (fused_ntt engines)
        for (int j = 0; j < ng; j++)
            if (gkeys[j]) last = j;
        aesfhe_ct* fused_out = nullptr;
        for (int j = 0; j < ng; j++) {
            if (!gkeys[j]) {
                if (!sumq) {
                    sumq = parts[j];
                    parts[j] = nullptr;
                } else {
                    aesfhe_ct* s2 = ct_new(e, B, 2, l2);
                    hipLaunchKernelGGL(k_addsub, ew_grid(e, l2 + 1, B * 2), dim3(256), 0, e->stream, opnd(view_of(sumq), B), opnd(view_of(parts[j]), B), out_of(s2), 2, e->q, 0, e->logN);
                    HIPC(hipGetLastError());
                    aesfhe_ct_free(sumq);
                    sumq = s2;
                }
                continue;
            }
            Tmp sg(e, (size_t)B * 2 * l2N);
            Span src = span_s(parts[j]->d, l2N, l2 + 1, l2 + 1, 0, e->Lp1), dst = span_s(sg.p, l2N, l2 + 1, l2 + 1, 0, e->Lp1);
            hipLaunchKernelGGL(k_galois, dim3(N / 256, B * 2 * (l2 + 1)), dim3(256), 0, e->stream, src, dst, (u64)gkeys[j]->galois, e->logN, e->Lp1);
            HIPC(hipGetLastError());
            Opnd s0{sg.p, 2 * l2N, l2N, 1};
            Tmp ext(e, (size_t)ks_beta(e, l2) * B * ne2N);
            ks_modup(e, sg.p + l2N, 2 * l2N, B, l2, ext.p, fuse);
            const bool first = !accg;
            if (first) accg.reset(new Tmp(e, (size_t)B * 2 * ne2N));
            if (fuse && j == last) {
                // the sum's ModDown by P fused into this key switch's row pass (ks_finish_fused):
                // the kept limbs' accumulators are finished in registers, with sumq added
                fused_out = ct_new(e, B, 2, l2);
                Opnd add = sumq ? opnd(view_of(sumq), B) : Opnd{nullptr, 0, 0, 0};
                try {
                    ks_finish_fused(e, sg.p + l2N, 2 * l2N, ext.p, B, l2, gkeys[j], s0, true, 0, add, fused_out,
                                    nullptr, nullptr, nullptr, accg->p, !first);
                } catch (...) {
                    aesfhe_ct_free(fused_out);
                    throw;
                }
                if (sumq) aesfhe_ct_free(sumq);
                sumq = fused_out;
                continue;
            }
            ks_inner_acc(e, sg.p + l2N, 2 * l2N, ext.p, B, l2, gkeys[j], s0, true, accg->p, fuse, !first);
        }
        if (accg && !fused_out) {
            aesfhe_ct* r = ct_new(e, B, 2, l2);
            Opnd add = sumq ? opnd(view_of(sumq), B) : Opnd{nullptr, 0, 0, 0};
            moddown_acc(e, accg->p, B, l2, 0, add, r);
            if (sumq) aesfhe_ct_free(sumq);
            sumq = r;
        }
    } catch (...) {
        for (auto* p : parts) aesfhe_ct_free(p);
        if (sumq) aesfhe_ct_free(sumq);
        throw;
    }
    for (auto* p : parts) aesfhe_ct_free(p);
    *out = sumq;
    API_END
}

// Power basis of one ciphertext (B = 1, fused-NTT engines) by depth.  The products of depth j,
// x^{2^j + k2} = x^{2^j} * x^{k2} for k2 = 1..m_j (m_j = min(2^j, d - 2^j)), all at level l0 - j,
// run as ONE batched product with x^{2^j} broadcast: the relinearisation key streams once per
// depth instead of once per product, and every launch covers m_j ciphertexts instead of one.
// The depth-j operand block O_j holds slot s = x^{s+1} at level l0 - j (s < 2^j): its upper half
// is depth j-1's product output, written there directly; its lower half is x^{1..2^{j-1}}
// level-downed straight from each power's own level (one batched level-down per source depth,
// written into the block).  O_{j+1} is split in the pool (no copies): its upper half is returned,
// its lower half freed once depth j+1 is enqueued.  Every product and level-down is the
// arithmetic of the sequential basis below (and of oracle/ckks_oracle.c aesfhe_power_basis), so
// each output is bit-identical to it.
static void power_basis_batched(aesfhe_engine* e, const aesfhe_ct* c, int d, const aesfhe_key* rlk, aesfhe_ct** outs) {
    const int N = e->N, l0 = c->level;
    int need = 0;
    while ((1 << need) < d) need++;
    auto pview = [&](const u64* p, int B, int lv) {
        const long ps = (long)(lv + 1) * N;
        return View{p, B, 2, lv, ps, 2 * ps, false};
    };
    for (int k = 0; k < d; k++) outs[k] = nullptr;
    std::vector<aesfhe_ct*> lower, nxt;  // lower halves of O_j (temporaries), parts of O_{j+1}
    auto drop = [&](std::vector<aesfhe_ct*>& v) {
        for (auto* p : v) aesfhe_ct_free(p);
        v.clear();
    };
    try {
        outs[0] = ct_new(e, 1, 2, l0);
        HIPC(hipMemcpyAsync(outs[0]->d, c->d, outs[0]->bytes, hipMemcpyDeviceToDevice, e->stream));
        const u64* opd = c->d;  // slot 0 of O_j (depth 0: x itself)
        for (int j = 0; j < need; j++) {
            const int S = 1 << j, lv = l0 - j, m = std::min(2 * S, d) - S;
            const size_t pw = (size_t)2 * (lv + 1) * N;
            const View va = pview(opd + (size_t)(S - 1) * pw, 1, lv), vb = pview(opd, m, lv);
            if (d > 2 * S) {  // another depth follows: the products fill the upper half of O_{j+1}
                nxt = ct_split_batch(e, ct_new(e, 2 * S, 2, lv - 1), 2 * S);
                aesfhe_ct alias{e, S, 2, lv - 1, 0, nxt[S]->d, 0};
                keyswitch_prod(e, opnd(va, S), opnd(vb, S), S, lv, rlk, &alias, 1);
                for (int t = 0; t < S; t++) outs[S + t] = nxt[S + t], nxt[S + t] = nullptr;
                nxt.resize(S);
                drop(lower);  // O_j's level-downed half: its last reader is enqueued
                // O_{j+1}'s lower half: x^{1..min(S, m_{j+1})} at level lv - 1, per source depth i
                // (x^{lo..hi} at level l0 - i) one batched level-down into the block
                const int mnext = std::min(4 * S, d) - 2 * S;
                for (int i = 0; i <= j; i++) {
                    const int lo = i ? (1 << (i - 1)) + 1 : 1, hi = std::min(1 << i, mnext);
                    if (hi < lo) break;
                    const int sl = l0 - i;
                    rescale_view(e, truncated(pview(outs[lo - 1]->d, hi - lo + 1, sl), lv), level_down_const(e, sl, lv - 1),
                                 nxt[lo - 1]->d);
                }
                lower.swap(nxt);
                opd = lower[0]->d;
            } else {  // last depth: the m outputs as one block, split
                aesfhe_ct* r = ct_new(e, m, 2, lv - 1);
                try {
                    keyswitch_prod(e, opnd(va, m), opnd(vb, m), m, lv, rlk, r, 1);
                } catch (...) {
                    aesfhe_ct_free(r);
                    throw;
                }
                std::vector<aesfhe_ct*> parts = m > 1 ? ct_split_batch(e, r, m) : std::vector<aesfhe_ct*>{r};
                for (int t = 0; t < m; t++) outs[S + t] = parts[t];
                drop(lower);
            }
        }
    } catch (...) {
        drop(lower);
        drop(nxt);
        for (int k = 0; k < d; k++) aesfhe_ct_free(outs[k]), outs[k] = nullptr;
        throw;
    }
}

extern "C" int aesfhe_power_basis(aesfhe_engine* e, const aesfhe_ct* c, int32_t d, const aesfhe_key* rlk, aesfhe_ct** outs) {
    API_BEGIN
    if (d < 1) throw_err(AESFHE_EARG, "degree must be >= 1");
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "power basis needs a relinearization key");
    if (c->np != 2) throw_err(AESFHE_EDEGREE, "power basis input should have 2 polynomials");
    int need = 0;
    while ((1 << need) < d) need++;
    if (c->level < need) throw_err(AESFHE_ELEVEL, "power basis of degree %d needs %d levels, have %d", d, need, c->level);
    if (d >= 2 && c->B == 1 && !c->is_zero && fused_ntt(e) && e->K + 1 <= kMdrMaxE) {
        power_basis_batched(e, c, d, rlk, outs);
        return AESFHE_OK;
    }
    std::vector<aesfhe_ct*> pw(d + 1, nullptr);
    // memo of level-downed powers: (k, level) -> ct
    std::map<std::pair<int, int>, aesfhe_ct*> memo;
    try {
        aesfhe_ct_copy(e, c, &pw[1]);
        auto at_level = [&](int k, int lv) -> aesfhe_ct* {
            if (pw[k]->level == lv) return pw[k];
            auto key = std::make_pair(k, lv);
            auto it = memo.find(key);
            if (it != memo.end()) return it->second;
            aesfhe_ct* x = level_down_view(e, view_of(pw[k]), lv);
            memo[key] = x;
            return x;
        };
        for (int k = 2; k <= d; k++) {
            int hi = 1;
            while (hi * 2 <= k) hi *= 2;
            int k1 = (hi == k) ? k / 2 : hi, k2 = (hi == k) ? k / 2 : k - hi;
            int lv = std::min(pw[k1]->level, pw[k2]->level);
            pw[k] = mul_ct(e, at_level(k1, lv), at_level(k2, lv), rlk);
        }
    } catch (...) {
        for (auto* p : pw) aesfhe_ct_free(p);
        for (auto& kv : memo) aesfhe_ct_free(kv.second);
        throw;
    }
    for (auto& kv : memo) aesfhe_ct_free(kv.second);
    for (int k = 1; k <= d; k++) outs[k - 1] = pw[k];
    API_END
}

extern "C" int aesfhe_lincomb(aesfhe_engine* e, const aesfhe_ct* const* cts, int32_t n, const double* re, const double* im, aesfhe_ct** out) {
    API_BEGIN
    if (n < 1) throw_err(AESFHE_EARG, "empty linear combination");
    if (n > 4096) throw_err(AESFHE_EARG, "linear combination too long");
    int l = cts[0]->level, B = 1, np = 2;
    for (int i = 0; i < n; i++) {
        l = std::min(l, cts[i]->level);
        B = std::max(B, cts[i]->B);
        np = std::max(np, cts[i]->np);
    }
    for (int i = 0; i < n; i++)
        if (cts[i]->B != B && cts[i]->B != 1) throw_err(AESFHE_EARG, "batch mismatch");
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a linear combination");
    const int nl = l + 1;
    const double s = aesfhe_engine_mul_scale(e, l);
    // gather the contributing inputs, each aligned to level l
    std::vector<std::unique_ptr<Aligned>> al;
    std::vector<const u64*> ptrs;
    std::vector<long> bstr;
    std::vector<int> npi;
    std::vector<u64> f;
    std::vector<double> ff;
    std::vector<long> pss;
    for (int i = 0; i < n; i++) {
        // inputs above l are truncated to its limbs, their scale compensated in the constant
        const double si = s * (e->chain.scale[l] / e->chain.scale[cts[i]->level]);
        int64_t A = llround(re[i] * si), Bc = llround(im[i] * si);
        if (cts[i]->is_zero || (A == 0 && Bc == 0)) continue;
        const View v = trunc_view(cts[i], l);
        ptrs.push_back(v.d);
        bstr.push_back(v.B == 1 && B > 1 ? 0 : v.bs);
        pss.push_back(v.ps);
        npi.push_back(v.np);
        std::vector<u64> fi;
        std::vector<double> ffi;
        const_factors(e, A, Bc, nl, fi, ffi);
        f.insert(f.end(), fi.begin(), fi.end());
        ff.insert(ff.end(), ffi.begin(), ffi.end());
    }
    if (ptrs.empty()) {
        *out = ct_zero_new(e, B, np, l - 1);
    } else {
        const int m = (int)ptrs.size();
        aesfhe_ct* acc = ct_new(e, B, np, l);
        auto dp = upload_small(e, ptrs.data(), ptrs.size());
        auto db = upload_small(e, bstr.data(), bstr.size());
        auto dps = upload_small(e, pss.data(), pss.size());
        auto dn = upload_small(e, npi.data(), npi.size());
        auto df = upload_small(e, f.data(), f.size());
        auto dff = upload_small(e, ff.data(), ff.size());
        {
            ProfScope ps_(e, FAM_EW, 8.0 * e->N * nl * (double)B * np * (m + 1), "lincomb");
            hipLaunchKernelGGL(k_lincomb, ew_grid(e, nl, B * np), dim3(256), 0, e->stream, (const u64* const*)dp, (const long*)db, (const int*)dn, m, (const long*)dps, (const u64*)df, (const double*)dff, out_of(acc), np, nl, e->q, e->qinv, e->logN);
        }
        HIPC(hipGetLastError());
        *out = rescale_view(e, view_of(acc));
        aesfhe_ct_free(acc);
    }
    API_END
}

extern "C" int aesfhe_lincomb_many(aesfhe_engine* e, const aesfhe_ct* const* cts, int32_t n, const double* re, const double* im, int32_t m, aesfhe_ct** outs) {
    if (n > kManyMax || m < 1) {
        for (int r = 0; r < m; r++) {
            int rc = aesfhe_lincomb(e, cts, n, re + (size_t)r * n, im + (size_t)r * n, &outs[r]);
            if (rc) return rc;
        }
        return 0;
    }
    API_BEGIN
    if (n < 1) throw_err(AESFHE_EARG, "empty linear combination");
    int l = cts[0]->level, B = 1, np = 2;
    for (int i = 0; i < n; i++) {
        l = std::min(l, cts[i]->level);
        B = std::max(B, cts[i]->B);
        np = std::max(np, cts[i]->np);
    }
    for (int i = 0; i < n; i++)
        if (cts[i]->B != B && cts[i]->B != 1) throw_err(AESFHE_EARG, "batch mismatch");
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a linear combination");
    const int nl = l + 1;
    const double s = aesfhe_engine_mul_scale(e, l);
    // rows whose constants all round to zero (or whose inputs are all zero) are zero outputs
    std::vector<int> live;
    std::vector<char> used(n, 0);
    for (int r = 0; r < m; r++) {
        bool any = false;
        for (int i = 0; i < n; i++) {
            const double si = s * (e->chain.scale[l] / e->chain.scale[cts[i]->level]);
            int64_t A = llround(re[(size_t)r * n + i] * si), Bc = llround(im[(size_t)r * n + i] * si);
            if (!cts[i]->is_zero && (A || Bc)) any = true, used[i] = 1;
        }
        if (any) live.push_back(r);
        else outs[r] = nullptr;
    }
    std::vector<int> cols;
    for (int i = 0; i < n; i++)
        if (used[i]) cols.push_back(i);
    std::vector<std::unique_ptr<Aligned>> al;
    std::vector<const u64*> ptrs;
    std::vector<long> bstr;
    std::vector<int> npi;
    std::vector<long> pss;
    for (int i : cols) {  // truncated to level l (scale compensated in F below)
        const View v = trunc_view(cts[i], l);
        ptrs.push_back(v.d);
        bstr.push_back(v.B == 1 && B > 1 ? 0 : v.bs);
        pss.push_back(v.ps);
        npi.push_back(v.np);
    }
    const int nc = (int)cols.size(), ml = (int)live.size();
    if (ml > 0) {
        std::vector<u64> F((size_t)ml * nc * nl * 2);
        std::vector<double> FF(F.size());
        for (int r = 0; r < ml; r++)
            for (int c = 0; c < nc; c++) {
                const size_t idx = (size_t)live[r] * n + cols[c];
                const double si = s * (e->chain.scale[l] / e->chain.scale[cts[cols[c]]->level]);
                int64_t A = llround(re[idx] * si), Bc = llround(im[idx] * si);
                if (cts[cols[c]]->is_zero) A = Bc = 0;
                std::vector<u64> fi;
                std::vector<double> ffi;
                const_factors(e, A, Bc, nl, fi, ffi);
                std::copy(fi.begin(), fi.end(), F.begin() + ((size_t)r * nc + c) * nl * 2);
                std::copy(ffi.begin(), ffi.end(), FF.begin() + ((size_t)r * nc + c) * nl * 2);
            }
        const long ps = (long)nl * e->N, obs = (long)np * ps, orow = (long)B * obs;
        Tmp acc(e, (size_t)ml * orow);
        auto dp = upload_small(e, ptrs.data(), ptrs.size());
        auto db = upload_small(e, bstr.data(), bstr.size());
        auto dps = upload_small(e, pss.data(), pss.size());
        auto dn = upload_small(e, npi.data(), npi.size());
        auto dF = upload_small(e, F.data(), F.size());
        auto dFF = upload_small(e, FF.data(), FF.size());
        {
            ProfScope ps_(e, FAM_EW, 8.0 * e->N * nl * (double)B * np * (nc + ml), "lincomb_many");
            hipLaunchKernelGGL(k_lincomb_many, ew_grid(e, nl, B * np), dim3(256), 0, e->stream, (const u64* const*)dp, (const long*)db, (const int*)dn, nc, (const long*)dps, (const u64*)dF, (const double*)dFF, ml, acc.p, orow, obs, np, nl, e->q, e->qinv, e->logN);
        }
        HIPC(hipGetLastError());
        std::vector<aesfhe_ct*> res = rescale_groups(e, acc.p, ml, B, np, l);
        for (int r = 0; r < ml; r++) outs[live[r]] = res[r];
    }
    for (int r = 0; r < m; r++)
        if (!outs[r]) outs[r] = ct_zero_new(e, B, np, l - 1);
    API_END
}

extern "C" int aesfhe_dot(aesfhe_engine* e, const aesfhe_ct* const* a, const aesfhe_ct* const* b, int32_t n, const aesfhe_key* rlk, aesfhe_ct** out) {
    API_BEGIN
    if (n < 1) throw_err(AESFHE_EARG, "empty dot product");
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "dot needs a relinearization key");
    int l = a[0]->level, B = 1;
    for (int i = 0; i < n; i++) {
        if (a[i]->np != 2 || b[i]->np != 2) throw_err(AESFHE_EDEGREE, "dot inputs should have 2 polynomials");
        l = std::min(l, std::min(a[i]->level, b[i]->level));
        B = std::max(B, std::max(a[i]->B, b[i]->B));
    }
    for (int i = 0; i < n; i++)
        if ((a[i]->B != B && a[i]->B != 1) || (b[i]->B != B && b[i]->B != 1)) throw_err(AESFHE_EARG, "batch mismatch");
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a dot product");
    const int nl = l + 1;
    std::vector<std::unique_ptr<Aligned>> al;
    std::vector<const u64*> pa, pb;
    std::vector<long> sa, sb;
    for (int i = 0; i < n; i++) {
        if (a[i]->is_zero || b[i]->is_zero) continue;
        al.emplace_back(new Aligned());
        align_to(e, a[i], l, *al.back());
        const View va = al.back()->v;
        al.emplace_back(new Aligned());
        align_to(e, b[i], l, *al.back());
        const View vb = al.back()->v;
        pa.push_back(va.d);
        pb.push_back(vb.d);
        sa.push_back(va.B == 1 && B > 1 ? 0 : va.bs);
        sb.push_back(vb.B == 1 && B > 1 ? 0 : vb.bs);
    }
    if (pa.empty()) {
        *out = ct_zero_new(e, B, 2, l - 1);
    } else {
        const int m = (int)pa.size();
        aesfhe_ct* acc = ct_new(e, B, 3, l);
        auto dpa = upload_small(e, pa.data(), pa.size());
        auto dpb = upload_small(e, pb.data(), pb.size());
        auto dsa = upload_small(e, sa.data(), sa.size());
        auto dsb = upload_small(e, sb.data(), sb.size());
        {
            ProfScope ps_(e, FAM_EW, 8.0 * e->N * nl * (double)B * (4.0 * m + 3), "dot");
            hipLaunchKernelGGL(k_dot, ew_grid(e, nl, B), dim3(256), 0, e->stream, (const u64* const*)dpa, (const long*)dsa, (const u64* const*)dpb, (const long*)dsb, m, (long)nl * e->N, out_of(acc), e->q, e->qinv, e->logN);
        }
        HIPC(hipGetLastError());
        *out = relin_rescale(e, acc, rlk, 1);
        aesfhe_ct_free(acc);
    }
    API_END
}

// sum_i a_i b_i + sum_j gamma_j c_j + beta, one relinearisation + rescale (include/aesfhe.h
// aesfhe_dot_fma): the k_dot tensor sum and the addends on d0 / d1 in one pass (k_dot_fma),
// then relin_rescale.  Bit-identical to the oracle's term-by-term sum.
extern "C" int aesfhe_dot_fma(aesfhe_engine* e, const aesfhe_ct* const* a, const aesfhe_ct* const* b, int32_t n,
                              const aesfhe_ct* const* c, const double* gamma, int32_t nc, double beta,
                              const aesfhe_key* rlk, aesfhe_ct** out) {
    API_BEGIN
    if (n < 1) throw_err(AESFHE_EARG, "empty dot product");
    if (nc < 0) throw_err(AESFHE_EARG, "negative addend count");
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "dot needs a relinearization key");
    int l = a[0]->level, B = 1;
    for (int i = 0; i < n; i++) {
        if (a[i]->np != 2 || b[i]->np != 2) throw_err(AESFHE_EDEGREE, "dot inputs should have 2 polynomials");
        l = std::min(l, std::min(a[i]->level, b[i]->level));
        B = std::max(B, std::max(a[i]->B, b[i]->B));
    }
    for (int j = 0; j < nc; j++) {
        if (c[j]->np != 2) throw_err(AESFHE_EDEGREE, "dot_fma addends should have 2 polynomials");
        B = std::max(B, c[j]->B);
    }
    for (int j = 0; j < nc; j++)
        if (c[j]->level < l) throw_err(AESFHE_ELEVEL, "dot_fma addend level %d below the product level %d", c[j]->level, l);
    for (int i = 0; i < n; i++)
        if ((a[i]->B != B && a[i]->B != 1) || (b[i]->B != B && b[i]->B != 1)) throw_err(AESFHE_EARG, "batch mismatch");
    for (int j = 0; j < nc; j++)
        if (c[j]->B != B && c[j]->B != 1) throw_err(AESFHE_EARG, "batch mismatch");
    if (l < 1) throw_err(AESFHE_ELEVEL, "no level left for a dot product");
    const int nl = l + 1;
    std::vector<std::unique_ptr<Aligned>> al;
    std::vector<const u64*> pa, pb;
    std::vector<long> sa, sb;
    for (int i = 0; i < n; i++) {
        if (a[i]->is_zero || b[i]->is_zero) continue;
        al.emplace_back(new Aligned());
        align_to(e, a[i], l, *al.back());
        const View va = al.back()->v;
        al.emplace_back(new Aligned());
        align_to(e, b[i], l, *al.back());
        const View vb = al.back()->v;
        pa.push_back(va.d);
        pb.push_back(vb.d);
        sa.push_back(va.B == 1 && B > 1 ? 0 : va.bs);
        sb.push_back(vb.B == 1 && B > 1 ? 0 : vb.bs);
    }
    // addends: truncated views, C_j per limb
    const double* D = e->chain.scale.data();
    std::vector<const u64*> cp;
    std::vector<long> cbs, cps;
    std::vector<u64> cf;
    for (int j = 0; j < nc; j++) {
        const int64_t Cc = llround(gamma[j] * (D[l] * (D[l] / D[c[j]->level])));
        if (c[j]->is_zero || Cc == 0) continue;
        const View v = trunc_view(c[j], l);
        cp.push_back(v.d);
        cbs.push_back(v.B == 1 && B > 1 ? 0 : v.bs);
        cps.push_back(v.ps);
        for (int i = 0; i < nl; i++) cf.push_back(h_smod(Cc, e->chain.q[i]));
    }
    const int64_t Rb = llround(beta * D[l]), R = llround(D[l]);
    std::vector<u64> km(nl);
    for (int i = 0; i < nl; i++) {
        const u64 q = e->chain.q[i];
        km[i] = h_mulmod(h_smod(Rb, q), h_smod(R, q), q);
    }
    aesfhe_ct* acc = ct_new(e, B, 3, l);
    try {
        const int m = (int)pa.size(), mc = (int)cp.size();
        const u64* const* dpa = m ? (const u64* const*)upload_small(e, pa.data(), pa.size()) : nullptr;
        const u64* const* dpb = m ? (const u64* const*)upload_small(e, pb.data(), pb.size()) : nullptr;
        const long* dsa = m ? upload_small(e, sa.data(), sa.size()) : nullptr;
        const long* dsb = m ? upload_small(e, sb.data(), sb.size()) : nullptr;
        const u64* const* dcp = mc ? (const u64* const*)upload_small(e, cp.data(), cp.size()) : nullptr;
        const long* dcb = mc ? upload_small(e, cbs.data(), cbs.size()) : nullptr;
        const long* dcs = mc ? upload_small(e, cps.data(), cps.size()) : nullptr;
        const u64* dcf = mc ? upload_small(e, cf.data(), cf.size()) : nullptr;
        const u64* dkm = upload_small(e, km.data(), km.size());
        {
            ProfScope ps_(e, FAM_EW, 8.0 * e->N * nl * (double)B * (4.0 * m + 2.0 * mc + 3), "dot");
            hipLaunchKernelGGL(k_dot_fma, ew_grid(e, nl, B), dim3(256), 0, e->stream, dpa, dsa, dpb, dsb, m, (long)nl * e->N,
                               dcp, dcb, dcs, mc, dcf, dkm, nl, out_of(acc), e->q, e->qinv, e->logN);
        }
        HIPC(hipGetLastError());
        *out = relin_rescale(e, acc, rlk, 1);
    } catch (...) {
        aesfhe_ct_free(acc);
        throw;
    }
    aesfhe_ct_free(acc);
    API_END
}

// Bivariate polynomial with shared power bases (fused BSGS):
//   out_t = sum_{i<nx, j<ny} C[t][i][j] x^i y^j,   xb = x^1..x^{nx-1}, yb = y^1..y^{ny-1}.
// Constants carry the integer scale S1 = Delta_{l-2} q_l q_{l-1} / Delta_l^2 (x^0, y^0 terms
// also R = round(Delta_l) per missing basis factor), so the inner sums are never rescaled: one
// tensor pass (k_poly2), one batched relinearisation of all m*B outputs, then two rescales land
// exactly on the canonical scale Delta_{l-2}.  Inputs above level l are truncated (limbs 0..l
// read in place, no rescale); their scale Delta_lev is compensated in the constants by the
// factor Delta_l / Delta_lev.  Constant rules: oracle/ckks_oracle.c aesfhe_poly2.
static TwD* poly2_table(aesfhe_engine* e, int l, int nx, int ny, int m, const std::vector<int64_t>& A,
                       const std::vector<int64_t>& Bc, int64_t R) {
    std::string key((const char*)&l, sizeof l);
    key.append((const char*)&nx, sizeof nx).append((const char*)&ny, sizeof ny).append((const char*)&m, sizeof m);
    key.append((const char*)A.data(), A.size() * 8).append((const char*)Bc.data(), Bc.size() * 8);
    auto it = e->poly2_tabs.find(key);
    if (it != e->poly2_tabs.end()) return it->second;
    if (e->poly2_tabs.size() >= 256) {
        HIPC(hipStreamSynchronize(e->stream));
        for (auto& kv : e->poly2_tabs) HIPC(hipFree(kv.second));
        e->poly2_tabs.clear();
    }
    const int nl = l + 1;
    const size_t per = (size_t)m * nx * ny;
    std::vector<TwD> T((size_t)nl * 2 * per);
    for (int li = 0; li < nl; li++) {
        const u64 q = e->chain.q[li];
        const u64 r1 = h_smod(R, q), r2 = h_mulmod(r1, r1, q), I = e->h_iroot[li];
        for (size_t c = 0; c < per; c++) {
            const int j = (int)(c % ny), i = (int)((c / ny) % nx);
            const u64 t = (i == 0 && j == 0) ? r2 : (i == 0 || j == 0) ? r1 : 1;
            const u64 a = h_mulmod(h_smod(A[c], q), t, q), b = h_mulmod(h_smod(Bc[c], q), t, q);
            const u64 bi = h_mulmod(b, I, q);
            const u64 f0 = h_addmod(a, bi, q), f1 = h_submod(a, bi, q);
            T[((size_t)li * 2 + 0) * per + c] = TwD{(double)f0, (double)f0 / (double)q};
            T[((size_t)li * 2 + 1) * per + c] = TwD{(double)f1, (double)f1 / (double)q};
        }
    }
    TwD* d = nullptr;
    HIPC(hipMalloc(&d, T.size() * sizeof(TwD)));
    HIPC(hipMemcpy(d, T.data(), T.size() * sizeof(TwD), hipMemcpyHostToDevice));
    e->poly2_tabs.emplace(key, d);
    return d;
}

extern "C" int aesfhe_poly2(aesfhe_engine* e, const aesfhe_ct* const* xb, int32_t nx, const aesfhe_ct* const* yb, int32_t ny, const double* re, const double* im, int32_t m, const aesfhe_key* rlk, aesfhe_ct** outs) {
    API_BEGIN
    if (nx < 1 || ny < 1 || nx > kPoly2Max || ny > kPoly2Max || m < 1)
        throw_err(AESFHE_EARG, "poly2 needs 1 <= nx, ny <= %d and m >= 1", kPoly2Max);
    if (nx + ny < 3) throw_err(AESFHE_EARG, "poly2 needs at least one basis ciphertext");
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "poly2 needs a relinearization key");
    std::vector<const aesfhe_ct*> all;
    for (int i = 0; i < nx - 1; i++) all.push_back(xb[i]);
    for (int j = 0; j < ny - 1; j++) all.push_back(yb[j]);
    int l = all[0]->level, B = 1;
    for (auto* c : all) {
        if (c->np != 2) throw_err(AESFHE_EDEGREE, "poly2 inputs should have 2 polynomials");
        if (c->is_zero) throw_err(AESFHE_EARG, "poly2 basis ciphertext is zero");
        l = std::min(l, c->level);
        B = std::max(B, c->B);
    }
    for (auto* c : all)
        if (c->B != B && c->B != 1) throw_err(AESFHE_EARG, "batch mismatch");
    if (l < 2) throw_err(AESFHE_ELEVEL, "no level left for a bivariate polynomial");
    const int nl = l + 1, N = e->N;
    const double* D = e->chain.scale.data();
    const double S1 = D[l - 2] / D[l] * ((double)e->chain.q[l] / D[l]) * (double)e->chain.q[l - 1];
    const int64_t R = llround(D[l]);
    const size_t per = (size_t)nx * ny;
    std::vector<double> rx(nx, 1.0), ry(ny, 1.0);
    for (int i = 1; i < nx; i++) rx[i] = D[l] / D[xb[i - 1]->level];
    for (int j = 1; j < ny; j++) ry[j] = D[l] / D[yb[j - 1]->level];
    auto coef = [&](const double* v, int t, size_t c) {
        return llround(v[t * per + c] * S1 * rx[c / ny] * ry[c % ny]);
    };
    std::vector<int> live;
    std::vector<int64_t> A, Bc;
    for (int t = 0; t < m; t++) {
        bool any = false;
        for (size_t c = 0; c < per; c++)
            if (coef(re, t, c) || coef(im, t, c)) any = true;
        if (!any) {
            outs[t] = nullptr;
            continue;
        }
        live.push_back(t);
        for (size_t c = 0; c < per; c++) {
            A.push_back(coef(re, t, c));
            Bc.push_back(coef(im, t, c));
        }
    }
    const int ml = (int)live.size();
    if (ml > 0) {
        std::vector<const u64*> px, py;
        std::vector<long> sx, sy, qx, qy;
        for (size_t a = 0; a < all.size(); a++) {
            const View v = view_of(all[a]);  // truncation: limbs 0..l read in place
            if (v.B > 1 && v.bs != (long)v.np * v.ps) throw_err(AESFHE_EARG, "poly2: non-compact basis view");
            const long bs = v.B == 1 && B > 1 ? 0 : v.bs;
            if ((int)a < nx - 1) px.push_back(v.d), sx.push_back(bs), qx.push_back(v.ps);
            else py.push_back(v.d), sy.push_back(bs), qy.push_back(v.ps);
        }
        if (px.empty()) px.push_back(nullptr), sx.push_back(0), qx.push_back(0);
        if (py.empty()) py.push_back(nullptr), sy.push_back(0), qy.push_back(0);
        const TwD* tab = poly2_table(e, l, nx, ny, ml, A, Bc, R);
        auto dpx = upload_small(e, px.data(), px.size());
        auto dpy = upload_small(e, py.data(), py.size());
        auto dsx = upload_small(e, sx.data(), sx.size());
        auto dsy = upload_small(e, sy.data(), sy.size());
        auto dqx = upload_small(e, qx.data(), qx.size());
        auto dqy = upload_small(e, qy.data(), qy.size());
        const int Bt = ml * B;
        const long obs = 3L * nl * N;
        aesfhe_ct* d3 = ct_new(e, Bt, 3, l);
        {
            ProfScope ps_(e, FAM_EW, 8.0 * N * nl * (double)B * (2.0 * (nx + ny - 2) + 3.0 * ml), "poly2");
            for (int t0 = 0; t0 < ml; t0 += kPoly2Out)
                hipLaunchKernelGGL(k_poly2, ew_grid(e, nl, B), dim3(256), 0, e->stream, (const u64* const*)dpx, (const long*)dsx, (const long*)dqx, nx, (const u64* const*)dpy, (const long*)dsy, (const long*)dqy, ny, tab, ml, t0, std::min(kPoly2Out, ml - t0), d3->d, (long)B * obs, obs, e->q, e->qinv, e->logN);
        }
        HIPC(hipGetLastError());
        aesfhe_ct* r2 = relin_rescale(e, d3, rlk, 2);
        aesfhe_ct_free(d3);
        std::vector<aesfhe_ct*> parts = ct_split_batch(e, r2, ml);  // no copies
        for (int t = 0; t < ml; t++) outs[live[t]] = parts[t];
    }
    for (int t = 0; t < m; t++)
        if (!outs[t]) outs[t] = ct_zero_new(e, B, 2, l - 2);
    API_END
}

// Integer-weight bivariate polynomial: out_t = sum_{i,j} (w[t][i][j] / den) x^i y^j (the Walsh
// spectra of Boolean functions are of this form).  Constant rule (oracle: aesfhe_poly2_int):
// classes cx(i) = 0 for i = 0, else 1 + rank of level(x^i) among the distinct x levels (highest
// first); cy likewise.  H(cx, cy) = llround(S1 * r_x * r_y / den) mod q, times R = llround(D_l)
// for cx = 0 and again for cy = 0, with S1, r_x, r_y as in aesfhe_poly2; F_ij = w_ij * H mod q.
// Output: level l - 2, scale exactly D_{l-2} (up to the rounding of H).
static void poly2_int_impl(aesfhe_engine* e, const aesfhe_ct* const* xb, int32_t nx, const aesfhe_ct* const* yb,
                           int32_t ny, const int32_t* w, int32_t den, int32_t m, const aesfhe_key* rlk,
                           aesfhe_ct** outs, int slab_rot);
extern "C" int aesfhe_poly2_int(aesfhe_engine* e, const aesfhe_ct* const* xb, int32_t nx, const aesfhe_ct* const* yb, int32_t ny, const int32_t* w, int32_t den, int32_t m, const aesfhe_key* rlk, aesfhe_ct** outs) {
    API_BEGIN
    poly2_int_impl(e, xb, nx, yb, ny, w, den, m, rlk, outs, 0);
    API_END
}
// the same with every output's batch rotated within slabs of 4: element 4 s + c of output t takes
// the polynomial's value at input element 4 s + ((c + slab_rot) mod 4) (the sliced AES state's
// ShiftRows of row r = slab_rot folded into its S-box)
extern "C" int aesfhe_poly2_int_rot(aesfhe_engine* e, const aesfhe_ct* const* xb, int32_t nx, const aesfhe_ct* const* yb, int32_t ny, const int32_t* w, int32_t den, int32_t m, const aesfhe_key* rlk, int32_t slab_rot, aesfhe_ct** outs) {
    API_BEGIN
    if (slab_rot < 0 || slab_rot > 3) throw_err(AESFHE_EARG, "slab rotation %d outside 0..3", slab_rot);
    poly2_int_impl(e, xb, nx, yb, ny, w, den, m, rlk, outs, slab_rot);
    API_END
}
static void poly2_int_impl(aesfhe_engine* e, const aesfhe_ct* const* xb, int32_t nx, const aesfhe_ct* const* yb,
                           int32_t ny, const int32_t* w, int32_t den, int32_t m, const aesfhe_key* rlk,
                           aesfhe_ct** outs, int slab_rot) {
    if (nx < 1 || ny < 1 || nx > kPoly2Max || ny > kPoly2Max || m < 1)
        throw_err(AESFHE_EARG, "poly2 needs 1 <= nx, ny <= %d and m >= 1", kPoly2Max);
    if (nx + ny < 3) throw_err(AESFHE_EARG, "poly2 needs at least one basis ciphertext");
    if (den < 1) throw_err(AESFHE_EARG, "poly2_int needs den >= 1");
    if (!rlk || rlk->kind != 2) throw_err(AESFHE_EARG, "poly2 needs a relinearization key");
    int l = INT32_MAX, B = 1;
    auto check = [&](const aesfhe_ct* c) {
        if (c->np != 2) throw_err(AESFHE_EDEGREE, "poly2 inputs should have 2 polynomials");
        if (c->is_zero) throw_err(AESFHE_EARG, "poly2 basis ciphertext is zero");
        l = std::min(l, c->level);
        B = std::max(B, c->B);
    };
    for (int i = 0; i < nx - 1; i++) check(xb[i]);
    for (int j = 0; j < ny - 1; j++) check(yb[j]);
    for (int i = 0; i < nx - 1; i++)
        if (xb[i]->B != B && xb[i]->B != 1) throw_err(AESFHE_EARG, "batch mismatch");
    for (int j = 0; j < ny - 1; j++)
        if (yb[j]->B != B && yb[j]->B != 1) throw_err(AESFHE_EARG, "batch mismatch");
    if (l < 2) throw_err(AESFHE_ELEVEL, "no level left for a bivariate polynomial");
    if (slab_rot && B % 4) throw_err(AESFHE_EARG, "slab rotation needs a batch of whole slabs (4 s), got %d", B);
    // wfac bounds an inner sum a = w_0 c0 + sum_j w_j y'_j (c0 < q, |y'| <= q/2 + 1) by wfac * q:
    // a limb takes the exact-FMA kernel (no folds) when wfac * q < 2^52, else the folding one
    double wfac = 1.0;
    for (int t = 0; t < m; t++)
        for (int i = 0; i < nx; i++) {
            long sum = 0;
            double f = 0.0;
            for (int j = 0; j < ny; j++) {
                const long a = std::labs((long)w[((size_t)t * nx + i) * ny + j]);
                sum += a;
                f += j == 0 ? (double)a : 0.5 * (double)a + 1e-3 * (double)a;
            }
            if (sum > 512) throw_err(AESFHE_EARG, "poly2_int: sum of |w| over a row exceeds 512");
            wfac = std::max(wfac, f);
        }
    const int nl = l + 1, N = e->N;
    const double* D = e->chain.scale.data();
    const double S1 = D[l - 2] / D[l] * ((double)e->chain.q[l] / D[l]) * (double)e->chain.q[l - 1];
    const int64_t R = llround(D[l]);
    // classes by level (highest first); y sorted so each class is a contiguous run of j
    auto classes = [&](const aesfhe_ct* const* b, int n, std::vector<int>& cls, std::vector<int>& lev) {
        lev.clear();
        for (int i = 0; i < n - 1; i++)
            if (std::find(lev.begin(), lev.end(), b[i]->level) == lev.end()) lev.push_back(b[i]->level);
        std::sort(lev.rbegin(), lev.rend());
        cls.assign(n, 0);
        for (int i = 1; i < n; i++) cls[i] = 1 + (int)(std::find(lev.begin(), lev.end(), b[i - 1]->level) - lev.begin());
    };
    std::vector<int> cx, cy0, lx, ly;
    classes(xb, nx, cx, lx);
    classes(yb, ny, cy0, ly);
    std::vector<int> perm(ny), permx(nx);  // perm[j'] = original j (classes contiguous)
    for (int j = 0; j < ny; j++) perm[j] = j;
    for (int i = 0; i < nx; i++) permx[i] = i;
    std::stable_sort(perm.begin() + 1, perm.end(), [&](int a, int b) { return cy0[a] < cy0[b]; });
    std::stable_sort(permx.begin() + 1, permx.end(), [&](int a, int b) { return cx[a] < cx[b]; });
    std::vector<int> cy(ny), cxs(nx);
    for (int j = 0; j < ny; j++) cy[j] = cy0[perm[j]];
    for (int i = 0; i < nx; i++) cxs[i] = cx[permx[i]];
    const int cxn = 1 + (int)lx.size(), cyn = 1 + (int)ly.size();
    // weights (permuted), live outputs
    std::vector<int> live;
    std::vector<double> Wt;
    for (int t = 0; t < m; t++) {
        bool any = false;
        for (size_t c = 0; c < (size_t)nx * ny; c++) any |= w[(size_t)t * nx * ny + c] != 0;
        if (!any) {
            outs[t] = nullptr;
            continue;
        }
        live.push_back(t);
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < ny; j++) Wt.push_back((double)w[((size_t)t * nx + permx[i]) * ny + perm[j]]);
    }
    const int ml = (int)live.size();
    if (ml > 0) {
        // y' factors Rt[c][cy] = H(c, cy), C0[c] = H(c, 0)
        std::vector<TwD> Rt((size_t)nl * cxn * cyn);
        std::vector<double> C0((size_t)nl * cxn);
        for (int li = 0; li < nl; li++) {
            const u64 q = e->chain.q[li];
            const u64 r1 = h_smod(R, q);
            std::vector<u64> H((size_t)cxn * cyn);
            for (int a = 0; a < cxn; a++)
                for (int b = 0; b < cyn; b++) {
                    const double rx = a == 0 ? 1.0 : D[l] / D[lx[a - 1]];
                    const double ry = b == 0 ? 1.0 : D[l] / D[ly[b - 1]];
                    u64 h = h_smod(llround(S1 * rx * ry / (double)den), q);
                    if (a == 0) h = h_mulmod(h, r1, q);
                    if (b == 0) h = h_mulmod(h, r1, q);
                    H[(size_t)a * cyn + b] = h;
                }
            for (int a = 0; a < cxn; a++) {
                C0[(size_t)li * cxn + a] = (double)H[(size_t)a * cyn];
                for (int b = 0; b < cyn; b++) {
                    const u64 v = H[(size_t)a * cyn + b];
                    Rt[((size_t)li * cxn + a) * cyn + b] = TwD{(double)v, (double)v / (double)q};
                }
            }
        }
        std::vector<const u64*> px, py;
        std::vector<long> sx, sy, qx, qy;
        for (int i = 1; i < nx; i++) {
            const View v = view_of(xb[permx[i] - 1]);
            if (v.B > 1 && v.bs != (long)v.np * v.ps) throw_err(AESFHE_EARG, "poly2: non-compact basis view");
            px.push_back(v.d), sx.push_back(v.B == 1 && B > 1 ? 0 : v.bs), qx.push_back(v.ps);
        }
        for (int j = 1; j < ny; j++) {
            const View v = view_of(yb[perm[j] - 1]);
            if (v.B > 1 && v.bs != (long)v.np * v.ps) throw_err(AESFHE_EARG, "poly2: non-compact basis view");
            py.push_back(v.d), sy.push_back(v.B == 1 && B > 1 ? 0 : v.bs), qy.push_back(v.ps);
        }
        if (px.empty()) px.push_back(nullptr), sx.push_back(0), qx.push_back(0);
        if (py.empty()) py.push_back(nullptr), sy.push_back(0), qy.push_back(0);
        auto dpx = upload_small(e, px.data(), px.size());
        auto dpy = upload_small(e, py.data(), py.size());
        auto dsx = upload_small(e, sx.data(), sx.size());
        auto dsy = upload_small(e, sy.data(), sy.size());
        auto dqx = upload_small(e, qx.data(), qx.size());
        auto dqy = upload_small(e, qy.data(), qy.size());
        std::vector<int> xstart(cxn + 1, nx);
        for (int i = nx - 1; i >= 0; i--) xstart[cxs[i]] = i;
        auto dcx = upload_small(e, xstart.data(), xstart.size());
        auto dcy = upload_small(e, cy.data(), cy.size());
        auto dW = upload_small(e, Wt.data(), Wt.size());
        auto dR = upload_small(e, Rt.data(), Rt.size());
        auto dC0 = upload_small(e, C0.data(), C0.size());
        const long obs = 3L * nl * N;
        aesfhe_ct* d3 = ct_new(e, ml * B, 3, l);
        // a < 2^52 and the unfolded tensor sums (a + 2 (nx - 1) products of <= 1.5 q) < 2^53
        auto is_big = [&](int li) {
            const double q = (double)e->chain.q[li];
            return wfac * q >= 0x1p52 * 0.999 || (wfac + 3.0 * nx) * q >= 0x1p53 * 0.999;
        };
        // the S-box shape (ny = 16, whole blocks of 4 outputs) takes k_poly2_int_s on its exact
        // limbs, with y' left unreduced where wfac_u = max_row (|w_0| + sum_j |w_j|) keeps the
        // doubled bound: |a| <= wfac_u q < 2^51 and the tensor sums (a + 2 (nx - 1) products of
        // <= 1.5 q) < 2^52
        double wfac_u = 1.0;
        for (int t = 0; t < ml; t++)
            for (int i = 0; i < nx; i++) {
                double f = 0.0;
                for (int j = 0; j < ny; j++) f += std::fabs(Wt[((size_t)t * nx + i) * ny + j]);
                wfac_u = std::max(wfac_u, f);
            }
        auto lazy_ok = [&](int li) {
            const double q = (double)e->chain.q[li];
            return wfac_u * q < 0x1p51 && (wfac_u + 3.0 * nx) * q < 0x1p52;
        };
        {
            ProfScope ps_(e, FAM_EW, 8.0 * N * nl * (double)B * (2.0 * (nx + ny - 2) + 3.0 * ml), "poly2_int");
            ps_.disp = 0;
            constexpr int mo = 4;  // outputs per thread (8: 219 VGPRs, 2 waves, measured slower)
            for (int t0 = 0; t0 < ml;) {
                // k_poly2_int_s: 2 blocks per launch, paired on XCDs by 8 workgroups (N >= 2^11)
                const bool sbox = ny == kPoly2Max && ml - t0 >= 2 * mo && (N / 256) % 8 == 0;
                for (int la = 0; la < nl;) {  // runs of limbs of one kernel class
                    const bool big = is_big(la), lz = !big && lazy_ok(la);
                    int lb = la + 1;
                    while (lb < nl && is_big(lb) == big && (big || lazy_ok(lb) == lz)) lb++;
                    const dim3 grid(N / 256, lb - la, B);
                    // the folding limbs (q_0) with split inner sums when q < 2^51 (k_poly2_int_split)
                    bool split = big;
                    for (int li = la; li < lb; li++) split &= (double)e->chain.q[li] < 0x1p51;
                    if (sbox && split) {
                        hipLaunchKernelGGL(k_poly2_int_split<mo>, dim3(2 * N / 256, lb - la, B), dim3(256), 0, e->stream,
                                           (const u64* const*)dpx, (const long*)dsx, (const long*)dqx, nx, (const u64* const*)dpy, (const long*)dsy, (const long*)dqy,
                                           (const int*)dcx, (const int*)dcy, cxn, cyn, (const double*)dW, (const TwD*)dR, (const double*)dC0, t0,
                                           d3->d, (long)B * obs, obs, e->q, e->qinv, la, nl, e->logN, slab_rot);
                        ps_.disp++;
                    } else if (sbox) {
                        hipLaunchKernelGGL((big ? k_poly2_int_s<mo, false, true> : lz ? k_poly2_int_s<mo, true> : k_poly2_int_s<mo, false>), dim3(2 * N / 256, lb - la, B), dim3(256), 0, e->stream,
                                           (const u64* const*)dpx, (const long*)dsx, (const long*)dqx, nx, (const u64* const*)dpy, (const long*)dsy, (const long*)dqy,
                                           (const int*)dcx, (const int*)dcy, cxn, cyn, (const double*)dW, (const TwD*)dR, (const double*)dC0, t0,
                                           d3->d, (long)B * obs, obs, e->q, e->qinv, la, nl, e->logN, slab_rot);
                        ps_.disp++;
                    } else {
                        auto kern = big ? (ny == kPoly2Max ? k_poly2_int<true, kPoly2Max, mo> : k_poly2_int<true, 0, mo>)
                                        : (ny == kPoly2Max ? k_poly2_int<false, kPoly2Max, mo> : k_poly2_int<false, 0, mo>);
                        for (int tb = t0; tb < (sbox ? t0 + 2 * mo : t0 + mo) && tb < ml; tb += mo) {
                            hipLaunchKernelGGL(kern, grid, dim3(256), 0, e->stream, (const u64* const*)dpx, (const long*)dsx, (const long*)dqx, nx, (const u64* const*)dpy, (const long*)dsy, (const long*)dqy, ny,
                                               (const int*)dcx, (const int*)dcy, cxn, cyn, (const double*)dW, (const TwD*)dR, (const double*)dC0, ml, tb, std::min(mo, ml - tb), d3->d, (long)B * obs, obs, e->q, e->qinv, la, nl, e->logN, slab_rot);
                            ps_.disp++;
                        }
                    }
                    la = lb;
                }
                t0 += sbox ? 2 * mo : mo;
            }
        }
        HIPC(hipGetLastError());
        aesfhe_ct* r2 = relin_rescale(e, d3, rlk, 2);
        aesfhe_ct_free(d3);
        std::vector<aesfhe_ct*> parts = ct_split_batch(e, r2, ml);  // no copies
        for (int t = 0; t < ml; t++) outs[live[t]] = parts[t];
    }
    for (int t = 0; t < m; t++)
        if (!outs[t]) outs[t] = ct_zero_new(e, B, 2, l - 2);
}

// -----------------------------------------------------------------------------------------------
// raw NTT entry points
extern "C" int aesfhe_ntt_host(aesfhe_engine* e, uint64_t* limbs, int32_t nlimb, const int32_t* pids, int32_t inv) {
    API_BEGIN
    const int N = e->N;
    for (int i = 0; i < nlimb; i++)
        if (pids[i] < 0 || pids[i] >= e->np) throw_err(AESFHE_EARG, "bad prime index");
    Tmp buf(e, (size_t)N);
    for (int i = 0; i < nlimb; i++) {
        HIPC(hipMemcpyAsync(buf.p, limbs + (size_t)i * N, (size_t)N * 8, hipMemcpyHostToDevice, e->stream));
        // one limb: a Q prime (nq = 1, qpid0 = pid) or a special prime (nq = 0, spid0 = pid)
        const int pid = pids[i];
        Span s = pid < e->Lp1 ? span_s(buf.p, N, 1, 1, pid, e->Lp1) : span_s(buf.p, N, 1, 0, 0, pid);
        ntt(e, s, s, 1, inv != 0);
        HIPC(hipMemcpyAsync(limbs + (size_t)i * N, buf.p, (size_t)N * 8, hipMemcpyDeviceToHost, e->stream));
        HIPC(hipStreamSynchronize(e->stream));
    }
    API_END
}

extern "C" int aesfhe_bench_ntt(aesfhe_engine* e, int32_t nlimb, int32_t iters, double* fwd_ms, double* inv_ms) {
    API_BEGIN
    const int N = e->N;
    const int nq = std::min(nlimb, e->Lp1);
    const int groups = (nlimb + nq - 1) / nq;
    Tmp buf(e, (size_t)groups * nq * N);
    HIPC(hipMemsetAsync(buf.p, 0, (size_t)groups * nq * N * 8, e->stream));
    Span s = span_s(buf.p, (long)nq * N, nq, nq, 0, e->Lp1);
    hipEvent_t a, b, c;
    HIPC(hipEventCreate(&a));
    HIPC(hipEventCreate(&b));
    HIPC(hipEventCreate(&c));
    ntt(e, s, s, groups * nq, false);  // warm up
    ntt(e, s, s, groups * nq, true);
    HIPC(hipEventRecord(a, e->stream));
    for (int i = 0; i < iters; i++) ntt(e, s, s, groups * nq, false);
    HIPC(hipEventRecord(b, e->stream));
    for (int i = 0; i < iters; i++) ntt(e, s, s, groups * nq, true);
    HIPC(hipEventRecord(c, e->stream));
    HIPC(hipEventSynchronize(c));
    float t1 = 0, t2 = 0;
    hipEventElapsedTime(&t1, a, b);
    hipEventElapsedTime(&t2, b, c);
    *fwd_ms = t1 / iters;
    *inv_ms = t2 / iters;
    hipEventDestroy(a);
    hipEventDestroy(b);
    hipEventDestroy(c);
    API_END
}
