/*
 * aesfhe.h -- C ABI of the MI355X-native RNS-CKKS engine behind the aes-fhe services.
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json: the reference
 * (songhayeong/aes-fhe) drives every homomorphic operation through the closed
 * `desilofhe.Engine` object, wrapped by `EngineContext` (engine_context.py:9-85) and
 * `EngineWrapper` (xor_service.py:36-129).  Each entry point below replaces one method
 * of that object as the reference calls it (file:line of the call site in the reference):
 *
 *   aesfhe_engine_create        Engine(...) three signatures        engine_context.py:32-58
 *   aesfhe_key_secret           engine.create_secret_key()          engine_context.py:62
 *   aesfhe_key_public           engine.create_public_key(sk)        engine_context.py:63
 *   aesfhe_key_relin            engine.create_relinearization_key   engine_context.py:64
 *   aesfhe_key_galois           create_conjugation_key /            engine_context.py:65-66
 *                               create_rotation_key /               engine_context.py:70
 *                               create_fixed_rotation_key
 *   aesfhe_encode/_decode       engine.encode(vec) (host codec)     xor_service.py:65-66,
 *                                                                    sbox/sbox_service.py:85-88
 *   aesfhe_encrypt/_decrypt     engine.encrypt(data, pk) / decrypt  engine_context.py:81-85
 *   aesfhe_encode_device, ...   utils.zeta_encode + encrypt and     utils.py:40-59,
 *     _decode/_encrypt/_decrypt decrypt + zeta_decode on device      engine_context.py:81-85
 *                               buffers (the client path)
 *   aesfhe_add / _sub / _add_pt engine.add(a, b)                    xor_service.py:75-76
 *   aesfhe_mul                  engine.multiply(ct, ct, rlk)        xor_service.py:68-71
 *   aesfhe_mul_pt               engine.multiply(ct, pt)             xor_service.py:73,285
 *   aesfhe_mul_const            engine.multiply(ct, scalar)         xor_service.py:282
 *   aesfhe_tensor/_relinearize  engine.relinearize(ct, rlk)         xor_service.py:107-118
 *   aesfhe_galois               engine.rotate(ct, key, k) /         xor_service.py:100-105
 *                               engine.conjugate(ct, cjk)           xor_service.py:88-89
 *   aesfhe_power_basis          engine.make_power_basis(ct, d, rlk) xor_service.py:85-86,
 *                                                                    sbox/sbox_service.py:93
 *   aesfhe_lincomb / aesfhe_dot  (no reference counterpart: fused BSGS building blocks used
 *                               by the optimised AES round; the reference's per-term loops
 *                               xor_service.py:283-285 / sbox_service.py:124-136 are the
 *                               unfused equivalent)
 *
 * Conventions
 *   - Plain C types only: pointers, sizes, int64 coefficients, doubles.  No torch types.
 *   - Every function returns 0 on success or a negative AESFHE_E* code; the message of the
 *     last failure on the calling thread is returned by aesfhe_last_error().  The Python
 *     facade maps codes to RuntimeError with desilofhe-compatible substrings (e.g.
 *     "should have 3 polynomials", matched at xor_service.py:116).
 *   - Handles are immutable values (every op returns a new handle, as desilofhe objects are);
 *     the caller frees them with the matching *_free.
 *   - A ciphertext handle holds a BATCH of B ciphertexts at one level; binary operations
 *     accept B_a == B_b or a broadcast operand with B == 1; aesfhe_mul and aesfhe_tensor also
 *     cycle through a smaller power-of-two batch dividing the larger one (element i takes
 *     element i mod B_small).
 *   - Residues are kept in the NTT (evaluation) domain, canonical in [0, q).
 *
 * Two implementations export exactly this ABI:
 *   libaesfhe.so        (aes-fhe_amd/csrc, HIP for gfx950)      -- the product
 *   oracle/_build/liboracle_ckks.so (oracle/ckks_oracle.c, CPU) -- test-only checker
 */
#ifndef AESFHE_H
#define AESFHE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision: bumped whenever a struct layout or an entry point's meaning changes (4: the
 * trailing aesfhe_params.digit_primes; a caller compiled against an older header passes a shorter
 * struct; 5: aesfhe_key_trim appended, and aesfhe_key_import accepts a switching key of 1..dnum
 * digits -- a trimmed key's export -- instead of exactly dnum).  Callers check
 * aesfhe_abi_version() == AESFHE_ABI_VERSION before anything else. */
#define AESFHE_ABI_VERSION 5

#define AESFHE_OK 0
#define AESFHE_EARG (-1)      /* bad argument / shape / level mismatch */
#define AESFHE_ENOMEM (-2)    /* host or device allocation failed */
#define AESFHE_EDEVICE (-3)   /* HIP runtime error */
#define AESFHE_EDEGREE (-4)   /* ciphertext has the wrong number of polynomials */
#define AESFHE_ELEVEL (-5)    /* out of levels */
#define AESFHE_EUNSUPPORTED (-6)

typedef struct aesfhe_engine aesfhe_engine;
typedef struct aesfhe_ct aesfhe_ct;
typedef struct aesfhe_pt aesfhe_pt;
typedef struct aesfhe_key aesfhe_key;

typedef struct aesfhe_params {
    int32_t log_n;          /* log2 of the ring degree N (slots = N/2) */
    int32_t max_level;      /* L: the ciphertext modulus chain has L+1 primes q_0..q_L */
    int32_t special_primes; /* K: special primes p_0..p_{K-1} (P = their product) */
    int32_t scale_bits;     /* log2 of the top-level scale Delta_L */
    int32_t base_bits;      /* bit size of q_0 */
    int32_t special_bits;   /* bit size of the special primes */
    int32_t device;         /* HIP device ordinal (ignored by the CPU oracle) */
    int32_t threads;        /* host threads (oracle only; 0 = default) */
    uint64_t seed;          /* engine seed: all key / encryption randomness derives from it */
    const uint64_t *primes; /* optional explicit chain q_0..q_L,p_0..p_{K-1} (NULL = generate) */
    uint64_t seed_ext[3];   /* with seed: the 256-bit ChaCha20 key of every random stream
                               (seed, ext[0], ext[1], ext[2]); zeros for a reproducible 64-bit seed */
    int32_t digit_primes;   /* alpha: primes per key-switch digit, 1..16 (0 = K); digit j covers
                               q_{j alpha} .. q_{j alpha + alpha - 1}, dnum = ceil((L+1)/alpha).
                               alpha > K is allowed while a digit's product stays below P */
} aesfhe_params;

/* ---- diagnostics ---------------------------------------------------------------------- */
const char *aesfhe_last_error(void);
const char *aesfhe_backend_name(void);
int32_t aesfhe_abi_version(void); /* AESFHE_ABI_VERSION of the library */

/* ---- engine ----------------------------------------------------------------------------- */
int aesfhe_engine_create(const aesfhe_params *params, aesfhe_engine **out);
void aesfhe_engine_destroy(aesfhe_engine *eng);
/* dims[0]=log_n dims[1]=max_level dims[2]=special_primes dims[3]=dnum */
int aesfhe_engine_dims(const aesfhe_engine *eng, int32_t dims[4]);
/* primes: L+1+K words; scales: L+1 doubles (canonical scale Delta_l of every level) */
int aesfhe_engine_primes(const aesfhe_engine *eng, uint64_t *primes_out);
int aesfhe_engine_scales(const aesfhe_engine *eng, double *scales_out);
/* Scale at which a plaintext/constant multiplied into a level-`level` ciphertext must be
 * encoded so that the rescaled product lands exactly on the canonical Delta_{level-1}. */
double aesfhe_engine_mul_scale(const aesfhe_engine *eng, int32_t level);
int aesfhe_engine_sync(aesfhe_engine *eng);
/* Per-kernel-family timing (HIP events on the engine stream; CPU wall time in the oracle).
 * family: "ntt" | "keyswitch" | "elementwise" | "all".  enable: bitmask of the families to
 * record (1 ntt, 2 keyswitch, 4 elementwise; -1 all), 0 stops.  Enabling resets the counters. */
int aesfhe_engine_profile(aesfhe_engine *eng, int32_t enable);
int aesfhe_engine_profile_read(aesfhe_engine *eng, const char *family, int64_t *launches,
                               double *total_ms, double *bytes);
/* Per kernel class of the recorded families since profiling was enabled, as JSON text
 * {"class": [launches, total_ms, algorithmic_bytes], ...} (classes: ntt_fwd_cols, ntt_fwd_rows,
 * ntt_fwd_rows_fin, ntt_fwd_cols_spread, ntt_inv_rows, ntt_inv_rows_prod, ntt_inv_cols, modup,
 * ks_rows_inner, moddown, poly2_int, lincomb, ...).  Writes at most cap bytes (NUL-terminated)
 * into buf (may be NULL) and the size needed into *need.  "{}" in the oracle. */
int aesfhe_engine_profile_kernels(aesfhe_engine *eng, char *buf, int64_t cap, int64_t *need);
/* device bytes currently held by the engine (keys + pool); 0 in the oracle */
int64_t aesfhe_engine_device_bytes(const aesfhe_engine *eng);
/* device arena counters (out holds 7 values): out[0] bytes held, [1] bytes live, [2] hipMalloc
 * calls, [3] trims, [4] blocks split off a larger free block, [5] peak bytes live since the engine
 * was created, [6] fragmentation = bytes of chunks that hold a live block minus the live bytes
 * (held but neither in use nor returnable by a trim); zeros in the oracle */
int aesfhe_engine_pool_stats(const aesfhe_engine *eng, int64_t *out);
/* release every cached (not live) device block (synchronises the engine's stream): between
 * workload phases whose buffer sizes differ, so the next phase does not evict in its timed path */
int aesfhe_engine_pool_trim(aesfhe_engine *eng);

/* ---- host codec (no engine / device needed) --------------------------------------------- */
/* Canonical-embedding encode: n_slots <= N/2 complex values (zero padded) -> N integer
 * coefficients round(scale * m_i). */
int aesfhe_encode(int32_t log_n, const double *re, const double *im, int64_t n_slots,
                  double scale, int64_t *coeffs_out);
/* Decode N centered integer coefficients (already divided by nothing) at `scale` -> N/2 slots */
int aesfhe_decode(int32_t log_n, const int64_t *coeffs, double scale, double *re_out,
                  double *im_out);

/* Prime chain + canonical scales the engine would generate for these parameters (host only):
 * primes_out L+1+K words, scales_out L+1 doubles. */
int aesfhe_chain(const aesfhe_params *params, uint64_t *primes_out, double *scales_out);

/* ---- keys ------------------------------------------------------------------------------- */
int aesfhe_key_secret(aesfhe_engine *eng, uint64_t seed, aesfhe_key **out);
int aesfhe_key_public(aesfhe_engine *eng, const aesfhe_key *sk, aesfhe_key **out);
int aesfhe_key_relin(aesfhe_engine *eng, const aesfhe_key *sk, aesfhe_key **out);
/* galois_elt odd in [1, 2N): conjugation = 2N-1, rotation by k slots (np.roll(v, k)) =
 * 5^(-k mod N/2) mod 2N.  Use aesfhe_galois_elt() to compute it. */
int aesfhe_key_galois(aesfhe_engine *eng, const aesfhe_key *sk, uint64_t galois_elt,
                      aesfhe_key **out);
uint64_t aesfhe_galois_elt(int32_t log_n, int64_t rotation, int32_t conjugate);
/* Hoisted rotation key for galois_elt g: a switching key s -> sigma_g^{-1}(s) (kind 5), for
 * aesfhe_rotate_hoisted.  (No reference counterpart: desilofhe's bootstrap keys are internal,
 * engine_context.py:72-73; used by the CoeffToSlot / SlotToCoeff baby steps.) */
int aesfhe_key_galois_hoisted(aesfhe_engine *eng, const aesfhe_key *sk, uint64_t galois_elt,
                              aesfhe_key **out);
/* Sparse ternary secret with exactly hw nonzeros (bootstrapping's ephemeral secret, for the
 * ModRaise overflow bound): key = derive(derive(seed_e, seed), 9); partial Fisher-Yates over
 * 0..N-1 -- step i swaps i with i + rnd(key, i) mod (N - i) and sets that coefficient to -1 if
 * rnd(key, N + i) is odd, else +1.  (Replaces desilofhe's internal bootstrap key material,
 * engine_context.py:62-73 create_bootstrap_key.) */
int aesfhe_key_secret_sparse(aesfhe_engine *eng, uint64_t seed, int32_t hw, aesfhe_key **out);
/* Key switching key sk_from -> sk_to; apply with aesfhe_galois (it is a galois-kind key with
 * element 1, the identity automorphism). */
int aesfhe_key_switch(aesfhe_engine *eng, const aesfhe_key *sk_from, const aesfhe_key *sk_to,
                      aesfhe_key **out);
/* kind: 0 secret 1 public 2 relin 3 galois; galois_elt for kind 3 */
int aesfhe_key_info(const aesfhe_key *key, int32_t *kind, uint64_t *galois_elt);
void aesfhe_key_free(aesfhe_key *key);
/* Key serialisation (desilofhe keeps keys inside its Engine object,
 * engine_context.py:62-73): kind, galois element, key seed (from which derived keys' randomness
 * is drawn) and the residues.  out NULL: only the header fields and *words are returned. */
int aesfhe_key_export(aesfhe_engine *eng, const aesfhe_key *key, int32_t *kind, uint64_t *galois_elt,
                      uint64_t *keyseed, int64_t *words, uint64_t *out);
int aesfhe_key_import(aesfhe_engine *eng, int32_t kind, uint64_t galois_elt, uint64_t keyseed,
                      const uint64_t *in, int64_t words, aesfhe_key **out);
/* Keep only the key-switch digits that a switch at level <= max_level reads (switching keys:
 * relinearization, galois / key-switch, hoisted rotation).  Digit d of a key is generated from
 * its own random streams, so the kept digits are word for word the full key's and every switch
 * at those levels is unchanged; a switch above max_level fails with AESFHE_ELEVEL.  A trimmed key
 * exports and imports with its digit count (words = digits x 2 x (L+1+K) x N).  No desilofhe
 * counterpart (its key memory is internal): the bootstrapper's SlotToCoeff keys only ever switch
 * at the bottom levels (bootstrap.py trim_bootstrap_keys). */
int aesfhe_key_trim(aesfhe_engine *eng, aesfhe_key *key, int32_t max_level);

/* ---- ciphertexts ------------------------------------------------------------------------ */
/* coeffs: batch*N integer coefficients (encoded at the canonical scale of `level`);
 * key: public key (or secret key: symmetric encryption).  nonce selects the randomness. */
int aesfhe_encrypt(aesfhe_engine *eng, const aesfhe_key *key, const int64_t *coeffs,
                   int32_t batch, int32_t level, uint64_t nonce, aesfhe_ct **out);
/* Decrypt to batch*N centred coefficients: limbs 0 and 1 CRT-combined modulo q_0 q_1 (a level-0
 * ciphertext: modulo q_0), saturated to +-(2^63 - 1). */
int aesfhe_decrypt(aesfhe_engine *eng, const aesfhe_key *sk, const aesfhe_ct *ct,
                   int64_t *coeffs_out);
/* ---- device-resident client path ----------------------------------
 * The codec and the encryption on buffers in the engine's device memory (the oracle: host
 * memory), stream-ordered on the engine's stream, for a client path with no host round trip
 * (reference: utils.zeta_encode/zeta_decode, utils.py:40-59, + EngineContext.encrypt/decrypt,
 * engine_context.py:81-85).  Results are bit-identical to aesfhe_encode / aesfhe_decode /
 * aesfhe_encrypt / aesfhe_decrypt on the same values. */
/* B slot vectors (re, im: row stride `stride` doubles, n_slots <= N/2 values each, zero padded;
 * im may be NULL) -> B x N int64 coefficients at `scale`.  Synchronises (overflow check). */
int aesfhe_encode_device(aesfhe_engine *eng, const double *re, const double *im, int32_t batch,
                         int64_t n_slots, int64_t stride, double scale, int64_t *coeffs_out);
/* B x N int64 coefficients -> B x N/2 slots (re_out, im_out: B x N/2 doubles each) */
int aesfhe_decode_device(aesfhe_engine *eng, const int64_t *coeffs, int32_t batch, double scale,
                         double *re_out, double *im_out);
/* aesfhe_encrypt with the coefficients in device memory (no host copy, no synchronisation) */
int aesfhe_encrypt_device(aesfhe_engine *eng, const aesfhe_key *key, const int64_t *coeffs,
                          int32_t batch, int32_t level, uint64_t nonce, aesfhe_ct **out);
/* aesfhe_decrypt into device memory (batch x N centred int64 coefficients; no synchronisation) */
int aesfhe_decrypt_device(aesfhe_engine *eng, const aesfhe_key *sk, const aesfhe_ct *ct,
                          int64_t *coeffs_out);

/* info[0]=batch info[1]=npoly info[2]=level info[3]=is_zero */
int aesfhe_ct_info(const aesfhe_ct *ct, int32_t info[4]);
/* NTT-domain residues, layout [batch][poly][limb 0..level][N] */
int aesfhe_ct_export(aesfhe_engine *eng, const aesfhe_ct *ct, uint64_t *out);
int aesfhe_ct_import(aesfhe_engine *eng, const uint64_t *in, int32_t batch, int32_t npoly,
                     int32_t level, aesfhe_ct **out);
/* Device-resident transfer for the multi-GPU batch scatter / gather (the
 * reference has no multi-GPU path -- it replaces the host round trip a desilofhe user would make
 * through ciphertext serialisation, xor_service.py:166-182 being the reader side the survey pairs
 * it with): residues of batch elements [start, start + count), layout as aesfhe_ct_export, to /
 * from a caller-owned buffer on the engine's device (host memory for the CPU oracle).  Both
 * synchronise the engine stream before returning. */
int aesfhe_ct_export_device(aesfhe_engine *eng, const aesfhe_ct *ct, int32_t start, int32_t count,
                            void *dst);
int aesfhe_ct_import_device(aesfhe_engine *eng, const void *src, int32_t batch, int32_t npoly,
                            int32_t level, aesfhe_ct **out);
int aesfhe_ct_copy(aesfhe_engine *eng, const aesfhe_ct *ct, aesfhe_ct **out);
/* batch slicing / concatenation (all parts at one level and npoly) */
int aesfhe_ct_slice(aesfhe_engine *eng, const aesfhe_ct *ct, int32_t start, int32_t count,
                    aesfhe_ct **out);
int aesfhe_ct_concat(aesfhe_engine *eng, const aesfhe_ct *const *parts, int32_t n,
                     aesfhe_ct **out);
/* batch permutation / repetition: element b of the result (batch n) is element idx[b] of ct
 * (0 <= idx[b] < batch).  One copy pass.  The fully sliced AES state (aes_round_bits
 * AESSlicedRound) carries the state columns as batch elements, so ShiftRows -- a rotation in
 * the reference's slot layouts (shiftrows_service.py:33-51) -- is this permutation, and a round
 * key held once per column is repeated over the batch with it. */
int aesfhe_ct_gather(aesfhe_engine *eng, const aesfhe_ct *ct, const int32_t *idx, int32_t n,
                     aesfhe_ct **out);
/* an all-zero ciphertext (flagged is_zero) */
int aesfhe_ct_zero(aesfhe_engine *eng, int32_t batch, int32_t level, aesfhe_ct **out);
void aesfhe_ct_free(aesfhe_ct *ct);

/* plaintext from N integer coefficients, materialised at `level` (NTT residues) */
int aesfhe_pt_create(aesfhe_engine *eng, const int64_t *coeffs, int32_t level,
                     aesfhe_pt **out);
/* the same over Q_level u P (level + 1 + K limbs): operands of aesfhe_linear_bsgs */
int aesfhe_pt_create_ext(aesfhe_engine *eng, const int64_t *coeffs, int32_t level,
                         aesfhe_pt **out);
void aesfhe_pt_free(aesfhe_pt *pt);

/* ---- arithmetic ------------------------------------------------------------------------- */
/* Operands at different levels are aligned by an exact-scale level-down of the higher one. */
int aesfhe_add(aesfhe_engine *eng, const aesfhe_ct *a, const aesfhe_ct *b, aesfhe_ct **out);
int aesfhe_sub(aesfhe_engine *eng, const aesfhe_ct *a, const aesfhe_ct *b, aesfhe_ct **out);
int aesfhe_negate(aesfhe_engine *eng, const aesfhe_ct *a, aesfhe_ct **out);
/* pt must be encoded at the canonical scale of ct's level and created at that level */
int aesfhe_add_pt(aesfhe_engine *eng, const aesfhe_ct *ct, const aesfhe_pt *pt,
                  aesfhe_ct **out);
/* ct + (re + i*im) at ct's level (constant encoded at the canonical scale, no level used) */
int aesfhe_add_const(aesfhe_engine *eng, const aesfhe_ct *ct, double re, double im,
                     aesfhe_ct **out);
/* pt encoded at aesfhe_engine_mul_scale(level); output rescaled to level-1 */
int aesfhe_mul_pt(aesfhe_engine *eng, const aesfhe_ct *ct, const aesfhe_pt *pt,
                  aesfhe_ct **out);
/* ct * (re + i*im), output at level-1 (exact canonical scale) */
int aesfhe_mul_const(aesfhe_engine *eng, const aesfhe_ct *ct, double re, double im,
                     aesfhe_ct **out);
/* ct (*) ct -> 3-polynomial ciphertext, same level, scale Delta^2 (no relin, no rescale) */
int aesfhe_tensor(aesfhe_engine *eng, const aesfhe_ct *a, const aesfhe_ct *b,
                  aesfhe_ct **out);
/* 3 -> 2 polynomials (fails with AESFHE_EDEGREE "should have 3 polynomials" otherwise) */
int aesfhe_relinearize(aesfhe_engine *eng, const aesfhe_ct *ct, const aesfhe_key *rlk,
                       aesfhe_ct **out);
int aesfhe_rescale(aesfhe_engine *eng, const aesfhe_ct *ct, aesfhe_ct **out);
/* tensor + relinearize + rescale */
int aesfhe_mul(aesfhe_engine *eng, const aesfhe_ct *a, const aesfhe_ct *b,
               const aesfhe_key *rlk, aesfhe_ct **out);
/* exact-scale level reduction */
int aesfhe_level_down(aesfhe_engine *eng, const aesfhe_ct *ct, int32_t level,
                      aesfhe_ct **out);
/* automorphism X -> X^g followed by key switching back to s (rotation / conjugation) */
/* n rotations of one ciphertext with hoisted keys: outs[i] = sigma_{g_i}((c0 + KS_i(c1)_0,
 * KS_i(c1)_1)), the ModUp of c1 computed once for all n (the same slots as aesfhe_galois with
 * the ordinary key of g_i; residues differ only in the key-switch noise). */
int aesfhe_rotate_hoisted(aesfhe_engine *eng, const aesfhe_ct *ct, const aesfhe_key *const *keys,
                          int32_t n, aesfhe_ct **outs);
/* out = alpha * a * b + gamma * c + beta, one relinearisation + rescale: level
 * l - 1 for l = min(level a, level b) (a, b level-downed to l), c (optional, level >= l) truncated
 * to l with C = llround(gamma * (D_l * (D_l / D_c))), beta added to d0 as
 * llround(beta * D_l) * llround(D_l) mod q.  (Fused T_{a+b} = 2 T_a T_b - T_{a-b} and double
 * angles of the bootstrapping's EvalMod; no reference counterpart.) */
int aesfhe_mul_fma(aesfhe_engine *eng, const aesfhe_ct *a, const aesfhe_ct *b, const aesfhe_key *rlk,
                   int64_t alpha, const aesfhe_ct *c, double gamma, double beta, aesfhe_ct **out);
int aesfhe_galois(aesfhe_engine *eng, const aesfhe_ct *ct, const aesfhe_key *gk,
                  aesfhe_ct **out);
/* outs[0..d-1] = ct^1 .. ct^d, ct^k at level(ct) - ceil(log2 k) */
int aesfhe_power_basis(aesfhe_engine *eng, const aesfhe_ct *ct, int32_t d,
                       const aesfhe_key *rlk, aesfhe_ct **outs);
/* sum_i (re_i + i*im_i) * cts[i] at the lowest input level l, output at l - 1.  Inputs above l
 * are truncated to its limbs (no rescale) and their scale D_level compensated in the constant:
 * A = llround(re * mul_scale(l) * (D_l / D_level)). */
int aesfhe_lincomb(aesfhe_engine *eng, const aesfhe_ct *const *cts, int32_t n,
                   const double *re, const double *im, aesfhe_ct **out);
/* m linear combinations of the same n inputs in one pass: outs[r] = lincomb(cts, re/im row r)
 * (re, im row-major [m][n]); bit-identical to m separate aesfhe_lincomb calls. */
int aesfhe_lincomb_many(aesfhe_engine *eng, const aesfhe_ct *const *cts, int32_t n,
                        const double *re, const double *im, int32_t m, aesfhe_ct **outs);
/* sum_i a_i (*) b_i, one relinearisation + one rescale for the whole sum */
int aesfhe_dot(aesfhe_engine *eng, const aesfhe_ct *const *a, const aesfhe_ct *const *b,
               int32_t n, const aesfhe_key *rlk, aesfhe_ct **out);
/* out = sum_i a_i (*) b_i + sum_j gamma_j c_j + beta with ONE relinearisation + rescale: level
 * l - 1 for l = min level of the a_i, b_i (level-downed to l like aesfhe_dot); every addend c_j
 * (2 polynomials, level >= l) is truncated to l and enters the tensor's d0 / d1 times
 * C_j = llround(gamma_j * (D_l * (D_l / D_cj))); beta is added to d0 as
 * llround(beta * D_l) * llround(D_l) mod q (the aesfhe_mul_fma rules, n products and nc addends).
 * A zero-coefficient (C_j = 0) or zero addend is skipped.  (Node sums of the depth-optimal
 * Chebyshev evaluation in the bootstrapping; no reference counterpart.) */
int aesfhe_dot_fma(aesfhe_engine *eng, const aesfhe_ct *const *a, const aesfhe_ct *const *b,
                   int32_t n, const aesfhe_ct *const *c, const double *gamma, int32_t nc,
                   double beta, const aesfhe_key *rlk, aesfhe_ct **out);
/* m bivariate polynomials over shared power bases (the 2-D LUT evaluation of the reference's
 * nibble services, xor_service.py:245-286 / sbox_service.py:116-138, fused):
 *   outs[t] = sum_{i<nx, j<ny} C[t][i][j] x^i y^j,  C = re + i*im row-major [m][nx][ny],
 * xb = x^1..x^{nx-1}, yb = y^1..y^{ny-1} (2 polynomials, aligned to the lowest level l >= 2).
 * Constants are scaled by S1 = D_{l-2} q_l q_{l-1} / D_l^2 (D = canonical scales) and
 * rounded: A = llround(re*S1), B = llround(im*S1); an x^0 or y^0 factor multiplies the
 * constant by R = llround(D_l) mod q (both: R^2).  Inner sums stay unrescaled; one
 * relinearisation and two rescales put every output at level l-2, scale D_{l-2}.
 * 1 <= nx, ny <= 16. */
int aesfhe_poly2(aesfhe_engine *eng, const aesfhe_ct *const *xb, int32_t nx,
                 const aesfhe_ct *const *yb, int32_t ny, const double *re, const double *im,
                 int32_t m, const aesfhe_key *rlk, aesfhe_ct **outs);
/* aesfhe_poly2 for integer-weight coefficients C[t][i][j] = w[t][i][j] / den (Walsh spectra of
 * Boolean functions -- the S-box bits of the bench round, aes_round_bits.py): constants
 * F_ij = w_ij * H(class_x(i), class_y(j)) mod q, one H = llround(S1 * r_x * r_y / den)
 * (x R for an x^0 / y^0 factor) per pair of basis levels, so inner sums are exact integer
 * combinations.  Classes: 0 for x^0 / y^0, then one per distinct basis level, highest first.
 * Requires sum_j |w[t][i][j]| <= 512.  Output level l - 2, scale D_{l-2}. */
int aesfhe_poly2_int(aesfhe_engine *eng, const aesfhe_ct *const *xb, int32_t nx,
                     const aesfhe_ct *const *yb, int32_t ny, const int32_t *w, int32_t den,
                     int32_t m, const aesfhe_key *rlk, aesfhe_ct **outs);
/* aesfhe_poly2_int with each output's batch rotated within slabs of 4 (batch a multiple of 4):
 * element 4s + c of an output holds the polynomial at input element 4s + ((c + slab_rot) mod 4),
 * slab_rot in 0..3.  The sliced AES state (aes_round_bits.AESSlicedRound) folds ShiftRows of
 * row r -- a rotation in the reference's layouts (shiftrows_service.py:33-51) -- into that
 * row's S-box this way. */
int aesfhe_poly2_int_rot(aesfhe_engine *eng, const aesfhe_ct *const *xb, int32_t nx,
                         const aesfhe_ct *const *yb, int32_t ny, const int32_t *w, int32_t den,
                         int32_t m, const aesfhe_key *rlk, int32_t slab_rot, aesfhe_ct **outs);

/* ---- bootstrapping primitives (Engine.bootstrap, xor_service.py:120-129) ----------------- */
/* ModRaise: limb 0 of ct (mod q_0, centred) lifted to every limb of `level`; the result encrypts
 * t = m + q_0 I (scale bookkeeping is the caller's). */
int aesfhe_mod_raise(aesfhe_engine *eng, const aesfhe_ct *ct, int32_t level, aesfhe_ct **out);
/* ct * X^{N/2} (sign >= 0) or ct * -X^{N/2}: every slot times i / -i, exact, no level used. */
int aesfhe_mul_i(aesfhe_engine *eng, const aesfhe_ct *ct, int32_t sign, aesfhe_ct **out);
/* sum_i cts[i] * pts[i] with one rescale (aligned to the lowest ciphertext level l; plaintexts
 * encoded at mul_scale(l) with >= l+1 limbs): the diagonal sums of homomorphic linear maps. */
int aesfhe_dot_pt(aesfhe_engine *eng, const aesfhe_ct *const *cts, const aesfhe_pt *const *pts,
                  int32_t n, aesfhe_ct **out);

/* Baby-step giant-step linear map with hoisted baby steps and lazy ModDown (bootstrapping's
 * CoeffToSlot / SlotToCoeff; no reference counterpart -- desilofhe's bootstrap is internal):
 *   out = sum_j rho_{gkeys[j]}( sum_{t in terms of j} pts[t] * rho_{bkeys[tbaby[t]]}(ct) )
 * rho_k = the rotation of key k (bkeys: hoisted keys, kind 5; gkeys: galois keys, kind 3),
 * rho_NULL = identity.  Terms of giant j are consecutive, nterm[j] of them, at most one per
 * baby (AESFHE_EARG otherwise).  Arithmetic: the
 * baby rotations stay in Q_l u P (E_i = sigma_i(P c0 + acc0_i, acc1_i), no ModDown), each giant's
 * term sum S_j = sum pts * E over Q_l u P (pts from aesfhe_pt_create_ext at level l, encoded at
 * mul_scale(l)) is ModDown'd together with one rescale (D = P q_l) to level l - 1, and the giant
 * rotations' key switches are summed in Q_{l-1} u P (acc0 += P sigma_j(part_j0)) with ONE final
 * ModDown by P; parts with a NULL giant key are added after it.  Output level l - 1. */
int aesfhe_linear_bsgs(aesfhe_engine *eng, const aesfhe_ct *ct, int32_t nb,
                       const aesfhe_key *const *bkeys, int32_t ng, const aesfhe_key *const *gkeys,
                       const int32_t *nterm, const int32_t *tbaby, const aesfhe_pt *const *pts,
                       aesfhe_ct **out);

/* ---- raw kernels (known-answer tests and roofline measurement) ------------------------- */
/* In-place forward (inverse=0) / inverse NTT of nlimb host limbs; limb i uses prime pids[i]
 * (index into the q_0..q_L,p_0.. chain). */
int aesfhe_ntt_host(aesfhe_engine *eng, uint64_t *limbs, int32_t nlimb, const int32_t *pids,
                    int32_t inverse);
/* Time `iters` forward+inverse NTT launches over `nlimb` device-resident limbs (primes
 * cycled over the Q chain).  Reports the average per-launch duration of each direction
 * measured with HIP events on the engine stream. */
int aesfhe_bench_ntt(aesfhe_engine *eng, int32_t nlimb, int32_t iters, double *fwd_ms,
                     double *inv_ms);

#ifdef __cplusplus
}
#endif
#endif /* AESFHE_H */
