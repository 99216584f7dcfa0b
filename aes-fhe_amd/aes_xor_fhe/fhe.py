"""desilofhe-compatible CKKS engine facade over the MI355X C ABI (include/aesfhe.h).

The reference drives all homomorphic arithmetic through ``desilofhe.Engine`` objects
(engine_context.py:6,32-85; xor_service.py:36-129).  This module provides the same object
surface -- ``Engine``, ``Ciphertext``, ``Plaintext`` and the key objects -- with the same
method names, argument meaning and error behaviour, backed by the HIP engine
(``libaesfhe.so``).  Swapping ``from desilofhe import Engine`` for
``from aes_xor_fhe.fhe import Engine`` is the whole integration.

Semantics pinned by the reference's tests:
  * ``slot_count == N/2`` (test/test_xor_service.py:40-43 assumes 32768 at N = 2^16);
  * ``rotate(ct, key, k)`` equals ``np.roll(v, k)`` (test/test_engine_rot.py:32-40);
  * ``relinearize`` of a 2-polynomial ciphertext raises RuntimeError containing
    "should have 3 polynomials" (matched at xor_service.py:114-118);
  * every multiplication (ct x ct, ct x pt, ct x scalar) consumes one level.
"""
from __future__ import annotations

import ctypes as C
import math
import os
from typing import Sequence

import numpy as np

from ._abi import Lib, Params, c_ct_p, c_key_p, c_pt_p, load_product

# HomomorphicEncryption.org 128-bit bound on log2(QP) for ternary secrets
SECURITY_BUDGET = {11: 54, 12: 109, 13: 218, 14: 438, 15: 881, 16: 1772, 17: 3544}

# seed None: a fresh 256-bit ChaCha20 engine key from the OS entropy pool (os.urandom) per
# engine, so that no two default engines derive the same keys; an explicit seed (an integer below
# 2^256 or 32 bytes) reproduces every key and encryption: a small integer for tests, a 256-bit
# value shared by the ranks that must hold the same keys (parallel.shared_seed, `nonce_start`).
# scale 44 with K = 8: log QP = 50 + 30 * 44 + 8 * 50 = 1770 <= 1772 (128-bit at N = 2^16).  The
# general-mode Engine.bootstrap the reference's services call (xor_service.py:120-129) needs it:
# measured at N = 2^16, L = 30 (tools/boot_general_diag.py): max slot error 4.7e-3 at scale 44,
# 1.16 (unusable) at scale 40, below the zeta-256 decision margin sin(pi/256) = 0.012 only at 44.
# The bench's bit-mode path keeps its own explicit 40-bit scale and K = 10.
DEFAULT_PARAMS = dict(log_n=16, max_level=30, special_primes=8, scale_bits=44, base_bits=50,
                      special_bits=50, seed=None)


_MAGIC = b"AESFHE\x01\x00"


def _urandom64() -> int:
    return int.from_bytes(os.urandom(8), "little")


def _params_for(log_n=None, max_level=None, special_primes=None, scale_bits=None,
                base_bits=None, special_bits=None, seed=None, threads=0, device=0, digit_primes=None):
    p = dict(DEFAULT_PARAMS)
    p["digit_primes"] = int(digit_primes or 0)  # key-switch digit width alpha (0: = special_primes)
    for k, v in dict(log_n=log_n, max_level=max_level, special_primes=special_primes,
                     scale_bits=scale_bits, base_bits=base_bits, special_bits=special_bits,
                     seed=seed).items():
        if v is not None:
            p[k] = v
    p["threads"] = threads
    p["device"] = device
    s = p["seed"]
    if s is None:  # a fresh 256-bit key
        s = int.from_bytes(os.urandom(32), "little")
    elif isinstance(s, (bytes, bytearray)):
        if len(s) != 32:
            raise ValueError("a bytes seed must be 32 bytes (256 bits)")
        s = int.from_bytes(bytes(s), "little")
    s = int(s)
    if not 0 <= s < 1 << 256:
        raise ValueError("seed must be an integer in [0, 2^256) or 32 bytes")
    m = (1 << 64) - 1
    # the ChaCha20 engine key: seed = bits 0..63, seed_ext = bits 64..255 (a 64-bit seed keeps the
    # zero extension: reproducible tests; multi-rank key sharing passes a 256-bit shared seed,
    # parallel.shared_seed)
    p["seed"], p["seed_ext"] = s & m, ((s >> 64) & m, (s >> 128) & m, (s >> 192) & m)
    return p


def widest_digits(log_n: int, max_level: int, special_primes: int, scale_bits: int,
                  base_bits: int = 50, special_bits: int = 50, lib: Lib | None = None) -> int:
    """The widest key-switch digit (aesfhe_params.digit_primes, <= 16 primes) whose product stays
    below P for this chain (the engines' digits_below_p rule, on the primes aesfhe_chain makes):
    fewer digits -- fewer extension limbs to convert, transform and multiply per key switch."""
    import math
    lib = lib if lib is not None else load_product()
    L1, K = max_level + 1, special_primes
    cp = Params(log_n, max_level, special_primes, scale_bits, base_bits, special_bits, 0, 0, 0, None)
    primes = (C.c_uint64 * (L1 + K))()
    scales = (C.c_double * L1)()
    lib.check(lib.chain(C.byref(cp), primes, scales))
    logp = sum(math.log2(float(primes[L1 + k])) for k in range(K))
    for a in range(16, K, -1):
        if all(sum(math.log2(float(primes[i])) for i in range(lo, min(lo + a, L1))) <= logp
               for lo in range(0, L1, a)):
            return a
    return K


def _as_ptr(a, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


class _Handle:
    """Owns one C handle; frees it when collected (desilofhe objects are GC-managed)."""

    __slots__ = ("_lib", "_h", "_free")

    def __init__(self, lib: Lib, h, free):
        self._lib, self._h, self._free = lib, h, free

    def __del__(self):
        try:
            if self._h:
                self._free(self._h)
                self._h = None
        except Exception:  # interpreter shutdown
            pass


# ------------------------------------------------------------------------------------------
# keys
class _Owned(_Handle):
    """A handle whose C free returns memory to the engine's device pool: it holds the engine,
    and its own __del__ (which runs before its slots are cleared) frees the handle first."""
    __slots__ = ("engine",)


class _Key(_Owned):
    __slots__ = ()


class SecretKey(_Key):
    __slots__ = ()


class PublicKey(_Key):
    __slots__ = ()


class RelinearizationKey(_Key):
    __slots__ = ()


class GaloisKey(_Key):
    __slots__ = ("galois_elt",)


class ConjugationKey(GaloisKey):
    __slots__ = ()


class FixedRotationKey(GaloisKey):
    __slots__ = ("delta",)


class RotationKey:
    """Key set for arbitrary rotations: galois keys for left rotations by +-2^i, generated on
    first use from the secret key (deterministically: same seed -> same keys) and cached."""

    def __init__(self, engine: "Engine", sk: SecretKey):
        self._engine, self._sk, self._keys = engine, sk, {}

    def left(self, step: int) -> GaloisKey:
        if step not in self._keys:
            eng = self._engine
            g = eng._lib.galois_elt(eng.log_coeff_count, -step, 0)
            self._keys[step] = eng._galois_key(self._sk, g, GaloisKey)
        return self._keys[step]


class BootstrapKey:
    """Returned by create_(small_)bootstrap_key (engine_context.py:72-73 creates both
    unconditionally).  The key material (sparse-secret switching keys, the CoeffToSlot /
    SlotToCoeff rotation keys) is generated on first use, by bootstrap.Bootstrapper, since most
    contexts never bootstrap.  `small` selects more, smaller linear-transform groups (fewer
    diagonals, one more level per transform)."""

    def __init__(self, engine: "Engine", sk: "SecretKey", small: bool):
        self.engine = engine
        self._sk = sk
        self.small = small
        self._bs = None

    def bootstrapper(self, relinearization_key, conjugation_key=None):
        if self._bs is None:
            from .bootstrap import Bootstrapper
            self._bs = Bootstrapper(self.engine, self._sk, relinearization_key, conjugation_key,
                                    groups=4 if self.small else 3)
        return self._bs


# ------------------------------------------------------------------------------------------
class Ciphertext(_Handle):
    """A batch of B ciphertexts at one level.  ``level`` mirrors desilofhe's attribute read at
    xor_service.py:274-277."""

    __slots__ = ("engine", "level", "batch", "npoly", "is_zero")

    def __init__(self, engine: "Engine", h):
        super().__init__(engine._lib, h, engine._lib.ct_free)
        self.engine = engine
        info = (C.c_int32 * 4)()
        engine._lib.ct_info(h, info)
        self.batch, self.npoly, self.level, self.is_zero = info[0], info[1], info[2], bool(info[3])

    def __repr__(self):
        return f"Ciphertext(level={self.level}, batch={self.batch}, npoly={self.npoly})"


class _ProductCiphertext(Ciphertext):
    """A deferred relinearised product a * b (``Engine.multiply(a, b, rlk)``): level, batch and
    is_zero are the eager result's; the first use of the handle evaluates it as the eager
    ``aesfhe_mul`` would (same residues).  Only `multiply(product, constant)` looks inside:
    such terms, summed by ``add`` (``_LinearCiphertext``), are materialised together as ONE
    fused bivariate evaluation (``aesfhe_poly2``: one relinearisation and two rescales for all
    of them), the reference's per-coefficient loop of xor_service.py:271-286 in one launch
    sequence."""

    __slots__ = ("_a", "_b", "_rlk", "_mat", "__weakref__")

    def __init__(self, engine: "Engine", a: Ciphertext, b: Ciphertext, rlk):
        self._lib, self._free = engine._lib, None
        self.engine = engine
        self._a, self._b, self._rlk, self._mat = a, b, rlk, None
        self.level, self.batch, self.npoly = min(a.level, b.level) - 1, max(a.batch, b.batch), 2
        self.is_zero = a.is_zero or b.is_zero

    @property
    def _h(self):
        if self._mat is None:
            e = self.engine
            self._mat = e._call_ct(e._lib.mul, self._a._h, self._b._h, self._rlk._h)
            self._a = self._b = None  # release the operands
            e._pending.discard(self)
        return self._mat._h

    @property
    def pending(self) -> bool:
        return self._mat is None

    def __del__(self):  # the materialised ciphertext frees itself
        pass

    def __repr__(self):
        return f"Ciphertext(level={self.level}, batch={self.batch}, npoly=2, deferred product)"


class _GaloisCiphertext(Ciphertext):
    """A deferred automorphism + key switch (``Engine.conjugate``): level, batch and is_zero are
    the eager result's.  The first use of any pending one evaluates every pending automorphism
    of the same key and level together -- one ``aesfhe_galois`` over their concatenated batch,
    then split -- so the reference's runs of single-ciphertext conjugations
    (xor_service.py:245-254: seven per power basis, two bases per xor_cipher) become a few
    batched key switches.  The key switch is elementwise over the batch, so every output's
    residues equal the eager call's."""

    __slots__ = ("_src", "_key", "_mat", "__weakref__")

    def __init__(self, engine: "Engine", src: Ciphertext, key):
        self._lib, self._free = engine._lib, None
        self.engine = engine
        self._src, self._key, self._mat = src, key, None
        self.level, self.batch, self.npoly, self.is_zero = src.level, src.batch, 2, src.is_zero

    @property
    def _h(self):
        if self._mat is None:
            e = self.engine
            e._flush_galois(self._key)
            if self._mat is None:  # left out of an earlier flush that failed: on its own
                self._mat = e._call_ct(e._lib.galois, self._src._h, self._key._h)
                self._src = None
        return self._mat._h

    @property
    def pending(self) -> bool:
        return self._mat is None

    def __del__(self):  # the materialised ciphertext frees itself
        pass

    def __repr__(self):
        return f"Ciphertext(level={self.level}, batch={self.batch}, npoly=2, deferred galois)"


class _LinearCiphertext(Ciphertext):
    """A deferred linear combination: sum_i c_i * ct_i (each term one level below its input, as
    `multiply(ct, constant)` defines it) + sum of ciphertexts + a constant.

    ``Engine.multiply(ct, constant)`` returns one term; ``Engine.add`` of such objects (with each
    other, with ciphertexts or with constants) returns the merged sum; any other use of the
    handle (``_h``: a C call, decrypt, export, a product, a rotation ...) materialises it once
    as ONE fused ``aesfhe_lincomb`` (one rescale of the sum) plus the ciphertext addends and
    the constant.  ``level``, ``batch``, ``npoly`` and ``is_zero`` are those of the eager result,
    so callers that read them (the reference's ``level < 8`` bootstrap rule, xor_service.py:
    274-277) see the same values.  The reference's LUT evaluators (sbox/sbox_service.py:116-138,
    gf_service.py:46-64, xor_service.py:271-286) issue one multiply and one add per coefficient;
    this turns each such chain into the single fused launch sequence of `lincomb` instead of a
    rescale + add per term.  The residues equal `Engine.lincomb` of the same terms (rescale of the
    sum instead of the sum of rescales) on either backend, so the oracle stays the checker."""

    __slots__ = ("_terms", "_addends", "_const", "_mat")

    def __init__(self, engine: "Engine", terms, addends, const, level, batch):
        self._lib, self._free = engine._lib, None
        self.engine = engine
        self._terms, self._addends, self._const, self._mat = terms, addends, complex(const), None
        self.level, self.batch, self.npoly = level, batch, 2
        self.is_zero = not terms and not addends and self._const == 0

    @property
    def _h(self):
        if self._mat is None:
            self._mat = self.engine._materialize(self)
        return self._mat._h

    def __del__(self):  # the materialised ciphertext frees itself
        pass

    def __repr__(self):
        return (f"Ciphertext(level={self.level}, batch={self.batch}, npoly=2, deferred "
                f"{len(self._terms)} terms + {len(self._addends)} addends)")


class Plaintext:
    """Host-side slot vector; device encodings are materialised per (level, scale) on use.
    A constant vector (every slot equal) is multiplied as the polynomial a + b X^{N/2}."""

    def __init__(self, engine: "Engine", values: np.ndarray):
        self.engine = engine
        self.values = values
        self.is_const = bool(values.size and np.all(values == values[0]))
        self.const = complex(values[0]) if values.size else 0j
        self._dev = {}

    def device(self, level: int, scale: float, ext: bool = False):
        """Device encoding at (level, scale); ext: over Q_level u P (aesfhe_pt_create_ext)."""
        key = (level, scale, ext)
        h = self._dev.get(key)
        if h is None:
            eng = self.engine
            co = eng._encode_coeffs(self.values, scale)
            out = C.c_void_p()
            create = eng._lib.pt_create_ext if ext else eng._lib.pt_create
            eng._check(create(eng._h, _as_ptr(co, C.c_int64), level, C.byref(out)))
            h = _Owned(eng._lib, out.value, eng._lib.pt_free)
            h.engine = eng
            self._dev[key] = h
        return h._h


# ------------------------------------------------------------------------------------------
class Engine:
    """CKKS engine with desilofhe's constructor signatures (engine_context.py:27-31):

    1. ``Engine(mode='cpu', use_bootstrap=False, use_multiparty=False, thread_count=0, device_id=0)``
    2. ``Engine(max_level, mode='cpu', *, use_multiparty=False, thread_count=0, device_id=0)``
    3. ``Engine(log_coeff_count, special_prime_count, mode='cpu', ...)``

    ``mode`` is accepted for compatibility; execution is always the HIP engine on
    ``device_id`` (the product has no CPU path).  Extra keyword overrides (``log_n``,
    ``special_primes``, ``scale_bits``, ``base_bits``, ``special_bits``, ``seed``, ``digit_primes``
    -- the key-switch digit width alpha, default K) select explicit parameters; ``_lib`` injects
    another implementation of the ABI (tests use it for the CPU oracle).

    ``fuse_linear`` (default True): ``multiply(ct, constant)`` and the ``add`` calls that consume
    its result are deferred and materialised as one fused linear combination
    (``_LinearCiphertext``), and ``multiply(a, b, rlk)`` is deferred to its first use
    (``_ProductCiphertext``) so that products scaled by constants and summed become one fused
    bivariate evaluation; False evaluates every call eagerly (a rescale per product).  What can
    be checked at the call is checked there (operand levels, batch shapes, polynomial counts, the
    key's type and owning engine); an error of the evaluation itself (out of device memory, a
    device fault) surfaces at the first use of the deferred handle, as a RuntimeError naming the
    C call.  At most ``max_pending`` products (default 256) that no fused evaluation has taken
    wait unevaluated per engine: the next one evaluates the waiting ones first.  A product a
    fused sum has used no longer counts (it stays deferred; only a direct use of its handle
    evaluates it), so the cap never re-evaluates products whose value a poly2 result holds.

    Randomness: without ``seed`` the engine seed, every secret key created without a seed and
    the first encryption nonce are drawn from os.urandom.  With an explicit ``seed`` everything
    is reproducible and nonces count from ``nonce_start`` (default 0); engines that share a seed
    to share keys (one per rank) must use disjoint nonce ranges (parallel.rank_nonce_start),
    otherwise two encryptions would reuse the same (a, e) randomness.
    """

    def __init__(self, *args, mode: str = "cpu", use_bootstrap: bool = False,
                 use_multiparty: bool = False, thread_count: int = 0, device_id: int = 0,
                 max_level: int | None = None, log_coeff_count: int | None = None,
                 special_prime_count: int | None = None, log_n: int | None = None,
                 special_primes: int | None = None, scale_bits: int | None = None,
                 base_bits: int | None = None, special_bits: int | None = None,
                 seed: int | bytes | None = None, nonce_start: int | None = None,
                 fuse_linear: bool = True, digit_primes: int | None = None, max_pending: int = 256,
                 _lib: Lib | None = None):
        ints = [a for a in args if isinstance(a, (int, np.integer)) and not isinstance(a, bool)]
        strs = [a for a in args if isinstance(a, str)]
        if strs:
            mode = strs[0]
        if len(ints) == 1 and max_level is None:
            max_level = int(ints[0])
        elif len(ints) >= 2:
            log_coeff_count, special_prime_count = int(ints[0]), int(ints[1])
        if log_coeff_count is not None:          # signature 3
            ln = log_coeff_count
            k = special_prime_count or DEFAULT_PARAMS["special_primes"]
            budget = SECURITY_BUDGET.get(ln, 1772)
            lvl = max_level if max_level is not None else max(
                1, (budget - DEFAULT_PARAMS["base_bits"] - k * DEFAULT_PARAMS["special_bits"])
                // DEFAULT_PARAMS["scale_bits"])
            p = _params_for(log_n=log_n or ln, max_level=lvl, special_primes=special_primes or k,
                            scale_bits=scale_bits, base_bits=base_bits, special_bits=special_bits,
                            seed=seed, threads=thread_count, device=device_id, digit_primes=digit_primes)
        else:                                    # signatures 1 and 2
            p = _params_for(log_n=log_n, max_level=max_level, special_primes=special_primes,
                            scale_bits=scale_bits, base_bits=base_bits, special_bits=special_bits,
                            seed=seed, threads=thread_count, device=device_id, digit_primes=digit_primes)
        self.mode = mode
        self.use_bootstrap = use_bootstrap
        self.use_multiparty = use_multiparty
        self.thread_count = thread_count
        self.device_id = device_id
        self._lib = _lib if _lib is not None else load_product()
        self._params = p
        cp = Params(p["log_n"], p["max_level"], p["special_primes"], p["scale_bits"],
                    p["base_bits"], p["special_bits"], p["device"], p["threads"], p["seed"], None,
                    (C.c_uint64 * 3)(*p["seed_ext"]), p["digit_primes"])
        h = C.c_void_p()
        self._check(self._lib.engine_create(C.byref(cp), C.byref(h)))
        self._h = h.value
        dims = (C.c_int32 * 4)()
        self._lib.engine_dims(self._h, dims)
        self.log_coeff_count, self.max_level, self.special_prime_count, self.dnum = list(dims)
        # key-switch digit width alpha (aesfhe_params.digit_primes; 0 selects K)
        self.digit_primes = p["digit_primes"] or self.special_prime_count
        self.slot_count = 1 << (self.log_coeff_count - 1)
        np_ = self.max_level + 1 + self.special_prime_count
        primes = (C.c_uint64 * np_)()
        self._lib.engine_primes(self._h, primes)
        self.primes = [int(x) for x in primes]
        scales = (C.c_double * (self.max_level + 1))()
        self._lib.engine_scales(self._h, scales)
        self.scales = [float(x) for x in scales]
        self._random_keys = seed is None
        self._fuse_linear = bool(fuse_linear)
        import weakref
        self._pending = weakref.WeakSet()  # deferred products not yet evaluated
        self._pending_gal = []  # deferred automorphisms (weak references), in call order
        self._max_pending = int(max_pending)
        if nonce_start is None:
            nonce_start = _urandom64() >> 1 if seed is None else 0
        self._nonce = int(nonce_start)

    # -- plumbing ---------------------------------------------------------------------------
    def _check(self, rc):
        self._lib.check(rc)

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                self._lib.engine_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def _ct(self, h) -> Ciphertext:
        return Ciphertext(self, h)

    def _call_ct(self, fn, *args) -> Ciphertext:
        out = C.c_void_p()
        self._check(fn(self._h, *args, C.byref(out)))
        return self._ct(out.value)

    def _vec(self, data) -> np.ndarray:
        v = np.asarray(data)
        if v.ndim != 1:
            raise ValueError("expected a 1-D slot vector")
        if v.size > self.slot_count:
            raise ValueError(f"{v.size} values exceed slot_count {self.slot_count}")
        return v.astype(np.complex128, copy=False)

    def _encode_coeffs(self, values: np.ndarray, scale: float) -> np.ndarray:
        v = np.ascontiguousarray(values, dtype=np.complex128)
        re = np.ascontiguousarray(v.real)
        im = np.ascontiguousarray(v.imag)
        co = np.empty(1 << self.log_coeff_count, dtype=np.int64)
        self._check(self._lib.encode(self.log_coeff_count, _as_ptr(re, C.c_double),
                                     _as_ptr(im, C.c_double), v.size, scale,
                                     _as_ptr(co, C.c_int64)))
        return co

    def _galois_key(self, sk: SecretKey, g: int, cls):
        out = C.c_void_p()
        self._check(self._lib.key_galois(self._h, sk._h, g, C.byref(out)))
        k = self._key(cls, out.value)
        k.galois_elt = g
        return k

    # -- keys (engine_context.py:62-73) -------------------------------------------------------
    def _key(self, cls, h):
        """Key handles hold the engine: the C key's free returns its buffer to the engine's
        device pool, so the engine must outlive every key."""
        k = cls(self._lib, h, self._lib.key_free)
        k.engine = self
        return k

    def create_secret_key(self, seed: int | None = None) -> SecretKey:
        """Ternary secret key.  seed None: 0 for a seeded engine (reproducible), else a fresh
        os.urandom value -- engine_context.py:62 calls this without arguments."""
        if seed is None:
            seed = _urandom64() if self._random_keys else 0
        out = C.c_void_p()
        self._check(self._lib.key_secret(self._h, seed, C.byref(out)))
        return self._key(SecretKey, out.value)

    def create_public_key(self, sk: SecretKey) -> PublicKey:
        out = C.c_void_p()
        self._check(self._lib.key_public(self._h, sk._h, C.byref(out)))
        return self._key(PublicKey, out.value)

    def create_relinearization_key(self, sk: SecretKey) -> RelinearizationKey:
        out = C.c_void_p()
        self._check(self._lib.key_relin(self._h, sk._h, C.byref(out)))
        return self._key(RelinearizationKey, out.value)

    def create_conjugation_key(self, sk: SecretKey) -> ConjugationKey:
        g = self._lib.galois_elt(self.log_coeff_count, 0, 1)
        return self._galois_key(sk, g, ConjugationKey)

    def create_rotation_key(self, sk: SecretKey) -> RotationKey:
        return RotationKey(self, sk)

    def create_fixed_rotation_key(self, sk: SecretKey, delta: int) -> FixedRotationKey:
        g = self._lib.galois_elt(self.log_coeff_count, int(delta), 0)
        k = self._galois_key(sk, g, FixedRotationKey)
        k.delta = int(delta)
        return k

    def create_hoisted_rotation_key(self, sk: SecretKey, delta: int) -> FixedRotationKey:
        """Key for rotate_hoisted (aesfhe_key_galois_hoisted): same slots as
        create_fixed_rotation_key(sk, delta)."""
        g = self._lib.galois_elt(self.log_coeff_count, int(delta), 0)
        out = C.c_void_p()
        self._check(self._lib.key_galois_hoisted(self._h, sk._h, g, C.byref(out)))
        k = self._key(FixedRotationKey, out.value)
        k.galois_elt = g
        k.delta = int(delta)
        return k

    def rotate_hoisted(self, ct: Ciphertext, keys: Sequence[FixedRotationKey]) -> list:
        """Rotations of one ciphertext by every key (create_hoisted_rotation_key), the ModUp of
        c1 shared (aesfhe_rotate_hoisted)."""
        n = len(keys)
        arr = (c_key_p * n)(*[k._h for k in keys])
        outs = (C.c_void_p * n)()
        self._check(self._lib.rotate_hoisted(self._h, ct._h, arr, n, outs))
        return [self._ct(h) for h in outs]

    def create_sparse_secret_key(self, hw: int, seed: int | None = None) -> SecretKey:
        """Ternary secret with exactly hw nonzeros (aesfhe_key_secret_sparse)."""
        if seed is None:
            seed = _urandom64() if self._random_keys else 0
        out = C.c_void_p()
        self._check(self._lib.key_secret_sparse(self._h, seed, int(hw), C.byref(out)))
        return self._key(SecretKey, out.value)

    def create_switching_key(self, sk_from: SecretKey, sk_to: SecretKey) -> GaloisKey:
        """Key switching key sk_from -> sk_to, applied with switch_key (aesfhe_key_switch)."""
        out = C.c_void_p()
        self._check(self._lib.key_switch(self._h, sk_from._h, sk_to._h, C.byref(out)))
        k = self._key(GaloisKey, out.value)
        k.galois_elt = 1
        return k

    def switch_key(self, ct: Ciphertext, swk: GaloisKey) -> Ciphertext:
        return self._call_ct(self._lib.galois, ct._h, swk._h)

    def create_small_bootstrap_key(self, sk: SecretKey) -> BootstrapKey:
        return BootstrapKey(self, sk, small=True)

    def create_bootstrap_key(self, sk: SecretKey) -> BootstrapKey:
        return BootstrapKey(self, sk, small=False)

    # -- codec --------------------------------------------------------------------------------
    def encode(self, vec, level: int | None = None, scale: float | None = None) -> Plaintext:
        return Plaintext(self, self._vec(vec))

    def encrypt(self, data, key, level: int | None = None) -> Ciphertext:
        """Encrypt a slot vector (or a (B, <=slots) array as one batched ciphertext) under a
        public key (or, symmetrically, the secret key), zero-padded to slot_count
        (engine_context.py:81-85, xor_service.py:59-66).  The HIP engine copies the slots to the
        GPU once and encodes + encrypts there (encrypt_device: the device codec is bit-identical
        to the host one, same nonce sequence); the CPU oracle encodes on the host."""
        level = self.max_level if level is None else int(level)
        arr = np.asarray(data)
        rows = arr[None, :] if arr.ndim == 1 else arr
        if rows.ndim != 2 or rows.shape[1] > self.slot_count:
            raise ValueError(f"data must be (<= {self.slot_count},) or (B, <= {self.slot_count})")
        if self.on_device:
            import torch
            src = rows if np.iscomplexobj(rows) else rows.astype(np.float64, copy=False)
            return self.encrypt_device(torch.from_numpy(np.ascontiguousarray(src)), key, level)
        return self._encrypt_host(rows, key, level)

    def _encrypt_host(self, rows: np.ndarray, key, level: int) -> Ciphertext:
        """encrypt with the host codec (aesfhe_encode on the CPU, then aesfhe_encrypt)."""
        rows = np.asarray(rows)
        rows = rows[None, :] if rows.ndim == 1 else rows
        n = 1 << self.log_coeff_count
        co = np.empty((rows.shape[0], n), dtype=np.int64)
        for b in range(rows.shape[0]):
            co[b] = self._encode_coeffs(rows[b].astype(np.complex128), self.scales[level])
        nonce = self._nonce
        self._nonce += 1
        out = C.c_void_p()
        self._check(self._lib.encrypt(self._h, key._h, _as_ptr(co, C.c_int64), rows.shape[0],
                                      level, nonce, C.byref(out)))
        return self._ct(out.value)

    def decrypt(self, ct: Ciphertext, sk: SecretKey) -> np.ndarray:
        """Slot values of `ct` ((slot_count,) complex, or (B, slot_count) for a batch).  The HIP
        engine decrypts and decodes on the GPU (decrypt_device) and copies the slots back once."""
        if self.on_device:
            out = self.decrypt_device(ct, sk).cpu().numpy()
            return out[0] if ct.batch == 1 else out
        return self._decrypt_host(ct, sk)

    def _decrypt_host(self, ct: Ciphertext, sk: SecretKey) -> np.ndarray:
        """decrypt with the host codec (aesfhe_decrypt's coefficients decoded on the CPU)."""
        n = 1 << self.log_coeff_count
        co = np.empty((ct.batch, n), dtype=np.int64)
        self._check(self._lib.decrypt(self._h, sk._h, ct._h, _as_ptr(co, C.c_int64)))
        out = np.empty((ct.batch, self.slot_count), dtype=np.complex128)
        re = np.empty(self.slot_count)
        im = np.empty(self.slot_count)
        scale = self.scales[ct.level]
        for b in range(ct.batch):
            row = np.ascontiguousarray(co[b])
            self._check(self._lib.decode(self.log_coeff_count, _as_ptr(row, C.c_int64), scale,
                                         _as_ptr(re, C.c_double), _as_ptr(im, C.c_double)))
            out[b] = re + 1j * im
        return out[0] if ct.batch == 1 else out

    # -- arithmetic ---------------------------------------------------------------------------
    def _as_plain(self, x) -> Plaintext:
        if isinstance(x, Plaintext):
            return x
        if np.isscalar(x):
            return Plaintext(self, np.full(self.slot_count, complex(x), dtype=np.complex128))
        return Plaintext(self, self._vec(x))

    def add(self, a, b) -> Ciphertext:
        if isinstance(a, _LinearCiphertext) or isinstance(b, _LinearCiphertext):
            r = self._linear_add(a, b)
            if r is not None:
                return r
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            return self._call_ct(self._lib.add, a._h, b._h)
        if not isinstance(a, Ciphertext):
            a, b = b, a
        pt = self._as_plain(b)
        if pt.is_const:
            c = pt.const
            return self._call_ct(self._lib.add_const, a._h, c.real, c.imag)
        return self._call_ct(self._lib.add_pt, a._h, pt.device(a.level, self.scales[a.level]))

    def subtract(self, a, b) -> Ciphertext:
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            return self._call_ct(self._lib.sub, a._h, b._h)
        if isinstance(a, Ciphertext):
            return self.add(a, self._as_plain(b).values * -1)
        return self.add(self.negate(b), a)

    sub = subtract

    def negate(self, a: Ciphertext) -> Ciphertext:
        return self._call_ct(self._lib.negate, a._h)

    def multiply(self, a, b, relinearization_key: RelinearizationKey | None = None) -> Ciphertext:
        if isinstance(a, Ciphertext) and isinstance(b, Ciphertext):
            if relinearization_key is not None:
                if getattr(relinearization_key, "engine", self) is not self:
                    raise ValueError("multiply: the relinearization key belongs to another engine")
                if (self._fuse_linear and a.npoly == 2 and b.npoly == 2 and min(a.level, b.level) >= 1
                        and (a.batch == b.batch or 1 in (a.batch, b.batch))
                        and isinstance(relinearization_key, RelinearizationKey)):
                    if len(self._pending) >= self._max_pending:
                        Engine.materialize([p for p in list(self._pending) if p.pending])
                    p = _ProductCiphertext(self, a, b, relinearization_key)
                    self._pending.add(p)
                    return p
                return self._call_ct(self._lib.mul, a._h, b._h, relinearization_key._h)
            t = self._call_ct(self._lib.tensor, a._h, b._h)
            return self._call_ct(self._lib.rescale, t._h)
        if not isinstance(a, Ciphertext):
            a, b = b, a
        if not isinstance(a, Ciphertext):
            raise TypeError("multiply needs at least one Ciphertext")
        pt = self._as_plain(b)
        if pt.is_const:
            c = pt.const
            if self._fuse_linear and a.npoly == 2 and a.level >= 1:
                terms = [(a, c)] if c != 0 else []
                return _LinearCiphertext(self, terms, [], 0, a.level - 1, a.batch)
            return self._call_ct(self._lib.mul_const, a._h, c.real, c.imag)
        scale = self._lib.engine_mul_scale(self._h, a.level)
        return self._call_ct(self._lib.mul_pt, a._h, pt.device(a.level, scale))

    # -- deferred linear combinations (_LinearCiphertext) -------------------------------------
    def _linear_add(self, a, b):
        """a + b with at least one deferred operand: the merged deferred sum, or None when b is
        not linear in the sense above (a non-constant plaintext, a 3-polynomial ciphertext)."""
        L, o = (a, b) if isinstance(a, _LinearCiphertext) else (b, a)
        if isinstance(o, Ciphertext):
            if o.npoly != 2:
                return None
            if L.batch != o.batch and 1 not in (L.batch, o.batch):
                raise RuntimeError(f"batch mismatch {L.batch} vs {o.batch}")
            if isinstance(o, _LinearCiphertext):
                terms, adds, const = L._terms + o._terms, L._addends + o._addends, L._const + o._const
            else:
                terms, adds, const = L._terms, L._addends + [o], L._const
            return _LinearCiphertext(self, terms, adds, const, min(L.level, o.level), max(L.batch, o.batch))
        pt = self._as_plain(o)
        if not pt.is_const:
            return None
        return _LinearCiphertext(self, L._terms, L._addends, L._const + pt.const, L.level, L.batch)

    def _materialize(self, L: "_LinearCiphertext") -> Ciphertext:
        """One aesfhe_lincomb of the terms (one rescale of the sum), then the ciphertext addends
        (level-aligned adds) and the constant, at the deferred object's level."""
        x = None
        plain, prods = [], {}
        for c, k in L._terms:
            if isinstance(c, _ProductCiphertext) and c.pending:
                if not c.is_zero:
                    prods.setdefault(id(c._rlk), []).append((c, k))
            else:
                plain.append((c, k))
        for group in prods.values():
            y = self._product_sum(group)
            x = y if x is None else self._call_ct(self._lib.add, x._h, y._h)
        if plain:
            y = self.lincomb([c for c, _ in plain], [k for _, k in plain])
            x = y if x is None else self._call_ct(self._lib.add, x._h, y._h)
        for c in L._addends:
            x = c if x is None else self._call_ct(self._lib.add, x._h, c._h)
        if x is None:
            x = self.zeros(L.batch, L.level)
        if x.batch < L.batch:  # every part was a broadcast (B = 1) operand
            x = self.concat([x] * L.batch)
        if L._const != 0:
            x = self._call_ct(self._lib.add_const, x._h, L._const.real, L._const.imag)
        if x.level > L.level:
            x = self.level_down(x, L.level)
        return x

    def _product_sum(self, terms) -> Ciphertext:
        """sum_t k_t a_t b_t over deferred products of one relinearisation key: one aesfhe_poly2
        call (the distinct left operands as its x basis, the right ones as its y basis, at most
        15 each), else the products one by one."""
        xs, ys = {}, {}
        for p, _ in terms:
            xs.setdefault(id(p._a), p._a)
            ys.setdefault(id(p._b), p._b)
        if len(xs) > 15 or len(ys) > 15:
            return self.lincomb([p for p, _ in terms], [k for _, k in terms])
        # the fused evaluation has used these products: they no longer count against max_pending
        # (which bounds the products no evaluation has taken yet).  Each stays deferred: a later
        # direct use of its handle still evaluates it.
        for p, _ in terms:
            self._pending.discard(p)
        xi = {k: i + 1 for i, k in enumerate(xs)}
        yi = {k: j + 1 for j, k in enumerate(ys)}
        C = np.zeros((1, len(xs) + 1, len(ys) + 1), dtype=np.complex128)
        for p, k in terms:
            C[0, xi[id(p._a)], yi[id(p._b)]] += k
        return self.poly2(list(xs.values()), list(ys.values()), C, terms[0][0]._rlk)[0]

    def multiply_fma(self, a: Ciphertext, b: Ciphertext, relinearization_key: RelinearizationKey,
                     alpha: int = 1, c: Ciphertext | None = None, gamma: float = 0.0,
                     beta: float = 0.0) -> Ciphertext:
        """alpha * a * b + gamma * c + beta with one relinearisation + rescale (aesfhe_mul_fma);
        c (level >= the product's) is truncated, not level-downed."""
        return self._call_ct(self._lib.mul_fma, a._h, b._h, relinearization_key._h, int(alpha),
                             c._h if c is not None else None, float(gamma), float(beta))

    def relinearize(self, ct: Ciphertext, relinearization_key: RelinearizationKey) -> Ciphertext:
        return self._call_ct(self._lib.relinearize, ct._h, relinearization_key._h)

    def rescale(self, ct: Ciphertext) -> Ciphertext:
        return self._call_ct(self._lib.rescale, ct._h)

    def level_down(self, ct: Ciphertext, level: int) -> Ciphertext:
        return self._call_ct(self._lib.level_down, ct._h, int(level))

    def make_power_basis(self, ct: Ciphertext, degree: int,
                         relinearization_key: RelinearizationKey) -> list:
        outs = (c_ct_p * degree)()
        self._check(self._lib.power_basis(self._h, ct._h, int(degree), relinearization_key._h,
                                          outs))
        return [self._ct(outs[i]) for i in range(degree)]

    def conjugate(self, ct: Ciphertext, conjugation_key: ConjugationKey) -> Ciphertext:
        """Complex conjugation of the slots.  With fuse_linear the call is deferred and batched
        with the other pending conjugations of its level (_GaloisCiphertext)."""
        if getattr(conjugation_key, "engine", self) is not self:
            raise ValueError("conjugate: the key belongs to another engine")
        if self._fuse_linear and ct.npoly == 2 and not ct.is_zero:
            import weakref
            g = _GaloisCiphertext(self, ct, conjugation_key)
            self._pending_gal.append(weakref.ref(g))
            if len(self._pending_gal) > self._max_pending:
                self._flush_galois(None)
            return g
        return self._call_ct(self._lib.galois, ct._h, conjugation_key._h)

    def _flush_galois(self, key):
        """Evaluate the pending deferred automorphisms (of `key`, or all): per (key, level), the
        sources concatenated along the batch, one aesfhe_galois, the result split back."""
        live = [r() for r in self._pending_gal]
        live = [g for g in live if g is not None and g._mat is None]
        todo = [g for g in live if key is None or g._key is key]
        self._pending_gal = [r for r in self._pending_gal
                             if r() is not None and r()._mat is None and r() not in todo]
        groups = {}
        for g in todo:
            groups.setdefault((id(g._key), g.level), []).append(g)
        for grp in groups.values():
            k = grp[0]._key
            if len(grp) == 1:
                g = grp[0]
                g._mat = self._call_ct(self._lib.galois, g._src._h, k._h)
            else:
                cat = self.concat([g._src for g in grp])
                out = self._call_ct(self._lib.galois, cat._h, k._h)
                off = 0
                for g in grp:
                    g._mat = self.slice(out, off, g.batch)
                    off += g.batch
            for g in grp:
                g._src = None

    def rotate(self, ct: Ciphertext, key, delta: int | None = None) -> Ciphertext:
        """np.roll semantics: rotate(ct, key, k) decrypts to np.roll(v, k)."""
        if isinstance(key, FixedRotationKey):
            if delta is not None and int(delta) % self.slot_count != key.delta % self.slot_count:
                raise RuntimeError(f"fixed rotation key is for {key.delta}, not {delta}")
            return self._call_ct(self._lib.galois, ct._h, key._h)
        if not isinstance(key, RotationKey):
            raise TypeError("rotate needs a RotationKey or FixedRotationKey")
        n = self.slot_count
        left = (-int(delta)) % n
        out = ct
        for step in _naf_steps(left, n):
            out = self._call_ct(self._lib.galois, out._h, key.left(step)._h)
        if out is ct:
            out = self._call_ct(self._lib.ct_copy, ct._h)
        return out

    def bootstrap(self, ct: Ciphertext, relinearization_key: RelinearizationKey,
                  conjugation_key: ConjugationKey, bootstrap_key: BootstrapKey) -> Ciphertext:
        """Refresh `ct` (any level) to level max_level - depth (xor_service.py:120-129 calls
        this with the context's rlk, conjugation and bootstrap keys).  bootstrap.Bootstrapper
        states the algorithm; the slots come back with the precision DESIGN.md section 7 lists."""
        if not isinstance(bootstrap_key, BootstrapKey):
            raise TypeError("bootstrap needs the key from create_bootstrap_key")
        return bootstrap_key.bootstrapper(relinearization_key, conjugation_key).bootstrap(ct)

    # -- fused building blocks used by the optimised AES round ---------------------------------
    def mod_raise(self, ct: Ciphertext, level: int | None = None) -> Ciphertext:
        """Limb 0 lifted to every limb of `level` (aesfhe_mod_raise): encrypts m + q_0 I."""
        return self._call_ct(self._lib.mod_raise, ct._h, self.max_level if level is None else int(level))

    def multiply_i(self, ct: Ciphertext, sign: int = 1) -> Ciphertext:
        """Every slot times i (sign > 0) or -i, exactly, without using a level (aesfhe_mul_i)."""
        return self._call_ct(self._lib.mul_i, ct._h, 1 if sign > 0 else -1)

    def dot_plain(self, cts: Sequence[Ciphertext], plains: Sequence["Plaintext"]) -> Ciphertext:
        """sum_i cts[i] * plains[i] with one rescale (aesfhe_dot_pt)."""
        n = len(cts)
        lv = min(c.level for c in cts)
        s = self._lib.engine_mul_scale(self._h, lv)
        arr = (c_ct_p * n)(*[c._h for c in cts])
        pts = (c_pt_p * n)(*[p.device(lv, s) for p in plains])
        return self._call_ct(self._lib.dot_pt, arr, pts, n)

    def linear_bsgs(self, ct: Ciphertext, baby_keys: Sequence, giant_keys: Sequence,
                    terms: Sequence[Sequence]) -> Ciphertext:
        """sum_j rot_{giant_keys[j]}(sum_{(i, pt) in terms[j]} pt * rot_{baby_keys[i]}(ct)), one
        level (aesfhe_linear_bsgs: hoisted babies, lazy ModDown).  baby_keys: hoisted rotation
        keys or None (identity); giant_keys: fixed rotation keys or None; terms[j]: (baby index,
        Plaintext) pairs, encoded at mul_scale(ct.level) over Q u P."""
        nb, ng = len(baby_keys), len(giant_keys)
        s = self._lib.engine_mul_scale(self._h, ct.level)
        bk = (c_key_p * nb)(*[k._h if k is not None else None for k in baby_keys])
        gk = (c_key_p * ng)(*[k._h if k is not None else None for k in giant_keys])
        nterm = (C.c_int32 * ng)(*[len(t) for t in terms])
        flat = [x for t in terms for x in t]
        tb = (C.c_int32 * len(flat))(*[i for i, _ in flat])
        pts = (c_pt_p * len(flat))(*[p.device(ct.level, s, ext=True) for _, p in flat])
        return self._call_ct(self._lib.linear_bsgs, ct._h, nb, bk, ng, gk, nterm, tb, pts)

    def lincomb(self, cts: Sequence[Ciphertext], coeffs: Sequence[complex]) -> Ciphertext:
        n = len(cts)
        arr = (c_ct_p * n)(*[c._h for c in cts])
        co = np.asarray(coeffs, dtype=np.complex128)
        re = np.ascontiguousarray(co.real)
        im = np.ascontiguousarray(co.imag)
        return self._call_ct(self._lib.lincomb, arr, n, _as_ptr(re, C.c_double),
                             _as_ptr(im, C.c_double))

    def lincomb_many(self, cts: Sequence[Ciphertext], coeffs) -> list:
        """Rows of a (m, n) coefficient matrix applied to the same n ciphertexts in one pass."""
        n = len(cts)
        M = np.ascontiguousarray(np.asarray(coeffs, dtype=np.complex128).reshape(-1, n))
        m = M.shape[0]
        arr = (c_ct_p * n)(*[c._h for c in cts])
        re = np.ascontiguousarray(M.real)
        im = np.ascontiguousarray(M.imag)
        outs = (c_ct_p * m)()
        self._check(self._lib.lincomb_many(self._h, arr, n, _as_ptr(re, C.c_double),
                                           _as_ptr(im, C.c_double), m, outs))
        return [self._ct(outs[i]) for i in range(m)]

    def dot(self, a: Sequence[Ciphertext], b: Sequence[Ciphertext],
            relinearization_key: RelinearizationKey) -> Ciphertext:
        n = len(a)
        aa = (c_ct_p * n)(*[c._h for c in a])
        bb = (c_ct_p * n)(*[c._h for c in b])
        return self._call_ct(self._lib.dot, aa, bb, n, relinearization_key._h)

    def dot_fma(self, a: Sequence[Ciphertext], b: Sequence[Ciphertext], relinearization_key: RelinearizationKey,
                addends: Sequence = (), beta: float = 0.0) -> Ciphertext:
        """sum_i a_i b_i + sum_j gamma_j c_j + beta for addends [(c_j, gamma_j)] (real gamma, c_j at
        least at the products' level, truncated) with one relinearisation + rescale
        (aesfhe_dot_fma)."""
        n, nc = len(a), len(addends)
        aa = (c_ct_p * n)(*[c._h for c in a])
        bb = (c_ct_p * n)(*[c._h for c in b])
        cc = (c_ct_p * max(nc, 1))(*[c._h for c, _ in addends])
        g = np.ascontiguousarray([float(k) for _, k in addends] or [0.0], dtype=np.float64)
        return self._call_ct(self._lib.dot_fma, aa, bb, n, cc, _as_ptr(g, C.c_double), nc, float(beta),
                             relinearization_key._h)

    def poly2(self, x_basis: Sequence[Ciphertext], y_basis: Sequence[Ciphertext], coeffs,
              relinearization_key: RelinearizationKey) -> list:
        """outs[t] = sum_{i,j} C[t, i, j] x^i y^j for C of shape (m, nx, ny), with
        x_basis = [x^1..x^{nx-1}] and y_basis = [y^1..y^{ny-1}] (aesfhe_poly2: fused inner sums,
        one relinearisation per output, two levels)."""
        Cf = np.asarray(coeffs, dtype=np.complex128)
        if Cf.ndim == 2:
            Cf = Cf[None]
        m, nx, ny = Cf.shape
        if len(x_basis) != nx - 1 or len(y_basis) != ny - 1:
            raise ValueError("poly2: basis lengths must be nx-1 and ny-1")
        xa = (c_ct_p * max(nx - 1, 1))(*[c._h for c in x_basis])
        ya = (c_ct_p * max(ny - 1, 1))(*[c._h for c in y_basis])
        re = np.ascontiguousarray(Cf.real)
        im = np.ascontiguousarray(Cf.imag)
        outs = (c_ct_p * m)()
        self._check(self._lib.poly2(self._h, xa, nx, ya, ny, _as_ptr(re, C.c_double),
                                    _as_ptr(im, C.c_double), m, relinearization_key._h, outs))
        return [self._ct(outs[i]) for i in range(m)]

    def poly2_int(self, x_basis: Sequence[Ciphertext], y_basis: Sequence[Ciphertext], weights,
                  den: int, relinearization_key: RelinearizationKey, slab_rot: int = 0) -> list:
        """poly2 with integer-weight coefficients C = weights / den (aesfhe_poly2_int): exact
        integer inner sums, one constant per pair of basis levels.  slab_rot (aesfhe_poly2_int_rot):
        output element 4 s + c takes the value at input element 4 s + ((c + slab_rot) mod 4)."""
        Wi = np.asarray(weights)
        if Wi.ndim == 2:
            Wi = Wi[None]
        if not np.array_equal(Wi, np.round(Wi)):
            raise ValueError("poly2_int: weights must be integers")
        Wi = np.ascontiguousarray(Wi, dtype=np.int32)
        m, nx, ny = Wi.shape
        if len(x_basis) != nx - 1 or len(y_basis) != ny - 1:
            raise ValueError("poly2_int: basis lengths must be nx-1 and ny-1")
        xa = (c_ct_p * max(nx - 1, 1))(*[c._h for c in x_basis])
        ya = (c_ct_p * max(ny - 1, 1))(*[c._h for c in y_basis])
        outs = (c_ct_p * m)()
        if slab_rot:
            self._check(self._lib.poly2_int_rot(self._h, xa, nx, ya, ny, _as_ptr(Wi, C.c_int32), int(den), m,
                                                relinearization_key._h, int(slab_rot), outs))
        else:
            self._check(self._lib.poly2_int(self._h, xa, nx, ya, ny, _as_ptr(Wi, C.c_int32), int(den), m,
                                            relinearization_key._h, outs))
        return [self._ct(outs[i]) for i in range(m)]

    def align(self, cts: Sequence[Ciphertext], level: int | None = None) -> list:
        """Exact-scale level-down of every ciphertext to `level` (default: the lowest)."""
        level = min(c.level for c in cts) if level is None else level
        return [c if c.level == level else self.level_down(c, level) for c in cts]

    def zeros(self, batch: int = 1, level: int | None = None) -> Ciphertext:
        level = self.max_level if level is None else level
        return self._call_ct(self._lib.ct_zero, batch, level)

    def concat(self, cts: Sequence[Ciphertext]) -> Ciphertext:
        arr = (c_ct_p * len(cts))(*[c._h for c in cts])
        return self._call_ct(self._lib.ct_concat, arr, len(cts))

    def slice(self, ct: Ciphertext, start: int, count: int) -> Ciphertext:
        return self._call_ct(self._lib.ct_slice, ct._h, start, count)

    def gather(self, ct: Ciphertext, idx: Sequence[int]) -> Ciphertext:
        """Batch permutation / repetition: element b of the result is element idx[b] of ct
        (aesfhe_ct_gather, one copy pass)."""
        arr = (C.c_int32 * len(idx))(*[int(i) for i in idx])
        return self._call_ct(self._lib.ct_gather, ct._h, arr, len(idx))

    def export_residues(self, ct: Ciphertext) -> np.ndarray:
        n = 1 << self.log_coeff_count
        out = np.empty((ct.batch, ct.npoly, ct.level + 1, n), dtype=np.uint64)
        self._check(self._lib.ct_export(self._h, ct._h, _as_ptr(out, C.c_uint64)))
        return out

    def import_residues(self, arr: np.ndarray) -> Ciphertext:
        a = np.ascontiguousarray(arr, dtype=np.uint64)
        b, p, l1, _ = a.shape
        return self._call_ct(self._lib.ct_import, _as_ptr(a, C.c_uint64), b, p, l1 - 1)

    # -- device-resident client path (aesfhe_*_device) -------------------
    @property
    def client_device(self):
        """torch device of client-path buffers: the engine's GPU (HIP engine) or the CPU (the
        oracle, whose "device" memory is host memory)."""
        import torch
        return torch.device("cuda", self.device_id) if self.on_device else torch.device("cpu")

    def _torch_sync(self):
        import torch
        if self.on_device:
            torch.cuda.current_stream(self.client_device).synchronize()

    def encrypt_device(self, values, key, level: int | None = None) -> Ciphertext:
        """Encrypt a (B, <= slot_count) torch tensor of slot values (real or complex) that lives
        on `client_device`: device encode (aesfhe_encode_device, bit-identical to the host codec)
        and encryption (aesfhe_encrypt_device), no host copy.  Same nonce sequence as encrypt."""
        import torch
        level = self.max_level if level is None else int(level)
        dev = self.client_device
        t = values if isinstance(values, torch.Tensor) else torch.as_tensor(np.asarray(values))
        t = t.to(dev)
        if t.ndim == 1:
            t = t[None]
        if t.ndim != 2 or t.shape[1] > self.slot_count:
            raise ValueError(f"values must be (<= {self.slot_count},) or (B, <= {self.slot_count})")
        B, ns = t.shape
        if t.is_complex():
            re, im = t.real.to(torch.float64).contiguous(), t.imag.to(torch.float64).contiguous()
        else:
            re, im = t.to(torch.float64).contiguous(), None
        co = torch.empty((B, 1 << self.log_coeff_count), dtype=torch.int64, device=dev)
        self._torch_sync()  # the slot tensors are written on torch's stream
        self._check(self._lib.encode_device(self._h, re.data_ptr(), im.data_ptr() if im is not None else None,
                                            B, ns, ns, self.scales[level], co.data_ptr()))
        nonce = self._nonce
        self._nonce += 1
        out = C.c_void_p()
        self._check(self._lib.encrypt_device(self._h, key._h, co.data_ptr(), B, level, nonce, C.byref(out)))
        self.synchronize()  # co is read on the engine's stream; torch may recycle it on return
        return self._ct(out.value)

    def decrypt_device(self, ct: Ciphertext, sk: SecretKey):
        """Decrypt + decode into a (B, slot_count) complex128 torch tensor on `client_device`
        (aesfhe_decrypt_device + aesfhe_decode_device: no host copy)."""
        import torch
        dev = self.client_device
        n = self.slot_count
        co = torch.empty((ct.batch, 2 * n), dtype=torch.int64, device=dev)
        re = torch.empty((ct.batch, n), dtype=torch.float64, device=dev)
        im = torch.empty((ct.batch, n), dtype=torch.float64, device=dev)
        self._torch_sync()
        self._check(self._lib.decrypt_device(self._h, sk._h, ct._h, co.data_ptr()))
        self._check(self._lib.decode_device(self._h, co.data_ptr(), ct.batch, self.scales[ct.level],
                                            re.data_ptr(), im.data_ptr()))
        self.synchronize()
        return torch.complex(re, im)

    # -- device-resident transfer (parallel.py: RCCL scatter / gather) ------------------------
    @property
    def on_device(self) -> bool:
        """True for the HIP engine (buffers handed to export_into / import_from live in device
        memory); False for the CPU oracle (host memory)."""
        return self._lib.backend.startswith("hip")

    def export_into(self, ct: Ciphertext, ptr: int, start: int = 0, count: int | None = None):
        """Residues of batch elements [start, start + count) into the buffer at address `ptr`
        (device memory of this engine's GPU; aesfhe_ct_export_device)."""
        count = ct.batch - start if count is None else count
        self._check(self._lib.ct_export_device(self._h, ct._h, int(start), int(count), C.c_void_p(ptr)))

    def import_from(self, ptr: int, batch: int, npoly: int, level: int) -> Ciphertext:
        """A ciphertext copied from residues at address `ptr` (aesfhe_ct_import_device)."""
        return self._call_ct(self._lib.ct_import_device, C.c_void_p(ptr), int(batch), int(npoly), int(level))

    # -- serialisation --------------------------------------------------
    def key_fingerprint(self) -> int:
        """63-bit digest of the engine key (256-bit seed) and prime chain: equal on two engines
        iff they derive the same keys from the same key seeds (parallel.py checks it across
        ranks before moving ciphertexts between them)."""
        import hashlib
        p = self._params
        ident = (p["seed"], tuple(p["seed_ext"]), tuple(self.primes))
        if self.digit_primes != self.special_prime_count:  # another key layout (digits)
            ident += (self.digit_primes,)
        h = hashlib.sha256(repr(ident).encode()).digest()
        return int.from_bytes(h[:8], "little") >> 1

    def _fingerprint(self) -> dict:
        fp = {"log_n": self.log_coeff_count, "max_level": self.max_level,
              "special_primes": self.special_prime_count, "primes": self.primes}
        if self.digit_primes != self.special_prime_count:  # keys of another digit layout
            fp["digit_primes"] = self.digit_primes
        return fp

    def save(self, obj, path) -> None:
        """Write a Ciphertext or key (SecretKey, PublicKey, RelinearizationKey, GaloisKey and
        subclasses) to `path`: magic, a JSON header (kind, shape, the engine's prime chain) and
        the NTT-domain residues as little-endian u64.  A RotationKey is not saved: it is derived
        on use from its secret key."""
        import json
        hdr = {"fp": self._fingerprint()}
        if isinstance(obj, Ciphertext):
            data = self.export_residues(obj)
            hdr.update(type="ciphertext", batch=obj.batch, npoly=obj.npoly, level=obj.level)
        elif isinstance(obj, _Key):
            kind, g, seed, words = C.c_int32(), C.c_uint64(), C.c_uint64(), C.c_int64()
            self._check(self._lib.key_export(self._h, obj._h, C.byref(kind), C.byref(g), C.byref(seed),
                                             C.byref(words), None))
            data = np.empty(words.value, dtype=np.uint64)
            self._check(self._lib.key_export(self._h, obj._h, C.byref(kind), C.byref(g), C.byref(seed),
                                             C.byref(words), _as_ptr(data, C.c_uint64)))
            hdr.update(type="key", cls=type(obj).__name__, kind=kind.value, galois=g.value,
                       keyseed=seed.value, delta=getattr(obj, "delta", None))
        else:
            raise TypeError(f"cannot save {type(obj).__name__}")
        head = json.dumps(hdr).encode()
        with open(path, "wb") as f:
            f.write(_MAGIC + len(head).to_bytes(8, "little") + head)
            f.write(np.ascontiguousarray(data).astype("<u8", copy=False).tobytes())

    def load(self, path):
        """Read an object written by save(); raises RuntimeError if it was made by an engine with
        other parameters (prime chain)."""
        import json
        with open(path, "rb") as f:
            if f.read(len(_MAGIC)) != _MAGIC:
                raise RuntimeError(f"{path}: not an aes-fhe object file")
            hdr = json.loads(f.read(int.from_bytes(f.read(8), "little")))
            data = np.frombuffer(f.read(), dtype="<u8")
        if hdr["fp"] != self._fingerprint():
            raise RuntimeError(f"{path}: written by an engine with different parameters")
        if hdr["type"] == "ciphertext":
            n = 1 << self.log_coeff_count
            return self.import_residues(data.reshape(hdr["batch"], hdr["npoly"], hdr["level"] + 1, n))
        cls = {c.__name__: c for c in (SecretKey, PublicKey, RelinearizationKey, GaloisKey,
                                       ConjugationKey, FixedRotationKey)}[hdr["cls"]]
        arr = np.ascontiguousarray(data, dtype=np.uint64)
        out = C.c_void_p()
        self._check(self._lib.key_import(self._h, hdr["kind"], hdr["galois"], hdr["keyseed"],
                                         _as_ptr(arr, C.c_uint64), arr.size, C.byref(out)))
        k = self._key(cls, out.value)
        if isinstance(k, GaloisKey):
            k.galois_elt = hdr["galois"]
        if isinstance(k, FixedRotationKey):
            k.delta = hdr["delta"]
        return k

    def key_bytes(self, key) -> int:
        """Device bytes of a key's residues (aesfhe_key_export's word count x 8)."""
        kind, g, seed, words = C.c_int32(), C.c_uint64(), C.c_uint64(), C.c_int64()
        self._check(self._lib.key_export(self._h, key._h, C.byref(kind), C.byref(g), C.byref(seed),
                                         C.byref(words), None))
        return 8 * words.value

    def key_seed(self, key) -> int:
        """The key seed a key was derived from (aesfhe_key_export's keyseed): two secret keys of
        one engine with the same seed are the same key (Bootstrapper(share=) checks it)."""
        kind, g, seed, words = C.c_int32(), C.c_uint64(), C.c_uint64(), C.c_int64()
        self._check(self._lib.key_export(self._h, key._h, C.byref(kind), C.byref(g), C.byref(seed),
                                         C.byref(words), None))
        return int(seed.value)

    def trim_key(self, key, max_level: int):
        """Keep only the key-switch digits a switch at level <= max_level reads
        (aesfhe_key_trim): the kept digits are the full key's word for word; a later switch above
        max_level raises.  Used for the bootstrapper's SlotToCoeff keys (trim_bootstrap_keys)."""
        self._check(self._lib.key_trim(self._h, key._h, int(max_level)))
        return key

    def pool_stats(self) -> dict:
        """Device pool counters (aesfhe_engine_pool_stats): bytes held / live, hipMalloc calls,
        trims, reuses of a larger cached block."""
        a = (C.c_int64 * 7)()
        self._check(self._lib.engine_pool_stats(self._h, a))
        return dict(zip(("held", "live", "mallocs", "trims", "reuse_larger", "peak_live", "fragmentation"),
                        [int(x) for x in a]))

    def pool_trim(self):
        """Release the cached device blocks (aesfhe_engine_pool_trim), e.g. between workloads."""
        self._check(self._lib.engine_pool_trim(self._h))

    def synchronize(self):
        self._check(self._lib.engine_sync(self._h))

    @staticmethod
    def materialize(obj):
        """Evaluate every deferred ciphertext (products, linear combinations) in a ciphertext
        or a nested list / tuple of them now (enqueued on the engine's stream); returns obj."""
        if isinstance(obj, Ciphertext):
            obj._h
        elif isinstance(obj, (list, tuple)):
            for o in obj:
                Engine.materialize(o)
        return obj


def _naf_steps(r: int, n: int) -> list:
    """Signed power-of-two steps summing to r (mod n), fewest terms (NAF of r or r - n)."""
    def naf(x):
        out, i = [], 0
        while x:
            if x & 1:
                d = 2 - (x & 3)
                out.append(d << i)
                x -= d
            x >>= 1
            i += 1
        return out
    if r == 0:
        return []
    a, b = naf(r), [-s for s in naf(n - r)]
    return a if len(a) <= len(b) else b
