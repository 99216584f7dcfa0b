"""The CPU oracle pinned before it is trusted: the reference's engine-contract tests
(test/test_engine_rot.py:21-61) restated on it, NTT known answers against big-integer
schoolbook negacyclic convolution, canonical-embedding encode against direct evaluation."""
import ctypes as C

import numpy as np
import pytest

from aes_xor_fhe.fhe import Engine

KW = dict(log_n=10, max_level=6, special_primes=2, seed=5)


@pytest.fixture(scope="module")
def env(oracle_lib):
    e = Engine(_lib=oracle_lib, **KW)
    sk = e.create_secret_key()
    return e, sk, e.create_public_key(sk), e.create_relinearization_key(sk), e.create_rotation_key(sk)


def test_encrypt_decrypt_identity(env):            # test_engine_rot.py:21-29
    e, sk, pk, *_ = env
    vec = np.linspace(0.0, 1.0, num=e.slot_count)
    np.testing.assert_allclose(e.decrypt(e.encrypt(vec, pk), sk), vec, atol=1e-6)


@pytest.mark.parametrize("k", [5, -4, 1, 300, -511])
def test_rotate_is_np_roll(env, k):                # test_engine_rot.py:32-40
    e, sk, pk, _, rot = env
    base = np.arange(e.slot_count, dtype=np.float64)
    np.testing.assert_allclose(e.decrypt(e.rotate(e.encrypt(base, pk), rot, k), sk),
                               np.roll(base, k), atol=1e-6)


def test_relinearize_noop_and_error(env):          # test_engine_rot.py:43-50
    e, sk, pk, rlk, _ = env
    from aes_xor_fhe.xor_service import EngineWrapper
    vec = np.random.RandomState(0).rand(e.slot_count)
    ct = e.encrypt(vec, pk)
    with pytest.raises(RuntimeError, match="should have 3 polynomials"):
        e.relinearize(ct, rlk)

    class Ctx:  # EngineWrapper over an existing engine (xor_service.py:107-118 swallow path)
        engine, secret_key, public_key, relinearization_key = e, sk, pk, rlk
        conjugation_key = rotation_key = bootstrap_key = None
    ew = EngineWrapper(None, ctx=Ctx)
    np.testing.assert_allclose(e.decrypt(ew.relinearize(ct), sk), vec, atol=1e-6)


def test_square_after_relin(env):                  # test_engine_rot.py:53-61
    e, sk, pk, rlk, _ = env
    vec = np.random.RandomState(1).rand(e.slot_count)
    ct = e.encrypt(vec, pk)
    sq = e.multiply(ct, ct, rlk)
    assert sq.level == ct.level - 1
    np.testing.assert_allclose(e.decrypt(sq, sk), vec * vec, atol=1e-5)
    # unrelinearised product + explicit relinearize
    t3 = e.multiply(ct, ct)
    assert t3.npoly == 3
    np.testing.assert_allclose(e.decrypt(e.relinearize(t3, rlk), sk), vec * vec, atol=1e-5)


@pytest.mark.parametrize("log_n", [4, 6, 8])
def test_ntt_known_answer_schoolbook(oracle_lib, log_n):
    e = Engine(_lib=oracle_lib, log_n=log_n, max_level=2, special_primes=1, seed=1)
    N = 1 << log_n
    rng = np.random.default_rng(log_n)
    for pid, q in enumerate(e.primes):
        a = rng.integers(0, q, N, dtype=np.uint64)
        b = rng.integers(0, q, N, dtype=np.uint64)
        # schoolbook negacyclic product in Python integers
        ref = [0] * N
        for i in range(N):
            for j in range(N):
                k, v = i + j, int(a[i]) * int(b[j])
                if k >= N:
                    ref[k - N] -= v
                else:
                    ref[k] += v
        ref = np.array([x % q for x in ref], dtype=np.uint64)
        bufs = np.stack([a, b]).copy()
        pids = np.array([pid, pid], dtype=np.int32)
        e._check(oracle_lib.ntt_host(e._h, bufs.ctypes.data_as(C.POINTER(C.c_uint64)), 2,
                                     pids.ctypes.data_as(C.POINTER(C.c_int32)), 0))
        prod = np.array([(int(x) * int(y)) % q for x, y in zip(bufs[0], bufs[1])], dtype=np.uint64)
        prod = prod.reshape(1, N).copy()
        e._check(oracle_lib.ntt_host(e._h, prod.ctypes.data_as(C.POINTER(C.c_uint64)), 1,
                                     pids[:1].ctypes.data_as(C.POINTER(C.c_int32)), 1))
        np.testing.assert_array_equal(prod[0], ref)


@pytest.mark.parametrize("log_n", [6, 10])
def test_encode_is_canonical_embedding(oracle_lib, log_n):
    N, n = 1 << log_n, 1 << (log_n - 1)
    rng = np.random.default_rng(0)
    z = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    co = np.empty(N, np.int64)
    re_, im_ = np.ascontiguousarray(z.real), np.ascontiguousarray(z.imag)
    oracle_lib.check(oracle_lib.encode(log_n, re_.ctypes.data_as(C.POINTER(C.c_double)),
                                       im_.ctypes.data_as(C.POINTER(C.c_double)), n, 2.0 ** 30,
                                       co.ctypes.data_as(C.POINTER(C.c_int64))))
    M = 2 * N
    roots = np.exp(2j * np.pi * np.array([pow(5, j, M) for j in range(n)]) / M)
    vals = np.polyval(co[::-1].astype(np.float64), roots) / 2.0 ** 30
    np.testing.assert_allclose(vals, z, atol=1e-6)


def test_deterministic_keys_and_encryption(oracle_lib):
    outs = []
    for _ in range(2):
        e = Engine(_lib=oracle_lib, **KW)
        sk = e.create_secret_key(3)
        ct = e.encrypt(np.ones(4), e.create_public_key(sk))
        outs.append(e.export_residues(ct))
    np.testing.assert_array_equal(*outs)


def test_levels_and_scales(env):
    e, sk, pk, rlk, _ = env
    z = np.exp(-2j * np.pi * np.arange(e.slot_count) / 16)
    ct = e.encrypt(z, pk)
    pb = e.make_power_basis(ct, 8, rlk)
    assert [c.level for c in pb] == [6, 5, 4, 4, 3, 3, 3, 3]
    for k, c in enumerate(pb, 1):
        np.testing.assert_allclose(e.decrypt(c, sk), z ** k, atol=1e-6)
    lo = e.level_down(ct, 2)
    assert lo.level == 2
    np.testing.assert_allclose(e.decrypt(lo, sk), z, atol=1e-6)
    s = e.add(pb[7], ct)                                   # mixed levels align
    np.testing.assert_allclose(e.decrypt(s, sk), z ** 8 + z, atol=1e-6)
    np.testing.assert_allclose(e.decrypt(e.add(ct, 0.5 - 0.25j), sk), z + 0.5 - 0.25j, atol=1e-6)


def test_poly2_semantics(env):
    """aesfhe_poly2 = sum C[t,i,j] x^i y^j at level l-2 (include/aesfhe.h)."""
    e, sk, pk, rlk, _ = env
    rng = np.random.default_rng(9)
    zx = np.exp(-2j * np.pi * rng.integers(0, 16, e.slot_count) / 16)
    zy = np.exp(-2j * np.pi * rng.integers(0, 16, e.slot_count) / 16)
    xb = e.make_power_basis(e.encrypt(zx, pk), 3, rlk)
    yb = e.make_power_basis(e.encrypt(zy, pk), 3, rlk)
    C = rng.standard_normal((2, 4, 4)) + 1j * rng.standard_normal((2, 4, 4))
    outs = e.poly2(xb, yb, C, rlk)
    lv = min(c.level for c in xb + yb)
    for t in range(2):
        assert outs[t].level == lv - 2
        want = sum(C[t, i, j] * zx ** i * zy ** j for i in range(4) for j in range(4))
        np.testing.assert_allclose(e.decrypt(outs[t], sk), want, atol=1e-4)
    with pytest.raises(ValueError):
        e.poly2(xb[:2], yb, C, rlk)
    with pytest.raises(RuntimeError, match="at least one basis"):
        e._check(e._lib.poly2(e._h, None, 1, None, 1, None, None, 1, None, None))


def test_poly2_int_semantics(env):
    """aesfhe_poly2_int = sum (w/den) x^i y^j at level l-2, basis at mixed levels."""
    e, sk, pk, rlk, _ = env
    rng = np.random.default_rng(10)
    zx = np.exp(-2j * np.pi * rng.integers(0, 16, e.slot_count) / 16)
    zy = np.exp(-2j * np.pi * rng.integers(0, 16, e.slot_count) / 16)
    xb = e.make_power_basis(e.encrypt(zx, pk), 3, rlk)
    yb = e.make_power_basis(e.encrypt(zy, pk), 4, rlk)
    W = rng.integers(-8, 9, (3, 4, 5))
    W[1] = 0
    outs = e.poly2_int(xb, yb, W, 64, rlk)
    lv = min(c.level for c in xb + yb)
    for t in range(3):
        assert outs[t].level == lv - 2
        want = sum(W[t, i, j] / 64 * zx ** i * zy ** j for i in range(4) for j in range(5))
        np.testing.assert_allclose(e.decrypt(outs[t], sk), want, atol=1e-4)
    with pytest.raises(RuntimeError, match="exceeds 512"):
        e.poly2_int(xb, yb, np.full((1, 4, 5), 300), 64, rlk)


def test_dot_fma_semantics(env):
    """aesfhe_dot_fma = sum a_i b_i + sum gamma_j c_j + beta at level l - 1, products level-aligned,
    addends truncated (include/aesfhe.h); an addend below the products' level is refused."""
    e, sk, pk, rlk, _ = env
    rng = np.random.default_rng(12)
    z = [rng.uniform(-1, 1, e.slot_count) for _ in range(5)]
    a0, b0 = e.encrypt(z[0], pk, level=4), e.encrypt(z[1], pk, level=5)
    a1, b1 = e.encrypt(z[2], pk, level=6), e.encrypt(z[3], pk, level=4)
    c0 = e.encrypt(z[4], pk, level=6)
    out = e.dot_fma([a0, a1], [b0, b1], rlk, [(c0, -0.5), (a1, 2.0)], 0.25)
    assert out.level == 3
    want = z[0] * z[1] + z[2] * z[3] - 0.5 * z[4] + 2.0 * z[2] + 0.25
    np.testing.assert_allclose(e.decrypt(out, sk).real, want, atol=1e-5)
    only = e.dot_fma([a1], [a1], rlk)
    assert only.level == 5
    np.testing.assert_allclose(e.decrypt(only, sk).real, z[2] * z[2], atol=1e-5)
    with pytest.raises(RuntimeError, match="below the product level"):
        e.dot_fma([a1], [b0], rlk, [(a0, 1.0)])


def test_rotate_hoisted_oracle(oracle_lib):
    """Hoisted rotations (shared ModUp; DESIGN.md 3.16 / include/aesfhe.h) = np.roll, batched,
    and agree with the ordinary rotation up to key-switch noise."""
    e = Engine(log_n=10, max_level=6, special_primes=4, seed=3, _lib=oracle_lib)
    sk = e.create_secret_key(1)
    pk = e.create_public_key(sk)
    rng = np.random.default_rng(0)
    x = rng.uniform(-1, 1, (2, e.slot_count)) + 1j * rng.uniform(-1, 1, (2, e.slot_count))
    c = e.encrypt(x, pk, level=5)
    ds = (1, 5, -7, 100)
    outs = e.rotate_hoisted(c, [e.create_hoisted_rotation_key(sk, d) for d in ds])
    for d, o in zip(ds, outs):
        assert o.level == 5
        np.testing.assert_allclose(e.decrypt(o, sk), np.roll(x, d, axis=1), atol=1e-6)
        ref = e.rotate(c, e.create_fixed_rotation_key(sk, d))
        np.testing.assert_allclose(e.decrypt(o, sk), e.decrypt(ref, sk), atol=1e-6)
    with pytest.raises(RuntimeError):
        e.rotate_hoisted(c, [e.create_fixed_rotation_key(sk, 1)])


def test_mul_fma_and_mixed_level_lincomb_oracle(oracle_lib):
    """aesfhe_mul_fma = alpha a b + gamma c + beta (one relinearise + rescale, c truncated with
    its scale compensated) and lincomb over inputs at different levels (truncation, no
    level-down): values within CKKS noise of the plaintext formulas."""
    e = Engine(log_n=10, max_level=8, special_primes=4, seed=3, _lib=oracle_lib)
    sk = e.create_secret_key(1)
    pk = e.create_public_key(sk)
    rlk = e.create_relinearization_key(sk)
    rng = np.random.default_rng(0)
    x, y, z = [rng.uniform(-1, 1, (2, e.slot_count)) for _ in range(3)]
    a, b, c = (e.encrypt(x, pk, level=6), e.encrypt(y, pk, level=5), e.encrypt(z, pk, level=7))
    o = e.multiply_fma(a, b, rlk, alpha=2, c=c, gamma=-1.0, beta=-1.0)
    assert o.level == 4
    np.testing.assert_allclose(e.decrypt(o, sk), 2 * x * y - z - 1, atol=1e-6)
    o = e.multiply_fma(a, a, rlk, alpha=-3, beta=0.5)
    np.testing.assert_allclose(e.decrypt(o, sk), -3 * x * x + 0.5, atol=1e-6)
    with pytest.raises(RuntimeError):
        e.multiply_fma(a, a, rlk, c=b)  # addend below the product level
    li = e.lincomb([a, b, c], [0.5, -0.25j, 3.0])
    assert li.level == 4
    np.testing.assert_allclose(e.decrypt(li, sk), 0.5 * x - 0.25j * y + 3 * z, atol=1e-6)


def test_linear_bsgs_oracle(oracle_lib):
    """aesfhe_linear_bsgs (include/aesfhe.h): slots equal the plain baby-step giant-step sum,
    batch and identity steps included; one level used; a giant with two terms on one baby is an
    argument error (the HIP engine's single-pass term kernel relies on it)."""
    e = Engine(log_n=11, max_level=5, special_primes=2, seed=9, _lib=oracle_lib)
    n = e.slot_count
    rng = np.random.default_rng(8)
    sk = e.create_secret_key(2)
    z = rng.uniform(-1, 1, (3, n))
    c = e.encrypt(z, e.create_public_key(sk), level=4)
    diags = [rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n) for _ in range(4)]
    babies, plan = [0, 2, -7], [(0, [(1, 0), (2, 1)]), (5, [(0, 2), (1, 3), (2, 0)])]
    bk = [None if d == 0 else e.create_hoisted_rotation_key(sk, -d) for d in babies]
    gk = [None if d == 0 else e.create_fixed_rotation_key(sk, -d) for d, _ in plan]
    pts = [e.encode(v) for v in diags]
    out = e.linear_bsgs(c, bk, gk, [[(b, pts[i]) for b, i in tl] for _, tl in plan])
    want = sum(np.roll(sum(diags[i] * np.roll(z, -babies[b], axis=1) for b, i in tl), -d, axis=1)
               for d, tl in plan)
    assert out.level == 3 and out.batch == 3
    np.testing.assert_allclose(e.decrypt(out, sk), want, atol=1e-6)
    with pytest.raises(RuntimeError, match="same baby"):
        e.linear_bsgs(c, bk, gk[:1], [[(1, pts[0]), (1, pts[1])]])


def test_digit_width_oracle(oracle_lib):
    """Key-switch digits wider than K (aesfhe_params.digit_primes): at L = 30 with K = 10 special
    primes, 12-prime digits give dnum 3 instead of 4 (no one-limb digit at the top level) with the
    same precision through products and rotations; a digit whose product exceeds P is refused."""
    from aes_xor_fhe.fhe import Engine
    errs = {}
    for a in (0, 12):
        e = Engine(log_n=10, max_level=30, special_primes=10, scale_bits=40, digit_primes=a, seed=3,
                   _lib=oracle_lib)
        assert (e.dnum, e.digit_primes) == ((4, 10) if a == 0 else (3, 12))
        sk = e.create_secret_key(1)
        pk, rlk, rot = e.create_public_key(sk), e.create_relinearization_key(sk), e.create_rotation_key(sk)
        v = np.random.default_rng(0).uniform(-1, 1, e.slot_count)
        ct = e.encrypt(v, pk)
        x, ref, err = ct, v.copy(), []
        for _ in range(4):
            x, ref = e.multiply(x, ct, rlk), ref * v
            err.append(np.abs(np.real(e.decrypt(x, sk)) - ref).max())
        err.append(np.abs(np.real(e.decrypt(e.rotate(x, rot, 3), sk)) - np.roll(ref, 3)).max())
        errs[a] = np.array(err)
        assert errs[a].max() < 1e-7
        if a:
            assert e.key_fingerprint() != Engine(log_n=10, max_level=30, special_primes=10, scale_bits=40,
                                                 seed=3, _lib=oracle_lib).key_fingerprint()
    assert np.all(errs[12] < 2 * errs[0] + 1e-9)
    with pytest.raises(RuntimeError, match="exceeds P"):
        Engine(log_n=10, max_level=30, special_primes=10, scale_bits=40, digit_primes=16, seed=3, _lib=oracle_lib)


def test_cyclic_broadcast_mul_oracle(oracle_lib):
    """aesfhe_mul cycles through a smaller power-of-two batch (element i takes i mod B_small)."""
    from aes_xor_fhe.fhe import Engine
    e = Engine(log_n=10, max_level=4, special_primes=2, seed=5, _lib=oracle_lib)
    sk = e.create_secret_key(1)
    pk, rlk = e.create_public_key(sk), e.create_relinearization_key(sk)
    rng = np.random.default_rng(2)
    z8, z4 = rng.uniform(-1, 1, (8, e.slot_count)), rng.uniform(-1, 1, (4, e.slot_count))
    out = e.multiply(e.encrypt(z8, pk), e.encrypt(z4, pk), rlk)
    assert out.batch == 8
    np.testing.assert_allclose(np.real(e.decrypt(out, sk)), z8 * z4[np.arange(8) % 4], atol=1e-6)
    with pytest.raises(RuntimeError, match="batch mismatch"):
        e.multiply(e.encrypt(z8[:6], pk), e.encrypt(z4[:3], pk), rlk)
