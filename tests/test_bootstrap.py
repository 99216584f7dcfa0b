"""CKKS bootstrapping (aes_xor_fhe.bootstrap; Engine.bootstrap, called by the reference at
xor_service.py:120-129,274-277 and mixcolumns_service.py:72-75).

desilofhe's bootstrap is closed and absent, so parity is unpinned against the reference's engine:
these tests check the algorithm's own invariants -- the butterfly factorisation of the encoding
map against the codec's V, the key-switch rounding noise of the exact ModDown, decrypt(boot(ct))
~ decrypt(ct) within the precision DESIGN.md section 7 states, the quadratic error squash of the
bit mode -- on the CPU oracle, and residue-identical outputs of the HIP engine (integer work,
bit-exact) plus the precision at BASELINE's N = 2^16, L = 30 on the GPU."""
import math

import numpy as np
import pytest

from aes_xor_fhe.bootstrap import Bootstrapper, apply_diag, transform_groups
from aes_xor_fhe.fhe import Engine


def _brv(n):
    L = int(math.log2(n))
    return np.array([int(format(i, f"0{L}b")[::-1], 2) for i in range(n)])


@pytest.mark.parametrize("log_n,groups", [(6, 1), (8, 3), (10, 3), (10, 4)])
def test_transform_factorisation(log_n, groups):
    N = 1 << log_n
    n, M = N // 2, 2 * N
    xi = np.exp(2j * np.pi / M)
    rot = np.array([pow(5, j, M) for j in range(n)])
    V = xi ** (np.outer(rot, np.arange(n)) % M)  # z = V u / scale (the codec, fhe.decode)
    u = np.random.default_rng(0).standard_normal(n) + 1j
    x = u[_brv(n)]
    for Mx in transform_groups(n, N, groups, False):
        x = apply_diag(Mx, x)
    np.testing.assert_allclose(x, V @ u, atol=1e-9)
    y = V @ u
    for Mx in transform_groups(n, N, groups, True):
        y = apply_diag(Mx, y)
    np.testing.assert_allclose(y, u[_brv(n)], atol=1e-9)


def _engine(lib, log_n=10, scale_bits=44, max_level=24, **kw):
    kw = dict(dict(special_primes=4), **kw)
    e = Engine(log_n=log_n, max_level=max_level, scale_bits=scale_bits, seed=3, _lib=lib, **kw)
    sk = e.create_secret_key(1)
    return e, sk, e.create_public_key(sk), e.create_relinearization_key(sk)


def test_keyswitch_rounding_noise(oracle_lib):
    """Exact ModDown: the added noise is eps * s_to with |eps| <= 1/2 (std sqrt(h/12))."""
    e, sk, pk, _ = _engine(oracle_lib)
    n = e.slot_count
    x = np.random.default_rng(2).uniform(-1, 1, n) * 1e-2
    for s_to, h in ((e.create_secret_key(9), 2 * e.slot_count * 2 / 3),
                    (e.create_sparse_secret_key(32, 4), 32)):
        swk = e.create_switching_key(sk, s_to)
        c = e.encrypt(x, pk, level=10)
        e0 = e.decrypt(c, sk) - x
        add = (e.decrypt(e.switch_key(c, swk), s_to) - x) - e0
        co = e._encode_coeffs(add, e.scales[10]).astype(float)
        assert co.std() < 1.5 * math.sqrt(h / 12) + 1, (h, co.std())


def test_bootstrap_general_oracle(oracle_lib):
    e, sk, pk, rlk = _engine(oracle_lib)
    bk = e.create_bootstrap_key(sk)
    cjk = e.create_conjugation_key(sk)
    n = e.slot_count
    rng = np.random.default_rng(1)
    z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
    ct = e.encrypt(z, pk, level=2)
    out = e.bootstrap(ct, rlk, cjk, bk)
    bs = bk.bootstrapper(rlk, cjk)
    assert out.level == e.max_level - bs.depth
    assert np.abs(e.decrypt(out, sk) - z).max() < 1e-3


@pytest.mark.parametrize("opt", [True, False], ids=["bits_opt", "round2_path"])
def test_bootstrap_bits_oracle(oracle_lib, opt):
    """Bit mode: depth 11 with bits_opt (c_in in CtS, depth-optimal degree-15 EvalMod), 13 on the
    round-2 path; both square the input error."""
    e, sk, pk, rlk = _engine(oracle_lib)
    bs = Bootstrapper(e, sk, rlk, bits_opt=opt)
    n = e.slot_count
    rng = np.random.default_rng(4)
    a, b = rng.choice([-1.0, 1.0], n), rng.choice([-1.0, 1.0], n)
    noise = 0.03 * rng.standard_normal((2, n))
    ya, yb = bs.bootstrap_bits(e.encrypt(a + noise[0], pk, level=6),
                               e.encrypt(b + noise[1], pk, level=4))
    assert ya.level == yb.level == bs.bits_level == e.max_level - (11 if opt else 13)
    # the input error enters squared: 1 - cos(2 pi e / 4) <= 1.24 e^2
    for y, v, nz in ((ya, a, noise[0]), (yb, b, noise[1])):
        err = np.abs(e.decrypt(y, sk) - v)
        assert np.all(err <= 1.24 * nz ** 2 + 1e-5)
    # one ciphertext alone, constant slots (all coefficients but one zero)
    y1, none = bs.bootstrap_bits(e.encrypt(np.ones(n), pk, level=3))
    assert none is None and np.abs(e.decrypt(y1, sk) - 1).max() < 1e-5
    with pytest.raises(ValueError):
        bs.bootstrap_bits(e.encrypt(a, pk, level=2))


def test_bootstrapper_share(oracle_lib):
    """Bootstrapper(share=...): a 3-map CoeffToSlot bootstrapper built beside a 5-map one reuses
    its conjugation and sparse-secret keys, every rotation key of a common rotation and the
    SlotToCoeff plans (the bench's and the AES drivers' pair), creates only the keys it alone
    needs, and still squares the input error of the bit mode."""
    e, sk, pk, rlk = _engine(oracle_lib, max_level=30, scale_bits=40)
    b5 = Bootstrapper(e, sk, rlk, cts_groups=5)
    b3 = Bootstrapper(e, sk, rlk, cts_groups=3, share=b5)
    assert b3.cjk is b5.cjk and b3.to_sparse is b5.to_sparse and b3.from_sparse is b5.from_sparse
    assert b3.stc_bits is b5.stc_bits and b3.stc is b5.stc
    common = set(b3.hrot) & set(b5.hrot)
    assert common and all(b3.hrot[d] is b5.hrot[d] for d in common)
    assert all(b3.rot[d] is b5.rot[d] for d in set(b3.rot) & set(b5.rot))
    with pytest.raises(ValueError):
        e2, sk2, _, rlk2 = _engine(oracle_lib)
        Bootstrapper(e2, sk2, rlk2, share=b5)
    n = e.slot_count
    rng = np.random.default_rng(6)
    a, b = rng.choice([-1.0, 1.0], n), rng.choice([-1.0, 1.0], n)
    noise = 0.03 * rng.standard_normal((2, n))
    ya, yb = b3.bootstrap_bits(e.encrypt(a + noise[0], pk, level=3), e.encrypt(b + noise[1], pk, level=3))
    for y, v, nz in ((ya, a, noise[0]), (yb, b, noise[1])):
        assert np.all(np.abs(e.decrypt(y, sk) - v) <= 1.24 * nz ** 2 + 1e-5)
    # a share under another secret key, or one whose keys were trimmed, is refused
    # before any key is made (a trimmed CoeffToSlot key would fail mid-bootstrap)
    with pytest.raises(ValueError, match="same secret key"):
        Bootstrapper(e, e.create_secret_key(seed=99), rlk, share=b5)
    from aes_xor_fhe.bootstrap import trim_bootstrap_keys
    trim_bootstrap_keys([b5, b3])
    with pytest.raises(ValueError, match="trimmed"):
        Bootstrapper(e, sk, rlk, cts_groups=4, share=b5)


def test_trim_bootstrap_keys_residue_identical(oracle_lib):
    """trim_bootstrap_keys on a 5-map CoeffToSlot bootstrapper alone (config 5's): the
    SlotToCoeff-only rotation keys keep one digit of the three (L = 30, 12-prime digits);
    bootstrap_bits then returns residue for residue what the untrimmed keys give (same engine seed,
    same keys), the freed bytes are reported, general bootstrapping refuses, and a trimmed key
    holds a third of a whole key's bytes.  (Beside a 3-map bootstrapper nothing is freed: its
    CoeffToSlot uses the same rotations at the top levels.)"""
    from aes_xor_fhe.bootstrap import trim_bootstrap_keys
    outs = []
    for trim in (False, True):
        e, sk, pk, rlk = _engine(oracle_lib, max_level=30, scale_bits=40, special_primes=10, digit_primes=12)
        b5 = Bootstrapper(e, sk, rlk, cts_groups=5)
        stc_only = set()
        if trim:
            assert trim_bootstrap_keys([b5]) > 0
            stc_only = {id(k) for p in b5.stc_bits for k in b5.plan_keys(p)} - \
                       {id(k) for p in b5.cts + b5.cts_bits for k in b5.plan_keys(p)}
            k = next(k for p in b5.stc_bits for k in b5.plan_keys(p) if id(k) in stc_only)
            assert e.key_bytes(k) * 3 == e.key_bytes(b5.from_sparse)
        rng = np.random.default_rng(8)
        a, b = rng.choice([-1.0, 1.0], e.slot_count), rng.choice([-1.0, 1.0], e.slot_count)
        ya, yb = b5.bootstrap_bits(e.encrypt(a, pk, level=5), e.encrypt(b, pk, level=5))
        outs.append([e.export_residues(y) for y in (ya, yb)])
        if trim:  # (after the encryptions above: this one draws encryption randomness too)
            with pytest.raises(RuntimeError, match="trimmed"):
                b5.bootstrap(e.encrypt(np.zeros(e.slot_count), pk, level=0))
            # the trimmed key itself, switched above its level: the oracle returns AESFHE_ELEVEL
            # as the HIP engine does (it used to abort() the process)
            top = e.encrypt(np.zeros(e.slot_count), pk, level=30)
            kh = next(h for h in b5.hrot.values() if id(h) in stc_only)
            with pytest.raises(RuntimeError, match="trimmed to 1 digits"):
                e.rotate_hoisted(top, [kh])
    for h, o in zip(*outs):
        assert np.array_equal(h, o)


@pytest.mark.parametrize("deg", [3, 7, 15, 29])
def test_chebyshev_opt_depth_and_values(oracle_lib, deg):
    """chebyshev_opt (bootstrap.py): a random Chebyshev series of degree deg lands exactly
    ceil(log2(deg + 1)) levels down -- never deeper than the recursive `chebyshev`, one level
    shallower at degrees 7 and 15 -- and decrypts to numpy's chebval of the slots; both evaluators
    agree."""
    e, sk, pk, rlk = _engine(oracle_lib, max_level=12)
    bs = Bootstrapper(e, sk, rlk, groups=1)
    rng = np.random.default_rng(deg)
    c = rng.uniform(-1, 1, deg + 1) / (1 + np.arange(deg + 1))
    x = rng.uniform(-1, 1, e.slot_count)
    ct = e.encrypt(x, pk, level=10)
    y = bs.chebyshev_opt(ct, c)
    assert y.level == 10 - math.ceil(math.log2(deg + 1))
    want = np.polynomial.chebyshev.chebval(x, c)
    assert np.abs(e.decrypt(y, sk).real - want).max() < 1e-6
    if deg >= 7:
        z = bs.chebyshev(ct, c)
        assert z.level == (y.level - 1 if deg in (7, 15) else y.level)
        assert np.abs(e.decrypt(z, sk).real - want).max() < 1e-6


def test_bits_fit_error_at_the_evaluated_points():
    """_bits_fit: degree 15 with 4 double angles matches sin(2 pi t / q0) to 1e-6 wherever the bit
    mode evaluates it (t / q0 = I +- 1/4 + d, |I| <= K, |d| <= 1e-2), where the plain Chebyshev
    interpolant of rounds 1-2 was off by 5.4e-5 (at I = 0, +1/4)."""
    B, K, r = 13.0, 12.0, 4
    c = Bootstrapper._bits_fit(15, r, B, K)
    cheb = Bootstrapper._cheb_fit(15, r, B)
    I = np.arange(-int(K), int(K) + 1)
    pts = np.concatenate([(i + s + np.linspace(-1e-2, 1e-2, 41)) / B for i in I for s in (0.25, -0.25)])

    def post(cc):
        g = np.polynomial.chebyshev.chebval(pts, cc)
        for _ in range(r):
            g = 2 * g * g - 1
        return g
    ideal = np.cos(2 * np.pi * (B * pts - 0.25))  # = sin(2 pi B x)
    assert np.abs(post(c) - ideal).max() < 1e-6
    assert np.abs(post(cheb) - ideal).max() > 4e-5


def test_refresh_schedule():
    """AESRowRound.needs_refresh: ten rounds on three refreshes at L = 30 (bootstrap output 19)
    and at config 5's L = 35 (output 24); at most 2 middle rounds after a refresh."""
    from aes_xor_fhe.aes_round_bits import AESRowRound
    R = AESRowRound.__new__(AESRowRound)
    for L, out in ((30, 19), (35, 24)):
        lvl, since, nref, plan = L - 1, 0, 0, []
        for rnd in range(1, 11):
            final = rnd == 10
            if R.needs_refresh(lvl, final, since, nref > 0, 3):
                lvl, since, nref = out, 0, nref + 1
                plan.append("R")
            lvl -= R.FINAL_DEPTH if final else R.ROUND_DEPTH
            assert lvl >= 0
            since += 1
            plan.append(str(rnd))
        assert nref == 3, (L, plan)
        segs = "".join(plan).split("R")
        assert all(len([ch for ch in seg if ch != "0"]) <= 3 for seg in segs)


def test_pick_bootstrapper():
    """Per-refresh choice among bootstrappers (AESRowRound.pick_bootstrapper): at L = 30 the
    5-map CtS (output 17) serves the refresh before round 4 (two middle rounds + StC = 17 levels),
    the 3-map one (output 19) the refresh before round 6 -- two levels more, so the bits can be
    cleaned (CLEAN_LEVELS) before the last refresh -- and the one before rounds 8-10 (7 + 7 + 5);
    at L = 35 the cheaper one serves all three and leaves room to clean as well."""
    from types import SimpleNamespace as NS
    from aes_xor_fhe.aes_round_bits import AESRowRound
    R = AESRowRound.__new__(AESRowRound)
    for L, want in ((30, [17, 19, 19]), (35, [22, 22, 22])):
        bss = [NS(bits_level=L - 13, stc_bits=[0] * 3), NS(bits_level=L - 11, stc_bits=[0] * 3)]
        lvl, since, got, cleans = L - 1, 0, [], []
        for rnd in range(1, 11):
            final = rnd == 10
            if R.needs_refresh(lvl, final, since, bool(got), 3):
                b = R.pick_bootstrapper(bss, rnd)
                last = R.refreshes_after(rnd, b.bits_level, L - 11, 3) == 0
                cleans.append(last and R.can_clean(lvl, since, bool(got), 3))
                got.append(b.bits_level)
                lvl, since = b.bits_level, 0
            lvl -= R.FINAL_DEPTH if final else R.ROUND_DEPTH
            assert lvl >= 0
            since += 1
        assert got == want, (L, got)
        assert cleans == [False, False, True], (L, cleans)  # the last refresh's input is cleaned
    # a single bootstrapper is always taken
    assert R.pick_bootstrapper(bss[1:], 8) is bss[1]


BENCH_CHAIN = dict(scale_bits=40, max_level=30, special_primes=10, digit_primes=12)


@pytest.mark.gpu
@pytest.mark.parametrize("kw,groups", [({}, None), (BENCH_CHAIN, None), (BENCH_CHAIN, 5)],
                         ids=["K4", "K10A12", "K10A12G5"])
def test_bootstrap_bits_bit_exact_vs_oracle(product_lib, oracle_lib, gpu_available, kw, groups):
    """Bit-mode and general bootstrapping residue for residue; K10A12: the bench's chain (L = 30,
    K = 10 special primes, 12-prime key-switch digits) at N = 2^10; G5: the 5-map CoeffToSlot
    bootstrapper the bench's ten-round leg uses for its two middle refreshes (the 3-map one is
    the default of the other two cases)."""
    outs = []
    for lib in (product_lib, oracle_lib):
        e, sk, pk, rlk = _engine(lib, **kw)
        bs = Bootstrapper(e, sk, rlk, cts_groups=groups)
        if groups is not None:
            assert bs.cts_groups == groups and bs.bits_level == e.max_level - 13
        rng = np.random.default_rng(4)
        n = e.slot_count
        a, b = rng.choice([-1.0, 1.0], n), rng.choice([-1.0, 1.0], n)
        ya, yb = bs.bootstrap_bits(e.encrypt(a, pk, level=3), e.encrypt(b, pk, level=3))
        g = e.bootstrap(e.encrypt(a + 0.5j * b, pk, level=0), rlk, bs.cjk,
                        _key_for(e, sk, bs))
        outs.append([e.export_residues(c) for c in (ya, yb, g)])
    for h, o in zip(*outs):
        assert np.array_equal(h, o)


@pytest.mark.gpu
def test_trimmed_keys_bit_exact_vs_oracle(product_lib, oracle_lib, gpu_available):
    """Config 5's refresh path with the SlotToCoeff-only keys trimmed (trim_bootstrap_keys,
    aesfhe_key_trim: device copy of the first digit, the old block back to the arena): HIP and
    oracle residue for residue at the bench's chain, N = 2^10."""
    from aes_xor_fhe.bootstrap import trim_bootstrap_keys
    outs = []
    for lib in (product_lib, oracle_lib):
        e, sk, pk, rlk = _engine(lib, **BENCH_CHAIN)
        bs = Bootstrapper(e, sk, rlk, cts_groups=5)
        assert trim_bootstrap_keys([bs]) > 0
        rng = np.random.default_rng(9)
        a, b = rng.choice([-1.0, 1.0], e.slot_count), rng.choice([-1.0, 1.0], e.slot_count)
        ya, yb = bs.bootstrap_bits(e.encrypt(a, pk, level=4), e.encrypt(b, pk, level=4))
        outs.append([e.export_residues(c) for c in (ya, yb)])
        assert np.abs(e.decrypt(ya, sk) - a).max() < 1e-2
    for h, o in zip(*outs):
        assert np.array_equal(h, o)


def _key_for(e, sk, bs):
    k = e.create_bootstrap_key(sk)
    k._bs = bs
    return k


@pytest.mark.gpu
def test_bootstrap_bits_full_params(product_lib, gpu_available):
    """BASELINE's N = 2^16, L = 30 (44-bit scale, log QP = 1770 <= 1772)."""
    e = Engine(log_n=16, max_level=30, special_primes=8, scale_bits=44, seed=3, _lib=product_lib)
    sk = e.create_secret_key(1)
    pk = e.create_public_key(sk)
    bs = Bootstrapper(e, sk, e.create_relinearization_key(sk))
    n = e.slot_count
    rng = np.random.default_rng(5)
    a, b = rng.choice([-1.0, 1.0], n), rng.choice([-1.0, 1.0], n)
    ya, yb = bs.bootstrap_bits(e.encrypt(a, pk, level=3), e.encrypt(b, pk, level=3))
    assert ya.level == 19  # L - 11: c_in folded into CtS, depth-5 Chebyshev sum
    assert np.abs(e.decrypt(ya, sk) - a).max() < 1e-3
    assert np.abs(e.decrypt(yb, sk) - b).max() < 1e-3


@pytest.mark.gpu
def test_bootstrap_general_default_params_decodes_zeta256(product_lib, gpu_available):
    """The reference's Engine.bootstrap (xor_service.py:120-129) at the default engine
    parameters (N = 2^16, L = 30, K = 8, 44-bit scale -- fhe.DEFAULT_PARAMS): zeta-256 bytes come
    back within their decision margin sin(pi / 256) = 0.0123 (measured max error ~4.7e-3; at a
    40-bit scale it was 1.16, which is why the default is 44)."""
    from aes_xor_fhe.utils import zeta_decode
    e = Engine(seed=3, _lib=product_lib)
    assert (e.log_coeff_count, e.max_level, e.special_prime_count) == (16, 30, 8)
    sk = e.create_secret_key()
    pk, rlk, cjk = e.create_public_key(sk), e.create_relinearization_key(sk), e.create_conjugation_key(sk)
    bk = e.create_bootstrap_key(sk)
    x = np.random.default_rng(8).integers(0, 256, e.slot_count)
    z = np.exp(-2j * np.pi * x / 256)
    out = e.bootstrap(e.encrypt(z, pk, level=0), rlk, cjk, bk)
    got = e.decrypt(out, sk)
    err = np.abs(got - z).max()
    assert err < np.sin(np.pi / 256), err
    assert np.array_equal(zeta_decode(got, modulus=256), x.astype(np.uint8))
    assert out.level == e.max_level - bk.bootstrapper(rlk, cjk).depth
