"""GPU parity: the HIP engine (libaesfhe.so) against the CPU oracle, residue for residue.

Both implement include/aesfhe.h; the oracle restates the CKKS algorithm desilofhe performs for
the reference (see oracle/ckks_oracle.c header).  Every comparison here is bit-exact on the
NTT-domain residues (integer work), after identical seeded key generation and encryption.
"""
import numpy as np
import pytest

from aes_xor_fhe.fhe import Engine

pytestmark = pytest.mark.gpu

SMALL = dict(log_n=12, max_level=6, special_primes=2, seed=1234)
# key-switch digits wider than K (aesfhe_params.digit_primes): the bench's chain, alpha = 12 over
# K = 10 special primes (dnum 3 at every level from 24 to 30; the digit product stays below P)
DIGITS12 = dict(log_n=12, max_level=30, special_primes=10, digit_primes=12, scale_bits=40, seed=77)


def _pair(product_lib, oracle_lib, **kw):
    g = Engine(_lib=product_lib, **kw)
    o = Engine(_lib=oracle_lib, **kw)
    assert g.primes == o.primes
    assert g.scales == o.scales
    return g, o


def _keys(eng):
    sk = eng.create_secret_key(7)
    return dict(sk=sk, pk=eng.create_public_key(sk), rlk=eng.create_relinearization_key(sk),
                cjk=eng.create_conjugation_key(sk), rot=eng.create_rotation_key(sk))


def _same(g, o, cg, co):
    assert (cg.level, cg.batch, cg.npoly) == (co.level, co.batch, co.npoly)
    a, b = g.export_residues(cg), o.export_residues(co)
    if not np.array_equal(a, b):
        bad = np.argwhere(a != b)
        raise AssertionError(f"{len(bad)} residues differ; first at {bad[0].tolist()}")


@pytest.mark.parametrize("log_n,extreme", [(10, False), (12, False), (14, False), (16, False),
                                           (16, True), (17, True)])
def test_ntt_bit_exact(product_lib, oracle_lib, gpu_available, log_n, extreme):
    kw = dict(log_n=log_n, max_level=4, special_primes=2, seed=1)
    g, o = _pair(product_lib, oracle_lib, **kw)
    import ctypes as C
    n = 1 << log_n
    npr = len(g.primes)
    rng = np.random.default_rng(log_n)
    limbs = np.stack([rng.integers(0, q, n, dtype=np.uint64) for q in g.primes])
    if extreme:  # the range bounds of the lazy butterflies: runs of q - 1 and 0
        for r, q in enumerate(g.primes):
            limbs[r, : n // 2] = q - 1
            limbs[r, n // 2 :: 3] = 0
    pids = np.arange(npr, dtype=np.int32)
    for inverse in (0, 1):
        out = []
        for eng in (g, o):
            buf = limbs.copy()
            eng._check(eng._lib.ntt_host(eng._h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), npr,
                                         pids.ctypes.data_as(C.POINTER(C.c_int32)), inverse))
            out.append(buf)
        np.testing.assert_array_equal(out[0], out[1])


def test_keygen_encrypt_bit_exact(product_lib, oracle_lib, gpu_available):
    g, o = _pair(product_lib, oracle_lib, **SMALL)
    kg, ko = _keys(g), _keys(o)
    rng = np.random.default_rng(0)
    v = np.exp(-2j * np.pi * rng.integers(0, 16, g.slot_count) / 16)
    cg, co = g.encrypt(v, kg["pk"]), o.encrypt(v, ko["pk"])
    _same(g, o, cg, co)
    np.testing.assert_allclose(g.decrypt(cg, kg["sk"]), v, atol=1e-6)
    # symmetric encryption and batches
    vb = np.stack([v, np.roll(v, 3)])
    _same(g, o, g.encrypt(vb, kg["sk"]), o.encrypt(vb, ko["sk"]))


def test_ops_bit_exact(product_lib, oracle_lib, gpu_available):
    g, o = _pair(product_lib, oracle_lib, **SMALL)
    kg, ko = _keys(g), _keys(o)
    rng = np.random.default_rng(1)
    z = np.exp(-2j * np.pi * rng.integers(0, 16, g.slot_count) / 16)
    w = np.exp(-2j * np.pi * rng.integers(0, 16, g.slot_count) / 16)
    cg, co = g.encrypt(z, kg["pk"]), o.encrypt(z, ko["pk"])
    dg, do = g.encrypt(w, kg["pk"]), o.encrypt(w, ko["pk"])
    _same(g, o, g.multiply(cg, dg, kg["rlk"]), o.multiply(co, do, ko["rlk"]))
    _same(g, o, g.add(cg, dg), o.add(co, do))
    _same(g, o, g.subtract(cg, dg), o.subtract(co, do))
    _same(g, o, g.multiply(cg, 0.25 - 0.5j), o.multiply(co, 0.25 - 0.5j))
    mask = (np.arange(g.slot_count) % 4 == 1).astype(float)
    _same(g, o, g.multiply(cg, g.encode(mask)), o.multiply(co, o.encode(mask)))
    _same(g, o, g.add(cg, g.encode(mask)), o.add(co, o.encode(mask)))
    _same(g, o, g.conjugate(cg, kg["cjk"]), o.conjugate(co, ko["cjk"]))
    for k in (1, -4, 5, 1000):
        _same(g, o, g.rotate(cg, kg["rot"], k), o.rotate(co, ko["rot"], k))
    _same(g, o, g.level_down(cg, 3), o.level_down(co, 3))
    pg = g.make_power_basis(cg, 8, kg["rlk"])
    po = o.make_power_basis(co, 8, ko["rlk"])
    for a, b in zip(pg, po):
        _same(g, o, a, b)
    coeffs = [0.5, 0.25j, -1.0, 2.0 + 1j]
    _same(g, o, g.lincomb(pg[:4], coeffs), o.lincomb(po[:4], coeffs))
    M = np.array([coeffs, [0, 0, 0, 0], [1j, -0.5, 0.125, 0.3 - 0.7j]])
    for a, b in zip(g.lincomb_many(pg[:4], M), o.lincomb_many(po[:4], M)):
        _same(g, o, a, b)
    _same(g, o, g.dot(pg[:3], pg[1:4], kg["rlk"]), o.dot(po[:3], po[1:4], ko["rlk"]))
    # mixed levels: add aligns by exact-scale level-down
    _same(g, o, g.add(pg[7], cg), o.add(po[7], co))
    # 3-polynomial path and the reference's relinearize error string
    t3g, t3o = g.multiply(cg, dg), o.multiply(co, do)
    _same(g, o, t3g, t3o)
    _same(g, o, g.relinearize(t3g, kg["rlk"]), o.relinearize(t3o, ko["rlk"]))
    with pytest.raises(RuntimeError, match="should have 3 polynomials"):
        g.relinearize(cg, kg["rlk"])


def test_batched_ops_bit_exact(product_lib, oracle_lib, gpu_available):
    g, o = _pair(product_lib, oracle_lib, **SMALL)
    kg, ko = _keys(g), _keys(o)
    rng = np.random.default_rng(2)
    zb = np.exp(-2j * np.pi * rng.integers(0, 16, (3, g.slot_count)) / 16)
    cg, co = g.encrypt(zb, kg["pk"]), o.encrypt(zb, ko["pk"])
    kgc, koc = g.encrypt(zb[0], kg["pk"]), o.encrypt(zb[0], ko["pk"])  # broadcast operand
    _same(g, o, g.multiply(cg, kgc, kg["rlk"]), o.multiply(co, koc, ko["rlk"]))
    _same(g, o, g.rotate(cg, kg["rot"], -3), o.rotate(co, ko["rot"], -3))
    _same(g, o, g.conjugate(cg, kg["cjk"]), o.conjugate(co, ko["cjk"]))
    dec = g.decrypt(g.multiply(cg, kgc, kg["rlk"]), kg["sk"])
    np.testing.assert_allclose(dec, zb * zb[0], atol=1e-5)


@pytest.mark.parametrize("k,a", [(8, 0), (10, 0), (10, 12)], ids=["K8", "K10", "K10A12"])
def test_full_params_mul_bit_exact(product_lib, oracle_lib, gpu_available, k, a):
    """BASELINE.json's parameter set: N = 2^16, L = 30 (one ct x ct multiply + rotation), with
    K = 8 (dnum 4), K = 10 (alpha 10: dnum 4 at level 30, a one-limb digit) and the bench's
    K = 10 with 12-prime digits (dnum 3)."""
    kw = dict(log_n=16, max_level=30, special_primes=k, digit_primes=a, seed=99)
    if a:
        kw["scale_bits"] = 40  # the bench's chain (12 x 40-bit digits below P = 10 x 50 bits)
    g, o = _pair(product_lib, oracle_lib, **kw)
    kg, ko = _keys(g), _keys(o)
    rng = np.random.default_rng(3)
    z = np.exp(-2j * np.pi * rng.integers(0, 256, g.slot_count) / 256)
    cg, co = g.encrypt(z, kg["pk"]), o.encrypt(z, ko["pk"])
    mg, mo = g.multiply(cg, cg, kg["rlk"]), o.multiply(co, co, ko["rlk"])
    _same(g, o, mg, mo)
    np.testing.assert_allclose(g.decrypt(mg, kg["sk"]), z * z, atol=1e-5)
    _same(g, o, g.rotate(mg, kg["rot"], -2048), o.rotate(mo, ko["rot"], -2048))


def test_poly2_bit_exact(product_lib, oracle_lib, gpu_available):
    """Fused bivariate evaluation: m = 10 outputs (two kernel chunks), one all-zero output,
    nx != ny, a broadcast (B = 1) basis element, constant row/column terms."""
    g, o = _pair(product_lib, oracle_lib, **SMALL)
    kg, ko = _keys(g), _keys(o)
    rng = np.random.default_rng(7)
    zx = np.exp(-2j * np.pi * rng.integers(0, 16, (2, g.slot_count)) / 16)
    zy = np.exp(-2j * np.pi * rng.integers(0, 16, g.slot_count) / 16)
    C = (rng.standard_normal((10, 4, 3)) + 1j * rng.standard_normal((10, 4, 3))) * 0.2
    C[3] = 0
    res = []
    for eng, k in ((g, kg), (o, ko)):
        xb = eng.make_power_basis(eng.encrypt(zx, k["pk"]), 3, k["rlk"])
        yb = eng.make_power_basis(eng.encrypt(zy, k["pk"]), 2, k["rlk"])
        res.append(eng.poly2(xb, yb, C, k["rlk"]))
    for a, b in zip(*res):
        _same(g, o, a, b)
    dec = g.decrypt(res[0][0], kg["sk"])
    want = sum(C[0, i, j] * zx ** i * zy ** j for i in range(4) for j in range(3))
    np.testing.assert_allclose(dec, want, atol=1e-4)


@pytest.mark.parametrize("scale_bits", [40, 44])
def test_poly2_int_bit_exact(product_lib, oracle_lib, gpu_available, scale_bits):
    """Integer-weight bivariate evaluation: 6 outputs (two chunks), a zero output, mixed basis
    levels (power bases), a broadcast basis element, negative weights.  Scale 44 (config 5's
    chain): the 44-bit limbs take the exact-FMA kernel chosen from the weight bound, q_0 the
    folding one."""
    g, o = _pair(product_lib, oracle_lib, **dict(SMALL, scale_bits=scale_bits))
    kg, ko = _keys(g), _keys(o)
    rng = np.random.default_rng(8)
    zx = np.exp(-2j * np.pi * rng.integers(0, 16, (2, g.slot_count)) / 16)
    zy = np.exp(-2j * np.pi * rng.integers(0, 16, g.slot_count) / 16)
    W = rng.integers(-8, 9, (6, 4, 5))
    W[2] = 0
    res = []
    for eng, k in ((g, kg), (o, ko)):
        xb = eng.make_power_basis(eng.encrypt(zx, k["pk"]), 3, k["rlk"])
        yb = eng.make_power_basis(eng.encrypt(zy, k["pk"]), 4, k["rlk"])
        res.append(eng.poly2_int(xb, yb, W, 64, k["rlk"]))
    for a, b in zip(*res):
        _same(g, o, a, b)
    want = sum(W[0, i, j] / 64 * zx ** i * zy ** j for i in range(4) for j in range(5))
    np.testing.assert_allclose(g.decrypt(res[0][0], kg["sk"]), want, atol=1e-4)


@pytest.mark.parametrize("kw", [SMALL, DIGITS12], ids=["small", "digits12"])
def test_rotate_hoisted_bit_exact(product_lib, oracle_lib, gpu_available, kw):
    """aesfhe_rotate_hoisted (one ModUp shared by every key) against the oracle's per-key
    restatement; slots equal np.roll like the ordinary rotation."""
    g, o = _pair(product_lib, oracle_lib, **kw)
    outs = []
    rng = np.random.default_rng(3)
    z = rng.uniform(-1, 1, (2, g.slot_count))
    for eng in (g, o):
        sk = eng.create_secret_key(7)
        c = eng.encrypt(z, eng.create_public_key(sk), level=4)
        keys = [eng.create_hoisted_rotation_key(sk, d) for d in (1, -5, 64)]
        outs.append((eng.rotate_hoisted(c, keys), sk))
    for cg, co in zip(outs[0][0], outs[1][0]):
        _same(g, o, cg, co)
    for d, cg in zip((1, -5, 64), outs[0][0]):
        np.testing.assert_allclose(g.decrypt(cg, outs[0][1]), np.roll(z, d, axis=1), atol=1e-6)


def test_mul_fma_and_mixed_lincomb_bit_exact(product_lib, oracle_lib, gpu_available):
    g, o = _pair(product_lib, oracle_lib, **SMALL)
    res = []
    rng = np.random.default_rng(4)
    z = [rng.uniform(-1, 1, (3, g.slot_count)) for _ in range(3)]
    for eng in (g, o):
        k = _keys(eng)
        a, b, c = (eng.encrypt(z[0], k["pk"], level=5), eng.encrypt(z[1][:1], k["pk"], level=4),
                   eng.encrypt(z[2], k["pk"], level=6))
        res.append([eng.multiply_fma(a, b, k["rlk"], alpha=2, c=c, gamma=-1.0, beta=-1.0),
                    eng.multiply_fma(a, a, k["rlk"], alpha=2, beta=-1.0),
                    eng.lincomb([a, b, c], [0.5, -0.25j, 3.0])]
                   + eng.lincomb_many([a, b, c], [[1.0, 2.0, -1.0], [0.25, 0.0, 1j]]))
    for cg, co in zip(*res):
        _same(g, o, cg, co)


@pytest.mark.parametrize("kw", [SMALL, dict(log_n=16, max_level=8, special_primes=4, seed=5)],
                         ids=["n4096", "n65536"])
def test_dot_fma_bit_exact(product_lib, oracle_lib, gpu_available, kw):
    """aesfhe_dot_fma (the depth-optimal Chebyshev node sum): products at mixed levels and
    broadcast batches, addends above the product level (truncated), zero coefficients, beta; and
    its slots against the plain expression."""
    g, o = _pair(product_lib, oracle_lib, **kw)
    res = []
    rng = np.random.default_rng(11)
    L = kw["max_level"]
    z = [rng.uniform(-1, 1, (2, g.slot_count)) for _ in range(5)]
    for eng in (g, o):
        k = _keys(eng)
        a0, b0 = eng.encrypt(z[0], k["pk"], level=L - 2), eng.encrypt(z[1][:1], k["pk"], level=L - 2)
        a1, b1 = eng.encrypt(z[2], k["pk"], level=L - 1), eng.encrypt(z[3], k["pk"], level=L)
        c0 = eng.encrypt(z[4], k["pk"], level=L)
        outs = [eng.dot_fma([a0, a1], [b0, b1], k["rlk"], [(c0, 0.75), (a1, -1.5), (b1, 0.0)], -0.5),
                eng.dot_fma([a0], [a0], k["rlk"], [(b0, 2.0)]),
                eng.dot_fma([a1], [b1], k["rlk"], beta=1.25)]
        res.append((outs, k))
    for cg, co in zip(res[0][0], res[1][0]):
        _same(g, o, cg, co)
    sk = res[0][1]["sk"]
    want = [z[0] * z[1][:1] + z[2] * z[3] + 0.75 * z[4] - 1.5 * z[2] - 0.5, z[0] * z[0] + 2.0 * z[1][:1],
            z[2] * z[3] + 1.25]
    for cg, w, lv in zip(res[0][0], want, (L - 3, L - 3, L - 2)):
        assert cg.level == lv
        np.testing.assert_allclose(g.decrypt(cg, sk).real, w, atol=1e-4)


@pytest.mark.parametrize("kw", [SMALL, dict(log_n=16, max_level=3, special_primes=2, seed=5),
                                dict(log_n=16, max_level=12, special_primes=10, seed=5),
                                dict(log_n=16, max_level=30, special_primes=10, digit_primes=12,
                                     scale_bits=40, seed=5)],
                         ids=["n4096", "n65536", "n65536K10", "n65536K10A12"])
def test_linear_bsgs_bit_exact(product_lib, oracle_lib, gpu_available, kw):
    """aesfhe_linear_bsgs (hoisted babies and lazy ModDown; at N = 2^16 the giants go through the
    fused ext-NTT row pass with accumulation) against the oracle's restatement, and its slots
    against the plain BSGS sum it computes."""
    g, o = _pair(product_lib, oracle_lib, **kw)
    n = g.slot_count
    rng = np.random.default_rng(6)
    z = rng.uniform(-1, 1, (2, n))
    diags = [rng.uniform(-1, 1, n) for _ in range(5)]
    plan = [(0, [(0, 0), (1, 1), (2, 2)]), (-6, [(0, 3)]), (24, [(1, 4), (2, 0)])]  # (giant, [(baby, diag)])
    babies = [0, 1, -3]
    outs = []
    for eng in (g, o):
        sk = eng.create_secret_key(7)
        c = eng.encrypt(z, eng.create_public_key(sk), level=kw["max_level"])
        bk = [None if d == 0 else eng.create_hoisted_rotation_key(sk, -d) for d in babies]
        gk = [None if d == 0 else eng.create_fixed_rotation_key(sk, -d) for d, _ in plan]
        pts = [eng.encode(v) for v in diags]
        terms = [[(b, pts[i]) for b, i in tl] for _, tl in plan]
        outs.append((eng.linear_bsgs(c, bk, gk, terms), sk))
    _same(g, o, outs[0][0], outs[1][0])
    want = sum(np.roll(sum(diags[i] * np.roll(z, -babies[b], axis=1) for b, i in tl), -d, axis=1)
               for d, tl in plan)
    assert outs[0][0].level == kw["max_level"] - 1
    np.testing.assert_allclose(g.decrypt(outs[0][0], outs[0][1]), want, atol=1e-5)


@pytest.mark.parametrize("log_n,kx", [(16, {}), (17, {}),
                                      (16, dict(max_level=30, special_primes=10, digit_primes=12, scale_bits=40))],
                         ids=["16", "17", "16K10A12"])
def test_fused_product_bit_exact(product_lib, oracle_lib, gpu_available, log_n, kx):
    """The fused-NTT engines' ciphertext product (N = 2^16 / 2^17: d2 = a1 b1 formed in the INTT
    copy-in, d0 / d1 and the own digit's term in the key-switch prologue; no tensor ciphertext):
    K = 3 over 7 limbs (a partial last digit), a batch x broadcast product at mismatched levels
    (one operand level-downed first), a square, fused multiply-adds (alpha, a higher-level addend,
    beta) and products at every level down to 1 -- all residue for residue against the oracle's
    tensor + relinearise + rescale.  K10A12: the bench's chain with 12-prime digits (L = 30)."""
    kw = dict(dict(log_n=log_n, max_level=6, special_primes=3, seed=21), **kx)
    L = kw["max_level"]
    g, o = _pair(product_lib, oracle_lib, **kw)
    rng = np.random.default_rng(9)
    z = rng.uniform(-1, 1, (3, g.slot_count))
    w = rng.uniform(-1, 1, g.slot_count)
    res, sks = [], []
    for eng in (g, o):
        k = _keys(eng)
        a, b = eng.encrypt(z, k["pk"], level=L), eng.encrypt(w, k["pk"], level=L - 1)
        out = [eng.multiply(a, b, k["rlk"]), eng.multiply(b, a, k["rlk"]), eng.multiply(b, b, k["rlk"]),
               # fused multiply-adds (Chebyshev / double-angle steps): alpha, c at a higher level, beta
               eng.multiply_fma(a, b, k["rlk"], alpha=2, c=a, gamma=-1.0, beta=-1.0),
               eng.multiply_fma(b, b, k["rlk"], alpha=2, beta=-1.0),
               eng.multiply_fma(b, a, k["rlk"], alpha=-3, c=b, gamma=0.5),
               # rescales through the spread-fused column pass: constant products (plain
               # rescale) and exact-scale level-downs by one and by several levels
               eng.multiply(a, 0.37), eng.multiply(b, -1.5),
               eng.level_down(a, L - 1), eng.level_down(a, 2), eng.level_down(b, 1)]
        # grouped rescale (lincomb_many: the groups as one batch through the fused rescale)
        out += eng.lincomb_many([a, b, a], [[1.0, 2.0, -1.0], [0.25, 0.0, 1j], [-3.0, 0.5, 0.0]])
        x = a
        while x.level >= 1:
            x = eng.multiply(x, a, k["rlk"])
            out.append(x)
        res.append(out)
        sks.append(k["sk"])
    for cg, co in zip(*res):
        _same(g, o, cg, co)
    np.testing.assert_allclose(g.decrypt(res[0][0], sks[0]), z * w, atol=1e-5)


@pytest.mark.parametrize("kw", [SMALL, dict(log_n=16, max_level=4, special_primes=2, seed=5), DIGITS12],
                         ids=["n4096", "n65536", "digits12"])
def test_switching_key_export_bit_exact(product_lib, oracle_lib, gpu_available, kw):
    """Relinearisation, conjugation and hoisted rotation keys: aesfhe_key_export returns
    residues equal to the oracle's, and a saved + loaded key relinearises to the same residues."""
    import ctypes as C
    g, o = _pair(product_lib, oracle_lib, **kw)

    def words(eng, key):
        kind, gal, seed, n = C.c_int32(), C.c_uint64(), C.c_uint64(), C.c_int64()
        eng._check(eng._lib.key_export(eng._h, key._h, C.byref(kind), C.byref(gal), C.byref(seed), C.byref(n), None))
        out = np.empty(n.value, np.uint64)
        eng._check(eng._lib.key_export(eng._h, key._h, C.byref(kind), C.byref(gal), C.byref(seed), C.byref(n),
                                       out.ctypes.data_as(C.POINTER(C.c_uint64))))
        return out

    kg, ko = _keys(g), _keys(o)
    for name in ("rlk", "cjk"):
        np.testing.assert_array_equal(words(g, kg[name]), words(o, ko[name]))
    hg = g.create_hoisted_rotation_key(kg["sk"], -3)
    ho = o.create_hoisted_rotation_key(ko["sk"], -3)
    np.testing.assert_array_equal(words(g, hg), words(o, ho))
    import tempfile, os
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "rlk.bin")
        g.save(kg["rlk"], path)
        rl2 = g.load(path)
    rng = np.random.default_rng(12)
    z = rng.uniform(-1, 1, g.slot_count)
    cg, co = g.encrypt(z, kg["pk"]), o.encrypt(z, ko["pk"])
    _same(g, o, g.multiply(cg, cg, rl2), o.multiply(co, co, ko["rlk"]))


@pytest.mark.parametrize("degrees", [(2, 3, 5, 8, 13, 16, 17, 31, 33)])
def test_power_basis_batched_bit_exact(product_lib, oracle_lib, gpu_available, degrees):
    """aesfhe_power_basis at N = 2^16 (one ciphertext: the products of each depth run as one
    batched product with x^{2^j} broadcast, the lower powers level-downed straight into the
    operand block) against the oracle's sequential basis, residue for residue: full and partial
    last depths, powers of two and their neighbours."""
    kw = dict(log_n=16, max_level=7, special_primes=3, seed=31)
    g, o = _pair(product_lib, oracle_lib, **kw)
    rng = np.random.default_rng(13)
    z = np.exp(-2j * np.pi * rng.integers(0, 256, g.slot_count) / 256)
    res, sks = [], []
    for eng in (g, o):
        k = _keys(eng)
        c = eng.encrypt(z, k["pk"], level=6)
        res.append([eng.make_power_basis(c, d, k["rlk"]) for d in degrees])
        sks.append(k["sk"])
    for bg, bo, d in zip(res[0], res[1], degrees):
        assert len(bg) == len(bo) == d
        for cg, co in zip(bg, bo):
            _same(g, o, cg, co)
    top = res[0][-1]
    np.testing.assert_allclose(g.decrypt(top[-1], sks[0]), z ** degrees[-1], atol=1e-4)


def test_power_basis_255_full_params_bit_exact(product_lib, oracle_lib, gpu_available):
    """The S-box's make_power_basis(ct, 255) at BASELINE.json's N = 2^16, L = 30 (K = 10, the
    bench chain): every one of the 255 powers residue-identical to the oracle's sequential basis
    (reference: sbox/sbox_service.py:91-93, gf_service.py:55-64)."""
    kw = dict(log_n=16, max_level=30, special_primes=10, seed=99)
    g, o = _pair(product_lib, oracle_lib, **kw)
    rng = np.random.default_rng(14)
    x = rng.integers(0, 256, g.slot_count)
    z = np.exp(2j * np.pi * x / 256)
    res, sks = [], []
    for eng in (g, o):
        k = dict(sk=eng.create_secret_key(7))
        k["pk"] = eng.create_public_key(k["sk"])
        k["rlk"] = eng.create_relinearization_key(k["sk"])
        res.append(eng.make_power_basis(eng.encrypt(z, k["pk"]), 255, k["rlk"]))
        sks.append(k["sk"])
    for cg, co in zip(*res):
        _same(g, o, cg, co)
    assert [c.level for c in res[0]] == [30 - int(np.ceil(np.log2(k))) for k in range(1, 256)]
    for p in (1, 2, 127, 128, 255):
        np.testing.assert_allclose(g.decrypt(res[0][p - 1], sks[0]), z ** p, atol=1e-3)


@pytest.mark.parametrize("scale_bits,wmax", [(40, 8), (44, 16)], ids=["s40w8", "s44w16"])
def test_poly2_int_sbox_shape_bit_exact(product_lib, oracle_lib, gpu_available, scale_bits, wmax):
    """aesfhe_poly2_int with the S-box's shape at N = 2^16: 15 x and 15 y basis ciphertexts
    (ny = 16, the compile-time basis size), a full pair of output blocks of 4 (k_poly2_int_s,
    both blocks in one launch) and a partial block, integer weights in [-wmax, wmax] / 64, mixed
    basis levels, the top limb q_0 on the folding kernel -- residue for residue against the
    oracle.  s40w8: y' left unreduced (the AES S-box's case); s44w16: row sums too large for
    that on 44-bit limbs, so y' is reduced."""
    kw = dict(log_n=16, max_level=7, special_primes=3, seed=41, scale_bits=scale_bits)
    g, o = _pair(product_lib, oracle_lib, **kw)
    rng = np.random.default_rng(15)
    zx = rng.uniform(-1, 1, (2, g.slot_count))
    zy = rng.uniform(-1, 1, g.slot_count)
    W = rng.integers(-wmax, wmax + 1, (10, 16, 16))
    W[3] = 0
    res = []
    for eng in (g, o):
        k = _keys(eng)
        xb = eng.make_power_basis(eng.encrypt(zx, k["pk"], level=6), 15, k["rlk"])
        yb = eng.make_power_basis(eng.encrypt(zy, k["pk"], level=6), 15, k["rlk"])
        res.append(eng.poly2_int(xb, yb, W, 64, k["rlk"]))
    for a, b in zip(*res):
        _same(g, o, a, b)


@pytest.mark.parametrize("scale_bits", [40, 44], ids=["s40", "s44"])
def test_poly2_int_aes_sbox_weights_bit_exact(product_lib, oracle_lib, gpu_available, scale_bits):
    """aesfhe_poly2_int with exactly the AES S-box's Walsh weights (64 W, den 64, 8 outputs: the
    bench round's call, aes_round_bits.walsh_sbox) on +-1 bit inputs: residue for residue against
    the oracle at N = 2^16 with mixed basis levels, a slab rotation, and q_0 on the split kernel
    (reference: the S-box the bit-sliced round evaluates, sbox/sbox_service.py:116-138)."""
    from aes_xor_fhe.aes_round_bits import walsh_sbox
    W = np.rint(walsh_sbox() * 64).astype(np.int64)
    kw = dict(log_n=16, max_level=7, special_primes=3, seed=43, scale_bits=scale_bits)
    g, o = _pair(product_lib, oracle_lib, **kw)
    rng = np.random.default_rng(16)
    zx = rng.choice([-1.0, 1.0], (4, g.slot_count))
    zy = rng.choice([-1.0, 1.0], (4, g.slot_count))
    res = []
    for eng in (g, o):
        k = _keys(eng)
        xb = eng.make_power_basis(eng.encrypt(zx, k["pk"], level=6), 15, k["rlk"])
        yb = eng.make_power_basis(eng.encrypt(zy, k["pk"], level=6), 15, k["rlk"])
        res.append(eng.poly2_int(xb, yb, W, 64, k["rlk"], slab_rot=1))
    for a, b in zip(*res):
        _same(g, o, a, b)


@pytest.mark.parametrize("kw", [SMALL, dict(log_n=16, max_level=6, special_primes=3, seed=13)],
                         ids=["n4096", "n65536"])
def test_cyclic_broadcast_mul_bit_exact(product_lib, oracle_lib, gpu_available, kw):
    """aesfhe_mul with a smaller power-of-two batch cycled through (element i takes element
    i mod B_small: the sliced AES state's batch-4 round keys), at N = 2^12 (tensor + relinearise)
    and N = 2^16 (the fused product: cycled reads in the INTT copy-in and the key-switch
    prologue), either operand order, against the oracle; a non-dividing batch is refused."""
    g, o = _pair(product_lib, oracle_lib, **kw)
    rng = np.random.default_rng(21)
    z8, z4, z2 = (rng.uniform(-1, 1, (b, g.slot_count)) for b in (8, 4, 2))
    res, sks = [], []
    for eng in (g, o):
        k = _keys(eng)
        a8, a4, a2 = (eng.encrypt(z, k["pk"], level=lv) for z, lv in ((z8, 6), (z4, 6), (z2, 5)))
        res.append([eng._call_ct(eng._lib.mul, a8._h, a4._h, k["rlk"]._h),
                    eng._call_ct(eng._lib.mul, a2._h, a8._h, k["rlk"]._h)])
        sks.append(k["sk"])
        b6, b3 = eng.encrypt(z8[:6], k["pk"]), eng.encrypt(z8[:3], k["pk"])  # held: handles stay valid
        with pytest.raises(RuntimeError, match="batch mismatch"):
            eng._call_ct(eng._lib.mul, b6._h, b3._h, k["rlk"]._h)
    for cg, co in zip(*res):
        _same(g, o, cg, co)
    idx = np.arange(8)
    np.testing.assert_allclose(g.decrypt(res[0][0], sks[0]).real, z8 * z4[idx % 4], atol=1e-5)
    np.testing.assert_allclose(g.decrypt(res[0][1], sks[0]).real, z2[idx % 2] * z8, atol=1e-5)
