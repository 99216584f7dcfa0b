"""GPU parity at the bench's own shapes.

The other parity tests run the bootstrap and the sliced round at N = 2^10 / 2^12, where the fused
N = 2^16 kernels do not run (fused_ntt() is false), the BSGS order walk sees 4 blocks instead of
256 and k_bsgs_terms only ever gets partial batch blocks.  Here: N = 2^16 on the bench chain
(L = 30, K = 10 special primes, 12-prime key-switch digits, scale 40) with batches that fill the
kernels' full blocks, residue for residue against the oracle.

* linear_bsgs at B = 8 with 4 giants (k_bsgs_terms<4, 3, 4, 2>: two full BB = 4 batch blocks) and
  with 6 giants (<8, 3, 2, 1>: the G = 8, BB = 2 instantiation), babies on one Galois orbit (the
  256-block orbit walk), the fused ModUp / ModDown column kernels (bconv_cols.h) in every key switch;
* bit bootstrapping with both bench bootstrappers (5-map and 3-map CoeffToSlot, shared keys, as
  bench.py builds them) over B = 8 pairs: every batch element of the batched GPU run equals the
  GPU's one-element run of that element (full blocks against partial ones), and one element of the
  second batch block equals the oracle's bootstrap of it (the oracle takes ~1 min per element at
  this size, so it checks one; the chain of exact equalities covers the rest).
"""
import numpy as np
import pytest

from aes_xor_fhe.bootstrap import Bootstrapper
from aes_xor_fhe.fhe import Engine

pytestmark = pytest.mark.gpu

BENCH = dict(log_n=16, max_level=30, special_primes=10, digit_primes=12, scale_bits=40, seed=5)


def _pair(product_lib, oracle_lib):
    g, o = Engine(_lib=product_lib, **BENCH), Engine(_lib=oracle_lib, **BENCH)
    assert g.primes == o.primes
    return g, o


def _same(a, b, what):
    if not np.array_equal(a, b):
        bad = np.argwhere(a != b)
        raise AssertionError(f"{what}: {len(bad)} residues differ; first at {bad[0].tolist()}")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("ng", [4, 6], ids=["G4BB4", "G6BB2"])
def test_linear_bsgs_bench_shapes_bit_exact(product_lib, oracle_lib, gpu_available, ng):
    g, o = _pair(product_lib, oracle_lib)
    n = g.slot_count
    rng = np.random.default_rng(11 + ng)
    z = rng.uniform(-1, 1, (8, n))
    babies = [0, 1, 2, 3]  # one identity + keyed babies g, g^2, g^3: the orbit walk applies
    giants = [0, 4, 8, 12, 16, 20][:ng]
    diags = [rng.uniform(-1, 1, n) for _ in range(len(babies) * ng)]
    plan = [(d, [(b, j * len(babies) + b) for b in range(len(babies)) if (b + j) % 3 != 2]) for j, d in enumerate(giants)]
    outs = []
    for eng in (g, o):
        sk = eng.create_secret_key(7)
        c = eng.encrypt(z, eng.create_public_key(sk), level=30)
        bk = [None if d == 0 else eng.create_hoisted_rotation_key(sk, -d) for d in babies]
        gk = [None if d == 0 else eng.create_fixed_rotation_key(sk, -d) for d, _ in plan]
        pts = [eng.encode(v) for v in diags]
        terms = [[(b, pts[i]) for b, i in tl] for _, tl in plan]
        out = eng.linear_bsgs(c, bk, gk, terms)
        outs.append(eng.export_residues(out))
        if eng is g:
            want = sum(np.roll(sum(diags[i] * np.roll(z, -babies[b], axis=1) for b, i in tl), -d, axis=1)
                       for d, tl in plan)
            assert out.level == 29 and out.batch == 8
            np.testing.assert_allclose(g.decrypt(out, sk), want, atol=1e-4)
    _same(outs[0], outs[1], f"linear_bsgs B = 8, {ng} giants")


@pytest.mark.timeout(900)
def test_bootstrap_bits_bench_shapes(product_lib, oracle_lib, gpu_available):
    g, o = _pair(product_lib, oracle_lib)
    n = g.slot_count
    rng = np.random.default_rng(12)
    a, b = rng.choice([-1.0, 1.0], (8, n)), rng.choice([-1.0, 1.0], (8, n))
    noise = 0.02 * rng.standard_normal((2, 8, n))
    sk = g.create_secret_key(1)
    pk, rlk = g.create_public_key(sk), g.create_relinearization_key(sk)
    bss = []
    for groups in (5, 3):  # as bench.py builds them: the 3-map one shares the 5-map one's keys
        bss.append(Bootstrapper(g, sk, rlk, cts_groups=groups, share=bss[0] if bss else None))
    ca, cb = g.encrypt(a + noise[0], pk, level=5), g.encrypt(b + noise[1], pk, level=5)
    assert ca.batch == 8
    check = 5  # an element of the second BB = 4 block
    ref_in = [g.export_residues(g.slice(x, check, 1)) for x in (ca, cb)]
    got = {}
    for bs in bss:
        ya, yb = bs.bootstrap_bits(ca, cb)
        assert ya.batch == 8 and ya.level == bs.bits_level
        full = [g.export_residues(y) for y in (ya, yb)]
        for i in range(8):  # batched (full blocks) == one element alone (a partial block)
            sa, sb = bs.bootstrap_bits(g.slice(ca, i, 1), g.slice(cb, i, 1))
            _same(full[0][i:i + 1], g.export_residues(sa), f"{bs.cts_groups}-map element {i} (a)")
            _same(full[1][i:i + 1], g.export_residues(sb), f"{bs.cts_groups}-map element {i} (b)")
        for y, v, nz in ((ya, a, noise[0]), (yb, b, noise[1])):
            assert np.all(np.abs(g.decrypt(y, sk) - v) <= 1.24 * nz ** 2 + 3e-3)
        got[bs.cts_groups] = [f[check:check + 1] for f in full]
    del bss, ya, yb, sa, sb
    g.pool_trim()
    # the oracle: the same keys (same engine seed and key seeds), element `check` imported from the GPU
    osk = o.create_secret_key(1)
    orlk = o.create_relinearization_key(osk)
    obs = []
    for groups in (5, 3):
        obs.append(Bootstrapper(o, osk, orlk, cts_groups=groups, share=obs[0] if obs else None))
    xa, xb = (o.import_residues(r) for r in ref_in)
    for bs in obs:
        ya, yb = bs.bootstrap_bits(xa, xb)
        _same(got[bs.cts_groups][0], o.export_residues(ya), f"{bs.cts_groups}-map vs oracle (a)")
        _same(got[bs.cts_groups][1], o.export_residues(yb), f"{bs.cts_groups}-map vs oracle (b)")
