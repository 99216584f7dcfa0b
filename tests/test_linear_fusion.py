"""Deferred linear combinations in the facade (fhe._LinearCiphertext, Engine(fuse_linear=True)):
`multiply(ct, constant)` and the adds that consume it are materialised as one fused lincomb.

Checked on the CPU oracle: the same levels / is_zero flags / batch errors as the eager
evaluation (fuse_linear=False), decoded values equal to it, residues equal to an explicit
Engine.lincomb of the same terms, and the reference-order S-box LUT (sbox/sbox_service.py:116-138)
decoding to FIPS-197 with the reference's op trace either way."""
import json
from pathlib import Path

import numpy as np
import pytest

from aes_xor_fhe import aes_tables as T
from aes_xor_fhe.fhe import Engine, _LinearCiphertext

from _tracing import make_wrap

KW = dict(log_n=10, max_level=8, special_primes=3, seed=5)
TRACES = json.loads((Path(__file__).resolve().parent / "golden" / "traces.json").read_text())


def _engines(oracle_lib):
    out = []
    for fuse in (True, False):
        e = Engine(_lib=oracle_lib, fuse_linear=fuse, **KW)
        sk = e.create_secret_key(3)
        out.append((e, sk, e.create_public_key(sk)))
    return out


def test_levels_flags_and_values_match_eager(oracle_lib):
    (f, skf, pkf), (g, skg, pkg) = _engines(oracle_lib)
    rng = np.random.default_rng(0)
    z = rng.uniform(-1, 1, (2, f.slot_count)) + 1j * rng.uniform(-1, 1, (2, f.slot_count))
    res = []
    for e, pk in ((f, pkf), (g, pkg)):
        a = e.encrypt(z, pk, level=7)
        b = e.encrypt(z[:1], pk, level=5)  # broadcast operand, lower level
        t0 = e.multiply(a, 0.0)
        t1 = e.add(t0, e.multiply(a, 0.5 - 0.25j))
        t2 = e.add(t1, e.multiply(b, 2.0))           # term one level lower (5 -> 4)
        t3 = e.add(e.encode(np.full(e.slot_count, 0.125 + 1j)), t2)  # constant plaintext
        t4 = e.add(t3, b)                             # a ciphertext addend at level 5
        t5 = e.add(t4, 0.75)
        res.append([t0, t1, t2, t3, t4, t5])
    for lf, le in zip(*res):
        assert (lf.level, lf.batch, lf.npoly, lf.is_zero) == (le.level, le.batch, le.npoly, le.is_zero)
    assert isinstance(res[0][5], _LinearCiphertext) and not isinstance(res[1][5], _LinearCiphertext)
    want = 0.5 * z - 0.25j * z + 2.0 * z[:1] + (0.125 + 1j) + z[:1] + 0.75
    for e, sk, r in ((f, skf, res[0][5]), (g, skg, res[1][5])):
        np.testing.assert_allclose(e.decrypt(r, sk), want, atol=1e-4)
    assert res[0][0].is_zero and res[0][0].level == 6
    np.testing.assert_allclose(f.decrypt(res[0][0], skf), 0, atol=1e-6)


def test_materialised_residues_equal_lincomb(oracle_lib):
    (f, skf, pkf), _ = _engines(oracle_lib)
    rng = np.random.default_rng(1)
    cts = [f.encrypt(rng.uniform(-1, 1, f.slot_count), pkf, level=lv) for lv in (7, 6, 6, 4)]
    co = [0.5, -1.25j, 3.0 + 0.5j, 0.0625]
    acc = f.multiply(cts[0], co[0])
    for c, k in zip(cts[1:], co[1:]):
        acc = f.add(acc, f.multiply(c, k))
    assert isinstance(acc, _LinearCiphertext) and acc.level == 3
    np.testing.assert_array_equal(f.export_residues(acc), f.export_residues(f.lincomb(cts, co)))


def test_batch_mismatch_raises_like_eager(oracle_lib):
    (f, _, pkf), (g, _, pkg) = _engines(oracle_lib)
    for e, pk in ((f, pkf), (g, pkg)):
        a = e.encrypt(np.ones((2, 4)), pk)
        b = e.encrypt(np.ones((3, 4)), pk)
        with pytest.raises(RuntimeError, match="batch mismatch"):
            e.add(e.multiply(a, 2.0), e.multiply(b, 2.0))


@pytest.mark.parametrize("fuse", [True, False], ids=["deferred", "eager"])
def test_sbox_reference_order_either_way(oracle_lib, fuse):
    from aes_xor_fhe.sbox.sbox_service import SBoxService
    from aes_xor_fhe.utils import zeta_decode, zeta_encode
    w = make_wrap(oracle_lib, tracing=True, fuse_linear=fuse)
    sb = SBoxService(w.ctx)
    x = np.random.default_rng(2).integers(0, 256, w.engine.slot_count)
    enc = w.engine.encrypt(zeta_encode(x, modulus=256), w.public_key)
    w.engine.trace.clear()
    out = sb.sub_bytes_array(enc)
    trace = dict(w.engine.trace)
    assert trace == TRACES["sub_bytes_array"]
    assert np.array_equal(zeta_decode(w.engine.decrypt(out, w.secret_key), modulus=256), T.SBOX[x])


def test_deferred_product_errors(oracle_lib):
    """Deferred products (fhe._ProductCiphertext): what can be checked at the call is checked
    there -- a relinearization key of another engine raises at multiply(); an error of the
    evaluation itself surfaces as a RuntimeError at the first use of the handle; at most
    max_pending products wait unevaluated (the next one evaluates them first)."""
    e = Engine(_lib=oracle_lib, max_pending=3, **KW)
    sk = e.create_secret_key(3)
    rlk = e.create_relinearization_key(sk)
    other = Engine(_lib=oracle_lib, **KW)
    ct = e.encrypt(np.ones(8), e.create_public_key(sk), level=5)
    with pytest.raises(ValueError, match="another engine"):
        e.multiply(ct, ct, other.create_relinearization_key(other.create_secret_key(3)))
    # an evaluation error appears at first use (here: the C call reports a device error)
    real = e._lib.mul
    try:
        e._lib.mul = lambda *a: -3
        p = e.multiply(ct, ct, rlk)
        assert p.pending and p.level == 4
        with pytest.raises(RuntimeError, match="device error"):
            e.decrypt(p, sk)
    finally:
        e._lib.mul = real
    ps = [e.multiply(ct, ct, rlk) for _ in range(5)]
    assert sum(p.pending for p in ps) <= 3
    np.testing.assert_allclose(e.decrypt(ps[-1], sk)[:8].real, np.ones(8), atol=1e-3)


def test_deferred_conjugations_batched_residue_exact(oracle_lib):
    """Engine.conjugate is deferred (fhe._GaloisCiphertext) and the pending conjugations of one
    key and level run as one batched aesfhe_galois: the residues equal the eager calls' (the key
    switch is elementwise over the batch), levels / batches are the eager ones, and the
    reference's xor_cipher (seven conjugations per power basis) decodes the same."""
    (f, skf, pkf), (g, skg, pkg) = _engines(oracle_lib)
    rng = np.random.default_rng(4)
    z = rng.uniform(-1, 1, (3, f.slot_count)) + 1j * rng.uniform(-1, 1, (3, f.slot_count))
    outs = []
    for e, sk, pk in ((f, skf, pkf), (g, skg, pkg)):
        cjk = e.create_conjugation_key(sk)
        cts = [e.encrypt(z[:2], pk, level=7), e.encrypt(z[2], pk, level=7), e.encrypt(z[:2], pk, level=6),
               e.encrypt(z[1], pk, level=7)]
        cj = [e.conjugate(c, cjk) for c in cts]
        assert [(c.level, c.batch) for c in cj] == [(7, 2), (7, 1), (6, 2), (7, 1)]
        if e is f:
            assert all(c.pending for c in cj)
        outs.append([e.export_residues(c) for c in cj])
        np.testing.assert_allclose(e.decrypt(cj[1], sk), np.conj(z[2]), atol=1e-4)
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


def test_fused_products_leave_the_pending_cap(oracle_lib):
    """products a fused sum (aesfhe_poly2) has used no longer count against
    max_pending, so building more than max_pending products in fused groups never falls back
    to an eager aesfhe_mul per product -- and the fused results decode correctly."""
    e = Engine(_lib=oracle_lib, max_pending=4, **KW)
    sk = e.create_secret_key(3)
    pk, rlk = e.create_public_key(sk), e.create_relinearization_key(sk)
    z = np.random.default_rng(7).uniform(-1, 1, (3, e.slot_count))
    a, b, c = (e.encrypt(v, pk, level=6) for v in z)
    calls = []
    real = e._lib.mul
    e._lib.mul = lambda *args: (calls.append(1), real(*args))[1]
    try:
        outs = []
        for g in range(4):  # 4 groups x 3 products = 12 > max_pending
            k = 0.25 * (g + 1)
            s = e.add(e.add(e.multiply(e.multiply(a, b, rlk), k), e.multiply(e.multiply(a, c, rlk), -k)),
                      e.multiply(e.multiply(b, c, rlk), 0.5))
            outs.append((k, e.decrypt(s, sk)))  # materialised: one poly2 of the group
        assert not calls, f"{len(calls)} eager aesfhe_mul calls"
        assert len(e._pending) == 0
    finally:
        e._lib.mul = real
    for k, got in outs:
        want = k * z[0] * z[1] - k * z[0] * z[2] + 0.5 * z[1] * z[2]
        np.testing.assert_allclose(got.real, want, atol=1e-3)
