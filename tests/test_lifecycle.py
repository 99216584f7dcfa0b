"""Object lifecycle, randomness, serialisation and device transfer at the ABI boundary.

* default engines (no seed) draw their seed, secret keys and nonces from os.urandom: two of them
  never share a key (engine_context.py:62 calls create_secret_key() without arguments);
* the engine may be destroyed before its ciphertexts and keys (Python's cycle collector
  finalises them in any order; regression test for the teardown-order segfault fixed in
  commit 4619bd7): the C engine stays alive until its last object is freed;
* Engine.save / Engine.load round-trip ciphertexts and every key kind, and refuse files made
  under other parameters;
* aesfhe_ct_export_device / aesfhe_ct_import_device (parallel.py's RCCL path) move residues
  through a caller-owned buffer bit-exactly.
Each runs on the CPU oracle; the `gpu` variants run the same checks on the HIP engine.
"""
import ctypes as C
import gc

import numpy as np
import pytest

from aes_xor_fhe.fhe import Engine
from aes_xor_fhe.xor_service import ZetaEncoder

KW = dict(log_n=10, max_level=4, special_primes=2)


def _sk_words(e, sk):
    kind, g, seed, words = C.c_int32(), C.c_uint64(), C.c_uint64(), C.c_int64()
    e._check(e._lib.key_export(e._h, sk._h, C.byref(kind), C.byref(g), C.byref(seed),
                               C.byref(words), None))
    out = np.empty(words.value, np.uint64)
    e._check(e._lib.key_export(e._h, sk._h, C.byref(kind), C.byref(g), C.byref(seed), C.byref(words),
                               out.ctypes.data_as(C.POINTER(C.c_uint64))))
    return out


def _default_keys_differ(lib):
    a, b = Engine(_lib=lib, **KW), Engine(_lib=lib, **KW)
    assert a._params["seed"] != b._params["seed"]
    assert not np.array_equal(_sk_words(a, a.create_secret_key()), _sk_words(b, b.create_secret_key()))
    # two unseeded secret keys of the same engine differ too
    assert not np.array_equal(_sk_words(a, a.create_secret_key()), _sk_words(a, a.create_secret_key()))
    # seeded engines are reproducible
    s1, s2 = Engine(_lib=lib, seed=9, **KW), Engine(_lib=lib, seed=9, **KW)
    assert np.array_equal(_sk_words(s1, s1.create_secret_key()), _sk_words(s2, s2.create_secret_key()))
    # shared seed, disjoint nonce ranges: the same message encrypts differently
    from aes_xor_fhe.parallel import rank_nonce_start
    r0 = Engine(_lib=lib, seed=9, nonce_start=rank_nonce_start(0), **KW)
    r1 = Engine(_lib=lib, seed=9, nonce_start=rank_nonce_start(1), **KW)
    x = np.ones(8)
    c0 = r0.encrypt(x, r0.create_public_key(r0.create_secret_key()))
    c1 = r1.encrypt(x, r1.create_public_key(r1.create_secret_key()))
    assert not np.array_equal(r0.export_residues(c0), r1.export_residues(c1))


def _destroy_engine_first(lib):
    from aes_xor_fhe._abi import Params
    p = Params(10, 4, 2, 40, 50, 50, 0, 1, 5, None)
    h = C.c_void_p()
    lib.check(lib.engine_create(C.byref(p), C.byref(h)))
    sk = C.c_void_p()
    lib.check(lib.key_secret(h, 1, C.byref(sk)))
    co = np.zeros((2, 1 << 10), np.int64)
    ct = C.c_void_p()
    lib.check(lib.encrypt(h, sk, co.ctypes.data_as(C.POINTER(C.c_int64)), 2, 4, 0, C.byref(ct)))
    lib.engine_destroy(h)          # before its objects
    lib.ct_free(ct)
    lib.key_free(sk)
    # the same through Python's cycle collector: engine <-> ciphertext cycle
    e = Engine(_lib=lib, seed=1, **KW)
    c = e.encrypt(np.ones(4), e.create_public_key(e.create_secret_key()))
    e._cycle = c
    del e, c
    gc.collect()


def _save_load(lib, tmp_path):
    e = Engine(_lib=lib, seed=11, **KW)
    sk = e.create_secret_key(2)
    pk, rlk = e.create_public_key(sk), e.create_relinearization_key(sk)
    cjk, frk = e.create_conjugation_key(sk), e.create_fixed_rotation_key(sk, -3)
    x = ZetaEncoder.to_zeta(np.arange(e.slot_count) % 16, 16)
    ct = e.encrypt(x, pk)
    objs = dict(sk=sk, pk=pk, rlk=rlk, cjk=cjk, frk=frk, ct=ct)
    back = {}
    for k, o in objs.items():
        e.save(o, tmp_path / f"{k}.bin")
        back[k] = e.load(tmp_path / f"{k}.bin")
        assert type(back[k]) is type(o)
    assert np.array_equal(e.export_residues(back["ct"]), e.export_residues(ct))
    assert back["frk"].delta == -3 and back["cjk"].galois_elt == cjk.galois_elt
    # loaded keys compute the same residues as the originals
    for op in (lambda ks: e.multiply(ct, ct, ks["rlk"]), lambda ks: e.rotate(ct, ks["frk"], -3),
               lambda ks: e.conjugate(ct, ks["cjk"])):
        assert np.array_equal(e.export_residues(op(objs)), e.export_residues(op(back)))
    dec = ZetaEncoder.from_zeta(e.decrypt(e.encrypt(x, back["pk"]), back["sk"]), 16)
    assert np.array_equal(dec, np.arange(e.slot_count) % 16)
    other = Engine(_lib=lib, seed=11, log_n=10, max_level=5, special_primes=2)
    with pytest.raises(RuntimeError, match="different parameters"):
        other.load(tmp_path / "ct.bin")


def _device_roundtrip(lib, make_buf):
    e = Engine(_lib=lib, seed=4, **KW)
    sk = e.create_secret_key()
    ct = e.encrypt(np.random.default_rng(0).standard_normal((3, 16)), sk)
    res = e.export_residues(ct)
    per = res[0].size
    buf, ptr = make_buf(2 * per)
    e.export_into(ct, ptr, 1, 2)             # batch elements 1..2
    back = e.import_from(ptr, 2, ct.npoly, ct.level)
    assert np.array_equal(e.export_residues(back), res[1:3])
    with pytest.raises(RuntimeError):
        e.export_into(ct, ptr, 2, 2)          # out of range


def test_default_keys_differ_oracle(oracle_lib):
    _default_keys_differ(oracle_lib)


def test_engine_destroyed_before_objects_oracle(oracle_lib):
    _destroy_engine_first(oracle_lib)


def test_save_load_oracle(oracle_lib, tmp_path):
    _save_load(oracle_lib, tmp_path)


def test_device_transfer_oracle(oracle_lib):
    def host(words):
        a = np.empty(words, np.uint64)
        return a, a.ctypes.data
    _device_roundtrip(oracle_lib, host)


@pytest.mark.gpu
def test_default_keys_differ_gpu(product_lib, gpu_available):
    _default_keys_differ(product_lib)


@pytest.mark.gpu
def test_engine_destroyed_before_objects_gpu(product_lib, gpu_available):
    _destroy_engine_first(product_lib)


@pytest.mark.gpu
def test_save_load_gpu(product_lib, gpu_available, tmp_path):
    _save_load(product_lib, tmp_path)


@pytest.mark.gpu
def test_device_transfer_gpu(product_lib, gpu_available):
    import torch

    def dev(words):
        t = torch.empty(words, dtype=torch.int64, device="cuda:0")
        torch.cuda.synchronize()
        return t, t.data_ptr()
    _device_roundtrip(product_lib, dev)


@pytest.mark.gpu
def test_device_arena_reuse_gpu(product_lib, gpu_available):
    """The chunked best-fit arena (engine.hip Pool): ciphertexts of many sizes created and freed
    in random order leave every byte reusable (live returns to its baseline, no new chunk for a
    repeat of the same workload), split batched results (poly2 outputs) free independently, and
    trim returns the empty chunks; values stay intact throughout."""
    e = Engine(_lib=product_lib, log_n=12, max_level=8, special_primes=3, seed=5)
    sk = e.create_secret_key(1)
    pk, rlk = e.create_public_key(sk), e.create_relinearization_key(sk)
    rng = np.random.default_rng(9)
    z = np.exp(2j * np.pi * rng.integers(0, 16, e.slot_count) / 16)
    w = e.encrypt(z, pk)
    w = e.multiply(w, w, rlk)  # anything materialised on first use exists before the baseline
    del w
    gc.collect()
    e.synchronize()
    base = e.pool_stats()["live"]

    def workload():
        cts = [e.encrypt(z, pk, level=int(rng.integers(1, 9))) for _ in range(40)]
        cts += [e.concat([cts[i]] * int(rng.integers(1, 5))) for i in range(10)]
        prods = [e.multiply(cts[i], cts[i + 1], rlk) for i in range(0, 20, 2)]
        for i in rng.permutation(len(cts)):
            cts[i] = None
        np.testing.assert_allclose(e.decrypt(prods[3], sk), z * z, atol=1e-4)
        del prods, cts
        gc.collect()
        e.synchronize()

    workload()
    after1 = e.pool_stats()
    assert after1["live"] == base, (after1, base)
    workload()
    after2 = e.pool_stats()
    assert after2["live"] == base and after2["mallocs"] == after1["mallocs"], (after1, after2)
    # split results: poly2_int outputs share one block; freed in any order they merge back
    xb = e.make_power_basis(e.encrypt(z, pk), 3, rlk)
    yb = e.make_power_basis(e.encrypt(z, pk), 3, rlk)
    W = rng.integers(-4, 5, (4, 4, 4))
    outs = e.poly2_int(xb, yb, W, 64, rlk)
    want = sum(W[2, i, j] / 64 * z ** i * z ** j for i in range(4) for j in range(4))
    np.testing.assert_allclose(e.decrypt(outs[2], sk), want, atol=1e-3)
    for i in (1, 3, 0, 2):
        outs[i] = None
    del xb, yb, outs
    gc.collect()
    e.synchronize()
    assert e.pool_stats()["live"] == base
    held = e.pool_stats()["held"]
    e.pool_trim()
    assert e.pool_stats()["held"] <= held
