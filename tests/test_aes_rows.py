"""Row-sliced bit-domain AES round (aes_xor_fhe.aes_round_bits, the bench's default step).

CPU: the oracle engine runs every stage (ShiftRows, SubBytes as a Walsh polynomial over
nibble-bit monomials, MixColumns, AddRoundKey) and four chained rounds inside one 30-level
budget, each checked against FIPS-197 (aes_tables, itself pinned by the FIPS-197 appendix
vectors in test_aes_tables.py).
GPU: the HIP engine produces residue-identical ciphertexts to the oracle for a full round at
N = 2^12 (bit-exact, integer work), and correct chained rounds at BASELINE.json's N = 2^16,
L = 30."""
import numpy as np
import pytest

from aes_xor_fhe import aes_tables as T
from aes_xor_fhe.aes_round_bits import AESRowRound, AESSlicedRound, walsh_sbox
from aes_xor_fhe.fhe import Engine


def _setup(lib, log_n, seed=5, cls=AESRowRound, **kw):
    kw = dict(dict(special_primes=8), **kw)
    e = Engine(log_n=log_n, max_level=30, seed=seed, _lib=lib, **kw)
    sk = e.create_secret_key(3)
    R = cls(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk))
    return e, R


def test_layout_roundtrip():
    R = AESRowRound.__new__(AESRowRound)
    R.sc, R.n_blk = 64, 16
    b = np.random.default_rng(0).integers(0, 256, (3, 16, 16), dtype=np.uint8)
    rows = R.pack(b)
    assert rows[2][1, 3 * 16 + 5] == b[1, 5, 2 + 12]
    assert np.array_equal(R.unpack(rows), b)


def test_walsh_spectrum_reconstructs_sbox():
    W = walsh_sbox()
    x = np.arange(256)

    def mono(m, v):
        out = np.ones_like(v)
        for k in range(4):
            if (m >> k) & 1:
                out = out * (1 - 2 * ((v >> k) & 1))
        return out
    for t in range(8):
        f = sum(W[t, s, u] * mono(s, x >> 4) * mono(u, x & 15) for s in range(16) for u in range(16))
        np.testing.assert_allclose(f, 1 - 2 * ((T.SBOX[x].astype(int) >> t) & 1), atol=1e-12)


def test_row_round_stages_oracle(oracle_lib):
    e, R = _setup(oracle_lib, 10)
    rng = np.random.default_rng(1)
    blocks = rng.integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
    rk = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))[1]
    st = R.encrypt_blocks(blocks)
    assert np.array_equal(R.decrypt_blocks(st), blocks)
    sr = R.shift_rows(st)
    ref = T.shift_rows(blocks)
    assert np.array_equal(R.decrypt_blocks(sr), ref)
    mono = R.monomials(sr[1][0:4])
    vals = {m: np.real(e.decrypt(c, R.sk)) for m, c in mono.items()}
    assert max(30 - c.level for c in mono.values()) == 2
    assert np.allclose(vals[0b1111], vals[1] * vals[2] * vals[4] * vals[8], atol=1e-6)
    A = R.sub_bytes(sr)
    ref = T.sub_bytes(ref)
    assert np.array_equal(R.decrypt_blocks(A), ref)
    M = R.mix_columns(A)
    ref = T.mix_columns(ref)
    assert np.array_equal(R.decrypt_blocks(M), ref)
    assert 30 - M[0][0].level == 4 + 3          # SubBytes 4, MixColumns 3
    K = R.add_round_key(M, R.encrypt_round_key(rk))
    assert np.array_equal(R.decrypt_blocks(K), T.aes_round(blocks, rk))
    KM = R.mix_columns_add_round_key(A, R.encrypt_round_key(rk))
    assert np.array_equal(R.decrypt_blocks(KM), T.aes_round(blocks, rk))
    assert 30 - KM[0][0].level == 7              # depth per round


def test_four_chained_rounds_oracle(oracle_lib):
    e, R = _setup(oracle_lib, 10, seed=8)
    rng = np.random.default_rng(2)
    blocks = rng.integers(0, 256, (1, R.n_blk, 16), dtype=np.uint8)
    rks = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = R.encrypt_blocks(blocks)
    ref = blocks
    for r in (1, 2, 3, 4):
        st = R.round(st, R.encrypt_round_key(rks[r]))
        ref = T.aes_round(ref, rks[r])
        assert np.array_equal(R.decrypt_blocks(st), ref)
    assert st[0][0].level == 2


@pytest.mark.gpu
def test_row_round_bit_exact_vs_oracle(product_lib, oracle_lib, gpu_available):
    outs = []
    for lib in (product_lib, oracle_lib):
        e, R = _setup(lib, 12, seed=21)
        rng = np.random.default_rng(3)
        blocks = rng.integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
        rk = rng.integers(0, 256, 16, dtype=np.uint8)
        st = R.round(R.encrypt_blocks(blocks), R.encrypt_round_key(rk))
        outs.append((e, st))
        assert np.array_equal(R.decrypt_blocks(st), T.aes_round(blocks, rk))
    (g, sg), (o, so) = outs
    for rg, ro in zip(sg, so):
        for cg, co in zip(rg, ro):
            assert np.array_equal(g.export_residues(cg), o.export_residues(co))


@pytest.mark.gpu
def test_row_round_full_params(product_lib, gpu_available):
    e, R = _setup(product_lib, 16, seed=4)
    assert e._lib.backend == "hip-gfx950"
    rng = np.random.default_rng(4)
    blocks = rng.integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
    rks = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = R.encrypt_blocks(blocks)
    ref = blocks
    for r in (1, 2, 3, 4):                        # four rounds inside one 30-level budget
        st = R.round(st, R.encrypt_round_key(rks[r]))
        ref = T.aes_round(ref, rks[r])
        assert np.array_equal(R.decrypt_blocks(st), ref)


# ---- fully sliced layout (AESSlicedRound: the columns as batch elements) ----------------------
def test_sliced_layout_roundtrip():
    R = AESSlicedRound.__new__(AESSlicedRound)
    R.sc, R.n_blk = 64, 16
    for nb in (1, 3, 4, 6):
        b = np.random.default_rng(nb).integers(0, 256, (nb, 16, 16), dtype=np.uint8)
        rows = R.pack(b)
        assert rows[0].shape == (4 * R.slabs(nb), 64)
        # element 4 s + c, slot k: byte r + 4c of block k of slab s (sets 4s .. 4s + 3 in order)
        if nb > 1:
            assert rows[2][4 * 0 + 3, 16 + 5] == b[1, 5, 2 + 12]
        assert np.array_equal(R.unpack(rows, nb), b)


def test_sliced_round_stages_oracle(oracle_lib):
    """ShiftRows as a batch permutation (aesfhe_ct_gather), the batch-4 round key repeated over
    the slabs, over an odd number of sets (the last slab padded)."""
    e, R = _setup(oracle_lib, 10, cls=AESSlicedRound)
    rng = np.random.default_rng(11)
    blocks = rng.integers(0, 256, (5, R.n_blk, 16), dtype=np.uint8)
    rk = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))[1]
    st = R.encrypt_blocks(blocks)
    assert st[0][0].batch == 8
    assert np.array_equal(R.decrypt_blocks(st, 5), blocks)
    sr = R.shift_rows(st)
    assert all(c.level == 30 for row in sr for c in row)  # no key switch, no level
    ref = T.shift_rows(blocks)
    assert np.array_equal(R.decrypt_blocks(sr, 5), ref)
    A = R.sub_bytes(st)
    assert np.array_equal(R.decrypt_blocks(R.shift_rows(A), 5), T.sub_bytes(ref))
    key = R.encrypt_round_key(rk)
    assert key[0][0].batch == 4
    KM = R.mix_columns_add_round_key(R.shift_rows(A), key)
    assert np.array_equal(R.decrypt_blocks(KM, 5), T.aes_round(blocks, rk))
    assert 30 - KM[0][0].level == 7
    K = R.add_round_key(st, key)
    assert np.array_equal(R.decrypt_blocks(K, 5), blocks ^ rk[None, None, :])


def test_sliced_four_chained_rounds_oracle(oracle_lib):
    e, R = _setup(oracle_lib, 10, seed=8, cls=AESSlicedRound)
    rng = np.random.default_rng(2)
    blocks = rng.integers(0, 256, (4, R.n_blk, 16), dtype=np.uint8)
    rks = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = R.encrypt_blocks(blocks)
    ref = blocks
    for r in (1, 2, 3, 4):
        st = R.round(st, R.encrypt_round_key(rks[r]))
        ref = T.aes_round(ref, rks[r])
        assert np.array_equal(R.decrypt_blocks(st, 4), ref)
    assert st[0][0].level == 2


def test_gather_oracle(oracle_lib):
    """aesfhe_ct_gather: element b of the result is element idx[b] (permutation, repetition)."""
    e = Engine(log_n=10, max_level=3, special_primes=2, seed=1, _lib=oracle_lib)
    sk = e.create_secret_key()
    pk = e.create_public_key(sk)
    v = np.random.default_rng(0).standard_normal((3, e.slot_count))
    ct = e.encrypt(v, pk)
    res = e.export_residues(ct)
    for idx in ([2, 0, 1], [1, 1, 1, 1, 0], [0]):
        g = e.gather(ct, idx)
        assert g.batch == len(idx) and g.level == ct.level
        assert np.array_equal(e.export_residues(g), res[idx])
    with pytest.raises(RuntimeError):
        e.gather(ct, [3])


@pytest.mark.gpu
def test_gather_gpu(product_lib, oracle_lib, gpu_available):
    outs = []
    for lib in (product_lib, oracle_lib):
        e = Engine(log_n=16, max_level=6, special_primes=2, seed=9, _lib=lib)
        sk = e.create_secret_key()
        ct = e.encrypt(np.random.default_rng(1).standard_normal((4, e.slot_count)), e.create_public_key(sk))
        outs.append(e.export_residues(e.gather(ct, [3, 1, 1, 0, 2, 3, 3])))
    assert np.array_equal(outs[0], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [{}, dict(special_primes=10, digit_primes=12, scale_bits=40)], ids=["K8", "K10A12"])
def test_sliced_round_bit_exact_vs_oracle(product_lib, oracle_lib, gpu_available, kw):
    outs = []
    for lib in (product_lib, oracle_lib):
        e, R = _setup(lib, 12, seed=21, cls=AESSlicedRound, **kw)
        rng = np.random.default_rng(3)
        blocks = rng.integers(0, 256, (6, R.n_blk, 16), dtype=np.uint8)
        rk = rng.integers(0, 256, 16, dtype=np.uint8)
        st = R.round(R.encrypt_blocks(blocks), R.encrypt_round_key(rk))
        outs.append((e, st))
        assert np.array_equal(R.decrypt_blocks(st, 6), T.aes_round(blocks, rk))
    (g, sg), (o, so) = outs
    for rg, ro in zip(sg, so):
        for cg, co in zip(rg, ro):
            assert np.array_equal(g.export_residues(cg), o.export_residues(co))


@pytest.mark.gpu
def test_sliced_round_full_params(product_lib, gpu_available):
    e, R = _setup(product_lib, 16, seed=4, cls=AESSlicedRound)
    assert e._lib.backend == "hip-gfx950"
    rng = np.random.default_rng(4)
    blocks = rng.integers(0, 256, (8, R.n_blk, 16), dtype=np.uint8)
    rks = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = R.encrypt_blocks(blocks)
    ref = blocks
    for r in (1, 2, 3, 4):                        # four rounds inside one 30-level budget
        st = R.round(st, R.encrypt_round_key(rks[r]))
        ref = T.aes_round(ref, rks[r])
        assert np.array_equal(R.decrypt_blocks(st, 8), ref)


def test_sub_bytes_shift_rows_oracle(oracle_lib):
    """ShiftRows folded into the S-box's output order (aesfhe_poly2_int_rot) gives residue for
    residue what SubBytes followed by the ShiftRows gather gives (the rotation commutes with the
    batch-elementwise relinearisation)."""
    e, R = _setup(oracle_lib, 10, seed=9, cls=AESSlicedRound)
    rng = np.random.default_rng(14)
    blocks = rng.integers(0, 256, (8, R.n_blk, 16), dtype=np.uint8)
    st = R.encrypt_blocks(blocks)
    fused = R.sub_bytes_shift_rows(st)
    ref = R.shift_rows(R.sub_bytes(st))
    for rf, rr in zip(fused, ref):
        for cf, cr in zip(rf, rr):
            assert np.array_equal(e.export_residues(cf), e.export_residues(cr))
    assert np.array_equal(R.decrypt_blocks(fused, 8), T.shift_rows(T.sub_bytes(blocks)))
    with pytest.raises(RuntimeError, match="whole slabs"):
        odd = e.encrypt(np.ones((3, e.slot_count)), R.pk)
        e.poly2_int([odd], [odd], np.ones((1, 2, 2)), 64, R.rlk, slab_rot=1)
