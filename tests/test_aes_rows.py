"""Row-sliced bit-domain AES round (aes_xor_fhe.aes_round_bits, the bench's default step).

CPU: the oracle engine runs every stage (ShiftRows, SubBytes -> bits, MixColumns, AddRoundKey,
bits -> nibbles) and two chained rounds, each checked against FIPS-197 (aes_tables, itself
checked against the FIPS-197 appendix vectors in test_aes_tables.py).
GPU: the HIP engine produces residue-identical ciphertexts to the oracle for a full round at
N = 2^12 (bit-exact, integer work), and a correct round at BASELINE.json's N = 2^16, L = 30."""
import numpy as np
import pytest

from aes_xor_fhe import aes_tables as T
from aes_xor_fhe.aes_round_bits import AESRowRound
from aes_xor_fhe.fhe import Engine


def _setup(lib, log_n, seed=5):
    e = Engine(log_n=log_n, max_level=30, special_primes=8, seed=seed, _lib=lib)
    sk = e.create_secret_key(3)
    R = AESRowRound(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk),
                    e.create_conjugation_key(sk))
    return e, R


def test_layout_roundtrip():
    R = AESRowRound.__new__(AESRowRound)
    R.sc, R.n_blk = 64, 16
    b = np.random.default_rng(0).integers(0, 256, (3, 16, 16), dtype=np.uint8)
    rows = R.pack(b)
    assert rows[2][1, 3 * 16 + 5] == b[1, 5, 2 + 12]
    assert np.array_equal(R.unpack(rows), b)


def test_row_round_stages_oracle(oracle_lib):
    e, R = _setup(oracle_lib, 10)
    rng = np.random.default_rng(1)
    blocks = rng.integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
    rk = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))[1]
    st = R.encrypt_blocks(blocks)
    assert np.array_equal(R.decrypt_blocks(st), blocks)
    sr = R.shift_rows(st)
    assert np.array_equal(R.decrypt_blocks(sr), T.shift_rows(blocks))
    A = R.sub_bytes_bits(sr)
    ref = T.sub_bytes(T.shift_rows(blocks))
    assert np.array_equal(R.decrypt_bits(A), ref)
    M = R.mix_columns_bits(A)
    ref = T.mix_columns(ref)
    assert np.array_equal(R.decrypt_bits(M), ref)
    K = R.add_round_key_bits(M, R.encrypt_round_key(rk))
    ref = ref ^ rk
    assert np.array_equal(R.decrypt_bits(K), ref)
    out = [R.to_nibbles(K[r]) for r in range(4)]
    assert np.array_equal(R.decrypt_blocks(out), T.aes_round(blocks, rk))
    assert 30 - out[0][0].level == 13           # depth per round


def test_two_chained_rounds_oracle(oracle_lib):
    e, R = _setup(oracle_lib, 10, seed=8)
    rng = np.random.default_rng(2)
    blocks = rng.integers(0, 256, (1, R.n_blk, 16), dtype=np.uint8)
    rks = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = R.encrypt_blocks(blocks)
    ref = blocks
    for r in (1, 2):
        st = R.round(st, R.encrypt_round_key(rks[r]))
        ref = T.aes_round(ref, rks[r])
        assert np.array_equal(R.decrypt_blocks(st), ref)
    assert st[0][0].level == 4


@pytest.mark.gpu
def test_row_round_bit_exact_vs_oracle(product_lib, oracle_lib, gpu_available):
    outs = []
    for lib in (product_lib, oracle_lib):
        e, R = _setup(lib, 12, seed=21)
        rng = np.random.default_rng(3)
        blocks = rng.integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
        rk = rng.integers(0, 256, 16, dtype=np.uint8)
        st = R.round(R.encrypt_blocks(blocks), R.encrypt_round_key(rk))
        outs.append((e, R, st))
        assert np.array_equal(R.decrypt_blocks(st), T.aes_round(blocks, rk))
    (g, _, sg), (o, _, so) = outs
    for (gh, gl), (oh, ol) in zip(sg, so):
        assert np.array_equal(g.export_residues(gh), o.export_residues(oh))
        assert np.array_equal(g.export_residues(gl), o.export_residues(ol))


@pytest.mark.gpu
def test_row_round_full_params(product_lib, gpu_available):
    e, R = _setup(product_lib, 16, seed=4)
    assert e._lib.backend == "hip-gfx950"
    rng = np.random.default_rng(4)
    blocks = rng.integers(0, 256, (2, R.n_blk, 16), dtype=np.uint8)
    rks = T.expand_key(rng.integers(0, 256, 16, dtype=np.uint8))
    st = R.encrypt_blocks(blocks)
    ref = blocks
    for r in (1, 2):                              # two rounds inside one 30-level budget
        st = R.round(st, R.encrypt_round_key(rks[r]))
        ref = T.aes_round(ref, rks[r])
        assert np.array_equal(R.decrypt_blocks(st), ref)
