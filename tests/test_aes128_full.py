"""Full AES-128 (10 rounds, FIPS-197 section 5.1) on the row-sliced bit state with bit-mode
bootstrapping (AESRowRound.encrypt_aes128; BASELINE configs 4-5).

CPU: the oracle engine at N = 2^10 (128 blocks per ciphertext) encrypts random blocks (block 0 =
the FIPS-197 C.1 plaintext) under the C.1 key, checked block by block against aes_tables.encrypt_block (pinned by the FIPS-197
appendix vectors in test_aes_tables.py), and block 0 against the published C.1 ciphertext.
GPU: the same at BASELINE's N = 2^16, L = 30 (8192 blocks per ciphertext)."""
import numpy as np
import pytest

from aes_xor_fhe import aes_tables as T
from aes_xor_fhe.aes_round_bits import AESRowRound, AESSlicedRound
from aes_xor_fhe.bootstrap import Bootstrapper, trim_bootstrap_keys
from aes_xor_fhe.fhe import Engine

SCALE_BITS = 41
FIPS_C1_KEY = bytes(range(16))
FIPS_C1_PT = bytes.fromhex("00112233445566778899aabbccddeeff")
FIPS_C1_CT = bytes.fromhex("69c4e0d86a7b0430d8cdb78070b4c55a")


def _run(lib, log_n, nb=1, seed=3, cls=AESRowRound, cts_groups=(3,), key_levels=False, **kw):
    kw = dict(dict(special_primes=8 if log_n >= 14 else 4, scale_bits=SCALE_BITS), **kw)
    e = Engine(log_n=log_n, max_level=30, seed=seed, _lib=lib, **kw)
    sk = e.create_secret_key(1)
    rlk = e.create_relinearization_key(sk)
    R = cls(e, sk, e.create_public_key(sk), rlk)
    bs = []
    for g in cts_groups:  # later ones share the first's keys and SlotToCoeff plans, as in bench.py
        bs.append(Bootstrapper(e, sk, rlk, cts_groups=g, share=bs[0] if bs else None))
    trim_bootstrap_keys(bs)  # bit refreshes only
    rng = np.random.default_rng(seed)
    key = np.frombuffer(FIPS_C1_KEY, dtype=np.uint8)
    blocks = rng.integers(0, 256, (nb, R.n_blk, 16), dtype=np.uint8)
    blocks[0, 0] = np.frombuffer(FIPS_C1_PT, dtype=np.uint8)
    rks = T.expand_key(key)
    # key_levels: the state encrypted at the lowest level keeping three refreshes and each round
    # key at the level its product consumes (as the bench does)
    L0 = R.fresh_level(e.max_level, bs) if key_levels else None
    lv = R.key_levels(L0, bs) if key_levels else [None] * 11
    keys = [R.encrypt_round_key(rk, level=v) for rk, v in zip(rks, lv)]
    tm = {}
    out, nref = R.encrypt_aes128(R.encrypt_blocks(blocks, level=L0), keys, bs, timings=tm)
    # every round started at the level the precomputed schedule says (so the round keys, encrypted
    # at key_levels, met the state without a level-down): measured, not only planned
    sched = R.schedule(e.max_level if L0 is None else L0, bs)
    assert [lv for _, lv, _ in tm["per_round"]] == [lv for _, lv, _ in sched]
    if key_levels:
        assert L0 == 25 and sched[-1][1] == 5
    got = R.decrypt_blocks(out, nb)
    want = T.encrypt_block(blocks, key)  # vectorised over (..., 16)
    return got, want, nref, out


def test_aes128_fips_vector_plain():
    assert bytes(T.encrypt_block(np.frombuffer(FIPS_C1_PT, np.uint8), FIPS_C1_KEY)) == FIPS_C1_CT


def test_aes128_ten_rounds_oracle(oracle_lib):
    got, want, nref, out = _run(oracle_lib, 10)
    assert nref == 3
    assert np.array_equal(got, want)
    assert bytes(got[0, 0]) == FIPS_C1_CT


@pytest.mark.gpu
def test_aes128_ten_rounds_full_params(product_lib, gpu_available):
    got, want, nref, out = _run(product_lib, 16)
    assert nref == 3 and out[0][0].level == 0
    assert np.array_equal(got, want)
    assert bytes(got[0, 0]) == FIPS_C1_CT


# the bench's ten-round configuration: sliced state, 12-prime key-switch digits over K = 10,
# bootstrappers with 5 and 3 CoeffToSlot maps (the two middle refreshes take the 5-map one,
# output level 17; the last keeps 19 for rounds 8-10)
BENCH10 = dict(cls=AESSlicedRound, cts_groups=(5, 3), special_primes=10, digit_primes=12, scale_bits=40,
               key_levels=True)


def test_aes128_ten_rounds_sliced_two_bootstrappers_oracle(oracle_lib):
    got, want, nref, out = _run(oracle_lib, 10, nb=2, **BENCH10)
    assert nref == 3 and out[0][0].level == 0
    assert np.array_equal(got, want)
    assert bytes(got[0, 0]) == FIPS_C1_CT


@pytest.mark.gpu
def test_aes128_ten_rounds_sliced_full_params(product_lib, gpu_available):
    got, want, nref, out = _run(product_lib, 16, nb=4, **BENCH10)
    assert nref == 3 and out[0][0].level == 0
    assert np.array_equal(got, want)
    assert bytes(got[0, 0]) == FIPS_C1_CT


def test_clean_bits_oracle(oracle_lib):
    """AESRowRound.clean_bits: 3x - x^3 (twice the cleaning map (3x - x^3) / 2) in two levels --
    bits +-1 with a relative error e come back as +-2 with error ~3 e^2 (the refresh after it takes
    in_scale = 2: Bootstrapper.bootstrap_bits)."""
    from aes_xor_fhe.aes_round_bits import AESRowRound
    from aes_xor_fhe.fhe import Engine
    e = Engine(_lib=oracle_lib, log_n=10, max_level=6, special_primes=2, seed=3)
    sk = e.create_secret_key()
    R = AESRowRound(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk))
    rng = np.random.default_rng(5)
    sgn = rng.choice([-1.0, 1.0], size=(1, e.slot_count))
    x = sgn * (1.0 + rng.uniform(-0.05, 0.05, sgn.shape))
    cts = [[e.encrypt(x, sk)]]
    out = R.clean_bits(cts)
    assert out[0][0].level == cts[0][0].level - R.CLEAN_LEVELS
    got = np.real(np.atleast_2d(e.decrypt(out[0][0], sk)))
    np.testing.assert_allclose(got, 3 * x - x ** 3, atol=1e-4)
    assert np.abs(np.abs(got) - 2.0).max() < 3 * 0.05 ** 2 + 1e-3
