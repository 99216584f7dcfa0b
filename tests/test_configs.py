"""BASELINE.json configs 1, 4 and 5 at their own parameters.

Config 1 -- "Single AES round, 1 ciphertext, N=2^14, L=8, CPU engine_context (test_total.py
plumbing)": the reference's AddRoundKey driver (test_all_process.py:12-48: EngineContext ->
EngineWrapper -> XORService -> AESFHERound.full_round, seeds 25073101 / 25073102) at N = 2^14,
L = 8 (the 128-bit budget of N = 2^14 leaves K = 1 special prime), checked against the reference's
own decoded output for those seeds (tests/golden/golden.npz "ark16_*", made by
tests/golden/make_golden.py) and against state ^ key on a full 8192-byte ciphertext; on the CPU
oracle and on the HIP engine (residue-identical to each other).

Config 5 -- "Full AES-128 10 rounds, N=2^17, L=35, batch=512 ciphertexts over 8 GPUs": one
rank's shard runs on one GPU.  Bit-exact ct x ct multiply + rotation against the oracle at
N = 2^17, L = 35, and full AES-128 (ARK0 + 10 rounds with bit-mode bootstrapping) at those
parameters, FIPS-197 verified (C.1 vector in block 0).

Config 4 -- "Full AES-128 10 rounds end-to-end, N=2^16, L=30, batch=64 ciphertexts": the whole
131 072-block batch at the bench's parameters, FIPS-197 verified block by block.
"""
from pathlib import Path

import numpy as np
import pytest

from aes_xor_fhe import aes_tables as T
from aes_xor_fhe.engine_context import EngineContext
from aes_xor_fhe.new import AESFHERound
from aes_xor_fhe.xor_service import EngineWrapper, XORConfig, XORService

GOLD = np.load(Path(__file__).resolve().parent / "golden" / "golden.npz")
CONFIG1 = dict(log_n=14, special_primes=1)


def _config1(lib, seed=25073101):
    ctx = EngineContext(signature=2, max_level=8, seed=seed, _lib=lib, **CONFIG1)
    e = ctx.engine
    assert (e.log_coeff_count, e.max_level, e.slot_count) == (14, 8, 8192)
    wrap = EngineWrapper(XORConfig(max_level=8), ctx=ctx)
    ark = AESFHERound(wrap, XORService(wrap))
    out16 = ark.full_round(GOLD["ark16_state"], GOLD["ark16_key"], recombine=True)
    assert np.array_equal(out16, GOLD["ark16_out"])
    assert np.array_equal(out16, GOLD["ark16_state"] ^ GOLD["ark16_key"])
    rng = np.random.default_rng(25073102)
    st, ky = (rng.integers(0, 256, 8192, dtype=np.uint8) for _ in range(2))
    hi, lo = ark.full_round(st, ky, recombine=False)
    assert min(hi.level, lo.level) >= 0
    from aes_xor_fhe.new import decrypt_and_recombine
    assert np.array_equal(decrypt_and_recombine(hi, lo, wrap, length=8192), st ^ ky)
    return e.export_residues(hi)


def test_config1_ark_oracle(oracle_lib):
    _config1(oracle_lib)


@pytest.mark.gpu
def test_config1_ark_gpu_matches_oracle(product_lib, oracle_lib, gpu_available):
    assert np.array_equal(_config1(product_lib), _config1(oracle_lib))


# 44-bit scale: the 128-bit budget of N = 2^17 (log QP <= 3544) leaves room (50 + 35 * 44 + 12 * 50 =
# 2190), and at a 40-bit scale the slot error after a round was ~2x N = 2^16's (aes10_diag.py)
CONFIG5 = dict(log_n=17, max_level=35, special_primes=12, scale_bits=44)


@pytest.mark.gpu
def test_config5_mul_rotate_bit_exact(product_lib, oracle_lib, gpu_available):
    from aes_xor_fhe.fhe import Engine
    g = Engine(_lib=product_lib, seed=5, **CONFIG5)
    o = Engine(_lib=oracle_lib, seed=5, thread_count=8, **CONFIG5)
    assert g.primes == o.primes and g.slot_count == 65536
    res = []
    z = np.exp(-2j * np.pi * np.random.default_rng(3).integers(0, 256, g.slot_count) / 256)
    for e in (g, o):
        sk = e.create_secret_key(7)
        ct = e.encrypt(z, e.create_public_key(sk))
        m = e.multiply(ct, ct, e.create_relinearization_key(sk))
        r = e.rotate(m, e.create_fixed_rotation_key(sk, -4096), -4096)
        res.append((e.export_residues(m), e.export_residues(r)))
        if e is g:
            np.testing.assert_allclose(e.decrypt(r, sk), np.roll(z * z, -4096), atol=1e-5)
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])


@pytest.mark.gpu
def test_config5_aes128_ten_rounds(product_lib, gpu_available):
    from aes_xor_fhe.aes_round_bits import AESRowRound
    from aes_xor_fhe.bootstrap import Bootstrapper
    from aes_xor_fhe.fhe import Engine
    e = Engine(_lib=product_lib, seed=17, **CONFIG5)
    sk = e.create_secret_key()
    rlk = e.create_relinearization_key(sk)
    R = AESRowRound(e, sk, e.create_public_key(sk), rlk)
    assert R.n_blk == 16384
    bs = Bootstrapper(e, sk, rlk)
    key = np.arange(16, dtype=np.uint8)
    blocks = np.random.default_rng(5).integers(0, 256, (1, R.n_blk, 16), dtype=np.uint8)
    blocks[0, 0] = np.frombuffer(bytes.fromhex("00112233445566778899aabbccddeeff"), np.uint8)
    st = R.encrypt_blocks(blocks)
    one = R.round(st, R.encrypt_round_key(T.expand_key(key)[1]))       # one middle round
    assert np.array_equal(R.decrypt_blocks(one), T.aes_round(blocks, T.expand_key(key)[1]))
    out, nref = R.encrypt_aes128(st, [R.encrypt_round_key(k) for k in T.expand_key(key)], bs)
    got = R.decrypt_blocks(out)
    want = T.encrypt_block(blocks, key)  # vectorised over (..., 16)
    assert np.array_equal(got, want)
    assert bytes(got[0, 0]) == bytes.fromhex("69c4e0d86a7b0430d8cdb78070b4c55a")


@pytest.mark.gpu
def test_config5_sliced_round(product_lib, gpu_available):
    """Config 5's shard in the bench's layout (the config5_shard leg): the fully sliced state at
    N = 2^17, L = 35, K = 12 with the widest key-switch digits, one slab of 4 sets (65 536 blocks)
    through a middle round from the top level, FIPS-197 for every block."""
    from aes_xor_fhe.aes_round_bits import AESSlicedRound
    from aes_xor_fhe.fhe import Engine, widest_digits
    e = Engine(_lib=product_lib, seed=29, digit_primes=widest_digits(**CONFIG5, lib=product_lib), **CONFIG5)
    sk = e.create_secret_key()
    R = AESSlicedRound(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk))
    assert R.n_blk == 16384
    blocks = np.random.default_rng(31).integers(0, 256, (4, R.n_blk, 16), dtype=np.uint8)
    rk = np.random.default_rng(32).integers(0, 256, 16, dtype=np.uint8)
    out = R.round(R.encrypt_blocks(blocks), R.encrypt_round_key(rk))
    assert out[0][0].level == 35 - 7
    assert np.array_equal(R.decrypt_blocks(out, 4), T.aes_round(blocks, rk))


# config 4 at the bench's parameters (bench.py defaults: scale 40, K = 10)
CONFIG4 = dict(log_n=16, max_level=30, special_primes=10, scale_bits=40)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [23, 29])
def test_config4_full_batch_ten_rounds(product_lib, gpu_available, seed):
    """Config 4 -- "Full AES-128 10 rounds end-to-end, N=2^16, L=30, batch=64 ciphertexts" -- in
    exactly the shape bench.py's aes128_10_rounds leg times: the whole batch (64 reference
    ciphertexts of 2048 blocks = 16 sets of 8192 blocks = 131 072 blocks) in the fully sliced
    state (AESSlicedRound, 4 slabs), 12-prime key-switch digits over K = 10, the state encrypted
    at the fresh level (25) with each round key at the level its product consumes, the 5-map and
    3-map CoeffToSlot bootstrappers picked per refresh, 4 pairs per bootstrap call; every block
    checked against FIPS-197 and every round's input level against the schedule."""
    from aes_xor_fhe.aes_round_bits import AESSlicedRound
    from aes_xor_fhe.bootstrap import Bootstrapper, trim_bootstrap_keys
    from aes_xor_fhe.fhe import Engine, widest_digits
    alpha = widest_digits(**CONFIG4, lib=product_lib)
    assert alpha == 12
    e = Engine(_lib=product_lib, seed=seed, digit_primes=alpha, **CONFIG4)
    sk = e.create_secret_key()
    rlk = e.create_relinearization_key(sk)
    R = AESSlicedRound(e, sk, e.create_public_key(sk), rlk)
    bs5 = Bootstrapper(e, sk, rlk, cts_groups=5)
    bs = [bs5, Bootstrapper(e, sk, rlk, cts_groups=3, share=bs5)]  # as bench.py builds them
    trim_bootstrap_keys(bs)
    L0 = R.fresh_level(e.max_level, bs)
    klv = R.key_levels(L0, bs)
    assert L0 == 25
    key = np.random.default_rng(4).integers(0, 256, 16, dtype=np.uint8)
    blocks = np.random.default_rng(seed - 17).integers(0, 256, (16, R.n_blk, 16), dtype=np.uint8)
    assert blocks.shape[0] * R.n_blk == 64 * 2048
    keys = [R.encrypt_round_key(k, level=lv) for k, lv in zip(T.expand_key(key), klv)]
    tm = {}
    refresh_in = []
    out, nref = R.encrypt_aes128(R.encrypt_blocks(blocks, level=L0), keys, bs, timings=tm,
                                 pairs_per_call=4, consume=True,
                                 probe=lambda rnd, S, sc: refresh_in.append(R.bit_margin(S, sc)))
    assert nref == 3
    assert [lv for _, lv, _ in tm["per_round"]] == [lv for _, lv, _ in R.schedule(L0, bs)]
    want = T.encrypt_block(blocks, key)  # vectorised over (..., 16)
    assert np.array_equal(R.decrypt_blocks(out, 16), want)
    # the decision margin left by the final round (bits cleaned before the last refresh,
    # AESRowRound.clean_bits): max | |v| - 1 | measured 0.03; 0.7-0.8 without the cleaning (a
    # wrong block in ~1 of 7 runs).  bit_margin decrypts on the device; the host
    # decryption of one ciphertext cross-checks it
    dev = R.bit_margin(out)
    host = float(np.abs(np.abs(np.real(np.atleast_2d(e.decrypt(out[0][0], sk)))) - 1.0).max())
    assert host <= dev + 1e-9
    assert dev < 0.1, dev
    # every refresh input (after the cleaning of the last one) well inside the decision margin
    assert len(refresh_in) == 3 and max(refresh_in) < 0.5, refresh_in
