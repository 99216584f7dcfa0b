"""Plaintext AES pinned to FIPS-197 (Appendix B round-1 values, Appendix C.1) and to the
reference's own tables (S-box at sbox/sbox_service.py:31-49 via the golden run)."""
from pathlib import Path

import numpy as np

from aes_xor_fhe import aes_tables as T

GOLD = np.load(Path(__file__).resolve().parent / "golden" / "golden.npz")


def h(s):
    return np.frombuffer(bytes.fromhex(s.replace(" ", "")), dtype=np.uint8)


def test_fips197_c1():
    out = T.encrypt_block(h("00112233445566778899aabbccddeeff"), h("000102030405060708090a0b0c0d0e0f"))
    assert bytes(out).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_fips197_appendix_b_round1():
    start = h("19 3d e3 be a0 f4 e2 2b 9a c6 8d 2a e9 f8 48 08")
    sb = T.sub_bytes(start)
    assert bytes(sb).hex() == "d42711aee0bf98f1b8b45de51e415230"
    sr = T.shift_rows(sb)
    assert bytes(sr).hex() == "d4bf5d30e0b452aeb84111f11e2798e5"
    mc = T.mix_columns(sr)
    assert bytes(mc).hex() == "046681e5e0cb199a48f8d37a2806264c"
    rk = T.expand_key(h("2b7e151628aed2a6abf7158809cf4f3c"))
    assert bytes(rk[1]).hex() == "a0fafe1788542cb123a339392a6c7605"
    assert np.array_equal(T.aes_round(start, rk[1]), mc ^ rk[1])
    out = T.encrypt_block(h("3243f6a8885a308d313198a2e0370734"), h("2b7e151628aed2a6abf7158809cf4f3c"))
    assert bytes(out).hex() == "3925841d02dc09fbdc118597196a0b32"


def test_inverses():
    s = np.random.default_rng(0).integers(0, 256, (8, 16), dtype=np.uint8)
    assert np.array_equal(T.inv_shift_rows(T.shift_rows(s)), s)
    assert np.array_equal(T.inv_mix_columns(T.mix_columns(s)), s)
    assert np.array_equal(T.INV_SBOX[T.SBOX], np.arange(256))


def test_sbox_matches_reference_golden():
    # the reference's SubBytes (sbox_service.py:116-138) in exact arithmetic
    assert np.array_equal(GOLD["sbox_out"], T.SBOX[GOLD["sbox_in"]])


def test_gf_tables():
    for x in range(256):
        assert T.GF2[x] == ((x << 1) ^ (0x1B if x & 0x80 else 0)) & 0xFF
        assert T.GF3[x] == T.GF2[x] ^ x
