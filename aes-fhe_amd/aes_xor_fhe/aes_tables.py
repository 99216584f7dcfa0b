"""AES-128 constants and a plaintext FIPS-197 reference, derived from the field definition.

Nothing here is transcribed: the S-box is computed as the GF(2^8) inverse followed by the
FIPS-197 affine map, xtime / GF multiplications from the AES polynomial x^8+x^4+x^3+x+1.
tests/test_aes_tables.py checks them against FIPS-197 Appendix B/C known answers and against
the tables the reference ships (sbox/sbox_service.py:31-49,
generator/generate_gf2_gf3_coeffs.py:8-44).

Byte order: a 16-byte block maps to the 4x4 state column-major (FIPS-197 3.4), i.e. byte
index i = r + 4c -- the same convention as the reference's utils.bytes_to_state (utils.py:11-26).
"""
from __future__ import annotations

import numpy as np

AES_POLY = 0x11B


def gf_mul(a: int, b: int) -> int:
    """Multiply in GF(2^8) modulo the AES polynomial."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= AES_POLY
        b >>= 1
    return r


def xtime(a: int) -> int:
    return gf_mul(a, 2)


def _gf_inv(a: int) -> int:
    if a == 0:
        return 0
    r = 1
    for _ in range(254):  # a^254 = a^{-1}
        r = gf_mul(r, a)
    return r


def _affine(x: int) -> int:
    y = 0
    for i in range(8):
        bit = ((x >> i) ^ (x >> ((i + 4) % 8)) ^ (x >> ((i + 5) % 8)) ^ (x >> ((i + 6) % 8))
               ^ (x >> ((i + 7) % 8)) ^ (0x63 >> i)) & 1
        y |= bit << i
    return y


SBOX = np.array([_affine(_gf_inv(x)) for x in range(256)], dtype=np.uint8)
INV_SBOX = np.zeros(256, dtype=np.uint8)
INV_SBOX[SBOX] = np.arange(256, dtype=np.uint8)
AES_SBOX = [int(v) for v in SBOX]          # list form, as the reference exposes it
GF_MUL_TABLES = {k: np.array([gf_mul(x, k) for x in range(256)], dtype=np.uint8)
                 for k in (1, 2, 3, 9, 11, 13, 14)}
GF2 = GF_MUL_TABLES[2]
GF3 = GF_MUL_TABLES[3]

RCON = [0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1B, 0x36]


# ---------------------------------------------------------------------------------------------
# plaintext AES-128 on a (..., 16) byte array in FIPS byte order (index r + 4c)
def sub_bytes(s: np.ndarray) -> np.ndarray:
    return SBOX[s]


def shift_rows(s: np.ndarray) -> np.ndarray:
    """out(r, c) = in(r, c + r mod 4)."""
    idx = np.array([(r + 4 * ((c + r) % 4)) for c in range(4) for r in range(4)])
    # position r + 4c of the output takes input index idx[r + 4c]
    return s[..., idx]


def inv_shift_rows(s: np.ndarray) -> np.ndarray:
    idx = np.array([(r + 4 * ((c - r) % 4)) for c in range(4) for r in range(4)])
    return s[..., idx]


def mix_columns(s: np.ndarray) -> np.ndarray:
    out = np.empty_like(s)
    for c in range(4):
        a = [s[..., r + 4 * c] for r in range(4)]
        for r in range(4):
            out[..., r + 4 * c] = (GF2[a[r]] ^ GF3[a[(r + 1) % 4]] ^ a[(r + 2) % 4]
                                   ^ a[(r + 3) % 4])
    return out


def inv_mix_columns(s: np.ndarray) -> np.ndarray:
    m = GF_MUL_TABLES
    out = np.empty_like(s)
    for c in range(4):
        a = [s[..., r + 4 * c] for r in range(4)]
        for r in range(4):
            out[..., r + 4 * c] = (m[14][a[r]] ^ m[11][a[(r + 1) % 4]] ^ m[13][a[(r + 2) % 4]]
                                   ^ m[9][a[(r + 3) % 4]])
    return out


def expand_key(key: bytes | np.ndarray) -> np.ndarray:
    """FIPS-197 5.2 key expansion: 16-byte key -> (11, 16) round keys (the reference's
    key_expansion.py is empty; the harness does this step in plaintext)."""
    k = np.asarray(bytearray(key) if isinstance(key, (bytes, bytearray)) else key, dtype=np.uint8)
    w = [list(k[4 * i:4 * i + 4]) for i in range(4)]
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = t[1:] + t[:1]
            t = [int(SBOX[b]) for b in t]
            t[0] ^= RCON[i // 4 - 1]
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    return np.array([sum(w[4 * r:4 * r + 4], []) for r in range(11)], dtype=np.uint8)


def encrypt_block(block: np.ndarray, key: bytes | np.ndarray, rounds: int = 10) -> np.ndarray:
    rk = expand_key(key)
    s = np.asarray(block, dtype=np.uint8) ^ rk[0]
    for r in range(1, rounds + 1):
        s = shift_rows(sub_bytes(s))
        if r != 10:
            s = mix_columns(s)
        s = s ^ rk[r]
    return s


def aes_round(state: np.ndarray, round_key: np.ndarray) -> np.ndarray:
    """One full middle round: SubBytes -> ShiftRows -> MixColumns -> AddRoundKey."""
    return mix_columns(shift_rows(sub_bytes(state))) ^ round_key
