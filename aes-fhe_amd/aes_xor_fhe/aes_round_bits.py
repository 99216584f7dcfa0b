"""Row-sliced, bit-domain homomorphic AES-128 round (the fast path of the bench).

Same primitive kinds as the reference's services (Zeta-16 nibble LUT polynomials as in
xor_service.py:245-286 / sbox_service.py:116-138, slot rotations as in shiftrows_service.py:
33-51), arranged so that the expensive operations disappear:

* layout -- one ciphertext per state row r and nibble: slot = c * n_blk + block with
  n_blk = slot_count / 4 (8192 blocks at N = 2^16).  ShiftRows (out(r,c) = in(r, c+r)) is then a
  single whole-ciphertext rotation of row r by -r*n_blk slots, with no masks; as it commutes
  with SubBytes it is applied to the nibble inputs (6 rotations per 8192 blocks).
* SubBytes -- from the Zeta-16 nibble pair (h, l) straight to the 8 output bits in the +-1
  encoding B_j = (-1)^{bit_j}: eight 2-D LUT polynomials sharing the power bases of h and l
  (one fused Engine.poly2 call: inner sums never rescaled, one relinearisation per bit).
* MixColumns -- in the +-1 encoding XOR is multiplication.  With a_r the SubBytes bytes of row
  r: out_r = xtime(a_r ^ a_{r+1}) ^ a_r ^ t, t = a_0 ^ a_1 ^ a_2 ^ a_3.  Per bit j:
  U_rj = A_rj A_{r+1,j}; T_j = U_0j U_2j; xtime(u)_j = u_{j-1} (j = 0: u_7), times u_7 for
  j in {1, 3, 4}; OUT_rj = (A_rj T_j) XT_rj.  116 products, depth 4.
* AddRoundKey -- 32 products with the encrypted key bits (B = 1, broadcast), depth 1.
* back to nibbles -- Zeta16^h = prod_k (alpha_k + beta_k B_{4+k}) with alpha = (1 + zeta^{2^k})/2,
  beta = (1 - zeta^{2^k})/2: one product per bit pair, one linear combination, one product,
  depth 3 (same for the low nibble).
Round depth 5 + 4 + 1 + 3 = 13 (two rounds per 30-level budget); about 322 key switches per
8192 blocks against ~960 for the byte-major nibble-domain round (aes_round.py).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import aes_tables as T
from .coeffs_gen import lut_2d
from .fhe import Ciphertext, Engine

ZETA16 = np.exp(-2j * np.pi / 16)
XT_OF = {0: (7, False), 1: (0, True), 2: (1, False), 3: (2, True), 4: (3, True), 5: (4, False),
         6: (5, False), 7: (6, False)}  # xtime bit j = u[src] (* u[7] if flagged)



class AESRowRound:
    def __init__(self, engine: Engine, sk, pk, rlk, cjk, rotation_keys=None):
        self.e = engine
        self.sk, self.pk, self.rlk, self.cjk = sk, pk, rlk, cjk
        self.sc = engine.slot_count
        self.n_blk = self.sc // 4
        # SubBytes output bits as +-1 values: (-1)^{bit_j(S(16h + l))} = zeta_2^{bit}
        self.C_bits = [lut_2d(lambda h, l, j=j: (int(T.SBOX[16 * h + l]) >> j) & 1, 16, out_mod=2)
                       for j in range(8)]
        # bits -> Zeta-16 nibble: factor k maps B = (-1)^x to zeta^{2^k x}
        self.alpha = [(1 + ZETA16 ** (1 << k)) / 2 for k in range(4)]
        self.beta = [(1 - ZETA16 ** (1 << k)) / 2 for k in range(4)]
        if rotation_keys is None:
            rotation_keys = {r: engine.create_fixed_rotation_key(sk, -r * self.n_blk) for r in (1, 2, 3)}
        self.rot_keys = rotation_keys

    # ---- layout -----------------------------------------------------------------------------
    def pack(self, blocks: np.ndarray) -> List[np.ndarray]:
        """(NB, n_blk, 16) bytes -> 4 row arrays (NB, slot_count): slot c*n_blk + blk holds byte
        r + 4c (FIPS order) of block blk."""
        b = np.asarray(blocks, dtype=np.uint8)
        return [np.ascontiguousarray(b[:, :, [r + 4 * c for c in range(4)]].transpose(0, 2, 1)).reshape(b.shape[0], self.sc)
                for r in range(4)]

    def unpack(self, rows: Sequence[np.ndarray]) -> np.ndarray:
        nb = rows[0].shape[0]
        out = np.empty((nb, self.n_blk, 16), dtype=np.uint8)
        for r in range(4):
            v = np.asarray(rows[r], dtype=np.uint8).reshape(nb, 4, self.n_blk)
            for c in range(4):
                out[:, :, r + 4 * c] = v[:, c, :]
        return out

    def encrypt_blocks(self, blocks: np.ndarray) -> List[Tuple[Ciphertext, Ciphertext]]:
        out = []
        for row in self.pack(blocks):
            s = row.astype(np.int64)
            out.append((self.e.encrypt(ZETA16 ** (s >> 4), self.pk),
                        self.e.encrypt(ZETA16 ** (s & 15), self.pk)))
        return out

    def _dec16(self, ct):
        z = np.atleast_2d(self.e.decrypt(ct, self.sk))
        return np.mod(np.rint(-np.angle(z) * 16 / (2 * np.pi)), 16).astype(np.uint8)

    def decrypt_blocks(self, rows: Sequence[Tuple[Ciphertext, Ciphertext]]) -> np.ndarray:
        return self.unpack([(self._dec16(h) << 4) | self._dec16(l) for h, l in rows])

    def decrypt_bits(self, bits: Sequence[Sequence[Ciphertext]]) -> np.ndarray:
        """4 rows x 8 bit ciphertexts (+-1) -> blocks (debug / tests)."""
        rows = []
        for r in range(4):
            acc = 0
            for j in range(8):
                v = np.real(np.atleast_2d(self.e.decrypt(bits[r][j], self.sk)))
                acc = acc | ((v < 0).astype(np.uint8) << j)
            rows.append(acc)
        return self.unpack(rows)

    def encrypt_round_key(self, rk: np.ndarray, level: int | None = None) -> List[List[Ciphertext]]:
        """Key bits as +-1 per row (B = 1, broadcast over the batch)."""
        rk = np.asarray(rk, dtype=np.int64)
        keys = []
        for r in range(4):
            row = np.repeat(rk[[r + 4 * c for c in range(4)]], self.n_blk)
            keys.append([self.e.encrypt(1.0 - 2.0 * ((row >> j) & 1), self.pk, level=level)
                         for j in range(8)])
        return keys

    # ---- building blocks ---------------------------------------------------------------------
    def full_basis(self, x: Ciphertext) -> Dict[int, Ciphertext]:
        e = self.e
        pw = e.make_power_basis(x, 8, self.rlk)
        b = {k + 1: c for k, c in enumerate(pw)}
        for k in range(9, 16):
            b[k] = e.conjugate(b[16 - k], self.cjk)
        keys = sorted(b)
        return dict(zip(keys, e.align([b[k] for k in keys])))

    def mul(self, a: Ciphertext, b: Ciphertext) -> Ciphertext:
        return self.e.multiply(a, b, self.rlk)

    def lut2_bits(self, hb, lb) -> List[Ciphertext]:
        """The 8 S-box output bits from the power bases of h and l in one fused bivariate
        evaluation (Engine.poly2): out_j = sum_{i,k} C_j[i,k] h^i l^k."""
        C = np.stack(self.C_bits)
        return self.e.poly2([hb[k] for k in range(1, 16)], [lb[k] for k in range(1, 16)], C, self.rlk)

    # ---- round steps ---------------------------------------------------------------------------
    def shift_rows(self, rows):
        out = [rows[0]]
        for r in (1, 2, 3):
            h, l = rows[r]
            out.append((self.e.rotate(h, self.rot_keys[r]), self.e.rotate(l, self.rot_keys[r])))
        return out

    def sub_bytes_bits(self, rows) -> List[List[Ciphertext]]:
        return [self.lut2_bits(self.full_basis(h), self.full_basis(l)) for h, l in rows]

    def mix_columns_bits(self, A: List[List[Ciphertext]]) -> List[List[Ciphertext]]:
        U = [[self.mul(A[r][j], A[(r + 1) % 4][j]) for j in range(8)] for r in range(4)]
        Tt = [self.mul(U[0][j], U[2][j]) for j in range(8)]
        out = []
        for r in range(4):
            row = []
            for j in range(8):
                src, carry = XT_OF[j]
                xt = self.mul(U[r][src], U[r][7]) if carry else U[r][src]
                row.append(self.mul(self.mul(A[r][j], Tt[j]), xt))
            out.append(row)
        return out

    def add_round_key_bits(self, S: List[List[Ciphertext]], key) -> List[List[Ciphertext]]:
        return [[self.mul(S[r][j], key[r][j]) for j in range(8)] for r in range(4)]

    def to_nibbles(self, bits: Sequence[Ciphertext]) -> Tuple[Ciphertext, Ciphertext]:
        """8 +-1 bit ciphertexts of one row -> (Zeta16^hi, Zeta16^lo)."""
        e = self.e
        outs = []
        for base in (4, 0):
            pairs = []
            for k0 in (0, 2):
                b0, b1 = bits[base + k0], bits[base + k0 + 1]
                a0, be0 = self.alpha[k0], self.beta[k0]
                a1, be1 = self.alpha[k0 + 1], self.beta[k0 + 1]
                p = e.lincomb([b0, b1, self.mul(b0, b1)], [be0 * a1, a0 * be1, be0 * be1])
                pairs.append(e.add(p, complex(a0 * a1)))
            outs.append(self.mul(pairs[0], pairs[1]))
        return outs[0], outs[1]

    def round(self, rows, key, timings: dict | None = None):
        """ShiftRows -> SubBytes -> MixColumns -> AddRoundKey on the row-sliced state;
        input and output are 4 (hi, lo) Zeta-16 nibble ciphertext pairs."""
        import time

        def mark(name, t0):
            if timings is None:
                return t0
            self.e.synchronize()
            t1 = time.perf_counter()
            timings[name] = timings.get(name, 0.0) + (t1 - t0)
            return t1
        t = mark("start", 0.0) if timings is not None else 0.0
        rows = self.shift_rows(rows)
        t = mark("shift_rows", t)
        A = self.sub_bytes_bits(rows)
        t = mark("sub_bytes", t)
        M = self.mix_columns_bits(A)
        t = mark("mix_columns", t)
        K = self.add_round_key_bits(M, key)
        t = mark("add_round_key", t)
        out = [self.to_nibbles(K[r]) for r in range(4)]
        mark("to_nibbles", t)
        return out
