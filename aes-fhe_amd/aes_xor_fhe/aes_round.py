"""A correct homomorphic AES-128 round on the MI355X CKKS engine (nibble domain, batched).

The reference composes its round from LUT services (xor_service.py:271-286 XOR,
sbox/sbox_service.py:116-138 SubBytes, gf_service.py:55-78 GF LUTs,
shiftrows_service.py:33-51 / shift_mix_zeta.py:14-69 ShiftRows+MixColumns), but its
ShiftRows wraps wrongly and both merged ShiftRows+MixColumns variants are degenerate or
diverge.  This module composes the same primitive kinds -- Zeta-domain LUT
polynomials, 4-bit XOR LUT, plaintext masks and slot rotations -- into a round that is
correct against FIPS-197, within the 30-level budget of BASELINE.json's N = 2^16, L = 30:

  state  : two ciphertexts per batch element, hi and lo nibble of every byte, Zeta-16 encoded
  layout : byte-major -- slot = byte_index * n_blk + block, byte_index = r + 4c (FIPS order);
           one ciphertext pair carries n_blk = slot_count / 16 AES blocks (2048 at N = 2^16)
  round  : SubBytes      2-D LUTs S_hi(h, l), S_lo(h, l)                     depth 5
           ShiftRows +   T_i(r, c) = s(r+i, c+r+i): rotations of S by whole   depth 1
           MixColumns    byte-chunks + target-row masks
                         out = xtime(T0 ^ T1) ^ T1 ^ T2 ^ T3                 depth 15
           AddRoundKey   4-bit XOR with the encrypted round key              depth 5

Every LUT is evaluated baby-step / giant-step: P(x, y) = sum_i x^i L_i(y) with the inner
L_i(y) = sum_j c_ij y^j as one fused linear combination (engine.lincomb) and the outer sum as
one fused dot product with a single relinearisation (engine.dot).  Powers x^9..x^15 are
conjugates of x^7..x^1 (x^16 = 1 on the Zeta-16 circle), as the reference's XOR basis does
(xor_service.py:245-254).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import aes_tables as T
from .coeffs_gen import lut_2d
from .fhe import Ciphertext, Engine

ZETA16 = np.exp(-2j * np.pi / 16)


def _nz(c: complex) -> bool:
    return abs(c) > 1e-12


@dataclass
class RoundKey:
    """Encrypted round key, key-side XOR inner polynomials precomputed (B = 1, broadcast)."""
    inner_hi: Dict[int, Ciphertext]
    inner_lo: Dict[int, Ciphertext]


class AESRoundEngine:
    def __init__(self, engine: Engine, sk, pk, rlk, cjk, rotation_keys: Dict[int, object] | None = None):
        self.e = engine
        self.sk, self.pk, self.rlk, self.cjk = sk, pk, rlk, cjk
        self.sc = engine.slot_count
        self.n_blk = self.sc // 16
        # LUT coefficient matrices (16 x 16, Zeta-16 in, Zeta-16 out)
        self.C_sbox_hi = lut_2d(lambda h, l: int(T.SBOX[16 * h + l]) >> 4, 16)
        self.C_sbox_lo = lut_2d(lambda h, l: int(T.SBOX[16 * h + l]) & 15, 16)
        self.C_x2_hi = lut_2d(lambda h, l: int(T.GF2[16 * h + l]) >> 4, 16)
        self.C_x2_lo = lut_2d(lambda h, l: int(T.GF2[16 * h + l]) & 15, 16)
        self.C_xor = lut_2d(lambda a, b: a ^ b, 16)
        # ShiftRows+MixColumns plan: for term i, target row r reads source chunk r' + 4c' with
        # r' = r + i, c' = c + r + i  ->  shift of delta = (r - r') - 4 (r + i) chunks (mod 16)
        chunk = np.arange(self.sc) // self.n_blk
        row = chunk % 4
        self.plan: List[List[Tuple[int, object]]] = []
        deltas = set()
        for i in range(4):
            groups: Dict[int, List[int]] = {}
            for r in range(4):
                rp = (r + i) % 4
                d = ((r - rp) - 4 * (r + i)) % 16
                groups.setdefault(d, []).append(r)
            terms = []
            for d, rows in sorted(groups.items()):
                mask = np.isin(row, rows).astype(float)
                terms.append((d, engine.encode(mask)))
                if d:
                    deltas.add(d)
            self.plan.append(terms)
        self.deltas = sorted(deltas)
        if rotation_keys is None:
            rotation_keys = {d: engine.create_fixed_rotation_key(sk, d * self.n_blk) for d in self.deltas}
        self.rot_keys = rotation_keys

    # ---- layout ---------------------------------------------------------------------------
    def pack(self, blocks: np.ndarray) -> np.ndarray:
        """(NB, n_blk, 16) bytes -> (NB, slot_count) bytes in the byte-major layout."""
        b = np.asarray(blocks, dtype=np.uint8)
        return np.ascontiguousarray(b.transpose(0, 2, 1)).reshape(b.shape[0], self.sc)

    def unpack(self, slots: np.ndarray) -> np.ndarray:
        s = np.asarray(slots, dtype=np.uint8).reshape(-1, 16, self.n_blk)
        return np.ascontiguousarray(s.transpose(0, 2, 1))

    def encrypt_blocks(self, blocks: np.ndarray) -> Tuple[Ciphertext, Ciphertext]:
        """(NB, n_blk, 16) plaintext blocks -> batched (hi, lo) nibble ciphertexts."""
        s = self.pack(blocks).astype(np.int64)
        zh, zl = ZETA16 ** (s >> 4), ZETA16 ** (s & 15)
        return self.e.encrypt(zh, self.pk), self.e.encrypt(zl, self.pk)

    def decrypt_blocks(self, hi: Ciphertext, lo: Ciphertext) -> np.ndarray:
        def dec(ct):
            z = np.atleast_2d(self.e.decrypt(ct, self.sk))
            return np.mod(np.rint(-np.angle(z) * 16 / (2 * np.pi)), 16).astype(np.uint8)
        return self.unpack((dec(hi) << 4) | dec(lo))

    def encrypt_round_key(self, rk: np.ndarray) -> RoundKey:
        """16-byte round key replicated over every block (B = 1); the key side of the XOR
        LUT (L_i(k) = sum_j c_ij k^j, i odd) is evaluated once per key."""
        kb = np.repeat(np.asarray(rk, dtype=np.int64), self.n_blk)
        out = []
        for nib in (kb >> 4, kb & 15):
            ct = self.e.encrypt(ZETA16 ** nib, self.pk)
            out.append(self._xor_inner(self.odd_basis(ct)))
        return RoundKey(out[0], out[1])

    # ---- power bases ------------------------------------------------------------------------
    def odd_basis(self, x: Ciphertext) -> Dict[int, Ciphertext]:
        """x^1, x^3, ..., x^15 (5 products + 4 conjugations), aligned to one level."""
        e, rlk = self.e, self.rlk
        x2 = e.multiply(x, x, rlk)
        x4 = e.multiply(x2, x2, rlk)
        x3 = e.multiply(x2, x, rlk)
        x5 = e.multiply(x4, x, rlk)
        x7 = e.multiply(x4, x3, rlk)
        b = {1: x, 3: x3, 5: x5, 7: x7}
        for k in (1, 3, 5, 7):
            b[16 - k] = e.conjugate(b[k], self.cjk)
        return self._aligned(b)

    def full_basis(self, x: Ciphertext) -> Dict[int, Ciphertext]:
        """x^1..x^15 (7 products + 7 conjugations), aligned to one level."""
        e = self.e
        pw = e.make_power_basis(x, 8, self.rlk)
        b = {k + 1: c for k, c in enumerate(pw)}
        for k in range(9, 16):
            b[k] = e.conjugate(b[16 - k], self.cjk)
        return self._aligned(b)

    def _aligned(self, b: Dict[int, Ciphertext]) -> Dict[int, Ciphertext]:
        keys = sorted(b)
        al = self.e.align([b[k] for k in keys])
        return dict(zip(keys, al))

    # ---- LUT evaluation -------------------------------------------------------------------------
    def _inner(self, ybasis: Dict[int, Ciphertext], C: np.ndarray, rows: Sequence[int]):
        """L_i(y) = sum_{j>=1} C[i, j] y^j for the requested rows, all rows in one fused pass over
        the basis (engine.lincomb_many); rows whose y-part is empty are omitted (the y^0 column
        C[i, 0] is handled by _outer)."""
        js = sorted(j for j in ybasis if j >= 1)
        rows = [i for i in rows if any(_nz(C[i, j]) for j in js)]
        if not rows:
            return {}
        M = np.array([[C[i, j] for j in js] for i in rows], dtype=np.complex128)
        outs = self.e.lincomb_many([ybasis[j] for j in js], M)
        return dict(zip(rows, outs))

    def _xor_inner(self, ybasis):
        rows = [i for i in range(1, 16, 2)]
        return self._inner(ybasis, self.C_xor, rows)

    def _outer(self, xbasis: Dict[int, Ciphertext], inner: Dict[int, Ciphertext],
               C: np.ndarray | None = None):
        """sum_i x^i (L_i(y) + C[i, 0]): one fused dot product for the y-dependent part (x side
        levelled down once to the inner level), one fused linear combination over x for the
        y^0 column, the i = 0 row added as is."""
        e = self.e
        ks = sorted(k for k in inner if k != 0)
        parts = []
        if ks:
            lv = min(inner[k].level for k in ks)
            xs = [xbasis[k] for k in ks]
            if xs[0].level > lv:
                xs = e.align(xs, lv)
            parts.append(e.dot(xs, [inner[k] for k in ks], self.rlk))
        if 0 in inner:
            parts.append(inner[0])
        if C is not None:
            cx = [k for k in range(1, 16) if _nz(C[k, 0]) and k in xbasis]
            if cx:
                parts.append(e.lincomb([xbasis[k] for k in cx], [C[k, 0] for k in cx]))
        out = parts[0]
        for p in parts[1:]:
            out = e.add(out, p)
        if C is not None and _nz(C[0, 0]):
            out = e.add(out, complex(C[0, 0]))
        return out

    def lut2(self, xb, yb, C: np.ndarray) -> Ciphertext:
        return self.lut2_many(xb, yb, [C])[0]

    def lut2_many(self, xb, yb, Cs: Sequence[np.ndarray]) -> List[Ciphertext]:
        """Several 2-D LUTs over the same operand bases (x side aligned once)."""
        inners = []
        for C in Cs:
            rows = [i for i in range(16) if np.any(np.abs(C[i]) > 1e-12)]
            inners.append(self._inner(yb, C, rows))
        lv = min(ct.level for inn in inners for ct in inn.values())
        keys = sorted(xb)
        if xb[keys[0]].level > lv:
            xb = dict(zip(keys, self.e.align([xb[k] for k in keys], lv)))
        return [self._outer(xb, inn, C) for inn, C in zip(inners, Cs)]

    def xor(self, xb, yb) -> Ciphertext:
        return self._outer(xb, self._xor_inner(yb))

    def xor_pair(self, a, b):
        """(a_hi ^ b_hi, a_lo ^ b_lo) from odd bases of both operands."""
        return self.xor(a[0], b[0]), self.xor(a[1], b[1])

    # ---- round steps ------------------------------------------------------------------------
    def sub_bytes(self, h: Ciphertext, l: Ciphertext) -> Tuple[Ciphertext, Ciphertext]:
        hb, lb = self.full_basis(h), self.full_basis(l)
        sh, sl = self.lut2_many(hb, lb, [self.C_sbox_hi, self.C_sbox_lo])
        return sh, sl

    def shift_mix_terms(self, s: Ciphertext) -> List[Ciphertext]:
        """T_0..T_3 of one nibble ciphertext: rotations of s by whole byte-chunks, each
        masked to the target rows that read it (ShiftRows folded into the rotations)."""
        e = self.e
        rots = {0: s}
        for d in self.deltas:
            rots[d] = e.rotate(s, self.rot_keys[d])
        out = []
        for terms in self.plan:
            acc = None
            for d, mask in terms:
                part = e.multiply(rots[d], mask)
                acc = part if acc is None else e.add(acc, part)
            out.append(acc)
        return out

    def mix_columns(self, th: List[Ciphertext], tl: List[Ciphertext]):
        """out = xtime(T0 ^ T1) ^ (T1 ^ (T2 ^ T3)) on nibble pairs."""
        ob = [(self.odd_basis(th[i]), self.odd_basis(tl[i])) for i in range(4)]
        u = self.xor_pair(ob[0], ob[1])
        w = self.xor_pair(ob[2], ob[3])
        wb = (self.odd_basis(w[0]), self.odd_basis(w[1]))
        v = self.xor_pair(ob[1], wb)
        ub_h, ub_l = self.full_basis(u[0]), self.full_basis(u[1])
        x = tuple(self.lut2_many(ub_h, ub_l, [self.C_x2_hi, self.C_x2_lo]))
        xb = (self.odd_basis(x[0]), self.odd_basis(x[1]))
        vb = (self.odd_basis(v[0]), self.odd_basis(v[1]))
        return self.xor_pair(xb, vb)

    def add_round_key(self, h: Ciphertext, l: Ciphertext, key: RoundKey):
        return (self._outer(self.odd_basis(h), key.inner_hi),
                self._outer(self.odd_basis(l), key.inner_lo))

    def round(self, h: Ciphertext, l: Ciphertext, key: RoundKey, timings: dict | None = None):
        """SubBytes -> ShiftRows -> MixColumns -> AddRoundKey (a middle AES-128 round).
        With `timings`, the engine is synchronised after each step and wall times recorded."""
        import time

        def mark(name, t0):
            if timings is not None:
                self.e.synchronize()
                t1 = time.perf_counter()
                timings[name] = timings.get(name, 0.0) + (t1 - t0)
                return t1
            return t0
        t = mark("start", 0.0) if timings is not None else 0.0
        sh, sl = self.sub_bytes(h, l)
        t = mark("sub_bytes", t)
        th, tl = self.shift_mix_terms(sh), self.shift_mix_terms(sl)
        t = mark("shift_rows_terms", t)
        mh, ml = self.mix_columns(th, tl)
        t = mark("mix_columns", t)
        out = self.add_round_key(mh, ml, key)
        mark("add_round_key", t)
        return out
