"""Nibble-domain AES round plumbing (reference: new.py:8-227).

``full_round`` is the reference's AddRoundKey on hi/lo nibbles (new.py:186-227): split both
operands into nibbles, Zeta-16 encode, encrypt four ciphertexts, 4-bit XOR each half with
``XORService.xor_cipher``, then decrypt and recombine.  ``shift_rows`` works on the
byte-major layout of ``_get_shift_rows_masks`` (row r = slot chunks [4rB, 4(r+1)B), B =
slot_count/16 blocks) and fixes the reference's crash (new.py:115: no ``self``, rotate without
key) and its wrap-around: bytes with column c >= r move by -rB, the others by (4 - r)B.
"""
from __future__ import annotations

from typing import Any, Tuple

import numpy as np

from .engine_context import EngineContext
from .xor_service import EngineWrapper, XORService, ZetaEncoder


def _get_shift_rows_masks(ctx: EngineContext) -> dict:
    """Row masks of the byte-major layout, cached on the context (new.py:8-36)."""
    if hasattr(ctx, "_sr_masks"):
        return ctx._sr_masks
    sc = ctx.engine.slot_count
    nb = sc // 16
    chunk = np.arange(sc) // nb
    masks = {r: ctx.engine.encode((chunk // 4 == r).astype(float)) for r in range(4)}
    ctx._sr_masks = masks
    return masks


def split_nibbles(flat: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    b = np.asarray(flat).astype(np.uint8, copy=False)
    return (b >> 4).astype(np.uint8), (b & 0x0F).astype(np.uint8)


def decrypt_and_recombine(ct_hi: Any, ct_lo: Any, eng: EngineWrapper, length: int | None = None) -> np.ndarray:
    hi = ZetaEncoder.from_zeta(eng.decrypt(ct_hi), modulus=16)
    lo = ZetaEncoder.from_zeta(eng.decrypt(ct_lo), modulus=16)
    if length is not None:
        hi, lo = hi[:length], lo[:length]
    return ((hi.astype(np.uint8) << 4) | lo.astype(np.uint8)).astype(np.uint8)


class AESFHERound:
    def __init__(self, eng_wrap: EngineWrapper, xor_svc: XORService):
        self.eng = eng_wrap
        self.xor = xor_svc
        self.row_rot = [0, -4, -8, -12]
        sc = self.eng.engine.slot_count
        nb = sc // 16
        chunk = np.arange(sc) // nb
        row, col = chunk // 4, chunk % 4
        # byte-major ShiftRows plan: (mask, rotation) pairs, wrap-aware
        self._sr_plan = [(self.eng.encode((row == 0).astype(float)), 0)]
        for r in range(1, 4):
            self._sr_plan.append((self.eng.encode(((row == r) & (col >= r)).astype(float)), -r * nb))
            self._sr_plan.append((self.eng.encode(((row == r) & (col < r)).astype(float)), (4 - r) * nb))

    def encrypt_nibbles(self, hi: np.ndarray, lo: np.ndarray) -> Tuple[Any, Any]:
        return (self.eng.encrypt(ZetaEncoder.to_zeta(hi, modulus=16)),
                self.eng.encrypt(ZetaEncoder.to_zeta(lo, modulus=16)))

    def add_round_key(self, s_hi, s_lo, k_hi, k_lo):
        return self.xor.xor_cipher(s_hi, k_hi), self.xor.xor_cipher(s_lo, k_lo)

    def shift_rows(self, ct_hi: Any, ct_lo: Any) -> Tuple[Any, Any]:
        outs = []
        for ct in (ct_hi, ct_lo):
            acc = None
            for pt, k in self._sr_plan:
                part = self.eng.multiply(ct, pt)
                if k:
                    part = self.eng.rotate(part, k)
                acc = part if acc is None else self.eng.add(acc, part)
            outs.append(acc)
        return outs[0], outs[1]

    def mix_columns(self, ct_hi: Any, ct_lo: Any):
        raise NotImplementedError(
            "the reference's nibble MixColumns is unfinished (new.py:150-184, calls a missing "
            "self.gf2); the working round is aes_round.AESRoundEngine")

    def full_round(self, state: np.ndarray, key: np.ndarray, recombine: bool = True):
        s_hi, s_lo = split_nibbles(state)
        k_hi, k_lo = split_nibbles(key)
        enc = lambda v: self.eng.encrypt(ZetaEncoder.to_zeta(v, modulus=16))
        ct_s_hi, ct_s_lo, ct_k_hi, ct_k_lo = enc(s_hi), enc(s_lo), enc(k_hi), enc(k_lo)
        out_hi = self.xor.xor_cipher(ct_s_hi, ct_k_hi)
        out_lo = self.xor.xor_cipher(ct_s_lo, ct_k_lo)
        if not recombine:
            return out_hi, out_lo
        return decrypt_and_recombine(out_hi, out_lo, self.eng, length=np.asarray(state).shape[0])
