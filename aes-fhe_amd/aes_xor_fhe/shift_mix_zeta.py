"""``MixRow``: the reference's merged ShiftRows+MixColumns as rotate-mask-XOR in the Zeta-16
domain (reference: shift_mix_zeta.py:14-122), restated with the same operation sequence.

As SURVEY.md 0 records, this construction is degenerate in exact arithmetic (every output
slot is 0); it is kept for call-surface parity and op-trace parity only.  It chains 23
``xor_cipher`` calls, so it needs bootstrapping at L = 30 (xor_cipher bootstraps operands
below level 8): supply ``EngineWrapper.bootstrap``.  The correct
ShiftRows+MixColumns is aes_round.AESRoundEngine.
"""
from __future__ import annotations

import numpy as np

from .utils import zeta_decode, zeta_encode
from .xor_service import EngineWrapper, XORService

_FWD = [[2, 3, 1, 1], [1, 1, 2, 3], [3, 1, 1, 2], [1, 2, 3, 1]]
_INV = [[14, 11, 13, 9], [9, 14, 11, 13], [13, 9, 14, 11], [11, 13, 9, 14]]


class MixRow:
    def __init__(self, xor_service: XORService, engine_wrapper: EngineWrapper):
        self.xor_svc = xor_service
        self.eng = engine_wrapper

    def _first_of_four(self):
        return self.eng.encrypt(zeta_encode(np.array([1.0 if i % 4 == 0 else 0.0 for i in range(16)])))

    def _block(self, ct_s, ct_x):
        e, x = self.eng, self.xor_svc
        t = e.relinearize(e.multiply(ct_s, ct_x))
        r1, r2, r3 = e.rotate(t, -1), e.rotate(t, -2), e.rotate(t, -3)
        comp = x.xor_cipher(x.xor_cipher(x.xor_cipher(t, r1), r2), r3)
        return e.relinearize(e.multiply(comp, self._first_of_four()))

    def _collapse(self, ct_b):
        e, x = self.eng, self.xor_svc
        u1 = x.xor_cipher(ct_b, e.rotate(ct_b, -2))
        u2 = x.xor_cipher(u1, e.rotate(u1, -1))
        return e.relinearize(e.multiply(u2, self._first_of_four()))

    def _combine(self, cts):
        out = None
        for k, ct in zip((0, 5, 10, 15), cts):
            p = self.eng.rotate(ct, -k)
            out = p if out is None else self.xor_svc.xor_cipher(out, p)
        return out

    def merged_shift_mix_fhe(self, state_matrix):
        vec = np.array(state_matrix, dtype=np.float64).reshape(16, order="C")
        ct_state = self.eng.encrypt(zeta_encode(vec))
        rows = [self.eng.encrypt(zeta_encode(np.tile(r, 4).astype(np.float64))) for r in _FWD]
        blocks = [self._block(ct_state, r) for r in rows]
        return self._combine([self._collapse(b) for b in blocks])

    def merged_inv_mixshift_fhe_from_ct(self, ct_state):
        rows = [self.eng.encrypt(zeta_encode(np.tile(r, 4).astype(np.float64))) for r in _INV]
        blocks = [self._block(ct_state, r) for r in rows]
        out = self._combine([self._collapse(b) for b in blocks])
        vec = np.round(zeta_decode(self.eng.decrypt(out))).astype(np.int64)
        return vec[:16].reshape((4, 4), order="C")
