"""ShiftRows / InvShiftRows on ciphertexts holding AES states in contiguous 16-slot blocks
(reference: shiftrows_service.py:5-69; byte (r, c) of block b sits in slot 16 b + r + 4 c).

The reference masks row r and rotates the whole vector by -4r, which moves the wrapped bytes
of row r into the next block (6 of 16 slots wrong) and only masks block 0.  Here every row is
split by source column: bytes with c >= r move by -4r, bytes with c < r by 16 - 4r (and the
inverse mirrored), with masks tiled over every block of the ciphertext.
"""
from __future__ import annotations

import numpy as np

from .xor_service import EngineWrapper, XORService


def _masks(sc: int, forward: bool):
    """[(mask vector, rotation)] covering all 16 positions of every block."""
    out = []
    pos = np.arange(sc) % 16
    row, col = pos % 4, pos // 4
    for r in range(4):
        if r == 0:
            out.append(((row == 0).astype(float), 0))
            continue
        if forward:
            out.append((((row == r) & (col >= r)).astype(float), -4 * r))
            out.append((((row == r) & (col < r)).astype(float), 16 - 4 * r))
        else:
            out.append((((row == r) & (col < 4 - r)).astype(float), 4 * r))
            out.append((((row == r) & (col >= 4 - r)).astype(float), 4 * r - 16))
    return out


class AESFHEShiftRows:
    def __init__(self, engine_wrapper: EngineWrapper, xor_svc: XORService | None = None):
        self.eng = engine_wrapper
        self.xor_svc = xor_svc
        sc = self.eng.engine.slot_count
        self._fwd = [(self.eng.encode(m), k) for m, k in _masks(sc, True)]
        self._inv = [(self.eng.encode(m), k) for m, k in _masks(sc, False)]

    def _apply(self, ct, plan):
        out = None
        for pt, k in plan:
            part = self.eng.multiply(ct, pt)
            if k:
                part = self.eng.rotate(part, k)
            out = part if out is None else self.eng.add(out, part)
        return out

    def shift_rows(self, ct):
        return self._apply(ct, self._fwd)

    def inverse_shift_rows(self, ct):
        return self._apply(ct, self._inv)
