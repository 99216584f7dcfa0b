"""``AESFHETransformer``: merged ShiftRows+MixColumns via GF LUTs + recombine + XOR on
contiguous 16-slot blocks (reference: mixcolumns_service.py:11-88), same operation sequence:
rotations -1/-6/-11, per output block GF x2/x3 (hi, lo) -> recombine -> xor_cipher chain,
four bootstraps, final rotate-XOR.  As written in the reference it feeds 8-bit Zeta-256
values to the 4-bit XOR LUT and diverges; it needs bootstrapping.  Kept for
call-surface / op-trace parity (recombination included: XORService.recombine_nibbles_ref); the
correct round is aes_round.AESRoundEngine.
"""
from __future__ import annotations

from typing import Any

import numpy as np

from .gf_service import GFService
from .xor_service import EngineWrapper, XORService, ZetaEncoder

_SPECS = [[("A", "mul2"), ("A1", "mul3"), ("A6", "mul1")],
          [("A1", "mul2"), ("A6", "mul3"), ("A11", "mul1")],
          [("A6", "mul2"), ("A11", "mul3"), ("A1", "mul1")],
          [("A11", "mul2"), ("A1", "mul3"), ("A6", "mul1")]]


class AESFHETransformer:
    def __init__(self, engine_wrapper: EngineWrapper, xor_svc: XORService, gf_svc: GFService):
        self.eng = engine_wrapper
        self.xor_svc = xor_svc
        self.gf_svc = gf_svc

    def merged_shift_mix(self, state_bytes: np.ndarray) -> Any:
        eng = self.eng
        ct = eng.encrypt(ZetaEncoder.to_zeta(state_bytes, modulus=256))
        rts = {"A": ct, "A1": eng.rotate(ct, -1), "A6": eng.rotate(ct, -6),
               "A11": eng.rotate(ct, -11)}

        def apply_mix(spec):
            terms = []
            for key, fn in spec:
                c = rts[key]
                if fn == "mul1":
                    terms.append(c)
                else:
                    hi, lo = getattr(self.gf_svc, fn)(c)
                    terms.append(self.xor_svc.recombine_nibbles_ref(hi, lo))
            acc = terms[0]
            for t in terms[1:]:
                acc = self.xor_svc.xor_cipher(acc, t)
            return acc

        blocks = [eng.bootstrap(apply_mix(s)) for s in _SPECS]
        out = blocks[0]
        for k in (1, 2, 3):
            out = self.xor_svc.xor_cipher(out, eng.rotate(blocks[k], -k))
        return out

    def merged_inv_mixshift(self, ct_state: Any) -> Any:
        raise NotImplementedError(
            "InvMixColumns + InvShiftRows need gf9/11/13/14 LUTs (as in the reference)")
