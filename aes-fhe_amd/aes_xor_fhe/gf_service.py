"""GF(2^8) x2 / x3 as Zeta-domain LUT polynomials (reference: gf_service.py:21-78).

Each multiplier returns (hi, lo) = (zeta_256^{16 (g>>4)}, zeta_256^{g & 15}) for g = k*x in
GF(2^8), evaluated on a zeta_256 byte with its own degree-255 power basis.  The coefficient
files the reference loads (generator/coeffs/gf{2,3}_{hi,lo}_coeffs.json, gf_service.py:39-42)
are absent from its tree; they are regenerated here with the variant whose hi*lo product
decodes to k*x (generator/generate_gf2_gf3_coeffs.py:60-68), see coeffs_gen.py.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from .coeffs_gen import load_1d
from .xor_service import EngineWrapper, XORService

COEFF_DIR = Path(__file__).resolve().parent / "coeffs"


class GFService:
    def __init__(self, eng_wrap: EngineWrapper, xor_svc: XORService, base: Path = COEFF_DIR):
        self.eng = eng_wrap
        self.xor_svc = xor_svc
        self.coeffs2_hi = load_1d(base / "gf2_hi_coeffs.json")
        self.coeffs2_lo = load_1d(base / "gf2_lo_coeffs.json")
        self.coeffs3_hi = load_1d(base / "gf3_hi_coeffs.json")
        self.coeffs3_lo = load_1d(base / "gf3_lo_coeffs.json")
        sc = self.eng.engine.slot_count
        enc = lambda cs: [self.eng.encode(np.full(sc, c, dtype=np.complex128)) for c in cs]
        self.pt2_hi, self.pt2_lo = enc(self.coeffs2_hi), enc(self.coeffs2_lo)
        self.pt3_hi, self.pt3_lo = enc(self.coeffs3_hi), enc(self.coeffs3_lo)

    def _eval_1d_lut(self, ct, pt_list):
        """Reference op order (gf_service.py:55-64): power basis, then one ct x pt + add per
        coefficient (zero coefficients included), constant term added as a plaintext."""
        powers = self.eng.make_power_basis(ct, len(pt_list) - 1)
        out = self.eng.multiply(ct, 0.0)
        out = self.eng.add(out, pt_list[0])
        for i, pt in enumerate(pt_list[1:], start=1):
            out = self.eng.add(out, self.eng.multiply(powers[i - 1], pt, self.eng.relin_key))
        return out

    def mul1(self, ct):
        return ct

    def mul2(self, ct):
        return self._eval_1d_lut(ct, self.pt2_hi), self._eval_1d_lut(ct, self.pt2_lo)

    def mul3(self, ct):
        return self._eval_1d_lut(ct, self.pt3_hi), self._eval_1d_lut(ct, self.pt3_lo)
