"""AES SubBytes on Zeta-encoded bytes (reference: sbox/sbox_service.py:71-138).

Two 8->4 LUT polynomials share one degree-255 power basis: P_hi(x) = zeta_256^{16 (S>>4)}
and P_lo(x) = zeta_256^{S & 15}; their product is zeta_256^{S(x)}.  ``sub_bytes`` /
``sub_bytes_array`` keep the reference's op order (one ct x pt and one add per non-zero
coefficient); ``sub_bytes_fused`` evaluates the same polynomials with one fused linear
combination each.
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, List

import numpy as np

from ..aes_tables import AES_SBOX  # noqa: F401  (re-exported like the reference)
from ..coeffs_gen import load_1d
from ..engine_context import EngineContext

COEFF_DIR = Path(__file__).resolve().parents[1] / "coeffs"


def load_json_coeffs(path: Path) -> np.ndarray:
    """Dense complex coefficient vector from a {n, entries: [[i, re, im]]} file."""
    return load_1d(path)


class SBoxService:
    def __init__(self, ctx: EngineContext, hi_path: Path = COEFF_DIR / "sbox_hi_coeffs.json",
                 lo_path: Path = COEFF_DIR / "sbox_lo_coeffs.json"):
        self.ctx = ctx
        self.engine = ctx.engine
        self.rlk = ctx.relinearization_key
        self.coeffs_hi = load_json_coeffs(hi_path)
        self.coeffs_lo = load_json_coeffs(lo_path)
        sc = self.engine.slot_count
        self.pt_hi = [self.engine.encode(np.full(sc, c, dtype=np.complex128)) for c in self.coeffs_hi]
        self.pt_lo = [self.engine.encode(np.full(sc, c, dtype=np.complex128)) for c in self.coeffs_lo]

    def _build_power_basis(self, ct: Any) -> List[Any]:
        return self.engine.make_power_basis(ct, len(self.coeffs_hi) - 1, self.rlk)

    def _lut(self, ct, powers, coeffs, pts):
        out = self.engine.multiply(ct, 0.0)
        for i, pt in enumerate(pts):
            if abs(coeffs[i]) < 1e-12:
                continue
            term = pt if i == 0 else self.engine.multiply(powers[i - 1], pt)
            out = self.engine.add(out, term)
        return out

    def sub_bytes(self, enc_byte: Any) -> Any:
        powers = self._build_power_basis(enc_byte)
        hi = self._lut(enc_byte, powers, self.coeffs_hi, self.pt_hi)
        lo = self._lut(enc_byte, powers, self.coeffs_lo, self.pt_lo)
        return self.engine.multiply(hi, lo, self.rlk)

    def sub_bytes_array(self, enc_arr: Any) -> Any:
        """SIMD SubBytes: every slot of the ciphertext (same evaluation as sub_bytes)."""
        return self.sub_bytes(enc_arr)

    def sub_bytes_fused(self, enc_arr: Any) -> Any:
        """Same hi / lo polynomials, evaluated with half the basis.  The input slots are 256-th
        roots of unity (zeta_256^x), where x^(256-i) = conj(x^i); so with the powers x^1..x^128,
        P(x) = c_0 + sum_{i<=128} c_i x^i + conj(sum_{i<128} conj(c_{256-i}) x^i): 127 basis
        products instead of 254, the four sums in one lincomb_many pass, one conjugation per
        polynomial.  One level fewer than sub_bytes (x^128 needs 7 levels, x^255 eight).  Without
        a conjugation key in the context it falls back to one lincomb over the full basis."""
        e = self.engine
        cjk = getattr(self.ctx, "conjugation_key", None)
        hi, lo = self.coeffs_hi, self.coeffs_lo
        if cjk is None or len(hi) != 256 or len(lo) != 256:
            powers = self._build_power_basis(enc_arr)
            outs = []
            for c in (hi, lo):
                ks = [k for k in range(1, len(c)) if abs(c[k]) >= 1e-12]
                o = e.lincomb([powers[k - 1] for k in ks], [c[k] for k in ks])
                if abs(c[0]) >= 1e-12:
                    o = e.add(o, complex(c[0]))
                outs.append(o)
            return e.multiply(outs[0], outs[1], self.rlk)
        powers = e.make_power_basis(enc_arr, 128, self.rlk)
        rows = []
        for c in (hi, lo):
            c = np.asarray(c, dtype=np.complex128)
            rows.append(c[1:129])
            rows.append(np.concatenate([np.conj(c[255:128:-1]), [0.0]]))
        s = e.lincomb_many(powers, np.stack(rows))
        outs = []
        for t, c in enumerate((hi, lo)):
            o = e.add(s[2 * t], e.conjugate(s[2 * t + 1], cjk))
            if abs(c[0]) >= 1e-12:
                o = e.add(o, complex(c[0]))
            outs.append(o)
        return e.multiply(outs[0], outs[1], self.rlk)
