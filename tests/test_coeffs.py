"""LUT coefficients regenerated from first principles equal the reference's data files
(sbox/coeffs/*.json, generator/coeffs/xor_mono_coeffs.json) and decode exactly."""
from pathlib import Path

import numpy as np
import pytest

from aes_xor_fhe import coeffs_gen as G
from aes_xor_fhe.aes_tables import GF2, GF3, SBOX

REFC = Path(__file__).resolve().parent / "golden" / "ref_coeffs"


@pytest.mark.parametrize("name", ["sbox_hi_coeffs.json", "sbox_lo_coeffs.json"])
def test_sbox_coeffs_match_reference(name):
    assert np.abs(G.load_1d(G.COEFF_DIR / name) - G.load_1d(REFC / name)).max() <= 1e-15


def test_xor_coeffs_match_reference():
    ours, ref = G.load_2d(G.COEFF_DIR / "xor_mono_coeffs.json"), G.load_2d(REFC / "xor_mono_coeffs.json")
    assert np.abs(ours - ref).max() <= 1e-15
    assert np.count_nonzero(np.abs(ref) > 1e-12) == 64        # odd x odd terms only


def _eval1(c, x, n=256):
    z = np.exp(-2j * np.pi * x / n)
    return np.polyval(c[::-1], z)


def test_luts_decode_exactly():
    x = np.arange(256)
    dec = lambda v, m: np.mod(np.rint(-np.angle(v) * m / (2 * np.pi)), m).astype(int)
    hi, lo = G.load_1d(G.COEFF_DIR / "sbox_hi_coeffs.json"), G.load_1d(G.COEFF_DIR / "sbox_lo_coeffs.json")
    assert np.array_equal(dec(_eval1(hi, x) * _eval1(lo, x), 256), SBOX)
    for tab, nm in ((GF2, "gf2"), (GF3, "gf3")):
        ph = _eval1(G.load_1d(G.COEFF_DIR / f"{nm}_hi_coeffs.json"), x)
        pl = _eval1(G.load_1d(G.COEFF_DIR / f"{nm}_lo_coeffs.json"), x)
        assert np.array_equal(dec(ph * pl, 256), tab)
    C = G.xor_4bit()
    a, b = np.meshgrid(np.arange(16), np.arange(16), indexing="ij")
    za, zb = np.exp(-2j * np.pi * a / 16), np.exp(-2j * np.pi * b / 16)
    val = sum(C[i, j] * za ** i * zb ** j for i in range(16) for j in range(16))
    assert np.array_equal(dec(val, 16), a ^ b)
