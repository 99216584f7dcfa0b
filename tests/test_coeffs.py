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


def test_zeta_table_encode_bit_identical():
    """ZetaEncoder.to_zeta by a table of the m roots is word-for-word the elementwise
    exp(-2 pi i (k mod m) / m) the reference computes (xor_service.py:132-145), negative and
    out-of-range k included, for power-of-two and other moduli."""
    import numpy as np
    from aes_xor_fhe.xor_service import ZetaEncoder
    rng = np.random.default_rng(7)
    for m in (2, 4, 16, 256, 7, 10):
        a = rng.integers(-5000, 5000, 20000)
        ref = np.exp(-2j * np.pi * (a.astype(np.int64) % m) / m)
        got = ZetaEncoder.to_zeta(a, m)
        assert got.dtype == np.complex128 and np.array_equal(got.view(np.uint64), ref.view(np.uint64))
    u8 = rng.integers(0, 256, 1000).astype(np.uint8)
    assert np.array_equal(ZetaEncoder.to_zeta(u8, 256), np.exp(-2j * np.pi * (u8.astype(np.int64) % 256) / 256))
