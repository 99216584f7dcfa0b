"""LUT-polynomial coefficients for Zeta-domain table lookups, generated from first principles.

A function f: Z_n -> Z_m on Zeta-encoded inputs becomes P(z) = sum_k c_k z^k with
c = ifft([zeta^{f(x)}]_x) (reference: sbox/generate_sbox_coeffs.py:34-43); a two-input
function uses ifft2 (generator/generate_multivariate_coeffs.py:7-13).  Files keep the
reference's JSON layout ({n, tol, entries: [[i, re, im]]} / {shape, tol, entries:
[[i, j, re, im]]}) so either side's loaders read them.

Regenerate the shipped files with ``python -m aes_xor_fhe.coeffs_gen``; tests compare them to
the reference's own JSON files (tests/golden/ref_coeffs/) within 1e-15.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from .aes_tables import GF2, GF3, SBOX

COEFF_DIR = Path(__file__).resolve().parent / "coeffs"
TOL = 1e-12


def lut_1d(fn, n: int = 256, out_mod: int | None = None) -> np.ndarray:
    """c_k such that sum_k c_k zeta_n^{x k} = zeta_{out_mod}^{fn(x)} (zeta = exp(-2 pi i/.))."""
    out_mod = n if out_mod is None else out_mod
    root = np.exp(-2j * np.pi / out_mod)
    lut = np.array([root ** int(fn(x)) for x in range(n)], dtype=np.complex128)
    return np.fft.ifft(lut)


def lut_2d(fn, n: int = 16, out_mod: int | None = None) -> np.ndarray:
    out_mod = n if out_mod is None else out_mod
    root = np.exp(-2j * np.pi / out_mod)
    lut = np.array([[root ** int(fn(i, j)) for j in range(n)] for i in range(n)],
                   dtype=np.complex128)
    return np.fft.ifft2(lut)


def save_1d(coeffs: np.ndarray, path: Path, note: str = "", tol: float = TOL) -> None:
    entries = [[i, float(c.real), float(c.imag)] for i, c in enumerate(coeffs) if abs(c) > tol]
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_text(json.dumps({"n": len(coeffs), "tol": tol, "entries": entries, "note": note},
                               indent=1))


def save_2d(coeffs: np.ndarray, path: Path, tol: float = TOL) -> None:
    n, m = coeffs.shape
    entries = [[i, j, float(coeffs[i, j].real), float(coeffs[i, j].imag)]
               for i in range(n) for j in range(m) if abs(coeffs[i, j]) > tol]
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_text(json.dumps({"shape": [n, m], "tol": tol, "entries": entries}, indent=1))


def load_1d(path: Path) -> np.ndarray:
    data = json.loads(Path(path).read_text(encoding="utf-8"))
    out = np.zeros(data.get("n") or len(data["entries"]), dtype=np.complex128)
    for i, re, im in data["entries"]:
        out[int(i)] = re + 1j * im
    return out


def load_2d(path: Path) -> np.ndarray:
    data = json.loads(Path(path).read_text(encoding="utf-8"))
    out = np.zeros(tuple(data["shape"]), dtype=np.complex128)
    for i, j, re, im in data["entries"]:
        out[int(i), int(j)] = re + 1j * im
    return out


# The LUTs the services use ------------------------------------------------------------------
def sbox_hi() -> np.ndarray:      # zeta_256^{16 (S(x) >> 4)} on byte input (sbox_service)
    return lut_1d(lambda x: (int(SBOX[x]) >> 4) * 16, 256)


def sbox_lo() -> np.ndarray:      # zeta_256^{S(x) & 15}
    return lut_1d(lambda x: int(SBOX[x]) & 0xF, 256)


def xor_4bit() -> np.ndarray:     # zeta_16^{a ^ b} (xor_mono_coeffs.json)
    return lut_2d(lambda a, b: a ^ b, 16)


def gf_hi(table) -> np.ndarray:   # variant A (generator/generate_gf2_gf3_coeffs.py:60-68)
    return lut_1d(lambda x: (int(table[x]) >> 4) * 16, 256)


def gf_lo(table) -> np.ndarray:
    return lut_1d(lambda x: int(table[x]) & 0xF, 256)


def write_all(out: Path = COEFF_DIR) -> None:
    save_1d(sbox_hi(), out / "sbox_hi_coeffs.json", "8-to-4 S-Box LUT coefficients via IFFT")
    save_1d(sbox_lo(), out / "sbox_lo_coeffs.json", "8-to-4 S-Box LUT coefficients via IFFT")
    save_2d(xor_4bit(), out / "xor_mono_coeffs.json")
    for name, tab in (("gf2", GF2), ("gf3", GF3)):
        save_1d(gf_hi(tab), out / f"{name}_hi_coeffs.json", f"GF x{name[-1]} hi LUT")
        save_1d(gf_lo(tab), out / f"{name}_lo_coeffs.json", f"GF x{name[-1]} lo LUT")


if __name__ == "__main__":
    write_all()
    print("wrote", COEFF_DIR)
