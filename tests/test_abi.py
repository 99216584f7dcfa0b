"""The C-ABI boundary: both implementations load and export every symbol include/aesfhe.h
declares; host-only entry points (codec, prime chain) agree bit for bit; the product path
fails loudly when its extension is missing (no fallback)."""
import ctypes as C
import re
import subprocess

import numpy as np
import pytest

from conftest import ORACLE_SO, PKG, PRODUCT_SO, ROOT

HEADER = (ROOT / "include" / "aesfhe.h").read_text()
DECLARED = sorted(set(re.findall(r"\b(aesfhe_[a-z0-9_]+)\s*\(", HEADER)))


@pytest.fixture(scope="module")
def product_cdll():
    if not PRODUCT_SO.exists():
        subprocess.run(["make", "-C", str(PKG)], check=True)
    from aes_xor_fhe._abi import Lib
    return Lib(PRODUCT_SO)


def test_header_declares_the_boundary():
    for name in ("aesfhe_engine_create", "aesfhe_encrypt", "aesfhe_mul", "aesfhe_galois",
                 "aesfhe_power_basis", "aesfhe_ntt_host", "aesfhe_relinearize"):
        assert name in DECLARED


@pytest.mark.parametrize("which", ["product", "oracle"])
def test_exports_every_declared_symbol(which, product_cdll, oracle_lib):
    lib = product_cdll if which == "product" else oracle_lib
    missing = [s for s in DECLARED if not hasattr(lib.cdll, s)]
    assert not missing, missing
    from aes_xor_fhe._abi import SYMBOLS
    assert sorted(SYMBOLS) == DECLARED


def test_backend_names(product_cdll, oracle_lib):
    assert product_cdll.backend == "hip-gfx950"
    assert oracle_lib.backend == "oracle-cpu"


def test_abi_version(product_cdll, oracle_lib):
    """Both libraries report the header's ABI revision (the loader refuses any other)."""
    from aes_xor_fhe._abi import ABI_VERSION
    want = int(re.search(r"#define AESFHE_ABI_VERSION (\d+)", HEADER).group(1))
    assert ABI_VERSION == want
    assert product_cdll.abi_version() == want and oracle_lib.abi_version() == want


@pytest.mark.parametrize("body", ["", "int aesfhe_abi_version(void) { return 1; }",
                                  "int aesfhe_abi_version(void) { return %d; }"],
                         ids=["no-version-symbol", "old-revision", "missing-symbol"])
def test_stale_library_reads_as_rebuild(tmp_path, body):
    """A library built against an older header -- without aesfhe_abi_version, with an older
    revision, or with the current revision but a symbol missing -- is refused with a "rebuild it"
    RuntimeError before anything else is bound, not a ctypes AttributeError."""
    from aes_xor_fhe._abi import ABI_VERSION, Lib
    src = tmp_path / "stale.c"
    src.write_text((body % ABI_VERSION if "%d" in body else body) + "\nint aesfhe_unrelated(void) { return 0; }\n")
    so = tmp_path / "libstale.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    with pytest.raises(RuntimeError, match="rebuild it"):
        Lib(so)


@pytest.mark.parametrize("log_n", [10, 12, 16])
def test_host_codec_bit_identical(product_cdll, oracle_lib, log_n):
    n = 1 << (log_n - 1)
    rng = np.random.default_rng(log_n)
    re_, im_ = rng.standard_normal(n), rng.standard_normal(n)
    outs = []
    for lib in (product_cdll, oracle_lib):
        co = np.empty(2 * n, np.int64)
        lib.check(lib.encode(log_n, re_.ctypes.data_as(C.POINTER(C.c_double)),
                             im_.ctypes.data_as(C.POINTER(C.c_double)), n, 2.0 ** 40,
                             co.ctypes.data_as(C.POINTER(C.c_int64))))
        r2, i2 = np.empty(n), np.empty(n)
        lib.check(lib.decode(log_n, co.ctypes.data_as(C.POINTER(C.c_int64)), 2.0 ** 40,
                             r2.ctypes.data_as(C.POINTER(C.c_double)),
                             i2.ctypes.data_as(C.POINTER(C.c_double))))
        outs.append((co, r2, i2))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert np.array_equal(outs[0][1], outs[1][1]) and np.array_equal(outs[0][2], outs[1][2])
    np.testing.assert_allclose(outs[0][1] + 1j * outs[0][2], re_ + 1j * im_, atol=1e-9)


@pytest.mark.parametrize("log_n,L,K", [(12, 6, 2), (14, 8, 1), (16, 30, 8), (17, 35, 8)])
def test_prime_chain_identical(product_cdll, oracle_lib, log_n, L, K):
    from aes_xor_fhe._abi import Params
    p = Params(log_n, L, K, 40, 50, 50, 0, 0, 1, None)
    res = []
    for lib in (product_cdll, oracle_lib):
        q = (C.c_uint64 * (L + 1 + K))()
        s = (C.c_double * (L + 1))()
        lib.check(lib.chain(C.byref(p), q, s))
        res.append((list(q), list(s)))
    assert res[0] == res[1]
    q, s = res[0]
    M = 2 << log_n
    assert all(x % M == 1 for x in q) and len(set(q)) == len(q)
    assert all(x < 2 ** 51 for x in q)
    # canonical scales stay within 2^-10 of 2^40 (greedy prime choice tracks Delta_l)
    assert max(abs(np.log2(v) - 40) for v in s) < 2 ** -10


def test_galois_elements(product_cdll, oracle_lib):
    for lib in (product_cdll, oracle_lib):
        assert lib.galois_elt(16, 0, 1) == 2 ** 17 - 1
        assert lib.galois_elt(16, -1, 0) == 5            # left rotation by 1
        assert lib.galois_elt(16, 0, 0) == 1


def test_product_path_fails_loudly_without_extension(monkeypatch, tmp_path):
    import aes_xor_fhe._abi as abi
    monkeypatch.setattr(abi, "_PRODUCT", None)
    monkeypatch.setenv("AESFHE_LIB", str(tmp_path / "missing.so"))
    with pytest.raises(RuntimeError, match="HIP extension not found"):
        abi.load_product()


def test_load_product_refuses_another_backend():
    """AESFHE_LIB may select another build of the product, never another backend: pointing it at
    the CPU oracle must fail loudly instead of letting the GPU tests / bench run the checker."""
    import os
    import subprocess
    import sys
    from conftest import ORACLE_SO, PKG, _build_oracle
    _build_oracle()
    env = dict(os.environ, AESFHE_LIB=str(ORACLE_SO), PYTHONPATH=str(PKG))
    r = subprocess.run([sys.executable, "-c", "from aes_xor_fhe._abi import load_product; load_product()"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0 and "not the product" in r.stderr, r.stderr[-2000:]
