"""Shared fixtures.  `-m gpu` tests need an MI355X and the built HIP extension; everything
else runs on CPU against the oracle (test infrastructure, oracle/) and the host codec."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "aes-fhe_amd"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

ORACLE_SO = ROOT / "oracle" / "_build" / "liboracle_ckks.so"
PRODUCT_SO = PKG / "build" / "libaesfhe.so"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _build_oracle():
    if not ORACLE_SO.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    return ORACLE_SO


@pytest.fixture(scope="session")
def oracle_lib():
    from aes_xor_fhe._abi import Lib
    return Lib(_build_oracle())


@pytest.fixture(scope="session")
def product_lib():
    from aes_xor_fhe._abi import PRODUCT_BACKEND, load_product
    lib = load_product()
    assert lib.backend == PRODUCT_BACKEND, lib.backend
    return lib


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
