"""Byte-block / AES-state helpers and the Zeta (root-of-unity) codec.

Restates the reference's utils.py (utils.py:11-90) with identical behaviour:
  * a 16-byte block maps to the 4x4 AES state column-major (FIPS-197 3.4);
  * ``zeta_encode(k, m)`` = zeta_m ** (k mod m) with zeta_m = exp(-2 pi i / m), computed as a
    power of the primitive root (utils.py:40-47).  NB: the reference has a second encoder,
    ``ZetaEncoder.to_zeta`` = exp(-2 pi i k / m) (xor_service.py:137-139), whose values differ
    in the last bits; both are kept, bit-compatible with their originals;
  * ``zeta_decode`` rounds the phase: k = rint(-angle(z) m / 2 pi) mod m (utils.py:50-59).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

BLOCK = 16


def bytes_to_state(block: bytes) -> np.ndarray:
    if len(block) != BLOCK:
        raise ValueError("Block length must be 16 bytes")
    return np.frombuffer(block, dtype=np.uint8).reshape((4, 4), order="F")


def state_to_bytes(state: np.ndarray) -> bytes:
    if state.shape != (4, 4):
        raise ValueError("State must be a 4x4 array")
    return state.reshape(BLOCK, order="F").astype(np.uint8).tobytes()


def zeta_encode(arr: Sequence[int], modulus: int = 16) -> np.ndarray:
    k = np.asarray(arr, dtype=np.int64) % modulus
    root = np.exp(-2j * np.pi / modulus)
    return root ** k


def zeta_decode(z_arr: np.ndarray, modulus: int = 16) -> np.ndarray:
    k = -np.angle(z_arr) * modulus / (2 * np.pi)
    return np.mod(np.rint(k), modulus).astype(np.uint8)


def chunk_bytes(data: bytes, block_size: int = BLOCK) -> list:
    return [data[i:i + block_size] for i in range(0, len(data), block_size)]


def pkcs7_pad(block: bytes, block_size: int = BLOCK) -> bytes:
    n = block_size - len(block) % block_size
    return block + bytes([n]) * n


def pkcs7_unpad(data: bytes) -> bytes:
    if not data:
        return data
    n = data[-1]
    if not 1 <= n <= len(data) or data[-n:] != bytes([n]) * n:
        raise ValueError("Invalid PKCS#7 padding")
    return data[:-n]
