"""Nibble split of a byte vector (reference: byte_split_nibble.py:3-21)."""
import numpy as np


def split_nibbles(flatten: np.ndarray):
    """uint8 (N,) -> (upper, lower) nibble vectors, each uint8 in 0..15."""
    b = np.asarray(flatten).astype(np.uint8, copy=False)
    return (b >> 4).astype(np.uint8), (b & 0x0F).astype(np.uint8)
