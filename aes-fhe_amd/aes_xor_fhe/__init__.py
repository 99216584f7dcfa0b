"""aes_xor_fhe -- MI355X-native restatement of songhayeong/aes-fhe's homomorphic AES services.

The package name mirrors the reference's import root (its modules import
``aes_xor_fhe.<module>``, e.g. sbox/sbox_service.py:27-28), so the reference's call sites and
tests read unchanged.  All homomorphic arithmetic runs in the HIP engine behind
include/aesfhe.h (see fhe.py).
"""
__all__ = ["fhe"]
