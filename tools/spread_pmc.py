"""Level-downs and constant products at N = 2^16, L = 30 (dev tool for the PMC passes of the
spread-fused column pass k_nttf_fwd_cols_spread): B ciphertexts level-downed one
level at a time from 30 to 20 (SPREAD 2) and multiplied by a constant (SPREAD 1, plain rescale).
  rocprofv3 --pmc FETCH_SIZE --kernel-trace ... -- python tools/spread_pmc.py [B]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "aes-fhe_amd"))

import numpy as np  # noqa: E402

from aes_xor_fhe.fhe import Engine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    e = Engine(log_n=16, max_level=30, special_primes=10, scale_bits=40, seed=3)
    sk = e.create_secret_key(1)
    pk = e.create_public_key(sk)
    z = np.random.default_rng(1).uniform(-1, 1, (B, e.slot_count))
    c = e.encrypt(z, pk)
    x = c
    for lv in range(29, 19, -1):
        x = e.level_down(x, lv)
    y = c
    for _ in range(4):
        y = e.multiply(y, 0.5)
    e.synchronize()
    err = max(np.abs(e.decrypt(x, sk) - z).max(), np.abs(e.decrypt(y, sk) - z / 16).max())
    print("levels", x.level, y.level, "max err", err)
    assert err < 1e-4


if __name__ == "__main__":
    main()
