#!/usr/bin/env python3
"""General-mode (complex slots) bootstrap precision: Engine.bootstrap as the reference calls it
(xor_service.py:120-129), for random complex slots of modulus <= 1 and for zeta-16 / zeta-256
roots of unity (python tools/boot_general_diag.py log_n L K scale base_bits [hw])."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "aes-fhe_amd"))
from aes_xor_fhe.fhe import Engine  # noqa: E402

log_n, L, K, sb, bb = (int(x) for x in sys.argv[1:6])
e = Engine(log_n=log_n, max_level=L, special_primes=K, scale_bits=sb, base_bits=bb, seed=3)
sk = e.create_secret_key(1)
pk = e.create_public_key(sk)
rlk, cjk = e.create_relinearization_key(sk), e.create_conjugation_key(sk)
bk = e.create_bootstrap_key(sk)
if len(sys.argv) > 6:
    from aes_xor_fhe.bootstrap import Bootstrapper
    bk._bs = Bootstrapper(e, sk, rlk, cjk, hw=int(sys.argv[6]))
n = e.slot_count
rng = np.random.default_rng(1)
cases = {"uniform": rng.uniform(-1, 1, n) * 0.7 + 0.7j * rng.uniform(-1, 1, n),
         "zeta16": np.exp(-2j * np.pi * rng.integers(0, 16, n) / 16),
         "zeta256": np.exp(-2j * np.pi * rng.integers(0, 256, n) / 256)}
for name, z in cases.items():
    ct = e.encrypt(z, pk, level=0)
    t0 = time.time()
    out = e.bootstrap(ct, rlk, cjk, bk)
    e.synchronize()
    err = np.abs(e.decrypt(out, sk) - z)
    print(f"N=2^{log_n} L={L} K={K} scale={sb} q0 bits={bb}: {name:8s} level {out.level} "
          f"max err {err.max():.3e} rms {np.sqrt((err ** 2).mean()):.3e} ({time.time() - t0:.2f}s)", flush=True)
