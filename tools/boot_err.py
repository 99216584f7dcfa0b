"""Bit-mode bootstrap output error statistics (max, mean bias, std per bit value) for EvalMod
variants, at the bench parameters (dev tool; python tools/boot_err.py [noise])."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aes-fhe_amd"))

import numpy as np  # noqa: E402

from aes_xor_fhe.bootstrap import Bootstrapper  # noqa: E402
from aes_xor_fhe.fhe import Engine  # noqa: E402

noise = float(sys.argv[1]) if len(sys.argv) > 1 else 5e-3
e = Engine(log_n=16, max_level=30, special_primes=10, scale_bits=40, seed=3)
sk = e.create_secret_key(1)
pk = e.create_public_key(sk)
rlk = e.create_relinearization_key(sk)
n = e.slot_count
rng = np.random.default_rng(5)
a, b = rng.choice([-1.0, 1.0], n), rng.choice([-1.0, 1.0], n)
na, nb = noise * rng.standard_normal(n), noise * rng.standard_normal(n)
ca, cb = e.encrypt(a + na, pk, level=3), e.encrypt(b + nb, pk, level=3)
for kw in (dict(bits_deg=29, bits_r=3), dict(bits_deg=15, bits_r=4), dict(bits_opt=False)):
    bs = Bootstrapper(e, sk, rlk, **kw)
    ya, yb = bs.bootstrap_bits(ca, cb)
    out = {"variant": kw, "level": ya.level}
    for name, y, v, nz in (("a", ya, a, na), ("b", yb, b, nb)):
        d = (np.real(e.decrypt(y, sk)) - v) * v  # signed error towards zero: negative = shrink
        out[name] = {"max": float(np.abs(d).max()), "mean": float(d.mean()), "std": float(d.std()),
                     "mean_plus": float(d[v > 0].mean()), "mean_minus": float(d[v < 0].mean()),
                     "resid_vs_ideal": float(np.abs(d + (1 - np.cos(np.pi * nz / 2))).max())}
    print(json.dumps(out), flush=True)
    del bs
