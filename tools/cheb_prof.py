"""Kernel profile of the bit-mode EvalMod (Chebyshev + double angles) alone, at the bench's
bootstrap shape: B = 16 ciphertexts at level L - 1 - groups (run under rocprofv3 --stats).
python tools/cheb_prof.py [--batch 16] [--reps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aes-fhe_amd"))

import numpy as np  # noqa: E402

from aes_xor_fhe.bootstrap import Bootstrapper  # noqa: E402
from aes_xor_fhe.fhe import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
e = Engine(log_n=16, max_level=30, special_primes=10, scale_bits=40, seed=3)
sk = e.create_secret_key(1)
pk = e.create_public_key(sk)
bs = Bootstrapper(e, sk, e.create_relinearization_key(sk))
lv = e.max_level - 1 - len(bs.cts)
x = e.encrypt(np.random.default_rng(1).uniform(-1, 1, (a.batch, e.slot_count)), pk, level=lv)
bs.evalmod(x, bits=True)
e.synchronize()
t = time.time()
for _ in range(a.reps):
    y = bs.evalmod(x, bits=True)
e.synchronize()
print(f"evalmod B={a.batch} level {lv}: {1e3 * (time.time() - t) / a.reps:.1f} ms per call, out level {y.level}", flush=True)
