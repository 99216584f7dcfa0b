#!/usr/bin/env python3
"""Where the reference harness's full_round (new.py:186-227, bench reference_harness leg) spends its
time on the GPU: nibble split, Zeta-16 encode, encrypt x4, xor_cipher x2, decrypt x2, recombine,
each synchronised and timed alone (median of 5 after a warm-up)."""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "aes-fhe_amd"))
from aes_xor_fhe.new import AESFHERound, split_nibbles  # noqa: E402
from aes_xor_fhe.xor_service import EngineWrapper, XORConfig, XORService, ZetaEncoder  # noqa: E402

w = EngineWrapper(XORConfig(engine_kwargs=dict(seed=1)))
e = w.engine
svc = XORService(w)
ark = AESFHERound(w, svc)
rng = np.random.default_rng(1)
state = rng.integers(0, 256, 32768, dtype=np.uint8)
key = rng.integers(0, 256, 32768, dtype=np.uint8)
ark.full_round(state, key)
T = {}


def tm(name, fn):
    e.synchronize()
    t = time.perf_counter()
    r = fn()
    e.materialize(r)
    e.synchronize()
    T.setdefault(name, []).append(time.perf_counter() - t)
    return r


for _ in range(5):
    t0 = time.perf_counter()
    s_hi, s_lo = tm("split", lambda: split_nibbles(state))
    k_hi, k_lo = split_nibbles(key)
    z = tm("zeta_encode x4", lambda: [ZetaEncoder.to_zeta(v, modulus=16) for v in (s_hi, s_lo, k_hi, k_lo)])
    cts = tm("encrypt x4", lambda: [w.encrypt(v) for v in z])
    outs = tm("xor_cipher x2", lambda: [svc.xor_cipher(cts[0], cts[2]), svc.xor_cipher(cts[1], cts[3])])
    dec = tm("decrypt x2", lambda: [w.decrypt(o) for o in outs])
    tm("zeta_decode+recombine", lambda: ((ZetaEncoder.from_zeta(dec[0], modulus=16).astype(np.uint8) << 4)
                                         | ZetaEncoder.from_zeta(dec[1], modulus=16).astype(np.uint8)))
    T.setdefault("total (split steps)", []).append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    ark.full_round(state, key)
    T.setdefault("full_round", []).append(time.perf_counter() - t0)
for k, v in T.items():
    print(f"{k:28s} {1e3 * float(np.median(v)):8.2f} ms")
