"""Time bit-mode and general bootstrapping on the HIP engine at N = 2^16, L = 30 (44-bit scale).

python tools/boot_bench.py [--log-n 16] [--reps 3]  -> one JSON line per mode."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aes-fhe_amd"))

import numpy as np  # noqa: E402

from aes_xor_fhe.bootstrap import Bootstrapper  # noqa: E402
from aes_xor_fhe.fhe import Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--max-level", type=int, default=30)
    ap.add_argument("--scale-bits", type=int, default=44)
    ap.add_argument("--special-primes", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--general", action="store_true")
    ap.add_argument("--batch", type=int, default=1, help="ciphertext pairs per call")
    ap.add_argument("--phases", action="store_true", help="also time each bootstrap phase")
    ap.add_argument("--baby-scale", type=int, default=2, help="BSGS baby steps x this (lazy mode)")
    ap.add_argument("--stc-baby-scale", type=float, default=None, help="the same for the SlotToCoeff maps")
    ap.add_argument("--eager", action="store_true", help="rotate_hoisted + dot_pt + galois linear maps")
    ap.add_argument("--no-opt", action="store_true", help="bit mode without bits_opt (c_in multiply, depth-6 Chebyshev)")
    ap.add_argument("--cts-groups", type=int, default=None, help="CoeffToSlot maps (default: groups = 3)")
    ap.add_argument("--digit-primes", type=int, default=0, help="key-switch digit width (0: K)")
    a = ap.parse_args()
    e = Engine(log_n=a.log_n, max_level=a.max_level, special_primes=a.special_primes, scale_bits=a.scale_bits, seed=3,
               digit_primes=a.digit_primes)
    sk = e.create_secret_key(1)
    pk = e.create_public_key(sk)
    t = time.time()
    bs = Bootstrapper(e, sk, e.create_relinearization_key(sk), lazy=not a.eager, baby_scale=a.baby_scale, stc_baby_scale=a.stc_baby_scale,
                      bits_opt=not a.no_opt, cts_groups=a.cts_groups)
    e.synchronize()
    setup = time.time() - t
    n = e.slot_count
    rng = np.random.default_rng(5)
    bits = [rng.choice([-1.0, 1.0], n) for _ in range(2)]
    cts = [e.concat([e.encrypt(b, pk, level=3)] * a.batch) for b in bits]
    bs.bootstrap_bits(*cts)
    e.synchronize()
    ts = []
    for _ in range(a.reps):
        t = time.time()
        ya, yb = bs.bootstrap_bits(*cts)
        e.synchronize()
        ts.append(time.time() - t)
    err = max(np.abs(np.atleast_2d(e.decrypt(y, sk)) - b).max() for y, b in zip((ya, yb), bits))
    print(json.dumps({"mode": "bits", "log_n": a.log_n, "max_level": a.max_level,
                      "special_primes": a.special_primes, "scale_bits": a.scale_bits, "setup_s": round(setup, 2),
                      "ms_per_call": round(1e3 * min(ts), 1), "cts_per_call": 2 * a.batch,
                      "ms_per_ct": round(1e3 * min(ts) / (2 * a.batch), 2),
                      "out_level": ya.level, "max_err": float(err), "bits_opt": bs.bits_opt,
                      "rotation_keys": len(bs.rot), "cts_groups": bs.cts_groups,
                      "digit_primes": e.digit_primes}), flush=True)
    if a.phases:
        def timed(fn, *xs):
            e.synchronize()
            t0 = time.time()
            r = fn(*xs)
            e.synchronize()
            return r, 1e3 * (time.time() - t0)
        ph = {}
        x, ph["combine"] = timed(lambda p, q: e.add(p, e.multiply_i(q, 1)), *cts)
        for i, plan in enumerate(bs.stc_bits):
            x, ph[f"stc{i}"] = timed(bs.linear, x, plan)
        c, ph["to_sparse"] = timed(e.switch_key, x, bs.to_sparse)
        c, ph["mod_raise"] = timed(e.mod_raise, c, bs.L)
        c, ph["from_sparse"] = timed(e.switch_key, c, bs.from_sparse)
        if not bs.bits_opt:
            c, ph["c_in"] = timed(lambda v: e.materialize(e.multiply(v, bs.c_in)), c)
        for i, plan in enumerate(bs.cts_bits):
            c, ph[f"cts{i}"] = timed(bs.linear, c, plan)
        (xr, xi), ph["conj"] = timed(lambda v: (lambda cj: (e.add(v, cj), e.multiply_i(e.subtract(v, cj), -1)))(e.conjugate(v, bs.cjk)), c)
        xx, ph["concat"] = timed(lambda p, q: e.concat([p, q]), xr, xi)
        ch, ph["chebyshev"] = timed(bs.chebyshev_opt if bs.bits_opt else bs.chebyshev, xx, bs.cheb_bits)
        y = ch
        for i in range(bs.bits_r):
            y, ph[f"double{i}"] = timed(lambda v: (lambda sq: e.add(e.add(sq, sq), -1.0))(e.multiply(v, v, bs.rlk)), y)
        tot = sum(ph.values())
        print(json.dumps({"phases_ms": {k: round(v, 2) for k, v in ph.items()}, "total_ms": round(tot, 1)}), flush=True)
    if a.general:
        z = rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)
        c = e.encrypt(z, pk, level=0)
        bs.bootstrap(c)
        e.synchronize()
        t = time.time()
        y = bs.bootstrap(c)
        e.synchronize()
        dt = time.time() - t
        print(json.dumps({"mode": "general", "ms_per_bootstrap": round(1e3 * dt, 1),
                          "out_level": y.level,
                          "max_err": float(np.abs(e.decrypt(y, sk) - z).max())}), flush=True)


if __name__ == "__main__":
    main()
