#!/usr/bin/env python3
"""Ten AES rounds in the bench's config-4 shape (sliced, 16 sets, alpha 12, 5/3-map refreshes,
4 pairs per call) under a fixed seed, decrypting the whole state after every refresh and round:
prints the first step with a wrong bit, the decoded margin (min |v|, max ||v| - 1|) per step,
and a hash of the final state's decrypted bits.  Diagnostic tool (AESFHE_LIB selects the
library).  python tools/aes10_trace.py SEED [SETS]"""
import hashlib
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "aes-fhe_amd"))
from aes_xor_fhe import aes_tables as T  # noqa: E402
from aes_xor_fhe.aes_round_bits import AESSlicedRound  # noqa: E402
from aes_xor_fhe.bootstrap import Bootstrapper  # noqa: E402
from aes_xor_fhe.fhe import Engine, widest_digits  # noqa: E402

seed = int(sys.argv[1])
nsets = int(sys.argv[2]) if len(sys.argv) > 2 else 16
cfg = dict(log_n=16, max_level=30, special_primes=10, scale_bits=40)
e = Engine(seed=seed, digit_primes=widest_digits(**cfg), **cfg)
sk = e.create_secret_key()
rlk = e.create_relinearization_key(sk)
R = AESSlicedRound(e, sk, e.create_public_key(sk), rlk)
bs = [Bootstrapper(e, sk, rlk, cts_groups=g) for g in (5, 3)]
L0 = R.fresh_level(e.max_level, bs)
klv = R.key_levels(L0, bs)
rng = np.random.default_rng(seed)
key = rng.integers(0, 256, 16, dtype=np.uint8)
blocks = rng.integers(0, 256, (nsets, R.n_blk, 16), dtype=np.uint8)
rks = T.expand_key(key)
keys = [R.encrypt_round_key(k, level=lv) for k, lv in zip(rks, klv)]


def check(S, want, label):
    got = R.decrypt_blocks(S, nsets)
    vals = np.concatenate([np.real(np.atleast_2d(e.decrypt(c, sk))).ravel() for row in S for c in row])
    bad = np.any(got != want, axis=-1)
    print(f"{label:28s} level {min(c.level for row in S for c in row):2d}  wrong blocks {int(bad.sum()):4d} "
          f"bits {int(np.unpackbits(got ^ want).sum()):5d}  min|v| {np.abs(vals).min():.4f}  "
          f"max||v|-1| {np.abs(np.abs(vals) - 1).max():.4f}", flush=True)
    if bad.any():
        s, b = np.argwhere(bad)[0]
        print(f"   first wrong: set {s} block {b} bytes {np.nonzero(got[s, b] != want[s, b])[0].tolist()}", flush=True)
    return got


t0 = time.time()
state = blocks ^ rks[0]
S = R.add_round_key(R.encrypt_blocks(blocks, level=L0), keys[0])
check(S, state, "ARK0")
since, nref = 0, 0
stc = len(bs[0].stc_bits)
for rnd in range(1, 11):
    final = rnd == 10
    lvl = min(c.level for row in S for c in row)
    if R.needs_refresh(lvl, final, since, nref > 0, stc):
        S, b, cleaned = R.refresh_step(S, rnd, lvl, since, nref > 0, bs, 4)
        nref += 1
        since = 0
        check(S, state, f"refresh {nref} ({b.cts_groups} maps{', cleaned' if cleaned else ''})")
    if final:
        S = R.final_round(S, keys[rnd])
        state = T.shift_rows(T.sub_bytes(state)) ^ rks[rnd]
    else:
        S = R.round(S, keys[rnd])
        state = T.aes_round(state, rks[rnd])
    since += 1
    got = check(S, state, f"round {rnd}")
assert np.array_equal(state, T.encrypt_block(blocks, key))
print("final hash", hashlib.sha256(got.tobytes()).hexdigest()[:16], "ok", bool(np.array_equal(got, state)),
      f"{time.time() - t0:.0f} s", flush=True)
