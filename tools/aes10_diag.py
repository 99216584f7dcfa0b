#!/usr/bin/env python3
"""Step-by-step full AES-128 on the GPU with a decrypt-and-compare after every step
(python tools/aes10_diag.py log_n L K [scale])."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "aes-fhe_amd"))
from aes_xor_fhe import aes_tables as T  # noqa: E402
from aes_xor_fhe.aes_round_bits import AESRowRound  # noqa: E402
from aes_xor_fhe.bootstrap import Bootstrapper  # noqa: E402
from aes_xor_fhe.fhe import Engine  # noqa: E402

log_n, L, K = (int(x) for x in sys.argv[1:4])
sb = int(sys.argv[4]) if len(sys.argv) > 4 else 40
e = Engine(log_n=log_n, max_level=L, special_primes=K, scale_bits=sb, seed=17)
sk = e.create_secret_key()
rlk = e.create_relinearization_key(sk)
R = AESRowRound(e, sk, e.create_public_key(sk), rlk)
bs = Bootstrapper(e, sk, rlk)
key = np.arange(16, dtype=np.uint8)
rks = T.expand_key(key)
keys = [R.encrypt_round_key(k) for k in rks]
blocks = np.random.default_rng(5).integers(0, 256, (1, R.n_blk, 16), dtype=np.uint8)
st = R.encrypt_blocks(blocks)


def check(name, S, want):
    got = R.decrypt_blocks(S)
    lv = min(c.level for row in S for c in row)
    errs = []
    for r in range(4):
        for j in range(8):
            v = np.real(np.atleast_2d(e.decrypt(S[r][j], sk)))
            errs.append(np.abs(np.abs(v) - 1).max())
    print(f"{name:>12}: level {lv:2d} wrong bytes {(got != want).mean():.4f} max | |v|-1 | {max(errs):.2e}", flush=True)


plain = blocks ^ rks[0]
S = R.add_round_key(st, keys[0])
check("ark0", S, plain)
stc = len(bs.stc_bits)
since = 0
nref = 0
for rnd in range(1, 11):
    final = rnd == 10
    lvl = min(c.level for row in S for c in row)
    if R.needs_refresh(lvl, final, since, nref > 0, stc):
        since = 0
        nref += 1
        S = R.refresh(S, bs)
        check(f"refresh<{rnd}", S, plain)
    if final:
        plain = T.shift_rows(T.sub_bytes(plain)) ^ rks[rnd]
        S = R.final_round(S, keys[rnd])
    else:
        plain = T.aes_round(plain, rks[rnd])
        S = R.round(S, keys[rnd])
    since += 1
    check(f"round {rnd}", S, plain)
