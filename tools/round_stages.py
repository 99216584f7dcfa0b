"""Per-step wall time of the AES round on the GPU (dev tool).

    python tools/round_stages.py [rows|bytes] [B]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "aes-fhe_amd"))
from aes_xor_fhe.fhe import Engine  # noqa: E402

layout = sys.argv[1] if len(sys.argv) > 1 else "rows"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
import os
e = Engine(log_n=16, max_level=30, special_primes=8, scale_bits=int(os.environ.get("SCALE_BITS", 40)))
sk = e.create_secret_key(1)
args = (e, sk, e.create_public_key(sk), e.create_relinearization_key(sk), e.create_conjugation_key(sk))
if layout == "rows":
    from aes_xor_fhe.aes_round_bits import AESRowRound
    R = AESRowRound(*args)
else:
    from aes_xor_fhe.aes_round import AESRoundEngine
    R = AESRoundEngine(*args)
blocks = np.random.default_rng(0).integers(0, 256, (B, R.n_blk, 16), dtype=np.uint8)
st = R.encrypt_blocks(blocks)
key = R.encrypt_round_key(np.arange(16, dtype=np.uint8))
run = (lambda **kw: R.round(st, key, **kw)) if layout == "rows" else (lambda **kw: R.round(*st, key, **kw))
run()
tm = {}
for _ in range(2):
    run(timings=tm)
tm.pop("start", None)
tot = sum(tm.values())
for k, v in tm.items():
    print(f"{k:18s} {v/2*1e3:8.1f} ms  {100*v/tot:5.1f}%")
print(f"{layout} scale {e.scales[-1]:.3g}: total {tot/2*1e3:.1f} ms/round, B={B}, {B*R.n_blk/(tot/2):.0f} blocks/s")
