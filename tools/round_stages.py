"""Per-step wall time of the AES round on the GPU (dev tool)."""
import sys, time
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "aes-fhe_amd"))
from aes_xor_fhe.fhe import Engine
from aes_xor_fhe.aes_round import AESRoundEngine
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
e = Engine(log_n=16, max_level=30, special_primes=8)
sk = e.create_secret_key(1)
R = AESRoundEngine(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk), e.create_conjugation_key(sk))
blocks = np.random.default_rng(0).integers(0, 256, (B, R.n_blk, 16), dtype=np.uint8)
h, l = R.encrypt_blocks(blocks)
key = R.encrypt_round_key(np.arange(16, dtype=np.uint8))
R.round(h, l, key)
tm = {}
for _ in range(2):
    R.round(h, l, key, timings=tm)
tm.pop("start", None)
tot = sum(tm.values())
for k, v in tm.items():
    print(f"{k:18s} {v/2*1e3:8.1f} ms  {100*v/tot:5.1f}%")
print(f"total {tot/2*1e3:.1f} ms/round, B={B}")
