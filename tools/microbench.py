"""Per-primitive timings of the HIP engine at BASELINE.json's parameters (N=2^16, L=30).

Development tool (not the bench contract): prints one line per primitive with the average
wall time per call over a batch of B ciphertexts, plus the NTT roofline figure.
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "aes-fhe_amd"))
from aes_xor_fhe.fhe import Engine  # noqa: E402


def timeit(eng, fn, reps):
    fn()
    eng.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    eng.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--level", type=int, default=30)
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    eng = Engine(log_n=a.log_n, max_level=a.level, special_primes=8)
    N = 1 << a.log_n
    for nl in (31, 31 * 8):
        f, i = (np.zeros(1), np.zeros(1))
        import ctypes as C
        fm, im = C.c_double(), C.c_double()
        eng._check(eng._lib.bench_ntt(eng._h, nl, 20, C.byref(fm), C.byref(im)))
        gbs = 16.0 * N * nl / (fm.value * 1e-3) / 1e9
        gbsi = 16.0 * N * nl / (im.value * 1e-3) / 1e9
        print(f"ntt limbs={nl:4d} fwd {fm.value*1e3:9.1f} us ({gbs:7.1f} GB/s alg)  "
              f"inv {im.value*1e3:9.1f} us ({gbsi:7.1f} GB/s alg)")
    sk = eng.create_secret_key()
    pk = eng.create_public_key(sk)
    t0 = time.perf_counter()
    rlk = eng.create_relinearization_key(sk)
    cjk = eng.create_conjugation_key(sk)
    rot = eng.create_rotation_key(sk)
    eng.synchronize()
    print(f"keygen relin+conj {1e3*(time.perf_counter()-t0):.1f} ms")
    rng = np.random.default_rng(0)
    for B in a.batch:
        z = np.exp(-2j * np.pi * rng.integers(0, 16, (B, eng.slot_count)) / 16)
        ct = eng.encrypt(z if B > 1 else z[0], pk)
        ct2 = eng.encrypt(z if B > 1 else z[0], pk)
        res = {}
        res["mul"], m = timeit(eng, lambda: eng.multiply(ct, ct2, rlk), a.reps)
        res["tensor"], _ = timeit(eng, lambda: eng._call_ct(eng._lib.tensor, ct._h, ct2._h), a.reps)
        t3 = eng._call_ct(eng._lib.tensor, ct._h, ct2._h)
        res["relin"], _ = timeit(eng, lambda: eng.relinearize(t3, rlk), a.reps)
        res["rescale"], _ = timeit(eng, lambda: eng.rescale(ct), a.reps)
        res["rotate1"], _ = timeit(eng, lambda: eng.rotate(ct, rot, -1), a.reps)
        res["conj"], _ = timeit(eng, lambda: eng.conjugate(ct, cjk), a.reps)
        res["mul_const"], _ = timeit(eng, lambda: eng.multiply(ct, 0.3 + 0.1j), a.reps)
        res["add"], _ = timeit(eng, lambda: eng.add(ct, ct2), a.reps)
        pb = eng.make_power_basis(ct, 8, rlk)
        res["lincomb8"], _ = timeit(eng, lambda: eng.lincomb(pb, [0.1] * 8), a.reps)
        res["dot4"], _ = timeit(eng, lambda: eng.dot(pb[:4], pb[4:], rlk), a.reps)
        res["power_basis8"], _ = timeit(eng, lambda: eng.make_power_basis(ct, 8, rlk), max(1, a.reps // 2))
        print(f"B={B}: " + "  ".join(f"{k}={v:.2f}ms" for k, v in res.items()))
        err = np.abs(eng.decrypt(m, sk) - (z * z if B > 1 else z[0] ** 2)).max()
        print(f"  mul decrypt err {err:.2e}")


if __name__ == "__main__":
    main()
