#!/usr/bin/env python3
"""Benchmark: homomorphic AES-128 rounds on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]

One *step* = one full middle AES-128 round (ShiftRows -> SubBytes -> MixColumns ->
AddRoundKey) at N = 2^16, L = 30 over a batch of B ciphertext sets per GPU.  Default layout
"rows" (aes_xor_fhe.aes_round_bits.AESRowRound): a set is 4 state rows x 8 +-1 bit ciphertexts
carrying 8192 AES blocks; layout "bytes" (aes_xor_fhe.aes_round.AESRoundEngine): a set is one
byte-major (hi, lo) Zeta-16 nibble pair carrying 2048 blocks.  Inputs (encrypted synthetic
random AES states) and the encrypted round key are resident in HBM before the timed region.

Multi-GPU (torchrun, one process per GPU): every rank runs its own shard of ciphertexts --
the path is embarrassingly parallel (no data-path collective), so the scaling is weak.  The
barrier and the max-over-ranks reduction of the step time use torch.distributed (gloo).

Printed on rank 0: ONE JSON line with metric/value/... plus
  roofline     -- the NTT kernels (dominant family): algorithmic bytes per launch / average
                  launch duration, from HIP events recorded on the engine stream over the
                  timed region; peak 8 TB/s HBM3E (MI355X_MICROARCH.md);
  cpu_baseline -- the CPU oracle (oracle/, a C restatement of the same engine) running the
                  same round on a bounded sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "aes-fhe_amd"))

PEAK_HBM_GBS = 8000.0
METRIC = "AES-128 blocks/sec (homomorphic full round) at N=2^16, L=30; 1/2/4/8 MI355X"


PMC_FILE = ROOT / "profiles" / "r01" / "pmc" / "ntt_traffic.json"
PMC_NOTE = ("HBM bytes per NTT launch = algorithmic bytes x the HBM/algorithmic ratio measured by "
            "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 calibration) + WRITE_SIZE on the same NTT kernels "
            "at the same parameters (profiles/r01/pmc/ntt_traffic.json)")


def traffic_per_launch(alg_bytes):
    """HBM bytes per NTT launch from the committed PMC measurement (None if absent)."""
    try:
        ratio = json.loads(PMC_FILE.read_text())["traffic_over_alg"]
    except (OSError, ValueError, KeyError):
        return None
    return round(alg_bytes * ratio)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32, help="ciphertext sets per GPU per step (8192 blocks each)")
    ap.add_argument("--layout", choices=("rows", "bytes"), default="rows")
    ap.add_argument("--log-n", type=int, default=16)
    ap.add_argument("--max-level", type=int, default=30)
    ap.add_argument("--special-primes", type=int, default=10,
                    help="K special primes = key-switch digit size alpha (dnum = ceil((L+1)/K))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--check", action="store_true", help="decrypt and verify against FIPS-197")
    ap.add_argument("--aes10-ppc", type=int, default=0,
                    help="bit-ciphertext pairs per bootstrap call (0: 32 / aes10-batch)")
    ap.add_argument("--aes10-batch", type=int, default=8,
                    help="ciphertext sets for the full 10-round AES-128 measurement (0: skip)")
    return ap.parse_args()


class RoundDriver:
    """Uniform face over the two round implementations: encrypt / step / decrypt."""

    def __init__(self, layout, eng, sk, pk, rlk, cjk, rotation_keys=None):
        if layout == "rows":
            from aes_xor_fhe.aes_round_bits import AESRowRound
            self.R = AESRowRound(eng, sk, pk, rlk, cjk, rotation_keys=rotation_keys)
        else:
            from aes_xor_fhe.aes_round import AESRoundEngine
            self.R = AESRoundEngine(eng, sk, pk, rlk, cjk, rotation_keys=rotation_keys)
        self.layout = layout
        self.n_blk = self.R.n_blk

    def encrypt(self, blocks):
        st = self.R.encrypt_blocks(blocks)
        return st if self.layout == "rows" else tuple(st)

    def key(self, rk):
        return self.R.encrypt_round_key(rk)

    def round(self, st, key):
        return self.R.round(st, key) if self.layout == "rows" else self.R.round(st[0], st[1], key)

    def sub_bytes(self, st):
        """Bounded CPU sample: SubBytes of the first state row (rows) / the nibble pair (bytes)."""
        if self.layout == "rows":
            return self.R.sub_bytes(st[:1])
        return self.R.sub_bytes(st[0], st[1])

    def decrypt(self, st):
        return self.R.decrypt_blocks(st) if self.layout == "rows" else self.R.decrypt_blocks(*st)


def setup_engine(args, device):
    from aes_xor_fhe.fhe import Engine
    eng = Engine(log_n=args.log_n, max_level=args.max_level, special_primes=args.special_primes, device_id=device)
    sk = eng.create_secret_key(1)
    pk = eng.create_public_key(sk)
    rlk = eng.create_relinearization_key(sk)
    cjk = eng.create_conjugation_key(sk)
    drv = RoundDriver(args.layout, eng, sk, pk, rlk, cjk)
    drv.keys = (sk, rlk, cjk)
    return eng, drv


def aes128_full(args, eng, drv, rank, barrier, dist):
    """Full AES-128 (ARK0 + 10 rounds, FIPS-197 5.1) with bit-mode bootstrapping on the rows
    layout: a warm-up encryption of the same shape (bootstrap plaintexts, device pool), then one
    timed encryption of args.aes10_batch ciphertext sets (x 8192 blocks at N = 2^16)."""
    import torch

    from aes_xor_fhe import aes_tables as T
    from aes_xor_fhe.bootstrap import Bootstrapper
    R = drv.R
    sk, rlk, cjk = drv.keys
    t0 = time.perf_counter()
    bs = Bootstrapper(eng, sk, rlk, cjk)
    eng.synchronize()
    setup_s = time.perf_counter() - t0
    key = np.random.default_rng(25073103).integers(0, 256, 16, dtype=np.uint8)
    keys = [R.encrypt_round_key(rk) for rk in T.expand_key(key)]
    rng = np.random.default_rng(2000 + rank)
    nb = args.aes10_batch
    ppc = args.aes10_ppc or max(1, 32 // nb)  # ~32 ciphertexts per Bootstrapper call
    # warm-up of the same shape: materialises the bootstrap plaintexts and fills the device pool
    # with every buffer size of the run, so the timed run makes no hipMalloc
    warm = R.encrypt_aes128(R.encrypt_blocks(rng.integers(0, 256, (nb, R.n_blk, 16), dtype=np.uint8)),
                            keys, bs, pairs_per_call=ppc)
    del warm
    blocks = rng.integers(0, 256, (nb, R.n_blk, 16), dtype=np.uint8)
    st = R.encrypt_blocks(blocks)
    tm = {}
    barrier()
    m0 = eng.pool_stats()["mallocs"]
    t0 = time.perf_counter()
    out, nref = R.encrypt_aes128(st, keys, bs, timings=tm, pairs_per_call=ppc)
    barrier()
    el = time.perf_counter() - t0
    timed_mallocs = eng.pool_stats()["mallocs"] - m0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ok = None
    if args.check:
        got = R.decrypt_blocks(out)
        ok = bool(all((got[i] == np.stack([T.encrypt_block(b, key) for b in blocks[i]])).all()
                      for i in range(nb)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return {"metric": "AES-128 blocks/sec (10 rounds incl. bootstrapping)",
            "value": round(nb * R.n_blk * world / el, 2), "unit": "blocks/s",
            "ms": round(el * 1e3, 1), "ciphertext_sets_per_gpu": nb,
            "blocks_per_gpu": nb * R.n_blk, "refreshes": nref,
            "bootstrap_share": round(tm.get("bootstrap", 0.0) / max(el, 1e-9), 3),
            "bootstrap_ms_per_bit_ct": round(1e3 * tm.get("bootstrap", 0.0) / max(nref * 32 * nb, 1), 2),
            "bootstrap_setup_s": round(setup_s, 2), "verified": ok,
            "block_rounds_per_s": round(10 * nb * R.n_blk * world / el, 2),
            "per_round_level_ms": tm.get("per_round"), "pool": eng.pool_stats(),
            "timed_mallocs": timed_mallocs}


def cpu_baseline(args):
    """Oracle (CPU restatement) on a bounded sample of the same workload, scaled to blocks/s.

    The full round at N=2^16 takes minutes on the oracle, so the sample is: SubBytes of one
    state row (rows layout) / nibble pair (bytes layout) at N=2^16, L=30 (timed), scaled by the oracle's own full-round/SubBytes
    time ratio measured at N=2^12, L=30 on the same op sequence (same layout as the GPU run)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import subprocess
    so = ROOT / "oracle" / "_build" / "liboracle_ckks.so"
    if not so.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True, stdout=subprocess.DEVNULL)
    from aes_xor_fhe._abi import Lib
    from aes_xor_fhe.fhe import Engine
    lib = Lib(so)
    threads = int(os.environ.get("OMP_NUM_THREADS", min(16, os.cpu_count() or 1)))
    times = {}
    for log_n in (12, args.log_n):
        eng = Engine(log_n=log_n, max_level=args.max_level, special_primes=args.special_primes, thread_count=threads, _lib=lib)
        sk = eng.create_secret_key(1)
        pk = eng.create_public_key(sk)
        R = RoundDriver(args.layout, eng, sk, pk, eng.create_relinearization_key(sk),
                        eng.create_conjugation_key(sk),
                        rotation_keys={} if log_n != 12 else None)
        rng = np.random.default_rng(log_n)
        blocks = rng.integers(0, 256, (1, R.n_blk, 16), dtype=np.uint8)
        st = R.encrypt(blocks)
        t0 = time.perf_counter()
        R.sub_bytes(st)
        times[(log_n, "sb")] = time.perf_counter() - t0
        if log_n == 12:
            key = R.key(rng.integers(0, 256, 16, dtype=np.uint8))
            t0 = time.perf_counter()
            R.round(st, key)
            times[(log_n, "round")] = time.perf_counter() - t0
    ratio = times[(12, "round")] / times[(12, "sb")]
    est_round = times[(args.log_n, "sb")] * ratio
    n_blk = (1 << (args.log_n - 1)) // (4 if args.layout == "rows" else 16)
    return {
        "value": n_blk / est_round, "unit": "blocks/s", "cores": threads, "kind": "port",
        "sample": (f"oracle SubBytes of 1 row/pair ({args.layout} layout, {n_blk} blocks/set) at N=2^{args.log_n} "
                   f"L={args.max_level}: {times[(args.log_n, 'sb')]:.2f} s, scaled by the oracle's "
                   f"round/SubBytes ratio {ratio:.2f} measured at N=2^12 -> est. {est_round:.1f} s "
                   f"per round"),
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch

    from aes_xor_fhe import aes_tables as T

    # one rank per GPU; more ranks than GPUs (a multi-rank rehearsal on a 1-GPU box) share them
    ndev = torch.cuda.device_count() or 1
    device = local % ndev
    eng, R = setup_engine(args, device)
    if torch.cuda.is_available():
        torch.cuda.set_device(device)
    rng = np.random.default_rng(1000 + rank)
    blocks = rng.integers(0, 256, (args.batch, R.n_blk, 16), dtype=np.uint8)
    rk = np.random.default_rng(25073102).integers(0, 256, 16, dtype=np.uint8)
    st = R.encrypt(blocks)
    key = R.key(rk)
    eng.synchronize()

    def step():
        return R.round(st, key)

    for _ in range(args.warmup):
        out = step()
    eng.synchronize()

    def barrier():
        eng.synchronize()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    import ctypes as C
    eng._check(eng._lib.engine_profile(eng._h, 1 | 2))  # ntt + keyswitch families only
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    barrier()
    elapsed = time.perf_counter() - t0
    n_ntt, ms_ntt, by_ntt = C.c_int64(), C.c_double(), C.c_double()
    eng._check(eng._lib.engine_profile_read(eng._h, b"ntt", C.byref(n_ntt), C.byref(ms_ntt), C.byref(by_ntt)))
    n_ks, ms_ks, by_ks = C.c_int64(), C.c_double(), C.c_double()
    eng._check(eng._lib.engine_profile_read(eng._h, b"keyswitch", C.byref(n_ks), C.byref(ms_ks), C.byref(by_ks)))
    eng._check(eng._lib.engine_profile(eng._h, 0))

    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    round_pool = eng.pool_stats()
    ok = None
    if args.check:
        got = R.decrypt(out)
        ok = bool((got == T.aes_round(blocks, rk)).all())

    aes10 = None
    if args.aes10_batch > 0 and args.layout == "rows":
        # the round's buffers and cached blocks (other sizes) would otherwise crowd the device
        # inside the timed 10-round run; release them between the two workloads
        del st, out
        import gc
        gc.collect()
        eng.pool_trim()
        aes10 = aes128_full(args, eng, R, rank, barrier, dist)

    blocks_per_step = args.batch * R.n_blk * world
    value = blocks_per_step * args.steps / elapsed
    if rank == 0:
        avg_launch_ms = ms_ntt.value / max(n_ntt.value, 1)
        achieved = by_ntt.value / (ms_ntt.value * 1e-3) / 1e9 if ms_ntt.value else 0.0
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "blocks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic random AES states + random round key, encrypted",
            "config": {
                "workload": ("one full AES-128 middle round (ShiftRows+SubBytes+MixColumns+"
                             "AddRoundKey): " + ("row-sliced +-1 bit state, S-box as Walsh "
                             "polynomial over nibble-bit monomials, bit-domain MixColumns/AddRoundKey" if args.layout == "rows"
                             else "nibble-domain Zeta-16 LUTs, byte-major SIMD packing")),
                "layout": args.layout,
                "log_n": args.log_n, "max_level": args.max_level, "special_primes": args.special_primes,
                "ciphertext_sets_per_gpu": args.batch, "blocks_per_gpu_per_step": args.batch * R.n_blk,
                "parallelism": f"ciphertext-batch sharding x{world} (no data-path collective)",
                "verified": ok, "pool_after_round": round_pool,
            },
            "roofline": {
                "bound": "hbm", "kernel": "ntt (k_nttf_*_cols / k_nttf_*_rows pass launches)",
                "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                "frac_per_pass_rw": round(2 * achieved / PEAK_HBM_GBS, 4),  # each pass's own read+write
                "traffic": traffic_per_launch(by_ntt.value / max(n_ntt.value, 1)),
                "traffic_source": PMC_NOTE,
                "launches": n_ntt.value, "avg_launch_us": round(avg_launch_ms * 1e3, 2),
                "alg_bytes_per_launch": round(by_ntt.value / max(n_ntt.value, 1)),
                "ntt_share_of_step": round(ms_ntt.value / (elapsed * 1e3), 3),
                "keyswitch_kernels_gbs": round(by_ks.value / (ms_ks.value * 1e-3) / 1e9, 1) if ms_ks.value else None,
                "keyswitch_share_of_step": round(ms_ks.value / (elapsed * 1e3), 3),
            },
            "cpu_baseline": None,
            "aes128_10_rounds": aes10,
        }
        if not args.no_cpu_baseline and world == 1:
            try:
                rec["cpu_baseline"] = cpu_baseline(args)
            except Exception as ex:  # report, never hide
                rec["cpu_baseline"] = {"error": repr(ex)}
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
