"""Multi-rank path on CPU (gloo, world_size 2): ciphertext-batch scatter from the client rank,
one AES round per rank on its shard with identical seed-derived keys, gather, decrypt, check
against FIPS-197.  Same code drives the GPUs under torchrun (backend RCCL or gloo)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, so, result_q):
    sys.path.insert(0, str(ROOT / "aes-fhe_amd"))
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from aes_xor_fhe._abi import Lib
        from aes_xor_fhe.fhe import Engine
        from aes_xor_fhe.aes_round import AESRoundEngine
        from aes_xor_fhe.parallel import gather_ciphertext, scatter_ciphertext, shard_range
        from aes_xor_fhe import aes_tables as T
        e = Engine(_lib=Lib(so), log_n=10, max_level=30, special_primes=8, seed=77, thread_count=2)
        sk = e.create_secret_key(5)      # same seed on every rank -> same keys, no key traffic
        R = AESRoundEngine(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk),
                           e.create_conjugation_key(sk))
        rk = np.arange(16, dtype=np.uint8) * 7
        total = 2 * world
        blocks = np.random.default_rng(1).integers(0, 256, (total, R.n_blk, 16), dtype=np.uint8)
        hi = lo = None
        if rank == 0:
            hi, lo = R.encrypt_blocks(blocks)
        mh = scatter_ciphertext(e, hi)
        ml = scatter_ciphertext(e, lo)
        a, b = shard_range(total, world, rank)
        assert mh.batch == b - a
        oh, ol = R.round(mh, ml, R.encrypt_round_key(rk))
        gh, gl = gather_ciphertext(e, oh), gather_ciphertext(e, ol)
        if rank == 0:
            ok = bool((R.decrypt_blocks(gh, gl) == T.aes_round(blocks, rk)).all())
            result_q.put(ok)
    finally:
        dist.destroy_process_group()


def test_shard_range():
    from aes_xor_fhe.parallel import shard_range
    parts = [shard_range(10, 4, r) for r in range(4)]
    assert parts == [(0, 3), (3, 6), (6, 8), (8, 10)]


def test_two_rank_scatter_round_gather(oracle_lib):
    import torch.multiprocessing as mp
    from conftest import ORACLE_SO
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(ORACLE_SO), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
