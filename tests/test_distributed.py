"""Multi-rank path on CPU (gloo, world_size 2): ciphertext-batch scatter from the client rank,
AES on each rank's shard with identical seed-derived keys (and disjoint nonce ranges), gather,
decrypt, check against FIPS-197.  Same code (parallel.py) drives the GPUs under torchrun with
the nccl backend (RCCL), where the buffers are device tensors.

  * byte-major nibble round (aes_round.AESRoundEngine), even split;
  * the bench's row-sliced layout (aes_round_bits.AESRowRound) running full 10-round AES-128
    with bit-mode bootstrapping, uneven split (3 sets over 2 ranks), the C.1 vector in set 0."""
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


def _worker(rank, world, init, so, result_q):
    sys.path.insert(0, str(ROOT / "aes-fhe_amd"))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
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


def _worker_rows(rank, world, init, so, result_q):
    sys.path.insert(0, str(ROOT / "aes-fhe_amd"))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from aes_xor_fhe._abi import Lib
        from aes_xor_fhe.fhe import Engine
        from aes_xor_fhe.aes_round_bits import AESRowRound
        from aes_xor_fhe.bootstrap import Bootstrapper
        from aes_xor_fhe.parallel import (gather_ciphertext, rank_nonce_start, scatter_ciphertext,
                                          shard_range)
        from aes_xor_fhe import aes_tables as T
        e = Engine(_lib=Lib(so), log_n=10, max_level=30, special_primes=4, scale_bits=41, seed=3,
                   nonce_start=rank_nonce_start(rank), thread_count=4)
        sk = e.create_secret_key(1)
        rlk = e.create_relinearization_key(sk)
        R = AESRowRound(e, sk, e.create_public_key(sk), rlk)
        bs = Bootstrapper(e, sk, rlk)
        key = np.arange(16, dtype=np.uint8)
        total = 3
        blocks = np.random.default_rng(9).integers(0, 256, (total, R.n_blk, 16), dtype=np.uint8)
        blocks[0, 0] = np.frombuffer(bytes.fromhex("00112233445566778899aabbccddeeff"), np.uint8)
        st = R.encrypt_blocks(blocks) if rank == 0 else [[None] * 8 for _ in range(4)]
        mine = [[scatter_ciphertext(e, c) for c in row] for row in st]
        a, b = shard_range(total, world, rank)
        assert all(c.batch == b - a for row in mine for c in row)
        keys = [R.encrypt_round_key(rk) for rk in T.expand_key(key)]
        out, nref = R.encrypt_aes128(mine, keys, bs)
        full = [[gather_ciphertext(e, c) for c in row] for row in out]
        if rank == 0:
            got = R.decrypt_blocks(full)
            want = T.encrypt_block(blocks, key)
            ok = nref == 3 and bool(np.array_equal(got, want)) and \
                bytes(got[0, 0]) == bytes.fromhex("69c4e0d86a7b0430d8cdb78070b4c55a")
            result_q.put(ok)
    finally:
        dist.destroy_process_group()


def _worker_sliced(rank, world, init, so, result_q):
    """The bench's default state (AESSlicedRound, 12-prime digits over K = 10): rank 0 encrypts
    three slabs (12 sets, the last one partly padding), scattered in whole slabs
    (granule = AESSlicedRound.GRANULE = 4: rank 0 gets two slabs, rank 1 one -- an element split
    would put a slab's columns on two ranks), each rank runs one round (ShiftRows folded into the
    S-box, the batch-4 round key read cyclically), and rank 0 gathers and checks FIPS-197."""
    sys.path.insert(0, str(ROOT / "aes-fhe_amd"))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from aes_xor_fhe._abi import Lib
        from aes_xor_fhe.fhe import Engine
        from aes_xor_fhe.aes_round_bits import AESSlicedRound
        from aes_xor_fhe.parallel import gather_ciphertext, rank_nonce_start, scatter_ciphertext
        from aes_xor_fhe import aes_tables as T
        e = Engine(_lib=Lib(so), log_n=10, max_level=30, special_primes=10, digit_primes=12, scale_bits=40,
                   seed=5, nonce_start=rank_nonce_start(rank), thread_count=4)
        sk = e.create_secret_key(1)
        R = AESSlicedRound(e, sk, e.create_public_key(sk), e.create_relinearization_key(sk))
        nsets = 4 * (world + 1) - 1  # 3 slabs over 2 ranks, the last one padded by one set
        blocks = np.random.default_rng(12).integers(0, 256, (nsets, R.n_blk, 16), dtype=np.uint8)
        rk = np.random.default_rng(13).integers(0, 256, 16, dtype=np.uint8)
        st = R.encrypt_blocks(blocks) if rank == 0 else [[None] * 8 for _ in range(4)]
        mine = [[scatter_ciphertext(e, c, granule=R.GRANULE) for c in row] for row in st]
        assert all(c.batch == (8 if rank == 0 else 4) for row in mine for c in row)
        out = R.round(mine, R.encrypt_round_key(rk))
        full = [[gather_ciphertext(e, c) for c in row] for row in out]
        if rank == 0:
            result_q.put(bool(np.array_equal(R.decrypt_blocks(full, nsets), T.aes_round(blocks, rk))))
    finally:
        dist.destroy_process_group()


def _worker_keys(rank, world, init, so, result_q):
    """shared_seed is one 256-bit value on every rank; engines built from it pass the key check;
    engines with their own seeds make scatter raise on every rank; an all-empty gather is None."""
    sys.path.insert(0, str(ROOT / "aes-fhe_amd"))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        import torch
        from aes_xor_fhe._abi import Lib
        from aes_xor_fhe.fhe import Engine
        from aes_xor_fhe.parallel import gather_ciphertext, scatter_ciphertext, shared_seed
        lib = Lib(so)
        s = shared_seed()
        seeds = [torch.zeros(5, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(seeds, torch.tensor([(s >> (63 * i)) & ((1 << 63) - 1) for i in range(5)]))
        same = all(torch.equal(seeds[0], t) for t in seeds) and s >= 1 << 64
        kw = dict(log_n=10, max_level=3, special_primes=2)
        e = Engine(_lib=lib, seed=s, **kw)
        sk = e.create_secret_key(1)
        ct = e.encrypt(np.ones((2, 8)), sk) if rank == 0 else None
        got = scatter_ciphertext(e, ct)
        ok = same and got is not None and got.batch == 1
        ok = ok and gather_ciphertext(e, None) is None
        bad = Engine(_lib=lib, seed=1000 + rank, **kw)
        try:
            scatter_ciphertext(bad, bad.encrypt(np.ones((2, 8)), bad.create_secret_key(1)) if rank == 0 else None)
            ok = False
        except RuntimeError as ex:
            ok = ok and "different keys" in str(ex)
        oks = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(oks, torch.tensor([int(ok)]))
        if rank == 0:
            result_q.put(all(int(t) == 1 for t in oks))
    finally:
        dist.destroy_process_group()


def _worker_stream(rank, world, init, so, result_q):
    """Streaming scatter: the source sends each share point to point through
    one staging buffer, so its torch staging peak is one share (the old collective scatter built
    world padded copies); uneven shares (10 elements over 3 ranks: 4 + 3 + 3); the producing form
    (scatter_produced: the source encrypts each share on demand and never holds the batch);
    residues equal the source's slices, and a gather restores the batch."""
    sys.path.insert(0, str(ROOT / "aes-fhe_amd"))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        from aes_xor_fhe._abi import Lib
        from aes_xor_fhe.fhe import Engine
        from aes_xor_fhe import parallel as P
        e = Engine(_lib=Lib(so), log_n=10, max_level=4, special_primes=2, seed=91)
        sk = e.create_secret_key(3)
        n = e.slot_count
        vals = np.random.default_rng(2).uniform(-1, 1, (10, n))
        ct = e.encrypt(vals, sk) if rank == 0 else None
        mine = P.scatter_ciphertext(e, ct)
        a, b = P.shard_range(10, world, rank)
        per = ct.npoly * (ct.level + 1) * (1 << e.log_coeff_count) * 8 if ct is not None else None
        ok = mine.batch == b - a
        st = dict(P.last_scatter)
        if rank == 0:  # the source: one staging share (the largest other share), never world copies
            ok = ok and st["role"] == "src" and st["staging_peak_bytes"] == 3 * per
            ok = ok and st["staging_peak_bytes"] <= st["share_bytes_max"] < world * 4 * per
            ok = ok and np.array_equal(e.export_residues(mine), e.export_residues(e.slice(ct, a, b - a)))
        else:
            ok = ok and st["role"] == "dst" and st["staging_peak_bytes"] == st["share_bytes_max"]
        ok = ok and np.allclose(e.decrypt(mine, sk), vals[a:b], atol=1e-6)
        full = P.gather_ciphertext(e, mine)
        if rank == 0:
            ok = ok and np.array_equal(e.export_residues(full), e.export_residues(ct))
        # the producing form: shares encrypted on demand at the source
        made = []

        def produce(x, y):  # two ciphertexts per share (as an AES state's bit ciphertexts)
            made.append((x, y))
            return [e.encrypt(vals[x:y], sk, level=3), e.encrypt(-vals[x:y], sk, level=3)]
        got = P.scatter_produced(e, 10, 2, 3, produce if rank == 0 else None, nitems=2)
        ok = ok and len(got) == 2 and all(g.batch == b - a and g.level == 3 for g in got)
        ok = ok and np.allclose(e.decrypt(got[0], sk), vals[a:b], atol=1e-6)
        ok = ok and np.allclose(e.decrypt(got[1], sk), -vals[a:b], atol=1e-6)
        if rank == 0:  # every share made once, the source's own last
            ok = ok and sorted(made) == [P.shard_range(10, world, r) for r in range(world)] and made[-1] == (a, b)
            ok = ok and P.last_scatter["staging_peak_bytes"] == 3 * 2 * 4 * (1 << e.log_coeff_count) * 8
        oks = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(oks, torch.tensor([int(ok)]))
        if rank == 0:
            result_q.put(all(int(t) == 1 for t in oks))
    finally:
        dist.destroy_process_group()


def _spawn(target, so, world=2, timeout=900):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # a file store per test, not a probed TCP port: concurrent test processes (pytest -n) cannot
    # race for the same rendezvous port
    import tempfile
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="aesfhe_pg_"), "store")
    procs = [ctx.Process(target=target, args=(r, world, init, so, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return q.get(timeout=5)


def test_shard_range():
    from aes_xor_fhe.parallel import shard_range
    parts = [shard_range(10, 4, r) for r in range(4)]
    assert parts == [(0, 3), (3, 6), (6, 8), (8, 10)]
    # whole slabs of 4: 3 slabs over 2 ranks -> 2 + 1, never 6 + 6
    assert [shard_range(12, 2, r, 4) for r in range(2)] == [(0, 8), (8, 12)]
    assert [shard_range(8, 3, r, 4) for r in range(3)] == [(0, 4), (4, 8), (8, 8)]
    with pytest.raises(ValueError, match="whole granules"):
        shard_range(10, 2, 0, 4)


def _bench(*argv, env=None, timeout=300):
    import subprocess
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *argv], capture_output=True, text=True,
                          env=e, timeout=timeout, cwd=str(ROOT))


def test_bench_launcher_starts_n_ranks():
    """`python bench.py --gpus 2` (no torchrun) starts two ranks as child processes through
    torch.distributed.run and prints rank 0's line, which reports n_gpus 2 (--selftest-launch:
    the ranks only join the gloo group and all-reduce their count; no GPU, no engine)."""
    import json
    r = _bench("--gpus", "2", "--selftest-launch")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["selftest"] is True


def test_bench_launcher_rejects_mismatch():
    """A rank whose WORLD_SIZE differs from --gpus exits non-zero instead of timing a different
    world than it reports."""
    r = _bench("--gpus", "1", "--selftest-launch", env={"WORLD_SIZE": "2"}, timeout=60)
    assert r.returncode == 2 and "must agree" in r.stderr


def test_two_rank_shared_seed_and_key_check(oracle_lib):
    from conftest import ORACLE_SO
    assert _spawn(_worker_keys, str(ORACLE_SO)) is True


def test_three_rank_streaming_scatter_peak(oracle_lib):
    from conftest import ORACLE_SO
    assert _spawn(_worker_stream, str(ORACLE_SO), world=3, timeout=300) is True


def test_two_rank_scatter_round_gather(oracle_lib):
    from conftest import ORACLE_SO
    assert _spawn(_worker, str(ORACLE_SO)) is True


def test_two_rank_sliced_round(oracle_lib):
    from conftest import ORACLE_SO
    assert _spawn(_worker_sliced, str(ORACLE_SO)) is True


def test_two_rank_rows_aes128_with_bootstrap_uneven(oracle_lib):
    from conftest import ORACLE_SO
    assert _spawn(_worker_rows, str(ORACLE_SO)) is True


@pytest.mark.gpu
def test_rccl_device_scatter_gather_single_rank(product_lib, gpu_available):
    """The device-tensor path of parallel.py under the nccl backend (RCCL): scatter and gather
    through torch CUDA tensors filled / read by aesfhe_ct_export_device / import_device, uneven
    shares included (world 1 on the 1-GPU test box; the driver's 8-GPU bench runs world 8)."""
    import torch
    import torch.distributed as dist
    from aes_xor_fhe.fhe import Engine
    from aes_xor_fhe.parallel import gather_ciphertext, scatter_ciphertext
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        torch.cuda.set_device(0)
        e = Engine(_lib=product_lib, log_n=12, max_level=6, special_primes=2, seed=3)
        sk = e.create_secret_key()
        ct = e.encrypt(np.random.default_rng(0).standard_normal((3, 64)), sk)
        mine = scatter_ciphertext(e, ct)
        assert mine.batch == 3
        assert np.array_equal(e.export_residues(mine), e.export_residues(ct))
        back = gather_ciphertext(e, e.multiply(mine, 2.0))
        want = e.export_residues(e.multiply(ct, 2.0))
        assert np.array_equal(e.export_residues(back), want)
    finally:
        dist.destroy_process_group()
