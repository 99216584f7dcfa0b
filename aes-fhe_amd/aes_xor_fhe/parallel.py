"""Ciphertext-batch sharding across GPUs of one node.

The homomorphic AES path partitions perfectly: ciphertexts (each carrying n_blk AES blocks)
are independent, so a batch of B ciphertext pairs is split contiguously over the ranks and
every rank runs whole rounds locally -- no per-round collective.  The only data movement is
the scatter of input ciphertexts from the client rank and the gather of the results, done
with torch.distributed (RCCL over xGMI on GPUs, gloo on CPU) on the NTT-domain residues.
Keys are never moved: every rank derives the same keys from the shared engine seed.
"""
from __future__ import annotations

from typing import Optional

import numpy as np


def shard_range(total: int, world: int, rank: int):
    """Contiguous [start, stop) share of `total` items for `rank` (first ranks take +1)."""
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _meta(ct, world):
    return np.array([ct.batch, ct.npoly, ct.level], dtype=np.int64)


def scatter_ciphertext(engine, ct, src: int = 0, group=None, device=None):
    """Split a batched ciphertext held by rank `src` across all ranks (batch dimension).
    Non-source ranks pass ct=None.  Returns this rank's share as a Ciphertext."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    meta = torch.zeros(3, dtype=torch.int64)
    if rank == src:
        meta = torch.from_numpy(_meta(ct, world))
    dist.broadcast(meta, src, group=group)
    batch, npoly, level = (int(x) for x in meta)
    if batch % world:
        raise ValueError(f"batch {batch} not divisible by world size {world}")
    share = batch // world
    n = 1 << engine.log_coeff_count
    shape = (share, npoly, level + 1, n)
    dev = device if device is not None else torch.device("cpu")
    out = torch.empty(shape, dtype=torch.int64, device=dev)
    parts = None
    if rank == src:
        res = engine.export_residues(ct).view(np.int64)
        parts = [torch.from_numpy(np.ascontiguousarray(res[i * share:(i + 1) * share])).to(dev)
                 for i in range(world)]
    dist.scatter(out, parts, src=src, group=group)
    return engine.import_residues(out.cpu().numpy().view(np.uint64))


def gather_ciphertext(engine, ct, dst: int = 0, group=None, device=None):
    """Concatenate every rank's batched ciphertext (same shape on all ranks) on rank `dst`."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = device if device is not None else torch.device("cpu")
    res = torch.from_numpy(engine.export_residues(ct).view(np.int64)).to(dev)
    bufs = [torch.empty_like(res) for _ in range(world)] if rank == dst else None
    dist.gather(res, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    full = torch.cat(bufs, 0).cpu().numpy().view(np.uint64)
    return engine.import_residues(full)
