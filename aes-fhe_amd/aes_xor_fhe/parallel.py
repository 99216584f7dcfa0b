"""Ciphertext-batch sharding across GPUs of one node.

The homomorphic AES path partitions perfectly: ciphertexts (each carrying n_blk AES blocks)
are independent, so a batch is split contiguously over the ranks (`shard_range`) and every
rank runs whole rounds locally -- no per-round collective.  The only data movement is the
scatter of input ciphertexts from the client rank and the gather of the results.

Transfers are device-resident: residues go from the engine's device buffers into torch tensors
on the same GPU (aesfhe_ct_export_device, a device-to-device copy) and torch.distributed moves
those tensors -- with the "nccl" backend that is RCCL over xGMI, GPU to GPU, never through host
memory.  With the CPU oracle engine (tests, "gloo") the same code runs on host tensors; with the
HIP engine under gloo (several ranks rehearsing on one GPU, which RCCL refuses) the residues
are staged through host tensors.

Keys are never moved: every rank derives the same keys from one 256-bit engine seed that rank 0
draws and broadcasts (`shared_seed`); each rank encrypts with its own nonce range
(`rank_nonce_start`) so no two ranks reuse randomness.  Before the first transfer over a process
group the ranks compare `Engine.key_fingerprint()`: engines with different keys (e.g. default
engines, each with its own random key) raise instead of computing on ciphertexts they cannot
decrypt.
"""
from __future__ import annotations

import numpy as np


def shard_range(total: int, world: int, rank: int, granule: int = 1):
    """Contiguous [start, stop) share of `total` items for `rank`, in whole granules of `granule`
    items (the sliced AES state's slab of 4 batch elements: its columns must stay on one rank);
    the first (total / granule) % world ranks take one granule more.  Raises if `total` is not a
    whole number of granules."""
    granule = int(granule)
    if granule < 1 or total % granule:
        raise ValueError(f"shard_range: {total} items are not whole granules of {granule}")
    base, extra = divmod(total // granule, world)
    start = rank * base + min(rank, extra)
    stop = start + base + (1 if rank < extra else 0)
    return start * granule, stop * granule


def rank_nonce_start(rank: int) -> int:
    """First encryption nonce of `rank` for engines sharing one seed: disjoint 2^48 ranges."""
    return (int(rank) + 1) << 48


def shared_seed(group=None, src: int = 0) -> int:
    """A 256-bit engine seed drawn from os.urandom on rank `src` and broadcast to every rank (the
    same on all of them), or a fresh local one without torch.distributed."""
    import os
    seed = int.from_bytes(os.urandom(32), "little")
    try:
        import torch.distributed as dist
        if not dist.is_initialized():
            return seed
    except ImportError:
        return seed
    import torch
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    words = torch.tensor([(seed >> (63 * i)) & ((1 << 63) - 1) for i in range(5)], dtype=torch.int64, device=dev)
    dist.broadcast(words, src, group=group)
    return sum(int(w) << (63 * i) for i, w in enumerate(words.cpu().tolist())) & ((1 << 256) - 1)


def _check_keys(engine, group, dev):
    """Raise unless every rank's engine derives the same keys (once per engine and group)."""
    import torch
    import torch.distributed as dist
    # verified groups are held by weak reference: a destroyed group whose id() is reused by a
    # new one is checked again
    import weakref
    done = engine.__dict__.setdefault("_fp_groups", weakref.WeakSet())
    key = group if group is not None else dist.distributed_c10d._get_default_group()
    if key in done:
        return
    mine = torch.tensor([engine.key_fingerprint()], dtype=torch.int64, device=dev)
    allf = [torch.empty_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(allf, mine, group=group)
    if len({int(t.item()) for t in allf}) != 1:
        raise RuntimeError("ranks hold engines with different keys (engine seed / prime chain): "
                           "create every rank's Engine with one shared seed (parallel.shared_seed)")
    done.add(key)


def _torch_device(engine, group=None):
    """Where the transfer buffers live: the engine's GPU under the nccl backend (RCCL moves
    device memory), host memory otherwise (the CPU oracle; gloo, e.g. a multi-rank rehearsal
    sharing one GPU, where RCCL cannot run two ranks on one device)."""
    import torch
    import torch.distributed as dist
    if engine.on_device and dist.get_backend(group) == "nccl":
        return torch.device("cuda", engine.device_id)
    return torch.device("cpu")


def _export(engine, ct, buf, start=0, count=None):
    if buf.device.type == "cpu" and engine.on_device:  # gloo with the HIP engine: host staging
        import torch
        count = ct.batch - start if count is None else count
        res = engine.export_residues(ct)[start:start + count]
        buf[:count].copy_(torch.from_numpy(res.reshape(count, -1).view(np.int64)))
    else:
        engine.export_into(ct, buf.data_ptr(), start, count)


def _import(engine, buf, batch, npoly, level):
    if buf.device.type == "cpu" and engine.on_device:
        arr = buf[:batch].numpy().view(np.uint64)
        return engine.import_residues(arr.reshape(batch, npoly, level + 1, -1))
    return engine.import_from(buf.data_ptr(), batch, npoly, level)


def _sync(dev):
    """Finish torch's pending work on `dev` before the engine's own stream touches (or after RCCL
    has written) a torch-allocated buffer: the two are different HIP streams."""
    if dev.type == "cuda":
        import torch
        torch.cuda.current_stream(dev).synchronize()


def _words(engine, npoly, level):
    return npoly * (level + 1) * (1 << engine.log_coeff_count)


# the torch staging bytes the last scatter on this process held at once (tests assert the source
# rank's peak): {"staging_peak_bytes", "share_bytes_max", "role"}
last_scatter: dict = {}


def _scatter_stream(engine, src, group, granule, meta, fill, own, nitems=1):
    """Rank `src` sends every other rank its share point to point, one rank at a time, through ONE
    staging buffer (fill(a, b, k, buf) writes item k's elements [a, b) into it), and takes its own
    share last (own(a, b) -> the list of nitems Ciphertexts), so the source holds its batch (or
    nothing, for a producing source) plus one share -- never the world padded copies a collective
    scatter needs (config 5's 512-ciphertext batch would not fit twice in
    288 GB).  Receivers take each item into a buffer of their share's size and import it.
    meta = (batch, npoly, level) on src, the same for every item.  Returns the list of this rank's
    nitems shares (None for an empty share)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = _torch_device(engine, group)
    _check_keys(engine, group, dev)
    m = torch.zeros(3, dtype=torch.int64, device=dev)
    if rank == src:
        m = torch.tensor(list(meta), dtype=torch.int64, device=dev)
    dist.broadcast(m, src, group=group)
    batch, npoly, level = (int(x) for x in m.cpu())
    shares = [shard_range(batch, world, r, granule) for r in range(world)]  # raises alike everywhere
    per = _words(engine, npoly, level)
    gsrc = dist.get_global_rank(group, src) if group is not None else src
    a, b = shares[rank]
    if rank == src:
        big = max([bb - aa for r, (aa, bb) in enumerate(shares) if r != src] + [0])
        buf = torch.empty((big, per), dtype=torch.int64, device=dev) if big else None
        for r in range(world):
            ra, rb = shares[r]
            if r == src or rb == ra:
                continue
            dst = dist.get_global_rank(group, r) if group is not None else r
            for k in range(nitems):
                _sync(dev)  # the previous send has left buf
                fill(ra, rb, k, buf)
                dist.send(buf[:rb - ra], dst, group=group)
        _sync(dev)
        last_scatter.update(role="src", staging_peak_bytes=(buf.numel() * 8 if buf is not None else 0),
                            share_bytes_max=max(bb - aa for aa, bb in shares) * per * 8)
        del buf
        return own(a, b) if b > a else [None] * nitems
    if b == a:
        last_scatter.update(role="dst", staging_peak_bytes=0, share_bytes_max=0)
        return [None] * nitems
    out = torch.empty((b - a, per), dtype=torch.int64, device=dev)
    res = []
    for _ in range(nitems):
        dist.recv(out, gsrc, group=group)
        _sync(dev)  # the transfer wrote `out` on torch's stream
        res.append(_import(engine, out, b - a, npoly, level))
    last_scatter.update(role="dst", staging_peak_bytes=out.numel() * 8, share_bytes_max=(b - a) * per * 8)
    return res


def scatter_ciphertext(engine, ct, src: int = 0, group=None, granule: int = 1):
    """Split a batched ciphertext held by rank `src` across all ranks along the batch dimension
    (shard_range: uneven batches allowed, in whole granules of `granule` elements -- 4 for the
    sliced AES state, AESSlicedRound.GRANULE).  Non-source ranks pass ct=None.  Returns this
    rank's share (None for a rank whose share is empty).  Raises on every rank if the batch is not
    a whole number of granules.  Streaming (_scatter_stream): the source holds ct plus one share."""
    meta = (ct.batch, ct.npoly, ct.level) if ct is not None else None
    return _scatter_stream(engine, src, group, granule, meta,
                           lambda a, b, k, buf: _export(engine, ct, buf, a, b - a),
                           lambda a, b: [engine.slice(ct, a, b - a)])[0]


def scatter_produced(engine, batch: int, npoly: int, level: int, produce, src: int = 0, group=None,
                     granule: int = 1, nitems: int = 1):
    """The client form: rank `src` produces each rank's share on demand (produce(a, b) -> the
    list of `nitems` ciphertexts of batch elements [a, b), all of one shape -- e.g. an AES state's
    bit ciphertexts, those blocks encrypted) and sends them, so it never holds the whole batch:
    one share in flight plus its own.  Other ranks pass produce=None (batch / npoly / level are
    taken from src).  Returns this rank's list of nitems shares."""
    held = {}

    def fill(a, b, k, buf):
        if k == 0:
            held["cs"] = list(produce(a, b))
            if len(held["cs"]) != nitems:
                raise ValueError(f"scatter_produced: {len(held['cs'])} ciphertexts for {nitems} items")
        c = held["cs"][k]
        if (c.batch, c.npoly, c.level) != (b - a, npoly, level):
            raise ValueError(f"scatter_produced: share [{a}, {b}) came back as batch {c.batch}, "
                             f"npoly {c.npoly}, level {c.level}")
        _export(engine, c, buf, 0, b - a)
        held["cs"][k] = None  # sent: freed before the next is exported
    return _scatter_stream(engine, src, group, granule, (batch, npoly, level), fill,
                           lambda a, b: list(produce(a, b)), nitems)


def gather_ciphertext(engine, ct, dst: int = 0, group=None):
    """Concatenate every rank's batched ciphertext (same npoly / level on all ranks, batch may
    differ; a rank may pass None for an empty share) on rank `dst`, in rank order.  None on
    every rank if every share is empty."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    dev = _torch_device(engine, group)
    _check_keys(engine, group, dev)
    mine = torch.tensor([ct.batch if ct is not None else 0,
                         ct.npoly if ct is not None else -1,
                         ct.level if ct is not None else -1], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(metas, mine, group=group)
    metas = [m.cpu().tolist() for m in metas]
    shapes = {(p, l) for b, p, l in metas if b > 0}
    if not shapes:  # every share empty: nothing to gather
        return None
    if len(shapes) != 1:
        raise ValueError(f"gather_ciphertext: ranks disagree on (npoly, level): {sorted(shapes)}")
    npoly, level = shapes.pop()
    per = _words(engine, npoly, level)
    smax = max(b for b, _, _ in metas)
    buf = torch.zeros((smax, per), dtype=torch.int64, device=dev)
    _sync(dev)
    if ct is not None:
        _export(engine, ct, buf)
    bufs = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    full = torch.cat([bufs[r][:metas[r][0]] for r in range(world)], 0).contiguous()
    _sync(dev)
    return _import(engine, full, full.shape[0], npoly, level)
