"""Multi-GPU partitioning of a key batch and the gather of its hashes.

Keys are independent (lib/k2hashfunc.cc:49-59 has no cross-key state), so the
batch shards with no data-path collective: rank r hashes a contiguous key range.
The only exchange is returning the 64-bit hashes to whoever indexes the k2hash
table -- an RCCL gather over xGMI (torch.distributed "nccl" backend = RCCL on
ROCm), or all-gather when every rank needs every hash.  The same code runs over
gloo on CPU tensors for tests.
"""
from __future__ import annotations

from typing import Optional

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced key range [first, last) of rank `rank` (equal counts +-1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    q, r = divmod(n, world)
    first = rank * q + min(rank, r)
    return first, first + q + (1 if rank < r else 0)


def shard_csr_by_bytes(offsets, rank: int, world: int) -> tuple[int, int]:
    """Key range [first, last) of rank `rank` such that every rank gets about the same
    number of key BYTES (CSR keys differ in length).  Cuts fall on key
    boundaries: cut k is the first key that starts at or after byte (total * k / world), so
    a run of zero-length keys at a cut goes to the later rank.  `offsets` (n + 1 entries,
    non-decreasing, need not start at 0) is a numpy array or a torch tensor (a device
    tensor is searched on its device)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    is_torch = not isinstance(offsets, np.ndarray) and hasattr(offsets, "is_cuda")
    if not is_torch:
        offsets = np.asarray(offsets)
    n = (offsets.numel() if is_torch else offsets.size) - 1
    lo, hi = int(offsets[0]), int(offsets[-1])

    def cut(k: int) -> int:
        if k <= 0:
            return 0
        if k >= world:
            return n
        target = lo + (hi - lo) * k // world
        if is_torch:
            import torch

            t = torch.tensor([target], dtype=offsets.dtype, device=offsets.device)
            return int(torch.searchsorted(offsets[:-1], t, side="left").item())
        return int(np.searchsorted(offsets[:-1], target, side="left"))

    return cut(rank), cut(rank + 1)


def csr_cuts(offsets, world: int) -> list:
    """Every rank's [first, last) of shard_csr_by_bytes (rank order)."""
    return [shard_csr_by_bytes(offsets, r, world) for r in range(world)]


def rebase_offsets(offsets, first: int, last: int):
    """Offsets of keys [first, last) relative to their first byte (n_local + 1 entries):
    with the bytes [offsets[first], offsets[last]) as the shard's own buffer, they index it
    from 0.  numpy array or torch tensor in, the same kind out."""
    sub = offsets[first:last + 1]
    return sub - sub[0]


def _global_rank(group, r: int) -> int:
    """Global rank of group-local rank r (P2POp peers are global ranks)."""
    import torch.distributed as dist

    return r if group is None else dist.get_global_rank(group, r)


def shard_counts(n: int, world: int) -> list:
    """Per-rank key counts of shard_range(n, r, world), r = 0..world-1."""
    return [b - a for a, b in (shard_range(n, r, world) for r in range(world))]


def gather_hashes(h, dst: int = 0, group=None, counts: Optional[list] = None):
    """Gather every rank's hash vector to rank `dst` (group-local) in rank (= key) order.

    `h` is this rank's int64 tensor.  `counts` (per-rank lengths, e.g. shard_counts) is
    exchanged with one small all-gather when not given, so uneven shards work either way.
    Returns the concatenated tensor on dst, None elsewhere.  Implemented as point-to-point
    sends to the root (RCCL has no native gather; each peer uses its own xGMI link to the
    root), posted together so they overlap.  Over gloo, device tensors are staged
    through host memory (gloo's point-to-point ops take CPU tensors).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    staged = dist.get_backend(group) == "gloo" and h.is_cuda
    hh = h.detach().cpu() if staged else h.contiguous()
    if counts is None:
        mine = torch.tensor([h.numel()], dtype=torch.int64, device="cpu" if (staged or not h.is_cuda) else h.device)
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine, group=group)
        counts = [int(c.item()) for c in allc]
    if len(counts) != world or counts[rank] != h.numel():
        raise ValueError("counts must list every rank's length")
    if rank == dst:
        out = torch.empty(sum(counts), dtype=h.dtype, device=hh.device)
        pieces = list(torch.split(out, counts))
        ops = []
        for r in range(world):
            if r == dst:
                pieces[r].copy_(hh)
            elif counts[r]:
                ops.append(dist.P2POp(dist.irecv, pieces[r], _global_rank(group, r), group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return out.to(h.device) if staged else out
    if h.numel():
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, hh, _global_rank(group, dst), group)])
        for req in reqs:
            req.wait()
    return None


def all_gather_hashes(h, group=None):
    """Every rank receives all hashes (equal shard sizes), via all_gather_into_tensor."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    staged = dist.get_backend(group) == "gloo" and h.is_cuda
    hh = h.detach().cpu() if staged else h.contiguous()
    out = torch.empty(h.numel() * world, dtype=h.dtype, device=hh.device)
    dist.all_gather_into_tensor(out, hh, group=group)
    return out.to(h.device) if staged else out
