"""Multi-GPU partitioning and the hash gather (k2hash_amd/shard.py), exercised on CPU
with the gloo backend at world_size 2 (and 3 for uneven splits).  The same code runs
over RCCL ("nccl") with device tensors in bench.py --gpus N.

Per-rank hashes here come from the product's scalar path (k2hash_amd.k2h_hash, the
plugin body) since there is no GPU; the gathered vector is checked against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from k2hash_amd import shard


def test_shard_range_covers_and_balances():
    for n in (0, 1, 7, 1000, 2**30 + 3):
        for w in (1, 2, 3, 4, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_shard_csr_by_bytes(oracle):
    off = oracle.gen_offsets(100000, 8, 256)
    for w in (1, 2, 4, 8):
        cuts = [shard.shard_csr_by_bytes(off, r, w) for r in range(w)]
        assert cuts[0][0] == 0 and cuts[-1][1] == 100000
        assert all(cuts[i][1] == cuts[i + 1][0] for i in range(w - 1))
        nbytes = [int(off[b]) - int(off[a]) for a, b in cuts]
        total = int(off[-1])
        assert max(nbytes) - min(nbytes) <= 2 * 256 + total // 1000
        a, b = cuts[-1]
        loc = shard.rebase_offsets(off, a, b)
        assert loc[0] == 0 and loc.size == b - a + 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, key_len, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path
        root = Path(__file__).resolve().parents[1]
        sys.path.insert(0, str(root / "oracle"))
        import k2hash_amd
        import oracle
        first, last = shard.shard_range(n, rank, world)
        data = oracle.gen_bytes((last - first) * key_len, byte_off=first * key_len)
        h = torch.tensor([k2hash_amd.k2h_hash(data[i * key_len:(i + 1) * key_len].tobytes())
                          for i in range(last - first)], dtype=torch.uint64).view(torch.int64)
        counts = [shard.shard_range(n, r, world)[1] - shard.shard_range(n, r, world)[0] for r in range(world)]
        out = shard.gather_hashes(h, dst=0, counts=counts)
        if rank == 0:
            q.put(out.view(torch.uint64).numpy().copy() if hasattr(torch, "uint64") else out.numpy().copy())
        if len(set(counts)) == 1:
            allh = shard.all_gather_hashes(h)
            q.put((rank, allh.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (3, 1001)])
def test_gather_hashes_gloo(oracle, world, n):
    key_len = 32
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, key_len, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(1 + (world if n % world == 0 else 0))]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref, _ = oracle.hash_fixed(oracle.gen_bytes(n * key_len), key_len)
    gathered = [r for r in results if not isinstance(r, tuple)][0]
    assert np.array_equal(np.asarray(gathered).view(np.uint64), ref)
    for r in results:
        if isinstance(r, tuple):
            assert np.array_equal(r[1].view(np.uint64), ref)
