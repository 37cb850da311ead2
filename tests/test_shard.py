"""Multi-GPU partitioning and the hash gather (k2hash_amd/shard.py), exercised on CPU
with the gloo backend at world_size 2 (and 3 for uneven splits).  The same code runs
over RCCL ("nccl") with device tensors in bench.py --gpus N.

Per-rank hashes come from the product's scalar path (k2hash_amd.k2h_hash, the plugin
body) on CPU, and from the HIP kernel in the gpu-marked test; the gathered vector is
checked against the oracle."""
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


def _csr_batch(world: int, n: int = 30011):
    """One CSR batch (numpy uint64 offsets, uint8 bytes) with zero-length keys, built so
    that shard_csr_by_bytes puts a run of zero-length keys exactly on a cut: the first
    half's bytes equal the second half's, so the world-2 cut target is the first zero-length
    key's start; other world sizes cut through random lengths that include zeros."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
    import oracle
    rng = np.random.default_rng(4242)
    half = n // 2 - 3
    l1 = rng.integers(0, 300, size=half)
    l1[::97] = 0
    l2 = rng.integers(0, 300, size=n - half - 5)
    l2[::89] = 0
    l2[-1] += int(l1.sum() - l2.sum())  # the two halves hold the same bytes
    while l2[-1] < 0:  # keep lengths non-negative: spread the deficit backwards
        j = int(np.nonzero(l2[:-1] > 0)[0][-1])
        take = min(int(l2[j]), -int(l2[-1]))
        l2[j] -= take
        l2[-1] += take
    lens = np.concatenate([l1, np.zeros(5, dtype=l1.dtype), l2]).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    data = oracle.gen_bytes(int(off[-1]), byte_off=12345)
    return off, data


def _worker(rank, world, port, n, key_len, q, mode="cpu"):
    """mode: "cpu" (scalar plugin hashes, counts given), "auto" (counts exchanged by
    gather_hashes itself), "subgroup" (gather inside the group of global ranks 1..world-1
    to its local rank 0), "gpu" (hashes computed by the HIP kernel on cuda:0, device
    tensors gathered over gloo)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path
        root = Path(__file__).resolve().parents[1]
        sys.path.insert(0, str(root / "oracle"))
        import k2hash_amd
        import oracle
        if mode in ("csr_cpu", "csr_gpu"):  # one CSR batch cut by bytes, each shard rebased
            off, data = _csr_batch(world, n)
            cuts = shard.csr_cuts(off, world)
            first, last = cuts[rank]
            loc = shard.rebase_offsets(off, first, last)
            mine = data[int(off[first]):int(off[last])]
            if mode == "csr_gpu":
                h, _ = k2hash_amd.hash_csr(torch.from_numpy(mine.copy()).to("cuda:0"),
                                           torch.from_numpy(loc.astype(np.int64)).to("cuda:0"))
                torch.cuda.synchronize()
            else:
                h = torch.tensor([k2hash_amd.k2h_hash(mine[int(loc[i]):int(loc[i + 1])].tobytes())
                                  for i in range(last - first)], dtype=torch.uint64).view(torch.int64)
            out = shard.gather_hashes(h, dst=0, counts=[b - a for a, b in cuts])
            if rank == 0:
                q.put(("csr", cuts, out.cpu().numpy().copy()))
            return
        first, last = shard.shard_range(n, rank, world)
        data = oracle.gen_bytes((last - first) * key_len, byte_off=first * key_len)
        if mode == "gpu":
            keys = torch.from_numpy(data).to("cuda:0")
            h, _ = k2hash_amd.hash_fixed(keys, key_len)
            torch.cuda.synchronize()
        else:
            h = torch.tensor([k2hash_amd.k2h_hash(data[i * key_len:(i + 1) * key_len].tobytes())
                              for i in range(last - first)], dtype=torch.uint64).view(torch.int64)
        counts = shard.shard_counts(n, world)
        if mode == "subgroup":
            members = list(range(1, world))
            grp = dist.new_group(members)
            if rank in members:
                out = shard.gather_hashes(h, dst=0, group=grp)
                if rank == 1:
                    q.put(("sub", out.numpy().copy()))
            dist.barrier()
            return
        out = shard.gather_hashes(h, dst=0, counts=None if mode == "auto" else counts)
        if rank == 0:
            q.put(out.cpu().numpy().copy())
        if len(set(counts)) == 1:
            allh = shard.all_gather_hashes(h)
            q.put((rank, allh.cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


def _run(world, n, key_len, mode, expect):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, key_len, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=180) for _ in range(expect)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


@pytest.mark.parametrize("world,n,mode", [(2, 1000, "cpu"), (3, 1001, "cpu"), (3, 1001, "auto")])
def test_gather_hashes_gloo(oracle, world, n, mode):
    key_len = 32
    results = _run(world, n, key_len, mode, 1 + (world if n % world == 0 else 0))
    ref, _ = oracle.hash_fixed(oracle.gen_bytes(n * key_len), key_len)
    gathered = [r for r in results if not isinstance(r, tuple)][0]
    assert np.array_equal(np.asarray(gathered).view(np.uint64), ref)
    for r in results:
        if isinstance(r, tuple):
            assert np.array_equal(r[1].view(np.uint64), ref)


def test_gather_hashes_subgroup(oracle):
    """A non-default group: peers are translated to global ranks."""
    world, n, key_len = 3, 999, 32
    (tag, got), = _run(world, n, key_len, "subgroup", 1)
    ref, _ = oracle.hash_fixed(oracle.gen_bytes(n * key_len), key_len)
    lo = shard.shard_range(n, 1, world)[0]
    assert tag == "sub" and np.array_equal(got.view(np.uint64), ref[lo:])


@pytest.mark.gpu
def test_gather_hip_hashes(oracle):
    """HIP-computed hashes (two ranks sharing cuda:0) through gather_hashes and
    all_gather_hashes, staged over gloo; the gathered vector is the oracle's."""
    world, n, key_len = 2, 200000, 32
    results = _run(world, n, key_len, "gpu", 1 + world)
    ref, _ = oracle.hash_fixed(oracle.gen_bytes(n * key_len), key_len)
    gathered = [r for r in results if not isinstance(r, tuple)][0]
    assert np.array_equal(np.asarray(gathered).view(np.uint64), ref)
    assert all(np.array_equal(r[1].view(np.uint64), ref) for r in results if isinstance(r, tuple))


def _check_csr(world, mode):
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
    import oracle
    n = 30011
    (tag, cuts, got), = _run(world, n, 0, mode, 1)
    off, data = _csr_batch(world, n)
    ref, _ = oracle.hash_csr(data, off)
    assert tag == "csr" and [tuple(c) for c in cuts] == shard.csr_cuts(off, world)
    assert np.array_equal(got.view(np.uint64), ref)
    lens = np.diff(off.astype(np.int64))
    if world == 2:  # the cut falls on the run of zero-length keys, which rank 1 starts with
        c = cuts[1][0]
        assert lens[c] == 0 and lens[c - 1] > 0 and (ref[c:c + 5] == 0).all()
    nbytes = [int(off[b]) - int(off[a]) for a, b in cuts]
    assert max(nbytes) - min(nbytes) <= 2 * 300


@pytest.mark.parametrize("world", [2, 3])
def test_csr_shards_by_bytes_gathered(world):
    """One CSR batch cut by bytes (shard_csr_by_bytes), each shard's offsets rebased, each
    rank hashing only its own bytes (scalar plugin), gathered to rank 0 with the per-rank
    counts: bit-for-bit the oracle's hashes of the whole batch."""
    _check_csr(world, "csr_cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_csr_shards_by_bytes_hip_gathered(world):
    """The same with each rank's shard hashed by the HIP CSR kernel on cuda:0 (ranks share
    the card over gloo), a zero-length key run on the world-2 cut."""
    _check_csr(world, "csr_gpu")
