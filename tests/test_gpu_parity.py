"""GPU parity: the HIP kernels (through the C ABI) against the oracle and the
golden fixtures generated from the reference build.  Bit-exact (integer path).

Sizes: seeded inputs the oracle finishes in seconds are compared hash for hash;
BASELINE.json's full sizes (configs 2, 3, 5 and the 8-shard config 4) are compared
through order-sensitive digests (tests/golden/digests.json, computed from the
reference itself over the same synthetic inputs).
"""
import numpy as np
import pytest

from conftest import hexkey, u64

import k2hash_amd
from k2hash_amd import batch

pytestmark = pytest.mark.gpu


def dev_u8(torch, arr, device, pad_front=0):
    """Device copy of a host byte array, optionally starting `pad_front` bytes into
    the allocation (to exercise unaligned key buffers)."""
    t = torch.zeros(arr.size + pad_front + 16, dtype=torch.uint8, device=device)
    t[pad_front:pad_front + arr.size] = torch.from_numpy(np.ascontiguousarray(arr))
    return t[pad_front:pad_front + arr.size]


def host_u64(t):
    return t.cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 128, 129, 255, 257, 4099, 100003])
def test_fixed32_vs_oracle(cuda, oracle, n):
    import torch
    data = oracle.gen_bytes(32 * n, byte_off=32 * 12345)
    r1, r2 = oracle.hash_fixed(data, 32)
    keys = dev_u8(torch, data, cuda)
    h1, h2 = k2hash_amd.hash_fixed(keys, 32, second=True)
    g1, _ = k2hash_amd.hash_fixed(keys, 32, second=False)
    torch.cuda.synchronize()
    assert np.array_equal(host_u64(h1), r1)
    assert np.array_equal(host_u64(h2), r2)
    assert np.array_equal(host_u64(g1), r1)


@pytest.mark.parametrize("n", [(1 << 21) + 17, 3 << 20])
def test_fixed32_many_blocks(cuda, oracle, n):
    """Millions of keys hash for hash (the digests below cover the full sizes)."""
    import torch
    data = oracle.gen_bytes(32 * n, byte_off=32 * 777)
    r1, r2 = oracle.hash_fixed(data, 32)
    keys = dev_u8(torch, data, cuda)
    h1, h2 = k2hash_amd.hash_fixed(keys, 32, second=True)
    g1, _ = k2hash_amd.hash_fixed(keys, 32, second=False)
    torch.cuda.synchronize()
    assert np.array_equal(host_u64(h1), r1)
    assert np.array_equal(host_u64(h2), r2)
    assert np.array_equal(host_u64(g1), r1)


# 384 and 640: odd round counts (3, 5) of the line-DMA kernel (two-slot unrolled loop)
@pytest.mark.parametrize("key_len", list(range(1, 72)) + [95, 96, 97, 127, 128, 129, 255, 256, 257, 384, 640, 1000, 4095,
                                     4096])
def test_fixed_any_length_vs_oracle(cuda, oracle, key_len):
    import torch
    n = 517 if key_len < 1000 else 67
    data = oracle.gen_bytes(key_len * n, byte_off=7 * key_len)
    r1, r2 = oracle.hash_fixed(data, key_len)
    for pad in (0, 1, 6):
        keys = dev_u8(torch, data, cuda, pad_front=pad)
        h1, h2 = k2hash_amd.hash_fixed(keys, key_len, second=True)
        torch.cuda.synchronize()
        assert np.array_equal(host_u64(h1), r1), (key_len, pad)
        assert np.array_equal(host_u64(h2), r2), (key_len, pad)


def _csr(keys):
    data = np.frombuffer(b"".join(keys), np.uint8) if keys else np.zeros(0, np.uint8)
    off = np.zeros(len(keys) + 1, np.int64)
    off[1:] = np.cumsum([len(k) for k in keys])
    return data, off


def test_golden_vectors_csr(cuda, vectors):
    import torch
    for field, std in (("vectors", False), ("std_fnv_vectors", True)):
        vs = vectors[field]
        data, off = _csr([hexkey(v) for v in vs])
        d = torch.from_numpy(data.copy()).to(cuda) if data.size else torch.zeros(0, dtype=torch.uint8, device=cuda)
        h1, h2 = k2hash_amd.hash_csr(d, torch.from_numpy(off).to(cuda), second=True, std_fnv=std)
        torch.cuda.synchronize()
        a, b = host_u64(h1), host_u64(h2)
        for i, v in enumerate(vs):
            assert (int(a[i]), int(b[i])) == (u64(v["h1"]), u64(v["h2"])), (field, v["tag"], v["len"])


@pytest.mark.parametrize("lens", ["mixed", "zeros", "long", "uniform", "mixedtiles"])
def test_csr_vs_oracle(cuda, oracle, lens):
    import torch
    rng = np.random.default_rng(5)
    if lens == "mixedtiles":
        # 512-key tiles alternating between LDS-staged (short keys) and oversize (spans past
        # the 72 KiB stage: listed and hashed by the ring pass) in one call, last tile partial
        L = rng.integers(8, 129, 512 * 7 + 77)
        for t in (1, 4, 7):
            L[512 * t: 512 * (t + 1)] = rng.integers(150, 400, L[512 * t: 512 * (t + 1)].size)
    elif lens == "mixed":
        L = rng.integers(0, 300, 6000)
        L[rng.integers(0, 6000, 300)] = 0
    elif lens == "zeros":
        L = np.zeros(1000, np.int64)
        L[::7] = 1
    elif lens == "long":
        L = rng.integers(1000, 9000, 300)
    else:
        L = rng.integers(8, 257, 20000)
    off = np.zeros(L.size + 1, np.int64)
    off[1:] = np.cumsum(L)
    base = 3  # offsets need not start at 0
    off += base
    data = oracle.gen_bytes(int(off[-1]) + 5)
    r1, r2 = oracle.hash_csr(data, off.astype(np.uint64))
    d = dev_u8(torch, data, cuda, pad_front=1)
    h1, h2 = k2hash_amd.hash_csr(d, torch.from_numpy(off).to(cuda), second=True)
    torch.cuda.synchronize()
    assert np.array_equal(host_u64(h1), r1)
    assert np.array_equal(host_u64(h2), r2)


def test_std_fnv_flag(cuda, oracle):
    import torch
    data = oracle.gen_bytes(32 * 1000)
    r1, r2 = oracle.hash_fixed(data, 32, variant=1)
    h1, h2 = k2hash_amd.hash_fixed(dev_u8(torch, data, cuda), 32, second=True, std_fnv=True)
    torch.cuda.synchronize()
    assert np.array_equal(host_u64(h1), r1) and np.array_equal(host_u64(h2), r2)


def test_empty_and_null(cuda):
    import torch
    off = torch.tensor([0, 0, 0, 0], dtype=torch.int64, device=cuda)
    h1, h2 = k2hash_amd.hash_csr(torch.zeros(0, dtype=torch.uint8, device=cuda), off, second=True)
    torch.cuda.synchronize()
    assert not h1.any() and not h2.any()
    h1, _ = k2hash_amd.hash_csr(torch.zeros(4, dtype=torch.uint8, device=cuda),
                                torch.zeros(1, dtype=torch.int64, device=cuda))
    assert h1.numel() == 0


def test_non_default_stream(cuda, oracle):
    import torch
    data = oracle.gen_bytes(32 * 5000)
    r1, _ = oracle.hash_fixed(data, 32)
    keys = dev_u8(torch, data, cuda)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        h1, _ = k2hash_amd.hash_fixed(keys, 32)
    s.synchronize()
    assert np.array_equal(host_u64(h1), r1)


def test_synth_matches_oracle_generator(cuda, oracle):
    import torch
    for nbytes, off in ((1, 0), (37, 5), (4096, 3), (100000, 8 * 1000 + 1)):
        t = batch.synth_bytes(nbytes, cuda, byte_off=off)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), oracle.gen_bytes(nbytes, byte_off=off)), (nbytes, off)
    o = batch.synth_offsets(5000, cuda, first_key=77)
    assert np.array_equal(o.cpu().numpy().astype(np.uint64), oracle.gen_offsets(5000, first_key=77))


def test_host_api_vs_oracle(cuda, oracle):
    n = (1 << 21) + 12345  # spans two 64 MiB pipeline chunks at 32 B
    data = oracle.gen_bytes(32 * n)
    r1, r2 = oracle.hash_fixed(data, 32)
    h1, h2 = k2hash_amd.hash_fixed_host(data, 32, second=True)
    assert np.array_equal(h1, r1) and np.array_equal(h2, r2)
    h1, _ = k2hash_amd.hash_fixed_host(data[: 21 * 1000], 21)
    assert np.array_equal(h1, oracle.hash_fixed(data[: 21 * 1000], 21)[0])
    off = oracle.gen_offsets(400000)
    cdata = oracle.gen_bytes(int(off[-1]))
    c1, c2 = oracle.hash_csr(cdata, off)
    g1, g2 = k2hash_amd.hash_csr_host(cdata, off, second=True)
    assert np.array_equal(g1, c1) and np.array_equal(g2, c2)


# ---------------------------------------------------------------------------------------
# Full BASELINE sizes, checked through digests of the reference's own outputs.
# ---------------------------------------------------------------------------------------
def _check_digest(oracle, cfg, h1, h2, first=0, expect=None):
    d1 = oracle.digest(host_u64(h1), first)
    d2 = oracle.digest(host_u64(h2), first)
    exp = expect or cfg
    assert [f"{x:016x}" for x in d1] == exp["h1"]
    assert [f"{x:016x}" for x in d2] == exp["h2"]


@pytest.mark.parametrize("name", ["fixed32_16M", "fixed4096_1M", "fixed21_1M", "fixed32_64K"])
def test_full_size_fixed_digest(cuda, oracle, digests, name):
    import torch
    cfg = digests[name]
    keys = batch.synth_bytes(cfg["n"] * cfg["key_len"], cuda)
    h1, h2 = k2hash_amd.hash_fixed(keys, cfg["key_len"], second=True)
    torch.cuda.synchronize()
    _check_digest(oracle, cfg, h1, h2)
    g1, _ = k2hash_amd.hash_fixed(keys, cfg["key_len"])  # h1-only path (the bench path)
    torch.cuda.synchronize()
    assert torch.equal(g1, h1)


@pytest.mark.parametrize("name", ["csr_8_256_64M", "csr_8_256_64K"])
def test_full_size_csr_digest(cuda, oracle, digests, name):
    import torch
    cfg = digests[name]
    off = batch.synth_offsets(cfg["n"], cuda, cfg["min_len"], cfg["max_len"])
    data = batch.synth_bytes(int(off[-1].item()), cuda)
    h1, h2 = k2hash_amd.hash_csr(data, off, second=True)
    torch.cuda.synchronize()
    _check_digest(oracle, cfg, h1, h2)


def test_config4_shard_digests(cuda, oracle, digests):
    """Config 4 (1 B x 32 B over 8 GPUs): each of the eight ranks' shards, hashed here one at
    a time, matches the reference's digest of that shard."""
    import torch
    cfg = digests["fixed32_1G"]
    assert len(cfg["chunks"]) == 8
    for c in cfg["chunks"]:
        keys = batch.synth_bytes(c["count"] * 32, cuda, byte_off=c["first"] * 32)
        h1, h2 = k2hash_amd.hash_fixed(keys, 32, second=True)
        torch.cuda.synchronize()
        _check_digest(oracle, cfg, h1, h2, first=c["first"], expect=c)
        del keys, h1, h2


@pytest.mark.parametrize("pad", [0, 16])
@pytest.mark.parametrize("key_len,n", [(128, 1), (128, 64), (256, 517), (384, 130), (1024, 200), (4096, 67),
                                       (4096, 1000), (200, 300)])
def test_fixed_long_kernels_vs_oracle(cuda, oracle, key_len, n, pad):
    """Long fixed-length keys: the line-DMA ring kernel (multiples of 128 B at a 128-aligned
    base) and the cooperative line ring (any other base or length), partial last waves
    included; h1 and h2."""
    import torch
    data = oracle.gen_bytes(key_len * n, byte_off=3 * key_len + 1)
    r1, r2 = oracle.hash_fixed(data, key_len)
    keys = dev_u8(torch, data, cuda, pad_front=pad)
    assert (keys.data_ptr() % 128 == 0) == (pad == 0)
    h1, h2 = k2hash_amd.hash_fixed(keys, key_len, second=True)
    g1, _ = k2hash_amd.hash_fixed(keys, key_len)
    torch.cuda.synchronize()
    assert np.array_equal(host_u64(h1), r1)
    assert np.array_equal(host_u64(h2), r2)
    assert np.array_equal(host_u64(g1), r1)


def test_host_api_error_mid_call_leaves_no_stale_chunk(cuda, oracle):
    """a host call that fails after launching chunks (here: offsets that stop
    being non-decreasing inside the second 4M-key chunk) must not leave a pending chunk
    that a later call drains into its own output."""
    from k2hash_amd import _native
    n = (4 << 20) + 64
    off = np.arange(n + 1, dtype=np.uint64)  # one-byte keys
    data = oracle.gen_bytes(n)
    bad = off.copy()
    bad[(4 << 20) + 10] = 0
    with pytest.raises(_native.NativeError):
        k2hash_amd.hash_csr_host(data, bad)
    m = 1000
    small = oracle.gen_offsets(m, 1, 40)
    sdata = oracle.gen_bytes(int(small[-1]), byte_off=77)
    h1, h2 = k2hash_amd.hash_csr_host(sdata, small, second=True)
    r1, r2 = oracle.hash_csr(sdata, small)
    assert np.array_equal(h1, r1) and np.array_equal(h2, r2)
    g1, _ = k2hash_amd.hash_csr_host(data, off)  # and the full call still works
    assert np.array_equal(g1, oracle.hash_csr(data, off)[0])


def test_out_tensors_validated(cuda, oracle):
    """Caller-supplied output tensors are checked before the kernel writes n values into
    them: undersized, wrong dtype, non-contiguous, h2 given without second=True
    (or missing with it) -> ValueError, nothing launched."""
    import torch
    n = 1000
    data = oracle.gen_bytes(32 * n)
    keys = dev_u8(torch, data, cuda)
    ok = torch.empty(n, dtype=torch.int64, device=cuda)
    bad = [
        (torch.empty(n - 1, dtype=torch.int64, device=cuda), None),
        (torch.empty(n, dtype=torch.int32, device=cuda), None),
        (torch.empty(2 * n, dtype=torch.int64, device=cuda)[::2], None),
        (torch.empty(n, dtype=torch.int64), None),
    ]
    for out in bad:
        with pytest.raises(ValueError):
            k2hash_amd.hash_fixed(keys, 32, out=out)
    with pytest.raises(ValueError):
        k2hash_amd.hash_fixed(keys, 32, out=(ok, torch.empty(n, dtype=torch.int64, device=cuda)))
    with pytest.raises(ValueError):
        k2hash_amd.hash_fixed(keys, 32, second=True, out=(ok, None))
    off = torch.arange(0, 32 * n + 1, 32, dtype=torch.int64, device=cuda)
    with pytest.raises(ValueError):
        k2hash_amd.hash_csr(keys, off, out=(torch.empty(n - 1, dtype=torch.int64, device=cuda), None))
    with pytest.raises(ValueError):
        batch.hash_fixed_index(keys, 32, 0xFF, 0xF, out=(ok, None, torch.empty(7, dtype=torch.int64, device=cuda), None))
    with pytest.raises(ValueError):
        batch.hash_csr_index(keys, off, 0xFF, 0xF, out=(ok, None, None, torch.empty(n + 1, dtype=torch.int64, device=cuda)))
    with pytest.raises(ValueError):
        batch.bucket_index(ok, 0xFF, 0xF, out=(torch.empty(n - 1, dtype=torch.int64, device=cuda), None))
    h1, _ = k2hash_amd.hash_fixed(keys, 32, out=(ok, None))  # the valid form still works
    torch.cuda.synchronize()
    assert np.array_equal(host_u64(h1), oracle.hash_fixed(data, 32)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 65, 130])
def test_fixed32_writes_nothing_past_n(cuda, oracle, n):
    """The fixed32 kernels clamp lanes past the end to key n-1 (they re-hash it and store its
    identical hash): no output element past n may change, with or without h2 / the index."""
    import torch
    data = oracle.gen_bytes(32 * n, byte_off=32 * 4242)
    r1, r2 = oracle.hash_fixed(data, 32)
    keys = dev_u8(torch, data, cuda)
    sentinel = -0x0123456789ABCDEF
    bufs = [torch.full((n + 256,), sentinel, dtype=torch.int64, device=cuda) for _ in range(6)]
    k2hash_amd.hash_fixed(keys, 32, second=False, out=(bufs[0][:n], None))
    k2hash_amd.hash_fixed(keys, 32, second=True, out=(bufs[1][:n], bufs[2][:n]))
    batch.hash_fixed_index(keys, 32, (1 << 28) - 1, 0xF, out=(bufs[3][:n], None, bufs[4][:n], bufs[5][:n]))
    torch.cuda.synchronize()
    for b, ref in ((bufs[0], r1), (bufs[1], r1), (bufs[2], r2), (bufs[3], r1)):
        assert np.array_equal(host_u64(b[:n]), ref)
    for b in bufs:
        assert bool((b[n:] == sentinel).all())
