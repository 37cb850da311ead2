"""Bucket-index epilogue: K2HShm::GetKIndexPos's stateless part
(lib/k2hshm.cc:810-833, MakeMask / GetMaskBitCount :78-90) and the collision slot
(lib/k2hshm.cc:1093), standalone and fused into the hash kernels.

Parity: the HIP epilogue is compared bit-for-bit with the oracle's loop-for-loop
restatement.  The reference functions are K2HShm members that need the mapped table and
libfullock, so they cannot be compiled here; the restatement is pinned by the reference's
own fixture tests/test_linetool_dsave.cmd (k2hlinetool -mask 2 -cmask 2) with its log
tests/test_linetool.log:2756-2768: key1\\0 and key27\\0 land in one CKINDEX, and `dsave 3`
(GetElementsByHash from start hash 3, lib/k2hshmdirect.cc:280-323) reaches it.
"""
import numpy as np
import pytest

import k2hash_amd
from k2hash_amd import batch

MASKS = [(0x3, 0x3), (0xFF, 0xF), (0x0, 0x0), (0x1, 0x0), ((1 << 28) - 1, 0xF), ((1 << 20) - 1, (1 << 12) - 1),
         ((1 << 58) - 1, 0x0), (0xFF, (1 << 63) | 0xF), (0x7, 0xFFFFFFFFFFFFFFFF)]


def _keys_h(oracle, keys):
    return [oracle.k2h_hash(k) for k in keys]


# ------------------------------------------------------------------------- CPU
def test_mask_helpers_match_reference_loops(oracle):
    for b in range(0, 65):
        m = oracle.lib().oracle_make_mask(b)
        assert m == ((1 << b) - 1 if b < 64 else (1 << 64) - 1)
        assert oracle.lib().oracle_mask_bitcount(m) == b


def test_known_positions(oracle):
    # 0x0b2bb3288cdb4d49 = k2h_hash("KEY-0000000000000000\0"); default masks 0xFF / 0xF
    assert oracle.kindex_pos(0x0B2BB3288CDB4D49, 0xFF, 0xF) == (8, 0x54, 0x9)
    assert oracle.kindex_pos(0, 0xFF, 0xF) == (0, 0, 0)
    assert oracle.kindex_pos(1 << 4, 0xFF, 0xF) == (1, 0, 0)
    assert oracle.kindex_pos(0x30, 0xFF, 0xF) == (2, 1, 0)


def test_linetool_dsave_fixture_pin(oracle):
    """tests/test_linetool_dsave.cmd runs k2hlinetool with -mask 2 -cmask 2 (cur_mask 0x3,
    collision_mask 0x3) and its log shows key1 and key27 saved together by `dsave 3` and
    restored together (tests/test_linetool.log:2756-2768)."""
    cur, cm = 0x3, 0x3
    b1 = oracle.kindex_pos(oracle.k2h_hash(b"key1\0"), cur, cm)
    b27 = oracle.kindex_pos(oracle.k2h_hash(b"key27\0"), cur, cm)
    assert b1 == b27  # one CKINDEX holds both elements
    # GetElementsByHash walks test_hash from 3 to cur_max_hash = (cur << bitcount(cm)) | cm
    cur_max = (cur << 2) | cm
    reach = [t for t in range(0, cur_max + 1) if oracle.kindex_pos(t, cur, cm) == b1]
    assert reach and min(reach) >= 3


def _ki_array_count(area: int) -> int:
    """KIArrayCount of key_index_area[area]: the table at lib/k2hshm.cc:800-808 lists
    area 0 -> PKINDEX[1], 1 -> [1], 2 -> [2], 3 -> [4]: 2^(area-1) from area 1 on.  (Its last
    two rows, 0x7FFFFFFF -> area 30 and 0xFFFFFFFF -> area 31, are one lower than
    GetKIndexPos's loop at :822-826 gives for 31- and 32-bit masks; the loop is what runs,
    so the rule of the first rows is extended.)"""
    return 1 if area == 0 else 1 << (area - 1)


@pytest.mark.parametrize("cmask", [0x0, 0x3, 0xF, (1 << 12) - 1])
def test_key_index_area_table_pin(oracle, cmask):
    """Second pin of the restatement: the reference's own key_index_area table
    (lib/k2hshm.cc:800-808).  For every cur_mask of the form 2^m - 1 the table admits:
    KIPtrArrayPos <= m; KIArrayPos < KIArrayCount(KIPtrArrayPos); and -- checked
    exhaustively over every shifted hash below 2^m for m <= 12 -- area p (p >= 1) is hit
    by exactly KIArrayCount(p) distinct KIArrayPos, area 0 by one, so the table's counts
    are exactly the index space GetKIndexPos addresses."""
    cshift = int(cmask).bit_length()
    rng = np.random.default_rng(cmask)
    for m in range(0, 33):
        cur = (1 << m) - 1
        hs = rng.integers(0, 2**63, 2000, dtype=np.int64).view(np.uint64) * np.uint64(5)
        hs[:3] = [0, 0xFFFFFFFFFFFFFFFF, np.uint64(cur) << np.uint64(cshift)]
        k, _ = oracle.bucket_index(hs, cur, cmask)
        pos, arr = batch.unpack_kindex(k)
        assert int(pos.max()) <= m
        assert int(pos[1]) == m and int(pos[2]) == m  # all mask bits set -> the table's last area
        assert all(int(a) < _ki_array_count(int(p)) for p, a in zip(pos, arr))
        if m <= 12:
            every = (np.arange(1 << m, dtype=np.uint64) << np.uint64(cshift)) | np.uint64(cmask & 0x5)
            k, _ = oracle.bucket_index(every, cur, cmask)
            pos, arr = batch.unpack_kindex(k)
            for area in range(0, m + 1):
                hit = {int(a) for p, a in zip(pos, arr) if int(p) == area}
                assert len(hit) == _ki_array_count(area), (m, area)


def test_kindex_packing_helpers():
    kv = np.array([(8 << 58) | 0x54, 0, (58 << 58) | ((1 << 58) - 1)], np.uint64)
    pos, arr = batch.unpack_kindex(kv)
    assert list(pos) == [8, 0, 58]
    assert list(arr) == [0x54, 0, (1 << 58) - 1]


# ------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("cur,cm", MASKS)
def test_standalone_vs_oracle(cuda, oracle, cur, cm):
    import torch
    rng = np.random.default_rng(cur ^ (cm & 0xFFFF))
    h = rng.integers(0, 2**63, 100003, dtype=np.int64).view(np.uint64) * np.uint64(3)
    h[:8] = [0, 1, 2, 3, 0xFFFFFFFFFFFFFFFF, 1 << 63, 0x0B2BB3288CDB4D49, 16]
    d = torch.from_numpy(h.view(np.int64).copy()).to(cuda)
    k, c = k2hash_amd.bucket_index(d, cur, cm)
    torch.cuda.synchronize()
    rk, rc = oracle.bucket_index(h, cur, cm)
    assert np.array_equal(k.cpu().numpy().view(np.uint64), rk)
    assert np.array_equal(c.cpu().numpy().view(np.uint64), rc)


@pytest.mark.gpu
def test_standalone_optional_outputs_and_errors(cuda):
    import torch
    d = torch.arange(1000, dtype=torch.int64, device=cuda)
    k, c = k2hash_amd.bucket_index(d, 0xFF, 0xF, kindex=False)
    assert k is None and c is not None
    k, c = k2hash_amd.bucket_index(d, 0xFF, 0xF, ckindex=False)
    assert c is None and k is not None
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError):
        k2hash_amd.bucket_index(d, (1 << 59) - 1, 0xF)  # cur_mask does not fit the packing


@pytest.mark.gpu
@pytest.mark.parametrize("key_len", [32, 21, 4096, 100, 256])
def test_fused_fixed_vs_oracle(cuda, oracle, key_len):
    import torch
    n = 70001 if key_len < 1000 else 3001
    data = oracle.gen_bytes(key_len * n, byte_off=99)
    r1, r2 = oracle.hash_fixed(data, key_len)
    keys = torch.from_numpy(data).to(cuda)
    for cur, cm in [(0xFF, 0xF), ((1 << 28) - 1, 0xF), (0x3, 0x3)]:
        h1, h2, k, c = k2hash_amd.hash_fixed_index(keys, key_len, cur, cm, second=True)
        torch.cuda.synchronize()
        rk, rc = oracle.bucket_index(r1, cur, cm)
        assert np.array_equal(h1.cpu().numpy().view(np.uint64), r1)
        assert np.array_equal(h2.cpu().numpy().view(np.uint64), r2)
        assert np.array_equal(k.cpu().numpy().view(np.uint64), rk)
        assert np.array_equal(c.cpu().numpy().view(np.uint64), rc)


@pytest.mark.gpu
def test_fused_csr_vs_oracle(cuda, oracle):
    import torch
    rng = np.random.default_rng(11)
    L = rng.integers(0, 300, 20000)
    L[::17] = 0
    off = np.zeros(L.size + 1, np.int64)
    off[1:] = np.cumsum(L)
    data = oracle.gen_bytes(int(off[-1]) + 3)
    r1, _ = oracle.hash_csr(data, off.astype(np.uint64))
    h1, h2, k, c = k2hash_amd.hash_csr_index(torch.from_numpy(data).to(cuda), torch.from_numpy(off).to(cuda),
                                             0xFFFF, 0xF, ckindex=False)
    torch.cuda.synchronize()
    rk, _ = oracle.bucket_index(r1, 0xFFFF, 0xF)
    assert h2 is None and c is None
    assert np.array_equal(h1.cpu().numpy().view(np.uint64), r1)
    assert np.array_equal(k.cpu().numpy().view(np.uint64), rk)


@pytest.mark.gpu
def test_fused_csr_oversize_tiles_vs_oracle(cuda, oracle):
    """The fused epilogue on both CSR paths in one call: LDS-staged tiles and tiles whose
    span exceeds the stage (hashed by the ring pass with the epilogue fused there too),
    with h2 and both index outputs."""
    import torch
    rng = np.random.default_rng(12)
    L = rng.integers(0, 129, 512 * 5 + 33)
    for t in (0, 3):
        L[512 * t: 512 * (t + 1)] = rng.integers(160, 420, 512)
    off = np.zeros(L.size + 1, np.int64)
    off[1:] = np.cumsum(L)
    data = oracle.gen_bytes(int(off[-1]) + 3)
    r1, r2 = oracle.hash_csr(data, off.astype(np.uint64))
    h1, h2, k, c = k2hash_amd.hash_csr_index(torch.from_numpy(data).to(cuda), torch.from_numpy(off).to(cuda),
                                             (1 << 20) - 1, 0x7, second=True)
    torch.cuda.synchronize()
    rk, rc = oracle.bucket_index(r1, (1 << 20) - 1, 0x7)
    assert np.array_equal(h1.cpu().numpy().view(np.uint64), r1)
    assert np.array_equal(h2.cpu().numpy().view(np.uint64), r2)
    assert np.array_equal(k.cpu().numpy().view(np.uint64), rk)
    assert np.array_equal(c.cpu().numpy().view(np.uint64), rc)


@pytest.mark.gpu
@pytest.mark.parametrize("cfgname,cur,cm", [("fixed32_16M", 0xFF, 0xF), ("fixed32_16M", (1 << 28) - 1, 0xF),
                                             ("csr_8_256_64M", (1 << 24) - 1, 0x3F)])
def test_fused_full_size_vs_oracle(cuda, oracle, digests, cfgname, cur, cm):
    """Configs 2 and 3 at full size: h1 from the fused kernel matches the reference's digest
    (so it IS the reference's h1, key for key up to digest collisions), and the fused kindex /
    ckindex equal the oracle's restatement applied to that h1 -- not a self-comparison with
    the standalone kernel."""
    import torch
    cfg = digests[cfgname]
    if cfg["kind"] == "fixed":
        keys = batch.synth_bytes(cfg["n"] * cfg["key_len"], cuda)
        h1, _, k, c = k2hash_amd.hash_fixed_index(keys, cfg["key_len"], cur, cm)
    else:
        off = batch.synth_offsets(cfg["n"], cuda, cfg["min_len"], cfg["max_len"])
        keys = batch.synth_bytes(int(off[-1].item()), cuda)
        h1, _, k, c = k2hash_amd.hash_csr_index(keys, off, cur, cm)
    torch.cuda.synchronize()
    hh = h1.cpu().numpy().view(np.uint64)
    assert [f"{x:016x}" for x in oracle.digest(hh)] == cfg["h1"]
    rk, rc = oracle.bucket_index(hh, cur, cm)
    assert np.array_equal(k.cpu().numpy().view(np.uint64), rk)
    assert np.array_equal(c.cpu().numpy().view(np.uint64), rc)


# ---------------------------------------------------------------------------
# Table state: K2HShm::GetKIndex(hash, isMergeCurmask = false) over a snapshot of the
# assigned K_INDEX entries (lib/k2hshm.cc:862-907).  Parity is UNPINNED beyond the
# restatement: K2HShm::GetKIndex needs the mapped table and libfullock, so the reference
# function is not executed; the oracle's walk (oracle/fnv_oracle.c oracle_get_kindex) is
# checked here against an independent Python restatement, and with every entry assigned
# it must reduce to the pinned stateless GetKIndexPos.
# ---------------------------------------------------------------------------
def _py_get_kindex(h, cur_mask, cmask, flags):
    """lib/k2hshm.cc:882-907 in Python: flags[(p, a)] = assigned."""
    res, found = None, -1
    m = cur_mask
    while m > 0:
        shifted = h >> (cmask.bit_length() % 64)  # GetMaskBitCount, shift count mod 64
        tmp = shifted & m
        p = tmp.bit_length()
        a = shifted & ((1 << (p - 1)) - 1 if p else 0)
        res = (p, a)
        if flags(p, a):
            return res, 1
        found = 0
        m >>= 1
    return res, found


def _bitmap_from(flags_fn, cur_mask):
    bits = np.zeros(((cur_mask + 1 + 31) // 32) * 32, dtype=np.uint8)
    for v in range(cur_mask + 1):
        p = v.bit_length()
        a = v - (1 << (p - 1)) if p else 0
        bits[v] = flags_fn(p, a)
    return np.packbits(bits.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").astype(np.uint32).reshape(-1)


@pytest.mark.parametrize("cur_mask,cmask", [(0x3, 0x3), (0xFF, 0xF), (0x1, 0x0), (0x0, 0xF), (0x3FF, 0x0),
                                            ((1 << 12) - 1, (1 << 8) - 1)])
def test_get_kindex_restatement(oracle, cur_mask, cmask):
    rng = np.random.default_rng(cur_mask ^ cmask)
    h = rng.integers(0, 2**63, size=3000, dtype=np.int64).view(np.uint64) * np.uint64(2) + np.uint64(1)
    for density in (0.0, 0.3, 0.9, 1.0):
        table = {}

        def flags(p, a, _d=density):
            if (p, a) not in table:
                table[(p, a)] = bool(rng.random() < _d)
            return table[(p, a)]
        bm = _bitmap_from(flags, cur_mask)
        k, c, f = oracle.bucket_index_table(h, cur_mask, cmask, bm)
        for i in range(0, 3000, 7):
            (res, fnd) = _py_get_kindex(int(h[i]), cur_mask, cmask, lambda p, a: table[(p, a)])
            if fnd < 0:
                assert int(k[i]) == (1 << 64) - 1 and f[i] == 0
            else:
                assert (int(k[i]) >> 58, int(k[i]) & ((1 << 58) - 1)) == res and f[i] == fnd
            assert int(c[i]) == int(h[i]) & cmask
    # every entry assigned: GetKIndex == GetKIndexPos (the pinned stateless part)
    full = _bitmap_from(lambda p, a: True, cur_mask)
    k, c, f = oracle.bucket_index_table(h, cur_mask, cmask, full)
    ks, cs = oracle.bucket_index(h, cur_mask, cmask)
    if cur_mask:
        assert np.array_equal(k, ks) and np.array_equal(c, cs) and f.all()


def test_expanded_table_bitmap_layout():
    bm = batch.expanded_table_bitmap(0xFF, 0.5, seed=3)
    assert bm.dtype == np.uint32 and bm.size == 8
    bits = np.unpackbits(bm.astype(">u4").view(np.uint8).reshape(-1, 4), axis=1).reshape(-1, 32)[:, ::-1].reshape(-1)
    assert bits[:128].all() and 0 < bits[128:].sum() < 128


# ------------------------------------------------------------------------- GPU
TABLES = [(0xFF, 0xF, 0.5), ((1 << 20) - 1, 0xF, 0.3), ((1 << 16) - 1, 0x0, 0.0), (0x3, 0x3, 0.9),
          ((1 << 24) - 1, (1 << 4) - 1, 1.0), (0x0, 0xF, 1.0), (0x1, 0x0, 0.0)]


@pytest.mark.gpu
@pytest.mark.parametrize("cur_mask,cmask,frac", TABLES)
def test_table_index_gpu_vs_oracle(cuda, oracle, cur_mask, cmask, frac):
    """Standalone and fused (fixed 32 B, CSR) table-state index vs the oracle's GetKIndex
    walk, on tables just expanded to cur_mask (top area partly arranged) and on random
    per-entry bitmaps."""
    import torch
    n = 200003
    data = oracle.gen_bytes(32 * n, byte_off=99)
    r1, _ = oracle.hash_fixed(data, 32)
    bms = [batch.expanded_table_bitmap(cur_mask, frac, seed=7)]
    rng = np.random.default_rng(cur_mask)
    bms.append(rng.integers(0, 2**32, size=(cur_mask + 1 + 31) // 32, dtype=np.uint64).astype(np.uint32))
    keys = torch.from_numpy(data).to(cuda)
    h1 = torch.from_numpy(r1.view(np.int64).copy()).to(cuda)
    off = oracle.gen_offsets(20011, 0, 300)
    cdata = oracle.gen_bytes(int(off[-1]))
    c1, _ = oracle.hash_csr(cdata, off)
    for bm in bms:
        ok, oc, of = oracle.bucket_index_table(r1, cur_mask, cmask, bm)
        assigned = torch.from_numpy(bm.view(np.int32).copy()).to(cuda)
        k, c, f = batch.bucket_index_table(h1, cur_mask, cmask, assigned)
        g1, _, gk, gc, gf = batch.hash_fixed_index_table(keys, 32, cur_mask, cmask, assigned)
        torch.cuda.synchronize()
        for kk, cc, ff in ((k, c, f), (gk, gc, gf)):
            assert np.array_equal(kk.cpu().numpy().view(np.uint64), ok)
            assert np.array_equal(cc.cpu().numpy().view(np.uint64), oc)
            assert np.array_equal(ff.cpu().numpy(), of)
        assert np.array_equal(g1.cpu().numpy().view(np.uint64), r1)
        ck, cc_, cf = oracle.bucket_index_table(c1, cur_mask, cmask, bm)
        x1, x2, xk, xc, xf = batch.hash_csr_index_table(torch.from_numpy(cdata).to(cuda),
                                                        torch.from_numpy(off.astype(np.int64)).to(cuda),
                                                        cur_mask, cmask, assigned, second=True)
        torch.cuda.synchronize()
        assert np.array_equal(x1.cpu().numpy().view(np.uint64), c1)
        assert np.array_equal(xk.cpu().numpy().view(np.uint64), ck)
        assert np.array_equal(xc.cpu().numpy().view(np.uint64), cc_)
        assert np.array_equal(xf.cpu().numpy(), cf)


@pytest.mark.gpu
def test_table_index_null_bitmap_is_stateless(cuda, oracle):
    """assigned = NULL: every entry assigned, so the table form equals the stateless one."""
    import torch
    h = oracle.gen_bytes(8 * 50000).view(np.uint64)
    th = torch.from_numpy(h.view(np.int64).copy()).to(cuda)
    k, c, f = batch.bucket_index_table(th, 0xFFFF, 0xF, None)
    ks, cs = batch.bucket_index(th, 0xFFFF, 0xF)
    torch.cuda.synchronize()
    assert torch.equal(k, ks) and torch.equal(c, cs) and bool((f == 1).all())
    with pytest.raises(ValueError):  # bitmap shorter than cur_mask + 1 bits
        batch.bucket_index_table(th, 0xFFFF, 0xF, torch.zeros(100, dtype=torch.int32, device=cuda))
    # cur_mask 0: GetKIndex returns NULL (lib/k2hshm.cc:882-907) -> K2H_AMD_KINDEX_NONE and
    # found 0, the same with a NULL bitmap as with an all-ones one, in the
    # standalone and both fused forms
    ones = torch.full((1,), -1, dtype=torch.int32, device=cuda)
    keys = torch.from_numpy(oracle.gen_bytes(32 * 5000)).to(cuda)
    off = oracle.gen_offsets(3000, 0, 200)
    cdata = torch.from_numpy(oracle.gen_bytes(int(off[-1]))).to(cuda)
    coff = torch.from_numpy(off.astype(np.int64)).to(cuda)
    for assigned in (None, ones):
        outs = [batch.bucket_index_table(th, 0, 0xF, assigned)[:3],
                batch.hash_fixed_index_table(keys, 32, 0, 0xF, assigned)[2:],
                batch.hash_csr_index_table(cdata, coff, 0, 0xF, assigned)[2:]]
        torch.cuda.synchronize()
        for k0, c0, f0 in outs:
            assert bool((k0 == -1).all()) and bool((f0 == 0).all()), assigned
    # offsets on another device than the bytes: rejected before any launch
    with pytest.raises(ValueError):
        batch.hash_csr_index_table(cdata, coff.cpu(), 0xFF, 0xF)
