"""RALLEDATA producer: GPU-built direct-set blobs vs the
reference layout.

Pins: tests/golden/ralledata.json is written by oracle/gen_ralledata.cc, which is
compiled against the REFERENCE's own lib/k2hash.h + lib/k2hshmdirect.h (struct
RALLEDATA, ralledata_init, calc_ralledata_length) and hashes with the reference's
lib/k2hashfunc.cc build, laying blobs out as K2HShm::GetElementToBinary does
(lib/k2hshmdirect.cc:59-88).  The oracle restatement (oracle_build_ralledata) must equal
it byte for byte; the HIP producer must equal both.
"""
import json

import numpy as np
import pytest

from conftest import GOLDEN

from k2hash_amd import ralledata


@pytest.fixture(scope="module")
def golden():
    g = json.loads((GOLDEN / "ralledata.json").read_text())
    recs = g["records"]
    b = bytes.fromhex
    return g, [b(r["key"]) for r in recs], [b(r["val"]) for r in recs], [b(r["skey"]) for r in recs], \
        [b(r["attrs"]) for r in recs], b"".join(b(r["blob"]) for r in recs)


# ------------------------------------------------------------------------- CPU
def test_reference_struct_layout(golden):
    g = golden[0]
    assert g["sizeof_RALLEDATA"] == ralledata.HEADER == 80
    assert [g["offsets"][f] for f in ralledata._FIELDS] == list(range(0, 80, 8))


def test_oracle_matches_reference_fixture(oracle, golden):
    _, k, v, s, a, blob = golden
    out, boff = oracle.build_ralledata(k, v, s, a)
    assert out.tobytes() == blob
    assert int(boff[-1]) == len(blob)


def test_parse_blob_fields(oracle, golden):
    _, k, v, s, a, blob = golden
    o = 0
    for i in range(len(k)):
        n = 80 + len(k[i]) + len(v[i]) + len(s[i]) + len(a[i])
        p = ralledata.parse_blob(blob[o:o + n])
        assert (p.key, p.val, p.skey, p.attrs) == (k[i], v[i], s[i], a[i])
        assert p.hash == oracle.k2h_hash(k[i]) and p.subhash == oracle.k2h_second_hash(k[i])
        o += n
    assert o == len(blob)


def test_empty_batch_needs_no_gpu():
    out, boff = ralledata.build_ralledata_host([])
    assert out.size == 0 and list(boff) == [0]


# ------------------------------------------------------------------------- GPU
def _dev(torch, cuda, parts):
    data = np.frombuffer(b"".join(parts), np.uint8).copy() if any(parts) else np.zeros(1, np.uint8)
    off = np.zeros(len(parts) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in parts])
    return torch.from_numpy(data).to(cuda), torch.from_numpy(off).to(cuda)


@pytest.mark.gpu
def test_device_matches_reference_fixture(cuda, golden):
    import torch
    _, k, v, s, a, blob = golden
    segs = [_dev(torch, cuda, x) for x in (k, v, s, a)]
    out, boff = ralledata.build_ralledata(*segs[0], *segs[1], *segs[2], *segs[3])
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == blob
    o = boff.cpu().numpy()
    assert o[0] == 0 and o[-1] == len(blob)


@pytest.mark.gpu
def test_host_matches_reference_fixture(cuda, golden):
    _, k, v, s, a, blob = golden
    out, boff = ralledata.build_ralledata_host(k, v, s, a)
    assert out.tobytes() == blob and int(boff[-1]) == len(blob)


@pytest.mark.gpu
@pytest.mark.parametrize("segments", ["kv", "k", "kvsa", "ka"])
def test_device_vs_oracle_random(cuda, oracle, segments):
    import torch
    rng = np.random.default_rng(len(segments))
    n = 50021
    data = oracle.gen_bytes(n * 700, byte_off=1234)
    pos = 0

    def take(lo, hi, p_empty):
        nonlocal pos
        out = []
        for _ in range(n):
            L = 0 if rng.random() < p_empty else int(rng.integers(lo, hi))
            out.append(data[pos:pos + L].tobytes())
            pos += L
        return out
    k = take(1, 300, 0.0)
    v = take(0, 260, 0.2) if "v" in segments else None
    s = take(0, 40, 0.5) if "s" in segments else None
    a = take(0, 60, 0.5) if "a" in segments else None
    ref, rboff = oracle.build_ralledata(k, v, s, a)
    segs = []
    for x in (k, v, s, a):
        segs += list(_dev(torch, cuda, x)) if x is not None else [None, None]
    out, boff = ralledata.build_ralledata(*segs)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert np.array_equal(boff.cpu().numpy().view(np.uint64), rboff)


@pytest.mark.gpu
def test_device_nonzero_first_offsets(cuda, oracle):
    """Offsets relative to the byte pointers need not start at 0 (a window of a larger
    batch), and the blob offsets are relative to the window."""
    import torch
    k = [bytes([i % 251]) * (1 + i % 37) for i in range(3000)]
    v = [bytes([i % 13]) * (i % 50) for i in range(3000)]
    ref, rboff = oracle.build_ralledata(k[1000:], v[1000:])
    kd, ko = _dev(torch, cuda, k)
    vd, vo = _dev(torch, cuda, v)
    out, boff = ralledata.build_ralledata(kd, ko[1000:].contiguous(), vd, vo[1000:].contiguous())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert np.array_equal(boff.cpu().numpy().view(np.uint64), rboff)


def _random_records(oracle, n, segments, klen, vlen, slen=(0, 16), alen=(0, 24), big_every=0, seed=0):
    rng = np.random.default_rng(seed)
    data = oracle.gen_bytes(n * (klen[1] + vlen[1] + slen[1] + alen[1]) + 64 * 1024 + 16, byte_off=77)
    pos = 0

    def take(lo, hi, p_empty, big=0):
        nonlocal pos
        out = []
        for i in range(n):
            L = 0 if rng.random() < p_empty else int(rng.integers(lo, hi))
            if big and i % big == big - 1:
                L = 5000
            out.append(data[pos % (len(data) - 6000):][:L].tobytes())
            pos += L
        return out
    k = take(*klen, 0.02)
    v = take(*vlen, 0.2, big_every) if "v" in segments else None
    s = take(*slen, 0.5) if "s" in segments else None
    a = take(*alen, 0.5) if "a" in segments else None
    return k, v, s, a


@pytest.mark.gpu
@pytest.mark.parametrize("segments", ["kv", "k", "kvsa", "ka", "kv_big", "kv_unaligned"])
def test_device_gather_form_vs_oracle(cuda, oracle, segments):
    """BASELINE-like records (keys 0-64 B, values 0-200 B): blocks of 64 records are staged
    in LDS and written as aligned pieces (the gather form); `_big` puts a 5000-B value in
    every 97th record so some blocks take the group form next to staged ones;
    `_unaligned` offsets every input and the output by a few bytes."""
    import torch
    n = 20011
    k, v, s, a = _random_records(oracle, n, segments.split("_")[0], (0, 65), (0, 201),
                                 big_every=97 if segments.endswith("big") else 0, seed=len(segments))
    ref, rboff = oracle.build_ralledata(k, v, s, a)
    segs = []
    shift = 0
    for x in (k, v, s, a):
        if x is None:
            segs += [None, None]
            continue
        d, o = _dev(torch, cuda, x)
        if segments.endswith("unaligned"):
            shift += 3
            pad = torch.zeros(d.numel() + shift, dtype=torch.uint8, device=cuda)
            pad[shift:] = d
            d, o = pad, o + shift  # same bytes, data pointer still the tensor start: offsets move
            d = d[1:]
            o = o - 1
        segs += [d, o]
    if segments.endswith("unaligned"):
        total = len(ref)
        big = torch.zeros(total + 16, dtype=torch.uint8, device=cuda)
        out, boff = ralledata.build_ralledata(*segs, out=big[5:5 + total], total=total)
    else:
        out, boff = ralledata.build_ralledata(*segs)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(got, ref), f"first diff at {int(np.argmax(got != ref))}"
    assert np.array_equal(boff.cpu().numpy().view(np.uint64), rboff)
    if segments.endswith("unaligned"):
        b = big.cpu().numpy()
        assert not b[:5].any() and not b[5 + total:].any()  # nothing outside the blob span


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 1000])
@pytest.mark.parametrize("std_fnv", [False, True])
def test_device_small_batches_and_std_fnv(cuda, oracle, n, std_fnv):
    """Partial tiles (n not a multiple of 64), a single record, and the std::FNV seed
    (K2H_AMD_FLAG_STD_FNV, oracle variant 1) through the fused hash of the gather form."""
    import torch
    k, v, s, a = _random_records(oracle, n, "kvs", (0, 65), (0, 201), seed=n)
    ref, rboff = oracle.build_ralledata(k, v, s, a, variant=1 if std_fnv else 0)
    segs = []
    for x in (k, v, s, a):
        segs += list(_dev(torch, cuda, x)) if x is not None else [None, None]
    out, boff = ralledata.build_ralledata(*segs, std_fnv=std_fnv)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert np.array_equal(boff.cpu().numpy().view(np.uint64), rboff)


@pytest.mark.gpu
def test_device_stage_boundary(cuda, oracle):
    """Tiles whose staged spans sit right at the 12 KiB stage limit, on both sides: 64
    records per tile with values sized so a tile's key + value hull is 12288 +- 32 bytes;
    the tiles that do not fit take the group form in the same kernel."""
    import torch
    n = 64 * 40
    k, v = [], []
    data = oracle.gen_bytes(n * 300, byte_off=5)
    pos = 0
    for t in range(40):
        target = 12288 + (t % 5 - 2) * 16  # key + value bytes of the tile
        per = target // 64
        for j in range(64):
            kl = 8 + (j * 7 + t) % 24
            vl = max(0, per - kl + (1 if j < target - per * 64 else 0))
            k.append(data[pos:pos + kl].tobytes())
            pos += kl
            v.append(data[pos:pos + vl].tobytes())
            pos += vl
    ref, rboff = oracle.build_ralledata(k, v)
    kd, ko = _dev(torch, cuda, k)
    vd, vo = _dev(torch, cuda, v)
    out, boff = ralledata.build_ralledata(kd, ko, vd, vo)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert np.array_equal(boff.cpu().numpy().view(np.uint64), rboff)


@pytest.mark.gpu
def test_device_fuzz(cuda, oracle):
    """Seeded fuzz of the device producer: 40 batches with random record counts, segment
    sets, length ranges (empty segments included), input and output alignments -- every
    tile edge and piece/segment boundary position the gather form's alignment math meets."""
    import torch
    rng = np.random.default_rng(2024)
    data = oracle.gen_bytes(1 << 21, byte_off=99)
    for it in range(40):
        n = int(rng.integers(1, 1500))
        present = [True] + [bool(rng.integers(0, 2)) for _ in range(3)]
        hi = [int(rng.integers(1, 80)), int(rng.integers(1, 300)), int(rng.integers(1, 40)), int(rng.integers(1, 40))]
        segs_b, pos = [], int(rng.integers(0, 1000))
        for s in range(4):
            if not present[s]:
                segs_b.append(None)
                continue
            lens = rng.integers(0, hi[s] + 1, n)
            lens[rng.random(n) < 0.1] = 0
            parts = []
            for L in lens:
                parts.append(data[pos % (len(data) - 400):][:int(L)].tobytes())
                pos += int(L)
            segs_b.append(parts)
        ref, rboff = oracle.build_ralledata(*segs_b)
        args = []
        for parts in segs_b:
            if parts is None:
                args += [None, None]
                continue
            d, o = _dev(torch, cuda, parts)
            sh = int(rng.integers(0, 16))  # the bytes at a random alignment, offsets shifted to match
            pad = torch.zeros(d.numel() + sh, dtype=torch.uint8, device=cuda)
            pad[sh:] = d
            args += [pad, o + sh]
        total = len(ref)
        osh = int(rng.integers(0, 16))
        big = torch.zeros(total + 32, dtype=torch.uint8, device=cuda)
        out, boff = ralledata.build_ralledata(*args, out=big[osh:osh + total], total=total)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert np.array_equal(got, ref), f"batch {it}: n={n} segs={present} first diff {int(np.argmax(got != ref))}"
        assert np.array_equal(boff.cpu().numpy().view(np.uint64), rboff), f"batch {it}"
        b = big.cpu().numpy()
        assert not b[:osh].any() and not b[osh + total:].any(), f"batch {it}: bytes outside the span"
