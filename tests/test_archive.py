"""Bulk key streams: k2hash archive scan + GPU prehash, and keys
at arbitrary ranges (with the C-string form k2himport's loaders store).

Pins: tests/golden/archive.k2har holds records written by the REFERENCE's own
K2HCommandArchive (lib/k2hcommand.cc, compiled from /root/reference by
oracle/gen_archive.cc, appended as K2HArchive::Save does, lib/k2harchive.cc:166-185),
and tests/golden/archive.json their keys hashed by the reference's lib/k2hashfunc.cc.
"""
import json

import numpy as np
import pytest

from conftest import GOLDEN, u64

from k2hash_amd import archive


@pytest.fixture(scope="module")
def ar():
    return (GOLDEN / "archive.k2har").read_bytes(), json.loads((GOLDEN / "archive.json").read_text())


# ------------------------------------------------------------------------- CPU
def test_scan_matches_reference_archive(ar):
    f, g = ar
    assert g["sizeof_SCOM"] == 104 and g["size"] == len(f)
    r = archive.scan(f)
    assert r.size == len(g["records"])
    for x, e in zip(r, g["records"]):
        assert int(x["type"]) == e["type"] and int(x["offset"]) == e["offset"] and int(x["status"]) == 0
        assert f[int(x["key_off"]):int(x["key_off"]) + int(x["key_len"])].hex() == e["key"]
        assert (int(x["val_len"]), int(x["skey_len"]), int(x["attrs_len"]), int(x["exdata_len"])) == \
            (e["val_length"], e["skey_length"], e["attr_length"], e["exdata_length"])
        assert f[int(x["exdata_off"]):int(x["exdata_off"]) + int(x["exdata_len"])].hex() == e["exdata"]
        assert 104 + int(x["key_len"] + x["val_len"] + x["skey_len"] + x["attrs_len"] + x["exdata_len"]) == e["total"]
    assert {int(t) for t in r["type"]} == set(range(7))  # every SCOM type occurs


def test_scan_stops_like_load(ar):
    """K2HArchive::Load ends at the first offset where a whole 104-byte header cannot be
    read (lib/k2harchive.cc:293, 385-405); a record whose data runs past the end is
    reported TRUNCATED; an unknown type is reported BAD_TYPE and skipped over."""
    f, g = ar
    last = g["records"][-1]
    r = archive.scan(f[:last["offset"] + 50])  # partial header: not a record
    assert r.size == len(g["records"]) - 1
    r = archive.scan(f[:last["offset"] + 104 + 1])  # whole header, truncated data
    assert r.size == len(g["records"]) and int(r[-1]["status"]) == archive.STATUS_TRUNCATED
    bad = bytearray(f)
    bad[g["records"][3]["offset"] + 16] = 99  # type field of record 3
    r = archive.scan(bytes(bad))
    assert r.size == len(g["records"]) and int(r[3]["status"]) == archive.STATUS_BAD_TYPE
    assert archive.scan(b"").size == 0 and archive.scan(b"\0" * 103).size == 0


# ------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_prehash_matches_reference_hashes(ar, oracle):
    f, g = ar
    h1, h2, nh1, nh2 = archive.prehash(f, rename=True)
    for i, e in enumerate(g["records"]):
        assert (int(h1[i]), int(h2[i])) == (u64(e["h1"]), u64(e["h2"])), i
        if e["type"] == archive.SCOM_RENAME:
            new = bytes.fromhex(e["exdata"])
            assert (int(nh1[i]), int(nh2[i])) == (oracle.k2h_hash(new), oracle.k2h_second_hash(new))
        else:
            assert int(nh1[i]) == 0


@pytest.mark.gpu
def test_prehash_bad_records_hash_to_zero(ar):
    f, g = ar
    bad = bytearray(f)
    bad[g["records"][3]["offset"] + 16] = 99
    h1, h2 = archive.prehash(bytes(bad))
    assert int(h1[3]) == 0 and int(h2[3]) == 0
    assert int(h1[4]) == u64(g["records"][4]["h1"])


@pytest.mark.gpu
@pytest.mark.parametrize("cstr", [False, True])
def test_hash_ranges_vs_oracle(cuda, oracle, cstr):
    import torch
    rng = np.random.default_rng(3 + cstr)
    base = oracle.gen_bytes(1 << 20, byte_off=77)
    n = 20000
    lens = rng.integers(0, 120, n)
    lens[::13] = 0
    starts = rng.integers(0, base.size - 200, n)
    h1, h2 = archive.hash_ranges(torch.from_numpy(base).to(cuda), torch.from_numpy(starts).to(cuda),
                                 torch.from_numpy(lens).to(cuda), second=True, cstr=cstr)
    torch.cuda.synchronize()
    a, b = h1.cpu().numpy().view(np.uint64), h2.cpu().numpy().view(np.uint64)
    for i in range(0, n, 7):
        k = base[starts[i]:starts[i] + lens[i]].tobytes() + (b"\0" if cstr else b"")
        assert (int(a[i]), int(b[i])) == (oracle.k2h_hash(k), oracle.k2h_second_hash(k)), (i, lens[i])
