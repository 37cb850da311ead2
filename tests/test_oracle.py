"""The oracle (oracle/fnv_oracle.c) pinned against the reference.

Pins, in order of strength:
  1. the reference itself, compiled from /root/reference/lib/k2hashfunc.cc into
     oracle/_ref (skipped where that build is absent, e.g. on the GPU box);
  2. the committed golden vectors and digests in tests/golden/, generated from
     that build by oracle/gen_golden.c;
  3. the reference's own test pins: tests/test_linetool_dsave.cmd:29-50 with
     tests/test_linetool.log:2756-2768 (key1\\0 and key27\\0 share a collision
     slot at -cmask 2, i.e. the low 4 bits of their hashes agree) and the
     "0123456789" keys printed by tests/k2hexttest.cc:166-175.
"""
import random

import numpy as np
import pytest

from conftest import hexkey, u64


def test_vectors_default(oracle, vectors):
    assert vectors["version"] == "FNV-1A BUILTIN"
    for v in vectors["vectors"]:
        k = hexkey(v)
        assert oracle.k2h_hash(k) == u64(v["h1"]), v["tag"]
        assert oracle.k2h_second_hash(k) == u64(v["h2"]), v["tag"]


def test_vectors_std_fnv(oracle, vectors):
    assert vectors["std_fnv_version"] == "STD::FNV BUILTIN"
    for v in vectors["std_fnv_vectors"]:
        k = hexkey(v)
        assert oracle.k2h_hash(k, 1) == u64(v["h1"]), v["tag"]
        assert oracle.k2h_second_hash(k, 1) == u64(v["h2"]), v["tag"]


def test_version_strings(oracle):
    assert oracle.lib().oracle_k2h_hash_version(0) == b"FNV-1A BUILTIN"  # lib/k2hashfunc.cc:38
    assert oracle.lib().oracle_k2h_hash_version(1) == b"STD::FNV BUILTIN"  # lib/k2hashfunc.cc:36


def test_reference_dsave_pin(oracle):
    # tests/test_linetool_dsave.cmd:29-50: -mask 2 -cmask 2; key1 and key27 ("char*" keys,
    # hashed with their NUL, lib/k2hshm.cc:1238) land in the same collision slot.
    a, b = oracle.k2h_hash(b"key1\0"), oracle.k2h_hash(b"key27\0")
    assert a & 0xF == b & 0xF == 5


def test_sign_extension(oracle):
    # bytes >= 0x80 are sign-extended (lib/k2hashfunc.cc:53,55): differs from canonical FNV-1a
    canonical = 0xcbf29ce484222325
    canonical = ((canonical ^ 0x80) * 0x100000001b3) & (2**64 - 1)
    assert oracle.k2h_hash(b"\x80") == 0x509c0cb379fdec5f != canonical == 0xaf643d4c8602915f


def test_batch_forms_match_scalar(oracle):
    rng = random.Random(7)
    keys = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 70))) for _ in range(300)]
    data = np.frombuffer(b"".join(keys), np.uint8)
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    h1, h2 = oracle.hash_csr(data, off)
    for i, k in enumerate(keys):
        assert int(h1[i]) == oracle.k2h_hash(k)
        assert int(h2[i]) == oracle.k2h_second_hash(k)
    fx = oracle.gen_bytes(21 * 100)
    g1, g2 = oracle.hash_fixed(fx, 21)
    for i in range(100):
        k = fx[21 * i:21 * i + 21].tobytes()
        assert int(g1[i]) == oracle.k2h_hash(k) and int(g2[i]) == oracle.k2h_second_hash(k)


def test_generator_spec(oracle):
    # splitmix64 counter form: word j = j-th output of splitmix64(seed)
    seed = oracle.SEED_BYTES
    state = seed
    words = []
    for _ in range(4):
        state = (state + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        words.append(z ^ (z >> 31))
    b = oracle.gen_bytes(32, seed)
    assert b.tobytes() == b"".join(w.to_bytes(8, "little") for w in words)
    assert oracle.gen_bytes(7, seed, 5).tobytes() == b[5:12].tobytes()
    off = oracle.gen_offsets(1000)
    lens = np.diff(off.astype(np.int64))
    assert lens.min() >= 8 and lens.max() <= 256 and off[0] == 0


def _digest_fixed(oracle, key_len, n, first=0):
    data = oracle.gen_bytes(key_len * n, byte_off=key_len * first)
    h1, h2 = oracle.hash_fixed(data, key_len)
    return oracle.digest(h1, first), oracle.digest(h2, first)


@pytest.mark.parametrize("name", ["fixed32_64K", "fixed21_1M"])
def test_digests_fixed(oracle, digests, name):
    cfg = digests[name]
    d1, d2 = _digest_fixed(oracle, cfg["key_len"], cfg["n"])
    assert [f"{x:016x}" for x in d1] == cfg["h1"]
    assert [f"{x:016x}" for x in d2] == cfg["h2"]


def test_digests_chunks_combine(oracle, digests):
    # digest of a shard starting at global key `first` composes with the others
    cfg = digests["fixed21_1M"]
    c = cfg["chunks"][3]
    d1, _ = _digest_fixed(oracle, 21, c["count"], c["first"])
    assert [f"{x:016x}" for x in d1] == c["h1"]


def test_digest_csr(oracle, digests):
    cfg = digests["csr_8_256_64K"]
    off = oracle.gen_offsets(cfg["n"], cfg["min_len"], cfg["max_len"])
    data = oracle.gen_bytes(int(off[-1]))
    h1, h2 = oracle.hash_csr(data, off)
    assert [f"{x:016x}" for x in oracle.digest(h1)] == cfg["h1"]
    assert [f"{x:016x}" for x in oracle.digest(h2)] == cfg["h2"]
    assert oracle.digest(h1) == oracle.digest_np(h1)


# --- against the reference build itself (this container only) -------------------------
def _ref(oracle, path):
    if not path.exists() and not oracle.build_ref():
        pytest.skip("reference build unavailable (no /root/reference here)")
    return oracle.RefLib(path)


def test_against_reference_random(oracle):
    ref = _ref(oracle, oracle.REF_SO)
    assert ref.version() == "FNV-1A BUILTIN"
    rng = random.Random(1234)
    for n in list(range(0, 70)) + [127, 128, 129, 255, 256, 1000, 4096]:
        for _ in range(5):
            k = bytes(rng.getrandbits(8) for _ in range(n))
            assert oracle.k2h_hash(k) == ref.k2h_hash(k)
            assert oracle.k2h_second_hash(k) == ref.k2h_second_hash(k)


def test_against_reference_std_fnv(oracle):
    ref = _ref(oracle, oracle.REF_STD_SO)
    assert ref.version() == "STD::FNV BUILTIN"
    rng = random.Random(99)
    for n in range(0, 80):
        k = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.k2h_hash(k, 1) == ref.k2h_hash(k)
        assert oracle.k2h_second_hash(k, 1) == ref.k2h_second_hash(k)


def test_fnv_split_every_point(oracle):
    """The two-lane split of one key's chain (oracle_fnv_split): the
    low-byte chain v' = 0xB3 (v ^ b) plus the signed affine accumulation reproduce the
    direct chain at EVERY split point of a 4 KiB key -- the SURVEY vector
    b[i] = (i*131+7) & 0xFF and random keys full of bytes >= 0x80 -- for both seeds."""
    import ctypes

    L = oracle.lib()
    L.oracle_fnv_split_mismatches.restype = ctypes.c_size_t
    L.oracle_fnv_split_mismatches.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    L.oracle_fnv_split.restype = ctypes.c_uint64
    L.oracle_fnv_split.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint64]
    keys = [np.array([(i * 131 + 7) & 0xFF for i in range(4096)], np.uint8),
            np.random.default_rng(11).integers(0, 256, 4096, dtype=np.uint8),
            np.full(4096, 0xFF, np.uint8), np.full(300, 0x80, np.uint8)]
    keys += [np.random.default_rng(k).integers(0x70, 0x90, k, dtype=np.uint8) for k in range(0, 70)]
    for k in keys:
        for seed in (14695981039346656037, 2166136261):
            assert L.oracle_fnv_split_mismatches(k.ctypes.data, k.size, seed) == 0, (k.size, seed)
    k = keys[0]
    assert L.oracle_fnv_split(k.ctypes.data, 4096, 2048, 14695981039346656037) == 0x4dbdf6ea6a33a325
