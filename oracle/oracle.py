"""ORACLE -- TEST INFRASTRUCTURE ONLY.

ctypes wrapper over oracle/_build/libfnv_oracle.so (the plain-C restatement in
fnv_oracle.c) and, when present, oracle/_ref/libk2hfunc_ref.so (the reference's
own lib/k2hashfunc.cc compiled by oracle/Makefile).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by k2hash_amd/.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
BUILD = HERE / "_build"
REF = HERE / "_ref"
ORACLE_SO = BUILD / "libfnv_oracle.so"
CPUBENCH_SO = BUILD / "libk2h_cpubench.so"
REF_SO = REF / "libk2hfunc_ref.so"
REF_STD_SO = REF / "libk2hfunc_ref_stdfnv.so"
REF_TESTHASH_SO = REF / "libk2htesthash_ref.so"
REF_CONFORMANCE = REF / "dynlib_conformance"

SEED_BYTES = 0x6B32686173680001
SEED_LENS = 0x6B32686173680002

_u64, _p, _sz = ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t


def build() -> None:
    """Compile the restatement (always possible: gcc only)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def build_ref() -> bool:
    """Compile the reference's own hash path from /root/reference, if present."""
    if not Path("/root/reference/lib/k2hashfunc.cc").exists():
        return REF_SO.exists()
    subprocess.run(["make", "-s", "-C", str(HERE), "ref"], check=True)
    return True


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not ORACLE_SO.exists() or not CPUBENCH_SO.exists():
            build()
        L = ctypes.CDLL(str(ORACLE_SO))
        L.oracle_fnv.restype, L.oracle_fnv.argtypes = _u64, [_p, _sz, _u64]
        L.oracle_k2h_hash.restype, L.oracle_k2h_hash.argtypes = _u64, [_p, _sz, ctypes.c_int]
        L.oracle_k2h_second_hash.restype, L.oracle_k2h_second_hash.argtypes = _u64, [_p, _sz, ctypes.c_int]
        L.oracle_k2h_hash_version.restype, L.oracle_k2h_hash_version.argtypes = ctypes.c_char_p, [ctypes.c_int]
        L.oracle_hash_csr.restype = None
        L.oracle_hash_csr.argtypes = [_p, _p, _sz, _p, _p, ctypes.c_int]
        L.oracle_hash_fixed.restype = None
        L.oracle_hash_fixed.argtypes = [_p, _sz, _sz, _p, _p, ctypes.c_int]
        L.oracle_gen_bytes.restype = None
        L.oracle_gen_bytes.argtypes = [_u64, _u64, _sz, _p]
        L.oracle_gen_offsets.restype = None
        L.oracle_gen_offsets.argtypes = [_u64, _u64, _sz, ctypes.c_uint32, ctypes.c_uint32, _u64, _p]
        L.oracle_digest.restype = None
        L.oracle_digest.argtypes = [_p, _sz, _u64, _p]
        L.oracle_splitmix_word.restype, L.oracle_splitmix_word.argtypes = _u64, [_u64, _u64]
        L.oracle_make_mask.restype, L.oracle_make_mask.argtypes = _u64, [ctypes.c_int]
        L.oracle_mask_bitcount.restype, L.oracle_mask_bitcount.argtypes = ctypes.c_int, [_u64]
        L.oracle_kindex_pos.restype = None
        L.oracle_kindex_pos.argtypes = [_u64, _u64, _u64, _p, _p, _p]
        L.oracle_build_ralledata.restype = _u64
        L.oracle_build_ralledata.argtypes = [_p, _p, _p, _p, _p, _p, _p, _p, _sz, _p, _p, ctypes.c_int]
        L.oracle_bucket_index.restype = None
        L.oracle_bucket_index.argtypes = [_p, _sz, _u64, _u64, _p, _p]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(1)


def k2h_hash(data: bytes, variant: int = 0) -> int:
    return int(lib().oracle_k2h_hash(data, len(data), variant))


def k2h_second_hash(data: bytes, variant: int = 0) -> int:
    return int(lib().oracle_k2h_second_hash(data, len(data), variant))


def hash_fixed(keys: np.ndarray, key_len: int, variant: int = 0):
    keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
    n = keys.size // key_len
    h1 = np.empty(n, np.uint64)
    h2 = np.empty(n, np.uint64)
    lib().oracle_hash_fixed(_ptr(keys), key_len, n, _ptr(h1), _ptr(h2), variant)
    return h1, h2


def hash_csr(data: np.ndarray, offsets: np.ndarray, variant: int = 0):
    data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64).reshape(-1)
    n = offsets.size - 1
    h1 = np.empty(n, np.uint64)
    h2 = np.empty(n, np.uint64)
    lib().oracle_hash_csr(_ptr(data), _ptr(offsets), n, _ptr(h1), _ptr(h2), variant)
    return h1, h2


def gen_bytes(nbytes: int, seed: int = SEED_BYTES, byte_off: int = 0) -> np.ndarray:
    out = np.empty(nbytes, np.uint8)
    lib().oracle_gen_bytes(seed, byte_off, nbytes, _ptr(out))
    return out


def gen_offsets(n: int, min_len: int = 8, max_len: int = 256, seed: int = SEED_LENS, first_key: int = 0,
                base: int = 0) -> np.ndarray:
    out = np.empty(n + 1, np.uint64)
    lib().oracle_gen_offsets(seed, first_key, n, min_len, max_len, base, _ptr(out))
    return out


def digest(h: np.ndarray, first_index: int = 0) -> tuple[int, int, int]:
    h = np.ascontiguousarray(h).view(np.uint64)
    out = np.zeros(3, np.uint64)
    lib().oracle_digest(_ptr(h), h.size, first_index, _ptr(out))
    return int(out[0]), int(out[1]), int(out[2])


def digest_np(h: np.ndarray, first_index: int = 0) -> tuple[int, int, int]:
    """numpy restatement of oracle_digest (independent cross-check)."""
    h = np.ascontiguousarray(h).view(np.uint64)
    with np.errstate(over="ignore"):
        w = (2 * (np.arange(h.size, dtype=np.uint64) + np.uint64(first_index)) + np.uint64(1))
        return (int(np.bitwise_xor.reduce(h)) if h.size else 0, int(h.sum(dtype=np.uint64)),
                int((h * w).sum(dtype=np.uint64)))


class RefLib:
    """The reference's compiled hash functions (oracle/_ref), for parity pinning."""

    def __init__(self, path: Path = REF_SO):
        self.path = path
        L = ctypes.CDLL(str(path))
        L.k2h_hash.restype, L.k2h_hash.argtypes = _u64, [_p, _sz]
        L.k2h_second_hash.restype, L.k2h_second_hash.argtypes = _u64, [_p, _sz]
        L.k2h_hash_version.restype, L.k2h_hash_version.argtypes = ctypes.c_char_p, []
        self.L = L

    def k2h_hash(self, data: bytes) -> int:
        return int(self.L.k2h_hash(data, len(data)))

    def k2h_second_hash(self, data: bytes) -> int:
        return int(self.L.k2h_second_hash(data, len(data)))

    def version(self) -> str:
        return self.L.k2h_hash_version().decode()


def cpubench():
    """The CPU-baseline harness (cpu_bench.c)."""
    if not CPUBENCH_SO.exists():
        build()
    L = ctypes.CDLL(str(CPUBENCH_SO))
    if not hasattr(L, "cpu_bench_csr"):  # built before the CSR harness existed
        build()
        L = ctypes.CDLL(str(CPUBENCH_SO))
    L.cpu_bench_fixed.restype = ctypes.c_double
    L.cpu_bench_fixed.argtypes = [ctypes.c_char_p, _p, _u64, _u64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(_u64)]
    L.cpu_bench_csr.restype = ctypes.c_double
    L.cpu_bench_csr.argtypes = [ctypes.c_char_p, _p, _p, _u64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(_u64)]
    L.cpu_bench_k2hbench.restype = ctypes.c_double
    L.cpu_bench_k2hbench.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(_u64)]
    return L


def bucket_index_table(h, cur_mask: int, collision_mask: int, assigned):
    """GetKIndex(hash, false) over a table snapshot (oracle_bucket_index_table): returns
    (kindex, ckindex, found) numpy arrays; `assigned` is the uint32 bitmap of K_INDEX
    entries (fnv_oracle.c)."""
    h = np.ascontiguousarray(h, dtype=np.uint64)
    assigned = np.ascontiguousarray(assigned, dtype=np.uint32)
    n = h.size
    k = np.empty(n, np.uint64)
    c = np.empty(n, np.uint64)
    f = np.empty(n, np.uint8)
    L = lib()
    L.oracle_bucket_index_table.restype = None
    L.oracle_bucket_index_table.argtypes = [_p, _sz, _u64, _u64, _p, _p, _p, _p]
    L.oracle_bucket_index_table(_ptr(h), n, cur_mask, collision_mask, _ptr(assigned), _ptr(k), _ptr(c), _ptr(f))
    return k, c, f


def kindex_pos(h: int, cur_mask: int, collision_mask: int) -> tuple[int, int, int]:
    """(KIPtrArrayPos, KIArrayPos, ckindex) of one hash (lib/k2hshm.cc:810-833, 1093)."""
    p, a, c = _u64(), _u64(), _u64()
    lib().oracle_kindex_pos(h, cur_mask, collision_mask, ctypes.byref(p), ctypes.byref(a), ctypes.byref(c))
    return p.value, a.value, c.value


def bucket_index(h: np.ndarray, cur_mask: int, collision_mask: int):
    h = np.ascontiguousarray(h).view(np.uint64)
    k = np.empty(h.size, np.uint64)
    c = np.empty(h.size, np.uint64)
    lib().oracle_bucket_index(_ptr(h), h.size, cur_mask, collision_mask, _ptr(k), _ptr(c))
    return k, c


def _csr_of(parts):
    data = np.frombuffer(b"".join(parts), np.uint8) if any(parts) else np.zeros(1, np.uint8)
    off = np.zeros(len(parts) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in parts])
    return np.ascontiguousarray(data), off


def build_ralledata(keys, vals=None, skeys=None, attrs=None, variant: int = 0):
    """RALLEDATA blobs for records given as lists of bytes (None = segment empty for all).
    Returns (blob bytes as uint8 array, blob offsets n+1)."""
    n = len(keys)
    segs = [_csr_of(keys)] + [(_csr_of(x) if x is not None else (np.zeros(1, np.uint8), None))
                             for x in (vals, skeys, attrs)]
    total = 80 * n + sum(int(o[-1]) for _, o in segs if o is not None)
    out = np.zeros(max(total, 1), np.uint8)
    boff = np.zeros(n + 1, np.uint64)
    args = []
    for d, o in segs:
        args += [_ptr(d), _ptr(o) if o is not None else None]
    lib().oracle_build_ralledata(*args, n, _ptr(out), _ptr(boff), variant)
    return out[:total], boff
