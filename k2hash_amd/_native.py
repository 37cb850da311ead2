"""ctypes binding of the k2hash_amd C ABI (include/k2hash_amd.h).

The native libraries are built in-tree by ``k2hash_amd/csrc/Makefile`` into
``k2hash_amd/lib/``.  There is no Python fallback for the hash path: if the
library is missing this module raises, loudly, on first use.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_DIR = Path(__file__).resolve().parent / "lib"
BATCH_LIB = LIB_DIR / "libk2hash_amd.so"
PLUGIN_LIB = LIB_DIR / "libk2hfnv_plugin.so"

K2H_AMD_OK = 0
K2H_AMD_EINVAL = -1
K2H_AMD_EHIP = -2
K2H_AMD_ENOMEM = -3
K2H_AMD_ENODEV = -4
K2H_AMD_FLAG_STD_FNV = 0x1
K2H_AMD_FLAG_CSTR = 0x2
K2H_AMD_IMPORT_TSV, K2H_AMD_IMPORT_MDBM = 0, 1

_u64 = ctypes.c_uint64
_p = ctypes.c_void_p


class Table(ctypes.Structure):
    """k2h_amd_table (include/k2hash_amd.h section 3)."""
    _fields_ = [("cur_mask", ctypes.c_uint64), ("collision_mask", ctypes.c_uint64), ("assigned", ctypes.c_void_p)]


_tp = ctypes.POINTER(Table)

# name -> (restype, argtypes); mirrors include/k2hash_amd.h
SIGNATURES = {
    "k2h_hash": (_u64, [_p, ctypes.c_size_t]),
    "k2h_second_hash": (_u64, [_p, ctypes.c_size_t]),
    "k2h_hash_version": (ctypes.c_char_p, []),
    "k2h_amd_hash_fixed": (ctypes.c_int, [_p, _u64, _u64, _p, _p, ctypes.c_uint32, _p]),
    "k2h_amd_hash_csr": (ctypes.c_int, [_p, _p, _u64, _p, _p, ctypes.c_uint32, _p]),
    "k2h_amd_hash_fixed_host": (ctypes.c_int, [_p, _u64, _u64, _p, _p, ctypes.c_uint32, ctypes.c_int]),
    "k2h_amd_hash_csr_host": (ctypes.c_int, [_p, _p, _u64, _p, _p, ctypes.c_uint32, ctypes.c_int]),
    "k2h_amd_bucket_index": (ctypes.c_int, [_p, _u64, _u64, _u64, _p, _p, _p]),
    "k2h_amd_hash_fixed_index": (ctypes.c_int, [_p, _u64, _u64, _p, _p, ctypes.c_uint32, _u64, _u64, _p, _p, _p]),
    "k2h_amd_hash_csr_index": (ctypes.c_int, [_p, _p, _u64, _p, _p, ctypes.c_uint32, _u64, _u64, _p, _p, _p]),
    "k2h_amd_bucket_index_table": (ctypes.c_int, [_p, _u64, _tp, _p, _p, _p, _p]),
    "k2h_amd_hash_fixed_index_table": (ctypes.c_int, [_p, _u64, _u64, _p, _p, ctypes.c_uint32, _tp, _p, _p, _p, _p]),
    "k2h_amd_hash_csr_index_table": (ctypes.c_int, [_p, _p, _u64, _p, _p, ctypes.c_uint32, _tp, _p, _p, _p, _p]),
    "k2h_amd_ralledata_size": (_u64, [_u64, _u64, _u64, _u64, _u64]),
    "k2h_amd_build_ralledata": (ctypes.c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _u64, _p, _p, ctypes.c_uint32, _p]),
    "k2h_amd_build_ralledata_host": (ctypes.c_int,
                                     [_p, _p, _p, _p, _p, _p, _p, _p, _u64, _p, _p, ctypes.c_uint32, ctypes.c_int]),
    "k2h_amd_hash_ranges": (ctypes.c_int, [_p, _p, _p, _u64, _p, _p, ctypes.c_uint32, _p]),
    "k2h_amd_archive_scan": (ctypes.c_int, [_p, _u64, _p, _u64, _p]),
    "k2h_amd_archive_prehash_host": (ctypes.c_int, [_p, _u64, _p, _u64, _p, _p, _p, _p, ctypes.c_uint32, ctypes.c_int]),
    "k2h_amd_import_scan": (ctypes.c_int, [_p, _u64, ctypes.c_int, _p, _u64, _p]),
    "k2h_amd_import_prehash_host": (ctypes.c_int, [_p, _u64, _p, _u64, _p, _p, ctypes.c_uint32, ctypes.c_int]),
    "k2h_amd_import_scan_device": (ctypes.c_int, [_p, _u64, ctypes.c_int, _p, _u64, _p, _p]),
    "k2h_amd_import_prehash": (ctypes.c_int, [_p, _u64, _p, _u64, _p, _p, ctypes.c_uint32, _p]),
    "k2h_amd_import_scan_prehash_device": (ctypes.c_int, [_p, _u64, ctypes.c_int, _p, _u64, _p, _p, _p,
                                                          ctypes.c_uint32, _p]),
    "k2h_amd_version": (ctypes.c_char_p, []),
    "k2h_amd_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "k2h_amd_synth_bytes": (ctypes.c_int, [_p, _u64, _u64, _u64, _p]),
    "k2h_amd_synth_lengths": (ctypes.c_int, [_p, _u64, _u64, _u64, ctypes.c_uint32, ctypes.c_uint32, _p]),
}

PLUGIN_SYMBOLS = ("k2h_hash", "k2h_second_hash", "k2h_hash_version")

_batch = None


class NativeError(RuntimeError):
    """A k2hash_amd C-ABI call returned a negative K2H_AMD_E* code."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"k2hash_amd error {code}: {msg}")
        self.code = code


def _bind(lib: ctypes.CDLL, names) -> ctypes.CDLL:
    for name in names:
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = SIGNATURES[name]
    return lib


def batch_lib() -> ctypes.CDLL:
    """The batch library (HIP kernels + plugin symbols).  Raises if not built."""
    global _batch
    if _batch is None:
        # One HIP runtime per process: torch ships its own libamdhip64 (soname
        # libamdhip64.so.7, like /opt/rocm's).  Loading torch first lets this library's
        # libamdhip64.so.7 dependency bind to that copy; the other order leaves two
        # runtimes in the process and torch then sees no GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = BATCH_LIB
        if not path.exists():
            raise RuntimeError(
                f"k2hash_amd native library missing: {path} "
                "(build it with `make -C k2hash_amd/csrc` or __graft_entry__.build())")
        _batch = _bind(ctypes.CDLL(str(path)), SIGNATURES.keys())
    return _batch


def plugin_lib(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """A library exposing only the three plugin symbols (default: libk2hfnv_plugin.so)."""
    p = Path(path) if path else PLUGIN_LIB
    if not p.exists():
        raise RuntimeError(f"k2hash_amd plugin library missing: {p}")
    return _bind(ctypes.CDLL(str(p)), PLUGIN_SYMBOLS)


def check(rc: int) -> None:
    if rc != K2H_AMD_OK:
        msg = batch_lib().k2h_amd_strerror(rc).decode(errors="replace")
        raise NativeError(rc, msg)
