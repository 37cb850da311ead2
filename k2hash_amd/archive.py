"""Bulk key streams: keys at arbitrary ranges of a buffer, and
k2hash archive files (include/k2hash_amd.h section 5).

An archive is what K2HArchive::Save writes and K2HArchive::Load replays record by
record, hashing each key on the CPU inside ReplaceAll / Remove / Rename
(lib/k2harchive.cc:82-383).  scan() walks the records the way Load does; prehash()
hashes every key of the file in one GPU batch.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from .batch import FLAG_STD_FNV, _check_dev, _dev_ptr, _stream_handle, _torch

FLAG_CSTR = _native.K2H_AMD_FLAG_CSTR
SCOM_SET_ALL, SCOM_REPLACE_VAL, SCOM_REPLACE_SKEY, SCOM_DEL_KEY, SCOM_OW_VAL, SCOM_REPLACE_ATTRS, SCOM_RENAME = range(7)
STATUS_OK, STATUS_BAD_TYPE, STATUS_TRUNCATED = 0, 1, 2

# struct k2h_amd_archive_rec (include/k2hash_amd.h)
REC_DTYPE = np.dtype([("type", "<i8"), ("offset", "<u8"), ("key_off", "<u8"), ("key_len", "<u8"),
                      ("val_off", "<u8"), ("val_len", "<u8"), ("skey_off", "<u8"), ("skey_len", "<u8"),
                      ("attrs_off", "<u8"), ("attrs_len", "<u8"), ("exdata_off", "<u8"), ("exdata_len", "<u8"),
                      ("status", "<i4"), ("reserved", "<i4")])


def _buf(data) -> np.ndarray:
    return np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else \
        np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)


def scan(data) -> np.ndarray:
    """Records of an archive (structured array, REC_DTYPE), in file order."""
    f = _buf(data)
    ptr = ctypes.c_void_p(f.ctypes.data if f.size else 1)
    lib = _native.batch_lib()
    cnt = ctypes.c_uint64()
    _native.check(lib.k2h_amd_archive_scan(ptr, f.size, None, 0, ctypes.byref(cnt)))
    recs = np.zeros(cnt.value, REC_DTYPE)
    _native.check(lib.k2h_amd_archive_scan(ptr, f.size, ctypes.c_void_p(recs.ctypes.data if recs.size else 1),
                                           recs.size, ctypes.byref(cnt)))
    return recs


def prehash(data, recs=None, rename: bool = False, std_fnv: bool = False, device: int = 0):
    """(h1, h2[, new_h1, new_h2]) of every record's key (uint64 arrays, 0 for records whose
    status is not STATUS_OK); with rename=True also the new key of SCOM_RENAME records."""
    f = _buf(data)
    if recs is None:
        recs = scan(f)
    n = recs.size
    h1, h2 = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    nh1, nh2 = (np.zeros(n, np.uint64), np.zeros(n, np.uint64)) if rename else (None, None)
    p = lambda a: ctypes.c_void_p(a.ctypes.data) if a is not None else None  # noqa: E731
    if n:
        _native.check(_native.batch_lib().k2h_amd_archive_prehash_host(
            ctypes.c_void_p(f.ctypes.data if f.size else 1), f.size, p(recs), n, p(h1), p(h2), p(nh1), p(nh2),
            FLAG_STD_FNV if std_fnv else 0, device))
    return (h1, h2, nh1, nh2) if rename else (h1, h2)


def hash_ranges(base, starts, lens, second: bool = False, cstr: bool = False, std_fnv: bool = False, stream=None):
    """Device form: key i = base[starts[i] : starts[i] + lens[i]] (uint8 / int64 / int64
    device tensors).  cstr=True hashes key + NUL (K2HShm::Set(const char*))."""
    torch = _torch()
    _check_dev(base, "base", torch.uint8)
    _check_dev(starts, "starts", torch.int64)
    _check_dev(lens, "lens", torch.int64)
    n = starts.numel()
    h1 = torch.empty(n, dtype=torch.int64, device=base.device)
    h2 = torch.empty(n, dtype=torch.int64, device=base.device) if second else None
    flags = (FLAG_CSTR if cstr else 0) | (FLAG_STD_FNV if std_fnv else 0)
    rc = _native.batch_lib().k2h_amd_hash_ranges(ctypes.c_void_p(base.data_ptr() or 1), _dev_ptr(starts),
                                                 _dev_ptr(lens), n, _dev_ptr(h1),
                                                 _dev_ptr(h2) if h2 is not None else None, flags,
                                                 _stream_handle(stream))
    _native.check(rc)
    return h1, h2


# ---------------------------------------------------------------------------
# k2himport inputs (tests/k2himport.cc:74-117): TSV and mdbm_export files.
# ---------------------------------------------------------------------------
IMPORT_TSV, IMPORT_MDBM = _native.K2H_AMD_IMPORT_TSV, _native.K2H_AMD_IMPORT_MDBM
# struct k2h_amd_import_rec (include/k2hash_amd.h)
IMPORT_DTYPE = np.dtype([("key_off", "<u8"), ("key_len", "<u8"), ("val_off", "<u8"), ("val_len", "<u8")])


def import_scan(data, fmt: str = "tsv") -> np.ndarray:
    """Records of a k2himport input, split exactly as the tool's getline loops do, each key
    and value as the C string K2HShm::Set(const char*, const char*) stores (lengths are
    strlen).  fmt: "tsv" or "mdbm"; a bad mdbm header raises (the tool exits)."""
    f = _buf(data)
    code = {"tsv": IMPORT_TSV, "mdbm": IMPORT_MDBM}[fmt]
    ptr = ctypes.c_void_p(f.ctypes.data if f.size else 1)
    lib = _native.batch_lib()
    cnt = ctypes.c_uint64()
    _native.check(lib.k2h_amd_import_scan(ptr, f.size, code, None, 0, ctypes.byref(cnt)))
    recs = np.zeros(cnt.value, IMPORT_DTYPE)
    _native.check(lib.k2h_amd_import_scan(ptr, f.size, code, ctypes.c_void_p(recs.ctypes.data if recs.size else 1),
                                          recs.size, ctypes.byref(cnt)))
    return recs


def import_prehash(data, recs=None, fmt: str = "tsv", std_fnv: bool = False, device: int = 0):
    """(h1, h2) of every record's key hashed as key + NUL on the GPU -- the bytes
    K2HShm::Set(const char*) hashes (lib/k2hshm.cc:2081-2083)."""
    f = _buf(data)
    if recs is None:
        recs = import_scan(f, fmt)
    n = recs.size
    h1, h2 = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    if n:
        _native.check(_native.batch_lib().k2h_amd_import_prehash_host(
            ctypes.c_void_p(f.ctypes.data if f.size else 1), f.size, ctypes.c_void_p(recs.ctypes.data), n,
            ctypes.c_void_p(h1.ctypes.data), ctypes.c_void_p(h2.ctypes.data), FLAG_STD_FNV if std_fnv else 0,
            device))
    return h1, h2


def import_scan_device(file, fmt: str = "tsv", stream=None):
    """import_scan for a file already in device memory (uint8 device tensor), with no
    host pass (k2h_amd_import_scan_device).  Returns an (n, 4) int64 device tensor of
    (key_off, key_len, val_off, val_len) rows -- struct k2h_amd_import_rec."""
    torch = _torch()
    _check_dev(file, "file", torch.uint8)
    code = {"tsv": IMPORT_TSV, "mdbm": IMPORT_MDBM}[fmt]
    lib = _native.batch_lib()
    fp = ctypes.c_void_p(file.data_ptr() or 1)
    cnt = ctypes.c_uint64()
    # one pass when the guess holds (records of >= 64 bytes on average); otherwise the
    # call reports the count with K2H_AMD_EINVAL and a second pass fills exact storage
    cap = max(1024, file.numel() // 64)
    recs = torch.empty((cap, 4), dtype=torch.int64, device=file.device)
    rc = lib.k2h_amd_import_scan_device(fp, file.numel(), code, _dev_ptr(recs), cap, ctypes.byref(cnt),
                                        _stream_handle(stream))
    if rc == _native.K2H_AMD_EINVAL and cnt.value > cap:
        recs = torch.empty((cnt.value, 4), dtype=torch.int64, device=file.device)
        rc = lib.k2h_amd_import_scan_device(fp, file.numel(), code, _dev_ptr(recs), cnt.value, ctypes.byref(cnt),
                                            _stream_handle(stream))
    _native.check(rc)
    return recs[: cnt.value]


def import_prehash_device(file, recs, std_fnv: bool = False, stream=None):
    """(h1, h2) device tensors of every record's key hashed as key + NUL, from the
    device-resident file and the records of import_scan_device."""
    torch = _torch()
    _check_dev(file, "file", torch.uint8)
    _check_dev(recs, "recs", torch.int64)
    if recs.dim() != 2 or recs.shape[1] != 4 or not recs.is_contiguous():
        raise ValueError("recs must be a contiguous (n, 4) int64 tensor")
    n = recs.shape[0]
    h1 = torch.empty(n, dtype=torch.int64, device=file.device)
    h2 = torch.empty(n, dtype=torch.int64, device=file.device)
    _native.check(_native.batch_lib().k2h_amd_import_prehash(
        ctypes.c_void_p(file.data_ptr() or 1), file.numel(), _dev_ptr(recs), n, _dev_ptr(h1), _dev_ptr(h2),
        FLAG_STD_FNV if std_fnv else 0, _stream_handle(stream)))
    return h1, h2


def import_scan_prehash_device(file, fmt: str = "tsv", std_fnv: bool = False, stream=None):
    """import_scan_device + import_prehash_device in one call: the records and their keys'
    (h1, h2) from the same kernel (k2h_amd_import_scan_prehash_device)."""
    torch = _torch()
    _check_dev(file, "file", torch.uint8)
    code = {"tsv": IMPORT_TSV, "mdbm": IMPORT_MDBM}[fmt]
    lib = _native.batch_lib()
    fp = ctypes.c_void_p(file.data_ptr() or 1)
    flags = FLAG_STD_FNV if std_fnv else 0
    cnt = ctypes.c_uint64()
    rc = 0
    cap = max(1024, file.numel() // 64)  # as import_scan_device: one pass when the guess holds
    for _ in range(2):
        recs = torch.empty((cap, 4), dtype=torch.int64, device=file.device)
        h1 = torch.empty(cap, dtype=torch.int64, device=file.device)
        h2 = torch.empty(cap, dtype=torch.int64, device=file.device)
        rc = lib.k2h_amd_import_scan_prehash_device(fp, file.numel(), code, _dev_ptr(recs), cap, ctypes.byref(cnt),
                                                    _dev_ptr(h1), _dev_ptr(h2), flags, _stream_handle(stream))
        if not (rc == _native.K2H_AMD_EINVAL and cnt.value > cap):
            break
        cap = cnt.value
    _native.check(rc)
    n = cnt.value
    return recs[:n], h1[:n], h2[:n]
