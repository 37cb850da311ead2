"""Batch key hashing on MI355X through the k2hash_amd C ABI.

Device forms take torch tensors already resident in HBM and launch on the
current torch stream; host forms take numpy arrays and use the library's
pinned-staging pipeline.  Hashes are returned as int64 tensors/arrays holding
the 64-bit k2h_hash_t bit patterns (view as uint64 with numpy for printing).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _native

FLAG_STD_FNV = _native.K2H_AMD_FLAG_STD_FNV


def _torch():
    import torch  # deferred: host-only users need not import torch

    return torch


def _stream_handle(stream=None) -> ctypes.c_void_p:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _dev_ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def _check_dev(t, name: str, dtype) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _check_out(t, name: str, n: int, device, torch) -> None:
    """A caller-supplied output tensor the kernel will write n 8-byte values into: int64,
    contiguous, on the keys' device, exactly n entries (an undersized or
    wrong-device tensor would otherwise be written past its end by the GPU)."""
    _check_dev(t, name, torch.int64)
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, the keys on {device}")
    if t.numel() != n:
        raise ValueError(f"{name} must have exactly {n} entries, got {t.numel()}")


def _unpack_out(out, n: int, device, torch, second: bool, want: Tuple[str, ...]):
    """Validate a caller's `out` tuple: h2 present iff `second`; the other named slots may be
    None (that output is then not written)."""
    if len(out) != len(want):
        raise ValueError(f"out must be a tuple of {len(want)} tensors ({', '.join(want)})")
    if out[0] is None:
        raise ValueError("out: h1 is required")
    if (out[1] is not None) != bool(second):
        raise ValueError("out: pass an h2 tensor exactly when second=True")
    for t, name in zip(out, want):
        if t is not None:
            _check_out(t, f"out {name}", n, device, torch)
    return out


def hash_fixed(keys, key_len: int, second: bool = False, std_fnv: bool = False,
               out: Optional[Tuple] = None, stream=None):
    """Hash n = keys.numel() // key_len fixed-length keys held in a uint8 device tensor.

    Returns (h1, h2) int64 device tensors (h2 None unless second=True).
    """
    torch = _torch()
    _check_dev(keys, "keys", torch.uint8)
    if key_len <= 0:
        raise ValueError("key_len must be positive")
    n = keys.numel() // key_len
    if out is not None:
        h1, h2 = _unpack_out(out, n, keys.device, torch, second, ("h1", "h2"))
    else:
        h1 = torch.empty(n, dtype=torch.int64, device=keys.device)
        h2 = torch.empty(n, dtype=torch.int64, device=keys.device) if second else None
    flags = FLAG_STD_FNV if std_fnv else 0
    rc = _native.batch_lib().k2h_amd_hash_fixed(
        _dev_ptr(keys), key_len, n, _dev_ptr(h1), _dev_ptr(h2) if h2 is not None else None, flags,
        _stream_handle(stream))
    _native.check(rc)
    return h1, h2


def hash_csr(data, offsets, second: bool = False, std_fnv: bool = False, out: Optional[Tuple] = None,
             stream=None):
    """Hash CSR keys: key i = data[offsets[i]:offsets[i+1]] (uint8 / int64 device tensors)."""
    torch = _torch()
    _check_dev(data, "data", torch.uint8)
    _check_dev(offsets, "offsets", torch.int64)
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets must have n+1 entries")
    if offsets.device != data.device:
        raise ValueError("data and offsets must be on one device")
    if out is not None:
        h1, h2 = _unpack_out(out, n, data.device, torch, second, ("h1", "h2"))
    else:
        h1 = torch.empty(n, dtype=torch.int64, device=data.device)
        h2 = torch.empty(n, dtype=torch.int64, device=data.device) if second else None
    flags = FLAG_STD_FNV if std_fnv else 0
    base = _dev_ptr(data) if data.numel() > 0 else ctypes.c_void_p(data.data_ptr() or 1)
    rc = _native.batch_lib().k2h_amd_hash_csr(
        base, _dev_ptr(offsets), n, _dev_ptr(h1), _dev_ptr(h2) if h2 is not None else None, flags,
        _stream_handle(stream))
    _native.check(rc)
    return h1, h2


# ----------------------------------------------------------------------------
# Bucket-index epilogue (include/k2hash_amd.h section 3; lib/k2hshm.cc:78-90,
# 810-833, 1093): where each hash lands in a k2hash table with masks
# (cur_mask, collision_mask).  kindex packs KIPtrArrayPos << 58 | KIArrayPos.
# ----------------------------------------------------------------------------
KINDEX_POS_SHIFT = 58


def unpack_kindex(kindex):
    """(KIPtrArrayPos, KIArrayPos) from packed kindex values (numpy uint64 or torch int64)."""
    if isinstance(kindex, np.ndarray):
        v = kindex.view(np.uint64)
        return v >> np.uint64(KINDEX_POS_SHIFT), v & np.uint64((1 << KINDEX_POS_SHIFT) - 1)
    pos = (kindex >> KINDEX_POS_SHIFT) & 0x3F
    return pos, kindex & ((1 << KINDEX_POS_SHIFT) - 1)


def _index_outs(torch, n, device, kindex, ckindex, out):
    if out is not None:
        if len(out) != 2:
            raise ValueError("out must be (kindex, ckindex)")
        for t, name in zip(out, ("kindex", "ckindex")):
            if t is not None:
                _check_out(t, f"out {name}", n, device, torch)
        return out
    k = torch.empty(n, dtype=torch.int64, device=device) if kindex else None
    c = torch.empty(n, dtype=torch.int64, device=device) if ckindex else None
    return k, c


def bucket_index(h1, cur_mask: int, collision_mask: int, kindex: bool = True, ckindex: bool = True,
                 out=None, stream=None):
    """Bucket positions of hashes already in device memory (int64 tensor)."""
    torch = _torch()
    _check_dev(h1, "h1", torch.int64)
    n = h1.numel()
    k, c = _index_outs(torch, n, h1.device, kindex, ckindex, out)
    rc = _native.batch_lib().k2h_amd_bucket_index(
        _dev_ptr(h1), n, cur_mask, collision_mask, _dev_ptr(k) if k is not None else None,
        _dev_ptr(c) if c is not None else None, _stream_handle(stream))
    _native.check(rc)
    return k, c


def hash_fixed_index(keys, key_len: int, cur_mask: int, collision_mask: int, second: bool = False,
                     std_fnv: bool = False, kindex: bool = True, ckindex: bool = True, stream=None, out=None):
    """hash_fixed + bucket index in one pass: returns (h1, h2, kindex, ckindex).  `out`:
    preallocated (h1, h2, kindex, ckindex) tensors (h2 / kindex / ckindex may be None)."""
    torch = _torch()
    _check_dev(keys, "keys", torch.uint8)
    if key_len <= 0:
        raise ValueError("key_len must be positive")
    n = keys.numel() // key_len
    if out is not None:
        h1, h2, k, c = _unpack_out(out, n, keys.device, torch, second, ("h1", "h2", "kindex", "ckindex"))
    else:
        h1 = torch.empty(n, dtype=torch.int64, device=keys.device)
        h2 = torch.empty(n, dtype=torch.int64, device=keys.device) if second else None
        k, c = _index_outs(torch, n, keys.device, kindex, ckindex, None)
    rc = _native.batch_lib().k2h_amd_hash_fixed_index(
        _dev_ptr(keys), key_len, n, _dev_ptr(h1), _dev_ptr(h2) if h2 is not None else None,
        FLAG_STD_FNV if std_fnv else 0, cur_mask, collision_mask, _dev_ptr(k) if k is not None else None,
        _dev_ptr(c) if c is not None else None, _stream_handle(stream))
    _native.check(rc)
    return h1, h2, k, c


def hash_csr_index(data, offsets, cur_mask: int, collision_mask: int, second: bool = False,
                   std_fnv: bool = False, kindex: bool = True, ckindex: bool = True, stream=None, out=None):
    """hash_csr + bucket index in one pass: returns (h1, h2, kindex, ckindex)."""
    torch = _torch()
    _check_dev(data, "data", torch.uint8)
    _check_dev(offsets, "offsets", torch.int64)
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets must have n+1 entries")
    if offsets.device != data.device:
        raise ValueError("data and offsets must be on one device")
    if out is not None:
        h1, h2, k, c = _unpack_out(out, n, data.device, torch, second, ("h1", "h2", "kindex", "ckindex"))
    else:
        h1 = torch.empty(n, dtype=torch.int64, device=data.device)
        h2 = torch.empty(n, dtype=torch.int64, device=data.device) if second else None
        k, c = _index_outs(torch, n, data.device, kindex, ckindex, None)
    base = _dev_ptr(data) if data.numel() > 0 else ctypes.c_void_p(data.data_ptr() or 1)
    rc = _native.batch_lib().k2h_amd_hash_csr_index(
        base, _dev_ptr(offsets), n, _dev_ptr(h1), _dev_ptr(h2) if h2 is not None else None,
        FLAG_STD_FNV if std_fnv else 0, cur_mask, collision_mask, _dev_ptr(k) if k is not None else None,
        _dev_ptr(c) if c is not None else None, _stream_handle(stream))
    _native.check(rc)
    return h1, h2, k, c


# ----------------------------------------------------------------------------
# Table-state bucket index (include/k2hash_amd.h section 3, *_table forms): the K_INDEX
# K2HShm::GetKIndex(hash, false) reaches (lib/k2hshm.cc:862-907) for a snapshot of the
# table's assigned flags.  `assigned`: int32 device tensor, the bitmap of assigned
# K_INDEX entries (bit p ? 2^(p-1) + a : 0 for entry a of key_index_area[p]), or None
# (every entry assigned).  Returns (kindex, ckindex, found) -- found is uint8.
# ----------------------------------------------------------------------------
KINDEX_NONE = (1 << 64) - 1


def _table(torch, cur_mask: int, collision_mask: int, assigned, device):
    if assigned is not None:
        _check_dev(assigned, "assigned", torch.int32)
        if assigned.device != device:
            raise ValueError("assigned must be on the hashes' device")
        need = (cur_mask + 1 + 31) // 32
        if assigned.numel() < need:
            raise ValueError(f"assigned must hold cur_mask + 1 bits ({need} int32 words), got {assigned.numel()}")
    return _native.Table(cur_mask, collision_mask, assigned.data_ptr() if assigned is not None else None)


def _table_outs(torch, n, device, kindex, ckindex, found, out):
    if out is not None:
        if len(out) != 3:
            raise ValueError("out must be (kindex, ckindex, found)")
        for t, name, dt in zip(out, ("kindex", "ckindex", "found"), (torch.int64, torch.int64, torch.uint8)):
            if t is not None:
                _check_dev(t, f"out {name}", dt)
                if t.device != device or t.numel() != n:
                    raise ValueError(f"out {name} must have {n} entries on {device}")
        return out
    return (torch.empty(n, dtype=torch.int64, device=device) if kindex else None,
            torch.empty(n, dtype=torch.int64, device=device) if ckindex else None,
            torch.empty(n, dtype=torch.uint8, device=device) if found else None)


def _ptr_or_none(t):
    return _dev_ptr(t) if t is not None else None


def bucket_index_table(h1, cur_mask: int, collision_mask: int, assigned=None, kindex: bool = True,
                       ckindex: bool = True, found: bool = True, out=None, stream=None):
    """GetKIndex positions of hashes already in device memory, over a table snapshot."""
    torch = _torch()
    _check_dev(h1, "h1", torch.int64)
    n = h1.numel()
    tab = _table(torch, cur_mask, collision_mask, assigned, h1.device)
    k, c, f = _table_outs(torch, n, h1.device, kindex, ckindex, found, out)
    rc = _native.batch_lib().k2h_amd_bucket_index_table(_dev_ptr(h1), n, ctypes.byref(tab), _ptr_or_none(k),
                                                         _ptr_or_none(c), _ptr_or_none(f), _stream_handle(stream))
    _native.check(rc)
    return k, c, f


def hash_fixed_index_table(keys, key_len: int, cur_mask: int, collision_mask: int, assigned=None,
                           second: bool = False, std_fnv: bool = False, stream=None):
    """hash_fixed + the table-state bucket index in one pass: (h1, h2, kindex, ckindex, found)."""
    torch = _torch()
    _check_dev(keys, "keys", torch.uint8)
    if key_len <= 0:
        raise ValueError("key_len must be positive")
    n = keys.numel() // key_len
    tab = _table(torch, cur_mask, collision_mask, assigned, keys.device)
    h1 = torch.empty(n, dtype=torch.int64, device=keys.device)
    h2 = torch.empty(n, dtype=torch.int64, device=keys.device) if second else None
    k, c, f = _table_outs(torch, n, keys.device, True, True, True, None)
    rc = _native.batch_lib().k2h_amd_hash_fixed_index_table(
        _dev_ptr(keys), key_len, n, _dev_ptr(h1), _ptr_or_none(h2), FLAG_STD_FNV if std_fnv else 0,
        ctypes.byref(tab), _dev_ptr(k), _dev_ptr(c), _dev_ptr(f), _stream_handle(stream))
    _native.check(rc)
    return h1, h2, k, c, f


def hash_csr_index_table(data, offsets, cur_mask: int, collision_mask: int, assigned=None, second: bool = False,
                         std_fnv: bool = False, stream=None):
    """hash_csr + the table-state bucket index in one pass: (h1, h2, kindex, ckindex, found)."""
    torch = _torch()
    _check_dev(data, "data", torch.uint8)
    _check_dev(offsets, "offsets", torch.int64)
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets must have n+1 entries")
    if offsets.device != data.device:
        raise ValueError("data and offsets must be on one device")
    tab = _table(torch, cur_mask, collision_mask, assigned, data.device)
    h1 = torch.empty(n, dtype=torch.int64, device=data.device)
    h2 = torch.empty(n, dtype=torch.int64, device=data.device) if second else None
    k, c, f = _table_outs(torch, n, data.device, True, True, True, None)
    base = _dev_ptr(data) if data.numel() > 0 else ctypes.c_void_p(data.data_ptr() or 1)
    rc = _native.batch_lib().k2h_amd_hash_csr_index_table(
        base, _dev_ptr(offsets), n, _dev_ptr(h1), _ptr_or_none(h2), FLAG_STD_FNV if std_fnv else 0,
        ctypes.byref(tab), _dev_ptr(k), _dev_ptr(c), _dev_ptr(f), _stream_handle(stream))
    _native.check(rc)
    return h1, h2, k, c, f


def expanded_table_bitmap(cur_mask: int, frac_top: float, seed: int = 0):
    """Assigned-entry bitmap (numpy uint32) of a table just expanded to `cur_mask`: every
    entry below the top area assigned, a fraction `frac_top` of the top area's entries
    (those ArrangeToUpperKIndex has already split) assigned.  Test / bench helper."""
    bits = cur_mask + 1
    flags = np.ones(bits, dtype=bool)
    top = (cur_mask + 1) // 2
    if cur_mask:
        rng = np.random.default_rng(seed)
        flags[top:] = rng.random(bits - top) < frac_top
    words = np.zeros((bits + 31) // 32 * 32, dtype=bool)
    words[:bits] = flags
    return np.packbits(words.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").astype(np.uint32).reshape(-1)


def _np_ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _host_outs(n, second, out):
    if out is not None:
        h1, h2 = out
        if h1.dtype != np.uint64 or h1.size != n or not h1.flags.c_contiguous or \
                (second and (h2 is None or h2.dtype != np.uint64 or h2.size != n or not h2.flags.c_contiguous)):
            raise ValueError("out must be contiguous uint64 arrays of n entries")
        return h1, (h2 if second else None)
    return np.empty(n, dtype=np.uint64), (np.empty(n, dtype=np.uint64) if second else None)


def hash_fixed_host(keys: np.ndarray, key_len: int, second: bool = False, std_fnv: bool = False,
                    device: int = 0, out=None):
    """Host-memory form of hash_fixed (numpy uint8 in, numpy uint64 out; `out`: reuse
    (h1, h2) arrays)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1)
    n = keys.size // key_len
    h1, h2 = _host_outs(n, second, out)
    rc = _native.batch_lib().k2h_amd_hash_fixed_host(
        _np_ptr(keys), key_len, n, _np_ptr(h1), _np_ptr(h2) if h2 is not None else None,
        FLAG_STD_FNV if std_fnv else 0, device)
    _native.check(rc)
    return h1, h2


def hash_csr_host(data: np.ndarray, offsets: np.ndarray, second: bool = False, std_fnv: bool = False,
                  device: int = 0, out=None):
    """Host-memory form of hash_csr."""
    data = np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64).reshape(-1)
    n = offsets.size - 1
    h1, h2 = _host_outs(n, second, out)
    dptr = _np_ptr(data) if data.size else ctypes.c_void_p(1)
    rc = _native.batch_lib().k2h_amd_hash_csr_host(
        dptr, _np_ptr(offsets), n, _np_ptr(h1), _np_ptr(h2) if h2 is not None else None,
        FLAG_STD_FNV if std_fnv else 0, device)
    _native.check(rc)
    return h1, h2


# ----------------------------------------------------------------------------
# Synthetic workloads (bench/test harness): splitmix64 counter stream, same spec
# as oracle/fnv_oracle.c.  Generated on the device.
# ----------------------------------------------------------------------------
SEED_BYTES = 0x6B32686173680001
SEED_LENS = 0x6B32686173680002


def synth_bytes(nbytes: int, device, seed: int = SEED_BYTES, byte_off: int = 0, stream=None):
    torch = _torch()
    t = torch.empty(nbytes, dtype=torch.uint8, device=device)
    rc = _native.batch_lib().k2h_amd_synth_bytes(_dev_ptr(t), nbytes, seed, byte_off, _stream_handle(stream))
    _native.check(rc)
    return t


def synth_offsets(n: int, device, min_len: int = 8, max_len: int = 256, seed: int = SEED_LENS,
                  first_key: int = 0, stream=None):
    """CSR offsets (n+1, int64, starting at 0) for keys first_key .. first_key+n-1."""
    torch = _torch()
    lens = torch.empty(n, dtype=torch.int32, device=device)
    rc = _native.batch_lib().k2h_amd_synth_lengths(_dev_ptr(lens), n, seed, first_key, min_len, max_len,
                                                    _stream_handle(stream))
    _native.check(rc)
    off = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, dim=0, dtype=torch.int64, out=off[1:])
    return off


def version() -> str:
    return _native.batch_lib().k2h_amd_version().decode()
