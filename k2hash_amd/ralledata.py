"""RALLEDATA producer: packed direct-set blobs with precomputed
hashes, built on the GPU (include/k2hash_amd.h section 4).

A blob is what K2HShm::GetElementToBinary writes (lib/k2hshmdirect.cc:59-88) on the
packed struct of lib/k2hshmdirect.h:36-47, and what k2h_set_element_by_binary
(lib/k2hash.cc:1562-1581) consumes -- trusting the hash / subhash fields, so a bulk load
fed from these blobs never hashes a key on the CPU.
"""
from __future__ import annotations

import ctypes
import struct
from typing import NamedTuple, Optional, Sequence

import numpy as np

from . import _native
from .batch import FLAG_STD_FNV, _check_dev, _dev_ptr, _stream_handle, _torch

HEADER = 80  # sizeof(RALLEDATA)
_FIELDS = ("hash", "subhash", "key_length", "val_length", "skey_length", "attrs_length", "key_pos", "val_pos",
           "skey_pos", "attrs_pos")


class Blob(NamedTuple):
    hash: int
    subhash: int
    key: bytes
    val: bytes
    skey: bytes
    attrs: bytes


def parse_blob(b: bytes) -> Blob:
    """Decode one RALLEDATA blob (field order of lib/k2hshmdirect.h:36-47)."""
    f = dict(zip(_FIELDS, struct.unpack_from("<10Q", b, 0)))
    seg = lambda p, n: bytes(b[p:p + n])  # noqa: E731
    return Blob(f["hash"], f["subhash"], seg(f["key_pos"], f["key_length"]), seg(f["val_pos"], f["val_length"]),
                seg(f["skey_pos"], f["skey_length"]), seg(f["attrs_pos"], f["attrs_length"]))


def ralledata_size(n: int, key_bytes: int, val_bytes: int = 0, skey_bytes: int = 0, attr_bytes: int = 0) -> int:
    return int(_native.batch_lib().k2h_amd_ralledata_size(n, key_bytes, val_bytes, skey_bytes, attr_bytes))


def _seg_bytes(off) -> int:
    if off is None or off.numel() == 0:
        return 0
    return int(off[-1].item()) - int(off[0].item())


def build_ralledata(keys, key_off, vals=None, val_off=None, skeys=None, skey_off=None, attrs=None, attr_off=None,
                    std_fnv: bool = False, out=None, blob_off=None, stream=None, total: Optional[int] = None):
    """Device form.  Each segment is (uint8 bytes tensor, int64 offsets tensor of n+1) or
    (None, None).  Returns (blobs uint8 tensor, blob_off int64 tensor of n+1).

    The blob size is computed from the first and last offset of every segment, which
    reads them back from the device (a stream sync); a caller that already knows it
    (`ralledata_size`) passes `total` together with `out` and the call stays async."""
    torch = _torch()
    _check_dev(key_off, "key_off", torch.int64)
    n = key_off.numel() - 1
    segs = [(keys, key_off), (vals, val_off), (skeys, skey_off), (attrs, attr_off)]
    args = []
    nbytes = []
    for name, (b, o) in zip(("keys", "vals", "skeys", "attrs"), segs):
        if o is None:
            args += [None, None]
            nbytes.append(0)
            continue
        _check_dev(o, f"{name} offsets", torch.int64)
        _check_dev(b, name, torch.uint8)
        args += [ctypes.c_void_p(b.data_ptr() or 1), _dev_ptr(o)]
        nbytes.append(0 if total is not None and out is not None else _seg_bytes(o))
    if total is None or out is None:
        total = ralledata_size(n, *nbytes)
    elif out.numel() < total:
        raise ValueError("out is smaller than total")
    dev = key_off.device
    if out is None:
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    if blob_off is None:
        blob_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    rc = _native.batch_lib().k2h_amd_build_ralledata(*args, n, _dev_ptr(out), _dev_ptr(blob_off),
                                                     FLAG_STD_FNV if std_fnv else 0, _stream_handle(stream))
    _native.check(rc)
    return out[:total], blob_off


def _csr(parts: Optional[Sequence[bytes]]):
    if parts is None:
        return None, None
    data = np.frombuffer(b"".join(parts), np.uint8) if any(parts) else np.zeros(1, np.uint8)
    off = np.zeros(len(parts) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in parts])
    return np.ascontiguousarray(data), off


def build_ralledata_host(keys: Sequence[bytes], vals=None, skeys=None, attrs=None, std_fnv: bool = False,
                         device: int = 0):
    """Host form over lists of byte strings (None = segment empty for every record).
    Returns (blobs as one uint8 array, blob offsets n+1 uint64)."""
    n = len(keys)
    segs = [_csr(keys)] + [_csr(x) for x in (vals, skeys, attrs)]
    args, nbytes = [], []
    for d, o in segs:
        if o is None:
            args += [None, None]
            nbytes.append(0)
        else:
            args += [ctypes.c_void_p(d.ctypes.data), ctypes.c_void_p(o.ctypes.data)]
            nbytes.append(int(o[-1]))
    total = ralledata_size(n, *nbytes)
    out = np.zeros(max(total, 1), np.uint8)
    boff = np.zeros(n + 1, np.uint64)
    rc = _native.batch_lib().k2h_amd_build_ralledata_host(*args, n, ctypes.c_void_p(out.ctypes.data),
                                                          ctypes.c_void_p(boff.ctypes.data),
                                                          FLAG_STD_FNV if std_fnv else 0, device)
    _native.check(rc)
    return out[:total], boff
