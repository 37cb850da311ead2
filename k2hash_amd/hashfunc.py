"""Host-side mirror of k2hash's hash-function interface (lib/k2hashfunc.{h,cc}).

The reference exposes three C symbols plus a loader class:

  k2h_hash / k2h_second_hash / k2h_hash_version   lib/k2hashfunc.h:62-74
  K2HashDynLib::get/Load/Unload/get_k2h_*          lib/k2hashfunc.h:98-118, lib/k2hashfunc.cc:104-161
  K2H_HASH_FUNC / K2H_2ND_HASH_FUNC / K2H_HASH_VER_FUNC (dispatch macros)
                                                   lib/k2hashfunc.h:90-93

This module keeps those names, argument meanings and error behaviour so parity
tests read like the reference's own (tests/k2hexttest.cc:120-126, 166-175):
``K2HashDynLib.get().Load(path)`` dlopens a plugin and resolves the three symbols
all-or-nothing; the ``K2H_*`` dispatchers call the loaded plugin if one is loaded,
else the builtin (the k2hash_amd library's own symbols).
"""
from __future__ import annotations

import ctypes
from typing import Optional

from . import _native


def _buf(data) -> tuple[Optional[ctypes.c_void_p], int, object]:
    """(pointer, length, keepalive) for bytes-like `data`; None -> NULL."""
    if data is None:
        return None, 0, None
    mv = memoryview(data).cast("B")
    n = mv.nbytes
    if n == 0:
        # a valid non-NULL pointer with length 0 (reference returns 0 for length < 1)
        keep = ctypes.create_string_buffer(1)
        return ctypes.cast(keep, ctypes.c_void_p), 0, keep
    if mv.readonly:
        keep = ctypes.create_string_buffer(mv.tobytes(), n)
    else:
        keep = (ctypes.c_char * n).from_buffer(mv)
    return ctypes.cast(keep, ctypes.c_void_p), n, keep


def _call(fn, data, length: Optional[int]):
    ptr, n, keep = _buf(data)
    if length is not None:
        if length > n and ptr is not None:
            raise ValueError("length exceeds buffer")
        n = length
    r = fn(ptr, n)
    del keep
    return int(r)


def k2h_hash(data, length: Optional[int] = None) -> int:
    """lib/k2hashfunc.cc:62-74 -- builtin first hash (CPU, bit-exact)."""
    return _call(_native.batch_lib().k2h_hash, data, length)


def k2h_second_hash(data, length: Optional[int] = None) -> int:
    """lib/k2hashfunc.cc:76-91 -- builtin second hash."""
    return _call(_native.batch_lib().k2h_second_hash, data, length)


def k2h_hash_version() -> str:
    """lib/k2hashfunc.cc:93-96."""
    return _native.batch_lib().k2h_hash_version().decode()


class K2HashDynLib:
    """Mirror of K2HashDynLib (lib/k2hashfunc.h:98-118, lib/k2hashfunc.cc:104-161).

    Singleton via get(); Load() unloads any previous plugin, dlopens `path`
    (RTLD_LAZY like lib/k2hashfunc.cc:142) and resolves k2h_hash,
    k2h_second_hash and k2h_hash_version; if any is missing it unloads and
    returns False (lib/k2hashfunc.cc:149-156).
    """

    _instance: Optional["K2HashDynLib"] = None

    def __init__(self) -> None:
        self._lib: Optional[ctypes.CDLL] = None
        self.fp_k2h_hash = None
        self.fp_k2h_second_hash = None
        self.fp_k2h_hash_version = None

    @classmethod
    def get(cls) -> "K2HashDynLib":
        if cls._instance is None:
            cls._instance = cls()
        return cls._instance

    def Unload(self) -> bool:  # noqa: N802 (reference name)
        self._lib = None  # ctypes does not dlclose; dropping the handle is enough here
        self.fp_k2h_hash = self.fp_k2h_second_hash = self.fp_k2h_hash_version = None
        return True

    def Load(self, path) -> bool:  # noqa: N802 (reference name)
        if not path:
            return False
        self.Unload()
        try:
            lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_LOCAL)
        except OSError:
            return False
        try:
            fns = [getattr(lib, name) for name in _native.PLUGIN_SYMBOLS]
        except AttributeError:
            self.Unload()
            return False
        for fn, name in zip(fns, _native.PLUGIN_SYMBOLS):
            fn.restype, fn.argtypes = _native.SIGNATURES[name]
        self._lib = lib
        self.fp_k2h_hash, self.fp_k2h_second_hash, self.fp_k2h_hash_version = fns
        return True

    def get_k2h_hash(self):
        return self.fp_k2h_hash

    def get_k2h_second_hash(self):
        return self.fp_k2h_second_hash

    def get_k2h_hash_version(self):
        return self.fp_k2h_hash_version


def K2H_HASH_FUNC(data, length: Optional[int] = None) -> int:  # noqa: N802
    """lib/k2hashfunc.h:91: loaded plugin if any, else builtin."""
    fp = K2HashDynLib.get().get_k2h_hash()
    return _call(fp, data, length) if fp else k2h_hash(data, length)


def K2H_2ND_HASH_FUNC(data, length: Optional[int] = None) -> int:  # noqa: N802
    """lib/k2hashfunc.h:92."""
    fp = K2HashDynLib.get().get_k2h_second_hash()
    return _call(fp, data, length) if fp else k2h_second_hash(data, length)


def K2H_HASH_VER_FUNC() -> str:  # noqa: N802
    """lib/k2hashfunc.h:93."""
    fp = K2HashDynLib.get().get_k2h_hash_version()
    return fp().decode() if fp else k2h_hash_version()
