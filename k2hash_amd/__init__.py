"""k2hash_amd -- MI355X-native key-hash path for yahoojapan/k2hash.

Scope: the default FNV-1a key hash of lib/k2hashfunc.cc,
as (1) a bit-exact drop-in hash plugin (C ABI, include/k2hash_amd.h section 1)
and (2) a batch C ABI backed by hand-written gfx950 HIP kernels (section 2).

  hashfunc   mirror of the reference interface: k2h_hash, k2h_second_hash,
             k2h_hash_version, K2HashDynLib, K2H_HASH_FUNC ...
  batch      device/host batch hashing, the fused bucket-index epilogue
             (K2HShm::GetKIndexPos / GetCKIndex positions), synthetic workloads
  shard      multi-GPU partitioning and the RCCL gather of hashes
"""
from .hashfunc import (K2H_2ND_HASH_FUNC, K2H_HASH_FUNC, K2H_HASH_VER_FUNC, K2HashDynLib, k2h_hash,
                       k2h_hash_version, k2h_second_hash)
from .batch import (bucket_index, hash_csr, hash_csr_host, hash_csr_index, hash_fixed, hash_fixed_host,
                    hash_fixed_index, synth_bytes, synth_offsets, unpack_kindex, version)

__all__ = [
    "k2h_hash", "k2h_second_hash", "k2h_hash_version", "K2HashDynLib", "K2H_HASH_FUNC",
    "K2H_2ND_HASH_FUNC", "K2H_HASH_VER_FUNC", "hash_fixed", "hash_csr", "hash_fixed_host",
    "hash_csr_host", "synth_bytes", "synth_offsets", "version", "bucket_index", "hash_fixed_index",
    "hash_csr_index", "unpack_kindex",
]
