// k2hash_amd -- internal launch interface between the C-ABI (k2h_batch.cc) and the
// HIP kernels.  Not part of the public ABI (see include/k2hash_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/k2hash_amd.h"

namespace k2h {

constexpr uint64_t kSeedBuiltinValue = 14695981039346656037ULL;  // lib/k2hashfunc.cc:51
constexpr uint64_t kSeedStdValue = 2166136261ULL;                  // libstdc++ _Fnv_hash_impl seed

// Bucket-index epilogue: where a hash lands in a k2hash table with
// masks (cur_mask, collision_mask) -- the stateless part of K2HShm::GetKIndexPos
// (lib/k2hshm.cc:810-833, with MakeMask / GetMaskBitCount at :78-90) and the collision
// slot `hash & collision_mask` (lib/k2hshm.cc:1093).
//   shifted       = hash >> bitlen(collision_mask)   (shift count taken mod 64, as the
//                                                     x86-64 shr the reference compiles to)
//   KIPtrArrayPos = bitlen(shifted & cur_mask)        (the reference's bitmask loop)
//   KIArrayPos    = shifted & MakeMask(KIPtrArrayPos - 1)   (MakeMask(0) = 0)
// kindex[i] packs KIPtrArrayPos << 58 | KIArrayPos (bitlen(cur_mask) <= 58 checked by the
// ABI); ckindex[i] = hash & collision_mask.  Either output may be null.
// Table state (assigned != null): K2HShm::GetKIndex(hash, false) (lib/k2hshm.cc:882-907)
// -- cur_mask walked down (>>= 1) until the K_INDEX at the masked shifted hash is
// assigned; `assigned` has one bit per K_INDEX entry, entry (p, a) at bit p ? 2^(p-1)+a : 0,
// which is exactly the masked shifted hash v = (hash >> cshift) & m (p = bitlen(v),
// a = v without its top bit).  No assigned entry: the mask-1 probe (what the loop leaves);
// cur_mask 0: kindex = all ones (NULL).  found[i] = 1 when an assigned entry was reached.
struct BucketParams {
  uint64_t cur_mask = 0;
  uint64_t collision_mask = 0;
  uint32_t cshift = 0;
  uint64_t* kindex = nullptr;
  uint64_t* ckindex = nullptr;
  const uint32_t* assigned = nullptr;
  uint8_t* found = nullptr;
};
constexpr int kKindexPosShift = 58;

#ifdef __HIPCC__
// NT: nontemporal stores, for kernels whose lanes write consecutive i (a wave fills
// whole lines); kernels that write in a permuted order (CSR tiles, length-sorted) use
// plain stores so that L2 merges the partial lines before they reach HBM.
template <bool NT = true>
__device__ __forceinline__ void bucket_emit(const BucketParams& bp, uint64_t i, uint64_t h) {
  if (bp.assigned) {  // table state: GetKIndex's walk over the assigned K_INDEX entries
    const uint64_t shifted = h >> (bp.cshift & 63u);
    uint64_t tmp = 0;
    bool hit = false;
    for (uint64_t m = bp.cur_mask; m; m >>= 1) {
      tmp = shifted & m;
      if ((bp.assigned[tmp >> 5] >> (tmp & 31u)) & 1u) {
        hit = true;
        break;
      }
    }
    if (bp.kindex) {
      const uint64_t pos = tmp ? 64u - (uint64_t)__clzll((long long)tmp) : 0u;
      const uint64_t arr = pos ? tmp & ((1ull << (pos - 1)) - 1ull) : 0u;
      const uint64_t v = bp.cur_mask ? (pos << kKindexPosShift) | arr : ~0ull;
      if constexpr (NT) __builtin_nontemporal_store(v, bp.kindex + i);
      else bp.kindex[i] = v;
    }
    if (bp.found) bp.found[i] = hit;
  } else if (bp.kindex) {
    uint64_t shifted = h >> (bp.cshift & 63u);
    uint64_t tmp = shifted & bp.cur_mask;
    uint64_t pos = tmp ? 64u - (uint64_t)__clzll((long long)tmp) : 0u;
    uint64_t arr = pos ? shifted & ((1ull << (pos - 1)) - 1ull) : 0u;
    uint64_t v = (pos << kKindexPosShift) | arr;
    if constexpr (NT) __builtin_nontemporal_store(v, bp.kindex + i);
    else bp.kindex[i] = v;
  }
  if (bp.ckindex) {
    if constexpr (NT) __builtin_nontemporal_store(h & bp.collision_mask, bp.ckindex + i);
    else bp.ckindex[i] = h & bp.collision_mask;
  }
}
#endif

// Standalone epilogue over hashes already in device memory.
hipError_t launch_bucket_index(const uint64_t* h1, uint64_t n, const BucketParams& bp, hipStream_t stream);

// RALLEDATA producer inputs (k2h_ralledata.hip): four CSR streams; a null offsets
// array = that segment is empty for every record.
struct RalleInputs {
  const uint8_t* keys = nullptr;
  const uint64_t* koff = nullptr;
  const uint8_t* vals = nullptr;
  const uint64_t* voff = nullptr;
  const uint8_t* skeys = nullptr;
  const uint64_t* soff = nullptr;
  const uint8_t* attrs = nullptr;
  const uint64_t* aoff = nullptr;
};
hipError_t launch_ralledata(const RalleInputs& in, uint64_t n, uint64_t seed, uint8_t* out, uint64_t* blob_off,
                            hipStream_t stream);

// Keys at arbitrary (start, length) ranges (k2h_ranges.hip); cstr: hash key + NUL.
hipError_t launch_ranges(const void* base, const uint64_t* starts, const uint64_t* lens, uint64_t n, uint64_t seed,
                         bool cstr, uint64_t* h1, uint64_t* h2, hipStream_t stream);

// k2himport inputs already in device memory (k2h_import_dev.hip).  launch_import_scan
// returns a K2H_AMD_* code (the HIP error in *herr) and synchronises the stream.
// h1 != NULL: each written record's key is also hashed (key + NUL) by the same kernel.
int launch_import_scan(const void* file, uint64_t size, int format, k2h_amd_import_rec* recs, uint64_t cap,
                       uint64_t* count, hipStream_t stream, hipError_t* herr, uint64_t* h1 = nullptr,
                       uint64_t* h2 = nullptr, uint64_t seed = 0);
hipError_t launch_import_prehash(const void* file, uint64_t size, const k2h_amd_import_rec* recs, uint64_t n,
                                 uint64_t seed, uint64_t* h1, uint64_t* h2, hipStream_t stream);

// S_p = seed * P^-p (p = 0..15): start states for end-aligned chunking (k2h_csr.hip).
struct SpadTable {
  uint64_t v[16];
};
SpadTable make_spad(uint64_t seed);

// CSR tile kernel (k2h_csr.hip): 512-key LDS-staged tiles hashed two keys per lane; a
// tile whose bytes exceed the stage is hashed by the same block with the line ring.
hipError_t launch_csr_tile(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                           uint64_t* h2, hipStream_t stream, const BucketParams* bp = nullptr);
// Long fixed-length keys (> 32 B): the line-DMA kernel for multiples of 128 B at a
// 128-aligned base, else the cooperative line ring (>= 128 B) or direct loads (< 128 B).
bool fixed_lines_ok(const void* keys, uint64_t key_len);
hipError_t launch_fixed_long(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1,
                             uint64_t* h2, hipStream_t stream, const BucketParams* bp = nullptr);

hipError_t launch_fixed(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1, uint64_t* h2,
                        hipStream_t stream, const BucketParams* bp = nullptr);
hipError_t launch_csr(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                      uint64_t* h2, hipStream_t stream, const BucketParams* bp = nullptr);

// Synthetic inputs (bench/test harness; same spec as oracle/fnv_oracle.c generators).
hipError_t launch_synth_bytes(uint8_t* out, uint64_t nbytes, uint64_t seed, uint64_t byte_off, hipStream_t stream);
hipError_t launch_synth_lengths(uint32_t* lens, uint64_t n, uint64_t seed, uint64_t first_key, uint32_t min_len,
                                uint32_t max_len, hipStream_t stream);

}  // namespace k2h
