// k2hash_amd -- batched FNV-1a key-hash kernels for MI355X (gfx950).
//
// Bit-exact restatement of lib/k2hashfunc.cc:49-91 (k2h_Fnv_hash / k2h_hash /
// k2h_second_hash) over millions of independent keys per launch.  FNV-1a is a
// strictly serial chain per key, so one lane owns one key; a wave hashes 64 keys
// side by side.  Both hashes come from one pass: the reference's second hash is the
// FNV state after length-1 bytes (lib/k2hashfunc.cc:83-85), i.e. the state just
// before the final byte.
//
// Kernels:
//   fixed32      16M x 32-byte keys (BASELINE config 2).  Each lane loads its key
//                with two 16-byte loads; a wave reads one contiguous 2 KiB run.
//   fixed        any key length, any alignment; per-lane unaligned 16-byte loads.
//   csr          offsets+bytes (CSR) keys of any length (configs 3, 5); see k2h_csr.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "k2h_fnv_device.h"
#include "k2h_kernels.h"

namespace k2h {

typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));

__device__ __forceinline__ uint4 load16_ua(const uint8_t* p) {
  u32x4_ua v = *reinterpret_cast<const u32x4_ua*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Load up to 16 bytes at p without touching memory at or beyond `end` (bytes past
// the key are don't-care; the caller masks them by length).
__device__ __forceinline__ uint4 load16_guarded(const uint8_t* p, const uint8_t* end) {
  if (p + 16 <= end) return load16_ua(p);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16 && p + j < end; ++j) w[j >> 2] |= (uint32_t)p[j] << (8 * (j & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Hash the final 1..16 bytes of a key held in c (byte 0 first); returns h1 in (lo,hi)
// and the state before the last byte in (lo2,hi2).
__device__ __forceinline__ void fnv_tail(uint32_t& lo, uint32_t& hi, uint32_t& lo2, uint32_t& hi2, uint4 c,
                                         uint32_t r) {
  uint64_t q0 = ((uint64_t)c.y << 32) | c.x, q1 = ((uint64_t)c.w << 32) | c.z;
  for (uint32_t j = 0; j < r; ++j) {
    if (j + 1 == r) {
      lo2 = lo;
      hi2 = hi;
    }
    fnv_step_c(lo, hi, (uint32_t)q0 & 0xffu);
    q0 = (q0 >> 8) | (q1 << 56);
    q1 >>= 8;
  }
}

__device__ __forceinline__ uint64_t pack(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// Streaming (nontemporal) forms: every key byte is read once and every hash written
// once, so both bypass cache retention.  Measured on MI355X for the fixed32 access
// pattern (tools/mem_floor.hip): 104.9 us per 16M keys with nt loads + nt stores vs
// 114.6 us with default-policy accesses.
typedef uint32_t u32x4_v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  u32x4_v v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_v*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(uint64_t* p, uint64_t v) { __builtin_nontemporal_store(v, p); }

// ---------------------------------------------------------------------------
// fixed: key i = base[L*i .. L*i+L), any L >= 1, any alignment.  The loop trip
// count is wave-uniform (L is a kernel argument), so no lane diverges.
// ---------------------------------------------------------------------------
template <bool H2, bool EPI = false>
__global__ __launch_bounds__(256) void fnv_fixed_kernel(const uint8_t* __restrict__ base, uint64_t key_len, uint64_t n,
                                                        uint64_t seed, uint64_t* __restrict__ h1,
                                                        uint64_t* __restrict__ h2, BucketParams bp = {}) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = base + key_len * i;
  const uint8_t* end = base + key_len * n;
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2 = lo, hi2 = hi;
  uint64_t nfull = (key_len - 1) / 16;  // chunks strictly before the one holding the last byte
  for (uint64_t c = 0; c < nfull; ++c) fnv_chunk16(lo, hi, load16_ua(p + 16 * c));
  uint32_t r = (uint32_t)(key_len - 16 * nfull);
  fnv_tail(lo, hi, lo2, hi2, load16_guarded(p + 16 * nfull, end), r);
  if (key_len == 1) {  // length 1: the second hash is not shortened (lib/k2hashfunc.cc:83)
    lo2 = lo;
    hi2 = hi;
  }
  h1[i] = pack(lo, hi);
  if constexpr (H2) h2[i] = pack(lo2, hi2);
  if constexpr (EPI) bucket_emit(bp, i, pack(lo, hi));
}

// Standalone bucket-index epilogue over hashes in device memory.
__global__ __launch_bounds__(256) void bucket_index_kernel(const uint64_t* __restrict__ h1, uint64_t n,
                                                           BucketParams bp) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i < n) bucket_emit(bp, i, __builtin_nontemporal_load(h1 + i));
}

// ---------------------------------------------------------------------------
// zero fill (length-0 keys, NULL key buffers: lib/k2hashfunc.cc:66-68)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void fill_zero_kernel(uint64_t* __restrict__ p, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i < n) p[i] = 0;
}

static inline unsigned grid_for(uint64_t n) { return (unsigned)((n + 255) / 256); }

// fixed32 (BASELINE config 2): 32-byte keys at a 16-aligned base.  One-wave blocks, KPT
// keys per lane: block b owns keys [b*64*KPT, (b+1)*64*KPT), lane t hashes keys
// b*64*KPT + 64 j + t.  All 2*KPT nontemporal loads are issued before the first hash, so
// each wave keeps KPT*2 KiB in flight while it computes; one-wave blocks let a finished
// wave's slot be refilled at once (round-1 A/B: KPT = 2, 64-thread blocks, nt loads and
// stores).  The second key's registers sit below the asm window, so
// the kernel stays at 59 VGPRs (8 waves/SIMD).  The headline form (KPT = 2, h1 only) is one
// asm statement per lane (fnv_key32_pair_x): hipcc waited for all four loads before the
// first hash; there key 0 is hashed once its own two loads are in (vmcnt(2)) and key 1 in
// the registers it was loaded into (round 3: 118.0 -> 113.7 us on config 2 in A/B,
// profiles/r03af_fixed32_ab.txt).
template <bool H2, int KPT, bool EPI = false>
__global__ __launch_bounds__(64) void fnv_fixed32_kpt_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                             uint64_t seed, uint64_t* __restrict__ h1,
                                                             uint64_t* __restrict__ h2, BucketParams bp = {}) {
  constexpr int BS = 64;
  const uint64_t base = (uint64_t)blockIdx.x * (BS * KPT) + threadIdx.x;
  if constexpr (KPT == 2 && !H2 && !EPI) {  // the headline form: one asm statement per lane
    // lanes past the end re-hash key n-1 and store its (identical) hash to h1[n-1]
    const uint64_t i0 = base < n ? base : n - 1, i1 = base + BS < n ? base + BS : n - 1;
    fnv_key32_pair_x(keys + 2 * i0, keys + 2 * i1, h1 + i0, h1 + i1, seed);
    return;
  } else if constexpr (KPT == 2) {  // h2 and / or the fused index: the same statement, hashes returned
    const uint64_t i0 = base < n ? base : n - 1, j1 = base + BS, i1 = j1 < n ? j1 : n - 1;
    uint64_t r0, r1, s0, s1;
    fnv_key32_pair_r<H2>(keys + 2 * i0, keys + 2 * i1, seed, r0, r1, s0, s1);
    if (base < n) {
      st_nt(h1 + base, r0);
      if constexpr (H2) st_nt(h2 + base, s0);
      if constexpr (EPI) bucket_emit(bp, base, r0);
    }
    if (j1 < n) {
      st_nt(h1 + j1, r1);
      if constexpr (H2) st_nt(h2 + j1, s1);
      if constexpr (EPI) bucket_emit(bp, j1, r1);
    }
    return;
  }
  uint4 a[KPT], b[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint64_t i = base + BS * j;
    if (i < n) {
      a[j] = ld_nt(keys + 2 * i);
      b[j] = ld_nt(keys + 2 * i + 1);
    }
  }
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const uint64_t i = base + BS * j;
    if (i < n) {
      uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2, hi2;
      if constexpr (H2) {
        fnv_chunk32_last(lo, hi, lo2, hi2, a[j], b[j]);
        st_nt(h2 + i, pack(lo2, hi2));
      } else {
        fnv_chunk32(lo, hi, a[j], b[j]);
      }
      st_nt(h1 + i, pack(lo, hi));
      if constexpr (EPI) bucket_emit(bp, i, pack(lo, hi));
    }
  }
}

hipError_t launch_bucket_index(const uint64_t* h1, uint64_t n, const BucketParams& bp, hipStream_t stream) {
  if (n == 0 || !(bp.kindex || bp.ckindex || bp.found)) return hipSuccess;
  bucket_index_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n, bp);
  return hipGetLastError();
}

// Default kernel per shape (the product path).  32-byte keys at a 16-aligned base: one-wave
// blocks, two keys per lane with all four loads issued before the first hash (a wave keeps
// 4 KiB in flight and half as many waves need dispatching; round-1 A/B).
// Other lengths: up to 32 B the per-lane tail loop, below 128 B
// per-lane direct 16-byte loads, from 128 B on the line-DMA kernel (multiples of 128 B at a
// 128-aligned base) or the cooperative line ring.
hipError_t launch_fixed(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1, uint64_t* h2,
                        hipStream_t stream, const BucketParams* bp) {
  if (n == 0) return hipSuccess;
  const bool epi = bp && (bp->kindex || bp->ckindex || bp->found);
  if (!keys || key_len == 0) {
    fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n);
    if (h2) fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h2, n);
    if (epi) return launch_bucket_index(h1, n, *bp, stream);
    return hipGetLastError();
  }
  if (key_len == 32 && ((uintptr_t)keys & 15u) == 0) {
    const uint4* k = (const uint4*)keys;
    const unsigned g = (unsigned)((n + 127) / 128);
    if (epi) {
      if (h2) fnv_fixed32_kpt_kernel<true, 2, true><<<g, 64, 0, stream>>>(k, n, seed, h1, h2, *bp);
      else fnv_fixed32_kpt_kernel<false, 2, true><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr, *bp);
    } else {
      if (h2) fnv_fixed32_kpt_kernel<true, 2><<<g, 64, 0, stream>>>(k, n, seed, h1, h2);
      else fnv_fixed32_kpt_kernel<false, 2><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr);
    }
    return hipGetLastError();
  }
  if (key_len > 32)
    return launch_fixed_long(keys, key_len, n, seed, h1, h2, stream, epi ? bp : nullptr);
  const uint8_t* kb = (const uint8_t*)keys;
  if (epi) {
    if (h2) fnv_fixed_kernel<true, true><<<grid_for(n), 256, 0, stream>>>(kb, key_len, n, seed, h1, h2, *bp);
    else fnv_fixed_kernel<false, true><<<grid_for(n), 256, 0, stream>>>(kb, key_len, n, seed, h1, nullptr, *bp);
  } else {
    if (h2) fnv_fixed_kernel<true><<<grid_for(n), 256, 0, stream>>>(kb, key_len, n, seed, h1, h2);
    else fnv_fixed_kernel<false><<<grid_for(n), 256, 0, stream>>>(kb, key_len, n, seed, h1, nullptr);
  }
  return hipGetLastError();
}

// CSR keys: 512-key tiles staged in LDS and hashed two keys per lane (k2h_csr.hip); a NULL
// byte buffer hashes every key to 0 (lib/k2hashfunc.cc:66-68, 80-82).
hipError_t launch_csr(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                      uint64_t* h2, hipStream_t stream, const BucketParams* bp) {
  if (n == 0) return hipSuccess;
  const bool epi = bp && (bp->kindex || bp->ckindex || bp->found);
  if (!bytes) {
    fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n);
    if (h2) fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h2, n);
    if (epi) return launch_bucket_index(h1, n, *bp, stream);
    return hipGetLastError();
  }
  return launch_csr_tile(bytes, offsets, n, seed, h1, h2, stream, epi ? bp : nullptr);
}

}  // namespace k2h
