// k2hash_amd -- kernels for variable-length (CSR) keys and long fixed-length keys.
//
// FNV-1a (lib/k2hashfunc.cc:49-59) is serial per key, so one lane owns one key and a
// wave runs as long as its longest key.  Three measures keep a wave's 64 lanes busy
// and its memory traffic line-efficient:
//
//  1. End-aligned 16-byte chunks.  A key of len bytes is hashed as k = ceil(len/16)
//     whole chunks ending exactly at its last byte; the first chunk starts p = 16k-len
//     bytes early and its p leading bytes are zeroed.  A zero byte is a pure multiply
//     (h ^= 0; h *= P), so starting from S_p = seed * P^-p (mod 2^64) those p steps
//     land exactly on the seed.  Every lane therefore runs whole hand-scheduled chunk
//     steps with no per-byte tail loop, and the second hash -- the state before the
//     final byte (lib/k2hashfunc.cc:83-85) -- is always byte 15 of the last chunk.
//  2. Length sort per tile (CSR).  A 256-thread block takes a tile of 512 consecutive
//     keys, DMAs the tile's bytes into LDS, counting-sorts the keys by chunk count, and
//     lane i hashes sorted keys i and 511-i back to back (a short and a long one: pair
//     sums are nearly equal across a wave).
//  3. The line ring (ring_hash), for keys that are not staged in LDS.  Per-lane loads of
//     16 B at 64 scattered keys run at 2-3 TB/s on MI355X (tools/stream_floor2.hip);
//     instead every lane's key is streamed as whole 128-byte-aligned lines: each round
//     the wave loads one line per lane cooperatively (8 lanes x 16 B per line, 8 full
//     lines per load instruction -- 5.7 TB/s in the same probe) into a 2-line LDS ring
//     per lane, and the lane reads its next 8 chunks from the ring at its own byte
//     offset.  A line is only ever loaded if it holds a byte of some key, so no load can
//     leave the buffer's pages and no bounds checks are needed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "k2h_fnv_device.h"
#include "k2h_kernels.h"

namespace k2h {

namespace {

typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x4_v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4_v gvec4;

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  u32x4_ua v = *reinterpret_cast<const u32x4_ua*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// 16 bytes at p where bytes below `lo` must not be touched (they are don't-care).
__device__ __forceinline__ uint4 ld16_lowguard(const uint8_t* p, const uint8_t* lo) {
  if (p >= lo) return ld16(p);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int j = 0; j < 16; ++j)
    if (p + j >= lo) w[j >> 2] |= (uint32_t)p[j] << (8 * (j & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Zero the first p (0..15) bytes of a chunk.
__device__ __forceinline__ uint4 mask_lead(uint4 c, uint32_t p) {
  // word mask = low half of (~0 << clamp(8p - base, 0, 32)): sub, med3, 64-bit shift
  // (a 32-bit shift cannot produce the all-zero mask), no compares or selects
  int32_t sh = (int32_t)(8u * p);
  auto m = [sh](int32_t base) -> uint32_t {
    int32_t t = sh - base;
    t = t < 0 ? 0 : (t > 32 ? 32 : t);
    return (uint32_t)(~0ull << t);
  };
  return make_uint4(c.x & m(0), c.y & m(32), c.z & m(64), c.w & m(96));
}

__device__ __forceinline__ uint64_t pack2(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}
__device__ __forceinline__ uint64_t bperm64(uint64_t v, uint32_t src_lane) {
  return ((uint64_t)bperm((uint32_t)(v >> 32), src_lane) << 32) | bperm((uint32_t)v, src_lane);
}
// LDS atomics and barriers for the phases that run while a tile's LDS-DMA is in flight.
// hipcc (ROCm 7.2) puts an s_waitcnt vmcnt(0) in front of any LDS atomic and any
// __syncthreads() while a global_load_lds is outstanding (it cannot prove they do not
// alias the DMA target), which drained the whole tile DMA before the length sort
// started.  As asm they carry no such wait; the sort touches only s_hist / s_order /
// s_wsum, never the stage the DMA writes.
__device__ __forceinline__ void lds_add(uint32_t* p, uint32_t v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)p), "v"(v)
               : "memory");
}
__device__ __forceinline__ uint32_t lds_add_rtn(uint32_t* p, uint32_t v) {
  uint32_t r;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(r)
               : "v"((uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)p), "v"(v)
               : "memory");
  return r;
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    uint32_t o = (uint32_t)__shfl_xor((int)v, d, 64);
    v = o > v ? o : v;
  }
  return v;
}


// ---------------------------------------------------------------------------
// Direct per-lane walker (fixed keys of 33-127 bytes): each lane loads its own chunks.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void hash_key(const uint8_t* s, const uint8_t* e, const uint8_t* lo_bound,
                                         const uint64_t* spad, uint64_t& r1, uint64_t& r2) {
  uint64_t len = (uint64_t)(e - s);
  if (len == 0) {  // lib/k2hashfunc.cc:66-68, 80-82
    r1 = r2 = 0;
    return;
  }
  uint64_t k = (len + 15) >> 4;
  uint32_t p = (uint32_t)(16 * k - len);
  const uint8_t* cp = e - 16 * k;
  uint64_t st = spad[p];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2, hi2;
  uint4 c = mask_lead(ld16_lowguard(cp, lo_bound), p);
  for (uint64_t j = 1; j < k; ++j) {
    uint4 nx = ld16(cp + 16 * j);
    fnv_chunk16(lo, hi, c);
    c = nx;
  }
  fnv_chunk16_last(lo, hi, lo2, hi2, c);
  r1 = pack2(lo, hi);
  r2 = len == 1 ? r1 : pack2(lo2, hi2);  // length 1: second hash not shortened (lib/k2hashfunc.cc:83)
}


// ---------------------------------------------------------------------------
// The line ring.
// ---------------------------------------------------------------------------
constexpr int kRingRow = 272;  // 2 x 128-byte slots + 16-byte mirror of slot 0's head
struct alignas(16) Ring {
  uint8_t b[64][kRingRow];
};

// Hash key [s, e) of every valid lane of the wave.  All 64 lanes must call.
// `safe` is any readable 128-byte-aligned address (used by idle lanes' loads).
__device__ __forceinline__ void ring_hash(bool valid, const uint8_t* s, const uint8_t* e, uint64_t safe,
                                          const uint64_t* spad, Ring& ring, uint64_t& r1, uint64_t& r2) {
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t len = valid ? (uint64_t)(e - s) : 0;
  uint32_t k = (uint32_t)((len + 15) >> 4);  // chunks (0: empty key or idle lane)
  uint32_t p = (uint32_t)(16u * k - len);    // leading pad bytes of chunk 0
  uint64_t cp = (uint64_t)(uintptr_t)e - 16ull * k;  // chunk 0 (virtual start, may precede s)
  uint64_t blk0 = cp & ~127ull;
  uint32_t mis = (uint32_t)(cp & 127u);
  // lines of this lane's stream that hold key bytes: [first, last] (relative to blk0)
  uint32_t first = 0, last = 0;
  if (k) {
    first = (uint32_t)(((uint64_t)(uintptr_t)s - blk0) >> 7);
    last = (uint32_t)(((uint64_t)(uintptr_t)e - 1 - blk0) >> 7);
  } else {
    blk0 = safe;
  }
  const uint32_t rounds = (k + 7) >> 3;
  const uint32_t R = wave_max(rounds);
  uint64_t st = spad[p & 15u];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2 = lo, hi2 = hi;

  if (R) {
    // load instruction j: lane t fetches piece t&7 of line q of lane 8j + t/8
    const uint32_t piece = lane & 7u;
    uint64_t jb[8];
    uint32_t jf[8], jl[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint32_t src = 8u * j + (lane >> 3);
      jb[j] = bperm64(blk0, src) + 16u * piece;
      jf[j] = bperm(first, src);
      jl[j] = bperm(last, src);
    }
    auto load_line = [&](uint32_t q, uint4 (&v)[8]) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint32_t qq = q < jf[j] ? jf[j] : (q > jl[j] ? jl[j] : q);  // keep to lines holding key bytes
        u32x4_v x = __builtin_nontemporal_load((gvec4*)(uintptr_t)(jb[j] + 128ull * qq));
        v[j] = make_uint4(x.x, x.y, x.z, x.w);
      }
    };
    auto store_line = [&](uint32_t q, const uint4 (&v)[8]) {
      uint32_t off = (q & 1u) * 128u + 16u * piece;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint8_t* row = ring.b[8u * j + (lane >> 3)];
        *reinterpret_cast<uint4*>(row + off) = v[j];
        if (off == 0) *reinterpret_cast<uint4*>(row + 256) = v[j];  // mirror: reads may wrap
      }
    };
    uint4 va[8], vb[8];
    load_line(0, va);
    load_line(1, vb);
    store_line(0, va);
    store_line(1, vb);
    if (R >= 2) load_line(2, va);
    asm volatile("" ::: "memory");
    const uint8_t* row = ring.b[lane];
    for (uint32_t r = 0; r < R; ++r) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        uint32_t q = 8u * r + m;
        if (q < k) {
          uint4 c = ld16(row + ((mis + 16u * q) & 255u));
          if (q == 0) c = mask_lead(c, p);
          if (q + 1 < k) {
            fnv_chunk16(lo, hi, c);
          } else {
            fnv_chunk16_last(lo, hi, lo2, hi2, c);
          }
        }
      }
      asm volatile("" ::: "memory");  // one wave's LDS ops execute in order; keep the compiler's
      if (r + 2 <= R) {
        store_line(r + 2, va);
        if (r + 3 <= R) load_line(r + 3, va);
      }
      asm volatile("" ::: "memory");
    }
  }
  if (k == 0) {  // empty key (lib/k2hashfunc.cc:66-68, 80-82) or idle lane
    r1 = r2 = 0;
    return;
  }
  r1 = pack2(lo, hi);
  r2 = len == 1 ? r1 : pack2(lo2, hi2);
}

}  // namespace


// Sort class of a key: its chunk count below 96 chunks (1536 B), then 4 sub-classes per
// octave of chunk count (128 classes).
__device__ __forceinline__ uint32_t len_bin128(uint64_t len) {
  if (len == 0) return 0;
  const uint64_t k = (len + 15) >> 4;
  if (k < 96) return (uint32_t)k;
  const uint32_t lg = 63u - (uint32_t)__clzll((long long)k);  // >= 6
  const uint32_t b = 96u + (lg - 6u) * 4u + (uint32_t)((k >> (lg - 2u)) & 3u);
  return b < 128u ? b : 127u;
}
__device__ __forceinline__ uint32_t len_bin128_32(uint32_t len) {
  if (len == 0) return 0;
  const uint32_t k = (len + 15u) >> 4;
  if (k < 96) return k;
  const uint32_t lg = 31u - (uint32_t)__clz((int)k);  // >= 6
  const uint32_t b = 96u + (lg - 6u) * 4u + ((k >> (lg - 2u)) & 3u);
  return b < 128u ? b : 127u;
}

// The reference's second hash from the first and the key's last byte: h1 = (h2 ^
// sext(b)) * P (lib/k2hashfunc.cc:53-56), P odd, so h2 = (h1 * P^-1) ^ sext(b); for a
// one-byte key h2 = h1 (lib/k2hashfunc.cc:83), for an empty one 0.
constexpr uint64_t prime_inverse() {
  uint64_t x = 1099511628211ULL;
  for (int i = 0; i < 6; ++i) x *= 2 - 1099511628211ULL * x;
  return x;
}
static_assert(prime_inverse() * 1099511628211ULL == 1, "P^-1 mod 2^64");
__device__ __forceinline__ uint64_t second_from_first(uint64_t h1v, uint32_t len, const uint8_t* key_end) {
  if (len <= 1) return h1v;  // 0 for an empty key, h1 for a one-byte key
  const int64_t sb = (int64_t)(int8_t)key_end[-1];
  return (h1v * prime_inverse()) ^ (uint64_t)sb;
}

// Two keys per lane, back to back: key 0 (k0 >= 1 chunks unless the lane is idle) then
// key 1 (k1 chunks, 0 = none), end-aligned chunks read from LDS, the switch to key 1
// (save key 0's state, restart from key 1's S_p with its masked chunk 0) in a branch
// that only the lanes switching at that step take.  Chunk reads alternate between the
// two asm register banks with the next read in flight under the current chunk's steps.
// Returns the two h1 values.
__device__ __forceinline__ void pair_walk(uint32_t k0, uint32_t p0, const uint8_t* cp0, uint32_t k1, uint32_t p1,
                                          const uint8_t* cp1, const uint64_t* spad, const uint4* masks, uint64_t& h0,
                                          uint64_t& h1v) {
  const uint32_t T = k0 + k1, sw = k0;
  uint64_t st = spad[p0];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32);
  const uint8_t* cp = cp0;
  uint4 m = masks[p0];
  uint4 c0 = ld16(cp0);
  c0 = make_uint4(c0.x & m.x, c0.y & m.y, c0.z & m.z, c0.w & m.w);
  uint4 c1 = c0;
  uint64_t saved = 0;
  bool odd = false;
  if (T > 1) {
    uint32_t t = 0;
    for (;;) {
      c1 = ld16(cp + 16u * (t + 1));
      fnv_chunk16<0>(lo, hi, c0);
      ++t;
      if (t == sw) {
        saved = pack2(lo, hi);
        st = spad[p1];
        lo = (uint32_t)st;
        hi = (uint32_t)(st >> 32);
        cp = cp1 - 16 * (int32_t)t;
        m = masks[p1];
        c1 = ld16(cp1);
        c1 = make_uint4(c1.x & m.x, c1.y & m.y, c1.z & m.z, c1.w & m.w);
      }
      if (t + 1 >= T) {
        odd = true;
        break;
      }
      c0 = ld16(cp + 16u * (t + 1));
      fnv_chunk16<1>(lo, hi, c1);
      ++t;
      if (t == sw) {
        saved = pack2(lo, hi);
        st = spad[p1];
        lo = (uint32_t)st;
        hi = (uint32_t)(st >> 32);
        cp = cp1 - 16 * (int32_t)t;
        m = masks[p1];
        c0 = ld16(cp1);
        c0 = make_uint4(c0.x & m.x, c0.y & m.y, c0.z & m.z, c0.w & m.w);
      }
      if (t + 1 >= T) break;
    }
  }
  if (odd) c0 = c1;
  fnv_chunk16<0>(lo, hi, c0);  // the last chunk of the lane's last key
  if (k1) {
    h0 = saved;
    h1v = pack2(lo, hi);
  } else {
    h0 = pack2(lo, hi);
    h1v = 0;
  }
}

constexpr uint32_t kTileKeys = 512;
constexpr uint32_t kStageBytes = 72 * 1024u;
constexpr uint32_t kNumClasses = 128;
static_assert(4 * sizeof(Ring) <= 16 + kStageBytes, "the oversize path's four line rings fit the stage");

// A tile whose bytes exceed the LDS stage (keys averaging > ~144 B): the block sorts its
// keys by class from their 64-bit offsets and each wave hashes groups of 64 sorted keys
// with the line ring, the four rings laid over the stage.  Block-uniform; no LDS-DMA in
// flight, so plain LDS atomics and barriers.
template <bool H2, bool EPI>
__device__ __forceinline__ void oversize_tile(uint64_t t0, uint32_t cnt, const uint8_t* __restrict__ bytes,
                                           const uint64_t* __restrict__ offsets, const uint64_t* s_spad,
                                           uint16_t* s_order, uint32_t* s_hist, Ring* rings,
                                           uint64_t* __restrict__ h1, uint64_t* __restrict__ h2,
                                           const BucketParams& bp) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  uint32_t bins[2];
#pragma unroll
  for (uint32_t j = 0; j < 2; ++j) {
    const uint32_t k = tid + 256u * j;
    if (k < cnt) {
      bins[j] = len_bin128(offsets[t0 + k + 1] - offsets[t0 + k]);
      atomicAdd(&s_hist[bins[j]], 1u);
    }
  }
  __syncthreads();
  if (wave == 0) {  // exclusive scan of the 128 class counts, two per lane
    const uint32_t v0 = s_hist[2 * lane], v1 = s_hist[2 * lane + 1], sum = v0 + v1;
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    s_hist[2 * lane] = incl - sum;
    s_hist[2 * lane + 1] = incl - sum + v0;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < 2; ++j) {
    const uint32_t k = tid + 256u * j;
    if (k < cnt) s_order[atomicAdd(&s_hist[bins[j]], 1u)] = (uint16_t)k;
  }
  __syncthreads();
  const uint64_t safe = (uint64_t)(uintptr_t)(bytes + offsets[0]) & ~127ull;
  const uint32_t ngroups = (cnt + 63u) >> 6;
  // groups are in length order: wave w takes groups w, 7-w, 8+w, 15-w, ... (snake)
  for (uint32_t it = 0; it * 4 < ngroups; ++it) {
    const uint32_t g = it * 4 + ((it & 1) ? 3 - wave : wave);
    if (g >= ngroups) continue;  // wave-uniform
    const uint32_t idx = g * 64u + lane;
    const bool valid = idx < cnt;
    const uint32_t k = s_order[valid ? idx : cnt - 1];
    uint64_t r1, r2;
    ring_hash(valid, bytes + offsets[t0 + k], bytes + offsets[t0 + k + 1], safe, s_spad, rings[wave], r1, r2);
    if (valid) {
      h1[t0 + k] = r1;
      if constexpr (H2) h2[t0 + k] = r2;
      if constexpr (EPI) bucket_emit<false>(bp, t0 + k, r1);
    }
  }
}

// ---------------------------------------------------------------------------
// CSR: one 256-thread block per tile of 512 consecutive keys (BASELINE config 3).
//  setup (at issue priority 1, so it does not queue behind the co-resident block's hash
//  instructions on the same SIMD): the tile's offsets as 32-bit tile-relative values in
//  LDS; the tile's byte span DMA'd into a 72 KiB LDS stage (global_load_lds, 16 B per
//  lane, no VGPR transit), in flight while the keys are counting-sorted by chunk count;
//  the 128-class scan by wave 0 alone.
//  walk (priority 0): lane i hashes sorted keys i and cnt-1-i back to back (pair_walk);
//  h2 is derived from h1 and the key's last byte (second_from_first).
// Two blocks fit a CU (2 x ~76 KiB of LDS): 2 waves per SIMD.  A tile whose span exceeds
// the stage takes the line-ring path in the same block (oversize_tile), so one launch
// covers every input and the call needs no scratch memory.
// ---------------------------------------------------------------------------
template <bool H2, bool EPI>
__global__ __launch_bounds__(256) void fnv_csr_staged_kernel(const uint8_t* __restrict__ bytes,
                                                           const uint64_t* __restrict__ offsets, uint64_t n,
                                                           SpadTable spad_tab, uint64_t* __restrict__ h1,
                                                           uint64_t* __restrict__ h2, BucketParams bp) {
  constexpr uint32_t TK = kTileKeys, NT = 256, NB = kNumClasses;
  __shared__ uint32_t s_rel[TK + 1];
  __shared__ uint16_t s_order[TK];
  __shared__ uint32_t s_hist[NB];
  __shared__ uint64_t s_spad[16];
  __shared__ uint4 s_mask[16];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[16 + kStageBytes];

  __builtin_amdgcn_s_setprio(1);
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t t0 = (uint64_t)blockIdx.x * TK;
  const uint32_t cnt = (uint32_t)(n - t0 < (uint64_t)TK ? n - t0 : (uint64_t)TK);
  const uint64_t o0 = offsets[t0], oN = offsets[t0 + cnt];  // block-uniform
  const uint64_t kb = (uint64_t)(uintptr_t)bytes + o0;
  const uint64_t span_lo = kb & ~15ull;
  const uint32_t delta = (uint32_t)(kb & 15u);
  const uint64_t span = oN - o0 + delta;  // stage bytes up to the tile's last key byte
  if (tid < 16) s_spad[tid] = spad_tab.v[tid];
  if (tid < NB) s_hist[tid] = 0;
  if (span > kStageBytes) {  // block-uniform
    __syncthreads();
    __builtin_amdgcn_s_setprio(0);
    oversize_tile<H2, EPI>(t0, cnt, bytes, offsets, s_spad, s_order, s_hist, reinterpret_cast<Ring*>(s_stage), h1,
                           h2, bp);
    return;
  }
  if (tid < 16) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // bytes >= p kept: chunk 0's p pad bytes zeroed
      const int32_t sh = 8 * ((int32_t)tid - 4 * i);
      w[i] = sh <= 0 ? ~0u : sh >= 32 ? 0u : ~0u << sh;
    }
    s_mask[tid] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  {  // a thread's three offset loads in flight together (a loop waited for each in turn:
     // round-3 lab A/B, -2 % on config 3, profiles/r03r_csr_ab.json)
    uint32_t r[3];
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      const uint32_t k = tid + NT * q;
      r[q] = k <= cnt ? (uint32_t)offsets[t0 + k] : 0u;
    }
#pragma unroll
    for (uint32_t q = 0; q < 3; ++q) {
      const uint32_t k = tid + NT * q;
      if (k <= cnt) s_rel[k] = r[q] - (uint32_t)o0;
    }
  }
  static_assert(3 * NT >= TK + 1, "three offsets per thread cover the tile");
  __syncthreads();

  // DMA of the tile span (16-byte pieces; pieces past the span re-read its last piece
  // into stage bytes nobody reads), in flight during the sort
  if (oN > o0) {
    const uint32_t npieces = (uint32_t)((span + 1023) >> 10);
    const uint32_t lastp = ((uint32_t)span - 1u) & ~15u;
    const uint8_t* src0 = (const uint8_t*)(uintptr_t)span_lo;
    uint32_t off = 1024u * wave + 16u * lane;
    for (uint32_t c = wave; c < npieces; c += 4, off += 4096u) {
      const uint32_t o = off < lastp ? off : lastp;
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src0 + o),
                                       (__attribute__((address_space(3))) void*)(s_stage + 16 + 1024u * c), 16, 0, 0);
    }
  }
  // counting sort by class (LDS atomics and barriers in asm: no compiler vmcnt drain of
  // the DMA in flight, see lds_add)
  uint32_t bins[2];
#pragma unroll
  for (uint32_t j = 0; j < 2; ++j) {
    const uint32_t k = tid + NT * j;
    if (k < cnt) {
      bins[j] = len_bin128_32(s_rel[k + 1] - s_rel[k]);
      lds_add(&s_hist[bins[j]], 1u);
    }
  }
  lds_barrier();
  if (wave == 0) {  // exclusive scan of the 128 class counts, two per lane
    const uint32_t v0 = s_hist[2 * lane], v1 = s_hist[2 * lane + 1], sum = v0 + v1;
    uint32_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    s_hist[2 * lane] = incl - sum;
    s_hist[2 * lane + 1] = incl - sum + v0;
  }
  lds_barrier();
#pragma unroll
  for (uint32_t j = 0; j < 2; ++j) {
    const uint32_t k = tid + NT * j;
    if (k < cnt) s_order[lds_add_rtn(&s_hist[bins[j]], 1u)] = (uint16_t)k;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces have landed
  __syncthreads();                                   // ... and every other wave's
  __builtin_amdgcn_s_setprio(0);

  // Pair walk: lane i (0..255) takes sorted keys i and cnt-1-i, a short and a long one,
  // and hashes them back to back; sums of the pair lengths are nearly equal across a
  // wave, so the wave's length waste drops from 10.8 % (groups of 64 equal-class keys)
  // to ~3.4 % on BASELINE config 3.
  const uint8_t* key0 = s_stage + 16 + delta;
  const uint32_t i = wave * 64u + lane;
  const bool has_a = i < (cnt + 1u) / 2u, has_b = i < cnt / 2u;
  const uint32_t ka = s_order[has_a ? i : 0u], kbi = s_order[has_b ? cnt - 1u - i : 0u];
  const uint32_t ra = s_rel[ka], rae = s_rel[ka + 1], rb = s_rel[kbi], rbe = s_rel[kbi + 1];
  const uint32_t la = has_a ? rae - ra : 0u, lb = has_b ? rbe - rb : 0u;
  const uint32_t kA = (la + 15u) >> 4, kB = (lb + 15u) >> 4;
  const uint32_t pA = (0u - la) & 15u, pB = (0u - lb) & 15u;
  const uint8_t* cpA = key0 + (int32_t)(rae - 16u * kA);
  const uint8_t* cpB = key0 + (int32_t)(rbe - 16u * kB);
  const bool only_b = kA == 0;  // key A empty (or absent): walk B alone
  uint64_t hw0, hw1;
  pair_walk(only_b ? kB : kA, only_b ? pB : pA, only_b ? cpB : cpA, only_b ? 0u : kB, pB, cpB, s_spad, s_mask, hw0,
            hw1);
  const uint64_t hA = kA ? hw0 : 0, hB = kB ? (only_b ? hw0 : hw1) : 0;
  if (has_a) {
    h1[t0 + ka] = hA;
    if constexpr (H2) h2[t0 + ka] = second_from_first(hA, la, key0 + rae);
    if constexpr (EPI) bucket_emit<false>(bp, t0 + ka, hA);
  }
  if (has_b) {
    h1[t0 + kbi] = hB;
    if constexpr (H2) h2[t0 + kbi] = second_from_first(hB, lb, key0 + rbe);
    if constexpr (EPI) bucket_emit<false>(bp, t0 + kbi, hB);
  }
}

// ---------------------------------------------------------------------------
// Fixed-length keys other than the 32-byte fast path (e.g. BASELINE config 5,
// 4 KiB): one lane per key, the same chunk walker, uniform trip count.
// ---------------------------------------------------------------------------
template <bool H2, bool DIRECT, bool EPI = false>
__global__ __launch_bounds__(256) void fnv_fixed_long_kernel(const uint8_t* __restrict__ base, uint64_t key_len,
                                                             uint64_t n, SpadTable spad_tab,
                                                             uint64_t* __restrict__ h1, uint64_t* __restrict__ h2,
                                                             BucketParams bp = {}) {
  __shared__ uint64_t s_spad[16];
  __shared__ Ring s_ring[DIRECT ? 1 : 4];
  if (threadIdx.x < 16) s_spad[threadIdx.x] = spad_tab.v[threadIdx.x];
  __syncthreads();
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  bool valid = i < n;
  uint64_t r1, r2;
  if constexpr (DIRECT) {
    if (!valid) return;
    hash_key(base + key_len * i, base + key_len * (i + 1), base, s_spad, r1, r2);
  } else {
    if ((uint64_t)blockIdx.x * 256u + (threadIdx.x & ~63u) >= n) return;  // whole wave idle
    uint64_t ii = valid ? i : n - 1;
    ring_hash(valid, base + key_len * ii, base + key_len * (ii + 1), (uint64_t)(uintptr_t)base & ~127ull, s_spad,
              s_ring[threadIdx.x >> 6], r1, r2);
    if (!valid) return;
  }
  __builtin_nontemporal_store(r1, h1 + i);
  if constexpr (H2) __builtin_nontemporal_store(r2, h2 + i);
  if constexpr (EPI) bucket_emit(bp, i, r1);
}

// ---------------------------------------------------------------------------
// Fixed-length keys of a multiple of 128 bytes from a 128-aligned base (BASELINE
// config 5, 4 KiB): one lane per key; the keys are DMA'd into a per-wave LDS ring of two
// rounds, round q = bytes [128 q, 128 q + 128) of every lane's key (a whole line; 8 KiB
// per round), the next round in flight while the wave hashes the current one.  No VGPR
// transit (global_load_lds), no per-chunk address math (chunks are 16-aligned, so none
// straddles a round).
//
// Instruction i of a round loads the pieces of lanes 8i .. 8i+7: lane t fetches piece
// ((t % 8) + rot_L) % 8 of lane L = 8i + t/8, rot_L = (L/2) % 8, into LDS byte 1024 i +
// 16 t.  Lane L's round then sits at (L/8)*1024 + (L%8)*128 with piece j at position
// (j - rot_L) % 8, and when all lanes read piece j together the 16 lanes of each
// ds_read_b128 pass hit 16 distinct 4-bank groups (the row offset (L%8)*128 takes two
// bank phases, the rotation the other eight).
//
// The round loop issues no VALU besides the hash (round 3; the round-2 form spent 21 per
// round, 3 per chunk, on addresses and copies): a round's DMAs are an SGPR base + the
// lane's fixed 32-bit offsets (line_dma8), the LDS reads fixed per-lane addresses with the
// slot as the immediate offset (the loop unrolled over the two slots), and the state and
// the mad64 zero half stay pinned in v48-v50 across the loop.
//
// Wait invariant: the only vector-memory operations a wave issues inside the round loop
// are its DMA loads (8 per round, in order) -- no stores, no other loads -- so
// `s_waitcnt vmcnt(8)` after issuing round q+1 means exactly "rounds <= q have landed".
// The hash stores come after the loop.  tests/test_kernel_source.py checks the loop body
// for stores.
// ---------------------------------------------------------------------------
template <bool H2, bool EPI = false>
__global__ __launch_bounds__(64) void fnv_fixed_lines_kernel(const uint8_t* __restrict__ base, uint64_t key_len,
                                                             uint64_t n, uint64_t seed, uint64_t* __restrict__ h1,
                                                             uint64_t* __restrict__ h2, BucketParams bp = {}) {
  constexpr uint32_t RB = 128, NP = 8, SLOT = 64 * RB;
  __shared__ __attribute__((aligned(1024))) uint8_t ring[2 * SLOT];
  const uint32_t t = threadIdx.x;
  const uint64_t key0 = (uint64_t)blockIdx.x * 64u;
  const uint32_t last = (uint32_t)(n - key0 < 64u ? n - key0 - 1 : 63u);  // highest lane holding a key
  const uint32_t R = (uint32_t)(key_len / RB);                            // rounds per key (>= 1)
  const uint32_t kl = (uint32_t)key_len;                                  // 64 * key_len < 2^32 (host check)

  uint32_t voff[NP];
#pragma unroll
  for (uint32_t i = 0; i < NP; ++i) {
    const uint32_t L = 8u * i + t / NP;
    const uint32_t piece = ((t % NP) + (L / 2u) % NP) % NP;
    voff[i] = (L < last ? L : last) * kl + 16u * piece;  // lanes past the end re-read the last key
  }
  const uint32_t rot = (t / 2u) % NP;
  const uint32_t rb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)ring;
  const uint32_t rowb = rb + (t / 8u) * 1024u + (t % 8u) * RB;
  uint32_t a[NP];
#pragma unroll
  for (uint32_t j = 0; j < NP; ++j) a[j] = rowb + 16u * ((j + NP - rot) % NP);
  const uint64_t wbase = (uint64_t)(uintptr_t)(base + key0 * key_len);
  auto issue = [&](uint32_t q, uint32_t slot) {  // round q into slot (wave-uniform source base)
    const uint64_t s = wbase + (uint64_t)RB * q;
    // (readfirstlane returns int: each half goes through uint32_t so the low one is not
    // sign-extended into the high one)
    const uint64_t src = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(s >> 32)) << 32) |
                         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)s);
    line_dma8(src, rb + slot * SLOT, voff);
  };

  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2 = lo, hi2 = hi, z = 0;
  issue(0, 0);
  uint32_t q = 0;
  for (; q + 2 < R; q += 2) {  // rounds q (slot 0) and q+1 (slot 1), neither the key's last
    asm volatile("" ::: "memory");
    issue(q + 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // round q has landed (invariant above)
    fnv_lds_round8o<0>(lo, hi, z, a);
    asm volatile("" ::: "memory");  // slot 0's reads completed inside that statement
    issue(q + 2, 0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    fnv_lds_round8o<SLOT>(lo, hi, z, a);
  }
  asm volatile("" ::: "memory");
  if (q + 1 < R) {  // two rounds left: q (slot 0), then the last, q+1 (slot 1)
    issue(q + 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    fnv_lds_round8o<0>(lo, hi, z, a);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fnv_lds_round8o_last<SLOT>(lo, hi, z, lo2, hi2, a);  // the state before the key's final byte
  } else {  // one round left: q, the last (slot 0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fnv_lds_round8o_last<0>(lo, hi, z, lo2, hi2, a);
  }
  if (t > last) return;
  const uint64_t i = key0 + t;
  const uint64_t r1 = pack2(lo, hi);
  __builtin_nontemporal_store(r1, h1 + i);
  if constexpr (H2) __builtin_nontemporal_store(pack2(lo2, hi2), h2 + i);
  if constexpr (EPI) bucket_emit(bp, i, r1);
}

// S_p = seed * P^-p mod 2^64, p = 0..15 (P = 1099511628211 is odd, so invertible).
SpadTable make_spad(uint64_t seed) {
  const uint64_t P = 1099511628211ULL;
  uint64_t inv = P;  // Newton: inv = inv * (2 - P*inv); P*P = 1 mod 8, 5 doublings reach 64 bits
  for (int i = 0; i < 6; ++i) inv *= 2 - P * inv;
  SpadTable t;
  uint64_t s = seed;
  for (int p = 0; p < 16; ++p) {
    t.v[p] = s;
    s *= inv;
  }
  return t;
}

hipError_t launch_csr_tile(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                           uint64_t* h2, hipStream_t stream, const BucketParams* bp) {
  const SpadTable t = make_spad(seed);
  const unsigned g = (unsigned)((n + kTileKeys - 1) / kTileKeys);
  const uint8_t* b = (const uint8_t*)bytes;
  const BucketParams none{};
  if (bp) {
    if (h2) fnv_csr_staged_kernel<true, true><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2, *bp);
    else fnv_csr_staged_kernel<false, true><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, *bp);
  } else {
    if (h2) fnv_csr_staged_kernel<true, false><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2, none);
    else fnv_csr_staged_kernel<false, false><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, none);
  }
  return hipGetLastError();
}

bool fixed_lines_ok(const void* keys, uint64_t key_len) {
  return key_len >= 128 && (key_len & 127u) == 0 && ((uintptr_t)keys & 127u) == 0 && key_len < (1ull << 26);
}

// Long fixed-length keys: multiples of 128 B at a 128-aligned base take the line-DMA
// kernel, other keys of >= 128 B the cooperative line ring, shorter ones (33-127 B)
// per-lane direct loads.
hipError_t launch_fixed_long(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1,
                             uint64_t* h2, hipStream_t stream, const BucketParams* bp) {
  const uint8_t* k = (const uint8_t*)keys;
  if (fixed_lines_ok(keys, key_len)) {  // 2 rounds of whole 128-byte lines per lane in the LDS ring
    const unsigned g = (unsigned)((n + 63) / 64);
    if (bp) {
      if (h2) fnv_fixed_lines_kernel<true, true><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, h2, *bp);
      else fnv_fixed_lines_kernel<false, true><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr, *bp);
    } else {
      if (h2) fnv_fixed_lines_kernel<true><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, h2);
      else fnv_fixed_lines_kernel<false><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
    }
    return hipGetLastError();
  }
  const SpadTable t = make_spad(seed);
  const unsigned g = (unsigned)((n + 255) / 256);
  const BucketParams none{};
  const BucketParams& p = bp ? *bp : none;
  if (key_len < 128) {  // per-lane direct loads
    if (bp) {
      if (h2) fnv_fixed_long_kernel<true, true, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, h2, p);
      else fnv_fixed_long_kernel<false, true, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, nullptr, p);
    } else {
      if (h2) fnv_fixed_long_kernel<true, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, h2);
      else fnv_fixed_long_kernel<false, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, nullptr);
    }
  } else {  // the cooperative line ring
    if (bp) {
      if (h2) fnv_fixed_long_kernel<true, false, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, h2, p);
      else fnv_fixed_long_kernel<false, false, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, nullptr, p);
    } else {
      if (h2) fnv_fixed_long_kernel<true, false><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, h2);
      else fnv_fixed_long_kernel<false, false><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, nullptr);
    }
  }
  return hipGetLastError();
}

}  // namespace k2h
