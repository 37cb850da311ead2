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
//     keys, counting-sorts them in LDS by chunk count, and each wave hashes groups of 64
//     keys of (nearly) the same chunk count.
//  3. The line ring (ring_hash).  Per-lane loads of 16 B at 64 scattered keys, or even
//     cooperative loads of 80-byte windows that straddle 128-byte lines, run at 2-3 TB/s
//     on MI355X (tools/stream_floor2.hip).  Instead every lane's key is streamed as whole
//     128-byte-aligned lines: each round the wave loads one line per lane cooperatively
//     (8 lanes x 16 B per line, 8 full lines per load instruction -- 5.7 TB/s in the same
//     probe) into a 2-line LDS ring per lane, and the lane reads its next 8 chunks from
//     the ring at its own byte offset.  A line is only ever loaded if it holds a byte of
//     some key, so no load can leave the buffer's pages and no bounds checks are needed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

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

[[maybe_unused]] __device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    uint32_t o = (uint32_t)__shfl_xor((int)v, d, 64);
    v = o < v ? o : v;
  }
  return v;
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
// Direct per-lane walker (A/B variant kVariantDirect): each lane loads its own chunks.
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

// Hash key [s, e) whose bytes are staged in LDS at `lds + (x - tile_base)` for every
// byte address x of the tile (lds has 16 readable bytes below its start for chunk 0's
// pad).  Chunk reads are unaligned ds_read_b128.
template <int WALK>  // 1: one chunk per statement (default), 0: uniform asm run + divergent tail, 2: pairs
__device__ __forceinline__ void lds_hash(bool valid, uint64_t s, uint64_t e, uint64_t tile_base, const uint8_t* lds,
                                         const uint64_t* spad, uint64_t& r1, uint64_t& r2) {
  uint64_t len = valid ? e - s : 0;
  uint32_t k = (uint32_t)((len + 15) >> 4);
  uint32_t p = (uint32_t)(16u * k - len);
  // idle / empty-key lanes walk from the stage start (harmless reads, result discarded)
  const uint8_t* cp = k ? lds + (int64_t)(e - 16ull * k - tile_base) : lds;
  if constexpr (WALK == 3) cp = (const uint8_t*)((uintptr_t)cp & ~(uintptr_t)15);  // timing probe: aligned reads
  uint64_t st = spad[p & 15u];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2 = lo, hi2 = hi;
  // chunk j of the key is at cp + 16 j; body chunks 0..k-2, then the last chunk k-1
  // takes the snapshot for the second hash
  uint4 c0 = mask_lead(ld16(cp), p);
  uint32_t j = 0;
  if constexpr (WALK == 0) {
    // body chunks every lane has: a wave-uniform asm run
    uint32_t kmin = wave_min(k ? k : 0xffffffffu);
    if (kmin != 0xffffffffu && kmin >= 2) {
      uint32_t run = __builtin_amdgcn_readfirstlane(kmin - 1);
      fnv_lds_run(lo, hi, c0, (uint32_t)(uintptr_t)(cp + 16), run);
      j = run;
    }
  }
  if constexpr (WALK == 2) {
    for (; j + 2 < k; j += 2) {
      uint4 c1 = ld16(cp + 16u * (j + 1)), c2 = ld16(cp + 16u * (j + 2));
      fnv_chunk32(lo, hi, c0, c1);
      c0 = c2;
    }
  }
  // two chunks per trip, alternating register banks (no copies between the read of
  // the next chunk and its hash); the read for the chunk after is in flight meanwhile
  // (a lane may stop after either half, so a wave whose lanes differ by one chunk still
  // costs max(k) - 1 body chunks; the last chunk is then in c1 or c0)
  uint4 c1 = c0;
  bool odd = false;
  for (; j + 1 < k; j += 2) {
    c1 = ld16(cp + 16u * (j + 1));
    fnv_chunk16<0>(lo, hi, c0);
    if (j + 2 >= k) {
      odd = true;
      break;
    }
    c0 = ld16(cp + 16u * (j + 2));
    fnv_chunk16<1>(lo, hi, c1);
  }
  if (odd) c0 = c1;
  fnv_chunk16_last(lo, hi, lo2, hi2, c0);
  if (k == 0) {
    r1 = r2 = 0;
    return;
  }
  r1 = pack2(lo, hi);
  r2 = len == 1 ? r1 : pack2(lo2, hi2);
}

constexpr int kTileKeys = 512;
constexpr int kBins = 256;
// LDS image of a whole tile's bytes (staged mode).  Sized so two 256-thread blocks fit a
// CU (160 KiB) and a tile of 512 keys of BASELINE config 3 (8-256 B, mean 132 B: 67.6 KB
// per tile, sd 1.7 KB) fits with > 99 % probability; larger tiles take the ring path.
constexpr int kStageBytes = 73 * 1024;
union TileLds {
  Ring ring[4];
  uint8_t stage[16 + kStageBytes];
};

// Sort class of a key: its chunk count for up to 127 chunks (2032 B), then 4
// sub-classes per octave of chunk count.
__device__ __forceinline__ uint32_t len_bin(uint64_t len) {
  if (len == 0) return 0;
  uint64_t k = (len + 15) >> 4;
  if (k < 128) return (uint32_t)k;
  uint32_t lg = 63u - (uint32_t)__clzll((long long)k);  // >= 7
  uint32_t b = 128u + (lg - 7u) * 4u + (uint32_t)((k >> (lg - 2u)) & 3u);
  return b < (uint32_t)kBins ? b : (uint32_t)kBins - 1u;
}

}  // namespace

// ---------------------------------------------------------------------------
// CSR: one 256-thread block per tile of 512 keys.
// ---------------------------------------------------------------------------
enum {
  kModeStaged = 0, kModeDirect = 1, kModeRing = 2, kModeStagedPairs = 3, kModeStagedSingle = 4, kModeStagedProf = 5,
  kModeLean256 = 6, kModeLean512x8 = 7, kModeLean512x4 = 8, kModeLeanAlignProbe = 9, kModeLeanRing = 10,
  kModeLean2Ring = 11, kModeLean2Pin = 12, kModeLean2Step = 13, kModeLean2Group = 14,
  kModePair2 = 15, kModePair2P = 16, kModePair4P = 17, kModePair4 = 18, kModePair4PS = 19, kModePair2PS = 20, kModePair4W2 = 21, kModePair4Z = 22, kModeLean2Clock = 23,
  kModeDbuf = 24, kModeDbufProbeNoHash = 25, kModeDbufProbeNoFeed = 26, kModeQueue = 27,
  kModeQueueProbeNoHash = 28, kModeQueueProbeNoFeed = 29, kModeQueuePrio = 30,
  kModeLean2Prio = 31, kModeLean2Prio3 = 32, kModeLean2Prio1 = 33, kModeLean2Scan1 = 34, kModeLean2Runs = 35, kModeLean3 = 36, kModeLean2Desync1 = 37, kModeLean2Desync2 = 38, kModeQueue320 = 39, kModeLean2PrioSetup = 40, kModeLean2Ballot = 41
};

// Phase stamps of the profiling mode (kModeStagedProf; tools/csr_phases.py): 100 MHz
// wall clock per block at the phase boundaries, and each wave's finish time.
#define K2H_PROF_STAMP(SLOT)                                                               \
  if constexpr (MODE == kModeStagedProf) {                                                 \
    if (tid == 0) prof[(uint64_t)blockIdx.x * 16u + (SLOT)] = __builtin_amdgcn_s_memrealtime(); \
  }

template <bool H2, int MODE, bool EPI, int TK = kTileKeys>
__device__ __forceinline__ void csr_tile(uint64_t tile, const uint8_t* __restrict__ bytes,
                                         const uint64_t* __restrict__ offsets, uint64_t n, const SpadTable& spad_tab,
                                         uint64_t* __restrict__ h1, uint64_t* __restrict__ h2, const BucketParams& bp) {
  __shared__ uint64_t s_off[TK + 1];
  __shared__ uint16_t s_order[TK];
  __shared__ uint32_t s_hist[kBins];
  __shared__ uint32_t s_wsum[4];
  __shared__ uint64_t s_spad[16];
  __shared__ TileLds s_u;

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint64_t t0 = tile * TK;
  uint64_t* const prof = h2;  // profiling mode only: h2 is the stamp buffer (16 per block)
  (void)prof;
  K2H_PROF_STAMP(0)
  const uint32_t cnt = (uint32_t)(n - t0 < (uint64_t)TK ? n - t0 : (uint64_t)TK);
  const uint8_t* lo_bound = bytes + offsets[0];
  const uint64_t safe = (uint64_t)(uintptr_t)lo_bound & ~127ull;

  if (tid < 16) s_spad[tid] = spad_tab.v[tid];
  for (uint32_t k = tid; k <= cnt; k += 256) s_off[k] = offsets[t0 + k];
  s_hist[tid] = 0;
  __syncthreads();
  K2H_PROF_STAMP(1)

  // staged mode: DMA the tile's whole byte span into LDS (lane-linear 1 KiB pieces,
  // no registers), in flight while the tile is sorted
  const uint64_t span_lo = ((uint64_t)(uintptr_t)bytes + s_off[0]) & ~15ull;
  const uint64_t span_hi = (uint64_t)(uintptr_t)bytes + s_off[cnt];
  const bool staged = (MODE == kModeStaged || MODE == kModeStagedPairs || MODE == kModeStagedSingle ||
                       MODE == kModeStagedProf) &&
                      span_hi - span_lo <= (uint64_t)kStageBytes;
  if (staged) {
    // a tile of empty keys has no bytes to stage (and `bytes` need not point anywhere)
    const uint32_t npieces = s_off[cnt] > s_off[0] ? (uint32_t)((span_hi - span_lo + 1023) >> 10) : 0u;
    for (uint32_t c = wave; c < npieces; c += 4) {
      uint64_t src = span_lo + 1024ull * c + 16u * lane;
      if (src >= span_hi) src = span_lo;  // past the span's last 16-byte piece: re-read a safe one
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(uintptr_t)src,
                                       (__attribute__((address_space(3))) void*)(s_u.stage + 16 + 1024u * c), 16, 0,
                                       0);
    }
  }

  K2H_PROF_STAMP(10)
  // 1. histogram of length classes
  constexpr int KPT = (TK + 255) / 256;  // keys per thread (TK need not be a multiple of 256)
  uint32_t bins[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    uint32_t k = tid + 256u * j;
    if (k < cnt) {
      bins[j] = len_bin(s_off[k + 1] - s_off[k]);
      lds_add(&s_hist[bins[j]], 1u);
    }
  }
  lds_barrier();
  K2H_PROF_STAMP(11)
  // 2. exclusive scan of the 256 class counts (one per thread)
  uint32_t v = s_hist[tid], incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  if (lane == 63) s_wsum[wave] = incl;
  lds_barrier();
  uint32_t base = 0;
  for (uint32_t w = 0; w < wave; ++w) base += s_wsum[w];
  s_hist[tid] = base + incl - v;  // becomes the scatter cursor
  lds_barrier();
  K2H_PROF_STAMP(12)
  // 3. scatter key indices in class order
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    uint32_t k = tid + 256u * j;
    if (k < cnt) s_order[lds_add_rtn(&s_hist[bins[j]], 1u)] = (uint16_t)k;
  }
  lds_barrier();
  // 4. each wave hashes groups of 64 class-sorted keys; results go straight to global
  //    (scattered 8-byte stores within the tile's 4 KiB output run merge in L2)
  K2H_PROF_STAMP(2)
  if (staged) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces have landed
    __syncthreads();                                   // ... and every other wave's
  }
  K2H_PROF_STAMP(3)
  // Groups are in length order, so wave w takes groups w, 7-w, 8+w, 15-w, ... (snake):
  // every wave gets the same total work and the block's waves finish together.  (Rotating
  // the start by block, as the lean kernel does, measured 8 % slower here.)
  const uint32_t ngroups = (cnt + 63u) >> 6;
  for (uint32_t it = 0; it * 4 < ngroups; ++it) {
    uint32_t g = it * 4 + ((it & 1) ? 3 - wave : wave);
    if (g >= ngroups) continue;
    uint32_t idx = g * 64u + lane;
    bool valid = idx < cnt;
    uint32_t k = s_order[valid ? idx : cnt - 1];
    uint64_t r1 = 0, r2 = 0;
    if constexpr (MODE == kModeDirect) {
      if (valid) hash_key(bytes + s_off[k], bytes + s_off[k + 1], lo_bound, s_spad, r1, r2);
    } else {
      if (staged)
        lds_hash<MODE == kModeStagedSingle ? 0 : MODE == kModeStagedPairs ? 2 : 1>(valid, (uint64_t)(uintptr_t)bytes + s_off[k], (uint64_t)(uintptr_t)bytes + s_off[k + 1], span_lo,
                 s_u.stage + 16, s_spad, r1, r2);
      else
        ring_hash(valid, bytes + s_off[k], bytes + s_off[k + 1], safe, s_spad, s_u.ring[wave], r1, r2);
    }
    if (valid) {
      h1[t0 + k] = r1;
      if constexpr (H2) h2[t0 + k] = r2;
      if constexpr (EPI) bucket_emit<false>(bp, t0 + k, r1);
    }
  }
  if constexpr (MODE == kModeStagedProf) {
    if (lane == 0) {
      uint32_t hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      prof[(uint64_t)blockIdx.x * 16u + 4u + wave] = __builtin_amdgcn_s_memrealtime();
      if (wave == 0) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        prof[(uint64_t)blockIdx.x * 16u + 8u] = ((uint64_t)xcc << 32) | hw;
        prof[(uint64_t)blockIdx.x * 16u + 9u] = staged;
      }
    }
  }
}

template <bool H2, int MODE, bool EPI = false>
__global__ __launch_bounds__(256) void fnv_csr_tile_kernel(const uint8_t* __restrict__ bytes,
                                                           const uint64_t* __restrict__ offsets, uint64_t n,
                                                           SpadTable spad_tab, uint64_t* __restrict__ h1,
                                                           uint64_t* __restrict__ h2, BucketParams bp = {}) {
  csr_tile<H2, MODE, EPI>(blockIdx.x, bytes, offsets, n, spad_tab, h1, h2, bp);
}

// The tiles listed by the lean kernel as too large for its stage (tile_list[0 ..
// *tile_count)), each hashed with the line ring; a grid-stride loop, since the count is
// only known on the device.
template <bool H2, bool EPI = false, int TK = kTileKeys>
__global__ __launch_bounds__(256) void fnv_csr_ring_list_kernel(const uint8_t* __restrict__ bytes,
                                                                const uint64_t* __restrict__ offsets, uint64_t n,
                                                                SpadTable spad_tab, uint64_t* __restrict__ h1,
                                                                uint64_t* __restrict__ h2,
                                                                const uint32_t* __restrict__ tile_list,
                                                                const uint32_t* __restrict__ tile_count,
                                                                BucketParams bp = {}) {
  const uint32_t count = *tile_count;
  for (uint32_t li = blockIdx.x; li < count; li += gridDim.x) {
    csr_tile<H2, kModeRing, EPI, TK>(tile_list[li], bytes, offsets, n, spad_tab, h1, h2, bp);
    __syncthreads();  // the next tile reuses the shared arrays
  }
}

// ---------------------------------------------------------------------------
// CSR, lean staged tiles: TK keys per block of NW waves, the tile's bytes DMA'd into
// an LDS stage of STAGE_KIB KiB with no line-ring union, so that several blocks fit a
// CU (4 x 256-key tiles at 36 KiB: four tiles in flight per CU, one loading / sorting
// while the others hash -- the 512-key kernel above fits two, and a tile spends about
// half its life in latency-bound load / sort / DMA phases, tools/csr_phases.py).
// Oversize tiles (span > stage) hash with per-lane direct loads.  Length classes are
// 128 bins (exact chunk counts below 96).  Wave w of block b takes sorted groups
// starting from (w + b) mod NW, snaking, so short and long groups spread over SIMDs.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t len_bin128(uint64_t len) {
  if (len == 0) return 0;
  uint64_t k = (len + 15) >> 4;
  if (k < 96) return (uint32_t)k;
  uint32_t lg = 63u - (uint32_t)__clzll((long long)k);  // >= 6
  uint32_t b = 96u + (lg - 6u) * 4u + (uint32_t)((k >> (lg - 2u)) & 3u);
  return b < 128u ? b : 127u;
}

// over_list / over_count (default path): a tile whose span exceeds the stage is not
// hashed here but appended to over_list, for fnv_csr_ring_list_kernel; without a list
// such tiles hash with per-lane direct loads (A/B variants).
template <bool H2, int TK, int NW, int STAGE_KIB, int WALK = 1, bool EPI = false>
__global__ __launch_bounds__(NW * 64) void fnv_csr_lean_kernel(const uint8_t* __restrict__ bytes,
                                                               const uint64_t* __restrict__ offsets, uint64_t n,
                                                               SpadTable spad_tab, uint64_t* __restrict__ h1,
                                                               uint64_t* __restrict__ h2,
                                                               uint32_t* __restrict__ over_list = nullptr,
                                                               uint32_t* __restrict__ over_count = nullptr,
                                                               BucketParams bp = {}) {
  constexpr int NT = NW * 64;
  constexpr int NB = 128;
  constexpr uint32_t kStage = STAGE_KIB * 1024u;
  static_assert(NT >= NB, "one thread per length class in the scan");
  __shared__ uint64_t s_off[TK + 1];
  __shared__ uint16_t s_order[TK];
  __shared__ uint32_t s_hist[NB];
  __shared__ uint32_t s_wsum[NW];
  __shared__ uint64_t s_spad[16];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[16 + kStage];

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint64_t t0 = (uint64_t)blockIdx.x * TK;
  const uint32_t cnt = (uint32_t)(n - t0 < (uint64_t)TK ? n - t0 : (uint64_t)TK);
  const uint8_t* lo_bound = bytes + offsets[0];

  if (tid < 16) s_spad[tid] = spad_tab.v[tid];
  for (uint32_t k = tid; k <= cnt; k += NT) s_off[k] = offsets[t0 + k];
  if (tid < NB) s_hist[tid] = 0;
  __syncthreads();

  const uint64_t span_lo = ((uint64_t)(uintptr_t)bytes + s_off[0]) & ~15ull;
  const uint64_t span_hi = (uint64_t)(uintptr_t)bytes + s_off[cnt];
  const bool staged = span_hi - span_lo <= (uint64_t)kStage;
  if (!staged && over_list) {  // block-uniform
    if (tid == 0) over_list[atomicAdd(over_count, 1u)] = blockIdx.x;
    return;
  }
  if (staged) {
    const uint32_t npieces = s_off[cnt] > s_off[0] ? (uint32_t)((span_hi - span_lo + 1023) >> 10) : 0u;
    for (uint32_t c = wave; c < npieces; c += NW) {
      uint64_t src = span_lo + 1024ull * c + 16u * lane;
      if (src >= span_hi) src = span_lo;
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(uintptr_t)src,
                                       (__attribute__((address_space(3))) void*)(s_stage + 16 + 1024u * c), 16, 0, 0);
    }
  }
  constexpr int KPT = (TK + NT - 1) / NT;
  uint32_t bins[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    uint32_t k = tid + NT * j;
    if (k < cnt) {
      bins[j] = len_bin128(s_off[k + 1] - s_off[k]);
      lds_add(&s_hist[bins[j]], 1u);
    }
  }
  lds_barrier();
  uint32_t v = tid < NB ? s_hist[tid] : 0u, incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  if (lane == 63) s_wsum[wave] = incl;
  lds_barrier();
  uint32_t base = 0;
  for (uint32_t w = 0; w < wave; ++w) base += s_wsum[w];
  if (tid < NB) s_hist[tid] = base + incl - v;
  lds_barrier();
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    uint32_t k = tid + NT * j;
    if (k < cnt) s_order[lds_add_rtn(&s_hist[bins[j]], 1u)] = (uint16_t)k;
  }
  if (staged) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const uint32_t ngroups = (cnt + 63u) >> 6;
  const uint32_t wr = (wave + blockIdx.x) % NW;
  for (uint32_t it = 0; it * NW < ngroups; ++it) {
    uint32_t g = it * NW + ((it & 1) ? NW - 1 - wr : wr);
    if (g >= ngroups) continue;
    uint32_t idx = g * 64u + lane;
    bool valid = idx < cnt;
    uint32_t k = s_order[valid ? idx : cnt - 1];
    uint64_t r1 = 0, r2 = 0;
    if (staged) {
      lds_hash<WALK>(valid, (uint64_t)(uintptr_t)bytes + s_off[k], (uint64_t)(uintptr_t)bytes + s_off[k + 1], span_lo,
                     s_stage + 16, s_spad, r1, r2);
    } else if (valid) {
      hash_key(bytes + s_off[k], bytes + s_off[k + 1], lo_bound, s_spad, r1, r2);
    }
    if (valid) {
      h1[t0 + k] = r1;
      if constexpr (H2) h2[t0 + k] = r2;
      if constexpr (EPI) bucket_emit<false>(bp, t0 + k, r1);
    }
  }
}

// ---------------------------------------------------------------------------
// CSR lean tiles, trimmed of non-hash VALU work (the kernel is bound by its VALU
// instruction count): 32-bit tile-relative offsets in LDS, a DMA
// loop with one 32-bit clamp per piece and a wave-uniform trip count, and the chunk-0
// lead mask from a 16-entry table.  Same tile
// shape as fnv_csr_lean_kernel<512, 4, 72>; oversize tiles go to the ring list.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t len_bin128_32(uint32_t len) {
  if (len == 0) return 0;
  uint32_t k = (len + 15u) >> 4;
  if (k < 96) return k;
  uint32_t lg = 31u - (uint32_t)__clz((int)k);  // >= 6
  uint32_t b = 96u + (lg - 6u) * 4u + ((k >> (lg - 2u)) & 3u);
  return b < 128u ? b : 127u;
}

// Key [rs, re) of the tile (byte offsets relative to the tile's first key byte, which
// sits at `key0` in LDS; 16 readable bytes precede the stage for chunk 0's pad).
template <bool PIN>
__device__ __forceinline__ void lds_hash32(bool valid, uint32_t rs, uint32_t re, const uint8_t* key0,
                                           const uint64_t* spad, const uint4* masks, uint64_t& r1,
                                           uint64_t& r2) {
  const uint32_t len = valid ? re - rs : 0u;
  const uint32_t k = (len + 15u) >> 4;
  const uint32_t p = (0u - len) & 15u;
  const uint8_t* cp = key0 + (int32_t)(re - 16u * k);  // chunk 0 (idle lanes: harmless reads)
  const uint64_t st = spad[p];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2 = lo, hi2 = hi;
  const uint4 m = masks[p];
  uint4 c0 = ld16(cp);
  c0 = make_uint4(c0.x & m.x, c0.y & m.y, c0.z & m.z, c0.w & m.w);
  // PIN (A/B): pin the chunk registers to the asm banks (v[40:43] / v[44:47]) so the LDS
  // reads land there directly -- but the pin waits for each read (lgkmcnt(0)) right
  // after issuing it, which costs more than the copies it saves
  auto pin0 = [](uint4& c) {
    if constexpr (PIN) asm volatile("" : "+{v40}"(c.x), "+{v41}"(c.y), "+{v42}"(c.z), "+{v43}"(c.w));
  };
  auto pin1 = [](uint4& c) {
    if constexpr (PIN) asm volatile("" : "+{v44}"(c.x), "+{v45}"(c.y), "+{v46}"(c.z), "+{v47}"(c.w));
  };
  pin0(c0);
  uint4 c1 = c0;
  bool odd = false;
  for (uint32_t j = 0; j + 1 < k; j += 2) {
    c1 = ld16(cp + 16u * (j + 1));
    pin1(c1);
    fnv_chunk16<0>(lo, hi, c0);
    if (j + 2 >= k) {
      odd = true;
      break;
    }
    c0 = ld16(cp + 16u * (j + 2));
    pin0(c0);
    fnv_chunk16<1>(lo, hi, c1);
  }
  if (odd) c0 = c1;
  fnv_chunk16_last(lo, hi, lo2, hi2, c0);
  if (k == 0) {
    r1 = r2 = 0;
    return;
  }
  r1 = pack2(lo, hi);
  r2 = len == 1 ? r1 : pack2(lo2, hi2);
}

// The same walk with the chunk registers held in the asm banks across the loop
// (fnv_step_read: each step hashes one bank while its asm reads the next chunk into the
// other): no copies in the loop (≈3 fewer VALU ops per chunk), yet 3 % slower than the
// compiler-scheduled walk in A/B (variant 53), so it is not the default.
__device__ __forceinline__ void lds_hash32s(bool valid, uint32_t rs, uint32_t re, const uint8_t* key0,
                                            const uint64_t* spad, const uint4* masks, uint64_t& r1, uint64_t& r2) {
  const uint32_t len = valid ? re - rs : 0u;
  const uint32_t k = (len + 15u) >> 4;
  const uint32_t p = (0u - len) & 15u;
  const uint8_t* cp = key0 + (int32_t)(re - 16u * k);
  const uint64_t st = spad[p];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2 = lo, hi2 = hi;
  const uint4 m = masks[p];
  uint4 a = ld16(cp);
  a = make_uint4(a.x & m.x, a.y & m.y, a.z & m.z, a.w & m.w);
  fnv_bank0_pin(a);
  uint4 b = a;
  const uint32_t a0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint8_t*)cp;
  bool from1 = false;
  for (uint32_t j = 0; j + 1 < k; j += 2) {
    fnv_step_read<0>(lo, hi, a, b, a0 + 16u * (j + 1));
    if (j + 2 >= k) {
      from1 = true;
      break;
    }
    fnv_step_read<1>(lo, hi, a, b, a0 + 16u * (j + 2));
  }
  fnv_step_last(lo, hi, lo2, hi2, a, b, from1);
  if (k == 0) {
    r1 = r2 = 0;
    return;
  }
  r1 = pack2(lo, hi);
  r2 = len == 1 ? r1 : pack2(lo2, hi2);
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
// that only the lanes switching at that step take.  Returns the two h1 values.
template <bool Z = false>
__device__ __forceinline__ void pair_walk(uint32_t k0, uint32_t p0, const uint8_t* cp0, uint32_t k1, uint32_t p1,
                                          const uint8_t* cp1, const uint64_t* spad, const uint4* masks,
                                          uint64_t& h0, uint64_t& h1v) {
  const uint32_t T = k0 + k1, sw = k0;
  uint64_t st = spad[p0];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), z = 0;  // Z: the mad64 zero half kept in v50
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
      if constexpr (Z) fnv_chunk16z<0>(lo, hi, c0, z);
      else fnv_chunk16<0>(lo, hi, c0);
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
      if constexpr (Z) fnv_chunk16z<1>(lo, hi, c1, z);
      else fnv_chunk16<1>(lo, hi, c1);
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
  if constexpr (Z) fnv_chunk16z<0>(lo, hi, c0, z);  // the last chunk of the lane's last key
  else fnv_chunk16<0>(lo, hi, c0);
  if (k1) {
    h0 = saved;
    h1v = pack2(lo, hi);
  } else {
    h0 = pack2(lo, hi);
    h1v = 0;
  }
}

// Uniform-trip pair walk (round 2; A/B variant 68, measured slower than pair_walk: the end
// event needs the same branch as the switch, and its state copies cost more VALU than the
// per-step compares it saves -- SQ_INSTS_VALU 1.026e9 vs 0.994e9).  Every lane runs tmax = max over the wave of k0 + k1
// chunk steps; chunk t of the lane's sequence (key 0's chunks, then key 1's) is read at
// base + 16 t, the next one in flight under the current one's hash, the chunk registers
// alternating between the two asm banks.  One compare per step against the lane's next
// event -- the end of key 0 (save it, restart from key 1's S_p with its masked chunk 0)
// or the end of key 1 (save it) -- in a branch only the lanes at that event take.  Lanes
// past their end re-read the stage start (results dropped).  Outside the hash: the address
// add and the compare per chunk, and the zero half of the mad64 addend pair stays in v50
// across the loop (pair_walk: ~5 VALU per chunk and an exec-mask dance per step).
__device__ __forceinline__ void pair_walk2(uint32_t k0, uint32_t p0, const uint8_t* cp0, uint32_t k1, uint32_t p1,
                                           const uint8_t* cp1, const uint8_t* safe, const uint64_t* spad,
                                           const uint4* masks, uint64_t& h0, uint64_t& h1v) {
  const uint32_t T = k0 + k1;
  const uint32_t tmax = __builtin_amdgcn_readfirstlane(wave_max(T));
  h0 = 0;
  h1v = 0;
  if (tmax == 0) return;
  uint64_t st = spad[p0];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), z = 0;
  const uint8_t* base = T ? cp0 : safe;
  uint32_t ev = T ? k0 : 0xFFFFFFFFu;  // next event: end of key 0, then of key 1
  bool second = false;
  uint4 m = masks[p0];
  uint4 a = ld16(base);
  a = make_uint4(a.x & m.x, a.y & m.y, a.z & m.z, a.w & m.w);
  uint4 b;
  // at the end of a key (state = its hash): save it, then restart on key 1 (c becomes its
  // masked chunk 0, read from cp1) or retire the lane
  auto event = [&](uint32_t t, uint4& c) {
    if (!second) {
      h0 = ((uint64_t)hi << 32) | lo;
      if (k1) {
        second = true;
        st = spad[p1];
        lo = (uint32_t)st;
        hi = (uint32_t)(st >> 32);
        base = cp1 - 16 * (int32_t)t;
        m = masks[p1];
        c = ld16(cp1);
        c = make_uint4(c.x & m.x, c.y & m.y, c.z & m.z, c.w & m.w);
        ev = T;
        return;
      }
    } else {
      h1v = ((uint64_t)hi << 32) | lo;
    }
    ev = 0xFFFFFFFFu;
    base = safe - 16 * (int32_t)t;
  };
  for (uint32_t t = 0;; t += 2) {
    b = ld16(base + 16u * (t + 1));
    fnv_chunk16z<0>(lo, hi, a, z);
    if (t + 1 == ev) event(t + 1, b);
    if (t + 1 >= tmax) break;
    a = ld16(base + 16u * (t + 2));
    fnv_chunk16z<1>(lo, hi, b, z);
    if (t + 2 == ev) event(t + 2, a);
    if (t + 2 >= tmax) break;
  }
}

#if K2H_AMD_LAB
#include "k2h_csr_lab_walk.inc"
#endif

// CLK (lab clock probe, H2 false): h2 receives per wave the shader-clock / 100 MHz stamps
// at entry and after the hash (tools/clock_probe.py).  PRIO (lab): the load / sort phase at
// raised issue priority, back to normal for the hash walk, so a tile's setup is not queued
// behind the other block's hash instructions on the same SIMD.
// SCAN1 (lab): the 128-class scan by wave 0 alone, two classes per lane (one barrier fewer).
template <bool H2, bool EPI = false, int WALK = 0, bool CLK = false, int PRIO = 0, bool SCAN1 = false, int WALK4 = 0,
          int DESYNC = 0>
__global__ __launch_bounds__(256) void fnv_csr_lean2_kernel(const uint8_t* __restrict__ bytes,
                                                            const uint64_t* __restrict__ offsets, uint64_t n,
                                                            SpadTable spad_tab, uint64_t* __restrict__ h1,
                                                            uint64_t* __restrict__ h2, uint32_t* __restrict__ over_list,
                                                            uint32_t* __restrict__ over_count, BucketParams bp = {},
                                                            uint32_t ncu = 0) {
  constexpr uint32_t TK = 512, NW = 4, NT = 256, NB = 128;
  constexpr uint32_t kStage = 72 * 1024u;
  __shared__ uint32_t s_rel[TK + 1];
  __shared__ uint16_t s_order[TK];
  __shared__ uint32_t s_hist[NB];
  __shared__ uint32_t s_wsum[NW];
  __shared__ uint64_t s_spad[16];
  __shared__ uint4 s_mask[16];
  __shared__ __attribute__((aligned(16))) uint8_t s_stage[16 + kStage];

  uint64_t clk0 = 0, rt0 = 0;
  if constexpr (CLK) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(PRIO == 4 ? 1 : PRIO);  // 4 (lab): 1, dropped at the walk
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // DESYNC (lab; ncu = CU count): some blocks of the first wave take half tiles, so the two
  // tiles resident on a CU start half a tile apart (1: blocks [0, ncu); 2: even blocks of
  // [0, 2 ncu)).  Measured: no change (the one-shot grid's turnover already desyncs them).
  const uint64_t bx = blockIdx.x, C = ncu;
  uint64_t t0 = bx * TK;
  uint32_t tk = TK;
  if constexpr (DESYNC == 1) {
    t0 = bx < C ? bx * (TK / 2) : C * (TK / 2) + (bx - C) * TK;
    tk = bx < C ? TK / 2 : TK;
  } else if constexpr (DESYNC == 2) {
    t0 = bx < 2 * C ? (bx / 2) * (TK + TK / 2) + ((bx & 1) ? TK / 2 : 0) : C * (TK + TK / 2) + (bx - 2 * C) * TK;
    tk = (bx < 2 * C && !(bx & 1)) ? TK / 2 : TK;
  }
  const uint32_t cnt = (uint32_t)(n - t0 < (uint64_t)tk ? n - t0 : (uint64_t)tk);
  const uint64_t o0 = offsets[t0], oN = offsets[t0 + cnt];  // block-uniform
  const uint64_t kb = (uint64_t)(uintptr_t)bytes + o0;
  const uint64_t span_lo = kb & ~15ull;
  const uint32_t delta = (uint32_t)(kb & 15u);
  const uint64_t span = oN - o0 + delta;  // stage bytes up to the tile's last key byte
  if (span > kStage) {                    // block-uniform
    if (tid == 0) over_list[atomicAdd(over_count, 1u)] = blockIdx.x;
    return;
  }
  if (tid < 16) {
    s_spad[tid] = spad_tab.v[tid];
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // bytes >= p kept: chunk 0's p pad bytes zeroed
      int32_t sh = 8 * ((int32_t)tid - 4 * i);
      w[i] = sh <= 0 ? ~0u : sh >= 32 ? 0u : ~0u << sh;
    }
    s_mask[tid] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  for (uint32_t k = tid; k <= cnt; k += NT) s_rel[k] = (uint32_t)(offsets[t0 + k] - o0);
  if (tid < NB) s_hist[tid] = 0;
  __syncthreads();

  // DMA of the tile span (16-byte pieces; pieces past the span re-read its last piece
  // into stage bytes nobody reads), in flight during the sort
  if (oN > o0) {
    const uint32_t npieces = (uint32_t)((span + 1023) >> 10);
    const uint32_t lastp = ((uint32_t)span - 1u) & ~15u;
    const uint8_t* src0 = (const uint8_t*)(uintptr_t)span_lo;
    uint32_t off = 1024u * wave + 16u * lane;
    for (uint32_t c = wave; c < npieces; c += NW, off += 1024u * NW) {
      const uint32_t o = off < lastp ? off : lastp;
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src0 + o),
                                       (__attribute__((address_space(3))) void*)(s_stage + 16 + 1024u * c), 16, 0, 0);
    }
  }
  constexpr uint32_t KPT = (TK + NT - 1) / NT;
  uint32_t bins[KPT];
#pragma unroll
  for (uint32_t j = 0; j < KPT; ++j) {
    uint32_t k = tid + NT * j;
    if (k < cnt) {
      bins[j] = len_bin128_32(s_rel[k + 1] - s_rel[k]);
      lds_add(&s_hist[bins[j]], 1u);
    }
  }
  lds_barrier();
  if constexpr (SCAN1) {
    static_assert(NB == 128, "two classes per lane of wave 0");
    if (wave == 0) {
      const uint32_t v0 = s_hist[2 * lane], v1 = s_hist[2 * lane + 1], sum = v0 + v1;
      uint32_t incl = sum;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
      }
      s_hist[2 * lane] = incl - sum;
      s_hist[2 * lane + 1] = incl - sum + v0;
    }
  } else {
    uint32_t v = tid < NB ? s_hist[tid] : 0u, incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      uint32_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    if (lane == 63) s_wsum[wave] = incl;
    lds_barrier();
    uint32_t base = 0;
    for (uint32_t w = 0; w < wave; ++w) base += s_wsum[w];
    if (tid < NB) s_hist[tid] = base + incl - v;
  }
  lds_barrier();
#pragma unroll
  for (uint32_t j = 0; j < KPT; ++j) {
    uint32_t k = tid + NT * j;
    if (k < cnt) s_order[lds_add_rtn(&s_hist[bins[j]], 1u)] = (uint16_t)k;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces have landed
  __syncthreads();                                   // ... and every other wave's

  const uint8_t* key0 = s_stage + 16 + delta;
  if constexpr (PRIO && PRIO != 4) __builtin_amdgcn_s_setprio(0);
  if constexpr (WALK == 3) {
    // Pair walk: lane i (0..255) takes sorted keys i and cnt-1-i, a short and a long one,
    // and hashes them back to back; sums of the pair lengths are nearly equal across a
    // wave, so the wave's length waste drops from 10.8 % (groups of 64 equal-class keys)
    // to ~3.4 % on BASELINE config 3.
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
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(0);
#if K2H_AMD_LAB
    if constexpr (WALK4 == 1)
      pair_walk3(only_b ? kB : kA, only_b ? pB : pA, only_b ? cpB : cpA, only_b ? 0u : kB, pB, cpB, s_stage + 16,
                 s_spad, s_mask, hw0, hw1);
    else if constexpr (WALK4 == 2)
      pair_walk4(only_b ? kB : kA, only_b ? pB : pA, only_b ? cpB : cpA, only_b ? 0u : kB, pB, cpB, s_stage + 16,
                 s_spad, s_mask, hw0, hw1);
    else
#endif
      pair_walk(only_b ? kB : kA, only_b ? pB : pA, only_b ? cpB : cpA, only_b ? 0u : kB, pB, cpB, s_spad, s_mask,
                hw0, hw1);
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
    if constexpr (CLK) {
      const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
      if (lane == 0) {
        uint64_t* o = h2 + 4ull * (blockIdx.x * NW + wave);
        o[0] = clk0;
        o[1] = clk1;
        o[2] = rt0;
        o[3] = rt1;
      }
    }
    return;
  }
  const uint32_t ngroups = (cnt + 63u) >> 6;
  const uint32_t wr = (wave + blockIdx.x) % NW;
  for (uint32_t it = 0; it * NW < ngroups; ++it) {
    uint32_t g = it * NW + ((it & 1) ? NW - 1 - wr : wr);
    if (g >= ngroups) continue;
    uint32_t idx = g * 64u + lane;
    bool valid = idx < cnt;
    uint32_t k = s_order[valid ? idx : cnt - 1];
    uint64_t r1, r2;
    if constexpr (WALK == 2)
      lds_hash32s(valid, s_rel[k], s_rel[k + 1], key0, s_spad, s_mask, r1, r2);
    else
      lds_hash32<WALK == 1>(valid, s_rel[k], s_rel[k + 1], key0, s_spad, s_mask, r1, r2);
    if (valid) {
      h1[t0 + k] = r1;
      if constexpr (H2) h2[t0 + k] = r2;
      if constexpr (EPI) bucket_emit<false>(bp, t0 + k, r1);
    }
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
// config 5, 4 KiB): one lane per key; the keys are DMA'd into a per-wave LDS ring of D
// rounds, round q = bytes [RB q, RB q + RB) of every lane's key (RB = 128: a whole line,
// 64: half of one; 64 RB bytes per round), D-1 rounds in flight while the wave hashes
// the current one.  No VGPR transit (global_load_lds), no per-chunk address math
// (chunks are 16-aligned, so none straddles a round), and the DMA addresses are a
// uniform base + fixed per-lane offsets.
//
// With NP = RB/16 pieces per round and LPI = 1024/RB lanes per DMA instruction,
// instruction i of a round loads the pieces of lanes LPI i .. LPI i + LPI-1: lane t
// fetches piece ((t % NP) + rot_L) % NP of lane L = LPI i + t / NP, rot_L =
// (L / (256/RB)) % NP, into LDS byte 1024 i + 16 t.  Lane L's round then sits at
// (L / LPI)*1024 + (L % LPI)*RB with piece j at position (j - rot_L) % NP, and when all
// lanes read piece j together the 16 lanes of each ds_read_b128 pass hit 16 distinct
// 4-bank groups (the row offset (L % LPI)*RB takes 256/RB bank phases, the rotation the
// other NP).
// ---------------------------------------------------------------------------
// PROBE (timing probes only, wrong hashes): 1 = no DMA (hash whatever LDS holds),
// 2 = no hashing (DMA + waits only).
// PROBE 4 (lab, correct hashes): each round's DMA issued at raised issue priority.
template <bool H2, int D, int RB, bool EPI = false, int PROBE = 0>
__global__ __launch_bounds__(64) void fnv_fixed_lines_kernel(const uint8_t* __restrict__ base, uint64_t key_len,
                                                             uint64_t n, uint64_t seed, uint64_t* __restrict__ h1,
                                                             uint64_t* __restrict__ h2, BucketParams bp = {}) {
  constexpr uint32_t NP = RB / 16, LPI = 1024 / RB, PH = 256 / RB;
  static_assert((RB == 256 || RB == 128 || RB == 64) && D >= 2 && NP * (D - 1) <= 63,
                "vmcnt holds at most 63 loads");
  __shared__ __attribute__((aligned(1024))) uint8_t ring[D * 64 * RB];
  const uint32_t t = threadIdx.x;
  const uint64_t key0 = (uint64_t)blockIdx.x * 64u;
  const uint32_t last = (uint32_t)(n - key0 < 64u ? n - key0 - 1 : 63u);  // highest lane holding a key
  const uint32_t R = (uint32_t)(key_len / RB);                            // rounds per key (>= 1)
  const uint32_t kl = (uint32_t)key_len;                                  // 64 * key_len < 2^32 (host check)

  uint32_t voff[NP];
#pragma unroll
  for (uint32_t i = 0; i < NP; ++i) {
    uint32_t L = LPI * i + t / NP;
    uint32_t piece = ((t % NP) + (L / PH) % NP) % NP;
    voff[i] = (L < last ? L : last) * kl + 16u * piece;  // lanes past the end re-read the last key
  }
  const uint32_t rot = (t / PH) % NP;
  const uint32_t rowb = (t / LPI) * 1024u + (t % LPI) * RB;
  uint32_t pofs[NP];
#pragma unroll
  for (uint32_t j = 0; j < NP; ++j) pofs[j] = rowb + 16u * ((j + NP - rot) % NP);
  const uint8_t* wbase = base + key0 * key_len;

  auto issue = [&](uint32_t q) {
    if constexpr (PROBE == 1) return;
    uint8_t* slot = ring + (q % D) * (64u * RB);
    const uint8_t* src = wbase + (uint64_t)RB * q;
    if constexpr (PROBE == 4) __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (uint32_t i = 0; i < NP; ++i)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src + voff[i]),
                                       (__attribute__((address_space(3))) void*)(slot + 1024u * i), 16, 0, 0);
    if constexpr (PROBE == 4) __builtin_amdgcn_s_setprio(0);
  };

  uint64_t clk0 = 0, rt0 = 0;
  if constexpr (PROBE == 3) {  // clock probe: h2 receives per wave the shader-clock / 100 MHz stamps
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  for (uint32_t q = 0; q < D - 1 && q < R; ++q) issue(q);
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2 = lo, hi2 = hi;
  for (uint32_t q = 0; q < R; ++q) {
    // slot (q+D-1) % D held round q-1, whose reads completed inside the previous round's
    // asm statement (lgkmcnt(0) before its last chunk)
    asm volatile("" ::: "memory");
    if (q + D - 1 < R) {
      issue(q + D - 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NP * (D - 1)) : "memory");  // round q has landed
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // LDS reads in asm (fnv_lds_round): the compiler's own waits would drain every DMA
    const uint32_t sb = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(ring + (q % D) * (64u * RB));
    uint32_t a[NP];
#pragma unroll
    for (uint32_t j = 0; j < NP; ++j) a[j] = sb + pofs[j];
    if constexpr (PROBE == 2) {
      lo ^= a[0];
    } else if (q + 1 < R) {
      fnv_lds_round<NP>(lo, hi, a);
    } else {
      fnv_lds_round_last<NP>(lo, hi, lo2, hi2, a);  // the state before the key's final byte
    }
  }
  if constexpr (PROBE == 3) {
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (t == 0) {
      uint64_t* o = h2 + 4ull * blockIdx.x;
      o[0] = clk0;
      o[1] = clk1;
      o[2] = rt0;
      o[3] = rt1;
    }
  }
  if (t > last) return;
  const uint64_t i = key0 + t;
  const uint64_t r1 = pack2(lo, hi);
  __builtin_nontemporal_store(r1, h1 + i);
  if constexpr (H2 && PROBE != 3) __builtin_nontemporal_store(pack2(lo2, hi2), h2 + i);
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

// lean2 tile kernel (walk WALK) + the ring pass over its oversize-tile list.
// Issue priority of lean2's load / sort phase (s_setprio; the hash walk runs at 0): a tile's
// offset loads, DMA issue and length sort then do not queue behind the other block's hash
// instructions on the same SIMD.  -2.8 % kernel time on config 3 in same-process A/B
// (lab variants 88-90, priorities 1-3 equal; profiles/r02ba_csr_dbuf_queue_ab.json).
constexpr int kLean2Prio = 1;
// The 128-class scan by wave 0 alone (two classes per lane, one barrier fewer than the
// four-wave scan): -0.6 % (lab variant 93 vs 90, profiles/r02ba_csr_dbuf_queue_ab.json).
constexpr bool kLean2Scan1 = true;

template <int WALK>
static hipError_t launch_lean2(const uint8_t* b, const uint64_t* offsets, uint64_t n, const SpadTable& t, uint64_t* h1,
                               uint64_t* h2, uint32_t* scratch, unsigned g, unsigned gl, const BucketParams* bp,
                               hipStream_t stream) {
  if (bp) {
    if (h2) {
      fnv_csr_lean2_kernel<true, true, WALK, false, kLean2Prio, kLean2Scan1><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch, *bp);
      fnv_csr_ring_list_kernel<true, true><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch, *bp);
    } else {
      fnv_csr_lean2_kernel<false, true, WALK, false, kLean2Prio, kLean2Scan1><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch, *bp);
      fnv_csr_ring_list_kernel<false, true><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch, *bp);
    }
  } else {
    if (h2) {
      fnv_csr_lean2_kernel<true, false, WALK, false, kLean2Prio, kLean2Scan1><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch);
      fnv_csr_ring_list_kernel<true><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch);
    } else {
      fnv_csr_lean2_kernel<false, false, WALK, false, kLean2Prio, kLean2Scan1><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch);
      fnv_csr_ring_list_kernel<false><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch);
    }
  }
  return hipGetLastError();
}

#if K2H_AMD_LAB
#include "k2h_csr_lab.inc"

static hipError_t launch_csr_tile_lab(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                           uint64_t* h2, int mode, hipStream_t stream, const BucketParams* bp) {
  SpadTable t = make_spad(seed);
  if (mode == kModeDbufProbeNoHash) return launch_dbuf<1>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModeDbufProbeNoFeed) return launch_dbuf<2>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModeQueueProbeNoHash) return launch_dbuf<1, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModeQueueProbeNoFeed) return launch_dbuf<2, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModeLean2Prio) return launch_lean2_prio<2>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2Prio3) return launch_lean2_prio<3>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2Ballot) return launch_lean2_prio<1, true, 2>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2PrioSetup) return launch_lean2_prio<4, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeQueue320) return launch_queue320((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2Desync1) return launch_lean2_prio<1, true, false, 1>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2Desync2) return launch_lean2_prio<1, true, false, 2>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean3) return launch_lean3((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2Runs) return launch_lean2_prio<1, true, 1>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2Scan1) return launch_lean2_prio<1, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeLean2Prio1) return launch_lean2_prio<1>((const uint8_t*)bytes, offsets, n, t, h1, h2, stream);
  if (mode == kModeQueuePrio) return launch_dbuf<3, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModeQueue) return launch_dbuf<0, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModeDbuf) return launch_dbuf((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair2) return launch_pair<2, 36, false>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair2P) return launch_pair<2, 36, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair4P) return launch_pair<4, 72, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair4) return launch_pair<4, 72, false>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair4Z) return launch_pair<4, 72, false, false, false, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair4W2) return launch_pair<4, 72, false, false, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair4PS) return launch_pair<4, 72, true, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModePair2PS) return launch_pair<2, 36, true, true>((const uint8_t*)bytes, offsets, n, t, h1, h2, bp, stream);
  if (mode == kModeLean2Clock) {  // h2 = stamp buffer (4 words per wave), tiles past the stage not hashed
    if (!h2) return hipErrorInvalidValue;
    const unsigned gc = (unsigned)((n + kTileKeys - 1) / kTileKeys);
    uint32_t* scratch = nullptr;
    hipError_t e = hipMallocAsync((void**)&scratch, 4ull * (gc + 1), stream);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(scratch, 0, 4, stream);
    if (e == hipSuccess) {
      fnv_csr_lean2_kernel<false, false, 3, true><<<gc, 256, 0, stream>>>((const uint8_t*)bytes, offsets, n, t, h1, h2,
                                                                         scratch + 1, scratch);
      e = hipGetLastError();
    }
    hipError_t f = hipFreeAsync(scratch, stream);
    return e != hipSuccess ? e : f;
  }
  unsigned g = (unsigned)((n + kTileKeys - 1) / kTileKeys);
  const uint8_t* b = (const uint8_t*)bytes;
  if (mode == kModeLeanRing || mode == kModeLean2Ring || mode == kModeLean2Pin || mode == kModeLean2Step ||
      mode == kModeLean2Group) {
    // Default: 512-key tiles staged by the lean kernel (62 VGPRs, no ring code); tiles
    // whose bytes exceed its 72 KiB stage are listed and hashed by the line-ring kernel
    // in a second launch on the same stream (none for BASELINE config 3).
    uint32_t* scratch = nullptr;  // [0] = count, [1..] = tile list
    hipError_t e = hipMallocAsync((void**)&scratch, 4ull * (g + 1), stream);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(scratch, 0, 4, stream);
    const BucketParams none{};
    const BucketParams& p = bp ? *bp : none;
    const unsigned gl = g < 512u ? g : 512u;  // ring kernel: ~78 KiB LDS, two blocks per CU
    if (e == hipSuccess && mode != kModeLeanRing) {
      e = mode == kModeLean2Pin    ? launch_lean2<1>(b, offsets, n, t, h1, h2, scratch, g, gl, bp, stream)
          : mode == kModeLean2Step ? launch_lean2<2>(b, offsets, n, t, h1, h2, scratch, g, gl, bp, stream)
          : mode == kModeLean2Group ? launch_lean2<0>(b, offsets, n, t, h1, h2, scratch, g, gl, bp, stream)
                                    : launch_lean2<3>(b, offsets, n, t, h1, h2, scratch, g, gl, bp, stream);
    } else if (e == hipSuccess) {
      if (bp) {
        if (h2) {
          fnv_csr_lean_kernel<true, 512, 4, 72, 1, true><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch, p);
          fnv_csr_ring_list_kernel<true, true><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch, p);
        } else {
          fnv_csr_lean_kernel<false, 512, 4, 72, 1, true><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch, p);
          fnv_csr_ring_list_kernel<false, true><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch, p);
        }
      } else {
        if (h2) {
          fnv_csr_lean_kernel<true, 512, 4, 72><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch);
          fnv_csr_ring_list_kernel<true><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, h2, scratch + 1, scratch);
        } else {
          fnv_csr_lean_kernel<false, 512, 4, 72><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch);
          fnv_csr_ring_list_kernel<false><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, scratch + 1, scratch);
        }
      }
      e = hipGetLastError();
    }
    hipError_t f = hipFreeAsync(scratch, stream);
    return e != hipSuccess ? e : f;
  }
  if (bp && mode == kModeStaged) {  // fused epilogue on the round-1 tile kernel
    if (h2) fnv_csr_tile_kernel<true, kModeStaged, true><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2, *bp);
    else fnv_csr_tile_kernel<false, kModeStaged, true><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr, *bp);
    return hipGetLastError();
  }
#define K2H_CSR_LAUNCH(M)                                                                      \
  if (h2) fnv_csr_tile_kernel<true, M><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2);       \
  else fnv_csr_tile_kernel<false, M><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr);
  switch (mode) {
    case kModeDirect: K2H_CSR_LAUNCH(kModeDirect) break;
    case kModeRing: K2H_CSR_LAUNCH(kModeRing) break;
    case kModeStagedPairs: K2H_CSR_LAUNCH(kModeStagedPairs) break;
    case kModeStagedSingle: K2H_CSR_LAUNCH(kModeStagedSingle) break;
    case kModeStagedProf:  // h2 = stamp buffer of 16 x ceil(n/512) words, required
      if (!h2) return hipErrorInvalidValue;
      fnv_csr_tile_kernel<false, kModeStagedProf><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2);
      break;
    case kModeLean256: {
      unsigned gl = (unsigned)((n + 255) / 256);
      if (h2) fnv_csr_lean_kernel<true, 256, 4, 36><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, h2);
      else fnv_csr_lean_kernel<false, 256, 4, 36><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr);
      break;
    }
    case kModeLeanAlignProbe: {  // timing probe only: wrong hashes
      unsigned gl = (unsigned)((n + 255) / 256);
      fnv_csr_lean_kernel<false, 256, 4, 36, 3><<<gl, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr);
      break;
    }
    case kModeLean512x8: {
      if (h2) fnv_csr_lean_kernel<true, 512, 8, 72><<<g, 512, 0, stream>>>(b, offsets, n, t, h1, h2);
      else fnv_csr_lean_kernel<false, 512, 8, 72><<<g, 512, 0, stream>>>(b, offsets, n, t, h1, nullptr);
      break;
    }
    case kModeLean512x4: {
      if (h2) fnv_csr_lean_kernel<true, 512, 4, 72><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, h2);
      else fnv_csr_lean_kernel<false, 512, 4, 72><<<g, 256, 0, stream>>>(b, offsets, n, t, h1, nullptr);
      break;
    }
    default: K2H_CSR_LAUNCH(kModeStaged) break;
  }
#undef K2H_CSR_LAUNCH
  if (bp) return launch_bucket_index(h1, n, *bp, stream);  // A/B modes: unfused epilogue
  return hipGetLastError();
}
#endif  // K2H_AMD_LAB

static_assert(kCsrDefaultMode == kModeLean2Ring, "product CSR mode");

hipError_t launch_csr_tile(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                           uint64_t* h2, int mode, hipStream_t stream, const BucketParams* bp) {
#if K2H_AMD_LAB
  if (mode != kModeLean2Ring) return launch_csr_tile_lab(bytes, offsets, n, seed, h1, h2, mode, stream, bp);
#else
  (void)mode;
#endif
  // 512-key tiles staged by the lean2 kernel (pair walk); tiles whose bytes exceed its
  // 72 KiB stage are listed and hashed by the line-ring kernel in a second launch on the
  // same stream (none for BASELINE config 3).
  const SpadTable t = make_spad(seed);
  const unsigned g = (unsigned)((n + kTileKeys - 1) / kTileKeys);
  uint32_t* scratch = nullptr;  // [0] = count, [1..] = tile list
  hipError_t e = hipMallocAsync((void**)&scratch, 4ull * (g + 1), stream);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(scratch, 0, 4, stream);
  const unsigned gl = g < 512u ? g : 512u;  // ring kernel: ~78 KiB LDS, two blocks per CU
  if (e == hipSuccess) e = launch_lean2<3>((const uint8_t*)bytes, offsets, n, t, h1, h2, scratch, g, gl, bp, stream);
  hipError_t f = hipFreeAsync(scratch, stream);
  return e != hipSuccess ? e : f;
}

bool fixed_lines_ok(const void* keys, uint64_t key_len) {
  return key_len >= 128 && (key_len & 127u) == 0 && ((uintptr_t)keys & 127u) == 0 && key_len < (1ull << 26);
}

#if K2H_AMD_LAB
static hipError_t launch_fixed_long_lab(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1,
                             uint64_t* h2, int mode, hipStream_t stream, const BucketParams* bp) {
  const uint8_t* k = (const uint8_t*)keys;
  if (mode == kLongAuto) mode = fixed_lines_ok(keys, key_len) ? kLongLines2 : kLongRing;
  if (mode >= kLongLines2 && !fixed_lines_ok(keys, key_len)) mode = kLongRing;
  if (mode >= kLongLines2) {
    unsigned g = (unsigned)((n + 63) / 64);
#define K2H_LINES(DD, RR)                                                                                         \
  if (bp) {                                                                                                       \
    if (h2) fnv_fixed_lines_kernel<true, DD, RR, true><<<g, 64, pad, stream>>>(k, key_len, n, seed, h1, h2, *bp);    \
    else fnv_fixed_lines_kernel<false, DD, RR, true><<<g, 64, pad, stream>>>(k, key_len, n, seed, h1, nullptr, *bp); \
  } else {                                                                                                          \
    if (h2) fnv_fixed_lines_kernel<true, DD, RR><<<g, 64, pad, stream>>>(k, key_len, n, seed, h1, h2);               \
    else fnv_fixed_lines_kernel<false, DD, RR><<<g, 64, pad, stream>>>(k, key_len, n, seed, h1, nullptr);            \
  }
    // kLongLines2Pad / Pad2: 4 / 2 KiB of dynamic LDS on top of the 16 KiB ring, i.e. 8 or
    // 9 instead of 10 waves per CU (occupancy probes)
    const unsigned pad = mode == kLongLines2Pad ? 4096u : mode == kLongLines2Pad2 ? 2048u : 0u;
    if ((mode >= kLongProbeCompute && mode <= kLongProbeMemHalf4) || mode == kLongProbeClock || mode == kLongPrio) {  // probes
      if (mode == kLongProbeCompute)
        fnv_fixed_lines_kernel<false, 2, 128, false, 1><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
      else if (mode == kLongProbeMemory)
        fnv_fixed_lines_kernel<false, 2, 128, false, 2><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
      else if (mode == kLongProbeMem3)
        fnv_fixed_lines_kernel<false, 3, 128, false, 2><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
      else if (mode == kLongProbeMem4)
        fnv_fixed_lines_kernel<false, 4, 128, false, 2><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
      else if (mode == kLongProbeMem256)
        fnv_fixed_lines_kernel<false, 2, 256, false, 2><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
      else if (mode == kLongProbeMemHalf4)
        fnv_fixed_lines_kernel<false, 4, 64, false, 2><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
      else if (mode == kLongPrio)
        fnv_fixed_lines_kernel<false, 2, 128, false, 4><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
      else if (mode == kLongProbeClock && h2)
        fnv_fixed_lines_kernel<true, 2, 128, false, 3><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, h2);
      return hipGetLastError();
    }
    if (mode == kLongLines256 && key_len % 256 != 0) mode = kLongLines2;
    if (mode == kLongLines256) {
      K2H_LINES(2, 256)
    } else
    switch (mode) {
      case kLongLines3: K2H_LINES(3, 128) break;
      case kLongHalf5: K2H_LINES(5, 64) break;
      case kLongHalf3: K2H_LINES(3, 64) break;
      case kLongHalf2: K2H_LINES(2, 64) break;
      case kLongHalf4: K2H_LINES(4, 64) break;
      case kLongHalf6: K2H_LINES(6, 64) break;
      default: K2H_LINES(2, 128) break;
    }
#undef K2H_LINES
    return hipGetLastError();
  }
  SpadTable t = make_spad(seed);
  unsigned g = (unsigned)((n + 255) / 256);
  const bool direct = mode == kLongDirect;
  if (bp && !direct) {  // fused epilogue on the line ring kernel
    if (h2) fnv_fixed_long_kernel<true, false, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, h2, *bp);
    else fnv_fixed_long_kernel<false, false, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, nullptr, *bp);
    return hipGetLastError();
  }
  if (direct) {
    if (h2) fnv_fixed_long_kernel<true, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, h2);
    else fnv_fixed_long_kernel<false, true><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, nullptr);
  } else {
    if (h2) fnv_fixed_long_kernel<true, false><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, h2);
    else fnv_fixed_long_kernel<false, false><<<g, 256, 0, stream>>>(k, key_len, n, t, h1, nullptr);
  }
  if (bp) return launch_bucket_index(h1, n, *bp, stream);
  return hipGetLastError();
}
#endif  // K2H_AMD_LAB

hipError_t launch_fixed_long(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1,
                             uint64_t* h2, int mode, hipStream_t stream, const BucketParams* bp) {
#if K2H_AMD_LAB
  if (mode > kLongLines2) return launch_fixed_long_lab(keys, key_len, n, seed, h1, h2, mode, stream, bp);
#endif
  const uint8_t* k = (const uint8_t*)keys;
  if (mode == kLongAuto) mode = fixed_lines_ok(keys, key_len) ? kLongLines2 : kLongRing;
  if (mode == kLongLines2 && !fixed_lines_ok(keys, key_len)) mode = kLongRing;
  if (mode == kLongLines2) {  // 2 rounds of whole 128-byte lines per lane in the LDS ring
    const unsigned g = (unsigned)((n + 63) / 64);
    if (bp) {
      if (h2) fnv_fixed_lines_kernel<true, 2, 128, true><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, h2, *bp);
      else fnv_fixed_lines_kernel<false, 2, 128, true><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr, *bp);
    } else {
      if (h2) fnv_fixed_lines_kernel<true, 2, 128><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, h2);
      else fnv_fixed_lines_kernel<false, 2, 128><<<g, 64, 0, stream>>>(k, key_len, n, seed, h1, nullptr);
    }
    return hipGetLastError();
  }
  const SpadTable t = make_spad(seed);
  const unsigned g = (unsigned)((n + 255) / 256);
  const BucketParams none{};
  const BucketParams& p = bp ? *bp : none;
  if (mode == kLongDirect) {  // per-lane direct loads (keys below 128 B)
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
