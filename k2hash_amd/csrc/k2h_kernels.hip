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

#if K2H_AMD_LAB  // measurement-lab variants (tools/lab), not in libk2hash_amd.so
// ---------------------------------------------------------------------------
// fixed32: key i = keys[32*i .. 32*i+32), keys 16-byte aligned.
// ---------------------------------------------------------------------------
template <bool H2, bool ASM, bool NT = false, bool EPI = false, int BS = 256>
__global__ __launch_bounds__(BS) void fnv_fixed32_kernel(const uint4* __restrict__ keys, uint64_t n, uint64_t seed,
                                                         uint64_t* __restrict__ h1, uint64_t* __restrict__ h2,
                                                         BucketParams bp = {}) {
  uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  uint4 a, b;
  if constexpr (NT) {
    a = ld_nt(keys + 2 * i);
    b = ld_nt(keys + 2 * i + 1);
  } else {
    a = keys[2 * i];
    b = keys[2 * i + 1];
  }
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2, hi2;
  if constexpr (ASM) {
    if constexpr (H2) {
      fnv_chunk32_last(lo, hi, lo2, hi2, a, b);
    } else {
      fnv_chunk32(lo, hi, a, b);
    }
  } else {
    uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int j = 0; j < 7; ++j) fnv_word_c(lo, hi, w[j]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k == 3) {
        lo2 = lo;
        hi2 = hi;
      }
      fnv_step_c(lo, hi, (w[7] >> (8 * k)) & 0xffu);
    }
  }
  if constexpr (NT) {
    st_nt(h1 + i, pack(lo, hi));
    if constexpr (H2) st_nt(h2 + i, pack(lo2, hi2));
  } else {
    h1[i] = pack(lo, hi);
    if constexpr (H2) h2[i] = pack(lo2, hi2);
  }
  if constexpr (EPI) bucket_emit(bp, i, pack(lo, hi));
}

// fixed32, whole key in one asm statement (fnv_key32_x): explicit registers, 64-bit
// shift sign smear, nt load/store inside the statement.
template <bool H2>
__global__ __launch_bounds__(256) void fnv_fixed32_x_kernel(const uint4* __restrict__ keys, uint64_t n, uint64_t seed,
                                                            uint64_t* __restrict__ h1, uint64_t* __restrict__ h2) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  if constexpr (H2) fnv_key32_x2(keys + 2 * i, h1 + i, h2 + i, seed);
  else fnv_key32_x(keys + 2 * i, h1 + i, seed);
}

#endif  // K2H_AMD_LAB

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

__device__ __forceinline__ void fixed32_hash_store(uint4 a, uint4 b, uint64_t seed, uint64_t i, uint64_t* h1,
                                                   uint64_t* h2, bool want_h2) {
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2, hi2;
  if (want_h2) {
    fnv_chunk32_last(lo, hi, lo2, hi2, a, b);
    h2[i] = pack(lo2, hi2);
  } else {
    fnv_chunk32(lo, hi, a, b);
  }
  h1[i] = pack(lo, hi);
}

#if K2H_AMD_LAB  // measurement-lab variants (tools/lab), not in libk2hash_amd.so
template <bool H2>
__global__ __launch_bounds__(256) void fnv_fixed32_persist_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                                  uint64_t seed, uint64_t* __restrict__ h1,
                                                                  uint64_t* __restrict__ h2) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint4 a = keys[2 * i], b = keys[2 * i + 1];
  for (;;) {
    uint64_t nx = i + stride;
    bool more = nx < n;
    uint4 na = a, nb = b;
    if (more) {
      na = keys[2 * nx];
      nb = keys[2 * nx + 1];
    }
    fixed32_hash_store(a, b, seed, i, h1, h2, H2);
    if (!more) break;
    i = nx;
    a = na;
    b = nb;
  }
}

// Same, but each wave reads its 64 keys as two fully coalesced 1 KiB loads (lane l:
// bytes 16l and 1024+16l of the wave's 2 KiB run) and transposes them through a
// wave-private 2 KiB LDS slot, so every global load instruction touches 8 whole
// 128-byte lines instead of 16 half lines.
template <bool H2>
__global__ __launch_bounds__(256) void fnv_fixed32_lds_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                              uint64_t seed, uint64_t* __restrict__ h1,
                                                              uint64_t* __restrict__ h2) {
  __shared__ uint4 slot[4][128];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t waves = (uint64_t)gridDim.x * 4u;
  const uint64_t ntiles = (n + 63) / 64;
  uint64_t t = (uint64_t)blockIdx.x * 4u + wave;
  if (t >= ntiles) return;
  const uint64_t nchunks = 2 * n;  // 16-byte chunks in the key buffer
  auto ld = [&](uint64_t tile, uint4& x, uint4& y) {
    uint64_t c0 = tile * 128 + lane, c1 = c0 + 64;
    x = c0 < nchunks ? keys[c0] : make_uint4(0, 0, 0, 0);
    y = c1 < nchunks ? keys[c1] : make_uint4(0, 0, 0, 0);
  };
  uint4 x, y;
  ld(t, x, y);
  for (;;) {
    uint64_t nt = t + waves;
    bool more = nt < ntiles;
    uint4 nx = x, ny = y;
    if (more) ld(nt, nx, ny);
    slot[wave][lane] = x;
    slot[wave][lane + 64] = y;
    __builtin_amdgcn_wave_barrier();
    uint4 a = slot[wave][2 * lane], b = slot[wave][2 * lane + 1];
    __builtin_amdgcn_wave_barrier();
    uint64_t i = t * 64 + lane;
    if (i < n) fixed32_hash_store(a, b, seed, i, h1, h2, H2);
    if (!more) break;
    t = nt;
    x = nx;
    y = ny;
  }
}



#endif  // K2H_AMD_LAB

// fixed32, flat grid, KPT keys per thread: block b owns keys [b*256*KPT, (b+1)*256*KPT);
// thread t hashes keys b*256*KPT + j*256 + t.  All 2*KPT loads are issued before the
// first hash, so each wave keeps KPT*2 KiB in flight while it computes.
// PRIO (lab): the loads issued at raised issue priority, the hash at 0.
template <bool H2, int KPT, int BS = 256, bool NT = false, bool EPI = false, bool CLK = false, int PRIO = 0>
__global__ __launch_bounds__(BS) void fnv_fixed32_kpt_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                             uint64_t seed, uint64_t* __restrict__ h1,
                                                             uint64_t* __restrict__ h2, BucketParams bp = {}) {
  // CLK (lab clock probe, h1 only): h2 receives per wave the shader-clock and 100 MHz
  // counters at its start and end (tools/clock_probe.py)
  uint64_t clk0 = 0, rt0 = 0;
  if constexpr (CLK) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  const uint64_t base = (uint64_t)blockIdx.x * (BS * KPT) + threadIdx.x;
  uint4 a[KPT], b[KPT];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    uint64_t i = base + BS * j;
    if (i < n) {
      if constexpr (NT) {
        a[j] = ld_nt(keys + 2 * i);
        b[j] = ld_nt(keys + 2 * i + 1);
      } else {
        a[j] = keys[2 * i];
        b[j] = keys[2 * i + 1];
      }
    }
  }
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    uint64_t i = base + BS * j;
    if (i < n) {
      if constexpr (NT) {
        uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2, hi2;
        if constexpr (H2) {
          fnv_chunk32_last(lo, hi, lo2, hi2, a[j], b[j]);
          st_nt(h2 + i, pack(lo2, hi2));
        } else {
          fnv_chunk32(lo, hi, a[j], b[j]);
        }
        st_nt(h1 + i, pack(lo, hi));
        if constexpr (EPI) bucket_emit(bp, i, pack(lo, hi));
      } else {
        fixed32_hash_store(a[j], b[j], seed, i, h1, h2, H2);
      }
    }
  }
  if constexpr (CLK) {
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63u) == 0) {
      uint64_t* o = h2 + 4ull * (blockIdx.x * (BS / 64) + threadIdx.x / 64);
      o[0] = clk0;
      o[1] = clk1;
      o[2] = rt0;
      o[3] = rt1;
    }
  }
}

#if K2H_AMD_LAB  // measurement-lab variants (tools/lab), not in libk2hash_amd.so
// ---------------------------------------------------------------------------
// fixed32, software-pipelined persistent blocks: each block walks tiles of 2*BS keys
// (two keys per lane) with a grid stride, and the loads of its next tile are issued
// before it hashes the current one, so every wave always has 4 KiB in flight (the flat
// kernel has loads in flight only while it waits).  Loads are unconditional (past the
// last tile a block re-reads its current one), so the compiler's vmcnt waits are exact.
// ---------------------------------------------------------------------------
template <bool H2, int BS>
__global__ __launch_bounds__(BS) void fnv_fixed32_pipe_kernel(const uint4* __restrict__ keys, uint64_t n,
                                                              uint64_t seed, uint64_t* __restrict__ h1,
                                                              uint64_t* __restrict__ h2) {
  const uint64_t ntiles = (n + 2 * BS - 1) / (2 * BS);
  const uint64_t stride = gridDim.x;
  uint64_t t = blockIdx.x;
  if (t >= ntiles) return;
  auto load = [&](uint64_t tile, uint4(&v)[4]) {
    const uint64_t i0 = tile * (2 * BS) + threadIdx.x, i1 = i0 + BS;
    const uint64_t a = i0 < n ? i0 : n - 1, b = i1 < n ? i1 : n - 1;
    v[0] = ld_nt(keys + 2 * a);
    v[1] = ld_nt(keys + 2 * a + 1);
    v[2] = ld_nt(keys + 2 * b);
    v[3] = ld_nt(keys + 2 * b + 1);
  };
  auto work = [&](uint64_t tile, const uint4(&v)[4]) {
    const uint64_t i0 = tile * (2 * BS) + threadIdx.x;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint64_t i = i0 + BS * j;
      uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2, hi2;
      if constexpr (H2) fnv_chunk32_last(lo, hi, lo2, hi2, v[2 * j], v[2 * j + 1]);
      else fnv_chunk32(lo, hi, v[2 * j], v[2 * j + 1]);
      if (i < n) {
        st_nt(h1 + i, pack(lo, hi));
        if constexpr (H2) st_nt(h2 + i, pack(lo2, hi2));
      }
    }
  };
  uint4 A[4], B[4];
  load(t, A);
  for (;;) {
    const uint64_t t1 = t + stride;
    load(t1 < ntiles ? t1 : t, B);
    work(t, A);
    if (t1 >= ntiles) break;
    const uint64_t t2 = t1 + stride;
    load(t2 < ntiles ? t2 : t1, A);
    work(t1, B);
    if (t2 >= ntiles) break;
    t = t2;
  }
}

template <bool H2, int BS>
static unsigned pipe_grid(uint64_t ntiles) {
  static int per_cu = 0, cus = 0;
  if (!per_cu) {
    int dev = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fnv_fixed32_pipe_kernel<H2, BS>, BS, 0) !=
            hipSuccess ||
        per_cu <= 0)
      per_cu = 2048 / BS;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || cus <= 0)
      cus = 256;
  }
  const uint64_t g = (uint64_t)cus * (uint64_t)per_cu;
  return (unsigned)(ntiles < g ? ntiles : g);
}

// ---------------------------------------------------------------------------
// fixed32, LDS-DMA ring: one-wave blocks, persistent.  Wave w hashes tiles of 64 keys
// (2 KiB) w, w + W, w + 2W, ... and streams them through a private ring of S LDS slots
// with global_load_lds_dwordx4 (two fully coalesced 1 KiB pieces per tile, no VGPRs
// held), so each wave keeps S-1 tiles in flight while it hashes the current one --
// the flat kernel holds at most one key per lane in flight and only while it waits.
// Ordering: loads, LDS-DMA and stores share the in-order vmcnt counter
// (MI355X_MICROARCH.md, s_waitcnt), and every iteration issues exactly two DMA pieces
// (a dummy re-read of one line past the wave's last tile), so the wait that retires
// tile j is vmcnt(2(S-1) + min(j, S-1) * stores per tile).
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void lds_read32(uint4& a, uint4& b, uint32_t addr) {
  asm volatile(
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %2 offset:16\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=v"(a), "=v"(b)
      : "v"(addr)
      : "memory");
}

template <bool H2, int S>
__global__ __launch_bounds__(64) void fnv_fixed32_ring_kernel(const uint8_t* __restrict__ keys, uint64_t n,
                                                              uint64_t seed, uint64_t* __restrict__ h1,
                                                              uint64_t* __restrict__ h2) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[S][2048];
  constexpr int kSt = H2 ? 2 : 1;  // stores per tile
  const uint32_t lane = threadIdx.x;
  const uint64_t ntiles = (n + 63) / 64;
  const uint64_t W = gridDim.x;
  const uint64_t t0 = blockIdx.x;
  if (t0 >= ntiles) return;
  const uint64_t m = (ntiles - t0 + W - 1) / W;  // tiles of this wave
  const uint64_t last_chunk = 2 * n - 1;          // 16-byte pieces of the key buffer
  auto issue = [&](uint64_t j) {
    uint32_t slot = (uint32_t)(j % S);
    uint64_t c0, c1;
    if (j < m) {
      uint64_t t = t0 + j * W;
      c0 = t * 128 + lane;
      c1 = c0 + 64;
      c0 = c0 > last_chunk ? last_chunk : c0;
      c1 = c1 > last_chunk ? last_chunk : c1;
    } else {  // dummy: keeps the per-iteration vmcnt arithmetic uniform
      c0 = c1 = t0 * 128;
    }
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(uintptr_t)(keys + 16 * c0),
                                     (__attribute__((address_space(3))) void*)&ring[slot][0], 16, 0, 0);
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(uintptr_t)(keys + 16 * c1),
                                     (__attribute__((address_space(3))) void*)&ring[slot][1024], 16, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);
  for (uint64_t j = 0; j < m; ++j) {
    issue(j + S - 1);
    if (j >= S - 1) {
      wait_vmcnt<2 * (S - 1) + (S - 1) * kSt>();
    } else if constexpr (S >= 3) {
      if (j == 0) wait_vmcnt<2 * (S - 1)>();
      else if (j == 1) wait_vmcnt<2 * (S - 1) + kSt>();
      else if constexpr (S >= 4) {
        if (j == 2) wait_vmcnt<2 * (S - 1) + 2 * kSt>();
        else wait_vmcnt<0>();
      } else {
        wait_vmcnt<0>();
      }
    } else {
      wait_vmcnt<2 * (S - 1)>();
    }
    // the LDS reads are asm: hipcc would otherwise put a vmcnt(0) in front of any
    // ds_read that may alias a pending LDS-DMA, draining the whole ring every tile
    uint4 a, b;
    lds_read32(a, b, (uint32_t)(uintptr_t)&ring[j % S][32u * lane]);
    uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2, hi2;
    uint64_t i = (t0 + j * W) * 64 + lane;
    if constexpr (H2) {
      fnv_chunk32_last(lo, hi, lo2, hi2, a, b);
    } else {
      fnv_chunk32(lo, hi, a, b);
    }
    // lane 0 of every tile of this wave is a real key (t < ntiles), so the store
    // instruction is always issued and the per-iteration vmcnt arithmetic holds
    if (i < n) {
      st_nt(h1 + i, pack(lo, hi));
      if constexpr (H2) st_nt(h2 + i, pack(lo2, hi2));
    }
  }
  wait_vmcnt<0>();
}

static unsigned persist_grid(uint64_t units_of_256) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  uint64_t g = (uint64_t)cus * 8;  // 8 x 256-thread blocks = 32 waves per CU
  return (unsigned)(units_of_256 < g ? units_of_256 : g);
}

// Resident one-wave blocks of the ring kernel per CU (occupancy query, LDS-bound), times
// the CU count; never more blocks than tiles.
static unsigned ring_grid(int variant, bool h2, uint64_t ntiles) {
  static int cache[3][2] = {};
  int v = variant == kVariantFixed32Ring2 ? 0 : variant == kVariantFixed32Ring3 ? 1 : 2;
  int& per_cu = cache[v][h2];
  if (!per_cu) {
    const void* f = nullptr;
    switch (v) {
      case 0: f = h2 ? (const void*)fnv_fixed32_ring_kernel<true, 2> : (const void*)fnv_fixed32_ring_kernel<false, 2>; break;
      case 1: f = h2 ? (const void*)fnv_fixed32_ring_kernel<true, 3> : (const void*)fnv_fixed32_ring_kernel<false, 3>; break;
      default: f = h2 ? (const void*)fnv_fixed32_ring_kernel<true, 4> : (const void*)fnv_fixed32_ring_kernel<false, 4>; break;
    }
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 64, 0) != hipSuccess || per_cu <= 0) per_cu = 16;
  }
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  uint64_t g = (uint64_t)cus * (uint64_t)per_cu;
  return (unsigned)(ntiles < g ? ntiles : g);
}

#endif  // K2H_AMD_LAB

hipError_t launch_bucket_index(const uint64_t* h1, uint64_t n, const BucketParams& bp, hipStream_t stream) {
  if (n == 0 || !(bp.kindex || bp.ckindex)) return hipSuccess;
  bucket_index_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n, bp);
  return hipGetLastError();
}

#if K2H_AMD_LAB
static hipError_t launch_fixed_lab(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1, uint64_t* h2,
                        int variant, hipStream_t stream, const BucketParams* bp) {
  if (n == 0) return hipSuccess;
  const bool epi = bp && (bp->kindex || bp->ckindex);
  if (!keys || key_len == 0) {
    fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n);
    if (h2) fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h2, n);
    if (epi) return launch_bucket_index(h1, n, *bp, stream);
    return hipGetLastError();
  }
  bool aligned16 = ((uintptr_t)keys & 15u) == 0;
  if (key_len == 32 && aligned16 && variant != kVariantGeneric) {
    const uint4* k = (const uint4*)keys;
    switch (variant) {
      case kVariantCompiler:
        if (h2) fnv_fixed32_kernel<true, false><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_kernel<false, false><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      case kVariantAuto: {
        // One-wave blocks (a finished wave's slot is refilled at once instead of when the
        // slowest of a block's four waves ends: 3-4 %), two keys per lane with all four
        // loads issued before the first hash (a wave keeps 4 KiB in flight and half as
        // many waves need dispatching: 5 % more).  Round-1 A/B, tools/variants.py,
        // variants 0/23/27/29-31.  The second key's registers sit below the asm window,
        // so the kernel stays at 59 VGPRs (8 waves/SIMD).
        unsigned g = (unsigned)((n + 127) / 128);
        if (epi) {
          if (h2) fnv_fixed32_kpt_kernel<true, 2, 64, true, true><<<g, 64, 0, stream>>>(k, n, seed, h1, h2, *bp);
          else fnv_fixed32_kpt_kernel<false, 2, 64, true, true><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr, *bp);
          return hipGetLastError();
        }
        if (h2) fnv_fixed32_kpt_kernel<true, 2, 64, true><<<g, 64, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_kpt_kernel<false, 2, 64, true><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
      case kVariantFixed32Prio: {
        unsigned g = (unsigned)((n + 127) / 128);
        if (h2) fnv_fixed32_kpt_kernel<true, 2, 64, true, false, false, 1><<<g, 64, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_kpt_kernel<false, 2, 64, true, false, false, 1><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
      case kVariantFixed32Pipe64: {
        const uint64_t nt = (n + 127) / 128;
        if (h2) fnv_fixed32_pipe_kernel<true, 64><<<pipe_grid<true, 64>(nt), 64, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_pipe_kernel<false, 64><<<pipe_grid<false, 64>(nt), 64, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
      case kVariantFixed32Pipe256: {
        const uint64_t nt = (n + 511) / 512;
        if (h2) fnv_fixed32_pipe_kernel<true, 256><<<pipe_grid<true, 256>(nt), 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_pipe_kernel<false, 256><<<pipe_grid<false, 256>(nt), 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
      case kVariantFixed32Nt256:
        if (h2) fnv_fixed32_kernel<true, true, true><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_kernel<false, true, true><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      case kVariantFixed32W64Kpt2:
      case kVariantFixed32W64Kpt3:
      case kVariantFixed32W64Kpt4: {
        const int kpt = variant == kVariantFixed32W64Kpt2 ? 2 : variant == kVariantFixed32W64Kpt3 ? 3 : 4;
        unsigned g = (unsigned)((n + 64 * kpt - 1) / (64 * kpt));
#define K2H_KPT(KK)                                                                                             \
  if (h2) fnv_fixed32_kpt_kernel<true, KK, 64, true><<<g, 64, 0, stream>>>(k, n, seed, h1, h2);                 \
  else fnv_fixed32_kpt_kernel<false, KK, 64, true><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr);
        if (kpt == 2) { K2H_KPT(2) }
        else if (kpt == 3) { K2H_KPT(3) }
        else { K2H_KPT(4) }
#undef K2H_KPT
        break;
      }
      case kVariantFixed32Blk64:
      case kVariantFixed32Blk128:
      case kVariantFixed32Blk512:
      case kVariantFixed32Blk1024: {
#define K2H_BLK(BSZ)                                                                                          \
  {                                                                                                          \
    unsigned gb = (unsigned)((n + BSZ - 1) / BSZ);                                                           \
    if (h2) fnv_fixed32_kernel<true, true, true, false, BSZ><<<gb, BSZ, 0, stream>>>(k, n, seed, h1, h2);     \
    else fnv_fixed32_kernel<false, true, true, false, BSZ><<<gb, BSZ, 0, stream>>>(k, n, seed, h1, nullptr); \
  }
        if (variant == kVariantFixed32Blk64) K2H_BLK(64)
        else if (variant == kVariantFixed32Blk128) K2H_BLK(128)
        else if (variant == kVariantFixed32Blk512) K2H_BLK(512)
        else K2H_BLK(1024)
#undef K2H_BLK
        break;
      }
      case kVariantFixed32Asm:
        if (h2) fnv_fixed32_x_kernel<true><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_x_kernel<false><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      case kVariantFixed32Clock: {  // clock probe: h2 = stamps (4 per wave), h1 hashes
        if (!h2) return hipErrorInvalidValue;
        unsigned g = (unsigned)((n + 127) / 128);
        fnv_fixed32_kpt_kernel<false, 2, 64, true, false, true><<<g, 64, 0, stream>>>(k, n, seed, h1, h2);
        break;
      }
      case kVariantFixed32Flat:
        if (h2) fnv_fixed32_kernel<true, true><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_kernel<false, true><<<grid_for(n), 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      case kVariantFixed32Kpt2: {
        unsigned g = (unsigned)((n + 511) / 512);
        if (h2) fnv_fixed32_kpt_kernel<true, 2><<<g, 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_kpt_kernel<false, 2><<<g, 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
      case kVariantFixed32Kpt4: {
        unsigned g = (unsigned)((n + 1023) / 1024);
        if (h2) fnv_fixed32_kpt_kernel<true, 4><<<g, 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_kpt_kernel<false, 4><<<g, 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
      case kVariantFixed32Lds: {
        unsigned g = persist_grid((n + 255) / 256);
        if (h2) fnv_fixed32_lds_kernel<true><<<g, 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_lds_kernel<false><<<g, 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
      case kVariantFixed32Ring3:
      case kVariantFixed32Ring4:
      case kVariantFixed32Ring2: {
        unsigned g = ring_grid(variant, h2 != nullptr, (n + 63) / 64);
#define K2H_RING(SS)                                                                                      \
  if (h2) fnv_fixed32_ring_kernel<true, SS><<<g, 64, 0, stream>>>((const uint8_t*)keys, n, seed, h1, h2); \
  else fnv_fixed32_ring_kernel<false, SS><<<g, 64, 0, stream>>>((const uint8_t*)keys, n, seed, h1, nullptr);
        if (variant == kVariantFixed32Ring2) { K2H_RING(2) }
        else if (variant == kVariantFixed32Ring4) { K2H_RING(4) }
        else { K2H_RING(3) }
#undef K2H_RING
        break;
      }
      default: {  // kVariantFixed32Persist
        unsigned g = persist_grid((n + 255) / 256);
        if (h2) fnv_fixed32_persist_kernel<true><<<g, 256, 0, stream>>>(k, n, seed, h1, h2);
        else fnv_fixed32_persist_kernel<false><<<g, 256, 0, stream>>>(k, n, seed, h1, nullptr);
        break;
      }
    }
    if (epi) return launch_bucket_index(h1, n, *bp, stream);  // A/B variants: unfused epilogue
    return hipGetLastError();
  }
  // Routing by key length (tools/fixed_sweep.py on MI355X, 512 MiB of keys per launch):
  // up to 32 B the per-lane tail loop is fastest, below 128 B per-lane direct 16-byte
  // loads, from 128 B on the cooperative line ring.
  // From 128 B on, keys of a multiple of 128 bytes at a 128-aligned base take the line-DMA
  // kernel, everything else the cooperative line ring.
  if (variant == kVariantAuto) variant = key_len <= 32 ? kVariantFixedTail : key_len < 128 ? kVariantDirect : 0;
  if (variant != kVariantFixedTail) {
    const int mode = variant == kVariantDirect       ? kLongDirect
                     : variant == kVariantLongRing   ? kLongRing
                     : variant == kVariantLongLines2 ? kLongLines2
                     : variant == kVariantLongLines3 ? kLongLines3
                     : variant == kVariantLongHalf3  ? kLongHalf3
                     : variant == kVariantLongHalf2  ? kLongHalf2
                     : variant == kVariantLongClock  ? kLongProbeClock
                     : variant == kVariantLongPrio   ? kLongPrio
                     : variant == kVariantLongHalf4  ? kLongHalf4
                     : variant == kVariantLongHalf6  ? kLongHalf6
                     : variant == kVariantLongHalf5  ? kLongHalf5
                     : variant == kVariantLongLines2Pad ? kLongLines2Pad
                     : variant == kVariantLongLines2Pad2 ? kLongLines2Pad2
                     : variant == kVariantLongProbeCompute ? kLongProbeCompute
                     : variant == kVariantLongProbeMemory ? kLongProbeMemory
                     : variant == kVariantLongProbeMem3 ? kLongProbeMem3
                     : variant == kVariantLongProbeMem4 ? kLongProbeMem4
                     : variant == kVariantLongProbeMem256 ? kLongProbeMem256
                     : variant == kVariantLongProbeMemHalf4 ? kLongProbeMemHalf4
                     : variant == kVariantLongLines256 ? kLongLines256
                                                     : kLongAuto;
    return launch_fixed_long(keys, key_len, n, seed, h1, h2, mode, stream, epi ? bp : nullptr);
  }
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
#endif  // K2H_AMD_LAB

// Default kernel per shape (the product path).  32-byte keys at a 16-aligned base: one-wave
// blocks, two keys per lane with all four loads issued before the first hash (a wave keeps
// 4 KiB in flight and half as many waves need dispatching; round-1 A/B).
// Other lengths (tools/fixed_sweep.py): up to 32 B the per-lane tail loop, below 128 B
// per-lane direct 16-byte loads, from 128 B on the line-DMA kernel (multiples of 128 B at a
// 128-aligned base) or the cooperative line ring.
hipError_t launch_fixed(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1, uint64_t* h2,
                        int variant, hipStream_t stream, const BucketParams* bp) {
  if (n == 0) return hipSuccess;
  const bool epi = bp && (bp->kindex || bp->ckindex);
  if (!keys || key_len == 0) {
    fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n);
    if (h2) fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h2, n);
    if (epi) return launch_bucket_index(h1, n, *bp, stream);
    return hipGetLastError();
  }
#if K2H_AMD_LAB
  if (variant != kVariantAuto) return launch_fixed_lab(keys, key_len, n, seed, h1, h2, variant, stream, bp);
#else
  (void)variant;
#endif
  if (key_len == 32 && ((uintptr_t)keys & 15u) == 0) {
    const uint4* k = (const uint4*)keys;
    const unsigned g = (unsigned)((n + 127) / 128);
    if (epi) {
      if (h2) fnv_fixed32_kpt_kernel<true, 2, 64, true, true><<<g, 64, 0, stream>>>(k, n, seed, h1, h2, *bp);
      else fnv_fixed32_kpt_kernel<false, 2, 64, true, true><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr, *bp);
    } else {
      if (h2) fnv_fixed32_kpt_kernel<true, 2, 64, true><<<g, 64, 0, stream>>>(k, n, seed, h1, h2);
      else fnv_fixed32_kpt_kernel<false, 2, 64, true><<<g, 64, 0, stream>>>(k, n, seed, h1, nullptr);
    }
    return hipGetLastError();
  }
  if (key_len > 32)
    return launch_fixed_long(keys, key_len, n, seed, h1, h2, key_len < 128 ? kLongDirect : kLongAuto, stream,
                             epi ? bp : nullptr);
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

#if K2H_AMD_LAB
// ---------------------------------------------------------------------------
// csr v0: one lane per key in input order (no length balancing).
// ---------------------------------------------------------------------------
template <bool H2>
__global__ __launch_bounds__(256) void fnv_csr_simple_kernel(const uint8_t* __restrict__ bytes,
                                                             const uint64_t* __restrict__ offsets, uint64_t n,
                                                             uint64_t seed, uint64_t* __restrict__ h1,
                                                             uint64_t* __restrict__ h2) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint64_t s = offsets[i], e = offsets[i + 1];
  uint64_t len = e - s;
  if (len == 0) {
    h1[i] = 0;
    if constexpr (H2) h2[i] = 0;
    return;
  }
  const uint8_t* p = bytes + s;
  const uint8_t* end = bytes + offsets[n];
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32), lo2 = lo, hi2 = hi;
  uint64_t nfull = (len - 1) / 16;
  for (uint64_t c = 0; c < nfull; ++c) fnv_chunk16(lo, hi, load16_ua(p + 16 * c));
  uint32_t r = (uint32_t)(len - 16 * nfull);
  fnv_tail(lo, hi, lo2, hi2, load16_guarded(p + 16 * nfull, end), r);
  if (len == 1) {  // length 1: the second hash is not shortened (lib/k2hashfunc.cc:83)
    lo2 = lo;
    hi2 = hi;
  }
  h1[i] = pack(lo, hi);
  if constexpr (H2) h2[i] = pack(lo2, hi2);
}

hipError_t launch_csr_simple(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                             uint64_t* h2, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (!bytes) {
    fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n);
    if (h2) fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h2, n);
    return hipGetLastError();
  }
  if (h2)
    fnv_csr_simple_kernel<true><<<grid_for(n), 256, 0, stream>>>((const uint8_t*)bytes, offsets, n, seed, h1, h2);
  else
    fnv_csr_simple_kernel<false><<<grid_for(n), 256, 0, stream>>>((const uint8_t*)bytes, offsets, n, seed, h1,
                                                                    nullptr);
  return hipGetLastError();
}

static hipError_t launch_csr_lab(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                      uint64_t* h2, int variant, hipStream_t stream, const BucketParams* bp) {
  if (n == 0) return hipSuccess;
  const bool epi = bp && (bp->kindex || bp->ckindex);
  if (variant == kVariantSimpleCsr || !bytes) {
    hipError_t e = launch_csr_simple(bytes, offsets, n, seed, h1, h2, stream);
    if (e == hipSuccess && epi) e = launch_bucket_index(h1, n, *bp, stream);
    return e;
  }
  return launch_csr_tile(bytes, offsets, n, seed, h1, h2,
                         variant == kVariantDirect      ? 1
                         : variant == kVariantCsrRing   ? 2
                         : variant == kVariantCsrPairs  ? 3
                         : variant == kVariantCsrSingle ? 4
                         : variant == kVariantCsrProf   ? 5
                         : variant == kVariantCsrLean256  ? 6
                         : variant == kVariantCsrLean512x8 ? 7
                         : variant == kVariantCsrLean512x4 ? 8
                         : variant == kVariantCsrAlignProbe ? 9
                         : variant == kVariantCsrTile   ? 0
                         : variant == kVariantCsrLeanRing ? 10
                         : variant == kVariantCsrLean2Pin ? 12
                         : variant == kVariantCsrLean2Step ? 13
                         : variant == kVariantCsrLean2Group ? 14
                         : variant == kVariantCsrPair2 ? 15
                         : variant == kVariantCsrPair2P ? 16
                         : variant == kVariantCsrPair4P ? 17
                         : variant == kVariantCsrPair4 ? 18
                         : variant == kVariantCsrPair4PS ? 19
                         : variant == kVariantCsrPair2PS ? 20
                         : variant == kVariantCsrPair4W2 ? 21
                         : variant == kVariantCsrPair4Z ? 22
                         : variant == kVariantCsrClock ? 23
                         : variant == kVariantCsrDbuf ? 24
                         : variant == kVariantCsrQueue ? 27
                         : variant == kVariantCsrQueuePrio ? 30
                         : variant == kVariantCsrLean2Prio ? 31
                         : variant == kVariantCsrLean2Prio3 ? 32
                         : variant == kVariantCsrLean2Prio1 ? 33
                         : variant == kVariantCsrLean2Scan1 ? 34
                         : variant == kVariantCsrLean2Runs ? 35
                         : variant == kVariantCsrLean3 ? 36
                         : variant == kVariantCsrLean2Desync1 ? 37
                         : variant == kVariantCsrLean2Desync2 ? 38
                         : variant == kVariantCsrQueue320 ? 39
                         : variant == kVariantCsrLean2PrioSetup ? 40
                         : variant == kVariantCsrLean2Ballot ? 41
                         : variant == kVariantCsrQueueProbeNoHash ? 28
                         : variant == kVariantCsrQueueProbeNoFeed ? 29
                         : variant == kVariantCsrDbufProbeNoHash ? 25
                         : variant == kVariantCsrDbufProbeNoFeed ? 26
                                                        : 11,
                         stream, epi ? bp : nullptr);
}
#endif  // K2H_AMD_LAB

// CSR keys: 512-key tiles staged in LDS and hashed two keys per lane (k2h_csr.hip); a NULL
// byte buffer hashes every key to 0 (lib/k2hashfunc.cc:66-68, 80-82).
hipError_t launch_csr(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                      uint64_t* h2, int variant, hipStream_t stream, const BucketParams* bp) {
  if (n == 0) return hipSuccess;
  const bool epi = bp && (bp->kindex || bp->ckindex);
#if K2H_AMD_LAB
  if (variant != kVariantAuto) return launch_csr_lab(bytes, offsets, n, seed, h1, h2, variant, stream, bp);
#else
  (void)variant;
#endif
  if (!bytes) {
    fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h1, n);
    if (h2) fill_zero_kernel<<<grid_for(n), 256, 0, stream>>>(h2, n);
    if (epi) return launch_bucket_index(h1, n, *bp, stream);
    return hipGetLastError();
  }
  return launch_csr_tile(bytes, offsets, n, seed, h1, h2, kCsrDefaultMode, stream, epi ? bp : nullptr);
}

}  // namespace k2h
