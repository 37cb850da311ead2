// k2hash_amd -- k2himport input scan on the GPU.
//
// The same records as the host scanner (k2h_import.cc, restating the std::getline loops
// of tests/k2himport.cc:74-117) for a file that already sits in HBM, without a host pass.
// Both formats are one two-mode machine, scanned over the bytes (see "TSV as the getline
// loop's own machine" below): the file read once, 32 B per record written, one
// synchronisation per call.
// TSV (ConvertfromTsv, tests/k2himport.cc:74-89): mode K reads a key up to its TAB, mode V
// a value up to its newline; keys hashed from LDS by pass A.
// mdbm (ConvertfromMdbm, tests/k2himport.cc:95-117): key lines and value lines alternate;
// the five header lines are the machine's first records (the fifth, "HEADER=END", checked
// where it ends); the EOF rules of the host scanner (an empty value after a key line that
// ends the file with '\n', the previous record's value after a key line that ends at EOF).
// Round 4: mdbm moved onto the TSV machinery (round 1-3: newline-position and line arrays,
// hipcub device scans, three synchronisations and seven per-call pool allocations).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>

#include "../../include/k2hash_amd.h"
#include "k2h_fnv_device.h"
#include "k2h_kernels.h"

namespace k2h {
namespace {

constexpr int kThreads = 256;

// One lane per record: the key straight from the file (no gather) as k = ceil(len/16)
// 16-byte chunks that END at its last byte (the CSR kernels' end-aligned form): chunk 0
// starts p = 16k - len bytes early with those bytes zeroed, and the state starts at
// S_p = seed * P^-p, which the p zero bytes (bare multiplies) carry exactly to the seed
// -- no byte-by-byte tail.  Then the NUL that K2HShm::Set(const char*) hashes with the
// key (lib/k2hshm.cc:2081-2083): a zero byte is a bare multiply, so h1 = state * P and
// h2 = state (lib/k2hashfunc.cc:83-85); the empty key is the one-byte "\0", h1 = h2 =
// seed * P.
typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));

__device__ inline uint4 ld16(const uint8_t* p) {
  const u32x4_ua v = *reinterpret_cast<const u32x4_ua*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// The key [off, off + len) + NUL.  Callers go through hash_cstr_checked below, never this.
__device__ inline void hash_cstr_unchecked(const uint8_t* __restrict__ f, uint64_t off, uint64_t len,
                                           const SpadTable& sp, uint64_t& h1, uint64_t& h2) {
  uint64_t raw = sp.v[0];  // the seed
  if (len) {
    const uint64_t k = (len + 15) / 16;
    const uint32_t p = (uint32_t)(16 * k - len);
    const uint8_t* c0 = f + off - p;  // chunk 0 (its first p bytes are not the key's)
    uint4 c;
    if (off >= p) {
      c = ld16(c0);
    } else {  // the key starts the file: no bytes before it to over-read
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t j = p; j < 16; ++j) w[j >> 2] |= (uint32_t)f[off - p + j] << (8 * (j & 3));
      c = make_uint4(w[0], w[1], w[2], w[3]);
    }
    // zero bytes [0, p)
    const uint32_t m0 = p >= 4 ? 0u : ~0u << (8 * p), m1 = p >= 8 ? 0u : p <= 4 ? ~0u : ~0u << (8 * (p - 4));
    const uint32_t m2 = p >= 12 ? 0u : p <= 8 ? ~0u : ~0u << (8 * (p - 8)), m3 = p <= 12 ? ~0u : ~0u << (8 * (p - 12));
    c.x &= m0, c.y &= m1, c.z &= m2, c.w &= m3;
    uint32_t lo = (uint32_t)sp.v[p], hi = (uint32_t)(sp.v[p] >> 32);
    // chunks 1-3 loaded before any is hashed, later ones one ahead (round 5: one load per
    // loop trip, each waited for in turn, cost the miss-heavy mdbm pass B a round trip per chunk)
    uint4 c1 = c, c2 = c, c3 = c;
    if (k > 1) c1 = ld16(c0 + 16);
    if (k > 2) c2 = ld16(c0 + 32);
    if (k > 3) c3 = ld16(c0 + 48);
    fnv_chunk16(lo, hi, c);
    if (k > 1) fnv_chunk16(lo, hi, c1);
    if (k > 2) fnv_chunk16(lo, hi, c2);
    if (k > 3) {
      uint4 nx = c3;
      for (uint64_t q = 4; q < k; ++q) {
        const uint4 cur = nx;
        nx = ld16(c0 + 16 * q);
        fnv_chunk16(lo, hi, cur);
      }
      fnv_chunk16(lo, hi, nx);
    }
    raw = ((uint64_t)hi << 32) | lo;
  }
  h1 = raw * 1099511628211ULL;  // lib/k2hashfunc.cc:56
  h2 = len ? raw : h1;
}

// The only entry to the file hash: a key range outside the file -- impossible for
// a correct scan state -- gives zero hashes (wrong records that parity catches), never a read
// past the file.
__device__ inline void hash_cstr_checked(const uint8_t* __restrict__ f, uint64_t size, uint64_t off, uint64_t len,
                                         const SpadTable& sp, uint64_t& h1, uint64_t& h2) {
  if (off <= size && len <= size - off) {
    hash_cstr_unchecked(f, off, len, sp, h1, h2);
  } else {
    h1 = h2 = 0;
  }
}

__global__ __launch_bounds__(kThreads) void import_hash_kernel(const uint8_t* __restrict__ f, uint64_t size,
                                                               const k2h_amd_import_rec* __restrict__ recs,
                                                               uint64_t n, SpadTable sp, uint64_t* __restrict__ h1,
                                                               uint64_t* __restrict__ h2) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = recs[i].key_off, len = recs[i].key_len;
  uint64_t a, b;
  hash_cstr_checked(f, size, off, len, sp, a, b);
  __builtin_nontemporal_store(a, h1 + i);  // (consecutive lanes, consecutive i; never read back here)
  if (h2) __builtin_nontemporal_store(b, h2 + i);
}

unsigned blocks_for(uint64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

// ---------------------------------------------------------------------------
// TSV as the getline loop's own machine.  ConvertfromTsv (tests/k2himport.cc:78-86)
// alternates getline(key, '\t') and getline(value): mode K reads a key up to its TAB
// (newlines included), mode V a value up to its newline (TABs included).  A record ends
// at every newline read in mode V, and one more at EOF if the file stops in mode V (the
// value getline hits EOF after the key's TAB); a key getline that hits EOF drops its
// bytes.  Set stores C strings (lib/k2hshm.cc:2081-2083), so a field is cut at its first
// NUL: a NUL is its field's first iff the last NUL before it lies before the field's
// start.  A span of bytes therefore acts on the state (mode, record index, field start,
// last NUL) as a small function: per entry mode, the exit mode, the record ends passed and
// the last field boundary (a TAB read in K, a newline read in V); plus its last NUL.
// These functions compose associatively (positions only grow, so "last" combines with
// max), so each 16 KiB block gets its entry state from a device scan of block functions
// and each thread from a block scan of the functions of its 128 bytes.
//
// The file is read ONCE (round 3; round 2 read it twice): pass A stages a block, finds
// each span's events (NL / TAB / NUL) and packs up to six of them per span into one word,
// computes the block function, and -- speculatively, since it does not know the mode at
// the block's start -- hashes the key that would follow each of the block's newlines
// (kSpec below).  Pass B needs no file bytes: from the packed events it rebuilds the span
// functions, scans them, walks the events, writes every record and takes each key's hash
// from pass A's state (or, for the rare key pass A could not cover, from the file).
// ---------------------------------------------------------------------------
constexpr uint32_t kTThreads = 128;
constexpr uint32_t kTBytes = 128;                               // bytes per thread
constexpr uint32_t kTChunk = kTThreads * kTBytes;               // 16 KiB per block
// pass B (and the entry-state scan) works in units of one wave's spans: 8 KiB
constexpr uint32_t kUnit = 64 * kTBytes;
constexpr uint32_t kUnitsPerBlock = kTChunk / kUnit;

// Block-local function of a span; positions are block-relative + 1 (0: none).  Every
// field is a pair of 16-bit halves, low = entering in K, high = entering in V:
//   sel:  the exit mode, as a v_perm byte selector (0x0100 = K, 0x0302 = V), so that
//         "take y's half for x's exit mode" is one v_perm_b32 with x.sel -- for y's modes,
//         record ends and boundaries alike (round 3: ~30 ops per compose -> 6);
//   cnt:  record ends passed;  last: last field boundary;  c: last NUL (one 32-bit value).
struct LFn {
  uint32_t sel, cnt, last, c;
};
constexpr uint32_t kSelK = 0x0100u, kSelV = 0x0302u;
__device__ inline LFn lfn_id() { return LFn{kSelK | (kSelV << 16), 0u, 0u, 0u}; }
__device__ inline uint32_t lfn_mode(uint32_t sel, uint32_t entry) { return (sel >> (16 * entry + 1)) & 1u; }
struct LCompose {  // x, then y
  __device__ LFn operator()(const LFn& x, const LFn& y) const {
    typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
    const uint32_t yc = __builtin_amdgcn_perm(y.cnt, y.cnt, x.sel), yl = __builtin_amdgcn_perm(y.last, y.last, x.sel);
    const u16x2 cnt = __builtin_bit_cast(u16x2, x.cnt) + __builtin_bit_cast(u16x2, yc);
    const u16x2 last = __builtin_elementwise_max(__builtin_bit_cast(u16x2, x.last), __builtin_bit_cast(u16x2, yl));
    return LFn{__builtin_amdgcn_perm(y.sel, y.sel, x.sel), __builtin_bit_cast(uint32_t, cnt),
               __builtin_bit_cast(uint32_t, last), max(x.c, y.c)};
  }
};

// The same function over the whole file (absolute positions + 1, 0: none).
struct alignas(16) GFn {
  uint32_t map, pad;
  uint64_t cnt0, cnt1, last0, last1, lnul;
};
__host__ __device__ inline GFn gfn_id() { return GFn{2u, 0u, 0, 0, 0, 0, 0}; }
struct GCompose {
  __host__ __device__ GFn operator()(const GFn& x, const GFn& y) const {
    const uint32_t mk = x.map & 1u, mv = (x.map >> 1) & 1u;
    GFn r;
    r.map = ((y.map >> mk) & 1u) | (((y.map >> mv) & 1u) << 1);
    r.pad = 0;
    r.cnt0 = x.cnt0 + (mk ? y.cnt1 : y.cnt0);
    r.cnt1 = x.cnt1 + (mv ? y.cnt1 : y.cnt0);
    const uint64_t yk = mk ? y.last1 : y.last0, yv = mv ? y.last1 : y.last0;
    r.last0 = x.last0 > yk ? x.last0 : yk;
    r.last1 = x.last1 > yv ? x.last1 : yv;
    r.lnul = x.lnul > y.lnul ? x.lnul : y.lnul;
    return r;
  }
};

struct TState {
  uint32_t m;   // mode (1 = V)
  uint64_t r;   // record being read
  uint64_t fs;  // its current field's start
  uint64_t ln;  // last NUL position + 1 (0: none)
};
__device__ inline TState gapply(const GFn& g, const TState& s) {
  TState t;
  t.m = (g.map >> s.m) & 1u;
  t.r = s.r + (s.m ? g.cnt1 : g.cnt0);
  const uint64_t l = s.m ? g.last1 : g.last0;
  t.fs = l ? l : s.fs;  // the boundary's position + 1 = the next field's start
  t.ln = s.ln > g.lnul ? s.ln : g.lnul;
  return t;
}

// lanes of the wave below this one with their bit set in b
__device__ inline uint32_t lanes_below(uint64_t b) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// Pass B: the state entering each lane's span of a wave (one pass-B unit) whose entry state
// su is known, and the record ends of the whole unit -- from ballots (round 6), instead of a
// wave scan of the span functions (hipcub, ~86 VALU per wave) and a gfn_of / gapply per
// lane.  Positions are unit-relative + 1, as in LFn.  The mode entering lane l is that of
// the nearest lane below l whose exit mode is fixed (or su.m), flipped by every lane in
// between that swaps the modes; each lane then takes its own record ends, last boundary and
// last NUL for its entry mode: the record index is a prefix count (mbcnt of one ballot per
// bit), the field start and the last NUL the nearest lane below that has one (ds_bpermute).
__device__ inline TState wave_state_in(const LFn& a, const TState& su, uint64_t base, uint32_t& ends) {
  const uint32_t l = threadIdx.x & 63u;
  const uint64_t below = (1ull << l) - 1ull;
  const uint32_t exk = lfn_mode(a.sel, 0), exv = lfn_mode(a.sel, 1);
  const uint64_t bfix = __ballot(exk == exv), bk = __ballot(exk != 0), bswap = __ballot(exk != 0 && exv == 0);
  const uint64_t mf = bfix & below;
  const uint32_t jf = mf ? 63u - (uint32_t)__builtin_clzll(mf) : 0u;  // (jf < l <= 63)
  const uint64_t flips = bswap & below & (mf ? ~((2ull << jf) - 1ull) : ~0ull);
  const uint32_t m = ((mf ? (uint32_t)(bk >> jf) : su.m) ^ (uint32_t)__builtin_popcountll(flips)) & 1u;
  const uint32_t cnt = (a.cnt >> (16 * m)) & 0xFFFFu, last = (a.last >> (16 * m)) & 0xFFFFu;
  // record ends below the lane, a ballot per bit (a packed span ends at most 3 records; a
  // span re-read from the file, up to 64: the wave-uniform test adds the other bits)
  uint32_t pc = 0;
  ends = 0;
  const uint32_t nb = __ballot(cnt > 3u) ? 7u : 2u;
  for (uint32_t b = 0; b < nb; ++b) {
    const uint64_t bb = __ballot((cnt >> b) & 1u);
    pc += lanes_below(bb) << b;
    ends += (uint32_t)__builtin_popcountll(bb) << b;
  }
  const uint64_t hl = __ballot(last != 0) & below, hn = __ballot(a.c != 0) & below;
  const uint32_t jl = hl ? 63u - (uint32_t)__builtin_clzll(hl) : 0u, jn = hn ? 63u - (uint32_t)__builtin_clzll(hn) : 0u;
  const uint32_t vl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(jl << 2), (int)last);  // (every lane)
  const uint32_t vn = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(jn << 2), (int)a.c);
  TState t;
  t.m = m;
  t.r = su.r + pc;
  t.fs = hl ? base + vl : su.fs;
  t.ln = hn ? base + vn : su.ln;  // (a NUL in the unit lies after every position before it)
  return t;
}

// Stage block `blk` into lds[PRE + 16 .. PRE + 16 + 16 KiB) with coalesced 16-byte loads
// (bytes past the file read as 0x01, no event; the 16 bytes below are chunk 0's pad for
// the hashes), and the PRE bytes before the block into lds[16 .. 16 + PRE) (block 0: 0x01).
template <uint32_t PRE>
__device__ inline void tsv_stage(const uint8_t* __restrict__ f, uint64_t size, uint64_t blk, uint8_t* lds) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t base = blk * kTChunk;
  const bool aligned = (((uintptr_t)(f + base)) & 15) == 0;
  constexpr int Q = (int)(kTChunk / 16 / kTThreads);
  const bool pre = PRE && threadIdx.x < PRE / 16;
  u32x4 pv = u32x4{0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
  if (aligned && base + kTChunk <= size) {  // block-uniform: every load in flight at once
    u32x4 v[Q];                              // (a per-piece branch waited for each in turn)
    if (pre && base) pv = *reinterpret_cast<const u32x4*>(f + base - PRE + 16 * threadIdx.x);
#pragma unroll
    for (int q = 0; q < Q; ++q)
      v[q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(f + base + 16ull * (threadIdx.x + kTThreads * q)));
    if (pre) *reinterpret_cast<u32x4*>(lds + 16 + 16 * threadIdx.x) = pv;
#pragma unroll
    for (int q = 0; q < Q; ++q) *reinterpret_cast<u32x4*>(lds + PRE + 16 + 16 * (threadIdx.x + kTThreads * q)) = v[q];
    __syncthreads();
    return;
  }
  if (pre) {
    if (base) {
      const uint8_t* p = f + base - PRE + 16 * threadIdx.x;  // (base >= 16 KiB > PRE)
      uint32_t x[4];
      for (int k = 0; k < 4; ++k)
        x[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
               ((uint32_t)p[4 * k + 3] << 24);
      pv = u32x4{x[0], x[1], x[2], x[3]};
    }
    *reinterpret_cast<u32x4*>(lds + 16 + 16 * threadIdx.x) = pv;
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const uint32_t piece = threadIdx.x + kTThreads * q;
    const uint64_t o = base + 16ull * piece;
    u32x4 v;
    if (aligned && o + 16 <= size) {
      v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(f + o));
    } else {
      uint32_t x[4];
      for (int k = 0; k < 4; ++k) {
        x[k] = 0x01010101u;
        for (int j = 0; j < 4; ++j) {
          const uint64_t i = o + 4 * k + j;
          if (i < size) x[k] = (x[k] & ~(0xFFu << (8 * j))) | ((uint32_t)f[i] << (8 * j));
        }
      }
      v = u32x4{x[0], x[1], x[2], x[3]};
    }
    *reinterpret_cast<u32x4*>(lds + PRE + 16 + 16 * piece) = v;
  }
  __syncthreads();
}

// Candidate event bytes (value < 0x0B: NUL, TAB, newline and the rare 0x01-0x08) of a
// span's 32 words as two 64-bit masks, one bit per byte in byte order.  Each word's
// candidates are bit 7 of its bytes (two ops); a v_dot4_u32_u8 gathers two words' eight
// bits into one byte (multipliers 1, 2, 4, 8 and 16, 32, 64, 128), shifted left by 7.
// (Round 3: a v_mul_lo_u32 nibble gather per word, a quarter-rate multiply, ~7.7 VALU per
// word; now ~4.5.)
// Round 6: two ops per word, not three -- (w - 0x0B0B0B0B) & ~w & 0x80808080 (v_sub, v_bitop3)
// sets bit 7 of every byte below 0x0B exactly, and of a byte 0x0B whose lower neighbour is
// below 0x0B (the borrow); such a false candidate has type 0, which every walk skips.
__device__ inline uint32_t cand_bits(uint32_t w) {
  return (w - 0x0B0B0B0Bu) & ~w & 0x80808080u;  // bit 7 of each byte < 0x0B (+ rare 0x0B)
}
__device__ inline void cand_masks(const uint32_t (&w)[32], uint64_t& m0, uint64_t& m1) {
  uint32_t mk[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = 4 * k + i;  // bytes [8p, 8p + 8)
      r[i] = __builtin_amdgcn_udot4(cand_bits(w[2 * p + 1]), 0x80402010u,
                                    __builtin_amdgcn_udot4(cand_bits(w[2 * p]), 0x08040201u, 0u, false), false);
    }
    mk[k] = (r[0] >> 7) | (r[1] << 1) | (r[2] << 9) | (r[3] << 17);
  }
  m0 = mk[0] | ((uint64_t)mk[1] << 32);
  m1 = mk[2] | ((uint64_t)mk[3] << 32);
}
// ... of the thread's 128 bytes staged in LDS.  The spans of a wave's lanes lie 128 B apart,
// so the lanes of a ds_read_b128 group (16 lanes, banks (a / 4) mod 64) reading the same
// 16-byte piece of their spans hit two bank sets: 8-way conflicts, 32 LDS cycles per read
// instead of 4 (SQ_LDS_BANK_CONFLICT 46 M cycles per call, round 4).  Lane l reads its
// pieces starting at piece (l / 2) mod 8 instead -- within every group of 16 lanes (their
// indices are distinct mod 16) each lane then has its own (span parity, piece) pair and its
// own four banks -- and the mask is rotated back: read slot q holds piece (q + s) mod 8,
// so the masks in slot order are the span's rotated right by 16 s bits.
__device__ inline void tsv_events(const uint8_t* span, uint64_t& m0, uint64_t& m1) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const uint32_t s = (threadIdx.x >> 1) & 7u;
  uint32_t w[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(span + 16 * ((q + s) & 7u));
    w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
  }
  uint64_t r0, r1;
  cand_masks(w, r0, r1);
  // rotate the 128 bits left by 16 s = right by 16 (s & 1), then left by 32 ((s + 1) / 2)
  // dwords (round 6: the 16-bit step is one alignbit per dword with a per-lane shift of 0 or
  // 16 -- alignbit(hi, lo, 0) is lo -- instead of an alignbit and a select)
  uint32_t d[4] = {(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
  uint32_t e[4];
  const uint32_t sh = 16u * (s & 1u), q = ((s + 1u) >> 1) & 3u;
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __builtin_amdgcn_alignbit(d[(i + 1) & 3], d[i], sh);
  // the dword steps as v_perm with a per-lane selector (bytes of src1 = the other dword, or
  // of src0 = this one): written as selects, hipcc turned them into a private array indexed
  // by q -- 32 bytes of scratch per lane, +23 MB of HBM writes per call
  const uint32_t p2 = (q & 2u) ? 0x03020100u : 0x07060504u, p1 = (q & 1u) ? 0x03020100u : 0x07060504u;
#pragma unroll
  for (int i = 0; i < 4; ++i) d[i] = __builtin_amdgcn_perm(e[i], e[(i + 2) & 3], p2);
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __builtin_amdgcn_perm(d[i], d[(i + 3) & 3], p1);
  m0 = e[0] | ((uint64_t)e[1] << 32);
  m1 = e[2] | ((uint64_t)e[3] << 32);
}

// Consume the lowest event of the 128-bit mask pair: its offset, or 128 when none is left.
__device__ inline uint32_t next_event(uint64_t& m0, uint64_t& m1) {
  const bool lo = m0 != 0;
  const uint64_t x = lo ? m0 : m1;
  const uint32_t b = x ? (uint32_t)__builtin_ctzll(x) + (lo ? 0u : 64u) : 128u;
  const uint64_t xn = x & (x - 1);
  m0 = lo ? xn : 0;
  m1 = lo ? m1 : xn;
  return b;
}

// Events of a thread's span: NL / TAB / NUL bytes (types 1 / 2 / 3) in byte order.  Pass A
// packs up to kEvCap of them into one word per thread for pass B: entry j = offset (7 bits)
// | type << 7 at bits [9j, 9j + 9) (unused entries 0), bit 54 set for a span with more
// (pass B reads it back from the file; the entries are then empty), and at bits [55, 63)
// the length of the head key pass A hashed for the span's first cut (0xFF: none; see
// kSlots).  Round 6: six entries, not five and a count -- the keys pass A hashes after an
// in-span newline need no length byte (pass B finds them from the entries).
constexpr uint32_t kEvCap = 6;
constexpr uint64_t kEvOver = 1ull << 54;
constexpr uint64_t kHeadNone = 0xFFull << 55;
// 0x0A -> 1, 0x09 -> 2 (TSV only: a TAB is an ordinary byte of an mdbm line), 0x00 -> 3,
// other bytes 0: two bits per byte value below 11
template <bool MDBM>
__device__ inline uint32_t ev_type(uint32_t c) {
  return c < 11u ? ((MDBM ? 0x100003u : 0x180003u) >> (2 * c)) & 3u : 0u;
}
// ... of a candidate byte (c <= 11, as the masks guarantee; 11 is the rare false candidate: type 0)
template <bool MDBM>
__device__ inline uint32_t cand_type(uint32_t c) {
  return ((MDBM ? 0x100003u : 0x180003u) >> (2 * c)) & 3u;
}

// The function of one event at position p1 (block-relative + 1), composed onto a span's
// accumulated function without branches (round 3; the per-type branches cost ~50 SALU and
// ~45 VALU instructions per event):
//   newline: entered in K, part of the key (exit K); entered in V, the record ends (exit K,
//            one record end, boundary p1);
//   TAB:     entered in K, the key ends (exit V, boundary p1); entered in V, part of the value;
//   NUL:     the last NUL; any other byte (type 0): the identity.
// mdbm (ConvertfromMdbm, tests/k2himport.cc:107-112) is the same machine with lines for
// fields: a key line and a value line alternate, so a newline entered in K ends the key
// (exit V, boundary p1) and entered in V ends the record (exit K, one record end, boundary
// p1); TABs are ordinary bytes.
template <bool MDBM>
__device__ inline LFn ev_fn(uint32_t t, uint32_t p1) {
  const bool nl = t == 1u, tab = t == 2u;
  if constexpr (MDBM)
    return LFn{nl ? (kSelV | (kSelK << 16)) : (kSelK | (kSelV << 16)), nl ? 0x10000u : 0u,
               nl ? p1 | (p1 << 16) : 0u, t == 3u ? p1 : 0u};
  return LFn{nl ? (kSelK | (kSelK << 16)) : tab ? (kSelV | (kSelV << 16)) : (kSelK | (kSelV << 16)),
             nl ? 0x10000u : 0u, nl ? p1 << 16 : tab ? p1 : 0u, t == 3u ? p1 : 0u};
}

// A span's function with one more event of type t at p1 composed onto it: LCompose(a,
// ev_fn(t, p1)) with the event's constants folded in (TSV; ~16 VALU instead of ~22).  The
// halves whose exit mode is V (sel half 0x0302: bit 1 set) take a newline's record end and
// boundary, the halves in K a TAB's boundary; positions only grow, so the max is the new one.
template <bool MDBM>
__device__ inline LFn lfn_push(const LFn& a, uint32_t t, uint32_t p1) {
  if constexpr (MDBM) return LCompose()(a, ev_fn<MDBM>(t, p1));
  const uint32_t vm = (a.sel >> 1) & 0x00010001u;  // 1 per half in V
  const uint32_t hm = vm * 0xFFFFu;                // 0xFFFF per half in V
  const bool nl = t == 1u, tab = t == 2u;
  const uint32_t take = nl ? hm : tab ? ~hm : 0u;
  return LFn{nl ? (kSelK | (kSelK << 16)) : tab ? (kSelV | (kSelV << 16)) : a.sel, a.cnt + (nl ? vm : 0u),
             (a.last & ~take) | ((p1 | (p1 << 16)) & take), t == 3u ? p1 : a.c};
}

// The function of a span's packed events (at most kEvCap, pass A's word) by table (round 5):
// it depends on their types and offsets only, so a 4096-entry table indexed by the six
// 2-bit types (0: none) gives, per entry mode, the exit mode, the record ends and the index
// of the last field boundary, plus the index of the last NUL; the offsets come from the
// word.  Pass B built it with one lfn_push per event, and a wave ran as many as its busiest
// lane (4.7 per span against a mean of 1.9).  Entry bits: 0 / 1 exit mode entering in K /
// V, [2, 4) / [4, 6) record ends, [6, 9) / [9, 12) boundary index (7: none), [12, 15) the
// last NUL's index (7: none); TSV, round 6: [15, 18), [18, 21), [21, 24) the index of the
// span's cut 0, 1, 2 when the event before it is a newline -- the in-span keys pass A
// hashes for slots 0-2 (7: none); [24, 27) the number of events; round 6, for pass A's
// newline state: [27, 30) the index of the last newline (7: none), bit 30 a cut (TAB / NUL)
// after it (or, with no newline, anywhere in the span).
template <bool MDBM>
struct SpanTab {
  uint32_t v[4096];
  constexpr SpanTab() : v() {
    for (uint32_t s = 0; s < 4096; ++s) {
      uint32_t out = 0, nul = 7, ins[3] = {7, 7, 7}, ncut = 0, prev = 0, ne = 0, lnl = 7, cut_after = 0;
      for (uint32_t m = 0; m < 2; ++m) {
        uint32_t mode = m, cnt = 0, last = 7;
        for (uint32_t i = 0; i < kEvCap; ++i) {
          const uint32_t t = (s >> (2 * i)) & 3u;
          if (t == 1u && mode == 1u) {  // a newline read in V ends the record
            ++cnt;
            last = i;
            mode = 0;
          } else if (MDBM ? t == 1u : (t == 2u && mode == 0u)) {  // the key's delimiter
            last = i;
            mode = 1;
          }
        }
        out |= (mode << m) | (cnt << (2 + 2 * m)) | (last << (6 + 3 * m));
      }
      for (uint32_t i = 0; i < kEvCap; ++i) {
        const uint32_t t = (s >> (2 * i)) & 3u;
        if (t == 3u) nul = i;
        if (!MDBM && t >= 2u) {
          if (ncut < 3 && prev == 1u) ins[ncut] = i;
          ++ncut;
        }
        ne += t ? 1u : 0u;
        if (t == 1u) lnl = i, cut_after = 0;
        if (t >= 2u) cut_after = 1;
        prev = t;
      }
      v[s] = out | (nul << 12) | (ins[0] << 15) | (ins[1] << 18) | (ins[2] << 21) | (ne << 24) | (lnl << 27) |
             (cut_after << 30);
    }
  }
};
__device__ const SpanTab<false> kSpanTabTsv{};
__device__ const SpanTab<true> kSpanTabMdbm{};
template <bool MDBM>
__device__ inline uint32_t span_tab(uint64_t pk) {
  static_assert(kEvCap == 6, "six 2-bit types index the table");
  const uint32_t lo = (uint32_t)pk, hi = (uint32_t)(pk >> 32);
  // types at bits 9 j + 7 of the word
  const uint32_t s = ((lo >> 7) & 3u) | ((lo >> 14) & 0xCu) | ((lo >> 21) & 0x30u) | ((hi << 4) & 0xC0u) |
                     ((hi >> 3) & 0x300u) | ((hi >> 10) & 0xC00u);
  return MDBM ? kSpanTabMdbm.v[s] : kSpanTabTsv.v[s];
}
template <bool MDBM>
__device__ inline LFn lfn_of_packed(uint64_t pk, uint32_t rel, uint32_t e) {
  auto p1 = [&](uint32_t i) { return i < kEvCap ? rel + ((uint32_t)(pk >> (9 * i)) & 127u) + 1u : 0u; };
  return LFn{((e & 1u) ? kSelV : kSelK) | (((e & 2u) ? kSelV : kSelK) << 16), ((e >> 2) & 3u) | (((e >> 4) & 3u) << 16),
             p1((e >> 6) & 7u) | (p1((e >> 9) & 7u) << 16), p1((e >> 12) & 7u)};
}

// Walk the candidate bytes of a span staged at `span`, calling f(offset, type) for each
// (type 0 for a candidate that is no event: f must treat it as none).
template <bool MDBM, class F>
__device__ inline void span_events(const uint8_t* span, F&& f) {
  uint64_t mm[2];
  tsv_events(span, mm[0], mm[1]);
  uint32_t o = next_event(mm[0], mm[1]), c = span[o & 127u];
  while (o < 128) {
    const uint32_t on = next_event(mm[0], mm[1]), cn = span[on & 127u];
    f(o, cand_type<MDBM>(c));
    o = on;
    c = cn;
  }
}

// Key of the C string a record stores, from LDS: raw FNV state of the key's bytes (the
// second hash of key + NUL; the first is raw * P), seed for the empty key.
__device__ inline uint64_t key_raw_lds(const uint8_t* lds_key, uint32_t len, const SpadTable& sp) {
  if (!len) return sp.v[0];
  const uint32_t k = (len + 15) / 16, p = 16 * k - len;
  const uint8_t* c0 = lds_key - p;
  uint4 c = ld16(c0);
  const uint32_t m0 = p >= 4 ? 0u : ~0u << (8 * p), m1 = p >= 8 ? 0u : p <= 4 ? ~0u : ~0u << (8 * (p - 4));
  const uint32_t m2 = p >= 12 ? 0u : p <= 8 ? ~0u : ~0u << (8 * (p - 8)), m3 = p <= 12 ? ~0u : ~0u << (8 * (p - 12));
  c.x &= m0, c.y &= m1, c.z &= m2, c.w &= m3;
  uint32_t lo = (uint32_t)sp.v[p], hi = (uint32_t)(sp.v[p] >> 32);
  for (uint32_t q = 1; q < k; ++q) {
    const uint4 nx = ld16(c0 + 16 * q);
    fnv_chunk16(lo, hi, c);
    c = nx;
  }
  fnv_chunk16(lo, hi, c);
  return ((uint64_t)hi << 32) | lo;
}

// Speculative keys: pass A does not know the mode at its block's start, but a key starts
// exactly after every newline the value getline reads, and ends at the first TAB or NUL
// after it (the key getline's TAB, or the C-string cut).  So for the span's first three cut
// events (TAB / NUL) that follow a newline of the same span, pass A hashes the bytes between
// them (round 6: three, not two; such a key needs no length byte -- pass B finds it from
// the packed events, the newline just before the cut), plus the head key below, whose
// length rides in the packed word.  Pass B, whose walk ends a key at cut event c of its
// span, takes slot c when the key's true length equals the slot's (same end, same length:
// the same bytes); every other key (one whose newline is in an earlier block beyond the
// head key's reach, a fourth cut in one span, a span with more than kEvCap events, a key of
// 255 bytes or more, a wave's slots past kUnitSlots) is hashed from the file.
// Round 4: slots indexed by span, so pass B loads its states with its packed word instead
// of after it (round 3: a per-block list indexed from the packed word, 10 B per key -- a
// second dependent HBM round trip at the start of every pass-B wave).
constexpr uint32_t kSlots = 2;  // slot states per span on average that a unit's region holds
// The head key: the key that ends at a block's first cut event when no newline precedes it
// in the block started in the bytes before the block (a key straddling the boundary, ~1 in
// 4 blocks on BASELINE-like files).  Pass A stages kPre bytes before the block too and
// hashes it from the byte after the last newline among them (start < 0, block-relative);
// before round 4 pass B hashed every such key from the file, one lane holding its wave
// (~47 us of a 0.62 ms call, profiles/r04d_import_probes.txt).  Block 0's head key starts
// at the file's first byte.  Round 6: 64 bytes, not 256 -- a head key of length L ending at
// block offset c is found when L <= c + 63 (every key of up to 64 bytes but one ending at
// offset 0), and the re-read of the bytes before each block drops from 1.6 % of the file to
// 0.4 %; a longer head key is hashed from the file in pass B.
constexpr uint32_t kPre = 64;
constexpr uint32_t kSpecLenMax = 254;  // longest key a slot holds (0xFF: no slot)
// Each span's slots: the FNV state after the key's bytes (h2 of key + NUL; h1 = raw * P)
// at raw[kSlots * span + j], written only for the slots its packed word names.
// Round 6: a unit's named slots are stored compacted, in span order (slot 0 before slot 1),
// at the front of the unit's region raw[kUnitSlots * unit ..]; pass B finds a span's entry
// from the named slots of the spans before it in its wave (slot_rank).
constexpr uint32_t kUnitSlots = 64 * kSlots;
struct SpecSlots {
  uint64_t* raw;  // [nblk * kUnitsPerBlock * kUnitSlots]
};
// A lane's named slots and their rank among its wave's: entries p (slot 0, if v0), p + v0
// (slot 1, if v1) and p + v0 + v1 (slot 2, if v2); n = the wave's total.  Only entries below
// kUnitSlots are stored (pass A) and taken (pass B); a key past them is hashed from the file.
struct SlotRank {
  uint32_t v0, v1, v2, p, n;
};
__device__ inline SlotRank slot_rank(bool v0, bool v1, bool v2) {
  const uint64_t b0 = __ballot(v0), b1 = __ballot(v1), b2 = __ballot(v2);
  return SlotRank{v0 ? 1u : 0u, v1 ? 1u : 0u, v2 ? 1u : 0u, lanes_below(b0) + lanes_below(b1) + lanes_below(b2),
                  (uint32_t)(__builtin_popcountll(b0) + __builtin_popcountll(b1) + __builtin_popcountll(b2))};
}

// Newline state of a span for the speculative keys: whether it holds a newline, whether
// the last one is still open (no cut after it), and its block-relative position; composed
// in file order (a later newline resets, a cut closes).
// (bit 0: has newline, bit 1: open, bits [2, 18): last newline position; identity 2.)
// compose(x, y) = y if y has a newline, else x with bit 1 cleared when y holds a cut.
// The block's exclusive prefix from two ballots (round 6; a hipcub block scan before, ~50
// VALU per wave of DPP steps and selects): a lane's prefix is the state of the nearest lane
// below it with a newline (fetched by ds_bpermute), closed if a lane in between holds a cut;
// with none below, the previous wave's aggregate (or the identity), closed likewise.  The
// waves' aggregates pass through s_agg under one barrier.
__device__ inline uint32_t nl_prefix_block(uint32_t v, uint32_t* s_agg) {
  const uint32_t l = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t bnl = __ballot((v & 1u) != 0), bcut = __ballot((v & 2u) == 0);
  // the wave's aggregate: its last newline lane, closed by a cut in a later lane
  uint32_t agg = (bcut != 0) ? 0u : 2u;
  if (bnl) {
    const uint32_t ja = 63u - (uint32_t)__builtin_clzll(bnl);
    const uint32_t vj = __builtin_amdgcn_readlane(v, ja);
    agg = ((bcut >> ja) >> 1) ? (vj & ~2u) : vj;
  }
  static_assert(kTThreads == 128, "two waves");
  if (threadIdx.x == 0) *s_agg = agg;
  __syncthreads();
  const uint32_t prev = w ? *s_agg : 2u;
  const uint64_t below = (1ull << l) - 1ull;
  const uint64_t m = bnl & below, cb = bcut & below;
  const uint32_t j = m ? 63u - (uint32_t)__builtin_clzll(m) : 0u;
  const uint32_t vj = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j << 2), (int)v);  // (every lane)
  const bool closed = m ? ((cb >> j) >> 1) != 0 : cb != 0;
  const uint32_t p = m ? vj : prev;
  return closed ? (p & ~2u) : p;
}

// A wave's function over the whole file (every lane gets it): pass A needs only the
// composition of its span functions (pass B rebuilds the per-span states), and each wave
// writes its own 8 KiB unit's (round 4).  Round 6: from ballots, as in wave_state_in, for
// both entry modes -- each lane's entry mode (the nearest fixed-exit lane below it, flipped
// by the swapping lanes in between), the record ends summed per bit, the last boundary and
// NUL taken from the highest lane that has one -- instead of a DPP reduction of the LFn
// (hipcub WarpReduce, ~60 VALU per wave).  Positions are block-relative + 1.
__device__ inline GFn wave_gfn(const LFn& a, uint64_t base) {
  const uint32_t l = threadIdx.x & 63u;
  const uint64_t below = (1ull << l) - 1ull;
  const uint32_t exk = lfn_mode(a.sel, 0), exv = lfn_mode(a.sel, 1);
  const uint64_t bfix = __ballot(exk == exv), bk = __ballot(exk != 0), bswap = __ballot(exk != 0 && exv == 0);
  const uint64_t mf = bfix & below;
  const uint32_t jf = mf ? 63u - (uint32_t)__builtin_clzll(mf) : 0u;
  const uint32_t par = (uint32_t)__builtin_popcountll(bswap & below & (mf ? ~((2ull << jf) - 1ull) : ~0ull)) & 1u;
  // the lane's entry mode when the wave enters in K (m0) or V (m1)
  const uint32_t m0 = mf ? ((uint32_t)(bk >> jf) ^ par) & 1u : par, m1 = mf ? m0 : par ^ 1u;
  const uint32_t c0 = (a.cnt >> (16 * m0)) & 0xFFFFu, c1 = (a.cnt >> (16 * m1)) & 0xFFFFu;
  const uint32_t l0 = (a.last >> (16 * m0)) & 0xFFFFu, l1 = (a.last >> (16 * m1)) & 0xFFFFu;
  GFn g = gfn_id();
  // the exit modes: the wave's last fixed-exit lane, flipped by the swapping lanes after it
  const uint32_t jw = bfix ? 63u - (uint32_t)__builtin_clzll(bfix) : 0u;
  const uint32_t pw = (uint32_t)__builtin_popcountll(bswap & (bfix ? ~((2ull << jw) - 1ull) : ~0ull)) & 1u;
  const uint32_t x0 = bfix ? ((uint32_t)(bk >> jw) ^ pw) & 1u : pw, x1 = bfix ? x0 : pw ^ 1u;
  g.map = x0 | (x1 << 1);
  // record ends (a span of at most kEvCap events ends at most 3; more from a longer span)
  const uint32_t nb = __ballot((c0 | c1) > 3u) ? 7u : 2u;
  uint64_t n0 = 0, n1 = 0;
  for (uint32_t b = 0; b < nb; ++b) {
    n0 += (uint64_t)__builtin_popcountll(__ballot((c0 >> b) & 1u)) << b;
    n1 += (uint64_t)__builtin_popcountll(__ballot((c1 >> b) & 1u)) << b;
  }
  g.cnt0 = n0;
  g.cnt1 = n1;
  const uint64_t h0 = __ballot(l0 != 0), h1 = __ballot(l1 != 0), hn = __ballot(a.c != 0);
  if (h0) g.last0 = base + __builtin_amdgcn_readlane(l0, 63 - __builtin_clzll(h0));
  if (h1) g.last1 = base + __builtin_amdgcn_readlane(l1, 63 - __builtin_clzll(h1));
  if (hn) g.lnul = base + __builtin_amdgcn_readlane(a.c, 63 - __builtin_clzll(hn));
  return g;
}

// Entry states of the blocks (tsv_scan_kernel, one launch instead of a device scan and a
// count kernel): blocks form tiles of kTile, each tile scanned by one block into each
// block's in-tile prefix; the last tile to finish scans the tile functions into each
// tile's entry state and the record count (the state after the whole file, plus the
// record a value getline ends at EOF).  The counter is zero between calls: the last
// block resets it.
constexpr uint32_t kTilePer = 4;
constexpr uint32_t kTile = kTilePer * kTThreads;  // blocks per tile
struct EntryScan {
  GFn* blk_fn;         // [2 nblk] each pass-B unit's (pass A wave's) function
  GFn* intile;         // [2 nblk] exclusive prefix of each unit's function within its tile
  GFn* tile_fn;        // [ntile]
  TState* tile_in;     // [ntile] state entering the tile
  uint32_t* done;      // tiles finished, zero between calls
  uint64_t* count;     // records in the file
  uint64_t* host_count;  // the same, into mapped pinned host memory (no read-back copy)
  uint64_t nblk, ntile;
  uint64_t size;
  uint32_t mdbm;  // the mdbm machine: starts in V (see kHdrRecs), counts a key line at EOF
};
// mdbm: the machine starts in mode V at the file's first byte, so the five header lines are
// "records" 0 (its value line 0), 1 (lines 1-2) and 2 (lines 3-4), and the key line after
// the header starts record kHdrRecs -- real record r is machine record r + kHdrRecs.  The
// fifth header line is record 2's value line (checked in pass B).
constexpr uint64_t kHdrRecs = 3;
constexpr uint32_t kStageRecs = 96;  // records a pass-B unit stages in LDS (BASELINE-like files: ~60 per 8 KiB)

// Exclusive scan of in(0) .. in(n - 1) by one block, thread t owning the run [t k, (t + 1) k):
// out(i, prefix of in(0 .. i - 1)); returns the whole reduction.  Runs of up to 4 are loaded
// at once and kept in registers (the tile scan's 4 and the tile-level scan of files up to
// 4 GiB); longer runs re-read their elements.
template <class Tmp, class In, class Out>
__device__ inline GFn block_scan_runs(Tmp& tmp, In&& in, uint64_t n, uint64_t k, Out&& out) {
  typedef hipcub::BlockScan<GFn, kTThreads, hipcub::BLOCK_SCAN_WARP_SCANS> GScan;
  const uint64_t i0 = (uint64_t)threadIdx.x * k, i1 = min(i0 + k, n);
  GFn x[4];
  GFn loc = gfn_id();
  if (k <= 4) {
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) x[q] = i0 + q < i1 ? in(i0 + q) : gfn_id();
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) loc = GCompose()(loc, x[q]);
  } else {
    for (uint64_t i = i0; i < i1; ++i) loc = GCompose()(loc, in(i));
  }
  GFn pre, agg;
  GScan(tmp).ExclusiveScan(loc, pre, gfn_id(), GCompose(), agg);
  if (k <= 4) {
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q)
      if (i0 + q < i1) {
        out(i0 + q, pre);
        pre = GCompose()(pre, x[q]);
      }
  } else {
    for (uint64_t i = i0; i < i1; ++i) {
      out(i, pre);
      pre = GCompose()(pre, in(i));
    }
  }
  return agg;
}

// Pass A: each block's function (for tsv_scan_kernel), each thread's packed events, and
// the speculative key states (TSV only: which mdbm lines are keys depends on the line
// count before the block, so pass B hashes mdbm keys from the file).
template <bool MDBM>
__global__ __launch_bounds__(kTThreads) void tsv_a_kernel(const uint8_t* __restrict__ f, uint64_t size,
                                                          GFn* __restrict__ blk_fn, uint64_t* __restrict__ ev,
                                                          SpecSlots spec, SpadTable sp) {
  constexpr uint32_t PRE = MDBM ? 0u : kPre;
  __shared__ __attribute__((aligned(16))) uint8_t lds[16 + PRE + kTChunk];
  // The block's speculative keys in chunk-count order, one word each: start (16 bits,
  // signed) | len << 16 | entry << 24, entry = the key's place in its unit's compacted slot
  // list (wave << 7 | rank, round 6; before: span * kSlots + cut index).  A span's (at most
  // kSlots) keys stay in its lane's registers until the sort (round 4; round 3: a list
  // filled by LDS atomics inside the event walk, each append a wave-wide wait for its
  // return).  (The block's LDS must stay within 17.5 KiB for 9 blocks per CU -- one
  // 512-byte granule more gave 8 and cost pass A 11 %, round 4.)
  __shared__ uint32_t s_sorted[kTThreads * kSlots];
  __shared__ uint32_t s_cls[8];        // keys per chunk-count class, then class offsets
  __shared__ uint32_t s_nlagg;  // wave 0's newline aggregate (nl_prefix_block)
  uint8_t* blk = lds + PRE;  // block byte i at blk[16 + i]; the kPre bytes before the block below it
  const uint64_t bid = blockIdx.x;
  if (threadIdx.x < 8) s_cls[threadIdx.x] = 0;
  const uint64_t base = bid * kTChunk;
  tsv_stage<PRE>(f, size, bid, lds);  // (its barrier publishes s_cls = 0)
  const uint32_t rel = kTBytes * threadIdx.x;
  const uint8_t* span = blk + 16 + rel;
  const bool live = base + rel < size;
  LFn acc = lfn_id();
  // the span's events, newest at bits [45, 54) and the older ones moved down 9 bits each
  // (round 6: one 64-bit shift per event instead of a variable shift and two guards); a span
  // of ne <= kEvCap events holds them at [54 - 9 ne, 54) after the walk, shifted down then
  uint64_t pk = 0;
  uint32_t ne = 0;
  // Speculative keys (round 4; round 3 walked the packed events a second time after the
  // block scan): a cut that follows a newline of this span ends the key that starts after
  // it; the span's first cut, if no newline precedes it here, waits for the scan (cut0) --
  // the entering state decides whether it ends a key, and where that key starts.  Round 6:
  // the walk only packs the events (a wave walks as many as its busiest lane, 2.5x the mean,
  // so each per-event instruction counts 2.5 times); the cuts, their keys and the span's
  // newline state are read off the packed word and its span_tab entry after the walk (a
  // span of more than kEvCap events names no key and reports no newline: only misses).
  constexpr uint32_t kNoKey = 0xFFFFFFFFu;
  uint32_t key0 = kNoKey, key1 = kNoKey, key2 = kNoKey;  // the span's keys at cuts 0-2: start | len << 16
  if (live)
    span_events<MDBM>(span, [&](uint32_t o, uint32_t t) {  // branch-free: t == 0 changes nothing
      // (selects throughout: the branches hipcc made of these cost ~40 SALU per event)
      pk = t ? (pk >> 9) | ((uint64_t)(o | (t << 7)) << 45) : pk;
      ne += t ? 1u : 0u;
    });
  const bool over = ne > kEvCap;
  pk = over ? kEvOver : pk >> (9 * (kEvCap - ne));
  // The span's function by table from the packed word, as pass B builds it (round 6; the
  // walk composed it per event, ~12 VALU each); a span of more than kEvCap events (rare)
  // walks its candidates again for it.
  const uint32_t te = span_tab<MDBM>(pk);
  acc = lfn_of_packed<MDBM>(pk, rel, te);
  if (over) {
    acc = lfn_id();
    span_events<MDBM>(span, [&](uint32_t o, uint32_t t) { acc = lfn_push<MDBM>(acc, t, rel + o + 1); });
  }
  uint32_t head_len = 0xFFu;  // the head key's length byte
  uint32_t cut0 = 0xFFFFFFFFu;  // the span's first cut when no newline precedes it
  uint32_t nl = 2u;  // newline state (NlSum): no newline, no cut
  if constexpr (!MDBM) {
    auto off = [&](uint32_t i) { return (uint32_t)(pk >> (9 * i)) & 127u; };
    uint32_t kk[3];
#pragma unroll
    for (uint32_t h = 0; h < 3; ++h) {
      const uint32_t x = (te >> (15 + 3 * h)) & 7u;  // cut h's event, a newline before it (7: none)
      const uint32_t st = off(x - 1u) + 1u;             // (x >= 1 when named)
      // (no length byte: pass B finds these keys from the packed events; in-span, len < 128)
      kk[h] = (x != 7u && !over) ? (rel + st) | ((off(x) - st) << 16) : kNoKey;
    }
    key0 = kk[0], key1 = kk[1], key2 = kk[2];
    cut0 = (!over && ne && (pk & 0x100u)) ? rel + off(0) : cut0;  // event 0 a cut (type >= 2: bit 8)
    const uint32_t lx = (te >> 27) & 7u, ca = (te >> 30) & 1u;
    nl = over ? 0u : lx != 7u ? 1u | (ca ? 0u : 2u) | ((rel + off(lx)) << 2) : (ca ? 0u : 2u);
  }
  const GFn wf = wave_gfn(acc, base);
  if ((threadIdx.x & 63u) == 0) blk_fn[bid * kUnitsPerBlock + (threadIdx.x >> 6)] = wf;
  if constexpr (MDBM) {
    ev[base / kTBytes + threadIdx.x] = pk | kHeadNone;
    return;
  }
  const uint32_t pre_nl = nl_prefix_block(live ? nl : 2u, &s_nlagg);
  // cut0 ends a key if the state entering the span is a newline with no cut after it
  // (open), or if nothing precedes the span in the block (head: the key started before the
  // block, after the last newline of the kPre bytes before it; block 0: at the file's start)
  const bool open = (pre_nl & 3u) == 3u, head = pre_nl == 2u;
  if (cut0 != 0xFFFFFFFFu && (open || head)) {
    bool ok = true;
    int32_t start = (int32_t)(pre_nl >> 2) + 1;
    if (head) {
      ok = base == 0;
      start = 0;
      for (int32_t w = (int32_t)PRE / 16 - 1; w >= 0 && !ok; --w) {
        const uint4 c = ld16(lds + 16 + 16 * w);
        const uint32_t wd[4] = {c.x, c.y, c.z, c.w};
        for (int32_t k = 3; k >= 0 && !ok; --k) {
          const uint32_t x = wd[k] ^ 0x0A0A0A0Au;
          const uint32_t m = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // bit 7 of 0x0A bytes
          if (m) {
            start = 16 * w + 4 * k + (31 - (int32_t)__clz(m)) / 8 + 1 - (int32_t)PRE;
            ok = true;
          }
        }
      }
    }
    const uint32_t len = (uint32_t)((int32_t)cut0 - start);
    if (ok && len <= kSpecLenMax) {
      key0 = ((uint32_t)start & 0xFFFFu) | (len << 16);
      head_len = len;
    }
  }
  // (a span with more than kEvCap events keeps its head key: pass B reads its length byte)
  ev[base / kTBytes + threadIdx.x] = pk | ((uint64_t)head_len << 55);
  // The keys in order of chunk count (counting sort over 8 classes), so that each wave's
  // hash loop runs as long as ITS longest key: on BASELINE-like files (keys 8-64 B, 1-4
  // chunks) wave 0 takes the short keys and runs 2 chunks instead of 4 (round 4).
  static_assert(kSpecLenMax < 256 && kUnitSlots * (kTThreads / 64) <= 256, "slot | len | start in 32 bits");
  // each key's entry in its unit's compacted slot list (span order; see SpecSlots): wave
  // bit 7, rank bits 0-6 -- carried in the sorted word instead of the raw slot index, so
  // the hashing lane stores the state straight into its compacted place (round 6); a wave's
  // entries past kUnitSlots are not hashed (pass B ranks the same way)
  const SlotRank sr = slot_rank(key0 != kNoKey, key1 != kNoKey, key2 != kNoKey);
  const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63u;
  const uint32_t rk[3] = {sr.p, sr.p + sr.v0, sr.p + sr.v0 + sr.v1};
  uint32_t cls[3], kk[3] = {key0, key1, key2};
#pragma unroll
  for (uint32_t h = 0; h < 3; ++h) {
    kk[h] = rk[h] < kUnitSlots ? kk[h] : kNoKey;
    cls[h] = (min(max((kk[h] >> 16) & 0xFFu, 1u), 128u) - 1u) >> 4;  // chunk-count class 0..7
    if (kk[h] != kNoKey) atomicAdd(&s_cls[cls[h]], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0;
#pragma unroll
    for (uint32_t c = 0; c < 8; ++c) {
      const uint32_t v = s_cls[c];
      s_cls[c] = a;
      a += v;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t h = 0; h < 3; ++h)
    if (kk[h] != kNoKey) s_sorted[atomicAdd(&s_cls[cls[h]], 1u)] = kk[h] | (((wv << 7) | rk[h]) << 24);
  __syncthreads();
  const uint32_t nk = s_cls[7];  // (each class's offset has moved to its end: the last is the count)
  // Right-aligned (round 6): the first round takes the LONGEST min(nk, 128) keys, lane 127
  // the longest, and a second round the rest (nk > 128), so wave 1 runs the long keys and
  // wave 0 only the nk - 64 shortest (~49 of ~113 on BASELINE-like files: their chunk count,
  // not the 64th key's); left-aligned, wave 0 ran keys 0-63 and wave 1 the 49 longest.
  uint64_t raw[2];
  uint32_t slot[2];
#pragma unroll
  for (uint32_t h = 0; h < 2; ++h) {
    const uint32_t q = h ? threadIdx.x : threadIdx.x + nk - kTThreads;  // (h = 0: valid from lane 128 - nk)
    slot[h] = 0xFFFFFFFFu;
    if (h ? q + kTThreads < nk : threadIdx.x + nk >= kTThreads) {
      const uint32_t k = s_sorted[q];
      raw[h] = key_raw_lds(blk + 16 + (int16_t)(k & 0xFFFFu), (k >> 16) & 0xFFu, sp);
      slot[h] = k >> 24;
    }
  }
  // The states go out compacted per unit (round 6): each wave's (pass-B unit's) named slots
  // in span order at the front of the unit's region of kUnitSlots entries, written as
  // consecutive 8-byte pieces across the wave -- only the ~60 states a unit holds, not 16 B
  // for each of its 64 spans (round 5: 1.34x the algorithmic bytes per call, over half of
  // the excess these slots).  Through the staged block's LDS, free once every key is hashed.
  __syncthreads();
  uint64_t* s_comp = reinterpret_cast<uint64_t*>(lds);  // [kTThreads / 64][kUnitSlots]
  static_assert(kUnitSlots == 128 && kTThreads / 64 <= 2, "wave bit 7 | rank bits 0-6");
#pragma unroll
  for (uint32_t h = 0; h < 2; ++h)
    if (slot[h] != 0xFFFFFFFFu) s_comp[slot[h]] = raw[h];
  __syncthreads();
  uint64_t* dst = spec.raw + (bid * kUnitsPerBlock + wv) * kUnitSlots;
  const uint32_t nst = min(sr.n, kUnitSlots);
  if (ln < nst) dst[ln] = s_comp[kUnitSlots * wv + ln];
  if (ln + 64u < nst) dst[ln + 64u] = s_comp[kUnitSlots * wv + ln + 64u];
}

// The entry-state scan between the passes, one block per tile: the tile's functions into
// each block's in-tile prefix; the last tile to finish (an arrival counter) scans the tile
// functions into each tile's entry state and the record count.  (Inside pass A this cost
// 3.4 ms instead of 0.45: an agent-scope release per 16 KiB block writes back the XCD's
// L2 each time, r03i.)
__global__ __launch_bounds__(kTThreads) void tsv_scan_kernel(EntryScan es) {
  typedef hipcub::BlockScan<GFn, kTThreads, hipcub::BLOCK_SCAN_WARP_SCANS> GScan;
  __shared__ typename GScan::TempStorage gtmp;
  __shared__ uint32_t s_last;
  const uint64_t tile = blockIdx.x, b0 = tile * kTile;
  // items are pass A's blocks, each the composition of its two waves' functions; each
  // block's prefix is written for both of its pass-B units (the second one past wave 0)
  const GFn* wfn = es.blk_fn + kUnitsPerBlock * b0;
  const GFn tf = block_scan_runs(
      gtmp, [&](uint64_t i) { return GCompose()(wfn[2 * i], wfn[2 * i + 1]); },
      min<uint64_t>(kTile, es.nblk - b0), kTilePer, [&](uint64_t i, const GFn& p) {
        es.intile[kUnitsPerBlock * (b0 + i)] = p;
        es.intile[kUnitsPerBlock * (b0 + i) + 1] = GCompose()(p, wfn[2 * i]);
      });
  static_assert(kUnitsPerBlock == 2, "two pass-B units per pass-A block");
  if (threadIdx.x == 0) {
    es.tile_fn[tile] = tf;
    __threadfence();
    s_last = atomicAdd(es.done, 1u) == es.ntile - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();  // acquire: every tile's function
  const uint64_t k = (es.ntile + kTThreads - 1) / kTThreads;
  const TState s0{es.mdbm, 0, 0, 0};
  const GFn all = block_scan_runs(gtmp, [&](uint64_t i) { return es.tile_fn[i]; }, es.ntile, k,
                                  [&](uint64_t i, const GFn& p) { es.tile_in[i] = gapply(p, s0); });
  if (threadIdx.x == 0) {
    const TState e = gapply(all, s0);
    // a value getline at EOF ends one more record; mdbm: so does a key line that ends at EOF
    // with bytes in it (tests/k2himport.cc:107-112: the key getline extracts them)
    uint64_t n = e.r + e.m;
    if (es.mdbm) {
      n += (!e.m && e.fs < es.size) ? 1u : 0u;
      n = n > kHdrRecs ? n - kHdrRecs : 0u;
    }
    es.count[0] = n;
    __hip_atomic_store(es.host_count, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    es.done[0] = 0;
  }
}

// Pass B: each thread's events (packed by pass A, or re-read from the file for a span with
// more than kEvCap), the block scan of the span functions again (from the events: no
// prefixes stored), the walk, the records, and every key's h1 / h2 -- pass A's state when
// its slot matches the key, else hashed from the file.  Fields are written only for
// records below min(count, cap), so a key cut off by EOF writes nothing.
// mdbm (MDBM): records are machine records - kHdrRecs; the thread that ends machine record
// 2's value line checks the fifth header line ("HEADER=END", tests/k2himport.cc:101-104)
// and sets hflags[1]; a last key line that ends at EOF takes the previous record's value
// (getline leaves the string as it was when it fails at EOF) -- the first record's
// directly, any later one by the host after the call (hflags[2], a 16-byte copy).
template <bool HASH, bool MDBM>
__global__ __launch_bounds__(64) void tsv_b_kernel(const uint8_t* __restrict__ f, uint64_t size,
                                                          const GFn* __restrict__ intile,
                                                          const TState* __restrict__ tile_in,
                                                          const uint64_t* __restrict__ ev,
                                                          const uint64_t* __restrict__ spec_raw,
                                                          const uint64_t* __restrict__ count, uint64_t cap,
                                                          k2h_amd_import_rec* __restrict__ recs, SpadTable sp,
                                                          uint64_t* __restrict__ h1, uint64_t* __restrict__ h2,
                                                          uint64_t* __restrict__ hflags) {
  // one wave per 8 KiB unit: the state entering each span from ballots (wave_state_in)
  // The unit's records, staged in LDS and written out as consecutive 16-byte pieces across
  // the wave (round 4; round 3: each lane stored its own records' halves, 1.31x the
  // algorithmic bytes written).  A unit with more than kStageRecs records stores directly.
  // (row kStageRecs: the dump row of the branch-free walk)
  __shared__ __attribute__((aligned(16))) uint64_t s_rec[(kStageRecs + 1) * 4];  // key_off, key_len, val_off, val_len
  // the lanes' slot states (3 per lane; round 6: the walk records which slot a key takes, and
  // the hashes are made from them as they are stored, instead of per event inside the walk)
  __shared__ uint64_t s_slot[64 * 3];
  // which parts this unit wrote; s_fh: a key's slot + 1 (its state in s_slot), 0xFF: hashed
  // from the file, 0: no key of this unit
  __shared__ uint8_t s_fk[kStageRecs + 1], s_fv[kStageRecs + 1], s_fh[kStageRecs + 1];
  constexpr uint64_t HDR = MDBM ? kHdrRecs : 0;
  const uint64_t base = (uint64_t)blockIdx.x * kUnit;
  const uint64_t blk = blockIdx.x / kUnitsPerBlock;  // pass A's block
  const uint32_t rel = kTBytes * threadIdx.x;
  const bool live = base + rel < size;
  const uint64_t ti = base / kTBytes + threadIdx.x;
  const uint64_t pk = ev[ti];
  const GFn ein = intile[blockIdx.x];
  const TState tin = tile_in[blk / kTile];
  const bool over = (pk & kEvOver) != 0;
  // The unit's compacted slot states (pass A): the first 64 loaded with the packed word, at
  // a fixed address (no dependent round trip); a span takes its entries from the lanes that
  // hold them once its packed word shows the named slots before it (a slot not named holds
  // 0, used only when the packed word names it).
  // a span's slots: their states and the key length each holds, 8 bits per slot (0xFF:
  // none; slots 0-1 from the packed word, slot 2 -- the third cut's key, when a newline is
  // the event before it -- found from the packed events, round 6)
  const uint32_t te = span_tab<MDBM>(pk);
  uint32_t slen = 0xFFFFFFu;
  uint64_t e_lo = 0;
  if constexpr (HASH && !MDBM) e_lo = spec_raw[(uint64_t)kUnitSlots * blockIdx.x + threadIdx.x];
  // a span with more than kEvCap events (rare): its candidate masks from the file, each
  // candidate's byte read back (no LDS, so the kernel keeps its occupancy)
  uint64_t om0 = 0, om1 = 0;
  if (over && live) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint32_t w[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint64_t o = base + rel + 16ull * q;
      if (o + 16 <= size && (((uintptr_t)(f + o)) & 15) == 0) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(f + o);
        w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
      } else {
        for (int k = 0; k < 4; ++k) {
          uint32_t x = 0x01010101u;
          for (int b = 0; b < 4; ++b)
            if (o + 4 * k + b < size) x = (x & ~(0xFFu << (8 * b))) | ((uint32_t)f[o + 4 * k + b] << (8 * b));
          w[4 * q + k] = x;
        }
      }
    }
    cand_masks(w, om0, om1);
  }
  if constexpr (HASH && !MDBM) {
    // slot c: the key at cut c that starts after the newline just before it (event index
    // i_c from the table; its length from the two offsets), or slot 0's head key (its byte)
    auto inspan = [&](uint32_t i) {
      return i < kEvCap ? ((uint32_t)(pk >> (9 * i)) & 127u) - ((uint32_t)(pk >> (9 * i - 9)) & 127u) - 1u : 0xFFu;
    };
    const uint32_t hb = (uint32_t)(pk >> 55) & 0xFFu;
    const uint32_t b0 = hb != 0xFFu ? hb : inspan((te >> 15) & 7u), b1 = inspan((te >> 18) & 7u),
                   b2 = inspan((te >> 21) & 7u);
    const SlotRank sr = slot_rank(b0 != 0xFFu, b1 != 0xFFu, b2 != 0xFFu);
    uint64_t e_hi = 0;
    if (sr.n > 64u) e_hi = spec_raw[(uint64_t)kUnitSlots * blockIdx.x + 64u + threadIdx.x];  // wave-uniform, rare
    auto pick = [&](uint32_t idx) -> uint64_t {  // entry idx of the unit, from the lane that loaded it
      const int a = (int)((idx & 63u) << 2);
      uint64_t v = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(e_lo >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)e_lo);
      if (sr.n > 64u) {
        const uint64_t w = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(e_hi >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)e_hi);
        v = idx < 64u ? v : w;
      }
      return v;
    };
    const uint32_t p1 = sr.p + sr.v0, p2 = p1 + sr.v1;
    s_slot[3 * threadIdx.x] = pick(sr.p);  // (all lanes: bpermute reads every lane)
    s_slot[3 * threadIdx.x + 1] = pick(p1);
    s_slot[3 * threadIdx.x + 2] = pick(p2);
    slen = (sr.p < kUnitSlots ? b0 : 0xFFu) | ((p1 < kUnitSlots ? b1 : 0xFFu) << 8) |
           ((p2 < kUnitSlots ? b2 : 0xFFu) << 16);
  }
  auto for_events = [&](auto&& fn) {
    if (!live) return;
    if (over) {
      uint64_t m0 = om0, m1 = om1;
      for (uint32_t o = next_event(m0, m1); o < 128 && base + rel + o < size; o = next_event(m0, m1)) {
        const uint32_t t = ev_type<MDBM>(f[base + rel + o]);  // (bytes past the file are 0x01 in the masks)
        if (t) fn(o, t);
      }
    } else {
      const uint32_t ne = (te >> 24) & 7u;
      for (uint32_t j = 0; j < ne; ++j) {
        const uint32_t e = (uint32_t)(pk >> (9 * j)) & 0x1FFu;
        fn(e & 127u, e >> 7);
      }
    }
  };
  LFn acc = lfn_of_packed<MDBM>(pk, rel, te);  // (a span past the file: no events, the identity)
  if (over) {  // more than kEvCap events (rare): from the file
    acc = lfn_id();
    for_events([&](uint32_t o, uint32_t t) { acc = lfn_push<MDBM>(acc, t, rel + o + 1); });
  }
  const TState su = gapply(ein, tin);  // the state entering the unit
  uint32_t ends;
  TState s = wave_state_in(acc, su, base, ends);
  const uint64_t lim = min(count[0], cap) + HDR;  // machine record indices below lim are written
  // the unit touches records su.r .. su.r + (its record ends), the last one possibly in part
  const uint32_t nrec = ends + 1u;
  const bool staged = nrec <= kStageRecs;
  if (staged)
    for (uint32_t q = threadIdx.x; q < nrec; q += 64) s_fk[q] = s_fv[q] = s_fh[q] = 0;
  __syncthreads();
  bool nulf = s.ln > s.fs;  // a NUL already cut the current field
  uint32_t j = 0;  // cut events of this span so far (slot j's length: byte j of slen)
  typedef uint64_t u64x2 __attribute__((ext_vector_type(2), aligned(8)));  // recs: 8-byte aligned
  auto key_end = [&](uint64_t e) {
    if (s.r < HDR || s.r >= lim) return;
    const uint64_t r = s.r - HDR;
    const uint32_t x = (uint32_t)(s.r - su.r);  // staged: its index in the unit
    if (staged) {
      s_rec[4 * x] = s.fs;
      s_rec[4 * x + 1] = e - s.fs;
      s_fk[x] = 1;
    } else {  // a unit with more records than the stage (rare): the key half straight out
      *reinterpret_cast<u64x2*>(&recs[r].key_off) = u64x2{s.fs, e - s.fs};
    }
    if constexpr (HASH) {
      // pass A's key for this cut event, if its length is this key's (0xFF: none)
      const uint64_t len = e - s.fs;
      const uint32_t sj = j < 3 ? (slen >> (8 * j)) & 0xFFu : 0xFFu;
      const bool hit = sj != 0xFFu && len == sj;
      if (staged) {  // (hashed as the unit's hashes are stored)
        s_fh[x] = hit ? 1 + 3 * threadIdx.x + j : 0xFFu;
      } else {
        uint64_t a, c;
        if (hit) {
          const uint64_t raw = s_slot[3 * threadIdx.x + j];
          a = raw * 1099511628211ULL;  // the NUL: a bare multiply (lib/k2hashfunc.cc:56)
          c = len ? raw : a;
        } else {  // a state outside the file (never for correct states): wrong records, not a fault
          hash_cstr_checked(f, size, s.fs, len, sp, a, c);
        }
        h1[r] = a;
        if (h2) h2[r] = c;
      }
    }
  };
  auto val_end = [&](uint64_t e, bool at_nul) {
    if constexpr (MDBM) {
      if (s.r == 2) {  // the fifth header line, compared whole (a NUL in it is a mismatch)
        static constexpr char kEnd[] = "HEADER=END";
        bool ok = !at_nul && e - s.fs == sizeof kEnd - 1;
        for (uint32_t i = 0; ok && i < sizeof kEnd - 1; ++i) ok = f[s.fs + i] == (uint8_t)kEnd[i];
        if (ok) __hip_atomic_store(hflags + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (s.r < HDR || s.r >= lim) return;
    const uint64_t r = s.r - HDR;
    if (staged) {
      const uint32_t x = (uint32_t)(s.r - su.r);
      s_rec[4 * x + 2] = s.fs;
      s_rec[4 * x + 3] = e - s.fs;
      s_fv[x] = 1;
    } else {
      *reinterpret_cast<u64x2*>(&recs[r].val_off) = u64x2{s.fs, e - s.fs};
    }
  };
  // The walk, one branch per event (round 4; round 3 branched on the event type and the mode,
  // ~60 SALU per event for the exec-mask bookkeeping): which field's C string ends here,
  // then the state by selects.  A field ends at its getline's delimiter (TSV: TAB for a
  // key, newline for a value; mdbm: newline for both) or at its first NUL; the delimiter
  // flips the mode, and a newline read in V ends the record.
  // A staged unit (nearly all) takes the walk without branches (round 5): every event writes
  // its record half and flag, to the dump row when no field of a record of this call ends
  // there, and only a key pass A could not hash branches (to hash it from the file); the
  // round-4 form branched on field ends, ~20 SALU per event of exec-mask bookkeeping.
  const bool staged_u = __builtin_amdgcn_readfirstlane(staged ? 1 : 0) != 0;
  typedef uint64_t u64x2a16 __attribute__((ext_vector_type(2)));
  for_events([&](uint32_t o, uint32_t t) {
    const uint64_t pos = base + rel + o;
    const bool nl = t == 1u, nul = t == 3u;
    const bool brk = MDBM ? nl : (s.m ? nl : t == 2u);  // the getline's delimiter
    const bool fe = !nulf && (brk || nul);             // a field's C string ends here
    if (staged_u) {
      const bool in = s.r >= HDR && s.r < lim;
      const bool ke = fe && !s.m && in, ve = fe && s.m && in;
      const uint32_t x = (uint32_t)(s.r - su.r);
      const uint32_t xk = ke ? x : kStageRecs, xv = ve ? x : kStageRecs, xr = ve ? xv : xk;
      *reinterpret_cast<u64x2a16*>(&s_rec[4 * xr + (ve ? 2u : 0u)]) = u64x2a16{s.fs, pos - s.fs};
      s_fk[xk] = 1;
      s_fv[xv] = 1;
      if constexpr (MDBM)
        if (fe && s.m && s.r == 2) val_end(pos, nul);  // the fifth header line's check (record 2 < HDR)
      if constexpr (HASH) {
        const uint32_t sj = j < 3 ? (slen >> (8 * j)) & 0xFFu : 0xFFu;
        const bool hit = sj != 0xFFu && pos - s.fs == sj;
        s_fh[xk] = hit ? 1 + 3 * threadIdx.x + j : 0xFFu;  // 0xFF: hashed from the file after the walk
      }
    } else if (fe) {
      if (s.m)
        val_end(pos, nul);
      else
        key_end(pos);
    }
    s.r += (nl && s.m) ? 1u : 0u;
    s.fs = brk ? pos + 1 : s.fs;
    nulf = !brk && (nulf || nul);
    s.m = brk ? s.m ^ 1u : s.m;
    j += nl ? 0u : 1u;  // cut events: TAB and NUL
  });
  if (live && base + rel + kTBytes >= size) {  // the thread holding the last byte
    if (s.m && !nulf) val_end(size, false);    // a value read to EOF
    if constexpr (MDBM) {
      if (!s.m && s.fs < size) {  // a key line at EOF: the key, and the previous record's value
        if (!nulf) key_end(size);
        if (s.r >= HDR && s.r < lim) {
          if (s.r == HDR && staged) {
            const uint32_t x = (uint32_t)(s.r - su.r);
            s_rec[4 * x + 2] = s.fs;
            s_rec[4 * x + 3] = 0;
            s_fv[x] = 1;
          } else if (s.r == HDR) {
            *reinterpret_cast<u64x2*>(&recs[0].val_off) = u64x2{s.fs, 0ull};
          }
          else
            __hip_atomic_store(hflags + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
  if (!staged) return;
  __syncthreads();
  // the staged parts, consecutive lanes on consecutive 16-byte pieces (a record's key half
  // or value half that another unit writes is skipped), as non-temporal stores: nothing in
  // the call reads them back (round 4: −31 us per call against plain stores)
  for (uint32_t q = threadIdx.x; q < 2 * nrec; q += 64) {
    const uint32_t x = q >> 1, half = q & 1u;
    if (half ? s_fv[x] : s_fk[x])
      __builtin_nontemporal_store(u64x2{s_rec[2 * q], s_rec[2 * q + 1]},
                                  reinterpret_cast<u64x2*>(&recs[su.r + x - HDR].key_off + 2 * half));
  }
  // keys pass A did not hash (0.8 % on BASELINE-like files), from the file: after the walk
  // (round 5), one lane per key and few live registers, instead of inside it, where the hash
  // raised the walk's register count (70 VGPRs, 7 waves per SIMD) and serialised the misses
  if constexpr (HASH) {
    for (uint32_t x = threadIdx.x; x < nrec; x += 64) {
      const uint32_t code = s_fh[x];
      if (!code) continue;
      uint64_t a, c;
      if (code == 0xFFu) {
        hash_cstr_checked(f, size, s_rec[4 * x], s_rec[4 * x + 1], sp, a, c);  // (a wrong state: wrong records, no fault)
      } else {
        const uint64_t raw = s_slot[code - 1];
        a = raw * 1099511628211ULL;  // the NUL: a bare multiply (lib/k2hashfunc.cc:56)
        c = s_rec[4 * x + 1] ? raw : a;
      }
      __builtin_nontemporal_store(a, h1 + su.r + x - HDR);
      if (h2) __builtin_nontemporal_store(c, h2 + su.r + x - HDR);
    }
  }
}

}  // namespace

// The scan's temporaries, one grow-only buffer per device held across calls (under a
// per-device lock for the call) while it stays within kScratchKeep: per-call pool
// allocations of this size cost ~0.15 ms per hipFreeAsync on MI355X (rocprofv3
// --runtime-trace, profiles/r03f_import_api_stats.csv), more than the scan itself.  Above
// kScratchKeep (a file of several GB) the buffer is freed at the end of the call, so a huge
// file does not pin its peak for the life of the process.
// The entry-state scan's counter lives in a second buffer that is never freed: it must be
// zero at every call (the scan leaves it zero), so it is cleared only when allocated.
// The record count and the mdbm flags come back through mapped pinned host memory.
constexpr uint64_t kScratchKeep = 512ull << 20;  // > the temporaries of a 1.2 GB TSV file (~20 % of its size)
struct ScanScratch {
  std::mutex mu;
  void* p = nullptr;
  size_t bytes = 0;
  void* cnt = nullptr;      // done (u32) at 0, count (u64) at 8
  uint64_t* hflags = nullptr;    // mapped pinned host memory: [0] count, [1] mdbm header ok, [2] mdbm fixup
  uint64_t* hflags_d = nullptr;  // ... and its device address
};
ScanScratch g_scan[64];

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// TSV and mdbm: pass A, the scan of block functions (and the count), pass B (mdbm always:
// it checks the header; TSV when records are wanted), one synchronisation.  Temporaries per
// 16 KiB block: its function and in-tile prefix (2 x 48 B), 8 B of events per 128 B span,
// and two speculative key states per span (TSV: 16 B per 128 B span); per tile
// of kTile blocks its function and entry state.
template <bool MDBM>
static int launch_scan(const uint8_t* f, uint64_t size, k2h_amd_import_rec* recs, uint64_t cap, uint64_t* count,
                       hipStream_t stream, hipError_t* herr, uint64_t* h1, uint64_t* h2, uint64_t seed) {
  const uint64_t nblk = (size + kTChunk - 1) / kTChunk;
  hipError_t e = nblk > 0x7FFFFFFFull ? hipErrorInvalidValue : hipSuccess;
  auto tr = [&](hipError_t x) {
    if (e == hipSuccess) e = x;
  };
  int dev = 0;
  tr(hipGetDevice(&dev));
  if (e == hipSuccess && (dev < 0 || dev >= 64)) e = hipErrorInvalidDevice;
  if (e != hipSuccess) {
    *herr = e;
    return K2H_AMD_EHIP;
  }
  const uint64_t nunit = (size + kUnit - 1) / kUnit;  // pass B's waves and the scan's items
  const uint64_t ntile = (nblk + kTile - 1) / kTile;  // tiles of pass-A blocks
  const size_t nfn = nblk * kUnitsPerBlock;  // pass A writes every wave's function, past-EOF ones too
  const size_t o_fn = 0, o_in = o_fn + align256(nfn * sizeof(GFn)), o_tf = o_in + align256(nfn * sizeof(GFn));
  const size_t o_ti = o_tf + align256(ntile * sizeof(GFn)), o_ev = o_ti + align256(ntile * sizeof(TState));
  const size_t nspec = MDBM ? 0 : nblk * kUnitsPerBlock * kUnitSlots;
  const size_t o_spec = o_ev + align256(nblk * kTThreads * 8);
  const size_t total = o_spec + align256(nspec * 8);
  ScanScratch& sc = g_scan[dev];
  std::lock_guard<std::mutex> lk(sc.mu);
  if (e == hipSuccess && sc.bytes < total) {
    if (sc.p) tr(hipFree(sc.p));
    sc.p = nullptr;
    sc.bytes = 0;
    tr(hipMalloc(&sc.p, total));
    if (e == hipSuccess) sc.bytes = total;
  }
  if (e == hipSuccess && !sc.cnt) {
    tr(hipMalloc(&sc.cnt, 256));
    tr(hipMemsetAsync(sc.cnt, 0, 256, stream));
    if (e != hipSuccess) sc.cnt = nullptr;
  }
  if (e == hipSuccess && !sc.hflags) {  // the count and flags come back without a copy command
    void* hp = nullptr;
    tr(hipHostMalloc(&hp, 64, hipHostMallocMapped));
    void* dp = nullptr;
    if (e == hipSuccess) tr(hipHostGetDevicePointer(&dp, hp, 0));
    if (e == hipSuccess) {
      sc.hflags = (uint64_t*)hp;
      sc.hflags_d = (uint64_t*)dp;
    } else if (hp) {
      (void)hipHostFree(hp);
    }
  }
  if (e != hipSuccess) {
    *herr = e;
    return K2H_AMD_EHIP;
  }
  sc.hflags[1] = 0;  // the previous call on this device has synchronised (the lock)
  sc.hflags[2] = 0;
  uint8_t* base = (uint8_t*)sc.p;
  uint8_t* cb = (uint8_t*)sc.cnt;
  EntryScan es;
  es.blk_fn = (GFn*)(base + o_fn);
  es.intile = (GFn*)(base + o_in);
  es.tile_fn = (GFn*)(base + o_tf);
  es.tile_in = (TState*)(base + o_ti);
  es.done = (uint32_t*)cb;
  es.count = (uint64_t*)(cb + 8);
  es.host_count = sc.hflags_d;
  es.nblk = nblk;
  es.ntile = ntile;
  es.size = size;
  es.mdbm = MDBM ? 1u : 0u;
  uint64_t* dcount = es.count;
  uint64_t* ev = (uint64_t*)(base + o_ev);
  const SpecSlots spec{(uint64_t*)(base + o_spec)};
  const bool walk = MDBM || (recs && cap);
  const uint64_t wcap = recs ? cap : 0;
  const SpadTable sp = make_spad(seed);
  tsv_a_kernel<MDBM><<<(unsigned)nblk, kTThreads, 0, stream>>>(f, size, es.blk_fn, ev, spec, sp);
  tr(hipGetLastError());
  if (e == hipSuccess) {
    tsv_scan_kernel<<<(unsigned)ntile, kTThreads, 0, stream>>>(es);
    tr(hipGetLastError());
  }
  if (e == hipSuccess && walk) {
    if (h1 && recs)
      tsv_b_kernel<true, MDBM><<<(unsigned)nunit, 64, 0, stream>>>(
          f, size, es.intile, es.tile_in, ev, spec.raw, dcount, wcap, recs, sp, h1, h2, sc.hflags_d);
    else
      tsv_b_kernel<false, MDBM><<<(unsigned)nunit, 64, 0, stream>>>(
          f, size, es.intile, es.tile_in, ev, spec.raw, dcount, wcap, recs, sp, nullptr, nullptr,
          sc.hflags_d);
    tr(hipGetLastError());
  }
  tr(hipStreamSynchronize(stream));
  const uint64_t n = e == hipSuccess ? __atomic_load_n(&sc.hflags[0], __ATOMIC_ACQUIRE) : 0;
  const bool hdr_ok = !MDBM || __atomic_load_n(&sc.hflags[1], __ATOMIC_ACQUIRE) != 0;
  // mdbm, a last key line at EOF after other records: the previous record's value (rare; a
  // second synchronisation only then)
  if (MDBM && e == hipSuccess && hdr_ok && __atomic_load_n(&sc.hflags[2], __ATOMIC_ACQUIRE) && recs && n >= 2 &&
      n <= cap) {
    tr(hipMemcpyAsync(&recs[n - 1].val_off, &recs[n - 2].val_off, 16, hipMemcpyDeviceToDevice, stream));
    tr(hipStreamSynchronize(stream));
  }
  if (sc.bytes > kScratchKeep) {  // the stream is synchronised: no kernel still reads it
    (void)hipFree(sc.p);
    sc.p = nullptr;
    sc.bytes = 0;
  }
  *herr = e;
  if (e != hipSuccess) return K2H_AMD_EHIP;
  if (!hdr_ok) return K2H_AMD_EINVAL;  // k2himport: "error: not a mdbm file."
  *count = n;
  return (recs && n > cap) ? K2H_AMD_EINVAL : K2H_AMD_OK;
}

// Returns K2H_AMD_* codes (the HIP error, if any, in *herr).
int launch_import_scan(const void* file, uint64_t size, int format, k2h_amd_import_rec* recs, uint64_t cap,
                       uint64_t* count, hipStream_t stream, hipError_t* herr, uint64_t* h1, uint64_t* h2,
                       uint64_t seed) {
  const uint8_t* f = (const uint8_t*)file;
  *herr = hipSuccess;
  *count = 0;
  // an empty file: no records (TSV), or no header (mdbm: "not a mdbm file"); no device work
  if (size == 0) return format == K2H_AMD_IMPORT_TSV ? K2H_AMD_OK : K2H_AMD_EINVAL;
  if (format == K2H_AMD_IMPORT_TSV) return launch_scan<false>(f, size, recs, cap, count, stream, herr, h1, h2, seed);
  return launch_scan<true>(f, size, recs, cap, count, stream, herr, h1, h2, seed);
}

hipError_t launch_import_prehash(const void* file, uint64_t size, const k2h_amd_import_rec* recs, uint64_t n,
                                 uint64_t seed, uint64_t* h1, uint64_t* h2, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  import_hash_kernel<<<blocks_for(n), kThreads, 0, stream>>>((const uint8_t*)file, size, recs, n, make_spad(seed),
                                                              h1, h2);
  return hipGetLastError();
}

}  // namespace k2h
