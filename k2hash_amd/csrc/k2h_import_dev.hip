// k2hash_amd -- k2himport input scan on the GPU.
//
// The same records as the host scanner (k2h_import.cc, restating the std::getline loops
// of tests/k2himport.cc:74-117) for a file that already sits in HBM, without a host pass:
//
// TSV (ConvertfromTsv, tests/k2himport.cc:74-89).  A record's key runs from the record
// start to the first TAB (across newlines), its value from there to the next '\n'.  So a
// record ends exactly at the newline of every line that holds a TAB, and the lines with
// no TAB in front of it belong to its key.  Record ends are therefore a per-line
// predicate and the loop needs no sequential walk: (1) per 16 KiB block, its newline
// count and its "span state" (newline seen; TAB / NUL / NUL-after-TAB seen since the
// last newline), scanned across blocks; (2) newline positions in order, and each line's
// first TAB and first NUL before / after that TAB (keys and values are cut there,
// c_str()/strlen) written directly, each thread knowing from the scanned state whether
// an event is the first of its kind in its line; (3) the TAB lines' indices written in
// order by the same pass (a per-block record count, taken in pass 1 for both possible
// incoming states, is scanned like the newline count), then one record per TAB line.  The bytes after the last newline form a last line whose
// value ends at EOF; if it holds no TAB the key getline hits EOF and it is dropped,
// as is a trailing run of newline-terminated lines with no TAB.
// mdbm (ConvertfromMdbm, tests/k2himport.cc:95-117).  Five header lines (the fifth
// "HEADER=END", checked on the host from the first newline positions), then line
// pairs; the EOF rules of the host scanner (an empty value after a key line that ends
// the file with '\n', the previous record's value after a key line that ends at EOF).
//
// Traffic: the file is read twice (pass 1: newline count, span state and record-end
// count per block; pass 2: newline positions, per-line TAB / NUL positions and the
// record-ending lines, written directly; a count-only TSV call stops after pass 1); outputs are 8 B per
// line plus 32 B per record.  Every pass is a streaming read.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <string.h>

#include <mutex>

#include "../../include/k2hash_amd.h"
#include "k2h_fnv_device.h"
#include "k2h_kernels.h"

namespace k2h {
namespace {

constexpr int kThreads = 256;
constexpr int kBytesPerThread = 64;
constexpr uint64_t kChunk = (uint64_t)kThreads * kBytesPerThread;  // 16 KiB per block
constexpr uint64_t kNone = ~0ull;

// Exact per-byte "equals c" mask of a 32-bit word: bit 7 of each matching byte.
__device__ inline uint32_t eq_mask(uint32_t w, uint32_t c4) {
  uint32_t v = w ^ c4;
  uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(t | v | 0x7F7F7F7Fu);
}

// Bytes [b, e) of this thread's 64-byte span, as 16 words with out-of-range bytes
// replaced by a non-newline value; aligned fast path when the span is whole.
__device__ inline void load_span(const uint8_t* f, uint64_t size, uint64_t b, uint32_t w[16]) {
  if (b + 64 <= size && (((uintptr_t)(f + b)) & 15) == 0) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* p = reinterpret_cast<const u32x4*>(f + b);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      u32x4 v = __builtin_nontemporal_load(p + q);
      w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint32_t x = 0x01010101u;
    for (int j = 0; j < 4; ++j) {
      uint64_t i = b + 4 * k + j;
      if (i < size) x = (x & ~(0xFFu << (8 * j))) | ((uint32_t)f[i] << (8 * j));
    }
    w[k] = x;
  }
}

struct LineInfo {
  uint64_t tab;       // first TAB in the line, or kNone
  uint64_t nul;       // first NUL in the line (anywhere), or kNone
  uint64_t nul_tab;   // first NUL after the first TAB, or kNone
};

__device__ inline uint64_t line_begin(const uint64_t* nl, uint64_t j) { return j ? nl[j - 1] + 1 : 0; }
__device__ inline uint64_t line_end(const uint64_t* nl, uint64_t nnl, uint64_t size, uint64_t j) {
  return j < nnl ? nl[j] : size;
}

// State of the line that is open at some point of the file, summarised over a span of
// bytes: whether the span holds a newline, and since its last newline (or its start)
// whether a TAB, a NUL, and a NUL after a TAB were seen.  Combining spans in file order
// is associative (a segmented "or"), so blocks and threads get their incoming state
// from scans: a thread then knows, for every TAB / NUL it holds, whether it is the
// first of its kind in its line.
enum : uint32_t { kHasNl = 1, kTab = 2, kNul = 4, kNulTab = 8 };
struct SpanOp {
  __host__ __device__ uint32_t operator()(uint32_t a, uint32_t b) const {
    if (b & kHasNl) return b;
    return (a & kHasNl) | ((a | b) & (kTab | kNul | kNulTab)) | (((a & kTab) && (b & kNul)) ? kNulTab : 0);
  }
};

struct CountStateOp {  // (newline count << 8 | span state) pairs, combined in file order
  __host__ __device__ uint32_t operator()(uint32_t a, uint32_t b) const {
    return (((a >> 8) + (b >> 8)) << 8) | SpanOp()(a & 0xFFu, b & 0xFFu);
  }
};

__device__ inline uint32_t nl_count(const uint32_t w[16]) {
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) c += __popc(eq_mask(w[k], 0x0A0A0A0Au));
  return c;
}

// Walk the span's events in byte order from state `st`; with Write, record each newline
// position and each line's first TAB / first NUL / first NUL after its first TAB, and
// (rl != NULL, TSV) the index of every line that ends a record -- a line holding a TAB --
// at rl[rec++].  Counts the record ends it passes.
struct Walk {
  uint32_t st;        // state after the span
  uint32_t recs;      // newlines that end a TAB line
  bool first_nl_tab;  // the first newline's line had a TAB (within the span)
  bool any_nl;
};

template <bool Write>
__device__ inline Walk span_walk(const uint32_t w[16], uint64_t b, uint32_t st, uint64_t line,
                                 uint64_t* __restrict__ nl, LineInfo* __restrict__ info, uint64_t* __restrict__ rl,
                                 uint64_t rec) {
  Walk r{st, 0, false, false};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    // masks per word, not kept for the span: fewer live registers, more waves
    const uint32_t mnl = eq_mask(w[k], 0x0A0A0A0Au);
    uint32_t x = mnl | eq_mask(w[k], 0x09090909u) | eq_mask(w[k], 0);
    while (x) {
      const int bit = __builtin_ctz(x);
      x &= x - 1;
      const uint64_t pos = b + 4 * k + (bit >> 3);
      if (mnl & (1u << bit)) {
        if constexpr (Write) nl[line] = pos;
        if (!r.any_nl) r.first_nl_tab = (st & kTab) != 0;
        r.any_nl = true;
        if (st & kTab) {
          if constexpr (Write) {
            if (rl) rl[rec++] = line;
          }
          ++r.recs;
        }
        ++line;
        st = kHasNl;
      } else if (((w[k] >> (bit - 7)) & 0xFFu) == 9) {  // TAB
        if (!(st & kTab)) {
          if constexpr (Write) info[line].tab = pos;
          st |= kTab;
        }
      } else {  // NUL
        if (!(st & kNul)) {
          if constexpr (Write) info[line].nul = pos;
          st |= kNul;
        }
        if ((st & kTab) && !(st & kNulTab)) {
          if constexpr (Write) info[line].nul_tab = pos;
          st |= kNulTab;
        }
      }
    }
  }
  r.st = st;
  return r;
}

// Record ends in a span given whether the line open at its start already holds a TAB
// (only the span's first newline depends on it).
__device__ inline uint32_t span_recs(const Walk& s, uint32_t in) {
  return s.recs + ((in & kTab) && s.any_nl && !s.first_nl_tab ? 1u : 0u);
}

// Pass 1: per block, the newline count, the span state, and the record-end count for
// both possible incoming states (low / high 32 bits: open line without / with a TAB).
__global__ __launch_bounds__(kThreads) void span_count_kernel(const uint8_t* __restrict__ f, uint64_t size,
                                                              uint64_t* __restrict__ block_cnt,
                                                              uint32_t* __restrict__ block_state,
                                                              uint64_t* __restrict__ block_recs) {
  const uint64_t b = (uint64_t)blockIdx.x * kChunk + (uint64_t)threadIdx.x * kBytesPerThread;
  uint32_t c = 0;
  Walk s{0, 0, false, false};
  if (b < size) {
    uint32_t w[16];
    load_span(f, size, b, w);
    c = nl_count(w);
    s = span_walk<false>(w, b, 0, 0, nullptr, nullptr, nullptr, 0);
  }
  typedef hipcub::BlockReduce<uint64_t, kThreads> Reduce;
  typedef hipcub::BlockScan<uint32_t, kThreads> Scan;
  __shared__ union {
    typename Reduce::TempStorage r;
    typename Scan::TempStorage s;
  } tmp;
  // incoming state assuming the block starts on a line with no TAB; assuming one with a
  // TAB differs only before the block's first newline: in1 has kTab iff in0 has, or no
  // newline precedes the thread
  uint32_t in0;
  Scan(tmp.s).ExclusiveScan(s.st, in0, 0u, SpanOp());
  __syncthreads();
  const uint32_t in1 = (in0 & kHasNl) ? in0 : (in0 | kTab);
  // newline count and both record counts fit 21 bits each (<= 16384 per block)
  const uint64_t packed = (uint64_t)c | ((uint64_t)span_recs(s, in0) << 21) | ((uint64_t)span_recs(s, in1) << 42);
  const uint64_t sum = Reduce(tmp.r).Sum(packed);
  if (threadIdx.x == kThreads - 1) block_state[blockIdx.x] = SpanOp()(in0, s.st);
  if (threadIdx.x == 0) {
    constexpr uint64_t m21 = (1ull << 21) - 1;
    block_cnt[blockIdx.x] = sum & m21;
    block_recs[blockIdx.x] = ((sum >> 21) & m21) | (((sum >> 42) & m21) << 32);
  }
}

// Record-end count of each block under its real incoming state.
__global__ __launch_bounds__(kThreads) void block_recs_kernel(const uint64_t* __restrict__ both,
                                                              const uint32_t* __restrict__ block_in, uint64_t nblk,
                                                              uint64_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nblk) return;
  out[i] = (block_in[i] & kTab) ? both[i] >> 32 : both[i] & 0xFFFFFFFFu;
}

// Pass 2 (block_base / block_in / rec_base = exclusive scans of pass 1): newline
// positions in order, every line's first TAB / NUL / NUL-after-TAB written straight
// into info, and (TSV) the record-ending line indices into rl -- including the bytes
// after the last newline when they hold a TAB (a record whose value ends at EOF).
__global__ __launch_bounds__(kThreads) void span_write_kernel(const uint8_t* __restrict__ f, uint64_t size,
                                                              const uint64_t* __restrict__ block_base,
                                                              const uint32_t* __restrict__ block_in,
                                                              const uint64_t* __restrict__ rec_base,
                                                              uint64_t* __restrict__ nl,
                                                              LineInfo* __restrict__ info,
                                                              uint64_t* __restrict__ rl) {
  const uint64_t b = (uint64_t)blockIdx.x * kChunk + (uint64_t)threadIdx.x * kBytesPerThread;
  uint32_t w[16];
  uint32_t c = 0;
  Walk s{0, 0, false, false};
  if (b < size) {
    load_span(f, size, b, w);
    c = nl_count(w);
    s = span_walk<false>(w, b, 0, 0, nullptr, nullptr, nullptr, 0);
  }
  typedef hipcub::BlockScan<uint32_t, kThreads> Scan;
  __shared__ typename Scan::TempStorage tmp;
  // newline count (<= 2^14 per block) above the 4 state bits: one scan for both
  uint32_t co, ro;
  Scan(tmp).ExclusiveScan((c << 8) | s.st, co, block_in[blockIdx.x], CountStateOp());
  __syncthreads();
  const uint32_t o = co >> 8, in = co & 0xFFu;
  Scan(tmp).ExclusiveSum(span_recs(s, in), ro);
  if (b >= size) return;
  const uint64_t line = block_base[blockIdx.x] + o, rec = rec_base[blockIdx.x] + ro;
  const Walk e = span_walk<true>(w, b, in, line, nl, info, rl, rec);
  // the thread holding the last byte: an open last line with a TAB is a record
  if (rl && b + kBytesPerThread >= size && f[size - 1] != '\n' && (e.st & kTab))
    rl[rec + e.recs] = line + c;
}

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

__device__ inline void hash_cstr(const uint8_t* __restrict__ f, uint64_t off, uint64_t len, const SpadTable& sp,
                                 uint64_t& h1, uint64_t& h2) {
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
    fnv_chunk16(lo, hi, c);
    for (uint64_t q = 1; q < k; ++q) fnv_chunk16(lo, hi, ld16(c0 + 16 * q));
    raw = ((uint64_t)hi << 32) | lo;
  }
  h1 = raw * 1099511628211ULL;  // lib/k2hashfunc.cc:56
  h2 = len ? raw : h1;
}

__global__ __launch_bounds__(kThreads) void import_hash_kernel(const uint8_t* __restrict__ f, uint64_t size,
                                                               const k2h_amd_import_rec* __restrict__ recs,
                                                               uint64_t n, SpadTable sp, uint64_t* __restrict__ h1,
                                                               uint64_t* __restrict__ h2) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const uint64_t off = recs[i].key_off, len = recs[i].key_len;
  uint64_t a = 0, b = 0;
  if (off <= size && len <= size - off) hash_cstr(f, off, len, sp, a, b);  // else: never read past the file
  h1[i] = a;
  if (h2) h2[i] = b;
}

// TSV: record r ends at TAB line rl[r]; its key starts after the previous TAB line.
// nul_from[k] = the first line j >= nlines - 1 - k whose bytes hold a NUL (kNone if none):
// a min-scan over the lines in reverse order, so a record whose key spans many TAB-less
// lines cuts it at its first NUL in O(1) (one lane used to walk those lines).
struct NulLineRev {
  const LineInfo* info;
  uint64_t nlines;
  __host__ __device__ uint64_t operator()(uint64_t k) const {
    const uint64_t j = nlines - 1 - k;
    return info[j].nul != kNone ? j : kNone;
  }
};
struct MinOp {
  __host__ __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a < b ? a : b; }
};

__global__ __launch_bounds__(kThreads) void tsv_records_kernel(const uint64_t* __restrict__ nl, uint64_t nnl,
                                                               uint64_t size, const LineInfo* __restrict__ info,
                                                               const uint64_t* __restrict__ nul_from, uint64_t nlines,
                                                               const uint64_t* __restrict__ rl, uint64_t nrec,
                                                               k2h_amd_import_rec* __restrict__ recs,
                                                               const uint8_t* __restrict__ f, SpadTable sp,
                                                               uint64_t* __restrict__ h1, uint64_t* __restrict__ h2) {
  const uint64_t r = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (r >= nrec) return;
  const uint64_t j1 = rl[r], j0 = r ? rl[r - 1] + 1 : 0;
  const uint64_t kb = line_begin(nl, j0);
  const LineInfo L = info[j1];
  uint64_t kend = L.tab;
  if (j1 > j0) {  // key lines before the TAB line (usually none): the first NUL in them, O(1)
    const uint64_t jn = nul_from[nlines - 1 - j0];  // first line >= j0 holding a NUL
    if (jn < j1) kend = info[jn].nul;
  }
  if (kend == L.tab && L.nul != kNone && L.nul < L.tab) kend = L.nul;
  const uint64_t vb = L.tab + 1, ve = L.nul_tab != kNone ? L.nul_tab : line_end(nl, nnl, size, j1);
  k2h_amd_import_rec o;
  o.key_off = kb;
  o.key_len = kend - kb;
  o.val_off = vb;
  o.val_len = ve - vb;  // a TAB that ends the file: getline fails, empty value at EOF
  recs[r] = o;
  if (h1) {  // fused prehash: the key as the C string Set stores
    uint64_t a, b;
    hash_cstr(f, o.key_off, o.key_len, sp, a, b);
    h1[r] = a;
    if (h2) h2[r] = b;
  }
}

// mdbm: key line 5 + 2r, value line 6 + 2r (see the header comment for the EOF rules).
__global__ __launch_bounds__(kThreads) void mdbm_records_kernel(const uint64_t* __restrict__ nl, uint64_t nnl,
                                                                uint64_t size, const LineInfo* __restrict__ info,
                                                                uint64_t nlines, uint64_t nrec, uint64_t body,
                                                                k2h_amd_import_rec* __restrict__ recs,
                                                                const uint8_t* __restrict__ f, SpadTable sp,
                                                                uint64_t* __restrict__ h1, uint64_t* __restrict__ h2) {
  const uint64_t r = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (r >= nrec) return;
  const uint64_t kl = 5 + 2 * r;
  auto cut = [&](uint64_t j) {  // strlen of line j's C string
    const uint64_t b = line_begin(nl, j), e = line_end(nl, nnl, size, j);
    return (info[j].nul != kNone ? info[j].nul : e) - b;
  };
  k2h_amd_import_rec o;
  o.key_off = line_begin(nl, kl);
  o.key_len = cut(kl);
  if (kl < nnl) {  // key line ends in '\n'
    const uint64_t vl = kl + 1;
    if (vl < nlines) {
      o.val_off = line_begin(nl, vl);
      o.val_len = cut(vl);
    } else {  // the file ends after the key line: the value getline fails
      o.val_off = size;
      o.val_len = 0;
    }
  } else if (r) {  // key line at EOF: the previous record's value (getline kept it)
    o.val_off = line_begin(nl, kl - 1);
    o.val_len = cut(kl - 1);
  } else {
    o.val_off = body;
    o.val_len = 0;
  }
  recs[r] = o;
  if (h1) {  // fused prehash: the key as the C string Set stores
    uint64_t a, b;
    hash_cstr(f, o.key_off, o.key_len, sp, a, b);
    h1[r] = a;
    if (h2) h2[r] = b;
  }
}

unsigned blocks_for(uint64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

}  // namespace

__global__ void scan_summary_kernel(const uint8_t* __restrict__ f, uint64_t size, const uint64_t* __restrict__ bbase,
                                    const uint64_t* __restrict__ rbase, const uint32_t* __restrict__ bst,
                                    const uint32_t* __restrict__ bin, uint64_t nblk, uint64_t* __restrict__ out) {
  out[0] = bbase[nblk];
  out[1] = rbase[nblk];
  out[2] = f[size - 1];
  out[3] = SpanOp()(bin[nblk - 1], bst[nblk - 1]);
}

// Scratch for the per-call temporaries: a library-private stream-ordered pool per device
// whose release threshold keeps up to kScratchKeep bytes of freed memory mapped (the
// default pool returns everything at every synchronisation, so each call would map its
// line / record arrays again).  Above the threshold, freed memory goes back to the device
// at the next synchronisation, so a call over a huge file does not pin its peak for the
// life of the process.
constexpr uint64_t kScratchKeep = 256ull << 20;  // ~ the temporaries of a 1 GB file of 140-byte lines

hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t stream) {
  constexpr int kMaxDev = 64;
  static hipMemPool_t pools[kMaxDev] = {};
  static std::once_flag once[kMaxDev];
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kMaxDev) return hipMallocAsync(p, bytes, stream);
  std::call_once(once[dev], [dev] {
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) return;
    uint64_t keep = kScratchKeep;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    pools[dev] = pool;
  });
  return pools[dev] ? hipMallocFromPoolAsync(p, bytes, pools[dev], stream) : hipMallocAsync(p, bytes, stream);
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
  const uint64_t nblk = (size + kChunk - 1) / kChunk;
  if (nblk > 0x7FFFFFFFull) return K2H_AMD_EINVAL;
  uint64_t* bcnt = nullptr;
  uint64_t *bbase = nullptr, *nl = nullptr, *rl = nullptr, *brec2 = nullptr, *brec = nullptr, *rbase = nullptr;
  LineInfo* info = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  uint32_t *bst = nullptr, *bin = nullptr;
  uint64_t nnl = 0, nlines = 0, nrec = 0;
  int rc = K2H_AMD_OK;
  hipError_t e = hipSuccess;
#define K2H_TRY(x) \
  do {             \
    if (e == hipSuccess) e = (x); \
  } while (0)
  const bool tsv = format == K2H_AMD_IMPORT_TSV;
  if (nblk) {
    K2H_TRY(scratch_alloc((void**)&bcnt, nblk * 8, stream));
    K2H_TRY(scratch_alloc((void**)&bbase, (nblk + 1) * 8, stream));
    K2H_TRY(scratch_alloc((void**)&bst, nblk * 4, stream));
    K2H_TRY(scratch_alloc((void**)&bin, nblk * 4, stream));
    K2H_TRY(scratch_alloc((void**)&brec2, nblk * 8, stream));
    K2H_TRY(scratch_alloc((void**)&brec, nblk * 8, stream));
    K2H_TRY(scratch_alloc((void**)&rbase, (nblk + 1) * 8, stream));
    if (e == hipSuccess) {
      span_count_kernel<<<(unsigned)nblk, kThreads, 0, stream>>>(f, size, bcnt, bst, brec2);
      e = hipGetLastError();
    }
    K2H_TRY(hipMemsetAsync(bbase, 0, 8, stream));
    K2H_TRY(hipMemsetAsync(rbase, 0, 8, stream));
    size_t t1 = 0, t2 = 0;
    K2H_TRY(hipcub::DeviceScan::InclusiveSum(nullptr, t1, bcnt, bbase + 1, nblk, stream));
    K2H_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, t2, bst, bin, SpanOp(), 0u, nblk, stream));
    tmp_bytes = t1 > t2 ? t1 : t2;
    K2H_TRY(scratch_alloc(&tmp, tmp_bytes ? tmp_bytes : 1, stream));
    K2H_TRY(hipcub::DeviceScan::InclusiveSum(tmp, t1, bcnt, bbase + 1, nblk, stream));
    K2H_TRY(hipcub::DeviceScan::ExclusiveScan(tmp, t2, bst, bin, SpanOp(), 0u, nblk, stream));
    if (e == hipSuccess) {
      block_recs_kernel<<<blocks_for(nblk), kThreads, 0, stream>>>(brec2, bin, nblk, brec);
      e = hipGetLastError();
    }
    K2H_TRY(hipcub::DeviceScan::InclusiveSum(tmp, t1, brec, rbase + 1, nblk, stream));  // same shape as bcnt
    // one read-back: newline count, newline record ends, last byte, final span state
    uint64_t sum[4] = {0, 0, '\n', 0};
    uint64_t* dsum = nullptr;
    K2H_TRY(scratch_alloc((void**)&dsum, sizeof sum, stream));
    if (e == hipSuccess) {
      scan_summary_kernel<<<1, 1, 0, stream>>>(f, size, bbase, rbase, bst, bin, nblk, dsum);
      e = hipGetLastError();
    }
    K2H_TRY(hipMemcpyAsync(sum, dsum, sizeof sum, hipMemcpyDeviceToHost, stream));
    K2H_TRY(hipStreamSynchronize(stream));
    if (dsum) (void)hipFreeAsync(dsum, stream);
    nnl = sum[0];
    const uint64_t nrec_nl = sum[1];
    const uint8_t last = (uint8_t)sum[2];
    const uint32_t st_final = (uint32_t)sum[3];
    // lines: one per newline, plus the bytes after the last newline if any
    nlines = nnl + (last != '\n' ? 1 : 0);
    // TSV records: newlines ending a TAB line, plus an open last line holding a TAB
    if (tsv) nrec = nrec_nl + ((last != '\n' && (st_final & kTab)) ? 1 : 0);
    // TSV needs pass 2 only to fill records; mdbm always (its header check reads nl)
    const bool pass2 = !tsv || (recs && nrec && nrec <= cap);
    if (pass2) {
      K2H_TRY(scratch_alloc((void**)&nl, (nnl ? nnl : 1) * 8, stream));
      K2H_TRY(scratch_alloc((void**)&info, (nlines ? nlines : 1) * sizeof(LineInfo), stream));
      if (tsv) K2H_TRY(scratch_alloc((void**)&rl, nrec * 8, stream));
      if (nlines) K2H_TRY(hipMemsetAsync(info, 0xFF, nlines * sizeof(LineInfo), stream));  // kNone
      if (e == hipSuccess) {
        span_write_kernel<<<(unsigned)nblk, kThreads, 0, stream>>>(f, size, bbase, bin, rbase, nl, info, rl);
        e = hipGetLastError();
      }
    }
  }
  uint64_t* nul_from = nullptr;
  void* tmp2 = nullptr;
  if (e == hipSuccess && tsv) {
    if (recs && nrec && nrec <= cap) {
      hipcub::CountingInputIterator<uint64_t> idx(0);
      hipcub::TransformInputIterator<uint64_t, NulLineRev, hipcub::CountingInputIterator<uint64_t>> nul_rev(
          idx, NulLineRev{info, nlines});
      size_t t3 = 0;
      K2H_TRY(scratch_alloc((void**)&nul_from, nlines * 8, stream));
      K2H_TRY(hipcub::DeviceScan::InclusiveScan(nullptr, t3, nul_rev, nul_from, MinOp(), nlines, stream));
      K2H_TRY(scratch_alloc(&tmp2, t3 ? t3 : 1, stream));
      K2H_TRY(hipcub::DeviceScan::InclusiveScan(tmp2, t3, nul_rev, nul_from, MinOp(), nlines, stream));
      if (e == hipSuccess) {
        tsv_records_kernel<<<blocks_for(nrec), kThreads, 0, stream>>>(nl, nnl, size, info, nul_from, nlines, rl, nrec,
                                                                      recs, f, make_spad(seed), h1, h2);
        e = hipGetLastError();
      }
    }
  } else if (e == hipSuccess && format == K2H_AMD_IMPORT_MDBM) {
    // header: five getline calls; the fifth must extract exactly "HEADER=END"
    static const char kEnd[] = "HEADER=END";
    uint64_t hb = 0, he = 0, body = 0;
    bool ok = nlines >= 5;
    if (ok) {
      uint64_t pos[5] = {0, 0, 0, 0, 0};
      const uint64_t m = nnl < 5 ? nnl : 5;
      if (m) K2H_TRY(hipMemcpyAsync(pos, nl, m * 8, hipMemcpyDeviceToHost, stream));
      K2H_TRY(hipStreamSynchronize(stream));
      hb = pos[3] + 1;
      he = nnl >= 5 ? pos[4] : size;  // the fifth line may end at EOF
      body = nnl >= 5 ? pos[4] + 1 : size;
      char hdr[sizeof kEnd] = {0};
      ok = he - hb == sizeof kEnd - 1;
      if (ok) K2H_TRY(hipMemcpyAsync(hdr, f + hb, sizeof kEnd - 1, hipMemcpyDeviceToHost, stream));
      K2H_TRY(hipStreamSynchronize(stream));
      ok = ok && memcmp(hdr, kEnd, sizeof kEnd - 1) == 0;
    }
    if (e == hipSuccess && !ok) rc = K2H_AMD_EINVAL;  // k2himport: "error: not a mdbm file."
    if (e == hipSuccess && ok) {
      nrec = nlines > 5 ? (nlines - 5 + 1) / 2 : 0;
      if (recs && nrec && nrec <= cap) {
        mdbm_records_kernel<<<blocks_for(nrec), kThreads, 0, stream>>>(nl, nnl, size, info, nlines, nrec, body,
                                                                          recs, f, make_spad(seed), h1, h2);
        e = hipGetLastError();
      }
    }
  }
  K2H_TRY(hipStreamSynchronize(stream));
#undef K2H_TRY
  for (void* p : {(void*)bcnt, (void*)bbase, (void*)bst, (void*)bin, (void*)brec2, (void*)brec, (void*)rbase, (void*)nl,
                  (void*)rl, (void*)info, tmp, (void*)nul_from, tmp2})
    if (p) (void)hipFreeAsync(p, stream);
  *herr = e;
  if (e != hipSuccess) return K2H_AMD_EHIP;
  if (rc != K2H_AMD_OK) return rc;
  *count = nrec;
  return (recs && nrec > cap) ? K2H_AMD_EINVAL : K2H_AMD_OK;
}

hipError_t launch_import_prehash(const void* file, uint64_t size, const k2h_amd_import_rec* recs, uint64_t n,
                                 uint64_t seed, uint64_t* h1, uint64_t* h2, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  import_hash_kernel<<<blocks_for(n), kThreads, 0, stream>>>((const uint8_t*)file, size, recs, n, make_spad(seed),
                                                              h1, h2);
  return hipGetLastError();
}

}  // namespace k2h
