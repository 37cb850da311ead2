// k2hash_amd -- RALLEDATA producer.
//
// k2hash's direct-set path takes elements as packed RALLEDATA blobs that already carry
// the key's hash and subhash (struct at lib/k2hshmdirect.h:36-47; consumed by
// K2HShm::SetElementByBinArray, lib/k2hshmdirect.cc:343-478, via
// k2h_set_element_by_binary, lib/k2hash.cc:1562-1581): a bulk loader that builds the
// blobs on the GPU never runs the scalar hash per key.  Blob layout = the one
// K2HShm::GetElementToBinary writes (lib/k2hshmdirect.cc:59-88):
//   [0]  hash  = k2h_hash(key)          [8]  subhash = k2h_second_hash(key)
//   [16] key_length  [24] val_length  [32] skey_length  [40] attrs_length
//   [48] key_pos = 80  [56] val_pos  [64] skey_pos  [72] attrs_pos   (from the blob top)
//   [80] key | value | subkeys | attrs
// Records come as four CSR streams (keys, values, subkeys, attributes: bytes + n+1
// offsets; a NULL offsets array means the segment is empty for every record).  Blobs are
// packed back to back, so blob i starts at the closed form
//   80 i + sum over segments of (seg_off[i] - seg_off[0])
// and no scan is needed.
//
// One kernel (ralledata_gather_kernel, below): tiles of 64 records staged in LDS, the keys
// hashed there, the blobs written as aligned 16-byte pieces; tiles too large to stage run
// the 8-lane group form inside the same kernel.  Blob and segment addresses are
// byte-aligned.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "k2h_fnv_device.h"
#include "k2h_kernels.h"

namespace k2h {
namespace {

typedef uint64_t u64_ua __attribute__((aligned(1)));
typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));

// Workgroup barrier over LDS only (see its use in ralledata_gather_kernel).
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ uint64_t seg_len(const uint64_t* off, uint64_t i) { return off ? off[i + 1] - off[i] : 0; }
__device__ __forceinline__ uint64_t seg_before(const uint64_t* off, uint64_t i) { return off ? off[i] - off[0] : 0; }


// Group form (oversize tiles): G lanes per record, 64/G records per wave.  Lane q of a group
// writes header piece q (5 x 16 B) and copies bytes [16q + 16Gj, +16) of each segment,
// so a group's loads and stores are consecutive 16-byte pieces instead of one lane
// streaming a whole record.  A segment's last partial piece is the 16 bytes ENDING at
// its last byte (they overlap the previous piece with the same bytes, so the order of
// the two stores does not matter); only segments shorter than 16 bytes are copied byte
// by byte.  G = 8 keeps most lanes busy on BASELINE-like records (keys 8-64 B, values
// 0-256 B).
template <int G>
__device__ __forceinline__ void group_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t len,
                                           uint32_t q) {
  uint64_t full = len & ~15ull;
  for (uint64_t j = 16ull * q; j < full; j += 16ull * G)
    *reinterpret_cast<u32x4_ua*>(dst + j) = *reinterpret_cast<const u32x4_ua*>(src + j);
  if (full == len) return;
  if (len >= 16) {
    if (q == G - 1)
      *reinterpret_cast<u32x4_ua*>(dst + len - 16) = *reinterpret_cast<const u32x4_ua*>(src + len - 16);
    return;
  }
  for (uint64_t t = full + q; t < len; t += G) dst[t] = src[t];  // the <= 15 tail bytes
}

// Gather form (round 2): output-driven.  A block takes R consecutive records; its blobs are
// one contiguous output span, and the records' key / value / subkey / attribute bytes are
// four contiguous input spans.  The block
//   1. stages the four input spans into LDS with aligned 16-byte loads (the aligned hull of
//      each span: every load holds a valid byte, so none leaves a mapped page) and builds
//      the R headers in LDS, plus a table of the span's segments (header, key, value,
//      subkeys, attrs of each record: where each starts in the span and where its bytes sit
//      in LDS) and, per aligned 16-byte output piece, the segment holding its first byte;
//   2. writes the span as aligned 16-byte pieces, consecutive lanes on consecutive pieces
//      (whole 128-byte lines per 8 lanes): a piece is one unaligned ds_read_b128 from the
//      segment that holds it, or, where segments meet inside it, one read per segment
//      merged under a byte mask.  Only the two pieces a block shares with its neighbours
//      are stored byte by byte.
// So every blob byte is stored once, aligned, and every input byte is loaded once, aligned;
// the group form's unaligned 16-byte accesses at ~2.3 TB/s are gone.  A block whose spans
// exceed the LDS image (records much larger than BASELINE-like ones) runs the group form.
constexpr int kGatherRecs = 64;                  // records per 256-thread block
constexpr int kGatherPool = 12288;               // staged segment bytes (BASELINE-like: ~10.5 KB, sd ~0.6 KB; 7 blocks per CU)
constexpr int kGatherHdr = 16;                   // LDS offset of the headers (16 readable bytes below)
constexpr int kGatherImg = kGatherHdr + 80 * kGatherRecs + kGatherPool + 16;
constexpr int kGatherPieces = (80 * kGatherRecs + kGatherPool) / 16 + 2;

// Key hash straight from HBM (the fused kernel's group-form blocks): the same end-aligned
// chunks; bytes below the key buffer are never read.
__device__ __forceinline__ void global_key_hash(const uint8_t* keys, uint64_t b, uint64_t e, const uint64_t* spad,
                                                uint64_t& r1, uint64_t& r2) {
  const uint64_t len = e - b, k = (len + 15) >> 4;
  const uint32_t p = (uint32_t)(16 * k - len);
  const uint8_t* cp = keys + e - 16 * k;
  const uint64_t st = spad[p & 15];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2 = lo, hi2 = hi;
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t j = p; j < 16 && k; ++j) w[j >> 2] |= (uint32_t)cp[j] << (8 * (j & 3));
  uint4 c = make_uint4(w[0], w[1], w[2], w[3]);
  for (uint64_t j = 1; j < k; ++j) {
    fnv_chunk16(lo, hi, c);
    const u32x4_ua v = *reinterpret_cast<const u32x4_ua*>(cp + 16 * j);
    c = make_uint4(v.x, v.y, v.z, v.w);
  }
  fnv_chunk16_last(lo, hi, lo2, hi2, c);
  r1 = k ? ((uint64_t)hi << 32) | lo : 0;
  r2 = k ? (len == 1 ? r1 : ((uint64_t)hi2 << 32) | lo2) : 0;
}

// one record by a group of G lanes, straight to HBM (the group form); lane 0 hashes the key
template <int G>
__device__ __forceinline__ void group_record(const RalleInputs& in, uint64_t n, uint8_t* __restrict__ out,
                                             uint64_t* __restrict__ blob_off, uint64_t i, uint32_t q,
                                             const uint64_t* spad) {
  const uint64_t kl = seg_len(in.koff, i), vl = seg_len(in.voff, i), sl = seg_len(in.soff, i), al = seg_len(in.aoff, i);
  const uint64_t o = 80ull * i + seg_before(in.koff, i) + seg_before(in.voff, i) + seg_before(in.soff, i) +
                     seg_before(in.aoff, i);
  uint8_t* b = out + o;
  if (q < 5) {
    uint64_t f0, f1;
    switch (q) {
      case 0:
        if (in.koff) global_key_hash(in.keys, in.koff[i], in.koff[i + 1], spad, f0, f1);
        else f0 = f1 = 0;
        break;
      case 1: f0 = kl; f1 = vl; break;
      case 2: f0 = sl; f1 = al; break;
      case 3: f0 = 80; f1 = 80 + kl; break;
      default: f0 = 80 + kl + vl; f1 = 80 + kl + vl + sl; break;
    }
    *reinterpret_cast<u32x4_ua*>(b + 16 * q) = u32x4_ua{(uint32_t)f0, (uint32_t)(f0 >> 32), (uint32_t)f1, (uint32_t)(f1 >> 32)};
  }
  if (kl) group_copy<G>(b + 80, in.keys + in.koff[i], kl, q);
  if (vl) group_copy<G>(b + 80 + kl, in.vals + in.voff[i], vl, q);
  if (sl) group_copy<G>(b + 80 + kl + vl, in.skeys + in.soff[i], sl, q);
  if (al) group_copy<G>(b + 80 + kl + vl + sl, in.attrs + in.aoff[i], al, q);
  if (blob_off && q == 0) {
    blob_off[i] = o;
    if (i + 1 == n) blob_off[n] = o + 80 + kl + vl + sl + al;
  }
}

// Key hash from the staged bytes: end-aligned 16-byte chunks (the CSR kernels'
// scheme): chunk 0 starts 16k - len bytes early with those bytes
// zeroed and the state started at S_p = seed * P^-p, so no byte tail; the last chunk's
// byte 15 step leaves the second hash (the state before the last byte).
__device__ __forceinline__ void staged_key_hash(const uint8_t* end, uint32_t len, const uint64_t* spad, uint64_t& r1,
                                                uint64_t& r2) {
  const uint32_t k = (len + 15) >> 4, p = 16 * k - len;
  const uint8_t* cp = end - 16 * k;
  const uint64_t st = spad[p & 15];
  uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2 = lo, hi2 = hi;
  u32x4_ua w = *reinterpret_cast<const u32x4_ua*>(cp);
  const int32_t sh = (int32_t)(8 * p);
  auto lead = [sh](int32_t b) -> uint32_t { return (uint32_t)(~0ull << min(max(sh - b, 0), 32)); };
  uint4 c = make_uint4(w.x & lead(0), w.y & lead(32), w.z & lead(64), w.w & lead(96));
  for (uint32_t j = 1; j < k; ++j) {
    fnv_chunk16(lo, hi, c);
    w = *reinterpret_cast<const u32x4_ua*>(cp + 16 * j);
    c = make_uint4(w.x, w.y, w.z, w.w);
  }
  fnv_chunk16_last(lo, hi, lo2, hi2, c);
  r1 = k ? ((uint64_t)hi << 32) | lo : 0;  // empty key hashes to 0 (lib/k2hashfunc.cc:66-68, 80-82)
  r2 = k ? (len == 1 ? r1 : ((uint64_t)hi2 << 32) | lo2) : 0;
}

// The key hashes are computed here from the staged keys (no hash kernel, no scratch).
// Wave 0 only waits for its records' offsets (the staged loads are issued by waves 1-3).
// 8 blocks per CU (8 waves/SIMD, <= 64 VGPRs): the block's LDS stays under 20 KiB -- the
// segment table packs (adj, end) into 16-bit halves, the piece table keeps the low byte of
// each piece's segment index plus the full index every 64 pieces (a 64-piece run, 1 KiB,
// meets at most 14 records -- every record carries an 80-byte header -- so fewer than 256
// segments, and the low byte and the run's base recover the index) -- where the round-2
// tables (int2, uint16) allowed 7 (A/B: 0.724 vs 0.733 ms, profiles/r03ad_ralle_ab.txt).
__device__ __forceinline__ uint32_t seg_pack(int32_t adj, int32_t end) {
  return (uint32_t)(uint16_t)(int16_t)adj | ((uint32_t)end << 16);
}
__device__ __forceinline__ int2 seg_unpack(uint32_t v) { return int2{(int32_t)(int16_t)(v & 0xffffu), (int32_t)(v >> 16)}; }

// KV: no subkeys and no attributes (both offset arrays NULL, the common direct-set call):
// the two empty streams fold away at compile time -- half the block-uniform setup (64-bit
// scalar address arithmetic, ~200 SALU per wave for four streams) and of the stream selects
// (round 4).
template <bool KV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void ralledata_gather_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  if constexpr (KV) {
    in.soff = in.aoff = nullptr;
    in.skeys = in.attrs = nullptr;
  }
  // segments per record: header, key, value, subkeys, attributes (KV: the first three)
  constexpr int NS = KV ? 3 : 5;
  constexpr int R = kGatherRecs, NSEG = NS * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ uint32_t seg[NSEG + 1];  // segment g: seg_pack(adj, end): span byte y sits at img[y + adj], end in the span
  constexpr int NRUN = (kGatherPieces + 63) / 64;
  __shared__ uint8_t tab[kGatherPieces + 1];  // low byte of the segment holding piece p's first byte (+ a dump slot)
  __shared__ uint16_t tbase[NRUN + 1];        // segment holding piece 64 j's first byte (+ a dump slot)
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
  static_assert(kGatherImg + 4 * (NSEG + 1) + kGatherPieces + 1 + 2 * (NRUN + 1) + 16 * 17 + 8 * 16 <= 20 * 1024,
                "8 blocks per CU");
  const uint32_t tid = threadIdx.x;
  const uint64_t r0 = (uint64_t)blockIdx.x * R;
  const uint32_t nr = (uint32_t)(n - r0 < (uint64_t)R ? n - r0 : (uint64_t)R);
  const uint64_t* offs[4] = {in.koff, in.voff, in.soff, in.aoff};
  const uint8_t* srcs[4] = {in.keys, in.vals, in.skeys, in.attrs};
  // the records' own offsets first: they do not depend on the span offsets below
  uint32_t ro0[4] = {0, 0, 0, 0}, ro1[4] = {0, 0, 0, 0};
  if (tid < nr) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ro0[s] = offs[s] ? (uint32_t)offs[s][r0 + tid] : 0u;
      ro1[s] = offs[s] ? (uint32_t)offs[s][r0 + tid + 1] : 0u;
    }
  }
  // block-uniform: each input span, its aligned hull, where it goes in the image
  uint64_t o_first = 80ull * r0, span = 80ull * nr, hull_total = 0;
  uint64_t sbase[4], hull_lo[4], hull_n[4];
  int32_t area[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    uint64_t b = 0, e = 0, f = 0;
    if (offs[s]) {
      b = offs[s][r0];
      e = offs[s][r0 + nr];
      f = offs[s][0];
    }
    sbase[s] = b;
    o_first += b - f;
    span += e - b;
    const uint64_t lo = (uint64_t)(uintptr_t)(srcs[s] + b) & ~15ull, hi = ((uint64_t)(uintptr_t)(srcs[s] + e) + 15) & ~15ull;
    hull_lo[s] = lo;
    hull_n[s] = e > b ? (hi - lo) >> 4 : 0;
    area[s] = kGatherHdr + 80 * R + (int32_t)(16 * hull_total) + (int32_t)((uintptr_t)(srcs[s] + b) - lo);
    hull_total += hull_n[s];
  }
  if (16 * hull_total > (uint64_t)kGatherPool) {  // block-uniform: too large to stage
    // the group form, one record per 8 lanes straight to HBM, lane 0 hashing the key
    if (tid < 16) spad[tid] = spad_tab.v[tid];
    __syncthreads();
    for (uint32_t rec = tid / 8; rec < nr; rec += 32) group_record<8>(in, n, out, blob_off, r0 + rec, tid % 8, spad);
    return;
  }
  // 1a. the staged pieces: up to 4 aligned loads per thread of waves 1-3 (wave 0's only
  // loads are its records' offsets, so its record work waits for nothing else)
  constexpr uint32_t SW = 64, NST = 256 - SW;
  constexpr int PPT = (kGatherPool / 16 + NST - 1) / NST;
  u32x4_al v[PPT];
  uint32_t dst[PPT];
  // (the stream of piece q by selects on 32-bit prefix counts: round 3 tested each stream's
  // 64-bit range under its own exec mask, ~16 SALU per piece)
  const uint32_t c1 = (uint32_t)hull_n[0], c2 = c1 + (uint32_t)hull_n[1], c3 = c2 + (uint32_t)hull_n[2];
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint32_t q = tid - SW + NST * u;
    dst[u] = 0xffffffffu;
    if (tid >= SW && q < (uint32_t)hull_total) {
      const bool b1 = q >= c1, b2 = q >= c2, b3 = q >= c3;
      const uint64_t lo = b3 ? hull_lo[3] : b2 ? hull_lo[2] : b1 ? hull_lo[1] : hull_lo[0];
      const uint32_t before = b3 ? c3 : b2 ? c2 : b1 ? c1 : 0u;
      const uint64_t addr = lo + 16ull * (q - before);
      // a global (not flat) load: hipcc must otherwise assume it may touch LDS and makes
      // the LDS reads after the barrier wait for every vector-memory operation; non-temporal:
      // every input byte is read once (round 4: 0.687 -> 0.673 ms in A/B)
      v[u] = __builtin_nontemporal_load(
          reinterpret_cast<const __attribute__((address_space(1))) u32x4_al*>((uintptr_t)addr));
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // 1b. one thread per record: header, segment table.  All
  // block-relative quantities fit 32 bits once the spans fit the image.
  const uint64_t a_out = (uint64_t)(uintptr_t)(out + o_first);
  const int32_t d0 = (int32_t)(a_out & 15u);
  if (tid < 17) {  // qmask[l] = bytes [l, 16) of a piece
    u32x4_al m;
    m.x = (uint32_t)(~0ull << (8 * min(max((int)tid - 0, 0), 4)));
    m.y = (uint32_t)(~0ull << (8 * min(max((int)tid - 4, 0), 4)));
    m.z = (uint32_t)(~0ull << (8 * min(max((int)tid - 8, 0), 4)));
    m.w = (uint32_t)(~0ull << (8 * min(max((int)tid - 12, 0), 4)));
    qmask[tid] = m;
  }
  if (tid < 16) spad[tid] = spad_tab.v[tid];
  if (tid < nr) {
    uint32_t rel[4], len[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      rel[s] = ro0[s] - (uint32_t)sbase[s];
      len[s] = ro1[s] - ro0[s];
    }
    const int32_t B = (int32_t)(80u * tid + rel[0] + rel[1] + rel[2] + rel[3]);
    const uint32_t kl = len[0], vl = len[1], sl = len[2], al = len[3];
    const uint32_t f[20] = {0, 0, 0, 0, kl, 0, vl, 0, sl, 0,  // hashes: filled in by wave 0 below
                            al, 0, 80, 0, 80 + kl, 0, 80 + kl + vl, 0, 80 + kl + vl + sl, 0};
#pragma unroll
    for (int c = 0; c < 5; ++c)
      *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid + 16 * c) = u32x4_al{f[4 * c], f[4 * c + 1], f[4 * c + 2], f[4 * c + 3]};
    int32_t start = B;
#pragma unroll
    for (int c = 0; c < NS; ++c) {
      const uint32_t g = NS * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = seg_pack(adj, start + L);
      start += L;
    }
    if (tid + 1 == nr) seg[NS * nr] = seg_pack(kGatherHdr, start);  // read (never used) as the last segment's successor
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  // The block's waves share only LDS, so the two barriers wait for LDS operations alone
  // (__syncthreads() also waits for every outstanding vector-memory operation).
  lds_sync();
  // the blob offsets by wave 1, idle while wave 0 hashes, from the segment table (a
  // record's header segment ends 80 bytes after its blob starts; the sentinel holds the
  // span's end): wave 0's critical path then carries no store whose acknowledgement a
  // later wait would include
  if (blob_off && tid >= 64 && tid - 64 < nr) {
    const uint32_t r = tid - 64;
    blob_off[r0 + r] = o_first + (uint64_t)(uint32_t)(seg_unpack(seg[NS * r]).y - 80);
    if (r0 + r + 1 == n) blob_off[n] = o_first + (uint64_t)(uint32_t)seg_unpack(seg[NS * nr]).y;
  }
  // 1c'. the piece table, by waves 1-3 while wave 0 hashes: each segment writes its index
  // for the pieces whose first byte it holds, four pieces per loop trip, the writes past the
  // segment's last piece sent to a dump slot (no per-piece branch).  Round 4 took one
  // divergent trip per piece (~15 per wave, the longest value segment) and branched round
  // the run-base write: ~120 SALU per wave of exec-mask bookkeeping.
  if (tid >= 64)
    for (uint32_t g = tid - 64; g < NS * nr; g += 192) {
      const int32_t end = seg_unpack(seg[g]).y, beg = g ? seg_unpack(seg[g - 1]).y : 0;
      const int32_t last = (end - 1 + d0) >> 4;
      for (int32_t p = g ? (beg + d0 + 15) >> 4 : 0; p <= last; p += 4) {
#pragma unroll
        for (int32_t u = 0; u < 4; ++u) tab[p + u <= last ? p + u : kGatherPieces] = (uint8_t)g;
        const int32_t r = (p + 63) & ~63;  // the run start among pieces p .. p + 3, if any
        tbase[r <= min(p + 3, last) ? r >> 6 : NRUN] = (uint16_t)g;
      }
    }
  // 1c. wave 0 hashes the block's keys from the image into the headers
  if (tid < nr) {
    const uint32_t kl = ro1[0] - ro0[0], ke = ro1[0] - (uint32_t)sbase[0];
    uint64_t h1, h2;
    staged_key_hash(img + area[0] + ke, kl, spad, h1, h2);
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid) =
        u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
  }
  lds_sync();
  // 2. aligned output pieces: the window of each segment in the piece, aligned with the
  // piece, merged forward (segment k supplies bytes [its start, 16) over what came before)
  const int32_t sp = (int32_t)span;
  const uint32_t np = (uint32_t)((d0 + sp + 15) >> 4);
  uint8_t* const base = out + (o_first - (uint64_t)d0);
  // piece p: its first segment s0 (= seg[g]) and the next s1, both windows already read;
  // further segments (a short or empty one between) are read here
  auto piece = [&](uint32_t p, uint32_t g, int2 s0, int2 s1, const u32x4_ua& w0, const u32x4_ua& w1) {
    const int32_t x = 16 * (int32_t)p - d0, end = min(x + 16, sp);
    u32x4_al acc = {w0.x, w0.y, w0.z, w0.w};
    int32_t pos = s0.y;
    auto merge = [&](const u32x4_ua& w) {  // bytes [pos - x, 16) from w
      const u32x4_al q = qmask[pos - x];
      acc.x = (w.x & q.x) | (acc.x & ~q.x);
      acc.y = (w.y & q.y) | (acc.y & ~q.y);
      acc.z = (w.z & q.z) | (acc.z & ~q.z);
      acc.w = (w.w & q.w) | (acc.w & ~q.w);
    };
    if (pos < end) {  // 18 % of pieces meet two segments, 0.4 % three or more
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg_unpack(seg[++g]);
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    return acc;
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  auto build = [&](uint32_t p) {
    const uint32_t gb = tbase[p >> 6];
    const uint32_t g = gb + ((tab[p] - gb) & 0xffu);
    const int2 s0 = seg_unpack(seg[g]), s1 = seg_unpack(seg[g + 1]);  // the piece's segment and the next
    return piece(p, g, s0, s1, window(s0, p), window(s1, p));
  };
  // pieces wholly inside the span: one aligned store each; the (at most two) pieces shared
  // with the neighbouring blocks: this block's bytes only, by two lanes of waves 2 and 3
  const uint32_t pf = d0 ? 1u : 0u, pl = ((d0 + sp) & 15) ? np - 1u : np;
  for (uint32_t p = pf + tid; p < pl; p += 256) __builtin_nontemporal_store(build(p), reinterpret_cast<u32x4_al*>(base + 16ull * p));
  const uint32_t pe = tid == 128 && pf ? 0u : tid == 192 && pl < np && (pl > 0 || !pf) ? np - 1u : ~0u;
  if (pe != ~0u) {
    const u32x4_al acc = build(pe);
    const int32_t x = 16 * (int32_t)pe - d0;
    const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
    for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * pe + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
  }
}

}  // namespace

hipError_t launch_ralledata(const RalleInputs& in, uint64_t n, uint64_t seed, uint8_t* out, uint64_t* blob_off,
                            hipStream_t stream) {
  if (n == 0) {
    if (blob_off) return hipMemsetAsync(blob_off, 0, 8, stream);
    return hipSuccess;
  }
  // one kernel, the key hashes computed from the staged keys
  const unsigned grid = (unsigned)((n + kGatherRecs - 1) / kGatherRecs);
  if (!in.soff && !in.aoff)
    ralledata_gather_kernel<true><<<grid, 256, 0, stream>>>(in, n, out, blob_off, make_spad(seed));
  else
    ralledata_gather_kernel<false><<<grid, 256, 0, stream>>>(in, n, out, blob_off, make_spad(seed));
  return hipGetLastError();
}

}  // namespace k2h
