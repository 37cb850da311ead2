// Round-3 lab: RALLEDATA gather-kernel variants, one TU with the product
// RALLEDATA source so the variants share its helpers.  Not part of the product.
//   variant 0: the product kernel; 1: wave 1 hashes the keys from HBM during the staging;
//   2: wave 1 stages the key span itself and hashes it before the block barrier;
//   3: the next segment's window read only for pieces that cross into it; 4: 3 with the
//   next piece's table entry read one piece ahead; 5: the product with the table entry one
//   piece ahead; 6: the product with the table entry and both segments one piece ahead;
//   7: the record offsets of every segment loaded without branches (one latency).
#include "k2h_ralledata.hip"

namespace k2h {
namespace {

// Variant 1: wave 1 hashes the block's keys straight from HBM (its own key-offset loads,
// then the key chunks, issued beside its share of the staged loads) while wave 0 does the
// record work, so the hash phase and the second barrier leave the tile's critical path.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void ralle_v1_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  constexpr int R = kGatherRecs, NSEG = 5 * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ int2 seg[NSEG + 1];     // segment g: .x = adj (span byte y sits at img[y + adj]), .y = its end in the span
  __shared__ uint16_t tab[kGatherPieces];  // segment holding piece p's first byte
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
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
  // wave 1: its record's key bounds (the same words wave 0 loads; L2 hits)
  uint64_t hk_b = 0, hk_e = 0;
  const uint32_t hrec = tid - 64;
  const bool hasher = tid >= 64 && tid < 128 && hrec < nr && in.koff;
  if (hasher) {
    hk_b = in.koff[r0 + hrec];
    hk_e = in.koff[r0 + hrec + 1];
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
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t q = (uint64_t)tid - SW + NST * u;
    dst[u] = 0xffffffffu;
    if (tid >= SW && q < hull_total) {
      uint64_t addr = 0, before = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (q >= before && q < before + hull_n[s]) addr = hull_lo[s] + 16 * (q - before);
        before += hull_n[s];
      }
      v[u] = *reinterpret_cast<const u32x4_al*>((uintptr_t)addr);
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // 1h. wave 1: the key hash from HBM (end-aligned chunks, the first one's lead bytes
  // masked; a key ending less than 16k bytes into the buffer reads its first chunk
  // bytewise).  The chunk loads go out behind the staged loads; the staged pieces are
  // written to the image first, so their registers are free during the hash.
  const bool hk = hasher && hk_e > hk_b;
  const uint64_t klen = hk_e - hk_b, kk = (klen + 15) >> 4;
  const uint32_t kp = (uint32_t)(16 * kk - klen);
  const uint8_t* kcp = in.keys + hk_e - 16 * kk;
  u32x4_ua w0 = {0, 0, 0, 0}, w1 = {0, 0, 0, 0}, w2 = {0, 0, 0, 0}, w3 = {0, 0, 0, 0};
  if (hk) {
    if (hk_e >= 16 * kk) {
      w0 = *reinterpret_cast<const u32x4_ua*>(kcp);
    } else {
      uint64_t a0 = 0, a1 = 0;
      for (uint32_t j = kp; j < 16; ++j) {
        const uint64_t b = kcp[j];
        if (j < 8) a0 |= b << (8 * j);
        else a1 |= b << (8 * (j - 8));
      }
      w0 = u32x4_ua{(uint32_t)a0, (uint32_t)(a0 >> 32), (uint32_t)a1, (uint32_t)(a1 >> 32)};
    }
    // chunks 1..3 issued with chunk 0 (BASELINE-like keys are <= 64 B)
    if (kk > 1) w1 = *reinterpret_cast<const u32x4_ua*>(kcp + 16);
    if (kk > 2) w2 = *reinterpret_cast<const u32x4_ua*>(kcp + 32);
    if (kk > 3) w3 = *reinterpret_cast<const u32x4_ua*>(kcp + 48);
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  uint64_t kh1 = 0, kh2 = 0;
  if (hk) {
    const uint64_t st = spad_tab.v[kp & 15];
    uint32_t lo = (uint32_t)st, hi = (uint32_t)(st >> 32), lo2 = lo, hi2 = hi;
    const int32_t sh = (int32_t)(8 * kp);
    auto lead = [sh](int32_t b) -> uint32_t { return (uint32_t)(~0ull << min(max(sh - b, 0), 32)); };
    uint4 c = make_uint4(w0.x & lead(0), w0.y & lead(32), w0.z & lead(64), w0.w & lead(96));
    if (kk > 1) {
      fnv_chunk16(lo, hi, c);
      c = make_uint4(w1.x, w1.y, w1.z, w1.w);
    }
    if (kk > 2) {
      fnv_chunk16(lo, hi, c);
      c = make_uint4(w2.x, w2.y, w2.z, w2.w);
    }
    if (kk > 3) {
      fnv_chunk16(lo, hi, c);
      c = make_uint4(w3.x, w3.y, w3.z, w3.w);
    }
    for (uint64_t j = 4; j < kk; ++j) {
      fnv_chunk16(lo, hi, c);
      const u32x4_ua v2 = *reinterpret_cast<const u32x4_ua*>(kcp + 16 * j);
      c = make_uint4(v2.x, v2.y, v2.z, v2.w);
    }
    fnv_chunk16_last(lo, hi, lo2, hi2, c);
    kh1 = ((uint64_t)hi << 32) | lo;
    kh2 = klen == 1 ? kh1 : ((uint64_t)hi2 << 32) | lo2;
  }
  // 1b. one thread per record: header, segment table, piece table, blob offset.  All
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
    const uint64_t i = r0 + tid;
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
    for (int c = 1; c < 5; ++c)  // (chunk 0, the hashes: wave 1)
      *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid + 16 * c) = u32x4_al{f[4 * c], f[4 * c + 1], f[4 * c + 2], f[4 * c + 3]};
    int32_t start = B;
    int32_t p = tid == 0 ? 0 : (B + d0 + 15) >> 4;  // first piece whose first byte is in this record
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const uint32_t g = 5 * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = int2{adj, start + L};
      for (; 16 * p - d0 < start + L; ++p) tab[p] = (uint16_t)g;  // pieces starting in this segment
      start += L;
    }
    if (tid + 1 == nr) seg[5 * nr] = int2{kGatherHdr, start};  // read (never used) as the last segment's successor
    if (blob_off) {
      blob_off[i] = o_first + B;
      if (i + 1 == n) blob_off[n] = o_first + start;
    }
  }
  if (tid >= 64 && tid < 128 && hrec < nr)
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * hrec) =
        u32x4_al{(uint32_t)kh1, (uint32_t)(kh1 >> 32), (uint32_t)kh2, (uint32_t)(kh2 >> 32)};
  __syncthreads();
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
    if (pos < end) {
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg[++g];
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    if (x >= 0 && x + 16 <= sp) {
      __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_al*>(base + 16ull * p));
    } else {  // shared with a neighbouring block: this block's bytes only
      const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * p + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
    }
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  for (uint32_t p = tid; p < np; p += 256) {
    const uint32_t g = tab[p];
    const int2 s0 = seg[g], s1 = seg[g + 1];  // the piece's segment and the next, one read
    piece(p, g, s0, s1, window(s0, p), window(s1, p));
  }
}


// Variant 2: wave 1 stages the key span alone and hashes the keys from it as soon as its
// own loads land (a wave-local wait, no block barrier); waves 2-3 stage the other spans;
// wave 0 does the record work.  One block barrier before the pieces.  Tiles whose key
// span exceeds wave 1's 4 pieces per lane run the product kernel's order.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void ralle_v2_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  constexpr int R = kGatherRecs, NSEG = 5 * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ int2 seg[NSEG + 1];     // segment g: .x = adj (span byte y sits at img[y + adj]), .y = its end in the span
  __shared__ uint16_t tab[kGatherPieces];  // segment holding piece p's first byte
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
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
  // 1a. the staged pieces.  Split form (key span <= 256 pieces): wave 1 loads the key
  // pieces (stride 64), waves 2-3 the others (stride 128); else waves 1-3 all pieces.
  constexpr uint32_t KPT = 4, VPT = (kGatherPool / 16 + 127) / 128;  // 4, 6
  const bool split = hull_n[0] <= 64 * KPT;
  u32x4_al v[VPT];
  uint32_t dst[VPT];
  auto piece_addr = [&](uint64_t q) {
    uint64_t addr = 0, before = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if (q >= before && q < before + hull_n[s]) addr = hull_lo[s] + 16 * (q - before);
      before += hull_n[s];
    }
    return addr;
  };
  const uint32_t wv = tid >> 6;
#pragma unroll
  for (int u = 0; u < (int)VPT; ++u) {
    uint64_t q;
    if (split) q = wv == 1 ? (u < (int)KPT ? (uint64_t)(tid - 64) + 64 * u : ~0ull)
                           : hull_n[0] + (uint64_t)(tid - 128) + 128 * u;
    else q = u < 4 ? (uint64_t)tid - 64 + 192 * u : ~0ull;
    const uint64_t qend = split && wv == 1 ? hull_n[0] : hull_total;
    dst[u] = 0xffffffffu;
    if (tid >= 64 && q < qend) {
      v[u] = *reinterpret_cast<const u32x4_al*>((uintptr_t)piece_addr(q));
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // wave 1, split form: its key pieces into the image, then the keys hashed from there
  if (split && wv == 1) {
#pragma unroll
    for (int u = 0; u < (int)VPT; ++u)
      if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
    if (tid < 80) spad[tid - 64] = spad_tab.v[tid - 64];  // (wave 0 writes the same values)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t hrec = tid - 64;
    if (hrec < nr) {
      const uint32_t kb = in.koff ? (uint32_t)in.koff[r0 + hrec] : 0u, ke = in.koff ? (uint32_t)in.koff[r0 + hrec + 1] : 0u;
      uint64_t h1 = 0, h2 = 0;
      if (ke > kb) staged_key_hash(img + area[0] + (ke - (uint32_t)sbase[0]), ke - kb, spad, h1, h2);
      *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * hrec) =
          u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
    }
#pragma unroll
    for (int u = 0; u < (int)VPT; ++u) dst[u] = 0xffffffffu;
  }
  // 1b. one thread per record: header, segment table, piece table, blob offset.  All
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
    const uint64_t i = r0 + tid;
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
    for (int c = 0; c < 5; ++c)  // (split form: chunk 0, the hashes, by wave 1)
      if (c > 0 || !split) *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid + 16 * c) = u32x4_al{f[4 * c], f[4 * c + 1], f[4 * c + 2], f[4 * c + 3]};
    int32_t start = B;
    int32_t p = tid == 0 ? 0 : (B + d0 + 15) >> 4;  // first piece whose first byte is in this record
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const uint32_t g = 5 * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = int2{adj, start + L};
      for (; 16 * p - d0 < start + L; ++p) tab[p] = (uint16_t)g;  // pieces starting in this segment
      start += L;
    }
    if (tid + 1 == nr) seg[5 * nr] = int2{kGatherHdr, start};  // read (never used) as the last segment's successor
    if (blob_off) {
      blob_off[i] = o_first + B;
      if (i + 1 == n) blob_off[n] = o_first + start;
    }
  }
#pragma unroll
  for (int u = 0; u < (int)VPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  __syncthreads();
  // 1c. (not split) wave 0 hashes the block's keys from the image into the headers
  if (!split && tid < nr) {
    const uint32_t kl = ro1[0] - ro0[0], ke = ro1[0] - (uint32_t)sbase[0];
    uint64_t h1, h2;
    staged_key_hash(img + area[0] + ke, kl, spad, h1, h2);
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid) =
        u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
  }
  if (!split) __syncthreads();
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
    if (pos < end) {
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg[++g];
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    if (x >= 0 && x + 16 <= sp) {
      __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_al*>(base + 16ull * p));
    } else {  // shared with a neighbouring block: this block's bytes only
      const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * p + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
    }
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  for (uint32_t p = tid; p < np; p += 256) {
    const uint32_t g = tab[p];
    const int2 s0 = seg[g], s1 = seg[g + 1];  // the piece's segment and the next, one read
    piece(p, g, s0, s1, window(s0, p), window(s1, p));
  }
}


// Variant 3: the product kernel with the next segment's window read only for pieces that
// cross into it (one unaligned 16-B LDS read fewer per interior piece).
// The key hashes are computed here from the staged keys (no hash kernel, no scratch).
// Wave 0 only waits for its records' offsets (the staged loads are issued by waves 1-3).
// 7 waves/SIMD (<= 72 VGPRs): the LDS image allows 7 blocks per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void ralle_v3_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  constexpr int R = kGatherRecs, NSEG = 5 * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ int2 seg[NSEG + 1];     // segment g: .x = adj (span byte y sits at img[y + adj]), .y = its end in the span
  __shared__ uint16_t tab[kGatherPieces];  // segment holding piece p's first byte
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
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
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t q = (uint64_t)tid - SW + NST * u;
    dst[u] = 0xffffffffu;
    if (tid >= SW && q < hull_total) {
      uint64_t addr = 0, before = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (q >= before && q < before + hull_n[s]) addr = hull_lo[s] + 16 * (q - before);
        before += hull_n[s];
      }
      v[u] = *reinterpret_cast<const u32x4_al*>((uintptr_t)addr);
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // 1b. one thread per record: header, segment table, piece table, blob offset.  All
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
    const uint64_t i = r0 + tid;
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
    int32_t p = tid == 0 ? 0 : (B + d0 + 15) >> 4;  // first piece whose first byte is in this record
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const uint32_t g = 5 * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = int2{adj, start + L};
      for (; 16 * p - d0 < start + L; ++p) tab[p] = (uint16_t)g;  // pieces starting in this segment
      start += L;
    }
    if (tid + 1 == nr) seg[5 * nr] = int2{kGatherHdr, start};  // read (never used) as the last segment's successor
    if (blob_off) {
      blob_off[i] = o_first + B;
      if (i + 1 == n) blob_off[n] = o_first + start;
    }
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  __syncthreads();
  // 1c. wave 0 hashes the block's keys from the image into the headers
  if (tid < nr) {
    const uint32_t kl = ro1[0] - ro0[0], ke = ro1[0] - (uint32_t)sbase[0];
    uint64_t h1, h2;
    staged_key_hash(img + area[0] + ke, kl, spad, h1, h2);
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid) =
        u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
  }
  __syncthreads();
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
    if (pos < end) {
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg[++g];
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    if (x >= 0 && x + 16 <= sp) {
      __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_al*>(base + 16ull * p));
    } else {  // shared with a neighbouring block: this block's bytes only
      const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * p + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
    }
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  for (uint32_t p = tid; p < np; p += 256) {
    const uint32_t g = tab[p];
    const int2 s0 = seg[g], s1 = seg[g + 1];  // the piece's segment and the next, one read
    // variant 3: the next segment's window only for a piece that reaches into it
    const int32_t x = 16 * (int32_t)p - d0;
    const bool cross = s0.y < min(x + 16, sp);
    const u32x4_ua w0 = window(s0, p);
    u32x4_ua w1 = w0;
    if (cross) w1 = window(s1, p);
    piece(p, g, s0, s1, w0, w1);
  }
}


// Variant 4: variant 3 with the next piece's table entry read one piece ahead.
// The key hashes are computed here from the staged keys (no hash kernel, no scratch).
// Wave 0 only waits for its records' offsets (the staged loads are issued by waves 1-3).
// 7 waves/SIMD (<= 72 VGPRs): the LDS image allows 7 blocks per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void ralle_v4_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  constexpr int R = kGatherRecs, NSEG = 5 * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ int2 seg[NSEG + 1];     // segment g: .x = adj (span byte y sits at img[y + adj]), .y = its end in the span
  __shared__ uint16_t tab[kGatherPieces];  // segment holding piece p's first byte
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
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
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t q = (uint64_t)tid - SW + NST * u;
    dst[u] = 0xffffffffu;
    if (tid >= SW && q < hull_total) {
      uint64_t addr = 0, before = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (q >= before && q < before + hull_n[s]) addr = hull_lo[s] + 16 * (q - before);
        before += hull_n[s];
      }
      v[u] = *reinterpret_cast<const u32x4_al*>((uintptr_t)addr);
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // 1b. one thread per record: header, segment table, piece table, blob offset.  All
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
    const uint64_t i = r0 + tid;
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
    int32_t p = tid == 0 ? 0 : (B + d0 + 15) >> 4;  // first piece whose first byte is in this record
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const uint32_t g = 5 * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = int2{adj, start + L};
      for (; 16 * p - d0 < start + L; ++p) tab[p] = (uint16_t)g;  // pieces starting in this segment
      start += L;
    }
    if (tid + 1 == nr) seg[5 * nr] = int2{kGatherHdr, start};  // read (never used) as the last segment's successor
    if (blob_off) {
      blob_off[i] = o_first + B;
      if (i + 1 == n) blob_off[n] = o_first + start;
    }
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  __syncthreads();
  // 1c. wave 0 hashes the block's keys from the image into the headers
  if (tid < nr) {
    const uint32_t kl = ro1[0] - ro0[0], ke = ro1[0] - (uint32_t)sbase[0];
    uint64_t h1, h2;
    staged_key_hash(img + area[0] + ke, kl, spad, h1, h2);
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid) =
        u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
  }
  __syncthreads();
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
    if (pos < end) {
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg[++g];
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    if (x >= 0 && x + 16 <= sp) {
      __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_al*>(base + 16ull * p));
    } else {  // shared with a neighbouring block: this block's bytes only
      const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * p + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
    }
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  uint32_t gnext = tid < np ? tab[tid] : 0u;
  for (uint32_t p = tid; p < np; p += 256) {
    const uint32_t g = gnext;
    const int2 s0 = seg[g], s1 = seg[g + 1];  // the piece's segment and the next, one read
    gnext = p + 256 < np ? tab[p + 256] : 0u;
    // variant 3: the next segment's window only for a piece that reaches into it
    const int32_t x = 16 * (int32_t)p - d0;
    const bool cross = s0.y < min(x + 16, sp);
    const u32x4_ua w0 = window(s0, p);
    u32x4_ua w1 = w0;
    if (cross) w1 = window(s1, p);
    piece(p, g, s0, s1, w0, w1);
  }
}



// The key hashes are computed here from the staged keys (no hash kernel, no scratch).
// Wave 0 only waits for its records' offsets (the staged loads are issued by waves 1-3).
// 7 waves/SIMD (<= 72 VGPRs): the LDS image allows 7 blocks per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void ralle_v5_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  constexpr int R = kGatherRecs, NSEG = 5 * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ int2 seg[NSEG + 1];     // segment g: .x = adj (span byte y sits at img[y + adj]), .y = its end in the span
  __shared__ uint16_t tab[kGatherPieces];  // segment holding piece p's first byte
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
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
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t q = (uint64_t)tid - SW + NST * u;
    dst[u] = 0xffffffffu;
    if (tid >= SW && q < hull_total) {
      uint64_t addr = 0, before = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (q >= before && q < before + hull_n[s]) addr = hull_lo[s] + 16 * (q - before);
        before += hull_n[s];
      }
      v[u] = *reinterpret_cast<const u32x4_al*>((uintptr_t)addr);
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // 1b. one thread per record: header, segment table, piece table, blob offset.  All
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
    const uint64_t i = r0 + tid;
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
    int32_t p = tid == 0 ? 0 : (B + d0 + 15) >> 4;  // first piece whose first byte is in this record
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const uint32_t g = 5 * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = int2{adj, start + L};
      for (; 16 * p - d0 < start + L; ++p) tab[p] = (uint16_t)g;  // pieces starting in this segment
      start += L;
    }
    if (tid + 1 == nr) seg[5 * nr] = int2{kGatherHdr, start};  // read (never used) as the last segment's successor
    if (blob_off) {
      blob_off[i] = o_first + B;
      if (i + 1 == n) blob_off[n] = o_first + start;
    }
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  __syncthreads();
  // 1c. wave 0 hashes the block's keys from the image into the headers
  if (tid < nr) {
    const uint32_t kl = ro1[0] - ro0[0], ke = ro1[0] - (uint32_t)sbase[0];
    uint64_t h1, h2;
    staged_key_hash(img + area[0] + ke, kl, spad, h1, h2);
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid) =
        u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
  }
  __syncthreads();
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
    if (pos < end) {
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg[++g];
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    if (x >= 0 && x + 16 <= sp) {
      __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_al*>(base + 16ull * p));
    } else {  // shared with a neighbouring block: this block's bytes only
      const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * p + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
    }
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  uint32_t gnext = tid < np ? tab[tid] : 0u;  // variant 5: the next piece's table entry one piece ahead
  for (uint32_t p = tid; p < np; p += 256) {
    const uint32_t g = gnext;
    const int2 s0 = seg[g], s1 = seg[g + 1];  // the piece's segment and the next, one read
    gnext = p + 256 < np ? tab[p + 256] : 0u;
    piece(p, g, s0, s1, window(s0, p), window(s1, p));
  }
}


// The key hashes are computed here from the staged keys (no hash kernel, no scratch).
// Wave 0 only waits for its records' offsets (the staged loads are issued by waves 1-3).
// 7 waves/SIMD (<= 72 VGPRs): the LDS image allows 7 blocks per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void ralle_v6_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  constexpr int R = kGatherRecs, NSEG = 5 * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ int2 seg[NSEG + 1];     // segment g: .x = adj (span byte y sits at img[y + adj]), .y = its end in the span
  __shared__ uint16_t tab[kGatherPieces];  // segment holding piece p's first byte
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
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
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t q = (uint64_t)tid - SW + NST * u;
    dst[u] = 0xffffffffu;
    if (tid >= SW && q < hull_total) {
      uint64_t addr = 0, before = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (q >= before && q < before + hull_n[s]) addr = hull_lo[s] + 16 * (q - before);
        before += hull_n[s];
      }
      v[u] = *reinterpret_cast<const u32x4_al*>((uintptr_t)addr);
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // 1b. one thread per record: header, segment table, piece table, blob offset.  All
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
    const uint64_t i = r0 + tid;
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
    int32_t p = tid == 0 ? 0 : (B + d0 + 15) >> 4;  // first piece whose first byte is in this record
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const uint32_t g = 5 * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = int2{adj, start + L};
      for (; 16 * p - d0 < start + L; ++p) tab[p] = (uint16_t)g;  // pieces starting in this segment
      start += L;
    }
    if (tid + 1 == nr) seg[5 * nr] = int2{kGatherHdr, start};  // read (never used) as the last segment's successor
    if (blob_off) {
      blob_off[i] = o_first + B;
      if (i + 1 == n) blob_off[n] = o_first + start;
    }
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  __syncthreads();
  // 1c. wave 0 hashes the block's keys from the image into the headers
  if (tid < nr) {
    const uint32_t kl = ro1[0] - ro0[0], ke = ro1[0] - (uint32_t)sbase[0];
    uint64_t h1, h2;
    staged_key_hash(img + area[0] + ke, kl, spad, h1, h2);
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid) =
        u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
  }
  __syncthreads();
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
    if (pos < end) {
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg[++g];
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    if (x >= 0 && x + 16 <= sp) {
      __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_al*>(base + 16ull * p));
    } else {  // shared with a neighbouring block: this block's bytes only
      const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * p + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
    }
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  // variant 6: the next piece's table entry and segments read one piece ahead
  uint32_t gn = 0;
  int2 s0n = int2{0, 0}, s1n = int2{0, 0};
  if (tid < np) {
    gn = tab[tid];
    s0n = seg[gn];
    s1n = seg[gn + 1];
  }
  for (uint32_t p = tid; p < np; p += 256) {
    const uint32_t g = gn;
    const int2 s0 = s0n, s1 = s1n;
    const u32x4_ua w0 = window(s0, p), w1 = window(s1, p);
    if (p + 256 < np) {
      gn = tab[p + 256];
      s0n = seg[gn];
      s1n = seg[gn + 1];
    }
    piece(p, g, s0, s1, w0, w1);
  }
}


__device__ uint64_t g_zero_pair[2] = {0, 0};  // (global, not constant: one address space with the offsets)
// The key hashes are computed here from the staged keys (no hash kernel, no scratch).
// Wave 0 only waits for its records' offsets (the staged loads are issued by waves 1-3).
// 7 waves/SIMD (<= 72 VGPRs): the LDS image allows 7 blocks per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void ralle_v7_kernel(
    RalleInputs in, uint64_t n, uint8_t* __restrict__ out, uint64_t* __restrict__ blob_off, SpadTable spad_tab) {
  constexpr int R = kGatherRecs, NSEG = 5 * R;
  typedef uint32_t u32x4_al __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) uint8_t img[kGatherImg];
  __shared__ int2 seg[NSEG + 1];     // segment g: .x = adj (span byte y sits at img[y + adj]), .y = its end in the span
  __shared__ uint16_t tab[kGatherPieces];  // segment holding piece p's first byte
  __shared__ u32x4_al qmask[17];
  __shared__ uint64_t spad[16];
  const uint32_t tid = threadIdx.x;
  const uint64_t r0 = (uint64_t)blockIdx.x * R;
  const uint32_t nr = (uint32_t)(n - r0 < (uint64_t)R ? n - r0 : (uint64_t)R);
  const uint64_t* offs[4] = {in.koff, in.voff, in.soff, in.aoff};
  const uint8_t* srcs[4] = {in.keys, in.vals, in.skeys, in.attrs};
  // the records' own offsets first: they do not depend on the span offsets below
  // variant 7: the record offsets of all segments loaded without branches (a NULL segment
  // reads its own lane's first offset of the key stream... or a zero word), so every load
  // is in flight together
  uint32_t ro0[4] = {0, 0, 0, 0}, ro1[4] = {0, 0, 0, 0};
  if (tid < nr) {
    uint64_t a0[4], a1[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint64_t* p = offs[s] ? offs[s] + r0 + tid : g_zero_pair;
      a0[s] = p[0];
      a1[s] = p[1];
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      ro0[s] = (uint32_t)a0[s];
      ro1[s] = (uint32_t)a1[s];
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
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t q = (uint64_t)tid - SW + NST * u;
    dst[u] = 0xffffffffu;
    if (tid >= SW && q < hull_total) {
      uint64_t addr = 0, before = 0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        if (q >= before && q < before + hull_n[s]) addr = hull_lo[s] + 16 * (q - before);
        before += hull_n[s];
      }
      v[u] = *reinterpret_cast<const u32x4_al*>((uintptr_t)addr);
      dst[u] = kGatherHdr + 80 * R + 16 * (uint32_t)q;
    }
  }
  // 1b. one thread per record: header, segment table, piece table, blob offset.  All
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
    const uint64_t i = r0 + tid;
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
    int32_t p = tid == 0 ? 0 : (B + d0 + 15) >> 4;  // first piece whose first byte is in this record
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      const uint32_t g = 5 * tid + c;
      const int32_t L = c == 0 ? 80 : (int32_t)len[c - 1];
      const int32_t adj = c == 0 ? kGatherHdr + 80 * (int32_t)tid - start : area[c - 1] + (int32_t)rel[c - 1] - start;
      seg[g] = int2{adj, start + L};
      for (; 16 * p - d0 < start + L; ++p) tab[p] = (uint16_t)g;  // pieces starting in this segment
      start += L;
    }
    if (tid + 1 == nr) seg[5 * nr] = int2{kGatherHdr, start};  // read (never used) as the last segment's successor
    if (blob_off) {
      blob_off[i] = o_first + B;
      if (i + 1 == n) blob_off[n] = o_first + start;
    }
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (dst[u] != 0xffffffffu) *reinterpret_cast<u32x4_al*>(img + dst[u]) = v[u];
  __syncthreads();
  // 1c. wave 0 hashes the block's keys from the image into the headers
  if (tid < nr) {
    const uint32_t kl = ro1[0] - ro0[0], ke = ro1[0] - (uint32_t)sbase[0];
    uint64_t h1, h2;
    staged_key_hash(img + area[0] + ke, kl, spad, h1, h2);
    *reinterpret_cast<u32x4_al*>(img + kGatherHdr + 80 * tid) =
        u32x4_al{(uint32_t)h1, (uint32_t)(h1 >> 32), (uint32_t)h2, (uint32_t)(h2 >> 32)};
  }
  __syncthreads();
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
    if (pos < end) {
      if (s1.y > pos) {
        merge(w1);
        pos = s1.y;
      }
      ++g;
      while (pos < end) {
        const int2 sn = seg[++g];
        if (sn.y > pos) {
          merge(*reinterpret_cast<const u32x4_ua*>(img + sn.x + x));
          pos = sn.y;
        }
      }
    }
    if (x >= 0 && x + 16 <= sp) {
      __builtin_nontemporal_store(acc, reinterpret_cast<u32x4_al*>(base + 16ull * p));
    } else {  // shared with a neighbouring block: this block's bytes only
      const uint32_t wv[4] = {acc.x, acc.y, acc.z, acc.w};
      for (int k = max(0, -x); k < 16 && x + k < sp; ++k) base[16ull * p + k] = (uint8_t)(wv[k >> 2] >> (8 * (k & 3)));
    }
  };
  // A piece's next segment is read before it is known to reach into the piece (the read is
  // then discarded), and its window can fall outside the image (e.g. a long pool segment
  // followed by the next record's header): clamp the index into the image.
  auto window = [&](int2 sg, uint32_t p) {
    const int32_t at = min(max(sg.x + 16 * (int32_t)p - d0, 0), kGatherImg - 16);
    return *reinterpret_cast<const u32x4_ua*>(img + at);
  };
  for (uint32_t p = tid; p < np; p += 256) {
    const uint32_t g = tab[p];
    const int2 s0 = seg[g], s1 = seg[g + 1];  // the piece's segment and the next, one read
    piece(p, g, s0, s1, window(s0, p), window(s1, p));
  }
}


}  // namespace
}  // namespace k2h

extern "C" __attribute__((visibility("default"))) int k2h_lab_ralle(int variant, const void* keys, const void* koff,
                                                                   const void* vals, const void* voff, uint64_t n,
                                                                   void* out, void* blob_off, void* stream) {
  using namespace k2h;
  RalleInputs in;
  in.keys = (const uint8_t*)keys;
  in.koff = (const uint64_t*)koff;
  in.vals = (const uint8_t*)vals;
  in.voff = (const uint64_t*)voff;
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = (unsigned)((n + kGatherRecs - 1) / kGatherRecs);
  if (variant == 0) return launch_ralledata(in, n, kSeedBuiltinValue, (uint8_t*)out, (uint64_t*)blob_off, st) == hipSuccess ? 0 : 1;
  if (variant == 1)
    ralle_v1_kernel<<<g, 256, 0, st>>>(in, n, (uint8_t*)out, (uint64_t*)blob_off, make_spad(kSeedBuiltinValue));
  else if (variant == 7)
    ralle_v7_kernel<<<g, 256, 0, st>>>(in, n, (uint8_t*)out, (uint64_t*)blob_off, make_spad(kSeedBuiltinValue));
  else if (variant == 5)
    ralle_v5_kernel<<<g, 256, 0, st>>>(in, n, (uint8_t*)out, (uint64_t*)blob_off, make_spad(kSeedBuiltinValue));
  else if (variant == 6)
    ralle_v6_kernel<<<g, 256, 0, st>>>(in, n, (uint8_t*)out, (uint64_t*)blob_off, make_spad(kSeedBuiltinValue));
  else if (variant == 4)
    ralle_v4_kernel<<<g, 256, 0, st>>>(in, n, (uint8_t*)out, (uint64_t*)blob_off, make_spad(kSeedBuiltinValue));
  else if (variant == 3)
    ralle_v3_kernel<<<g, 256, 0, st>>>(in, n, (uint8_t*)out, (uint64_t*)blob_off, make_spad(kSeedBuiltinValue));
  else if (variant == 2)
    ralle_v2_kernel<<<g, 256, 0, st>>>(in, n, (uint8_t*)out, (uint64_t*)blob_off, make_spad(kSeedBuiltinValue));
  else
    return 2;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
