/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of yahoojapan/k2hash's key-hash path, used as the parity
 * checker for the HIP kernels and as the CPU baseline ("port") in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this file's library; the product (k2hash_amd/) never links or calls it.
 *
 * Pinned: every function below is checked against (a) the reference itself,
 * compiled from /root/reference/lib/k2hashfunc.cc by oracle/Makefile into
 * oracle/_ref/ (tests/test_oracle.py), and (b) the committed golden vectors in
 * tests/golden/ generated from that build by oracle/gen_golden.c.
 *
 * Reference citations (paths relative to the reference root):
 *   seed 14695981039346656037, prime 1099511628211 ... lib/k2hashfunc.cc:51,56
 *   bytes read through `const char*` (signed on x86-64),
 *   XORed as a sign-extended 64-bit value ............. lib/k2hashfunc.cc:53,55
 *   NULL / length 0 -> 0 ................................ lib/k2hashfunc.cc:66-68, 80-82
 *   second hash = FNV over length-1 bytes if length>1 .. lib/k2hashfunc.cc:83-85
 *   version strings ..................................... lib/k2hashfunc.cc:35-39
 *   USE_STD_FNV_HASH_FUNCTION variant: libstdc++ _Fnv_hash_impl::hash, seed
 *   2166136261 (GCC 11 bits/functional_hash.h:212-217), same signed-char loop
 *   (libstdc++ _Fnv_hash_bytes) ......................... lib/k2hashfunc.cc:69-70, 86-87
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define ORACLE_FNV_SEED_BUILTIN 14695981039346656037ULL
#define ORACLE_FNV_SEED_STD 2166136261ULL
#define ORACLE_FNV_PRIME 1099511628211ULL

/* variant 0 = "FNV-1A BUILTIN" (default build), 1 = "STD::FNV BUILTIN" */
static uint64_t seed_of(int variant) {
  return variant ? ORACLE_FNV_SEED_STD : ORACLE_FNV_SEED_BUILTIN;
}

/* lib/k2hashfunc.cc:49-59: byte-serial xor/multiply over signed chars. */
uint64_t oracle_fnv(const void* ptr, size_t len, uint64_t seed) {
  const signed char* p = (const signed char*)ptr;
  uint64_t h = seed;
  for (size_t i = 0; i < len; ++i) {
    h ^= (uint64_t)(int64_t)p[i];
    h *= ORACLE_FNV_PRIME;
  }
  return h;
}

/* lib/k2hashfunc.cc:62-74 */
uint64_t oracle_k2h_hash(const void* ptr, size_t length, int variant) {
  if (!ptr || length < 1) return 0;
  return oracle_fnv(ptr, length, seed_of(variant));
}

/* lib/k2hashfunc.cc:76-91 */
uint64_t oracle_k2h_second_hash(const void* ptr, size_t length, int variant) {
  if (!ptr || length < 1) return 0;
  if (length > 1) length--;
  return oracle_fnv(ptr, length, seed_of(variant));
}

/* lib/k2hashfunc.cc:35-39, 93-96 */
const char* oracle_k2h_hash_version(int variant) {
  return variant ? "STD::FNV BUILTIN" : "FNV-1A BUILTIN";
}

/* Batch forms used as checkers: CSR (key i = bytes[offsets[i] .. offsets[i+1]))
 * and fixed-length (key i = bytes[i*key_len .. (i+1)*key_len)).  h2 may be NULL. */
void oracle_hash_csr(const uint8_t* bytes, const uint64_t* offsets, size_t n,
                     uint64_t* h1, uint64_t* h2, int variant) {
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* k = bytes + offsets[i];
    size_t len = (size_t)(offsets[i + 1] - offsets[i]);
    h1[i] = oracle_k2h_hash(k, len, variant);
    if (h2) h2[i] = oracle_k2h_second_hash(k, len, variant);
  }
}

void oracle_hash_fixed(const uint8_t* bytes, size_t key_len, size_t n,
                       uint64_t* h1, uint64_t* h2, int variant) {
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* k = bytes + i * key_len;
    h1[i] = oracle_k2h_hash(k, key_len, variant);
    if (h2) h2[i] = oracle_k2h_second_hash(k, key_len, variant);
  }
}

/* ------------------------------------------------------------------------
 * Synthetic-input generator (spec shared with the device generator in
 * k2hash_amd/csrc/k2h_synth.hip; independent implementation, cross-checked
 * by tests).  splitmix64 in counter form: word j of a stream with seed s is
 * mix(s + (j+1) * GAMMA), i.e. the j-th output of splitmix64 seeded with s.
 * ------------------------------------------------------------------------ */
#define GAMMA 0x9E3779B97F4A7C15ULL

uint64_t oracle_splitmix_word(uint64_t seed, uint64_t j) {
  uint64_t z = seed + (j + 1) * GAMMA;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* Bytes [byte_off, byte_off+nbytes) of the little-endian word stream. */
void oracle_gen_bytes(uint64_t seed, uint64_t byte_off, size_t nbytes, uint8_t* out) {
  size_t i = 0;
  while (i < nbytes) {
    uint64_t pos = byte_off + i;
    uint64_t w = oracle_splitmix_word(seed, pos >> 3);
    for (unsigned sh = (unsigned)(pos & 7); sh < 8 && i < nbytes; ++sh) out[i++] = (uint8_t)(w >> (8 * sh));
  }
}

/* CSR lengths: len_i = min_len + mix(seed, i) % (max_len - min_len + 1);
 * offsets[0] = 0, offsets[i+1] = offsets[i] + len_i. */
void oracle_gen_offsets(uint64_t seed, uint64_t first_key, size_t n, uint32_t min_len,
                        uint32_t max_len, uint64_t base, uint64_t* offsets) {
  uint64_t span = (uint64_t)(max_len - min_len) + 1;
  offsets[0] = base;
  for (size_t i = 0; i < n; ++i) {
    uint64_t len = min_len + oracle_splitmix_word(seed, first_key + i) % span;
    offsets[i + 1] = offsets[i] + len;
  }
}

/* Order-sensitive digest of a hash vector: {xor, wrapping sum, sum of h*(2i+1)}. */
void oracle_digest(const uint64_t* h, size_t n, uint64_t first_index, uint64_t out[3]) {
  uint64_t x = 0, s = 0, w = 0;
  for (size_t i = 0; i < n; ++i) {
    x ^= h[i];
    s += h[i];
    w += h[i] * (2 * (first_index + i) + 1);
  }
  out[0] = x;
  out[1] = s;
  out[2] = w;
}

/* ---------------------------------------------------------------------------
 * The exact split of one key's FNV-1a chain at byte m (the algebra a
 * two-lane hash of one long key would use).  Per byte b with s = sext(b) (lib/k2hashfunc.cc
 * :53-56) and v = h mod 256, w = v ^ b:
 *   h ^ s = +h + (w - v)          for b <  0x80   (only the low byte changes)
 *   h ^ s = -h + (v + w - 256)    for b >= 0x80   (~h = -h - 1 above the low byte)
 * so h' = P (sigma h + d) with sigma = +-1 and d depending on (v, b) only, and the low byte
 * runs its own chain v' = 0xB3 (v ^ b) mod 256 (P mod 256 = 0xB3).  Over bytes [m, N):
 *   h_N = K (P^(N-m) h_m + E),  K = prod sigma,  E_{n+1} = P (E_n + K_{n+1} d_n), E_m = 0
 * so a second lane that knows v_m (the 8-bit chain over [0, m)) computes (K, E) while the
 * first lane computes h_m, and h_N follows from one multiply-add.
 * ------------------------------------------------------------------------- */
static uint64_t fnv_pow(uint64_t b, uint64_t e) {
  uint64_t r = 1;
  for (; e; e >>= 1, b *= b)
    if (e & 1) r *= b;
  return r;
}

uint64_t oracle_fnv_split(const uint8_t* p, size_t len, size_t m, uint64_t seed) {
  const uint64_t P = 1099511628211ULL;
  /* lane A: the plain chain over [0, m) */
  uint64_t hm = seed;
  for (size_t i = 0; i < m; ++i) hm = (hm ^ (uint64_t)(int64_t)(signed char)p[i]) * P;
  /* lane B: the low byte over [0, m), then (K, E) over [m, len) */
  uint32_t v = (uint32_t)(seed & 0xFF);
  for (size_t i = 0; i < m; ++i) v = (0xB3u * (v ^ p[i])) & 0xFFu;
  int64_t K = 1;
  uint64_t E = 0;
  for (size_t i = m; i < len; ++i) {
    const uint32_t w = v ^ p[i];
    const int neg = p[i] >= 0x80;
    const int64_t d = neg ? (int64_t)v + (int64_t)w - 256 : (int64_t)w - (int64_t)v;
    if (neg) K = -K;
    E = P * (E + (uint64_t)(K * d));
    v = (0xB3u * w) & 0xFFu;
  }
  const uint64_t r = fnv_pow(P, (uint64_t)(len - m)) * hm + E;
  return K > 0 ? r : (uint64_t)0 - r;
}

/* Number of split points m in [0, len] where the split disagrees with the direct chain. */
size_t oracle_fnv_split_mismatches(const uint8_t* p, size_t len, uint64_t seed) {
  size_t bad = 0;
  for (size_t m = 0; m <= len; ++m)
    if (oracle_fnv_split(p, len, m, seed) != oracle_fnv(p, len, seed)) ++bad;
  return bad;
}

/* ---------------------------------------------------------------------------
 * Bucket index: the stateless part of K2HShm::GetKIndexPos and
 * the collision slot of K2HShm::GetCKIndex, restated loop for loop.  The reference
 * functions are K2HShm members needing the mapped table and libfullock, so they are
 * not compiled here; this restatement is the checker.
 * ------------------------------------------------------------------------- */
/* lib/k2hshm.cc:78-83 K2HShm::MakeMask */
uint64_t oracle_make_mask(int bitcnt) {
  uint64_t mask;
  for (mask = 0UL; 0 < bitcnt; mask = ((mask << 1) | 1UL), bitcnt--);
  return mask;
}

/* lib/k2hshm.cc:85-90 K2HShm::GetMaskBitCount */
int oracle_mask_bitcount(uint64_t mask) {
  int bitcnt;
  for (bitcnt = 0; 0 != mask; bitcnt++, mask = (mask >> 1));
  return bitcnt;
}

/* lib/k2hshm.cc:810-833 K2HShm::GetKIndexPos (cur_mask = *pCurMask or pHead->cur_mask)
 * and lib/k2hshm.cc:1093 (hash & collision_mask).  The reference shifts by
 * GetMaskBitCount(collision_mask), which is 64 for a full mask: x86-64 takes shift
 * counts mod 64, so `& 63` here states what the reference build computes. */
void oracle_kindex_pos(uint64_t hash, uint64_t cur_mask, uint64_t collision_mask, uint64_t* kiptr_pos,
                       uint64_t* kiarray_pos, uint64_t* ckindex) {
  uint64_t shifted_hash = hash >> (oracle_mask_bitcount(collision_mask) & 63);
  uint64_t bitmask, tmphash, pos;
  for (tmphash = shifted_hash & cur_mask, pos = 0UL, bitmask = 0UL; 0 != (tmphash & ~bitmask);
       pos++, bitmask = ((bitmask << 1) | 1UL));
  *kiptr_pos = pos;
  *kiarray_pos = shifted_hash & oracle_make_mask(0 < pos ? (int)(pos - 1) : 0);
  *ckindex = hash & collision_mask;
}

/* Batch form with the ABI's packing: kindex = KIPtrArrayPos << 58 | KIArrayPos. */
void oracle_bucket_index(const uint64_t* h, size_t n, uint64_t cur_mask, uint64_t collision_mask,
                         uint64_t* kindex, uint64_t* ckindex) {
  for (size_t i = 0; i < n; ++i) {
    uint64_t p, a, c;
    oracle_kindex_pos(h[i], cur_mask, collision_mask, &p, &a, &c);
    if (kindex) kindex[i] = (p << 58) | a;
    if (ckindex) ckindex[i] = c;
  }
}

/* lib/k2hshm.cc:862-907 K2HShm::GetKIndex(hash, isMergeCurmask = false): walk cur_mask
 * down (cur_mask >>= 1 while > 0), computing GetKIndexPos with each mask (the
 * pCurMask form, lib/k2hshm.cc:810-833), and stop at the first K_INDEX whose `assign` is
 * KINDEX_ASSIGNED (lib/k2hstructure.h:40-41, 160-165); if none is, the pointer of the
 * last probe (mask 1) is what the loop leaves in pKindex; with cur_mask 0 the loop does
 * not run and the result is NULL.  The isMergeCurmask = true form also rearranges the
 * table (ArrangeToUpperKIndex), a write this batch form does not model.
 *
 * Table state: `assigned` is a bitmap with one bit per K_INDEX entry of the mapped
 * table, entry KIArrayPos of key_index_area[KIPtrArrayPos] (CVT_ABS_PKINDEX,
 * lib/k2hshm.cc:50) at bit  KIPtrArrayPos ? 2^(KIPtrArrayPos-1) + KIArrayPos : 0
 * (area p holds 2^(p-1) entries, area 0 one: the table's cur_mask + 1 entries in area
 * order).  Returns 1 (assigned entry reached), 0 (walk ended on an unassigned entry),
 * -1 (cur_mask 0: NULL).  Parity of this walk is unpinned: K2HShm needs the mapped table
 * and libfullock, so the reference's GetKIndex is not executed here; only its stateless
 * part (GetKIndexPos) is pinned, by the dsave fixture and the key_index_area table. */
int oracle_get_kindex(uint64_t hash, uint64_t cur_mask, uint64_t collision_mask, const uint32_t* assigned,
                      uint64_t* kiptr_pos, uint64_t* kiarray_pos) {
  int found = -1;
  for (uint64_t m = cur_mask; 0 < m; m = m >> 1) {
    uint64_t p, a, c;
    oracle_kindex_pos(hash, m, collision_mask, &p, &a, &c);
    *kiptr_pos = p;
    *kiarray_pos = a;
    const uint64_t bit = p ? (1ull << (p - 1)) + a : 0;
    if ((assigned[bit >> 5] >> (bit & 31)) & 1u) return 1;
    found = 0;
  }
  return found;
}

/* Batch form: kindex packed as above, K2H_AMD_KINDEX_NONE (all ones) for NULL; found[i]
 * = 1 when an assigned entry was reached. */
void oracle_bucket_index_table(const uint64_t* h, size_t n, uint64_t cur_mask, uint64_t collision_mask,
                               const uint32_t* assigned, uint64_t* kindex, uint64_t* ckindex, uint8_t* found) {
  for (size_t i = 0; i < n; ++i) {
    uint64_t p = 0, a = 0;
    const int r = oracle_get_kindex(h[i], cur_mask, collision_mask, assigned, &p, &a);
    if (kindex) kindex[i] = r < 0 ? ~0ull : (p << 58) | a;
    if (ckindex) ckindex[i] = h[i] & collision_mask;
    if (found) found[i] = r > 0;
  }
}

/* ---------------------------------------------------------------------------
 * RALLEDATA producer, restated: one packed blob per record,
 * laid out as K2HShm::GetElementToBinary does (lib/k2hshmdirect.cc:59-88) on the
 * packed struct of lib/k2hshmdirect.h:36-47 (10 little-endian 8-byte fields:
 * hash, subhash, key/val/skey/attrs lengths, key/val/skey/attrs positions from the
 * struct top), hash/subhash = k2h_hash / k2h_second_hash of the key
 * (lib/k2hshm.cc:2184-2185).  Blobs are packed back to back: blob i starts at
 * 80*i + sum of the bytes of records < i.  Segment offset arrays may be NULL
 * (segment empty for every record).  Pinned by tests/golden/ralledata.json, which
 * oracle/gen_ralledata.cc writes from the reference's own header and hash build.
 * ------------------------------------------------------------------------- */
static void put64(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

uint64_t oracle_build_ralledata(const uint8_t* keys, const uint64_t* koff, const uint8_t* vals, const uint64_t* voff,
                                const uint8_t* skeys, const uint64_t* soff, const uint8_t* attrs,
                                const uint64_t* aoff, size_t n, uint8_t* out, uint64_t* blob_off, int variant) {
  uint64_t o = 0;
  for (size_t i = 0; i < n; ++i) {
    uint64_t kl = koff[i + 1] - koff[i];
    uint64_t vl = voff ? voff[i + 1] - voff[i] : 0;
    uint64_t sl = soff ? soff[i + 1] - soff[i] : 0;
    uint64_t al = aoff ? aoff[i + 1] - aoff[i] : 0;
    if (blob_off) blob_off[i] = o;
    uint8_t* b = out + o;
    put64(b + 0, oracle_k2h_hash(keys + koff[i], kl, variant));
    put64(b + 8, oracle_k2h_second_hash(keys + koff[i], kl, variant));
    put64(b + 16, kl);
    put64(b + 24, vl);
    put64(b + 32, sl);
    put64(b + 40, al);
    put64(b + 48, 80);
    put64(b + 56, 80 + kl);
    put64(b + 64, 80 + kl + vl);
    put64(b + 72, 80 + kl + vl + sl);
    if (kl) memcpy(b + 80, keys + koff[i], kl);
    if (vl) memcpy(b + 80 + kl, vals + voff[i], vl);
    if (sl) memcpy(b + 80 + kl + vl, skeys + soff[i], sl);
    if (al) memcpy(b + 80 + kl + vl + sl, attrs + aoff[i], al);
    o += 80 + kl + vl + sl + al;
  }
  if (blob_off) blob_off[n] = o;
  return o;
}
