/*
 * k2hash_amd -- MI355X-native key-hash path for yahoojapan/k2hash.
 *
 * C ABI of the two shared libraries built from k2hash_amd/csrc/:
 *
 *   libk2hfnv_plugin.so   the DROP-IN hash plugin.  Exports exactly the three
 *                         symbols k2hash's plugin loader resolves (section 1).
 *                         Pure C++, no HIP dependency, safe to dlopen from any
 *                         process/thread and across fork.
 *   libk2hash_amd.so      the same three symbols plus the batch ABI (section 2)
 *                         backed by hand-written CDNA4 HIP kernels.  Also a valid
 *                         plugin; HIP is initialised lazily by the first batch call.
 *
 * All hashes are bit-identical to the reference's default build
 * (lib/k2hashfunc.cc, "FNV-1A BUILTIN"), or, with K2H_AMD_FLAG_STD_FNV, to its
 * USE_STD_FNV_HASH_FUNCTION build ("STD::FNV BUILTIN").
 */
#ifndef K2HASH_AMD_H
#define K2HASH_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* lib/k2hash.h:37 */
typedef uint64_t k2h_hash_t;

/* ---------------------------------------------------------------------------
 * 1. Drop-in plugin ABI.
 *
 * Replaces the weak builtins declared at lib/k2hashfunc.h:62-74 and defined at
 * lib/k2hashfunc.cc:62-96.  K2HashDynLib::Load (lib/k2hashfunc.cc:132-161,
 * reached from k2h_load_hash_library, lib/k2hash.cc:106-117, and from the tools'
 * -ext options, e.g. tests/k2hlinetool.cc:4995-5008) dlopen()s the plugin with
 * RTLD_LAZY and dlsym()s these three names, all-or-nothing
 * (lib/k2hashfunc.cc:149-156).  The same symbols also override the builtins at
 * link time or through LD_PRELOAD (lib/k2hcommon.h:41-45, docs/k2hash.1:50-55).
 *
 * Semantics (identical to the reference):
 *   - ptr == NULL or length == 0 -> 0            (lib/k2hashfunc.cc:66-68, 80-82)
 *   - k2h_hash: FNV-1a-64 over `length` bytes, each byte read as signed char
 *     and sign-extended before the XOR               (lib/k2hashfunc.cc:49-59)
 *   - k2h_second_hash: same over length-1 bytes when length > 1
 *                                                     (lib/k2hashfunc.cc:83-85)
 *   - k2h_hash_version: "FNV-1A BUILTIN" -- the reference's own string, because
 *     the hashes are identical and the string is stamped into / checked against
 *     every k2hash file header (lib/k2hshminit.cc:405, 641-646).  < 32 bytes
 *     (lib/k2hash.h:69).
 * Reentrant, lock-free, allocation-free, never throws or logs; no GPU work.
 * ------------------------------------------------------------------------- */
k2h_hash_t k2h_hash(const void* ptr, size_t length);        /* lib/k2hashfunc.h:65 */
k2h_hash_t k2h_second_hash(const void* ptr, size_t length); /* lib/k2hashfunc.h:68 */
const char* k2h_hash_version(void);                         /* lib/k2hashfunc.h:72 */

/* ---------------------------------------------------------------------------
 * 2. Batch ABI (new surface; libk2hash_amd.so only).
 *
 * The reference has no batch entry point: every call site hashes one key
 * synchronously (lib/k2hshm.cc:1230-1231, 2184-2185, ...).  Bulk callers
 * (bulk loads, archive import, RALLEDATA producers, benches) use these.
 *
 * Return value: K2H_AMD_OK (0) or a negative K2H_AMD_E* code;
 * k2h_amd_strerror() describes the last failure on the calling thread.
 * Per-key results follow the plugin semantics above; a key of length 0 hashes
 * to 0 (h1 and h2), and so does every key when the byte buffer is NULL.
 * h2 may be NULL (second hash not wanted).  `stream` is a hipStream_t
 * (NULL = the null stream); device-pointer calls are asynchronous on it.
 * ------------------------------------------------------------------------- */
#define K2H_AMD_OK 0
#define K2H_AMD_EINVAL (-1)   /* bad argument (NULL output, overflow, ...) */
#define K2H_AMD_EHIP (-2)     /* HIP runtime error (see k2h_amd_strerror) */
#define K2H_AMD_ENOMEM (-3)   /* device / pinned host allocation failed */
#define K2H_AMD_ENODEV (-4)   /* no usable gfx950 device */

#define K2H_AMD_FLAG_STD_FNV 0x1u /* USE_STD_FNV_HASH_FUNCTION build: seed 2166136261
                                      (lib/k2hashfunc.cc:35-37, 69-70, 86-87) */

/* Fixed-length keys in device memory: key i = keys[i*key_len, (i+1)*key_len). */
int k2h_amd_hash_fixed(const void* keys, uint64_t key_len, uint64_t n, uint64_t* h1, uint64_t* h2, uint32_t flags,
                       void* stream);

/* CSR keys in device memory: key i = bytes[offsets[i], offsets[i+1]), offsets has n+1
 * non-decreasing entries (byte offsets relative to `bytes`). */
int k2h_amd_hash_csr(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1, uint64_t* h2,
                     uint32_t flags, void* stream);

/* Host-memory forms: same layouts, host pointers in and out.  The library stages
 * through pinned buffers and overlaps H2D / kernel / D2H in chunks on `device`.
 * Synchronous: returns when h1/h2 are filled.  The CSR form checks its offsets chunk
 * by chunk as it streams them; offsets that decrease return K2H_AMD_EINVAL, and the
 * contents of h1/h2 are then unspecified (earlier chunks may have been written). */
int k2h_amd_hash_fixed_host(const void* keys, uint64_t key_len, uint64_t n, uint64_t* h1, uint64_t* h2,
                            uint32_t flags, int device);
int k2h_amd_hash_csr_host(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1, uint64_t* h2,
                          uint32_t flags, int device);

/* ---------------------------------------------------------------------------
 * 3. Bucket-index epilogue (where each key lands in a k2hash table).
 *
 * For table masks (cur_mask, collision_mask) -- K2HSHM header fields, e.g. the
 * defaults 0xFF / 0xF of K2HShm::DEFAULT_MASK_BITCOUNT / DEFAULT_COLLISION_MASK_BITCOUNT
 * (lib/k2hshm.h:132-133) -- computes per hash h the stateless part of
 * K2HShm::GetKIndexPos (lib/k2hshm.cc:810-833, MakeMask / GetMaskBitCount at :78-90)
 * and the collision slot of K2HShm::GetCKIndex (lib/k2hshm.cc:1093):
 *   shifted       = h >> GetMaskBitCount(collision_mask)   (count taken mod 64)
 *   KIPtrArrayPos = GetMaskBitCount(shifted & cur_mask)
 *   KIArrayPos    = shifted & MakeMask(KIPtrArrayPos ? KIPtrArrayPos - 1 : 0)
 *   kindex[i]     = KIPtrArrayPos << 58 | KIArrayPos     (K2H_AMD_KINDEX_* below)
 *   ckindex[i]    = h & collision_mask
 * i.e. &key_index_area[KIPtrArrayPos][KIArrayPos] (CVT_ABS_PKINDEX, lib/k2hshm.cc:50)
 * and &ckey_list[ckindex].  The table-state part of GetKIndex (walking cur_mask down
 * past unassigned K_INDEX entries, lib/k2hshm.cc:882-907) is the *_table forms below.
 * kindex and ckindex may each be NULL; cur_mask must fit 58 bits when kindex is wanted.
 * The fused forms hash and index in one pass (the index costs no extra key read).
 * ------------------------------------------------------------------------- */
#define K2H_AMD_KINDEX_POS(v) ((uint64_t)(v) >> 58)                     /* KIPtrArrayPos */
#define K2H_AMD_KINDEX_ARR(v) ((uint64_t)(v) & ((1ull << 58) - 1ull))  /* KIArrayPos */

int k2h_amd_bucket_index(const uint64_t* h1, uint64_t n, uint64_t cur_mask, uint64_t collision_mask,
                         uint64_t* kindex, uint64_t* ckindex, void* stream);
int k2h_amd_hash_fixed_index(const void* keys, uint64_t key_len, uint64_t n, uint64_t* h1, uint64_t* h2,
                             uint32_t flags, uint64_t cur_mask, uint64_t collision_mask, uint64_t* kindex,
                             uint64_t* ckindex, void* stream);
int k2h_amd_hash_csr_index(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1, uint64_t* h2,
                           uint32_t flags, uint64_t cur_mask, uint64_t collision_mask, uint64_t* kindex,
                           uint64_t* ckindex, void* stream);

/* Table-state forms: the K_INDEX that K2HShm::GetKIndex(hash, isMergeCurmask = false)
 * returns (lib/k2hshm.cc:862-907) for a snapshot of the table's assigned flags: cur_mask
 * walked down (cur_mask >>= 1 while > 0) until the entry GetKIndexPos gives for that mask
 * has assign == KINDEX_ASSIGNED (lib/k2hstructure.h:40-41).  Without the side effect of
 * the isMergeCurmask = true form (ArrangeToUpperKIndex): the caller rearranges.
 *   table->assigned: device bitmap, one bit per K_INDEX entry of the mapped table, LSB
 *     first in 32-bit words: entry KIArrayPos of key_index_area[KIPtrArrayPos] at bit
 *     KIPtrArrayPos ? 2^(KIPtrArrayPos-1) + KIArrayPos : 0  (cur_mask + 1 bits).  NULL:
 *     every entry assigned (= the stateless forms above).
 *   kindex[i]: the entry reached, packed as above; when no probed entry is assigned, the
 *     last probe's (mask 1), as the reference's loop leaves it; K2H_AMD_KINDEX_NONE when
 *     cur_mask is 0 (the reference returns NULL).
 *   found[i] (may be NULL): 1 when an assigned entry was reached, else 0. */
#define K2H_AMD_KINDEX_NONE (~0ull)
typedef struct k2h_amd_table {
  uint64_t cur_mask;         /* K2HSHM cur_mask */
  uint64_t collision_mask;   /* K2HSHM collision_mask */
  const uint32_t* assigned;  /* device bitmap of assigned K_INDEX entries, or NULL */
} k2h_amd_table;

int k2h_amd_bucket_index_table(const uint64_t* h1, uint64_t n, const k2h_amd_table* table, uint64_t* kindex,
                               uint64_t* ckindex, uint8_t* found, void* stream);
int k2h_amd_hash_fixed_index_table(const void* keys, uint64_t key_len, uint64_t n, uint64_t* h1, uint64_t* h2,
                                   uint32_t flags, const k2h_amd_table* table, uint64_t* kindex, uint64_t* ckindex,
                                   uint8_t* found, void* stream);
int k2h_amd_hash_csr_index_table(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1,
                                 uint64_t* h2, uint32_t flags, const k2h_amd_table* table, uint64_t* kindex,
                                 uint64_t* ckindex, uint8_t* found, void* stream);

/* ---------------------------------------------------------------------------
 * 4. RALLEDATA producer (bulk direct-set input with precomputed hashes).
 *
 * k2h_set_element_by_binary (lib/k2hash.cc:1562-1581) -> K2HShm::SetElementByBinArray
 * (lib/k2hshmdirect.cc:343-478) inserts an element from a packed RALLEDATA blob
 * (lib/k2hshmdirect.h:36-47) and TRUSTS its hash / subhash fields: a bulk loader that
 * builds blobs here never runs the scalar hash per key.  Blob i (layout of
 * K2HShm::GetElementToBinary, lib/k2hshmdirect.cc:59-88):
 *   u64 hash = k2h_hash(key), subhash = k2h_second_hash(key),
 *   u64 key_length, val_length, skey_length, attrs_length,
 *   u64 key_pos = 80, val_pos, skey_pos, attrs_pos   (offsets from the blob top)
 *   then key | value | subkeys | attrs bytes.
 * Records are four CSR streams (bytes + n+1 offsets, offsets relative to the bytes
 * pointer); a NULL offsets array means that segment is empty for every record.  Blobs
 * are packed back to back in `out` (k2h_amd_ralledata_size bytes): blob i starts at
 * 80*i + the bytes of all earlier records, written to blob_off[i] (n+1 entries,
 * optional).  A K2HBIN for blob i is {out + blob_off[i], blob_off[i+1] - blob_off[i]}.
 * ------------------------------------------------------------------------- */
#define K2H_AMD_RALLEDATA_HEADER 80 /* sizeof(RALLEDATA), packed */

uint64_t k2h_amd_ralledata_size(uint64_t n, uint64_t key_bytes, uint64_t val_bytes, uint64_t skey_bytes,
                                uint64_t attr_bytes);
int k2h_amd_build_ralledata(const void* keys, const uint64_t* key_off, const void* vals, const uint64_t* val_off,
                            const void* skeys, const uint64_t* skey_off, const void* attrs, const uint64_t* attr_off,
                            uint64_t n, void* out, uint64_t* blob_off, uint32_t flags, void* stream);
int k2h_amd_build_ralledata_host(const void* keys, const uint64_t* key_off, const void* vals,
                                 const uint64_t* val_off, const void* skeys, const uint64_t* skey_off,
                                 const void* attrs, const uint64_t* attr_off, uint64_t n, void* out,
                                 uint64_t* blob_off, uint32_t flags, int device);

/* ---------------------------------------------------------------------------
 * 5. Bulk key streams: keys anywhere in a buffer, and k2hash archives.
 *
 * k2h_amd_hash_ranges hashes key i = base[starts[i], starts[i] + lens[i]) (device
 * pointers).  With K2H_AMD_FLAG_CSTR each key is hashed as the C string that
 * K2HShm::Set(const char*, ...) stores (lib/k2hshm.cc:2081-2083): the range plus a
 * terminating NUL (strlen + 1 bytes) -- the form k2himport's TSV / mdbm loaders use
 * (tests/k2himport.cc:81-112).  The call synchronises `stream` once (to size the
 * staging buffer the keys are packed into).
 *
 * k2h_amd_archive_scan walks a k2hash archive (K2HArchive::Save / Load,
 * lib/k2harchive.cc:82-383; record = packed 104-byte SCOM header + data,
 * lib/k2hcommand.h:64-79) as Load does and reports each record; recs may be NULL to
 * count only.  k2h_amd_archive_prehash_host then hashes every record's key on the GPU
 * (and, if new_h1/new_h2 are given, the new key of each SCOM_RENAME record), so a
 * loader can have all hashes before applying record one.  Host pointers.
 * ------------------------------------------------------------------------- */
#define K2H_AMD_FLAG_CSTR 0x2u /* hash each key as key + NUL (K2HShm::Set(const char*)) */

int k2h_amd_hash_ranges(const void* base, const uint64_t* starts, const uint64_t* lens, uint64_t n, uint64_t* h1,
                        uint64_t* h2, uint32_t flags, void* stream);

#define K2H_AMD_ARCHIVE_BAD_TYPE 1  /* type outside SCOM_TYPE_MIN..MAX (Load: skip / fail) */
#define K2H_AMD_ARCHIVE_TRUNCATED 2 /* a data segment runs past the end of the file */
typedef struct k2h_amd_archive_rec {
  int64_t type;    /* SCOM_SET_ALL .. SCOM_RENAME (lib/k2hcommand.h:47-55) */
  uint64_t offset; /* record start in the file */
  uint64_t key_off, key_len, val_off, val_len, skey_off, skey_len, attrs_off, attrs_len, exdata_off, exdata_len;
  /* absolute offsets in the file */
  int32_t status;  /* 0, K2H_AMD_ARCHIVE_BAD_TYPE or K2H_AMD_ARCHIVE_TRUNCATED */
  int32_t reserved;
} k2h_amd_archive_rec;

int k2h_amd_archive_scan(const void* file, uint64_t size, k2h_amd_archive_rec* recs, uint64_t cap,
                         uint64_t* count);
int k2h_amd_archive_prehash_host(const void* file, uint64_t size, const k2h_amd_archive_rec* recs, uint64_t count,
                                 uint64_t* h1, uint64_t* h2, uint64_t* new_h1, uint64_t* new_h2, uint32_t flags,
                                 int device);

/* k2himport inputs (tests/k2himport.cc:74-117): k2h_amd_import_scan splits a TSV
 * (key TAB value NEWLINE) or mdbm_export file (five header lines ending "HEADER=END",
 * then key line / value line) into records exactly as the tool's std::getline loops
 * do, and reports each key and value as the C string K2HShm::Set(const char*, const
 * char*) stores (lib/k2hshm.cc:2081-2083): *_len = strlen, i.e. cut at a NUL byte.
 * recs may be NULL to count only; a bad mdbm header returns K2H_AMD_EINVAL (the tool
 * exits).  Faithful to getline: an mdbm key line ending at EOF reports the previous
 * record's value range (the string a failed getline leaves untouched).  k2h_amd_import_prehash_host hashes every key as key + NUL on the GPU (the
 * bytes Set hashes).  Host pointers. */
#define K2H_AMD_IMPORT_TSV 0
#define K2H_AMD_IMPORT_MDBM 1
typedef struct k2h_amd_import_rec {
  uint64_t key_off, key_len; /* absolute offset in the file, strlen of the key */
  uint64_t val_off, val_len; /* likewise for the value */
} k2h_amd_import_rec;

int k2h_amd_import_scan(const void* file, uint64_t size, int format, k2h_amd_import_rec* recs, uint64_t cap,
                        uint64_t* count);
int k2h_amd_import_prehash_host(const void* file, uint64_t size, const k2h_amd_import_rec* recs, uint64_t count,
                                uint64_t* h1, uint64_t* h2, uint32_t flags, int device);

/* The same scan for a file already in device memory (file, recs: device pointers;
 * count: host), with no host pass: record ends are the newlines of the lines that hold
 * a TAB (TSV) or every second line after the header (mdbm), found by parallel passes
 * (k2hash_amd/csrc/k2h_import_dev.hip).  Same records, same errors as
 * k2h_amd_import_scan; synchronises `stream`.  k2h_amd_import_prehash hashes every
 * record's key as key + NUL straight from the device-resident file, one lane per
 * record (async on `stream`); a record whose key range is not inside [0, size) gets
 * h1 = h2 = 0 and nothing outside the file is read. */
int k2h_amd_import_scan_device(const void* file, uint64_t size, int format, k2h_amd_import_rec* recs, uint64_t cap,
                               uint64_t* count, void* stream);
int k2h_amd_import_prehash(const void* file, uint64_t size, const k2h_amd_import_rec* recs, uint64_t n, uint64_t* h1,
                           uint64_t* h2, uint32_t flags, void* stream);
/* Both in one call: the records and, from the same kernel, h1 / h2 (h2 may be NULL) of
 * every record's key + NUL -- the prehash without a second pass over the records.  h1
 * and h2 need room for cap entries; count / cap / errors as k2h_amd_import_scan_device. */
int k2h_amd_import_scan_prehash_device(const void* file, uint64_t size, int format, k2h_amd_import_rec* recs,
                                       uint64_t cap, uint64_t* count, uint64_t* h1, uint64_t* h2, uint32_t flags,
                                       void* stream);

/* Identity / diagnostics. */
const char* k2h_amd_version(void);     /* library + kernel identity, e.g. "k2hash_amd 0.1 gfx950" */
const char* k2h_amd_strerror(int code); /* message for `code`, with the last HIP error if any */

/* Synthetic-workload generator used by bench.py and the tests (not the hash
 * path): writes bytes [byte_off, byte_off+nbytes) of the splitmix64 word stream
 * with `seed`, and CSR lengths min_len + mix(seed, first_key+i) % (max_len-min_len+1).
 * Same spec as oracle/fnv_oracle.c. */
int k2h_amd_synth_bytes(void* out, uint64_t nbytes, uint64_t seed, uint64_t byte_off, void* stream);
int k2h_amd_synth_lengths(uint32_t* lens, uint64_t n, uint64_t seed, uint64_t first_key, uint32_t min_len,
                          uint32_t max_len, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* K2HASH_AMD_H */
