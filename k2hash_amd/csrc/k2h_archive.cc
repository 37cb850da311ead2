// k2hash_amd -- k2hash archive reader for the bulk-key-stream prehash (SURVEY.md 8f
// rank 3).  Pure C++ (no HIP): walks an archive the way K2HArchive::Load does
// (lib/k2harchive.cc:279-383) and reports every record's segments, so that all keys
// can be hashed in one GPU batch before the records are applied.
//
// Record format (lib/k2hcommand.h:64-79, packed): char szCommand[16]; long type;
// size_t key/val/skey/attr/exdata lengths; off_t key/val/skey/attrs/exdata positions
// (relative to the record start) = 104 bytes, then the data.  The next record starts
// scom_total_length() = 104 + the five lengths later (lib/k2hcommand.h:108-111), whatever
// the positions say.  Load stops at the first offset where a whole header cannot be read
// (ReadFile returns NULL on a short read, lib/k2harchive.cc:385-405); a record with an
// unknown type or a segment that cannot be read fully is skipped (isErrSkip) or ends the
// load -- reported here per record in `status` so the caller can apply either policy.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/k2hash_amd.h"

namespace {

constexpr uint64_t kScomSize = 104;  // sizeof(SCOM), packed

uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);  // little endian (x86-64 / the archive writer's host)
  return v;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) int k2h_amd_archive_scan(const void* file, uint64_t size,
                                                                k2h_amd_archive_rec* recs, uint64_t cap,
                                                                uint64_t* count) {
  if (!count || (size && !file)) return K2H_AMD_EINVAL;
  const uint8_t* f = (const uint8_t*)file;
  uint64_t n = 0;
  for (uint64_t off = 0; size >= kScomSize && off <= size - kScomSize;) {
    const uint8_t* h = f + off;
    k2h_amd_archive_rec r;
    r.type = (int64_t)rd64(h + 16);
    uint64_t len[5], pos[5];
    for (int j = 0; j < 5; ++j) len[j] = rd64(h + 24 + 8 * j);
    for (int j = 0; j < 5; ++j) pos[j] = rd64(h + 64 + 8 * j);
    r.offset = off;
    r.status = (r.type < 0 || r.type > 6) ? K2H_AMD_ARCHIVE_BAD_TYPE : 0;  // SCOM_TYPE_MIN..MAX, lib/k2hcommand.h:47-55
    uint64_t* o[5] = {&r.key_off, &r.val_off, &r.skey_off, &r.attrs_off, &r.exdata_off};
    uint64_t* l[5] = {&r.key_len, &r.val_len, &r.skey_len, &r.attrs_len, &r.exdata_len};
    uint64_t total = kScomSize;
    bool overflow = false;
    for (int j = 0; j < 5; ++j) {
      *l[j] = len[j];
      *o[j] = off + pos[j];
      if (len[j] > size || pos[j] > size || off + pos[j] + len[j] > size) {
        if (len[j] && !r.status) r.status = K2H_AMD_ARCHIVE_TRUNCATED;
      }
      if (total + len[j] < total) overflow = true;
      total += len[j];
    }
    if (recs && n < cap) recs[n] = r;
    ++n;
    if (overflow || total > size - off) break;  // the next header would start beyond the file
    off += total;
  }
  *count = n;
  return (recs && n > cap) ? K2H_AMD_EINVAL : K2H_AMD_OK;
}

// Hash every record's key (and, for SCOM_RENAME, the new key held in exdata) on the GPU:
// keys are gathered into one CSR batch on the host and sent through the pinned
// pipeline of k2h_amd_hash_csr_host.  Records whose status is non-zero hash to 0.
__attribute__((visibility("default"))) int k2h_amd_archive_prehash_host(const void* file, uint64_t size,
                                                                        const k2h_amd_archive_rec* recs,
                                                                        uint64_t count, uint64_t* h1, uint64_t* h2,
                                                                        uint64_t* new_h1, uint64_t* new_h2,
                                                                        uint32_t flags, int device) {
  if (count == 0) return K2H_AMD_OK;
  if (!recs || !h1 || (size && !file)) return K2H_AMD_EINVAL;
  const uint8_t* f = (const uint8_t*)file;
  const bool rename = new_h1 || new_h2;
  std::vector<uint64_t> off(count * (rename ? 2 : 1) + 1, 0);
  uint64_t bytes = 0;
  for (uint64_t i = 0; i < count; ++i) {
    if (!recs[i].status) bytes += recs[i].key_len;
    if (rename && !recs[i].status && recs[i].type == 6) bytes += recs[i].exdata_len;
  }
  std::vector<uint8_t> keys(bytes ? bytes : 1);
  uint64_t p = 0, m = 0;
  auto put = [&](uint64_t o, uint64_t l) {
    if (l) memcpy(keys.data() + p, f + o, l);
    p += l;
    off[++m] = p;
  };
  for (uint64_t i = 0; i < count; ++i) put(recs[i].key_off, recs[i].status ? 0 : recs[i].key_len);
  if (rename)
    for (uint64_t i = 0; i < count; ++i)
      put(recs[i].exdata_off, (!recs[i].status && recs[i].type == 6) ? recs[i].exdata_len : 0);
  std::vector<uint64_t> a(m), b(m);
  int rc = k2h_amd_hash_csr_host(keys.data(), off.data(), m, a.data(), b.data(), flags, device);
  if (rc) return rc;
  memcpy(h1, a.data(), count * 8);
  if (h2) memcpy(h2, b.data(), count * 8);
  if (new_h1) memcpy(new_h1, a.data() + count, count * 8);
  if (new_h2) memcpy(new_h2, b.data() + count, count * 8);
  return K2H_AMD_OK;
}

}  // extern "C"
