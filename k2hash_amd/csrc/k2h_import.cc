// k2hash_amd -- k2himport input scanner for the bulk-key-stream prehash (SURVEY.md 8f
// rank 3).  Pure C++ (no HIP): splits a TSV or mdbm_export file into records exactly as
// tests/k2himport.cc does with std::getline, and reports each record's key and value
// as the C strings K2HShm::Set(const char*, const char*) stores (lib/k2hshm.cc:2081-2083:
// strlen + 1 bytes), so that every key of the file can be hashed in one GPU batch before
// the records are applied.
//
// TSV (ConvertfromTsv, tests/k2himport.cc:74-89):
//   while (getline(ifs, key, '\t')) { if (ifs.eof()) break; getline(ifs, value); Set(...); }
//   - a key runs to the next TAB, across newlines; if no TAB follows, the trailing text
//     is dropped (eof inside the key getline);
//   - a value runs to the next '\n' or the end of the file; an empty value at the end of
//     the file still makes a record (getline fails, Set runs anyway), then the loop stops.
// mdbm (ConvertfromMdbm, tests/k2himport.cc:95-117): five header lines, the fifth must
// be exactly "HEADER=END" (else the tool exits with "not a mdbm file"), then key line /
// value line pairs; a last key line ending in a newline gets an empty value, one ending
// at EOF the previous record's value (getline does not clear its string when it fails
// on a stream already at EOF).
// The C-string view: a key or value holding a NUL byte is cut at its first NUL
// (c_str() + strlen), so `key_len` / `val_len` below are strlen(c_str()).
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/k2hash_amd.h"

namespace {

// std::getline(is, s, delim) over f[p, size): the extracted text [p, e), the new
// position, and whether the call fails (nothing extracted and no delimiter: EOF).
struct Line {
  uint64_t b, e;
  bool found;  // delimiter found (and consumed)
  bool fail;   // failbit: no character extracted
};

Line getline(const uint8_t* f, uint64_t size, uint64_t& p, uint8_t delim) {
  Line l{p, p, false, false};
  if (p >= size) {
    l.fail = true;
    return l;
  }
  const void* d = memchr(f + p, delim, size - p);
  if (d) {
    l.e = (uint64_t)((const uint8_t*)d - f);
    l.found = true;
    p = l.e + 1;
  } else {
    l.e = size;
    p = size;
  }
  return l;
}

uint64_t cstr_len(const uint8_t* f, uint64_t b, uint64_t e) {
  const void* z = memchr(f + b, 0, e - b);
  return z ? (uint64_t)((const uint8_t*)z - (f + b)) : e - b;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) int k2h_amd_import_scan(const void* file, uint64_t size, int format,
                                                               k2h_amd_import_rec* recs, uint64_t cap,
                                                               uint64_t* count) {
  if (!count || (size && !file) || (format != K2H_AMD_IMPORT_TSV && format != K2H_AMD_IMPORT_MDBM))
    return K2H_AMD_EINVAL;
  const uint8_t* f = (const uint8_t*)file;
  uint64_t n = 0, p = 0;
  auto emit = [&](const Line& k, uint64_t voff, uint64_t vlen) {
    if (recs && n < cap) {
      recs[n].key_off = k.b;
      recs[n].key_len = cstr_len(f, k.b, k.e);
      recs[n].val_off = voff;
      recs[n].val_len = vlen;
    }
    ++n;
  };
  if (format == K2H_AMD_IMPORT_TSV) {
    for (;;) {
      Line k = getline(f, size, p, '\t');
      if (k.fail) break;   // while (getline(...)) fails
      if (!k.found) break; // if (ifs->eof()) break;
      Line v = getline(f, size, p, '\n');  // the stream is good here, so the string is cleared
      emit(k, v.b, v.fail ? 0 : cstr_len(f, v.b, v.e));
      if (v.fail) break;   // the stream is in fail state: the next while test fails
    }
  } else {
    Line h[5];
    bool failed = false;
    for (int i = 0; i < 5; ++i) {
      h[i] = failed ? Line{p, p, false, true} : getline(f, size, p, '\n');
      failed = failed || h[i].fail;
    }
    static const char kEnd[] = "HEADER=END";
    if (h[4].fail || h[4].e - h[4].b != sizeof kEnd - 1 || memcmp(f + h[4].b, kEnd, sizeof kEnd - 1) != 0) {
      *count = 0;
      return K2H_AMD_EINVAL;  // k2himport: "error: not a mdbm file."
    }
    // std::getline leaves its string untouched when its sentry fails: a key line that
    // ends at EOF sets eofbit, so the value read after it fails and Set gets the
    // PREVIOUS record's value (the empty string before the first record)
    uint64_t pv_off = p, pv_len = 0;
    for (;;) {
      Line k = getline(f, size, p, '\n');
      if (k.fail) break;
      if (!k.found) {
        emit(k, pv_off, pv_len);
        break;
      }
      Line v = getline(f, size, p, '\n');
      pv_off = v.b;
      pv_len = v.fail ? 0 : cstr_len(f, v.b, v.e);
      emit(k, pv_off, pv_len);
      if (v.fail) break;
    }
  }
  *count = n;
  return (recs && n > cap) ? K2H_AMD_EINVAL : K2H_AMD_OK;
}

// Hash every record's key as the C string Set stores (key bytes + NUL) on the GPU, one
// CSR batch through the pinned pipeline of k2h_amd_hash_csr_host.
__attribute__((visibility("default"))) int k2h_amd_import_prehash_host(const void* file, uint64_t size,
                                                                       const k2h_amd_import_rec* recs, uint64_t count,
                                                                       uint64_t* h1, uint64_t* h2, uint32_t flags,
                                                                       int device) {
  if (count == 0) return K2H_AMD_OK;
  if (!recs || !h1 || (size && !file)) return K2H_AMD_EINVAL;
  const uint8_t* f = (const uint8_t*)file;
  uint64_t bytes = 0;
  for (uint64_t i = 0; i < count; ++i) {
    if (recs[i].key_off > size || recs[i].key_len > size - recs[i].key_off) return K2H_AMD_EINVAL;
    bytes += recs[i].key_len + 1;
  }
  std::vector<uint8_t> keys(bytes);
  std::vector<uint64_t> off(count + 1, 0);
  uint64_t p = 0;
  for (uint64_t i = 0; i < count; ++i) {
    if (recs[i].key_len) memcpy(keys.data() + p, f + recs[i].key_off, recs[i].key_len);
    p += recs[i].key_len;
    keys[p++] = 0;  // the terminating NUL is part of the stored key
    off[i + 1] = p;
  }
  return k2h_amd_hash_csr_host(keys.data(), off.data(), count, h1, h2, flags & ~K2H_AMD_FLAG_CSTR, device);
}

}  // extern "C"
