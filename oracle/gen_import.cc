// ORACLE -- TEST INFRASTRUCTURE ONLY (never linked into or called by the product).
//
// Fixture generator for the k2himport prehash.  Runs the two
// parse loops of the reference tool tests/k2himport.cc over std::getline -- the
// libstdc++ behaviour those loops are built on -- restated here:
//   TSV  (tests/k2himport.cc:74-89):  while (getline(is, key, '\t')) { if (is.eof()) break;
//                                     getline(is, value); Set(key.c_str(), value.c_str()); }
//   mdbm (tests/k2himport.cc:95-117): five header lines, the fifth must be "HEADER=END";
//                                     then while (getline(is, key)) { getline(is, value); Set(...); }
// and hashes every key the way K2HShm::Set(const char*, const char*) passes it on
// (lib/k2hshm.cc:2081-2083: the C string, strlen + 1 bytes) with the REFERENCE's own
// k2h_hash / k2h_second_hash (lib/k2hashfunc.cc:62-91), linked from
// oracle/_ref/libk2hfunc_ref.so.  Prints one JSON object: the records (stream offsets
// before each getline, C-string key / value bytes in hex, the two hashes) or an error.
//
//   gen_import tsv|mdbm <file>
//   gen_import tsv-digest|mdbm-digest <file>
//                                  the loop's records and hashes as order-sensitive digests
//                                  {xor, sum, sum of v * (2i + 1)} per field (the bench's
//                                  8M-record workloads, tests/golden/make_import_digest.py)
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <fstream>
#include <string>

extern "C" uint64_t k2h_hash(const void* ptr, size_t length);
extern "C" uint64_t k2h_second_hash(const void* ptr, size_t length);

static void hex(const char* p, size_t n) {
  for (size_t i = 0; i < n; ++i) printf("%02x", (unsigned)(unsigned char)p[i]);
}

struct Digest {  // oracle_digest (oracle/fnv_oracle.c), accumulated one value at a time
  uint64_t x = 0, s = 0, w = 0;
  void add(uint64_t v, uint64_t i) {
    x ^= v;
    s += v;
    w += v * (2 * i + 1);
  }
  void print(const char* name) const {
    printf("\"%s\": [\"%016llx\", \"%016llx\", \"%016llx\"]", name, (unsigned long long)x, (unsigned long long)s,
           (unsigned long long)w);
  }
};

// The loops of tests/k2himport.cc:81-86 (TSV) and :104-113 (mdbm, after the header check of
// :95-103) with every record folded into digests instead of printed.
static int loop_digest(std::ifstream& is, bool tsv) {
  Digest d[6];
  uint64_t n = 0;
  std::string key, value;
  if (!tsv) {
    std::string hdr[5];
    for (int i = 0; i < 5; ++i) std::getline(is, hdr[i]);
    if (hdr[4] != "HEADER=END") {
      printf("{\"format\": \"mdbm\", \"error\": true}\n");
      return 0;
    }
  }
  for (;;) {
    long long koff = (long long)is.tellg();
    if (tsv) {
      if (!std::getline(is, key, '\t')) break;
      if (is.eof()) break;
    } else if (!std::getline(is, key)) {
      break;
    }
    long long voff = (long long)is.tellg();
    std::getline(is, value);
    const char* kc = key.c_str();
    const size_t kl = strlen(kc), vl = strlen(value.c_str());
    d[0].add((uint64_t)koff, n);
    d[1].add(kl, n);
    d[2].add((uint64_t)voff, n);
    d[3].add(vl, n);
    d[4].add(k2h_hash(kc, kl + 1), n);
    d[5].add(k2h_second_hash(kc, kl + 1), n);
    ++n;
  }
  static const char* names[6] = {"key_off", "key_len", "val_off", "val_len", "h1", "h2"};
  printf("{\"format\": \"%s\", \"records\": %llu", tsv ? "tsv" : "mdbm", (unsigned long long)n);
  for (int k = 0; k < 6; ++k) {
    printf(", ");
    d[k].print(names[k]);
  }
  printf("}\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: gen_import tsv|mdbm|tsv-digest|mdbm-digest <file>\n");
    return 2;
  }
  if (strcmp(argv[1], "tsv-digest") == 0 || strcmp(argv[1], "mdbm-digest") == 0) {
    std::ifstream is(argv[2], std::ios::binary);
    if (!is) {
      fprintf(stderr, "cannot open %s\n", argv[2]);
      return 2;
    }
    return loop_digest(is, argv[1][0] == 't');
  }
  const bool tsv = strcmp(argv[1], "tsv") == 0;
  std::ifstream is(argv[2], std::ios::binary);
  if (!is) {
    fprintf(stderr, "cannot open %s\n", argv[2]);
    return 2;
  }
  bool first = true;
  auto emit = [&](long long koff, long long voff, const std::string& k, const std::string& v) {
    const char* kc = k.c_str();
    const char* vc = v.c_str();
    const size_t kl = strlen(kc), vl = strlen(vc);
    printf("%s\n  {\"key_off\": %lld, \"val_off\": %lld, \"key\": \"", first ? "" : ",", koff, voff);
    hex(kc, kl);
    printf("\", \"val\": \"");
    hex(vc, vl);
    printf("\", \"h1\": \"%016llx\", \"h2\": \"%016llx\"}", (unsigned long long)k2h_hash(kc, kl + 1),
           (unsigned long long)k2h_second_hash(kc, kl + 1));
    first = false;
  };
  std::string key, value;
  printf("{\"format\": \"%s\", ", argv[1]);
  if (tsv) {
    printf("\"error\": false, \"records\": [");
    for (;;) {
      long long koff = (long long)is.tellg();
      if (!std::getline(is, key, '\t')) break;
      if (is.eof()) break;
      long long voff = (long long)is.tellg();
      std::getline(is, value);
      emit(koff, voff, key, value);
    }
  } else {
    std::string hdr[5];
    for (int i = 0; i < 5; ++i) std::getline(is, hdr[i]);
    if (hdr[4] != "HEADER=END") {
      printf("\"error\": true, \"records\": []}\n");
      return 0;
    }
    printf("\"error\": false, \"records\": [");
    for (;;) {
      long long koff = (long long)is.tellg();
      if (!std::getline(is, key)) break;
      long long voff = (long long)is.tellg();
      std::getline(is, value);
      emit(koff, voff, key, value);
    }
  }
  printf("\n]}\n");
  return 0;
}
