/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Golden fixture for the RALLEDATA producer, built against the
 * REFERENCE's own headers where they lie under /root/reference (never copied):
 *   lib/k2hash.h        k2h_hash_t, K2HBIN
 *   lib/k2hshmdirect.h  RALLEDATA / BALLEDATA (packed, lines 36-56), ralledata_init
 *                       (63-75), calc_ralledata_length (85-88)
 * and the reference's hash functions from oracle/_ref/libk2hfunc_ref.so (dlsym, as
 * K2HashDynLib::Load does).  Each record's blob is laid out the way
 * K2HShm::GetElementToBinary does it (lib/k2hshmdirect.cc:59-88), with hash/subhash
 * = K2H_HASH_FUNC / K2H_2ND_HASH_FUNC of the key (as K2HShm::Set stores them,
 * lib/k2hshm.cc:2184-2185), so the struct layout, field order and packing come from
 * the reference build itself.
 *
 * usage: gen_ralledata <ref.so> <out.json>
 */
#include <dlfcn.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "k2hash.h"
#include "k2hshmdirect.h"

extern "C" void oracle_gen_bytes(uint64_t seed, uint64_t byte_off, size_t nbytes, uint8_t* out);
extern "C" uint64_t oracle_splitmix_word(uint64_t seed, uint64_t j);

typedef uint64_t (*hash_fn)(const void*, size_t);

static std::string hex(const unsigned char* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += d[p[i] >> 4];
    s += d[p[i] & 15];
  }
  return s;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <ref.so> <out.json>\n", argv[0]);
    return 2;
  }
  void* so = dlopen(argv[1], RTLD_LAZY);
  if (!so) return 2;
  hash_fn h1 = (hash_fn)dlsym(so, "k2h_hash"), h2 = (hash_fn)dlsym(so, "k2h_second_hash");
  if (!h1 || !h2) return 2;
  const uint64_t seed = 0x6B32686173680004ULL;
  FILE* f = fopen(argv[2], "w");
  fprintf(f, "{\n \"generator\": \"oracle/gen_ralledata.cc (reference lib/k2hshmdirect.h layout, lib/k2hashfunc.cc hashes)\",\n");
  fprintf(f, " \"sizeof_RALLEDATA\": %zu,\n \"offsets\": {\"hash\": %zu, \"subhash\": %zu, \"key_length\": %zu, "
             "\"val_length\": %zu, \"skey_length\": %zu, \"attrs_length\": %zu, \"key_pos\": %zu, \"val_pos\": %zu, "
             "\"skey_pos\": %zu, \"attrs_pos\": %zu},\n \"records\": [\n",
          sizeof(RALLEDATA), offsetof(RALLEDATA, hash), offsetof(RALLEDATA, subhash), offsetof(RALLEDATA, key_length),
          offsetof(RALLEDATA, val_length), offsetof(RALLEDATA, skey_length), offsetof(RALLEDATA, attrs_length),
          offsetof(RALLEDATA, key_pos), offsetof(RALLEDATA, val_pos), offsetof(RALLEDATA, skey_pos),
          offsetof(RALLEDATA, attrs_pos));
  const int N = 48;
  uint64_t byte_off = 0;
  for (int i = 0; i < N; ++i) {
    uint64_t r = oracle_splitmix_word(seed, (uint64_t)i);
    size_t kl = 1 + r % 40, vl = (r >> 8) % 5 == 0 ? 0 : (r >> 12) % 300, sl = (r >> 24) % 4 == 0 ? (r >> 28) % 50 : 0,
           al = (r >> 36) % 3 == 0 ? (r >> 40) % 60 : 0;
    if (i == 0) kl = 5, vl = 7, sl = 0, al = 0;  // "key1\0"-like small record
    if (i == 1) vl = 1500;                        // a long value
    if (i == 2) vl = sl = al = 0;                 // key only
    std::vector<unsigned char> k(kl), v(vl), s(sl), a(al);
    oracle_gen_bytes(seed, byte_off, kl, k.data());
    byte_off += kl;
    if (vl) oracle_gen_bytes(seed, byte_off, vl, v.data());
    byte_off += vl;
    if (sl) oracle_gen_bytes(seed, byte_off, sl, s.data());
    byte_off += sl;
    if (al) oracle_gen_bytes(seed, byte_off, al, a.data());
    byte_off += al;
    if (i == 0) memcpy(k.data(), "key1", 5);
    // GetElementToBinary's layout (lib/k2hshmdirect.cc:59-88) on the reference's struct
    size_t total = sizeof(RALLEDATA) + kl + vl + sl + al;
    PBALLEDATA bin = (PBALLEDATA)malloc(total);
    ralledata_init(bin->rawdata);
    bin->rawdata.hash = h1(k.data(), kl);
    bin->rawdata.subhash = h2(k.data(), kl);
    bin->rawdata.key_length = kl;
    bin->rawdata.val_length = vl;
    bin->rawdata.skey_length = sl;
    bin->rawdata.attrs_length = al;
    bin->rawdata.key_pos = (off_t)sizeof(RALLEDATA);
    bin->rawdata.val_pos = bin->rawdata.key_pos + (off_t)bin->rawdata.key_length;
    bin->rawdata.skey_pos = bin->rawdata.val_pos + (off_t)bin->rawdata.val_length;
    bin->rawdata.attrs_pos = bin->rawdata.skey_pos + (off_t)bin->rawdata.skey_length;
    unsigned char* top = reinterpret_cast<unsigned char*>(&bin->rawdata);
    if (kl) memcpy(top + bin->rawdata.key_pos, k.data(), kl);
    if (vl) memcpy(top + bin->rawdata.val_pos, v.data(), vl);
    if (sl) memcpy(top + bin->rawdata.skey_pos, s.data(), sl);
    if (al) memcpy(top + bin->rawdata.attrs_pos, a.data(), al);
    if (calc_ralledata_length(bin->rawdata) != total) return 3;
    fprintf(f, "  {\"key\": \"%s\", \"val\": \"%s\", \"skey\": \"%s\", \"attrs\": \"%s\", \"blob\": \"%s\"}%s\n",
            hex(k.data(), kl).c_str(), hex(v.data(), vl).c_str(), hex(s.data(), sl).c_str(), hex(a.data(), al).c_str(),
            hex(top, total).c_str(), i + 1 < N ? "," : "");
    free(bin);
  }
  fprintf(f, " ]\n}\n");
  fclose(f);
  return 0;
}
