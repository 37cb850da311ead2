/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Golden archive fixture for the bulk-key-stream prehash.  The
 * records are written by the REFERENCE's own K2HCommandArchive (lib/k2hcommand.cc,
 * compiled from /root/reference by oracle/Makefile, never copied) exactly as
 * K2HArchive::Save appends them (lib/k2harchive.cc:166-185: Get() then
 * scom_total_length(pBinCom->scom) bytes), and every key is hashed by the reference's
 * lib/k2hashfunc.cc build (dlsym, as K2HashDynLib::Load does).
 *
 * Writes <out>.k2har (the archive bytes) and <out>.json (per record: type, record
 * offset, key hex, h1, h2, lengths of the five data segments).
 *
 * usage: gen_archive <ref.so> <out-prefix>
 */
#include <dlfcn.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "k2hcommand.h"

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
  if (argc < 3) return 2;
  void* so = dlopen(argv[1], RTLD_LAZY);
  if (!so) return 2;
  hash_fn h1 = (hash_fn)dlsym(so, "k2h_hash"), h2 = (hash_fn)dlsym(so, "k2h_second_hash");
  if (!h1 || !h2) return 2;
  std::string pre = argv[2];
  FILE* ar = fopen((pre + ".k2har").c_str(), "wb");
  FILE* js = fopen((pre + ".json").c_str(), "w");
  if (!ar || !js) return 2;
  fprintf(js, "{\n \"generator\": \"oracle/gen_archive.cc (reference lib/k2hcommand.cc K2HCommandArchive, lib/k2hashfunc.cc)\",\n"
              " \"sizeof_SCOM\": %zu,\n \"records\": [\n", sizeof(SCOM));
  const uint64_t seed = 0x6B32686173680005ULL;
  uint64_t off = 0, boff = 0;
  const int N = 64;
  for (int i = 0; i < N; ++i) {
    uint64_t r = oracle_splitmix_word(seed, (uint64_t)i);
    size_t kl = 1 + r % 48, vl = (r >> 8) % 200, sl = (r >> 16) % 3 ? 0 : (r >> 20) % 40, al = (r >> 28) % 3 ? 0 : (r >> 32) % 30,
           xl = 1 + (r >> 40) % 24;
    std::vector<unsigned char> k(kl), v(vl + 1), s(sl + 1), a(al + 1), x(xl);
    oracle_gen_bytes(seed, boff, kl, k.data());
    boff += kl;
    oracle_gen_bytes(seed, boff, vl, v.data());
    boff += vl;
    oracle_gen_bytes(seed, boff, sl, s.data());
    boff += sl;
    oracle_gen_bytes(seed, boff, al, a.data());
    boff += al;
    oracle_gen_bytes(seed, boff, xl, x.data());
    boff += xl;
    if (i == 0) {  // a c-string key as k2hlinetool / K2HShm::Set(const char*) store it
      kl = 5;
      memcpy(k.data(), "key1", 5);
    }
    K2HCommandArchive com;
    long type = (long)(i % 7);  // SCOM_SET_ALL .. SCOM_RENAME in turn (lib/k2hcommand.h:47-55)
    bool ok = false;
    off_t valoffset = (off_t)((r >> 48) % 4096);
    switch (type) {
      case SCOM_SET_ALL: ok = com.SetAll(k.data(), kl, v.data(), vl, s.data(), sl, a.data(), al); break;
      case SCOM_REPLACE_VAL: ok = com.ReplaceVal(k.data(), kl, v.data(), vl); break;
      case SCOM_REPLACE_SKEY: ok = com.ReplaceSKey(k.data(), kl, s.data(), sl); break;
      case SCOM_DEL_KEY: ok = com.DelKey(k.data(), kl); break;
      case SCOM_OW_VAL: ok = com.OverWriteValue(k.data(), kl, v.data(), vl, valoffset); break;
      case SCOM_REPLACE_ATTRS: ok = com.ReplaceAttrs(k.data(), kl, a.data(), al); break;
      default: ok = com.Rename(k.data(), kl, x.data(), xl, a.data(), al); break;
    }
    if (!ok) return 3;
    const BCOM* b = com.Get();
    size_t len = scom_total_length(b->scom);
    if (fwrite(b->byData, 1, len, ar) != len) return 4;
    fprintf(js,
            "  {\"type\": %ld, \"offset\": %" PRIu64 ", \"key\": \"%s\", \"h1\": \"%016" PRIx64 "\", \"h2\": \"%016" PRIx64
            "\", \"val_length\": %zu, \"skey_length\": %zu, \"attr_length\": %zu, \"exdata_length\": %zu, "
            "\"exdata\": \"%s\", \"total\": %zu}%s\n",
            b->scom.type, off, hex(k.data(), kl).c_str(), h1(k.data(), kl), h2(k.data(), kl), b->scom.val_length,
            b->scom.skey_length, b->scom.attr_length, b->scom.exdata_length,
            hex(b->byData + b->scom.exdata_pos, b->scom.exdata_length).c_str(), len, i + 1 < N ? "," : "");
    off += len;
  }
  fprintf(js, " ],\n \"size\": %" PRIu64 "\n}\n", off);
  fclose(ar);
  fclose(js);
  return 0;
}
