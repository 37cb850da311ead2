// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// Drives the REFERENCE's own plugin loader against a candidate plugin: links the
// reference's K2HashDynLib (lib/k2hashfunc.cc:104-161, built into oracle/_ref) and
// uses its dispatch macros K2H_HASH_FUNC / K2H_2ND_HASH_FUNC / K2H_HASH_VER_FUNC
// (lib/k2hashfunc.h:90-93) exactly as tests/k2hexttest.cc:120-126,166-175 does.
//
// usage: dynlib_conformance <plugin.so> < keys.hex
//   prints "LOAD ok|fail", "VERSION <K2H_HASH_VER_FUNC()>", "BUILTIN <k2h_hash_version()>",
//   then one "h1 h2" line per input hex key (one key per line, "-" = empty key).
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "k2hashfunc.h"

static std::vector<unsigned char> unhex(const char* s) {
  std::vector<unsigned char> out;
  if (!strcmp(s, "-")) return out;
  for (size_t i = 0; s[i] && s[i + 1]; i += 2) {
    unsigned v;
    sscanf(s + i, "%2x", &v);
    out.push_back((unsigned char)v);
  }
  return out;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  bool ok = K2HashDynLib::get()->Load(argv[1]);
  printf("LOAD %s\n", ok ? "ok" : "fail");
  if (!ok) return 1;
  printf("VERSION %s\n", K2H_HASH_VER_FUNC());
  printf("BUILTIN %s\n", k2h_hash_version());
  static char line[1 << 16];
  while (fgets(line, sizeof line, stdin)) {
    line[strcspn(line, "\r\n")] = 0;
    std::vector<unsigned char> k = unhex(line);
    const unsigned char* p = k.empty() ? reinterpret_cast<const unsigned char*>("") : k.data();
    unsigned long long a = K2H_HASH_FUNC(p, k.size());
    unsigned long long b = K2H_2ND_HASH_FUNC(p, k.size());
    printf("%016llx %016llx\n", a, b);
  }
  K2HashDynLib::get()->Unload();
  return 0;
}
