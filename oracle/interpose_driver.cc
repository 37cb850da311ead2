// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// Driver over _ref/libk2hcaller_ref.so (interpose_caller.cc): prints which object the
// library's k2h_hash resolved to (dladdr), the version its call site stamps, and h1 / h2
// for each hex key on stdin ("-" = empty key) as the library's K2H_HASH_FUNC /
// K2H_2ND_HASH_FUNC call sites compute them.  Run with and without LD_PRELOAD.
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

extern "C" {
void caller_hash(const void* p, size_t n, uint64_t* h1, uint64_t* h2);
const char* caller_stamp_version(void);
const void* caller_hash_fn(void);
}

int main() {
  Dl_info info;
  memset(&info, 0, sizeof info);
  if (!dladdr(caller_hash_fn(), &info) || !info.dli_fname) return 2;
  printf("FN %s\n", info.dli_fname);
  printf("VERSION %s\n", caller_stamp_version());
  static char line[1 << 16];
  while (fgets(line, sizeof line, stdin)) {
    line[strcspn(line, "\r\n")] = 0;
    std::vector<unsigned char> k;
    if (strcmp(line, "-"))
      for (size_t i = 0; line[i] && line[i + 1]; i += 2) {
        unsigned v;
        sscanf(line + i, "%2x", &v);
        k.push_back((unsigned char)v);
      }
    uint64_t a, b;
    caller_hash(k.empty() ? "" : (const char*)k.data(), k.size(), &a, &b);
    printf("%016llx %016llx\n", (unsigned long long)a, (unsigned long long)b);
  }
  return 0;
}
