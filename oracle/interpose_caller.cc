// ORACLE -- TEST INFRASTRUCTURE ONLY.
//
// A stand-in for libk2hash's own call sites, compiled into ONE shared library together
// with the reference's lib/k2hashfunc.cc + lib/k2hdbg.cc (oracle/Makefile, _ref/
// libk2hcaller_ref.so) -- the way libk2hash.so carries the weak builtins beside the code
// that calls them (lib/Makefile.am:133-134).  The calls go exactly as K2HShm's do:
//   hash / subhash through K2H_HASH_FUNC / K2H_2ND_HASH_FUNC   (lib/k2hshm.cc:1230-1231)
//   the file stamp through k2h_hash_version() directly         (lib/k2hshminit.cc:405)
// so a strong k2h_hash / k2h_second_hash / k2h_hash_version interposed with LD_PRELOAD
// (the route k2hbench needs: it has no -ext option, tests/k2hbench.cc:297-333) is what
// these call sites reach.  tests/test_plugin_abi.py drives it via interpose_driver.
#include <stddef.h>
#include <stdint.h>

#include "k2hashfunc.h"

extern "C" {

__attribute__((visibility("default"))) void caller_hash(const void* p, size_t n, uint64_t* h1, uint64_t* h2) {
  *h1 = K2H_HASH_FUNC(p, n);
  *h2 = K2H_2ND_HASH_FUNC(p, n);
}

__attribute__((visibility("default"))) const char* caller_stamp_version(void) { return k2h_hash_version(); }

// the k2h_hash this library's call sites bind to (its GOT entry)
__attribute__((visibility("default"))) const void* caller_hash_fn(void) {
  return reinterpret_cast<const void*>(&k2h_hash);
}

}  // extern "C"
