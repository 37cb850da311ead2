// k2hash_amd -- scalar drop-in plugin body (CPU).
//
// The three symbols libk2hash resolves from a hash plugin (lib/k2hashfunc.h:62-74,
// lib/k2hashfunc.cc:149-151).  Every k2hash call site hashes one key synchronously on
// a CPU thread, so the plugin path stays on the CPU: a GPU launch per key would cost
// ~100x the hash itself.  Bulk callers use the batch ABI in k2h_batch.cc instead.
//
// Contract kept from the reference: NULL or length 0 -> 0 (lib/k2hashfunc.cc:66-68,
// 80-82); bytes are sign-extended before the XOR (lib/k2hashfunc.cc:53,55); the second
// hash covers length-1 bytes when length > 1 (lib/k2hashfunc.cc:83-85).  Reentrant,
// no allocation, no locks, no logging, nothing initialised at load time (safe under
// dlopen/dlclose at exit, lib/k2hashfunc.cc:114-117, and across fork,
// tests/k2hbench.cc:1170).
#include <stddef.h>
#include <stdint.h>

#include "../../include/k2hash_amd.h"

namespace {

constexpr uint64_t kSeed = 14695981039346656037ULL;
constexpr uint64_t kPrime = 1099511628211ULL;

inline uint64_t fnv_signed(const signed char* p, size_t n, uint64_t h) {
  // Four bytes per iteration keeps the loop overhead off the serial xor/imul chain.
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    h = (h ^ (uint64_t)(int64_t)p[i]) * kPrime;
    h = (h ^ (uint64_t)(int64_t)p[i + 1]) * kPrime;
    h = (h ^ (uint64_t)(int64_t)p[i + 2]) * kPrime;
    h = (h ^ (uint64_t)(int64_t)p[i + 3]) * kPrime;
  }
  for (; i < n; ++i) h = (h ^ (uint64_t)(int64_t)p[i]) * kPrime;
  return h;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) k2h_hash_t k2h_hash(const void* ptr, size_t length) {
  if (!ptr || length < 1) return 0;
  return fnv_signed(static_cast<const signed char*>(ptr), length, kSeed);
}

__attribute__((visibility("default"))) k2h_hash_t k2h_second_hash(const void* ptr, size_t length) {
  if (!ptr || length < 1) return 0;
  if (length > 1) --length;
  return fnv_signed(static_cast<const signed char*>(ptr), length, kSeed);
}

__attribute__((visibility("default"))) const char* k2h_hash_version(void) {
  // Same string as the reference builtin (lib/k2hashfunc.cc:38): the hashes are identical,
  // and k2hash stamps/checks this string in every file header (lib/k2hshminit.cc:405,
  // 641-646), so existing files stay attachable whichever override route is used.
  static const char kVersion[] = "FNV-1A BUILTIN";
  return kVersion;
}

}  // extern "C"
