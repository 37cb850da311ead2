// k2hash_amd -- hashing keys that sit anywhere in a buffer.
//
// Bulk key streams -- k2hash archives (K2HArchive::Load, lib/k2harchive.cc:279-383:
// records of a 104-byte SCOM header + key / value / subkeys / attrs / exdata,
// lib/k2hcommand.h:64-79) and import files -- interleave keys with other bytes, so
// the keys are given as (start, length) ranges instead of CSR.  The ranges are
// gathered into one packed CSR buffer (16 lanes per key, 16-byte pieces, one byte
// per lane for the tail) and hashed by the CSR kernels; the extra traffic is the key
// bytes twice, small next to the values an archive carries.
//
// K2H_AMD_FLAG_CSTR hashes each key as the C string K2HShm::Set(const char*, ...)
// passes (lib/k2hshm.cc:2081-2083: strlen(key) + 1 bytes, the NUL included).  The NUL
// is a zero byte, so h1 = state(key) * P and h2 = state(key) (the state before the last
// byte, lib/k2hashfunc.cc:83-85); an empty string is the one-byte key "\0", whose h1 and
// h2 are both seed * P.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "k2h_kernels.h"

namespace k2h {
namespace {

typedef uint32_t u32x4_ua __attribute__((ext_vector_type(4), aligned(1)));
constexpr int kGroup = 16;

__global__ __launch_bounds__(256) void gather_ranges_kernel(const uint8_t* __restrict__ base,
                                                            const uint64_t* __restrict__ starts,
                                                            const uint64_t* __restrict__ lens,
                                                            const uint64_t* __restrict__ off, uint64_t n,
                                                            uint8_t* __restrict__ packed) {
  const uint64_t i = ((uint64_t)blockIdx.x * 256u + threadIdx.x) / kGroup;
  const uint32_t q = threadIdx.x % kGroup;
  if (i >= n) return;
  const uint64_t len = lens[i];
  const uint8_t* src = base + starts[i];
  uint8_t* dst = packed + off[i];
  const uint64_t full = len & ~15ull;
  for (uint64_t j = 16ull * q; j < full; j += 16ull * kGroup)
    *reinterpret_cast<u32x4_ua*>(dst + j) = *reinterpret_cast<const u32x4_ua*>(src + j);
  const uint64_t t = full + q;
  if (t < len) dst[t] = src[t];
}

// C-string semantics on top of the raw hashes (see the header comment).
__global__ __launch_bounds__(256) void cstr_fixup_kernel(const uint64_t* __restrict__ lens, uint64_t n, uint64_t seed,
                                                         uint64_t* __restrict__ h1, uint64_t* __restrict__ h2) {
  const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint64_t P = 1099511628211ULL;  // lib/k2hashfunc.cc:56
  uint64_t raw = h1[i];
  uint64_t a = lens[i] ? raw * P : seed * P, b = lens[i] ? raw : seed * P;
  h1[i] = a;
  if (h2) h2[i] = b;
}

}  // namespace

hipError_t launch_ranges(const void* base, const uint64_t* starts, const uint64_t* lens, uint64_t n, uint64_t seed,
                         bool cstr, uint64_t* h1, uint64_t* h2, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  // offsets[0] = 0, offsets[i+1] = sum of lens[0..i]
  uint64_t* off = nullptr;
  hipError_t e = hipMallocAsync((void**)&off, (n + 1) * 8, stream);
  if (e != hipSuccess) return e;
  size_t tmp_bytes = 0;
  void* tmp = nullptr;
  uint8_t* packed = nullptr;
  uint64_t total = 0;
  e = hipMemsetAsync(off, 0, 8, stream);
  if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, lens, off + 1, n, stream);
  if (e == hipSuccess) e = hipMallocAsync(&tmp, tmp_bytes ? tmp_bytes : 1, stream);
  if (e == hipSuccess) e = hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, lens, off + 1, n, stream);
  if (e == hipSuccess) e = hipMemcpyAsync(&total, off + n, 8, hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);  // the packed size sizes the next allocation
  if (e == hipSuccess) e = hipMallocAsync((void**)&packed, total ? total : 16, stream);
  if (e == hipSuccess) {
    gather_ranges_kernel<<<(unsigned)((n * kGroup + 255) / 256), 256, 0, stream>>>((const uint8_t*)base, starts, lens,
                                                                                   off, n, packed);
    e = hipGetLastError();
  }
  // the CSR kernels treat a NULL byte buffer as "all keys empty"; packed is never NULL here
  if (e == hipSuccess) e = launch_csr(packed, off, n, seed, h1, cstr ? nullptr : h2, stream);
  if (e == hipSuccess && cstr) {
    cstr_fixup_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(lens, n, seed, h1, h2);
    e = hipGetLastError();
  }
  if (packed) (void)hipFreeAsync(packed, stream);
  if (tmp) (void)hipFreeAsync(tmp, stream);
  hipError_t f = hipFreeAsync(off, stream);
  return e != hipSuccess ? e : f;
}

}  // namespace k2h
