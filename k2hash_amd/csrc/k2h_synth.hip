// k2hash_amd -- synthetic workload generator (bench/test harness, not the hash path).
//
// Spec (shared with oracle/fnv_oracle.c, implemented independently there):
//   word j of a stream with seed s = splitmix64 output j = mix(s + (j+1)*0x9E3779B97F4A7C15),
//   bytes are the little-endian bytes of consecutive words;
//   CSR length of key i = min_len + mix(seed_len + (i+1)*GAMMA) % (max_len - min_len + 1).
// Generating on the device keeps multi-GiB inputs out of PCIe and host memory.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "k2h_kernels.h"

namespace k2h {

__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t j) {
  uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// out[i] = byte (byte_off + i) of the stream; one 8-byte word per thread-iteration.
__global__ __launch_bounds__(256) void synth_bytes_kernel(uint8_t* __restrict__ out, uint64_t nbytes, uint64_t seed,
                                                          uint64_t byte_off) {
  // process the stream in words aligned to the stream (not to `out`)
  uint64_t first_word = byte_off >> 3;
  uint64_t last_word = (byte_off + nbytes + 7) >> 3;
  uint64_t nwords = last_word - first_word;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  bool aligned = ((byte_off & 7) == 0) && (((uintptr_t)out & 7) == 0);
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nwords; t += stride) {
    uint64_t w = splitmix_word(seed, first_word + t);
    uint64_t pos = (first_word + t) << 3;  // stream byte position of byte 0 of w
    if (aligned && pos + 8 <= byte_off + nbytes) {
      *reinterpret_cast<uint64_t*>(out + (pos - byte_off)) = w;
    } else {
      for (int k = 0; k < 8; ++k) {
        uint64_t q = pos + k;
        if (q >= byte_off && q < byte_off + nbytes) out[q - byte_off] = (uint8_t)(w >> (8 * k));
      }
    }
  }
}

__global__ __launch_bounds__(256) void synth_lengths_kernel(uint32_t* __restrict__ lens, uint64_t n, uint64_t seed,
                                                            uint64_t first_key, uint32_t min_len, uint32_t span) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    lens[i] = min_len + (uint32_t)(splitmix_word(seed, first_key + i) % span);
}

hipError_t launch_synth_bytes(uint8_t* out, uint64_t nbytes, uint64_t seed, uint64_t byte_off, hipStream_t stream) {
  if (nbytes == 0) return hipSuccess;
  synth_bytes_kernel<<<4096, 256, 0, stream>>>(out, nbytes, seed, byte_off);
  return hipGetLastError();
}

hipError_t launch_synth_lengths(uint32_t* lens, uint64_t n, uint64_t seed, uint64_t first_key, uint32_t min_len,
                                uint32_t max_len, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  synth_lengths_kernel<<<4096, 256, 0, stream>>>(lens, n, seed, first_key, min_len, max_len - min_len + 1);
  return hipGetLastError();
}

}  // namespace k2h
