// Memory-floor variants for the fixed32 access pattern (read 32 B/key, write 8 B/key),
// trivial compute, timed interleaved in one process: which load/store forms move the
// 671 MB per 16M-key launch fastest on MI355X.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__device__ __forceinline__ uint64_t mix(uint4 a, uint4 b) {
  return ((uint64_t)(a.x ^ a.z ^ b.x ^ b.z) << 32) | (a.y ^ a.w ^ b.y ^ b.w);
}
template <int V>
__global__ __launch_bounds__(256) void k(const uint4* __restrict__ keys, uint64_t n, uint64_t* __restrict__ h1) {
  __shared__ uint4 slot[4][128];
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint4 a, b;
  if constexpr (V == 0 || V == 2 || V == 4) {        // per-lane 2x16B at 32B stride
    a = keys[2 * i]; b = keys[2 * i + 1];
  } else if constexpr (V == 1 || V == 3) {            // nt loads
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u* kv = reinterpret_cast<const v4u*>(keys);
    v4u x = __builtin_nontemporal_load(&kv[2 * i]), y = __builtin_nontemporal_load(&kv[2 * i + 1]);
    a = make_uint4(x.x, x.y, x.z, x.w); b = make_uint4(y.x, y.y, y.z, y.w);
  } else {                                            // V 5,6: coalesced 1 KiB + LDS transpose
    uint64_t t = i >> 6;
    slot[wave][lane] = keys[t * 128 + lane];
    slot[wave][lane + 64] = keys[t * 128 + 64 + lane];
    __builtin_amdgcn_wave_barrier();
    a = slot[wave][2 * lane]; b = slot[wave][2 * lane + 1];
  }
  uint64_t h = mix(a, b);
  if constexpr (V == 0 || V == 1 || V == 5) {
    h1[i] = h;
  } else if constexpr (V == 2 || V == 3 || V == 6) {
    __builtin_nontemporal_store(h, &h1[i]);
  } else {  // V == 4: pair lanes, even lanes store 16 B
    uint64_t o = __shfl_xor(h, 1, 64);
    if ((lane & 1) == 0) {
      uint4 v = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)o, (uint32_t)(o >> 32));
      *reinterpret_cast<uint4*>(&h1[i]) = v;
    }
  }
}

int main() {
  const uint64_t n = 1ull << 24;
  uint4 *k0, *k1; uint64_t *h;
  CHK(hipMalloc(&k0, n * 32)); CHK(hipMalloc(&k1, n * 32)); CHK(hipMalloc(&h, n * 8));
  CHK(hipMemset(k0, 0x5a, n * 32)); CHK(hipMemset(k1, 0xa5, n * 32));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const unsigned g = (unsigned)(n / 256);
  const char* names[] = {"ld 2x16B, st 8B", "ld nt, st 8B", "ld, st nt", "ld nt, st nt", "ld, st paired 16B",
                         "ld coalesced+LDS, st 8B", "ld coalesced+LDS, st nt"};
  const int NV = 7;
  std::vector<float> t[NV];
  for (int r = 0; r < 7; ++r)
    for (int v = 0; v < NV; ++v) {
      const int reps = 10;
      CHK(hipEventRecord(e0));
      for (int it = 0; it < reps; ++it) {
        const uint4* kk = (it & 1) ? k1 : k0;
        switch (v) {
          case 0: k<0><<<g, 256>>>(kk, n, h); break;
          case 1: k<1><<<g, 256>>>(kk, n, h); break;
          case 2: k<2><<<g, 256>>>(kk, n, h); break;
          case 3: k<3><<<g, 256>>>(kk, n, h); break;
          case 4: k<4><<<g, 256>>>(kk, n, h); break;
          case 5: k<5><<<g, 256>>>(kk, n, h); break;
          case 6: k<6><<<g, 256>>>(kk, n, h); break;
        }
      }
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms / reps);
    }
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    double med = t[v][t[v].size() / 2];
    printf("%-28s median %8.2f us  min %8.2f us  -> %7.1f GB/s (%.1f%% of 8 TB/s)\n", names[v], med * 1e3, t[v][0] * 1e3,
           40.0 * n / (med * 1e-3) / 1e9, 100.0 * 40.0 * n / (med * 1e-3) / 8e12);
  }
  return 0;
}
