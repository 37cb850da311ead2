// Floors for the fixed32 kernel on this MI355X: the memory floor (same loads/stores,
// trivial compute), the VALU floor (same hash, keys synthesised in registers, no loads),
// and the real kernel, timed interleaved in one process.  Also reports the in-kernel
// shader clock from s_memtime / s_memrealtime (100 MHz) in the VALU-floor kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "../k2hash_amd/csrc/k2h_fnv_device.h"
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
using namespace k2h;

__global__ __launch_bounds__(256) void k_mem(const uint4* __restrict__ keys, uint64_t n, uint64_t* __restrict__ h1) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint4 a = keys[2 * i], b = keys[2 * i + 1];
  h1[i] = ((uint64_t)(a.x ^ a.z ^ b.x ^ b.z) << 32) | (a.y ^ a.w ^ b.y ^ b.w);
}
__global__ __launch_bounds__(256) void k_alu(uint64_t n, uint64_t seed, uint64_t* __restrict__ h1, uint64_t* clk) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = (uint32_t)i * 0x9E3779B9u;
  uint4 a = make_uint4(x, x ^ 0x55555555u, x + 7u, x * 3u), b = make_uint4(x ^ 1u, x + 11u, ~x, x ^ 0xABCDEFu);
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
  fnv_chunk32(lo, hi, a, b);
  h1[i] = ((uint64_t)hi << 32) | lo;
  if (threadIdx.x == 0 && blockIdx.x % 1024 == 0) {
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    clk[2 * (blockIdx.x / 1024)] = t1 - t0;
    clk[2 * (blockIdx.x / 1024) + 1] = r1 - r0;
  }
}
__global__ __launch_bounds__(256) void k_full(const uint4* __restrict__ keys, uint64_t n, uint64_t seed, uint64_t* __restrict__ h1) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint4 a = keys[2 * i], b = keys[2 * i + 1];
  uint32_t lo = (uint32_t)seed, hi = (uint32_t)(seed >> 32);
  fnv_chunk32(lo, hi, a, b);
  h1[i] = ((uint64_t)hi << 32) | lo;
}
// read-only floor: loads, no per-key store (one store per block)
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ keys, uint64_t n, uint64_t* __restrict__ h1) {
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  uint4 a = keys[2 * i], b = keys[2 * i + 1];
  uint32_t v = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
  if (v == 0x12345678u) h1[i] = v;
}

int main() {
  const uint64_t n = 1ull << 24;
  uint4 *k0, *k1; uint64_t *h, *clk;
  CHK(hipMalloc(&k0, n * 32)); CHK(hipMalloc(&k1, n * 32)); CHK(hipMalloc(&h, n * 8)); CHK(hipMalloc(&clk, 64 * 8 * 2));
  CHK(hipMemset(k0, 0x5a, n * 32)); CHK(hipMemset(k1, 0xa5, n * 32));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const unsigned g = (unsigned)(n / 256);
  const char* names[] = {"memory floor (load 32B, store 8B)", "read-only floor (load 32B)", "VALU floor (no loads)", "full fixed32 (flat)"};
  std::vector<float> t[4];
  for (int r = 0; r < 7; ++r) {
    for (int v = 0; v < 4; ++v) {
      const int reps = 10;
      CHK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) {
        const uint4* k = (i & 1) ? k1 : k0;
        if (v == 0) k_mem<<<g, 256>>>(k, n, h);
        else if (v == 1) k_read<<<g, 256>>>(k, n, h);
        else if (v == 2) k_alu<<<g, 256>>>(n, 14695981039346656037ULL, h, clk);
        else k_full<<<g, 256>>>(k, n, 14695981039346656037ULL, h);
      }
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms / reps);
    }
  }
  for (int v = 0; v < 4; ++v) {
    std::sort(t[v].begin(), t[v].end());
    double med = t[v][t[v].size() / 2];
    printf("%-40s median %8.2f us  min %8.2f us  -> %7.1f GB/s at 40 B/key (%.1f%% of 8 TB/s)\n", names[v], med * 1e3,
           t[v][0] * 1e3, 40.0 * n / (med * 1e-3) / 1e9, 100.0 * 40.0 * n / (med * 1e-3) / 8e12);
  }
  uint64_t hc[128]; CHK(hipMemcpy(hc, clk, sizeof hc, hipMemcpyDeviceToHost));
  double s = 0; int c = 0;
  for (int j = 0; j < 64; ++j) if (hc[2 * j + 1]) { s += (double)hc[2 * j] / (double)hc[2 * j + 1] * 0.1; ++c; }
  printf("in-kernel shader clock (VALU floor kernel, %d samples): %.3f GHz\n", c, c ? s / c : 0.0);
  return 0;
}
