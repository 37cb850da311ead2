// Memory floor of candidate per-lane-key access patterns for 1M x 4 KiB keys
// (64 lanes = 64 keys per wave, keys at a 4 KiB stride), trivial compute:
//   coop<CH,P>: every round the wave loads each lane's P x 16 B window cooperatively
//               (consecutive lanes on consecutive pieces), through LDS; CH chunks/round
//   direct<C>:  each lane loads C x 16 B of its own key per round into registers
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef uint32_t v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4 gv4;

template <int CH, int P, bool NT>
__global__ __launch_bounds__(256) void coop(const uint8_t* __restrict__ base, uint64_t n, uint64_t* __restrict__ out) {
  __shared__ uint4 st[4][64 * P];
  const uint32_t rounds = 4096 / (16 * CH);
  uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t key0 = ((uint64_t)blockIdx.x * 4 + wave) * 64;
  if (key0 >= n) return;
  uint64_t paddr[P]; uint32_t poff[P];
#pragma unroll
  for (int j = 0; j < P; ++j) {
    uint32_t g = 64 * j + lane, src = g / P, c = g % P;
    paddr[j] = (uint64_t)(uintptr_t)base + (key0 + src) * 4096 + 16 * c;
    poff[j] = src * P + c;
  }
  uint32_t acc = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    uint4 pf[P];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      uint64_t a = paddr[j] + 16ull * CH * r;
      if (P > CH && r == rounds - 1 && (64 * j + lane) % P == P - 1) a -= 16;
      v4 v = NT ? __builtin_nontemporal_load((gv4*)(uintptr_t)a) : *(gv4*)(uintptr_t)a;
      pf[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
#pragma unroll
    for (int j = 0; j < P; ++j) st[wave][poff[j]] = pf[j];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int m = 0; m < CH; ++m) { uint4 c = st[wave][lane * P + m]; acc ^= c.x ^ c.y ^ c.z ^ c.w; }
    __builtin_amdgcn_wave_barrier();
  }
  out[key0 + lane] = acc;
}

template <int C, bool NT>
__global__ __launch_bounds__(256) void direct(const uint8_t* __restrict__ base, uint64_t n, uint64_t* __restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t a0 = (uint64_t)(uintptr_t)base + i * 4096;
  uint32_t acc = 0;
  for (uint32_t r = 0; r < 4096 / (16 * C); ++r) {
    v4 v[C];
#pragma unroll
    for (int m = 0; m < C; ++m) {
      gv4* p = (gv4*)(uintptr_t)(a0 + 16ull * (C * r + m));
      v[m] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int m = 0; m < C; ++m) acc ^= v[m].x ^ v[m].y ^ v[m].z ^ v[m].w;
  }
  out[i] = acc;
}

template <int C>
__global__ __launch_bounds__(256) void direct_ua(const uint8_t* __restrict__ base, uint64_t n, uint64_t* __restrict__ out) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4), aligned(1)));
  typedef __attribute__((address_space(1))) const v4u gv4u;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint64_t a0 = (uint64_t)(uintptr_t)base + i * 4096 + 5;
  uint32_t acc = 0;
  for (uint32_t r = 0; r < 4096 / (16 * C) - 1; ++r) {
    v4u v[C];
#pragma unroll
    for (int m = 0; m < C; ++m) v[m] = *(gv4u*)(uintptr_t)(a0 + 16ull * (C * r + m));
#pragma unroll
    for (int m = 0; m < C; ++m) acc ^= v[m].x ^ v[m].y ^ v[m].z ^ v[m].w;
  }
  out[i] = acc;
}
#include "../k2hash_amd/csrc/k2h_fnv_device.h"
// VALU floor at a forced occupancy (dynamic LDS per block limits blocks per CU)
__global__ __launch_bounds__(256) void valu_occ(uint64_t n, uint64_t* __restrict__ out) {
  extern __shared__ uint8_t dyn[];
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 0x9E3779B9u;
  uint32_t lo = 0x84222325u, hi = 0xcbf29ce4u;
  for (int r = 0; r < 32; ++r) {
    uint4 a = make_uint4(x, x ^ 0x55555555u, x + 7u, x * 3u);
    k2h::fnv_chunk16(lo, hi, a);
    x += lo;
  }
  if (lo == 0x12345) dyn[threadIdx.x] = 1;
  out[i] = ((uint64_t)hi << 32) | lo;
}
int main() {
  const uint64_t n = 1ull << 20;
  uint8_t* buf; uint64_t* out;
  CHK(hipMalloc(&buf, n * 4096)); CHK(hipMalloc(&out, n * 8));
  CHK(hipMemset(buf, 0x5a, n * 4096));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const unsigned g = (unsigned)(n / 256);
  struct V { const char* name; void (*f)(const uint8_t*, uint64_t, uint64_t*); };
  V vs[] = {
    {"coop CH4 P5 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<4, 5, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"coop CH8 P8 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<8, 8, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"coop CH8 P9 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<8, 9, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"coop CH8 P8 default", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<8, 8, false><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"coop CH16 P16 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<16, 16, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"coop CH16 P17 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<16, 17, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"direct C1 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { direct<1, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"direct C4 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { direct<4, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"direct C8 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { direct<8, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"direct C8 default", [](const uint8_t* b, uint64_t n, uint64_t* o) { direct<8, false><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"coop CH4 P4 nt (64B aligned)", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<4, 4, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"coop CH4 P4 default", [](const uint8_t* b, uint64_t n, uint64_t* o) { coop<4, 4, false><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"direct C8 default unaligned", [](const uint8_t* b, uint64_t n, uint64_t* o) { direct_ua<8><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"direct C4 default", [](const uint8_t* b, uint64_t n, uint64_t* o) { direct<4, false><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
    {"direct C16 nt", [](const uint8_t* b, uint64_t n, uint64_t* o) { direct<16, true><<<(unsigned)(n / 256), 256>>>(b, n, o); }},
  };
  (void)g;
  for (auto& v : vs) {
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
      CHK(hipEventRecord(e0));
      v.f(buf, n, out);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("%-22s %8.3f ms  -> %7.1f GB/s of key bytes\n", v.name, t[2], 4096.0 * n / (t[2] * 1e-3) / 1e9);
  }
  // VALU occupancy sweep: 1M lanes x 32 chunks (512 B) of hashing, no memory traffic
  for (int wps : {1, 2, 3, 4, 6, 8}) {
    int blocks_per_cu = wps;  // 256-thread blocks = 1 wave per SIMD each
    size_t lds = 160 * 1024 / blocks_per_cu - 1024;
    if (lds > 64 * 1024) lds = 64 * 1024;
    CHK(hipFuncSetAttribute((const void*)valu_occ, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    std::vector<float> t;
    for (int r = 0; r < 5; ++r) {
      CHK(hipEventRecord(e0));
      valu_occ<<<(unsigned)(n / 256), 256, lds>>>(n, out);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("VALU floor, ~%d waves/SIMD (lds %zu): %8.3f ms -> %7.1f GB/s of hashed bytes\n", wps, lds, t[2],
           512.0 * n / (t[2] * 1e-3) / 1e9);
  }
  return 0;
}
