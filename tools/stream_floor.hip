// Memory floor of the wave stream engine's access pattern for 4 KiB keys: each wave
// walks 64 keys (one per lane) in 64-byte rounds, loading every lane's 80-byte window
// cooperatively (5 x 16 B pieces per lane, consecutive lanes on consecutive pieces of
// one window).  Trivial compute.  Compares key strides 4096 (contiguous keys) and
// 4096 + pad, to expose HBM channel camping from a 4 KiB lockstep stride, and the same
// loads with the key rotated per lane (lane l starts at round l mod 64).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef uint32_t v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const v4 gv4;

template <bool ROT>
__global__ __launch_bounds__(256) void k(const uint8_t* __restrict__ base, uint64_t stride, uint64_t n, uint32_t rounds,
                                         uint64_t* __restrict__ out) {
  __shared__ uint4 st[4][64 * 5];
  uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t key0 = ((uint64_t)blockIdx.x * 4 + wave) * 64;
  if (key0 >= n) return;
  uint64_t paddr[5]; uint32_t poff[5];
  for (int j = 0; j < 5; ++j) {
    uint32_t g = 64 * j + lane, src = g / 5, c = g % 5;
    paddr[j] = (uint64_t)(uintptr_t)base + (key0 + src) * stride + 16 * c;
    poff[j] = src * 5 + c;
  }
  uint32_t acc = 0;
  for (uint32_t r = 0; r < rounds; ++r) {
    uint4 pf[5];
    for (int j = 0; j < 5; ++j) {
      uint32_t g = 64 * j + lane, src = g / 5;
      uint32_t rr = ROT ? (r + src) % rounds : r;
      uint64_t a = paddr[j] + 64ull * rr;
      if (rr == rounds - 1 && (g % 5) == 4) a -= 16;  // stay inside the key
      v4 v = __builtin_nontemporal_load((gv4*)(uintptr_t)a);
      pf[j] = make_uint4(v.x, v.y, v.z, v.w);
    }
    for (int j = 0; j < 5; ++j) st[wave][poff[j]] = pf[j];
    __builtin_amdgcn_wave_barrier();
    for (int m = 0; m < 4; ++m) { uint4 c = st[wave][lane * 5 + m]; acc ^= c.x ^ c.y ^ c.z ^ c.w; }
    __builtin_amdgcn_wave_barrier();
  }
  out[key0 + lane] = acc;
}

int main() {
  const uint64_t n = 1ull << 20;
  const uint32_t rounds = 64;  // 4096 B keys, 64 B per round
  uint64_t pads[] = {0, 64, 128, 256, 512};
  uint8_t* buf; uint64_t* out;
  CHK(hipMalloc(&buf, n * (4096 + 512) + 4096)); CHK(hipMalloc(&out, n * 8));
  CHK(hipMemset(buf, 0x5a, n * (4096 + 512) + 4096));
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const unsigned g = (unsigned)(n / 256);
  for (int rot = 0; rot < 2; ++rot)
    for (uint64_t pad : pads) {
      std::vector<float> t;
      for (int r = 0; r < 5; ++r) {
        CHK(hipEventRecord(e0));
        if (rot) k<true><<<g, 256>>>(buf, 4096 + pad, n, rounds, out);
        else k<false><<<g, 256>>>(buf, 4096 + pad, n, rounds, out);
        CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      double med = t[2];
      printf("stride %5llu rotated %d: %8.3f ms  -> %7.1f GB/s of key bytes\n", (unsigned long long)(4096 + pad), rot,
             med, 4096.0 * n / (med * 1e-3) / 1e9);
    }
  return 0;
}
