// Copy floor for the RALLEDATA shape: read R bytes, write W bytes, aligned 16-byte
// pieces, consecutive lanes on consecutive pieces, trivial compute -- the HBM rate a
// read+write kernel of this mix can reach on MI355X (bench config ralledata: R = 1.50 GB
// of keys + values + offsets, W = 2.11 GB of blobs + blob offsets).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/copy_floor tools/copy_floor.hip && /tmp/copy_floor
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// V0: one read piece + one write piece per thread (nt stores); V1: plain stores;
// V2: PPT pieces per thread, all loads first; V3: write-only; V4: read-only
template <int V, int PPT = 1>
__global__ __launch_bounds__(256) void k(const v4u* __restrict__ src, uint64_t nr, v4u* __restrict__ dst, uint64_t nw,
                                         v4u* __restrict__ sink) {
  const uint64_t t = (uint64_t)blockIdx.x * 256u * PPT + threadIdx.x;
  v4u a[PPT];
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t i = t + 256ull * u;
    a[u] = v4u{(uint32_t)i, 1, 2, 3};
    if (V != 3 && i < nr) a[u] = src[i];
  }
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const uint64_t i = t + 256ull * u;
    if (V == 4) {
      if (a[u].x == 0x12345678u && a[u].y == 7u) sink[0] = a[u];
    } else if (i < nw) {
      if (V == 1) dst[i] = a[u] ^ 0x5a5a5a5au;
      else __builtin_nontemporal_store(a[u] ^ 0x5a5a5a5au, &dst[i]);
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t R = argc > 1 ? strtoull(argv[1], 0, 0) : 1500000000ull;
  const uint64_t W = argc > 2 ? strtoull(argv[2], 0, 0) : 2110000000ull;
  const uint64_t nr = R / 16, nw = W / 16, nmax = nr > nw ? nr : nw;
  v4u *src, *dst, *sink;
  CHK(hipMalloc(&src, nr * 16));
  CHK(hipMalloc(&dst, nw * 16));
  CHK(hipMalloc(&sink, 64));
  CHK(hipMemset(src, 1, nr * 16));
  CHK(hipMemset(dst, 0, nw * 16));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto launch = [&](int v) {
    unsigned g1 = (unsigned)((nmax + 255) / 256), g4 = (unsigned)((nmax + 1023) / 1024);
    switch (v) {
      case 0: k<0><<<g1, 256>>>(src, nr, dst, nw, sink); break;
      case 1: k<1><<<g1, 256>>>(src, nr, dst, nw, sink); break;
      case 2: k<0, 4><<<g4, 256>>>(src, nr, dst, nw, sink); break;
      case 3: k<3><<<(unsigned)((nw + 255) / 256), 256>>>(src, 0, dst, nw, sink); break;
      case 4: k<4><<<(unsigned)((nr + 255) / 256), 256>>>(src, nr, dst, 0, sink); break;
    }
  };
  const char* name[] = {"read+write nt, 1 piece/thread", "read+write plain stores", "read+write nt, 4 pieces/thread",
                        "write only (W)", "read only (R)"};
  for (int w = 0; w < 30; ++w) launch(w % 5);
  float best[5] = {1e9, 1e9, 1e9, 1e9, 1e9};
  for (int r = 0; r < 5; ++r)
    for (int v = 0; v < 5; ++v) {
      CHK(hipEventRecord(e0));
      for (int i = 0; i < 10; ++i) launch(v);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms / 10 < best[v]) best[v] = ms / 10;
    }
  for (int v = 0; v < 5; ++v) {
    const double bytes = v == 3 ? (double)W : v == 4 ? (double)R : (double)(R + W);
    printf("%-34s %8.3f ms  %7.1f GB/s\n", name[v], best[v], bytes / best[v] / 1e6);
  }
  return 0;
}
