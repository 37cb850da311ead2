// Host-path probe: what each way of moving caller-owned (pageable) host memory to the
// GPU and back costs on this box -- pinned copies, pageable copies (runtime staging),
// hipHostRegister of the caller's buffer (+ mapped zero-copy reads by a kernel), and
// host memcpy into pinned staging at 1..16 threads.  Numbers feed the design of
// k2h_amd_hash_*_host.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/host_probe tools/host_probe.hip -lpthread
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include <thread>
#include <vector>

static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}
#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void sum_kernel(const uint4* __restrict__ p, uint64_t n16, uint64_t* out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, s = 0;
  for (; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x123456789ull) *out = s;
}

static void par_copy(void* dst, const void* src, size_t len, int threads) {
  std::vector<std::thread> th;
  size_t per = (len + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    size_t a = per * t, b = a + per < len ? a + per : len;
    if (a >= b) break;
    th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const size_t N = (argc > 1 ? atol(argv[1]) : 512) << 20;
  char* pageable = (char*)malloc(N);
  for (size_t i = 0; i < N; i += 4096) pageable[i] = (char)i;  // touch
  memset(pageable, 1, N);
  char *pinned, *dev;
  CK(hipHostMalloc((void**)&pinned, N, hipHostMallocDefault));
  CK(hipMalloc((void**)&dev, N));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto bw = [&](const char* what, void* d, const void* s, size_t n, hipMemcpyKind k) {
    double best = 1e9;
    for (int r = 0; r < 4; ++r) {
      double t0 = now();
      CK(hipMemcpyAsync(d, s, n, k, st));
      CK(hipStreamSynchronize(st));
      double t = now() - t0;
      if (r && t < best) best = t;
    }
    printf("%-44s %8.2f GB/s  (%zu MiB, %.2f ms)\n", what, n / best / 1e9, n >> 20, best * 1e3);
  };
  bw("H2D pinned", dev, pinned, N, hipMemcpyHostToDevice);
  bw("D2H pinned", pinned, dev, N, hipMemcpyDeviceToHost);
  bw("H2D pageable (runtime staging)", dev, pageable, N, hipMemcpyHostToDevice);
  bw("D2H pageable (runtime staging)", pageable, dev, N, hipMemcpyDeviceToHost);
  bw("H2D pageable 64 MiB", dev, pageable, 64 << 20, hipMemcpyHostToDevice);
  for (int th : {1, 2, 4, 8, 16}) {
    double best = 1e9;
    for (int r = 0; r < 3; ++r) {
      double t0 = now();
      par_copy(pinned, pageable, N, th);
      double t = now() - t0;
      if (t < best) best = t;
    }
    printf("memcpy pageable->pinned %2d threads             %8.2f GB/s\n", th, N / best / 1e9);
  }
  // hipHostRegister of the caller's (already touched) buffer, whole and in 64 MiB pieces
  for (size_t piece : {(size_t)N, (size_t)64 << 20, (size_t)16 << 20}) {
    double treg = 0, tunreg = 0;
    for (size_t off = 0; off < N; off += piece) {
      double t0 = now();
      CK(hipHostRegister(pageable + off, piece, hipHostRegisterDefault));
      double t1 = now();
      CK(hipHostUnregister(pageable + off));
      tunreg += now() - t1;
      treg += t1 - t0;
    }
    printf("hipHostRegister %4zu MiB pieces: register %.2f ms (%.1f GB/s), unregister %.2f ms\n", piece >> 20,
           treg * 1e3, N / treg / 1e9, tunreg * 1e3);
  }
  {
    CK(hipHostRegister(pageable, N, hipHostRegisterMapped));
    bw("H2D registered", dev, pageable, N, hipMemcpyHostToDevice);
    bw("D2H registered", pageable, dev, N, hipMemcpyDeviceToHost);
    void* dp = nullptr;
    CK(hipHostGetDevicePointer(&dp, pageable, 0));
    uint64_t* out;
    CK(hipMalloc((void**)&out, 8));
    for (int grid : {1024, 4096, 16384}) {
      double best = 1e9;
      for (int r = 0; r < 3; ++r) {
        double t0 = now();
        sum_kernel<<<grid, 256, 0, st>>>((const uint4*)dp, N / 16, out);
        CK(hipStreamSynchronize(st));
        double t = now() - t0;
        if (r && t < best) best = t;
      }
      printf("kernel reads mapped host memory, grid %5d   %8.2f GB/s\n", grid, N / best / 1e9);
    }
    CK(hipHostUnregister(pageable));
  }
  // a fresh, never-registered buffer (first registration of cold pages)
  {
    char* fresh = (char*)malloc(N);
    memset(fresh, 2, N);
    double t0 = now();
    CK(hipHostRegister(fresh, N, hipHostRegisterDefault));
    printf("hipHostRegister fresh %zu MiB: %.2f ms\n", N >> 20, (now() - t0) * 1e3);
    CK(hipHostUnregister(fresh));
    free(fresh);
  }
  printf("EXIT 0\n");
  return 0;
}
