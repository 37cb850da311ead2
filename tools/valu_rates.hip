// VALU issue-rate microbenchmark for the integer ops on the FNV-1a step (gfx950).
// Each lane runs 8 independent dependency chains of one instruction, so the
// loop is issue-bound, not latency-bound.  Prints cycles per wave-instruction
// per SIMD at 8 waves/SIMD (2048 threads/CU * 256 CUs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int OP>
__global__ __launch_bounds__(256) void kbench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,
           a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b0 = a0 * 3, b1 = a1 * 3, b2 = a2 * 3, b3 = a3 * 3, b4 = a4 * 3, b5 = a5 * 3, b6 = a6 * 3, b7 = a7 * 3;
  const uint32_t k = 0x1b3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if constexpr (OP == 0) {
#define X(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##i) : "v"(b##i));
        REP8(X)
#undef X
      } else if constexpr (OP == 1) {
#define X(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##i) : "s"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 2) {
#define X(i) asm volatile("v_mad_u64_u32 %0, s[0:1], %0, %2, 0" : "+v"(*(uint64_t*)&a##i), "+v"(b##i) : "s"(k) : "s0", "s1");
        // note: the 64-bit pair is formed from a##i only through the cast; use a proper 64-bit var below
#undef X
      } else if constexpr (OP == 3) {
#define X(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a##i) : "s"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 4) {
#define X(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a##i) : "s"(k), "v"(b##i));
        REP8(X)
#undef X
      } else if constexpr (OP == 5) {
#define X(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a##i) : "s"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 6) {
#define X(i) asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(a##i) : "v"(b##i));
        REP8(X)
#undef X
      } else if constexpr (OP == 7) {
#define X(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##i) : "v"(b##i), "s"(k));
        REP8(X)
#undef X
      } else if constexpr (OP == 8) {
#define X(i) asm volatile("v_xor_b32_sdwa %0, sext(%1), %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "+v"(a##i) : "v"(b##i));
        REP8(X)
#undef X
      } else if constexpr (OP == 9) {
#define X(i) asm volatile("v_mad_u32_u16 %0, %0, %1, %2" : "+v"(a##i) : "s"(k), "v"(b##i));
        REP8(X)
#undef X
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7;
}

// v_mad_u64_u32 needs 64-bit register pairs: separate kernel.
__global__ __launch_bounds__(256) void kbench_mad64(uint64_t* out, int iters, uint32_t seed) {
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const uint32_t k = 0x1b3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#define X(i) asm volatile("v_mad_u64_u32 %0, s[2:3], %1, %2, %0" : "+v"(a##i) : "v"((uint32_t)a##i), "s"(k) : "s2", "s3");
      REP8(X)
#undef X
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  int clk_khz = prop.clockRate;
  printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, cus, clk_khz);
  const int threads = 256, blocks = cus * 8;  // 8 blocks of 256 = 32 waves/CU = 8 waves/SIMD
  uint32_t* d32; uint64_t* d64;
  CHK(hipMalloc(&d32, sizeof(uint32_t) * threads * blocks));
  CHK(hipMalloc(&d64, sizeof(uint64_t) * threads * blocks));
  const int iters = 4096;
  const double insts_per_lane = (double)iters * 16 * 8;
  const char* names[] = {"v_xor_b32", "v_mul_lo_u32", "(unused)", "v_mul_u32_u24", "v_mad_u32_u24",
                         "v_mul_hi_u32", "v_lshl_add_u32", "v_perm_b32", "v_xor_b32_sdwa(sext BYTE_1)", "v_mad_u32_u16",
                         "v_mad_u64_u32"};
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  auto run = [&](int op) {
    for (int rep = 0; rep < 2; ++rep) {
      CHK(hipEventRecord(e0));
      switch (op) {
        case 0: kbench<0><<<blocks, threads>>>(d32, iters, 1); break;
        case 1: kbench<1><<<blocks, threads>>>(d32, iters, 1); break;
        case 3: kbench<3><<<blocks, threads>>>(d32, iters, 1); break;
        case 4: kbench<4><<<blocks, threads>>>(d32, iters, 1); break;
        case 5: kbench<5><<<blocks, threads>>>(d32, iters, 1); break;
        case 6: kbench<6><<<blocks, threads>>>(d32, iters, 1); break;
        case 7: kbench<7><<<blocks, threads>>>(d32, iters, 1); break;
        case 8: kbench<8><<<blocks, threads>>>(d32, iters, 1); break;
        case 9: kbench<9><<<blocks, threads>>>(d32, iters, 1); break;
        case 10: kbench_mad64<<<blocks, threads>>>(d64, iters, 1); break;
      }
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 1) {
        // wave-instructions per SIMD = waves per SIMD (8) * insts per lane
        double wave_insts_per_simd = 8.0 * insts_per_lane;
        double ns_per = ms * 1e6 / wave_insts_per_simd;
        double lane_ops = (double)blocks * threads * insts_per_lane / (ms * 1e-3);
        printf("%-30s %8.3f ms  %6.3f ns/wave-inst/SIMD  (= %5.2f cyc @2.4GHz)  %6.2f T lane-ops/s\n",
               names[op], ms, ns_per, ns_per * 2.4, lane_ops / 1e12);
      }
    }
  };
  int ops[] = {0, 6, 7, 8, 3, 4, 9, 1, 5, 10};
  for (int op : ops) run(op);
  return 0;
}
