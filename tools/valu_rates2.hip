// Second VALU issue-rate probe: which gfx950 integer ops issue in 2 vs 4 cycles per wave64,
// and whether a mixed stream's costs add.  8 waves/SIMD, 8 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

#define OPS(Y) \
  Y(0, "v_xor_b32_e32", "v_xor_b32_e32 %0, %0, %1") \
  Y(1, "v_xor_b32_e64", "v_xor_b32_e64 %0, %0, %1") \
  Y(2, "v_add_u32_e32", "v_add_u32_e32 %0, %0, %1") \
  Y(3, "v_lshlrev_b32_e32", "v_lshlrev_b32_e32 %0, 8, %0") \
  Y(4, "v_and_b32_e32", "v_and_b32_e32 %0, %0, %1") \
  Y(5, "v_mul_u32_u24_e32(v)", "v_mul_u32_u24_e32 %0, %0, %1") \
  Y(6, "v_or3_b32", "v_or3_b32 %0, %0, %1, %0") \
  Y(7, "v_add3_u32", "v_add3_u32 %0, %0, %1, %0") \
  Y(8, "v_bfe_i32", "v_bfe_i32 %0, %1, 8, 8") \
  Y(9, "v_alignbyte_b32", "v_alignbyte_b32 %0, %0, %1, 1") \
  Y(10, "v_cndmask_b32_e32", "v_cndmask_b32_e32 %0, %0, %1, vcc") \
  Y(11, "v_mov_b32_e32", "v_mov_b32_e32 %0, %1") \
  Y(12, "v_ashrrev_i32_e32", "v_ashrrev_i32_e32 %0, 31, %0") \
  Y(13, "v_or_b32_e32", "v_or_b32_e32 %0, %0, %1") \
  Y(14, "v_sub_u32_e32", "v_sub_u32_e32 %0, %0, %1") \
  Y(15, "v_mul_lo_u32(v,v)", "v_mul_lo_u32 %0, %0, %1") \
  Y(16, "v_lshl_or_b32", "v_lshl_or_b32 %0, %0, 8, %1") \
  Y(17, "v_xor_b32_sdwa BYTE_0 sext", "v_xor_b32_sdwa %0, sext(%1), %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD") \
  Y(18, "v_xad_u32", "v_xad_u32 %0, %0, %1, %0") \
  Y(19, "v_pk_mul_lo_u16", "v_pk_mul_lo_u16 %0, %0, %1") \
  Y(20, "v_pk_add_u16", "v_pk_add_u16 %0, %0, %1") \
  Y(21, "v_lshrrev_b64", "v_lshrrev_b64 %0, 8, %0") \
  Y(22, "v_mad_u64_u32 + v_xor_e32 (pair)", "") \
  Y(23, "v_mad_u64_u32 + 2 v_xor_e32", "") \
  Y(24, "v_mul_lo + v_xor_e32", "v_mul_lo_u32 %0, %0, %1\n v_xor_b32_e32 %0, %0, %1") \
  Y(25, "v_lshlrev_b64 (pair)", "")

template <int OP>
__global__ __launch_bounds__(256) void kb(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b0 = a0 * 3, b1 = a1 * 3, b2 = a2 * 3, b3 = a3 * 3, b4 = a4 * 3, b5 = a5 * 3, b6 = a6 * 3, b7 = a7 * 3;
  uint64_t c0 = a0, c1 = a1, c2 = a2, c3 = a3, c4 = a4, c5 = a5, c6 = a6, c7 = a7;
  asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#define Y(id, name, str) if constexpr (OP == id && id != 22 && id != 23 && id != 21 && id != 25) { \
      _Pragma("unroll") for (int z = 0; z < 1; ++z) { \
      asm volatile(str : "+v"(a0) : "v"(b0)); asm volatile(str : "+v"(a1) : "v"(b1)); \
      asm volatile(str : "+v"(a2) : "v"(b2)); asm volatile(str : "+v"(a3) : "v"(b3)); \
      asm volatile(str : "+v"(a4) : "v"(b4)); asm volatile(str : "+v"(a5) : "v"(b5)); \
      asm volatile(str : "+v"(a6) : "v"(b6)); asm volatile(str : "+v"(a7) : "v"(b7)); } }
      OPS(Y)
#undef Y
      if constexpr (OP == 21) {
#define X(i) asm volatile("v_lshrrev_b64 %0, 8, %0" : "+v"(c##i));
        REP8(X)
#undef X
      }
      if constexpr (OP == 25) {
#define X(i) asm volatile("v_lshlrev_b64 %0, 8, %0" : "+v"(c##i));
        REP8(X)
#undef X
      }
      if constexpr (OP == 22) {
#define X(i) asm volatile("v_mad_u64_u32 %0, s[2:3], %1, %2, %0\n v_xor_b32_e32 %1, %1, %2" : "+v"(c##i), "+v"(a##i) : "v"(b##i) : "s2", "s3");
        REP8(X)
#undef X
      }
      if constexpr (OP == 23) {
#define X(i) asm volatile("v_mad_u64_u32 %0, s[2:3], %1, %2, %0\n v_xor_b32_e32 %1, %1, %2\n v_xor_b32_e32 %2, %2, %1" : "+v"(c##i), "+v"(a##i), "+v"(b##i) :: "s2", "s3");
        REP8(X)
#undef X
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ b0 ^ b1 ^ b2 ^ b3 ^ b4 ^ b5 ^ b6 ^ b7 ^
      (uint32_t)(c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7) ^ (uint32_t)((c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7) >> 32);
}

typedef void (*KFn)(uint32_t*, int, uint32_t);
template <int N> struct Tab { static void fill(KFn* t) { t[N] = kb<N>; Tab<N - 1>::fill(t); } };
template <> struct Tab<-1> { static void fill(KFn*) {} };

int main() {
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  const int threads = 256, blocks = prop.multiProcessorCount * 8;
  uint32_t* d; CHK(hipMalloc(&d, sizeof(uint32_t) * threads * blocks));
  const int iters = 2048; const double insts_per_lane = (double)iters * 16 * 8;
  const char* names[26];
#define Y(id, name, str) names[id] = name;
  OPS(Y)
#undef Y
  KFn tab[26]; Tab<25>::fill(tab);
  hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  for (int op = 0; op < 26; ++op) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(e0));
      tab[op]<<<blocks, threads>>>(d, iters, 1);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); if (rep && ms < best) best = ms;
    }
    double ns_per = best * 1e6 / (8.0 * insts_per_lane);  // per asm-statement group per SIMD
    printf("%-36s %7.3f ms  %6.3f ns/asm-stmt/SIMD (= %5.2f cyc @2.4GHz)\n", names[op], best, ns_per, ns_per * 2.4);
  }
  return 0;
}
