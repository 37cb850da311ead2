// How fast does the hand-scheduled FNV byte step issue at low occupancy?  The LDS-heavy
// long-key kernels run at 2 waves/SIMD; a single dependent chain per lane may not fill
// the SIMD there.  Measures ns per 16-byte chunk per wave per SIMD, register-resident
// data, at 1/2/4/8 waves per SIMD (occupancy forced by dynamic LDS), with one chain per
// lane (ILP 1) and two interleaved independent chains (ILP 2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

// chain A: state v48/v49, v50 = 0, t v51, x v52, m v53, smear v54
// chain B: state v64/v65, v66 = 0, t v67, x v68, m v69, smear v70
#define SA(W, K) \
  "v_xor_b32_sdwa v52, sext(" W "), v48 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K " src1_sel:DWORD\n\t"
#define SB(W, K) \
  "v_xor_b32_sdwa v68, sext(" W "), v64 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K " src1_sel:DWORD\n\t"
#define HA(K) "v_xor_b32_sdwa v49, sext(v54), v49 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K " src1_sel:DWORD\n\t"
#define HB(K) "v_xor_b32_sdwa v65, sext(v70), v65 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K " src1_sel:DWORD\n\t"
#define MA "v_mul_lo_u32 v53, v49, s26\n\t"
#define MB "v_mul_lo_u32 v69, v65, s26\n\t"
#define TA "v_lshl_add_u32 v51, v52, 8, v53\n\t"
#define TB "v_lshl_add_u32 v67, v68, 8, v69\n\t"
#define DA "v_mad_u64_u32 v[48:49], s[20:21], v52, s26, v[50:51]\n\t"
#define DB "v_mad_u64_u32 v[64:65], s[22:23], v68, s26, v[66:67]\n\t"
#define STEP1(W, K) SA(W, K) HA(K) MA TA DA
#define STEP2(WA, WB, K) SA(WA, K) SB(WB, K) HA(K) HB(K) MA MB TA TB DA DB
#define SMA(W) "v_perm_b32 v54, " W ", " W ", s25\n\t"
#define SMB(W) "v_perm_b32 v70, " W ", " W ", s25\n\t"
#define WORD1(W) SMA(W) STEP1(W, 0) STEP1(W, 1) STEP1(W, 2) STEP1(W, 3)
#define WORD2(WA, WB) SMA(WA) SMB(WB) STEP2(WA, WB, 0) STEP2(WA, WB, 1) STEP2(WA, WB, 2) STEP2(WA, WB, 3)
#define CHUNK1 WORD1("v40") WORD1("v41") WORD1("v42") WORD1("v43")
#define CHUNK2 WORD2("v40", "v56") WORD2("v41", "v57") WORD2("v42", "v58") WORD2("v43", "v59")
#define CLOB "v40", "v41", "v42", "v43", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v56", "v57", "v58", "v59", \
  "v64", "v65", "v66", "v67", "v68", "v69", "v70", "s20", "s21", "s22", "s23"

template <int ILP>
__global__ __launch_bounds__(256) void kc(uint32_t* out, int iters, uint32_t seed) {
  extern __shared__ uint32_t pad[];
  uint32_t r0, r1;
  asm volatile(
      "v_mov_b32 v40, %2\n\tv_add_u32 v41, 1, v40\n\tv_add_u32 v42, 2, v40\n\tv_add_u32 v43, 3, v40\n\t"
      "v_add_u32 v56, 5, v40\n\tv_add_u32 v57, 6, v40\n\tv_add_u32 v58, 7, v40\n\tv_add_u32 v59, 8, v40\n\t"
      "v_mov_b32 v48, 0\n\tv_mov_b32 v49, 0\n\tv_mov_b32 v50, 0\n\tv_mov_b32 v64, 0\n\tv_mov_b32 v65, 0\n\t"
      "v_mov_b32 v66, 0\n\t"
      "s_mov_b32 s24, %3\n\t"
      "s_mov_b32 s25, 0x090b080a\n\t"
      "s_movk_i32 s26, 0x1b3\n"
      "1:\n\t"
      ".if %4 == 1\n\t" CHUNK1 CHUNK1 ".else\n\t" CHUNK2 ".endif\n\t"
      "s_sub_u32 s24, s24, 1\n\t"
      "s_cmp_eq_u32 s24, 0\n\t"
      "s_cbranch_scc0 1b\n\t"
      "v_xor_b32 %0, v48, v64\n\t"
      "v_xor_b32 %1, v49, v65\n\t"
      : "=v"(r0), "=v"(r1)
      : "v"(threadIdx.x ^ seed), "s"(iters), "n"(ILP)
      : CLOB, "s24", "s25", "s26", "scc");
  if (r0 == 0x12345678u && r1 == 0x9abcdef0u) out[0] = pad[0];  // keep pad
  out[blockIdx.x * blockDim.x + threadIdx.x] = r0 ^ r1;
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CHK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
  uint32_t* out;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  CHK(hipFuncSetAttribute((const void*)kc<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHK(hipFuncSetAttribute((const void*)kc<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int iters = 4000;  // 2 chunks (ILP 1: one chain, 32 B; ILP 2: two chains, 16 B each) per iteration
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int warm = 0; warm < 20; ++warm) kc<1><<<cus * 4, 256, 40 * 1024>>>(out, iters, 1);
  CHK(hipDeviceSynchronize());
  for (int w : {1, 2, 3, 4, 6, 8}) {
    size_t lds = w >= 8 ? 0 : (size_t)(160 * 1024 / w) - 1024;
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)kc<1>, 256, lds));
    for (int ilp : {1, 2}) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        CHK(hipEventRecord(a));
        if (ilp == 1) kc<1><<<cus * w, 256, lds>>>(out, iters, rep);
        else kc<2><<<cus * w, 256, lds>>>(out, iters, rep);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
      }
      // per SIMD: w waves each doing iters*2 chunk-steps (ILP 2: 2 chains x 1 chunk per iter)
      double chunks = (double)iters * 2.0 * w;
      double ns_per_chunk = best * 1e6 / chunks;
      double bytes = (double)cus * 4 * w * 64 * iters * 32;  // key bytes hashed chip-wide
      printf("waves/SIMD %d (occ %d blk/CU) ILP %d: %7.3f ms  %6.2f ns/chunk/wave/SIMD  (%5.1f cyc@2.13GHz per chunk-op slot %.2f)  chip %.2f TB/s key bytes\n",
             w, occ, ilp, best, ns_per_chunk, ns_per_chunk * 2.13, ns_per_chunk * 2.13 / 86.0, bytes / (best * 1e-3) / 1e12);
    }
  }
  printf("EXIT 0\n");
  return 0;
}
