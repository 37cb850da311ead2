// k2hash_amd -- device-side FNV-1a primitives for gfx950 (CDNA4).
//
// The reference hot loop (lib/k2hashfunc.cc:49-59) is, per key byte b,
//     h ^= (uint64_t)(int64_t)(signed char)b;   // sign-extended (lib/k2hashfunc.cc:53,55)
//     h *= 0x100000001b3;                        // 1099511628211 (lib/k2hashfunc.cc:56)
// with h seeded by 14695981039346656037 (lib/k2hashfunc.cc:51).
//
// On CDNA4 the 64-bit state lives in two VGPRs (lo, hi) and, with P = 2^40 + 435,
//     x_lo = lo ^ sext32(b)          x_hi = hi ^ sign(b)   (sign(b) = 0 or 0xffffffff)
//     h'   = x * P = x_lo*435 + ((x_hi*435 + (x_lo << 8)) << 32)
// which is five VALU ops per byte:
//     v_xor_b32_sdwa  x_lo, sext(w.BYTE_k), lo
//     v_xor_b32_sdwa  hi,   sext(u.BYTE_k), hi      u = per-byte sign smear of w (v_perm_b32)
//     v_mul_lo_u32    m, hi, 435
//     v_lshl_add_u32  t, x_lo, 8, m                  written into the odd half of a {0, t} pair
//     v_mad_u64_u32   {lo,hi}, x_lo, 435, {0, t}
// plus two ops per 4-byte word for the sign smear.  Measured on MI355X
// (tools/valu_rates*.hip, profiles/r01_valu_rates.txt) every one of these issues in
// ~4.2 cycles per wave64 per SIMD, so the mix is 5.5 slow-issue ops per byte.  hipcc's
// own lowering of the byte loop spends 6.5 (it materialises x_lo << 8 and uses v_add3).
//
// The {0, t} pair needs two adjacent physical VGPRs with the low one held at zero, which
// the compiler cannot be asked for through operand constraints, so the byte steps are
// written as one asm statement per 16-byte chunk over a fixed register window (v[48:55]
// below, declared as clobbers so the allocator keeps out).  The kernel stays under 64
// VGPRs, i.e. 8 waves/SIMD.  A portable C++ formulation (fnv_step_c) is kept for the
// tails and as an A/B variant.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace k2h {

constexpr uint64_t kSeedBuiltin = 14695981039346656037ULL;  // lib/k2hashfunc.cc:51
constexpr uint64_t kSeedStd = 2166136261ULL;                  // libstdc++ _Fnv_hash_impl default
constexpr uint32_t kPrimeLo = 0x1b3u;                         // 1099511628211 = 2^40 + 0x1b3
constexpr uint32_t kSmearSel = 0x090B080Au;                   // v_perm selector, see smear()

// Per-byte sign smear: byte k of the result is 0xff if byte k of w is >= 0x80, else 0.
// v_perm_b32 selectors 8..11 replicate the sign of bytes 1,3,5,7 of {src0:src1}; with
// src1 = w, src0 = w << 8 those are w.b1, w.b3, w.b0, w.b2.
__device__ __forceinline__ uint32_t smear(uint32_t w) {
  return __builtin_amdgcn_perm(w << 8, w, kSmearSel);
}

// Portable one-byte step on the split state (compiler-scheduled).
__device__ __forceinline__ void fnv_step_c(uint32_t& lo, uint32_t& hi, uint32_t byte) {
  int32_t sb = (int32_t)(int8_t)byte;
  uint32_t xlo = lo ^ (uint32_t)sb;
  uint32_t xhi = hi ^ (uint32_t)(sb >> 31);
  uint32_t t = xhi * kPrimeLo + (xlo << 8);
  uint64_t r = (uint64_t)xlo * kPrimeLo + ((uint64_t)t << 32);
  lo = (uint32_t)r;
  hi = (uint32_t)(r >> 32);
}

__device__ __forceinline__ void fnv_word_c(uint32_t& lo, uint32_t& hi, uint32_t w) {
  uint32_t u = smear(w);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int32_t sb = (int32_t)(int8_t)(w >> (8 * k));
    int32_t sm = (int32_t)(int8_t)(u >> (8 * k));
    uint32_t xlo = lo ^ (uint32_t)sb;
    uint32_t xhi = hi ^ (uint32_t)sm;
    uint32_t t = xhi * kPrimeLo + (xlo << 8);
    uint64_t r = (uint64_t)xlo * kPrimeLo + ((uint64_t)t << 32);
    lo = (uint32_t)r;
    hi = (uint32_t)(r >> 32);
  }
}

// ---------------------------------------------------------------------------
// Hand-scheduled chunk steps.  Register window (clobbered):
//   v48 lo, v49 hi   state pair (mad64 destination)
//   v50 = 0, v51 = t the {0, t} addend pair
//   v52 x_lo, v53 m, v54 u (sign smear), v55 w << 8
// ---------------------------------------------------------------------------
#define K2H_ASM_STEP(W, K)                                                                         \
  "v_xor_b32_sdwa v52, sext(%[" #W "]), v48 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K \
  " src1_sel:DWORD\n\t"                                                                            \
  "v_xor_b32_sdwa v49, sext(v54), v49 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K        \
  " src1_sel:DWORD\n\t"                                                                            \
  "v_mul_lo_u32 v53, v49, %[p]\n\t"                                                                \
  "v_lshl_add_u32 v51, v52, 8, v53\n\t"                                                            \
  "v_mad_u64_u32 v[48:49], vcc, v52, %[p], v[50:51]\n\t"

#define K2H_ASM_SMEAR(W)                \
  "v_lshlrev_b32 v55, 8, %[" #W "]\n\t" \
  "v_perm_b32 v54, v55, %[" #W "], %[sel]\n\t"

#define K2H_ASM_WORD(W) K2H_ASM_SMEAR(W) K2H_ASM_STEP(W, 0) K2H_ASM_STEP(W, 1) K2H_ASM_STEP(W, 2) K2H_ASM_STEP(W, 3)

#define K2H_ASM_BEGIN "v_mov_b32 v48, %[lo]\n\tv_mov_b32 v49, %[hi]\n\tv_mov_b32 v50, 0\n\t"
#define K2H_ASM_END "v_mov_b32 %[lo], v48\n\tv_mov_b32 %[hi], v49\n\t"
#define K2H_ASM_SNAP "v_mov_b32 %[lo2], v48\n\tv_mov_b32 %[hi2], v49\n\t"
#define K2H_ASM_CLOBBERS "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "vcc"

#define K2H_X_STEP(W, U, K)                                                                            \
  "v_xor_b32_sdwa v52, sext(" W "), v48 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K         \
  " src1_sel:DWORD\n\t"                                                                                \
  "v_xor_b32_sdwa v49, sext(" U "), v49 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_" #K          \
  " src1_sel:DWORD\n\t"                                                                                \
  "v_mul_lo_u32 v53, v49, %[p]\n\t"                                                                    \
  "v_lshl_add_u32 v51, v52, 8, v53\n\t"                                                                \
  "v_mad_u64_u32 v[48:49], vcc, v52, %[p], v[50:51]\n\t"
#define K2H_X_WORD(W, U) K2H_X_STEP(W, U, 0) K2H_X_STEP(W, U, 1) K2H_X_STEP(W, U, 2) K2H_X_STEP(W, U, 3)
#define K2H_X_SMEAR2(LO, HI, PAIR)                 \
  "v_lshlrev_b64 v[56:57], 8, " PAIR "\n\t"        \
  "v_perm_b32 v54, v56, " LO ", %[sel]\n\t"        \
  "v_perm_b32 v58, v57, " HI ", %[sel]\n\t"
#define K2H_X_PAIR(LO, HI, PAIR) K2H_X_SMEAR2(LO, HI, PAIR) K2H_X_WORD(LO, "v54") K2H_X_WORD(HI, "v58")
#define K2H_X_PAIR_LAST(LO, HI, PAIR)                                                                      \
  K2H_X_SMEAR2(LO, HI, PAIR) K2H_X_WORD(LO, "v54") K2H_X_STEP(HI, "v58", 0) K2H_X_STEP(HI, "v58", 1)        \
      K2H_X_STEP(HI, "v58", 2) "v_mov_b32 v60, v48\n\tv_mov_b32 v61, v49\n\t" K2H_X_STEP(HI, "v58", 3)

// The chunk helpers bind the state to v48/v49, the zero half of the addend pair to v50
// and the chunk words to v[40:43] (v[44:47] for the second chunk) through physical-
// register operand constraints ("{vN}"), so the allocator keeps the state in place from
// one statement to the next (no copies in or out of the window) and the words sit in
// adjacent pairs for the 64-bit-shift sign smear (K2H_X_SMEAR2 below).
#define K2H_P_PAIR(LO, HI, PAIR) K2H_X_PAIR(LO, HI, PAIR)
#define K2H_P_CLOBBERS "v51", "v52", "v53", "v54", "v56", "v57", "v58", "vcc", "memory"

// 16 bytes (one uint4 chunk) into the state; BANK 1 takes the chunk in v[44:47]
// instead of v[40:43], so a loop that alternates banks (ping-pong) needs no copies.
template <int BANK = 0>
__device__ __forceinline__ void fnv_chunk16(uint32_t& lo, uint32_t& hi, uint4 c) {
  if constexpr (BANK == 0) {
    asm(K2H_P_PAIR("v40", "v41", "v[40:41]") K2H_P_PAIR("v42", "v43", "v[42:43]")
        : "+{v48}"(lo), "+{v49}"(hi)
        : "{v40}"(c.x), "{v41}"(c.y), "{v42}"(c.z), "{v43}"(c.w), "{v50}"(0u), [p] "s"(kPrimeLo),
          [sel] "s"(kSmearSel)
        : K2H_P_CLOBBERS);
  } else {
    asm(K2H_P_PAIR("v44", "v45", "v[44:45]") K2H_P_PAIR("v46", "v47", "v[46:47]")
        : "+{v48}"(lo), "+{v49}"(hi)
        : "{v44}"(c.x), "{v45}"(c.y), "{v46}"(c.z), "{v47}"(c.w), "{v50}"(0u), [p] "s"(kPrimeLo),
          [sel] "s"(kSmearSel)
        : K2H_P_CLOBBERS);
  }
}

// Same, with the zero half of the mad64 addend pair passed in and out (z == 0 is never
// changed): kept in v50 across a loop of statements instead of re-materialised per chunk.
template <int BANK = 0>
__device__ __forceinline__ void fnv_chunk16z(uint32_t& lo, uint32_t& hi, uint4 c, uint32_t& z) {
  if constexpr (BANK == 0) {
    asm(K2H_P_PAIR("v40", "v41", "v[40:41]") K2H_P_PAIR("v42", "v43", "v[42:43]")
        : "+{v48}"(lo), "+{v49}"(hi), "+{v50}"(z)
        : "{v40}"(c.x), "{v41}"(c.y), "{v42}"(c.z), "{v43}"(c.w), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
        : K2H_P_CLOBBERS);
  } else {
    asm(K2H_P_PAIR("v44", "v45", "v[44:45]") K2H_P_PAIR("v46", "v47", "v[46:47]")
        : "+{v48}"(lo), "+{v49}"(hi), "+{v50}"(z)
        : "{v44}"(c.x), "{v45}"(c.y), "{v46}"(c.z), "{v47}"(c.w), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
        : K2H_P_CLOBBERS);
  }
}

// A chunk loop whose chunk registers stay in the asm banks: step<BANK> hashes the chunk
// held in bank BANK (v[40:43] or v[44:47]) while it issues the LDS read of the next
// chunk into the other bank (`next`, a 32-bit LDS address).  The read is in the asm, so
// the compiler neither waits for it nor copies it: the s_waitcnt lgkmcnt(1) inside waits
// only for the read the previous step issued into this step's bank.
template <int BANK>
__device__ __forceinline__ void fnv_step_read(uint32_t& lo, uint32_t& hi, uint4& a, uint4& b, uint32_t next) {
  if constexpr (BANK == 0) {
    asm volatile("ds_read_b128 v[44:47], %[nx]\n\ts_waitcnt lgkmcnt(1)\n\t" K2H_P_PAIR("v40", "v41", "v[40:41]")
                     K2H_P_PAIR("v42", "v43", "v[42:43]")
                 : "+{v48}"(lo), "+{v49}"(hi), "+{v40}"(a.x), "+{v41}"(a.y), "+{v42}"(a.z), "+{v43}"(a.w),
                   "+{v44}"(b.x), "+{v45}"(b.y), "+{v46}"(b.z), "+{v47}"(b.w)
                 : [nx] "v"(next), "{v50}"(0u), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
                 : K2H_P_CLOBBERS);
  } else {
    asm volatile("ds_read_b128 v[40:43], %[nx]\n\ts_waitcnt lgkmcnt(1)\n\t" K2H_P_PAIR("v44", "v45", "v[44:45]")
                     K2H_P_PAIR("v46", "v47", "v[46:47]")
                 : "+{v48}"(lo), "+{v49}"(hi), "+{v40}"(a.x), "+{v41}"(a.y), "+{v42}"(a.z), "+{v43}"(a.w),
                   "+{v44}"(b.x), "+{v45}"(b.y), "+{v46}"(b.z), "+{v47}"(b.w)
                 : [nx] "v"(next), "{v50}"(0u), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
                 : K2H_P_CLOBBERS);
  }
}

// Pin a chunk into bank 0 (before a step loop; waits for the value like any use).
__device__ __forceinline__ void fnv_bank0_pin(uint4& a) {
  asm volatile("" : "+{v40}"(a.x), "+{v41}"(a.y), "+{v42}"(a.z), "+{v43}"(a.w));
}

// After a step loop: the key's last chunk is in bank 0, or in bank 1 when `from1` (this
// lane's loop ended on a bank-0 step); hash it as the last chunk (second-hash snapshot).
__device__ __forceinline__ void fnv_step_last(uint32_t& lo, uint32_t& hi, uint32_t& lo2, uint32_t& hi2, uint4& a,
                                              uint4& b, bool from1) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (from1)
    asm volatile("v_mov_b32 v40, v44\n\tv_mov_b32 v41, v45\n\tv_mov_b32 v42, v46\n\tv_mov_b32 v43, v47"
                 : "+{v40}"(a.x), "+{v41}"(a.y), "+{v42}"(a.z), "+{v43}"(a.w)
                 : "{v44}"(b.x), "{v45}"(b.y), "{v46}"(b.z), "{v47}"(b.w));
  asm volatile(K2H_P_PAIR("v40", "v41", "v[40:41]") K2H_X_PAIR_LAST("v42", "v43", "v[42:43]")
               : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2), "+{v40}"(a.x), "+{v41}"(a.y),
                 "+{v42}"(a.z), "+{v43}"(a.w)
               : "{v50}"(0u), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
               : K2H_P_CLOBBERS);
}

// 32 bytes (two chunks), one statement.
__device__ __forceinline__ void fnv_chunk32(uint32_t& lo, uint32_t& hi, uint4 a, uint4 b) {
  asm(K2H_P_PAIR("v40", "v41", "v[40:41]") K2H_P_PAIR("v42", "v43", "v[42:43]")
          K2H_P_PAIR("v44", "v45", "v[44:45]") K2H_P_PAIR("v46", "v47", "v[46:47]")
      : "+{v48}"(lo), "+{v49}"(hi)
      : "{v40}"(a.x), "{v41}"(a.y), "{v42}"(a.z), "{v43}"(a.w), "{v44}"(b.x), "{v45}"(b.y), "{v46}"(b.z),
        "{v47}"(b.w), "{v50}"(0u), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
      : K2H_P_CLOBBERS);
}

// Last 16-byte chunk of a key: also returns the state before the final byte
// (the reference's second hash, lib/k2hashfunc.cc:83-85).
__device__ __forceinline__ void fnv_chunk16_last(uint32_t& lo, uint32_t& hi, uint32_t& lo2, uint32_t& hi2, uint4 c) {
  asm(K2H_P_PAIR("v40", "v41", "v[40:41]") K2H_X_PAIR_LAST("v42", "v43", "v[42:43]")
      : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2)
      : "{v40}"(c.x), "{v41}"(c.y), "{v42}"(c.z), "{v43}"(c.w), "{v50}"(0u), [p] "s"(kPrimeLo),
        [sel] "s"(kSmearSel)
      : K2H_P_CLOBBERS);
}

__device__ __forceinline__ void fnv_chunk16_lastz(uint32_t& lo, uint32_t& hi, uint32_t& lo2, uint32_t& hi2, uint4 c,
                                                  uint32_t& z) {
  asm(K2H_P_PAIR("v40", "v41", "v[40:41]") K2H_X_PAIR_LAST("v42", "v43", "v[42:43]")
      : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2), "+{v50}"(z)
      : "{v40}"(c.x), "{v41}"(c.y), "{v42}"(c.z), "{v43}"(c.w), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
      : K2H_P_CLOBBERS);
}

__device__ __forceinline__ void fnv_chunk32_last(uint32_t& lo, uint32_t& hi, uint32_t& lo2, uint32_t& hi2, uint4 a,
                                                 uint4 b) {
  asm(K2H_P_PAIR("v40", "v41", "v[40:41]") K2H_P_PAIR("v42", "v43", "v[42:43]")
          K2H_P_PAIR("v44", "v45", "v[44:45]") K2H_X_PAIR_LAST("v46", "v47", "v[46:47]")
      : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2)
      : "{v40}"(a.x), "{v41}"(a.y), "{v42}"(a.z), "{v43}"(a.w), "{v44}"(b.x), "{v45}"(b.y), "{v46}"(b.z),
        "{v47}"(b.w), "{v50}"(0u), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
      : K2H_P_CLOBBERS);
}

}  // namespace k2h

// ---------------------------------------------------------------------------
// Whole-key statement for 32-byte keys (fixed32 fast path): the two 16-byte loads, all
// 32 byte steps and the store in ONE asm statement over explicit registers, so that
//  - each pair of words gets its sign smear from one 64-bit shift + two v_perm_b32
//    (3 slow-issue ops per 8 bytes instead of 4), which needs the words in adjacent
//    registers -- something operand constraints cannot express;
//  - no moves in or out of the register window.
// Register window: v[40:47] key words, v48/v49 state, v50 = 0, v51 t, v52 x_lo,
// v53 m, v54/v58 smears, v[56:57] shifted pair, v[60:61] second-hash snapshot.
// ---------------------------------------------------------------------------
namespace k2h {

#define K2H_X_HEAD                                                     \
  "global_load_dwordx4 v[40:43], %[src], off nt\n\t"                   \
  "global_load_dwordx4 v[44:47], %[src], off offset:16 nt\n\t"         \
  "v_mov_b32 v48, %[slo]\n\t"                                          \
  "v_mov_b32 v49, %[shi]\n\t"                                          \
  "v_mov_b32 v50, 0\n\t"                                               \
  "s_waitcnt vmcnt(0)\n\t"
#define K2H_X_BODY                                                                                      \
  K2H_X_PAIR("v40", "v41", "v[40:41]") K2H_X_PAIR("v42", "v43", "v[42:43]") K2H_X_PAIR("v44", "v45", "v[44:45]")
#define K2H_X_CLOBBERS                                                                                   \
  "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", \
      "v55", "v56", "v57", "v58", "v59", "v60", "v61", "vcc", "memory"

// h1 only
__device__ __forceinline__ void fnv_key32_x(const void* src, uint64_t* dst1, uint64_t seed) {
  asm volatile(K2H_X_HEAD K2H_X_BODY K2H_X_PAIR("v46", "v47", "v[46:47]")
               "global_store_dwordx2 %[d1], v[48:49], off nt\n\t"
               "s_nop 1\n\t"
               :
               : [src] "v"(src), [d1] "v"(dst1), [slo] "s"((uint32_t)seed), [shi] "s"((uint32_t)(seed >> 32)),
                 [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
               : K2H_X_CLOBBERS);
}

// h1 + h2
__device__ __forceinline__ void fnv_key32_x2(const void* src, uint64_t* dst1, uint64_t* dst2, uint64_t seed) {
  asm volatile(K2H_X_HEAD K2H_X_BODY K2H_X_PAIR_LAST("v46", "v47", "v[46:47]")
               "global_store_dwordx2 %[d1], v[48:49], off nt\n\t"
               "global_store_dwordx2 %[d2], v[60:61], off nt\n\t"
               "s_nop 1\n\t"
               :
               : [src] "v"(src), [d1] "v"(dst1), [d2] "v"(dst2), [slo] "s"((uint32_t)seed),
                 [shi] "s"((uint32_t)(seed >> 32)), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
               : K2H_X_CLOBBERS);
}

// Two 32-byte keys per lane, h1 only, as ONE statement: the four nt loads issued together
// (key 0 into v[40:47], key 1 into v[32:39]), key 0 hashed as soon as ITS two loads have
// landed (vmcnt(2): loads return in order) while key 1's are still in flight, key 1 hashed
// in place (no copies into the window), both hashes stored at the end.  hipcc, given the
// loads as code, waited for all four before the first hash (vmcnt(0)).
#define K2H_X_KEY1 \
  K2H_X_PAIR("v32", "v33", "v[32:33]") K2H_X_PAIR("v34", "v35", "v[34:35]") K2H_X_PAIR("v36", "v37", "v[36:37]") \
      K2H_X_PAIR("v38", "v39", "v[38:39]")
__device__ __forceinline__ void fnv_key32_pair_x(const void* src0, const void* src1, uint64_t* dst0, uint64_t* dst1,
                                                 uint64_t seed) {
  asm volatile("global_load_dwordx4 v[40:43], %[s0], off nt\n\t"
               "global_load_dwordx4 v[44:47], %[s0], off offset:16 nt\n\t"
               "global_load_dwordx4 v[32:35], %[s1], off nt\n\t"
               "global_load_dwordx4 v[36:39], %[s1], off offset:16 nt\n\t"
               "v_mov_b32 v48, %[slo]\n\t"
               "v_mov_b32 v49, %[shi]\n\t"
               "v_mov_b32 v50, 0\n\t"
               "s_waitcnt vmcnt(2)\n\t" K2H_X_BODY K2H_X_PAIR("v46", "v47", "v[46:47]")
               "v_mov_b32 v62, v48\n\t"
               "v_mov_b32 v63, v49\n\t"
               "v_mov_b32 v48, %[slo]\n\t"
               "v_mov_b32 v49, %[shi]\n\t"
               "s_waitcnt vmcnt(0)\n\t" K2H_X_KEY1
               "global_store_dwordx2 %[d0], v[62:63], off nt\n\t"
               "global_store_dwordx2 %[d1], v[48:49], off nt\n\t"
               "s_nop 1\n\t"
               :
               : [s0] "v"(src0), [s1] "v"(src1), [d0] "v"(dst0), [d1] "v"(dst1), [slo] "s"((uint32_t)seed),
                 [shi] "s"((uint32_t)(seed >> 32)), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
               : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", K2H_X_CLOBBERS, "v62", "v63");
}

// The same two-key statement with the hashes returned in registers (stored by the caller,
// e.g. with the fused bucket-index epilogue); H2 also returns each key's second hash (the
// state before its last byte: key 0's parked in v55/v59 while key 1 is hashed).
#define K2H_X_KEY1_LAST \
  K2H_X_PAIR("v32", "v33", "v[32:33]") K2H_X_PAIR("v34", "v35", "v[34:35]") K2H_X_PAIR("v36", "v37", "v[36:37]") \
      K2H_X_PAIR_LAST("v38", "v39", "v[38:39]")
#define K2H_PAIR_HEAD                                   \
  "global_load_dwordx4 v[40:43], %[s0], off nt\n\t"          \
  "global_load_dwordx4 v[44:47], %[s0], off offset:16 nt\n\t" \
  "global_load_dwordx4 v[32:35], %[s1], off nt\n\t"          \
  "global_load_dwordx4 v[36:39], %[s1], off offset:16 nt\n\t" \
  "v_mov_b32 v48, %[slo]\n\t"                                 \
  "v_mov_b32 v49, %[shi]\n\t"                                 \
  "v_mov_b32 v50, 0\n\t"                                      \
  "s_waitcnt vmcnt(2)\n\t"
#define K2H_PAIR_INPUTS                                                                                     \
  [s0] "v"(src0), [s1] "v"(src1), [slo] "s"((uint32_t)seed), [shi] "s"((uint32_t)(seed >> 32)), [p] "s"(kPrimeLo), \
      [sel] "s"(kSmearSel)
template <bool H2>
__device__ __forceinline__ void fnv_key32_pair_r(const void* src0, const void* src1, uint64_t seed, uint64_t& r0,
                                                 uint64_t& r1, uint64_t& s0, uint64_t& s1) {
  uint32_t a0, a1, b0, b1;
  if constexpr (!H2) {
    asm volatile(K2H_PAIR_HEAD K2H_X_BODY K2H_X_PAIR("v46", "v47", "v[46:47]")
                 "v_mov_b32 v62, v48\n\t"
                 "v_mov_b32 v63, v49\n\t"
                 "v_mov_b32 v48, %[slo]\n\t"
                 "v_mov_b32 v49, %[shi]\n\t"
                 "s_waitcnt vmcnt(0)\n\t" K2H_X_KEY1
                 : "={v62}"(a0), "={v63}"(a1), "={v48}"(b0), "={v49}"(b1)
                 : K2H_PAIR_INPUTS
                 : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
                   "v46", "v47", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61",
                   "vcc", "memory");
    s0 = s1 = 0;
  } else {
    uint32_t c0, c1, d0, d1;
    asm volatile(K2H_PAIR_HEAD K2H_X_BODY K2H_X_PAIR_LAST("v46", "v47", "v[46:47]")
                 "v_mov_b32 v62, v48\n\t"
                 "v_mov_b32 v63, v49\n\t"
                 "v_mov_b32 v55, v60\n\t"
                 "v_mov_b32 v59, v61\n\t"
                 "v_mov_b32 v48, %[slo]\n\t"
                 "v_mov_b32 v49, %[shi]\n\t"
                 "s_waitcnt vmcnt(0)\n\t" K2H_X_KEY1_LAST
                 : "={v62}"(a0), "={v63}"(a1), "={v48}"(b0), "={v49}"(b1), "={v55}"(c0), "={v59}"(c1),
                   "={v60}"(d0), "={v61}"(d1)
                 : K2H_PAIR_INPUTS
                 : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45",
                   "v46", "v47", "v50", "v51", "v52", "v53", "v54", "v56", "v57", "v58", "vcc", "memory");
    s0 = ((uint64_t)c1 << 32) | c0;
    s1 = ((uint64_t)d1 << 32) | d0;
  }
  r0 = ((uint64_t)a1 << 32) | a0;
  r1 = ((uint64_t)b1 << 32) | b0;
}

}  // namespace k2h

// ---------------------------------------------------------------------------
// Wave-uniform run over chunks staged in LDS: hashes `cnt` (>= 1, the same in every
// lane) consecutive chunks -- the one already in `c`, then cnt-1 read from LDS at
// `lds` (byte address of the chunk after `c`) -- as ONE asm statement: the state stays
// in v48/v49, chunks alternate between v[40:43] and v[44:47] (no copies), the next
// chunk's ds_read_b128 is in flight under the current chunk's steps, and each pair of
// words takes its sign smear from one 64-bit shift + two v_perm_b32.  On return `c`
// holds the chunk that follows the run (read from LDS, not hashed).
// ---------------------------------------------------------------------------
namespace k2h {

#define K2H_X_CHUNK_A K2H_X_PAIR("v40", "v41", "v[40:41]") K2H_X_PAIR("v42", "v43", "v[42:43]")
#define K2H_X_CHUNK_B K2H_X_PAIR("v44", "v45", "v[44:45]") K2H_X_PAIR("v46", "v47", "v[46:47]")

__device__ __forceinline__ void fnv_lds_run(uint32_t& lo, uint32_t& hi, uint4& c, uint32_t lds, uint32_t cnt) {
  asm volatile(
      "v_mov_b32 v48, %[lo]\n\t"
      "v_mov_b32 v49, %[hi]\n\t"
      "v_mov_b32 v50, 0\n\t"
      "v_mov_b32 v40, %[c0]\n\t"
      "v_mov_b32 v41, %[c1]\n\t"
      "v_mov_b32 v42, %[c2]\n\t"
      "v_mov_b32 v43, %[c3]\n\t"
      "v_mov_b32 v62, %[lds]\n\t"
      "s_waitcnt lgkmcnt(0)\n"
      "k2h_run_loop_%=:\n\t"
      "ds_read_b128 v[44:47], v62\n\t" K2H_X_CHUNK_A
      "s_sub_u32 %[cnt], %[cnt], 1\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_cmp_eq_u32 %[cnt], 0\n\t"
      "s_cbranch_scc1 k2h_run_exit_b_%=\n\t"
      "ds_read_b128 v[40:43], v62 offset:16\n\t" K2H_X_CHUNK_B
      "v_add_u32_e32 v62, 32, v62\n\t"
      "s_sub_u32 %[cnt], %[cnt], 1\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_cmp_eq_u32 %[cnt], 0\n\t"
      "s_cbranch_scc0 k2h_run_loop_%=\n\t"
      "v_mov_b32 %[c0], v40\n\t"
      "v_mov_b32 %[c1], v41\n\t"
      "v_mov_b32 %[c2], v42\n\t"
      "v_mov_b32 %[c3], v43\n\t"
      "s_branch k2h_run_end_%=\n"
      "k2h_run_exit_b_%=:\n\t"
      "v_mov_b32 %[c0], v44\n\t"
      "v_mov_b32 %[c1], v45\n\t"
      "v_mov_b32 %[c2], v46\n\t"
      "v_mov_b32 %[c3], v47\n"
      "k2h_run_end_%=:\n\t"
      "v_mov_b32 %[lo], v48\n\t"
      "v_mov_b32 %[hi], v49\n\t"
      : [lo] "+v"(lo), [hi] "+v"(hi), [c0] "+v"(c.x), [c1] "+v"(c.y), [c2] "+v"(c.z), [c3] "+v"(c.w),
        [cnt] "+s"(cnt)
      : [lds] "v"(lds), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
      : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54",
        "v55", "v56", "v57", "v58", "v62", "vcc", "scc", "memory");
}

}  // namespace k2h

// ---------------------------------------------------------------------------
// Eight 16-byte chunks read from LDS at per-lane addresses a[0..7] (one line of a key),
// hashed in order as ONE asm statement: reads alternate between v[40:43] and v[44:47],
// the next chunk's ds_read_b128 is in flight under the current chunk's steps, and the
// lgkmcnt waits are explicit -- the compiler's own wait insertion would otherwise
// treat every LDS read as aliasing the LDS-DMA loads still in flight and drain them
// all (s_waitcnt vmcnt(0)) before the first read.  LAST: the eighth chunk is the key's
// final one and its pre-final-byte state (the second hash) is returned in lo2/hi2.
// ---------------------------------------------------------------------------
namespace k2h {

#define K2H_R8_BODY(LASTCHUNK)                                               \
  "ds_read_b128 v[40:43], %[a0]\n\t"                                         \
  "ds_read_b128 v[44:47], %[a1]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "ds_read_b128 v[40:43], %[a2]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_B                                   \
  "ds_read_b128 v[44:47], %[a3]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "ds_read_b128 v[40:43], %[a4]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_B                                   \
  "ds_read_b128 v[44:47], %[a5]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "ds_read_b128 v[40:43], %[a6]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_B                                   \
  "ds_read_b128 v[44:47], %[a7]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "s_waitcnt lgkmcnt(0)\n\t" LASTCHUNK

#define K2H_R8_INPUTS                                                                                        \
  [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [a4] "v"(a[4]), [a5] "v"(a[5]),              \
      [a6] "v"(a[6]), [a7] "v"(a[7]), "{v50}"(0u), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)
#define K2H_R8_CLOBBERS                                                                                      \
  "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v51", "v52", "v53", "v54", "v56", "v57", "v58", "vcc", \
      "memory"

#define K2H_R4_BODY(LASTCHUNK)                                               \
  "ds_read_b128 v[40:43], %[a0]\n\t"                                         \
  "ds_read_b128 v[44:47], %[a1]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "ds_read_b128 v[40:43], %[a2]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_B                                   \
  "ds_read_b128 v[44:47], %[a3]\n\t"                                         \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "s_waitcnt lgkmcnt(0)\n\t" LASTCHUNK
#define K2H_R4_INPUTS                                                                                        \
  [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), "{v50}"(0u), [p] "s"(kPrimeLo),             \
      [sel] "s"(kSmearSel)
#define K2H_LAST_B K2H_X_PAIR("v44", "v45", "v[44:45]") K2H_X_PAIR_LAST("v46", "v47", "v[46:47]")

// NP = 8 or 4 chunks per round (a full 128-byte line, or half of one).
template <int NP>
__device__ __forceinline__ void fnv_lds_round(uint32_t& lo, uint32_t& hi, const uint32_t (&a)[NP]);

// NP = 16 (two lines per round): two eight-chunk statements.
__device__ __forceinline__ void fnv_lds_round16(uint32_t& lo, uint32_t& hi, const uint32_t (&a16)[16], bool last,
                                                uint32_t& lo2, uint32_t& hi2) {
  {
    const uint32_t(&a)[8] = *reinterpret_cast<const uint32_t(*)[8]>(&a16[0]);
    asm volatile(K2H_R8_BODY(K2H_X_CHUNK_B) : "+{v48}"(lo), "+{v49}"(hi) : K2H_R8_INPUTS : K2H_R8_CLOBBERS);
  }
  const uint32_t(&a)[8] = *reinterpret_cast<const uint32_t(*)[8]>(&a16[8]);
  if (!last) {
    asm volatile(K2H_R8_BODY(K2H_X_CHUNK_B) : "+{v48}"(lo), "+{v49}"(hi) : K2H_R8_INPUTS : K2H_R8_CLOBBERS);
  } else {
    asm volatile(K2H_R8_BODY(K2H_LAST_B)
                 : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2)
                 : K2H_R8_INPUTS
                 : K2H_R8_CLOBBERS);
  }
}

template <int NP>
__device__ __forceinline__ void fnv_lds_round(uint32_t& lo, uint32_t& hi, const uint32_t (&a)[NP]) {
  if constexpr (NP == 16) {
    uint32_t d0, d1;
    fnv_lds_round16(lo, hi, a, false, d0, d1);
  } else if constexpr (NP == 8)
    asm volatile(K2H_R8_BODY(K2H_X_CHUNK_B) : "+{v48}"(lo), "+{v49}"(hi) : K2H_R8_INPUTS : K2H_R8_CLOBBERS);
  else
    asm volatile(K2H_R4_BODY(K2H_X_CHUNK_B) : "+{v48}"(lo), "+{v49}"(hi) : K2H_R4_INPUTS : K2H_R8_CLOBBERS);
}

template <int NP>
__device__ __forceinline__ void fnv_lds_round_last(uint32_t& lo, uint32_t& hi, uint32_t& lo2, uint32_t& hi2,
                                                   const uint32_t (&a)[NP]) {
  if constexpr (NP == 16)
    fnv_lds_round16(lo, hi, a, true, lo2, hi2);
  else if constexpr (NP == 8)
    asm volatile(K2H_R8_BODY(K2H_LAST_B)
                 : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2)
                 : K2H_R8_INPUTS
                 : K2H_R8_CLOBBERS);
  else
    asm volatile(K2H_R4_BODY(K2H_LAST_B)
                 : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2)
                 : K2H_R4_INPUTS
                 : K2H_R8_CLOBBERS);
}

__device__ __forceinline__ void fnv_lds_round8(uint32_t& lo, uint32_t& hi, const uint32_t (&a)[8]) {
  asm volatile(K2H_R8_BODY(K2H_X_CHUNK_B) : "+{v48}"(lo), "+{v49}"(hi) : K2H_R8_INPUTS : K2H_R8_CLOBBERS);
}

__device__ __forceinline__ void fnv_lds_round8_last(uint32_t& lo, uint32_t& hi, uint32_t& lo2, uint32_t& hi2,
                                                    const uint32_t (&a)[8]) {
  asm volatile(K2H_R8_BODY(K2H_X_PAIR("v44", "v45", "v[44:45]") K2H_X_PAIR_LAST("v46", "v47", "v[46:47]"))
               : "+{v48}"(lo), "+{v49}"(hi), "={v60}"(lo2), "={v61}"(hi2)
               : K2H_R8_INPUTS
               : K2H_R8_CLOBBERS);
}

// The same eight-chunk round with the LDS slot as the ds_read immediate offset O (the
// per-lane addresses a[] stay fixed across rounds: no address VALU per round) and the
// zero half of the mad64 addend pair carried in v50 by the caller (z, always 0; not
// re-materialised per statement).
#define K2H_R8O_BODY(LASTCHUNK)                                              \
  "ds_read_b128 v[40:43], %[a0] offset:%[o]\n\t"                             \
  "ds_read_b128 v[44:47], %[a1] offset:%[o]\n\t"                             \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "ds_read_b128 v[40:43], %[a2] offset:%[o]\n\t"                             \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_B                                   \
  "ds_read_b128 v[44:47], %[a3] offset:%[o]\n\t"                             \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "ds_read_b128 v[40:43], %[a4] offset:%[o]\n\t"                             \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_B                                   \
  "ds_read_b128 v[44:47], %[a5] offset:%[o]\n\t"                             \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "ds_read_b128 v[40:43], %[a6] offset:%[o]\n\t"                             \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_B                                   \
  "ds_read_b128 v[44:47], %[a7] offset:%[o]\n\t"                             \
  "s_waitcnt lgkmcnt(1)\n\t" K2H_X_CHUNK_A                                   \
  "s_waitcnt lgkmcnt(0)\n\t" LASTCHUNK
#define K2H_R8O_INPUTS                                                                                       \
  [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [a4] "v"(a[4]), [a5] "v"(a[5]),              \
      [a6] "v"(a[6]), [a7] "v"(a[7]), [o] "n"(O), [p] "s"(kPrimeLo), [sel] "s"(kSmearSel)

template <int O>
__device__ __forceinline__ void fnv_lds_round8o(uint32_t& lo, uint32_t& hi, uint32_t& z, const uint32_t (&a)[8]) {
  asm volatile(K2H_R8O_BODY(K2H_X_CHUNK_B)
               : "+{v48}"(lo), "+{v49}"(hi), "+{v50}"(z)
               : K2H_R8O_INPUTS
               : K2H_R8_CLOBBERS);
}

template <int O>
__device__ __forceinline__ void fnv_lds_round8o_last(uint32_t& lo, uint32_t& hi, uint32_t& z, uint32_t& lo2,
                                                     uint32_t& hi2, const uint32_t (&a)[8]) {
  asm volatile(K2H_R8O_BODY(K2H_LAST_B)
               : "+{v48}"(lo), "+{v49}"(hi), "+{v50}"(z), "={v60}"(lo2), "={v61}"(hi2)
               : K2H_R8O_INPUTS
               : K2H_R8_CLOBBERS);
}

// One round of line DMA for the line kernel: 8 global_load_lds_dwordx4, each an SGPR base
// (`src`, wave-uniform) + the lane's 32-bit offset v[i], LDS destination m + 1024 i in M0.
// As asm, the compiler neither counts these loads nor waits for them: every wait on them
// is the caller's explicit s_waitcnt vmcnt.  M0 is compiler-reserved (it cannot be
// declared clobbered) and is not restored here: the caller's kernel must have no other M0
// user -- tests/test_kernel_source.py checks the line-DMA kernel's code for any.
#define K2H_DMA1(I, OFF)             \
  "s_add_u32 m0, %[m], " #OFF "\n\t" \
  "s_nop 0\n\t"                      \
  "global_load_lds_dwordx4 %[v" #I "], %[s]\n\t"
__device__ __forceinline__ void line_dma8(uint64_t src, uint32_t m, const uint32_t (&v)[8]) {
  asm volatile(K2H_DMA1(0, 0) K2H_DMA1(1, 0x400) K2H_DMA1(2, 0x800) K2H_DMA1(3, 0xc00) K2H_DMA1(4, 0x1000)
                   K2H_DMA1(5, 0x1400) K2H_DMA1(6, 0x1800) K2H_DMA1(7, 0x1c00)
               :
               : [s] "s"(src), [m] "s"(m), [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]),
                 [v4] "v"(v[4]), [v5] "v"(v[5]), [v6] "v"(v[6]), [v7] "v"(v[7])
               : "memory", "scc");
}
#undef K2H_DMA1

}  // namespace k2h
