// k2hash_amd -- internal launch interface between the C-ABI (k2h_batch.cc) and the
// HIP kernels.  Not part of the public ABI (see include/k2hash_amd.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/k2hash_amd.h"

namespace k2h {

constexpr uint64_t kSeedBuiltinValue = 14695981039346656037ULL;  // lib/k2hashfunc.cc:51
constexpr uint64_t kSeedStdValue = 2166136261ULL;                  // libstdc++ _Fnv_hash_impl seed

// Kernel variant selector.  The product library (libk2hash_amd.so) always runs the
// default kernel per shape (kVariantAuto); the measurement lab (K2H_AMD_LAB=1 build,
// tools/lab/, k2h_amd_set_variant) compiles the round-1 A/B variants listed here.
enum { kVariantAuto = 0 };
#if K2H_AMD_LAB
// Kernel variant selector (A/B measurement knob, K2H_AMD_VARIANT env / k2h_amd_set_variant).
enum {
  kVariantCompiler = 1,  // fixed32: compiler-scheduled byte step instead of the hand-scheduled one
  kVariantGeneric = 2,   // fixed32: force the generic any-length kernel
  kVariantSimpleCsr = 3, // csr: one lane per key in input order (no length balancing)
  kVariantFixed32Flat = 4,     // fixed32: one 256-thread block per 256 keys (no prefetch)
  kVariantFixed32Persist = 5,  // fixed32: persistent grid, next keys prefetched into registers
  kVariantFixed32Lds = 6,      // fixed32: persistent + coalesced 1 KiB loads transposed through LDS
  kVariantFixed32Kpt2 = 7,     // fixed32: flat grid, 2 keys per thread, all loads issued up front
  kVariantFixed32Kpt4 = 8,     // fixed32: flat grid, 4 keys per thread
  kVariantFixedTail = 9,       // fixed (non-32): per-lane byte tail loop instead of end-aligned chunks
  kVariantDirect = 10,         // csr tile / fixed long: per-lane direct loads instead of the line ring
  kVariantCsrRing = 11,        // csr tile: line ring for every tile (no LDS staging of the tile)
  kVariantFixed32Asm = 12,     // fixed32: whole key (loads, 32 steps, store) in one asm statement
  kVariantCsrSingle = 13,      // csr staged: wave-uniform asm run over common chunks (lower VALU count,
                               // more dependency stalls at 2 waves/SIMD: slower, kept for A/B)
  kVariantCsrPairs = 14,       // csr staged: two chunks per asm statement (no uniform asm run)
  kVariantCsrProf = 15,        // csr staged, diagnostics: h2 receives per-tile phase stamps
                               // (16 words per 512-key tile, tools/csr_phases.py), not hashes
  kVariantFixed32Ring2 = 16,   // fixed32: persistent one-wave blocks, LDS-DMA ring of 2 tiles
  kVariantFixed32Ring3 = 17,   // fixed32: ... ring of 3 tiles (2 in flight while hashing)
  kVariantFixed32Ring4 = 18,   // fixed32: ... ring of 4 tiles
  kVariantCsrLean256 = 19,     // csr: 256-key tiles, 4 waves, 36 KiB stage, 4 blocks/CU, no ring union
  kVariantCsrLean512x8 = 20,   // csr: 512-key tiles, 8 waves (one group each), 72 KiB stage
  kVariantCsrLean512x4 = 21,   // csr: 512-key tiles, 4 waves, 72 KiB stage (the default kernel without the ring)
  kVariantCsrAlignProbe = 22,  // csr timing probe (WRONG hashes): lean256 with 16-aligned LDS chunk reads
  kVariantFixed32Blk64 = 23,   // fixed32 flat kernel with 64 / 128 / 512 / 1024-thread blocks
  kVariantFixed32Blk128 = 24,
  kVariantFixed32Blk512 = 25,
  kVariantFixed32Blk1024 = 26,
  kVariantFixed32Nt256 = 27,   // fixed32: the round-1 default (nt loads/stores, 256-thread blocks)
  kVariantRalleThread = 28,    // ralledata: one thread per record (round-1 A/B)
  kVariantFixed32W64Kpt2 = 29, // fixed32: one-wave blocks, 2 / 3 / 4 keys per lane, all loads issued first, nt
  kVariantFixed32W64Kpt3 = 30,
  kVariantFixed32W64Kpt4 = 31,
  kVariantLongRing = 32,       // fixed long keys: the cooperative line ring (the round-1 kernel)
  kVariantLongLines2 = 33,     // fixed long keys (len % 128 == 0): line DMA into a 2 / 3-round LDS ring
  kVariantLongLines3 = 34,
  kVariantLongHalf3 = 35,      // ... half-line rounds (64 B per lane), 3 / 4 / 6 of them
  kVariantLongHalf4 = 36,
  kVariantLongHalf6 = 37,
  kVariantLongHalf5 = 38,      // ... 5 half-line rounds (20 KiB: 8 waves per CU)
  kVariantLongLines2Pad = 39,  // 2 line rounds + 4 KiB / 2 KiB of LDS padding (8 / 9 waves per CU)
  kVariantLongLines2Pad2 = 40,
  kVariantLongProbeCompute = 41,  // timing probes (WRONG hashes): line-DMA kernel without DMA / without hashing
  kVariantLongProbeMemory = 42,
  kVariantLongProbeMem3 = 43,     // DMA-only probes at 3 / 4 line rounds, 2 double-line rounds, 4 half-line rounds
  kVariantLongProbeMem4 = 44,
  kVariantLongProbeMem256 = 45,
  kVariantLongProbeMemHalf4 = 46,
  kVariantLongLines256 = 47,      // fixed long keys (len % 256 == 0): 2 rounds of 256 B per lane (32 KiB)
  kVariantCsrTile = 48,           // csr: the round-1 default (512-key tile kernel with the ring inside)
  kVariantRalleGroup16 = 49,      // ralledata: 16 lanes per record, overlapped 16-byte tails
  kVariantRalleByteTail = 50,     // ralledata: the round-1 assembly (16 lanes, tails one byte per lane)
  kVariantCsrLeanRing = 51,       // csr: lean 512-key tiles + ring list, before the VALU trims (default: lean2)
  kVariantCsrLean2Pin = 52,       // csr: lean2 group walk with the chunk registers pinned to the asm banks (the pin
                                  // forces an lgkmcnt(0) per chunk read: 6 % slower)
  kVariantCsrLean2Step = 53,      // csr: lean2 group walk with the asm step walker (reads inside the hash asm, no copies)
  kVariantCsrLean2Group = 54,     // csr: lean2 with one key per lane in groups of 64 (default: two keys per lane,
                                  // short + long sorted partners, h2 from h1)
  kVariantRalleProbeAligned = 55, // ralledata timing probes (WRONG blobs): aligned segment stores / header only
  kVariantRalleProbeHeader = 56,
  kVariantRalleBatch4 = 57,       // ralledata: 4 / 2 records per 8-lane group, loads batched (slower, A/B)
  kVariantRalleBatch2 = 58,
  kVariantFixed32Pipe64 = 59,     // fixed32: persistent, next tile's loads issued before hashing the current
  kVariantFixed32Pipe256 = 60,    // (one-wave / 256-thread blocks, two keys per lane)
  kVariantCsrPair2 = 61,          // csr pair tiles: 256 keys, 2 waves, 36 KiB stage (4 blocks per CU)
  kVariantCsrPair2P = 62,         // ... persistent blocks, next tile's offsets prefetched during the hash
  kVariantCsrPair4P = 63,         // ... 512 keys, 4 waves, 72 KiB, persistent
  kVariantCsrPair4 = 64,          // ... 512 keys, 4 waves, 72 KiB
  kVariantCsrPair4PS = 66,        // csr pair tiles, persistent, second half of the grid starts half a tile late
  kVariantCsrPair2PS = 67,
  kVariantLongHalf2 = 70,         // fixed long keys: 2 half-line rounds (8 KiB ring per wave)
  kVariantFixed32Clock = 71,      // clock probes: the default fixed32 / 4 KiB kernels, h2 = per-wave stamps of the
  kVariantLongClock = 72,         // shader clock (s_memtime) and the 100 MHz counter (tools/clock_probe.py)
  kVariantCsrClock = 78,         // clock probe: the default CSR kernel (lean2), h2 = per-wave stamps (H2 off)
  kVariantRalleGroup8 = 73,       // ralledata: the round-1/2 group kernel (8 lanes per record, unaligned stores)
  kVariantRalleGather = 74,       // ralledata: output-driven gather from LDS-staged segments (aligned line stores)
  kVariantRalleGatherFused = 75,  // ... with the key hashes computed in the same kernel from the staged keys (default)
  kVariantRallePhases = 76,       // the one-shot gather form with per-block phase stamps in blob_off (tools/ralle_phases.py)
  kVariantRallePhasesNoStore = 77,  // ... and no piece stores (timing probe, wrong blobs)
  kVariantRallePieces2 = 79,      // gather form, two output pieces per loop trip
  kVariantRalleStageAll = 80,     // gather form, staged loads on all four waves
  kVariantCsrPair4Z = 69,         // csr pair tiles (512 keys), the mad64 zero half kept in v50 across the walk
  kVariantCsrDbuf = 81,           // csr: double-buffered 512-key tiles, one persistent block per CU, hash / sort /
                                  // DMA waves split by role
  kVariantCsrDbufProbeNoHash = 82,  // timing probes (WRONG hashes): dbuf without hashing / without feeding
  kVariantCsrDbufProbeNoFeed = 83,
  kVariantCsrQueue = 84,          // csr: queue tiles (8 hash waves claim 64-key groups, sort / DMA feeder waves)
  kVariantCsrQueueProbeNoHash = 85,  // timing probes (WRONG hashes): queue tiles without hashing / without feeding
  kVariantCsrQueueProbeNoFeed = 86,
  kVariantCsrQueuePrio = 87,      // csr queue tiles, feeder waves at raised issue priority
  kVariantCsrLean2Prio = 88,      // csr lean2 with its load / sort phase at raised issue priority (2; 89: 3, 90: 1)
  kVariantCsrLean2Prio3 = 89,
  kVariantCsrLean2Prio1 = 90,
  kVariantFixed32Prio = 91,       // fixed32 default kernel with its loads issued at raised priority
  kVariantLongPrio = 92,          // fixed long keys: line-DMA kernel, DMA issued at raised priority
  kVariantCsrLean2Scan1 = 93,     // csr lean2 (priority 1) with the class scan by wave 0 alone
  kVariantRallePrioLoads = 94,    // ralledata gather: loads at raised issue priority / all of phase 1 at raised priority
  kVariantRallePrioPhase1 = 95,
  kVariantCsrLean2Runs = 96,      // csr lean2 (priority 1, one-wave scan) with the pair walk in unchecked runs
  kVariantCsrLean3 = 97,          // csr lean3: persistent lean2, next tile's offsets LDS-DMA'd during the hash
  kVariantCsrLean2Desync1 = 98,   // csr lean2 (product settings), first-wave half tiles so co-resident tiles start out
  kVariantCsrLean2Desync2 = 99,   // of phase (98: blocks [0, #CU); 99: even blocks of [0, 2 #CU))
  kVariantCsrQueue320 = 100,      // csr queue tiles of 320 keys in three 46 KiB slots, feeders at raised priority
  kVariantCsrLean2PrioSetup = 101, // csr lean2 (one-wave scan) with priority 1 kept through the pair setup, dropped at the walk
  kVariantCsrLean2Ballot = 102,   // csr lean2 with the uniform-trip, ballot-guarded pair walk (pair_walk4)
  kVariantCsrPair4W2 = 68,        // csr pair tiles (512 keys) with the uniform-trip walk (pair_walk2)
  kVariantRalleStage = 65,        // ralledata: blobs of 64 records assembled in LDS, aligned line stores (slower)
};
#endif

// Bucket-index epilogue: where a hash lands in a k2hash table with
// masks (cur_mask, collision_mask) -- the stateless part of K2HShm::GetKIndexPos
// (lib/k2hshm.cc:810-833, with MakeMask / GetMaskBitCount at :78-90) and the collision
// slot `hash & collision_mask` (lib/k2hshm.cc:1093).
//   shifted       = hash >> bitlen(collision_mask)   (shift count taken mod 64, as the
//                                                     x86-64 shr the reference compiles to)
//   KIPtrArrayPos = bitlen(shifted & cur_mask)        (the reference's bitmask loop)
//   KIArrayPos    = shifted & MakeMask(KIPtrArrayPos - 1)   (MakeMask(0) = 0)
// kindex[i] packs KIPtrArrayPos << 58 | KIArrayPos (bitlen(cur_mask) <= 58 checked by the
// ABI); ckindex[i] = hash & collision_mask.  Either output may be null.
struct BucketParams {
  uint64_t cur_mask = 0;
  uint64_t collision_mask = 0;
  uint32_t cshift = 0;
  uint64_t* kindex = nullptr;
  uint64_t* ckindex = nullptr;
};
constexpr int kKindexPosShift = 58;

#ifdef __HIPCC__
// NT: nontemporal stores, for kernels whose lanes write consecutive i (a wave fills
// whole lines); kernels that write in a permuted order (CSR tiles, length-sorted) use
// plain stores so that L2 merges the partial lines before they reach HBM.
template <bool NT = true>
__device__ __forceinline__ void bucket_emit(const BucketParams& bp, uint64_t i, uint64_t h) {
  if (bp.kindex) {
    uint64_t shifted = h >> (bp.cshift & 63u);
    uint64_t tmp = shifted & bp.cur_mask;
    uint64_t pos = tmp ? 64u - (uint64_t)__clzll((long long)tmp) : 0u;
    uint64_t arr = pos ? shifted & ((1ull << (pos - 1)) - 1ull) : 0u;
    uint64_t v = (pos << kKindexPosShift) | arr;
    if constexpr (NT) __builtin_nontemporal_store(v, bp.kindex + i);
    else bp.kindex[i] = v;
  }
  if (bp.ckindex) {
    if constexpr (NT) __builtin_nontemporal_store(h & bp.collision_mask, bp.ckindex + i);
    else bp.ckindex[i] = h & bp.collision_mask;
  }
}
#endif

// Standalone epilogue over hashes already in device memory.
hipError_t launch_bucket_index(const uint64_t* h1, uint64_t n, const BucketParams& bp, hipStream_t stream);

// RALLEDATA producer inputs (k2h_ralledata.hip): four CSR streams; a null offsets
// array = that segment is empty for every record.
struct RalleInputs {
  const uint8_t* keys = nullptr;
  const uint64_t* koff = nullptr;
  const uint8_t* vals = nullptr;
  const uint64_t* voff = nullptr;
  const uint8_t* skeys = nullptr;
  const uint64_t* soff = nullptr;
  const uint8_t* attrs = nullptr;
  const uint64_t* aoff = nullptr;
};
hipError_t launch_ralledata(const RalleInputs& in, uint64_t n, uint64_t seed, uint8_t* out, uint64_t* blob_off,
                            int variant, hipStream_t stream);

// Keys at arbitrary (start, length) ranges (k2h_ranges.hip); cstr: hash key + NUL.
hipError_t launch_ranges(const void* base, const uint64_t* starts, const uint64_t* lens, uint64_t n, uint64_t seed,
                         bool cstr, uint64_t* h1, uint64_t* h2, int variant, hipStream_t stream);

// k2himport inputs already in device memory (k2h_import_dev.hip).  launch_import_scan
// returns a K2H_AMD_* code (the HIP error in *herr) and synchronises the stream.
// h1 != NULL: each written record's key is also hashed (key + NUL) by the same kernel.
int launch_import_scan(const void* file, uint64_t size, int format, k2h_amd_import_rec* recs, uint64_t cap,
                       uint64_t* count, hipStream_t stream, hipError_t* herr, uint64_t* h1 = nullptr,
                       uint64_t* h2 = nullptr, uint64_t seed = 0);
hipError_t launch_import_prehash(const void* file, uint64_t size, const k2h_amd_import_rec* recs, uint64_t n,
                                 uint64_t seed, uint64_t* h1, uint64_t* h2, hipStream_t stream);

// S_p = seed * P^-p (p = 0..15): start states for end-aligned chunking (k2h_csr.hip).
struct SpadTable {
  uint64_t v[16];
};
SpadTable make_spad(uint64_t seed);

// CSR tile kernels (k2h_csr.hip).  The product mode: 512-key LDS-staged tiles hashed two keys
// per lane, oversize tiles listed for a line-ring pass.  (Other modes: the lab build.)
constexpr int kCsrDefaultMode = 11;
hipError_t launch_csr_tile(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                           uint64_t* h2, int mode, hipStream_t stream, const BucketParams* bp = nullptr);
// Long fixed-length keys: mode kLongAuto picks the line-DMA kernel (key_len % 128 == 0,
// 128-aligned keys; 2 rounds of whole lines), else the cooperative line ring.
// kLongHalfD: rounds of half lines (64 B per lane), D of them.
enum { kLongAuto = 0, kLongDirect = 1, kLongRing = 2, kLongLines2 = 3,
#if K2H_AMD_LAB
       kLongLines3 = 4, kLongHalf3 = 5,
       kLongHalf4 = 6, kLongHalf6 = 7, kLongHalf5 = 8, kLongLines2Pad = 9, kLongLines2Pad2 = 10,
       kLongLines256 = 11,
       // timing probes (wrong hashes), keep last: no DMA / DMA only at (D, RB) =
       // (2,128) (2,128) (3,128) (4,128) (2,256) (4,64)
       kLongProbeCompute = 12, kLongProbeMemory = 13, kLongProbeMem3 = 14, kLongProbeMem4 = 15,
       kLongProbeMem256 = 16, kLongProbeMemHalf4 = 17,
       kLongHalf2 = 18,  // 2 half-line rounds (8 KiB per wave, 20 waves per CU)
       kLongProbeClock = 19,  // clock probe (h2 = per-wave shader-clock / 100 MHz stamps)
       kLongPrio = 20         // the default line-DMA kernel with each round's DMA issued at raised priority (h1 only)
#endif
};
bool fixed_lines_ok(const void* keys, uint64_t key_len);
hipError_t launch_fixed_long(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1,
                             uint64_t* h2, int mode, hipStream_t stream, const BucketParams* bp = nullptr);

hipError_t launch_fixed(const void* keys, uint64_t key_len, uint64_t n, uint64_t seed, uint64_t* h1, uint64_t* h2,
                        int variant, hipStream_t stream, const BucketParams* bp = nullptr);
hipError_t launch_csr(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                      uint64_t* h2, int variant, hipStream_t stream, const BucketParams* bp = nullptr);
#if K2H_AMD_LAB
hipError_t launch_csr_simple(const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t seed, uint64_t* h1,
                             uint64_t* h2, hipStream_t stream);
#endif

// Synthetic inputs (bench/test harness; same spec as oracle/fnv_oracle.c generators).
hipError_t launch_synth_bytes(uint8_t* out, uint64_t nbytes, uint64_t seed, uint64_t byte_off, hipStream_t stream);
hipError_t launch_synth_lengths(uint32_t* lens, uint64_t n, uint64_t seed, uint64_t first_key, uint32_t min_len,
                                uint32_t max_len, hipStream_t stream);

}  // namespace k2h
