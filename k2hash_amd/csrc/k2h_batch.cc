// k2hash_amd -- batch C-ABI (include/k2hash_amd.h section 2) over the HIP kernels.
//
// Device-pointer entry points validate arguments and launch on the caller's stream.
// Host-pointer entry points stage through pinned buffers and pipeline
// host-copy -> H2D -> kernel -> D2H over two streams in chunks, so a caller that holds
// keys in host memory (the k2hash process itself) gets the PCIe-bound rate without
// managing device memory.  HIP is touched only inside these calls (lazy init), never at
// library load, so libk2hash can dlopen this library as its plugin safely.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/k2hash_amd.h"
#include "k2h_kernels.h"

namespace {

thread_local char g_err[256];


int fail(int code, const char* what, hipError_t e = hipSuccess) {
  if (e != hipSuccess)
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
  else
    snprintf(g_err, sizeof g_err, "%s", what);
  return code;
}

uint64_t seed_for(uint32_t flags) {
  return (flags & K2H_AMD_FLAG_STD_FNV) ? k2h::kSeedStdValue : k2h::kSeedBuiltinValue;
}

// ---------------------------------------------------------------------------
// Device gate (include/k2hash_amd.h: K2H_AMD_ENODEV = "no usable gfx950 device").  The
// library carries gfx950 code objects only, so every entry point that launches checks the
// device's architecture once (cached per device) and returns ENODEV before any launch on a
// device without a gfx950 ISA.  K2H_AMD_TEST_ARCH, read once per process, replaces the name
// the runtime reports: a test hook that lets a gfx950 box exercise the refusal.
// ---------------------------------------------------------------------------
constexpr int kMaxDevices = 64;
std::atomic<int8_t> g_arch_ok[kMaxDevices];  // 0 unknown, 1 gfx950, -1 other

int gate_device(int device) {
  if (device < 0 || device >= kMaxDevices) return fail(K2H_AMD_EINVAL, "device index out of range");
  int8_t s = g_arch_ok[device].load(std::memory_order_relaxed);
  if (s == 0) {
    static const char* forced = getenv("K2H_AMD_TEST_ARCH");
    char name[256] = {0};
    if (forced) {
      snprintf(name, sizeof name, "%s", forced);
    } else {
      hipDeviceProp_t p;
      hipError_t e = hipGetDeviceProperties(&p, device);
      if (e != hipSuccess) return fail(K2H_AMD_ENODEV, "hipGetDeviceProperties", e);
      snprintf(name, sizeof name, "%s", p.gcnArchName);
    }
    // gcnArchName is "gfx950" or "gfx950:sramecc+:xnack-": the processor name before ':'
    s = (strncmp(name, "gfx950", 6) == 0 && (name[6] == 0 || name[6] == ':')) ? 1 : -1;
    g_arch_ok[device].store(s, std::memory_order_relaxed);
  }
  if (s < 0) return fail(K2H_AMD_ENODEV, "device is not gfx950 (this library holds gfx950 code only)");
  return K2H_AMD_OK;
}

// The caller's current device (device-pointer entry points launch there).
int gate_current() {
  int d = -1;
  hipError_t e = hipGetDevice(&d);
  if (e != hipSuccess) return fail(K2H_AMD_ENODEV, "no HIP device", e);
  return gate_device(d);
}

#define K2H_GATE()                          \
  do {                                      \
    if (int gate_rc_ = gate_current())      \
      return gate_rc_;                      \
  } while (0)

// ---------------------------------------------------------------------------
// Parallel host copies for the staging pipeline.  One core's memcpy into pinned memory
// runs at ~16 GB/s on the MI355X hosts, a third of PCIe (57 GB/s measured,
// tools/host_rate.py), so staging copies are split over a small worker pool.  The pool
// is created on the first host-path call (never at library load) and re-created in a
// forked child, whose copy of the pool has no threads.
// ---------------------------------------------------------------------------
class CopyPool {
 public:
  void copy(void* dst, const void* src, size_t len) {
    if (len < (4u << 20) || nthreads() <= 1) {
      memcpy(dst, src, len);
      return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    ensure();
    dst_ = (uint8_t*)dst;
    src_ = (const uint8_t*)src;
    len_ = len;
    piece_ = std::max<size_t>(1u << 20, (len + 4 * (nworkers_ + 1) - 1) / (4 * (nworkers_ + 1)));
    piece_ = (piece_ + 4095) & ~(size_t)4095;
    next_.store(0);
    busy_ = nworkers_;
    ++gen_;
    cv_.notify_all();
    lk.unlock();
    run();  // the caller copies too
    lk.lock();
    done_cv_.wait(lk, [&] { return busy_ == 0; });
  }

 private:
  static int nthreads() {
    static int n = [] {
      const char* e = getenv("K2H_AMD_COPY_THREADS");
      int v = e ? atoi(e) : (int)std::min(8u, std::max(1u, std::thread::hardware_concurrency() / 2));
      return v < 1 ? 1 : v;
    }();
    return n;
  }
  void ensure() {
    if (pid_ == getpid() && nworkers_) return;
    // (re)start: in a forked child the parent's workers do not exist.  Workers are
    // detached and the pool is never destroyed (see pool()), so process exit neither
    // joins nor terminates them.
    nworkers_ = 0;
    pid_ = getpid();
    gen_ = 0;
    for (int i = 0; i < nthreads() - 1; ++i, ++nworkers_)
      std::thread([this] {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
          cv_.wait(lk, [&] { return gen_ != seen; });
          seen = gen_;
          lk.unlock();
          run();
          lk.lock();
          if (--busy_ == 0) done_cv_.notify_all();
        }
      }).detach();
  }
  void run() {
    for (;;) {
      size_t off = next_.fetch_add(piece_);
      if (off >= len_) return;
      memcpy(dst_ + off, src_ + off, std::min(piece_, len_ - off));
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  size_t nworkers_ = 0;
  pid_t pid_ = 0;
  uint64_t gen_ = 0;
  size_t busy_ = 0;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  size_t len_ = 0, piece_ = 0;
  std::atomic<size_t> next_{0};
};

CopyPool& pool() {
  static CopyPool* p = new CopyPool;  // never destroyed: detached workers may outlive statics
  return *p;
}

// ---------------------------------------------------------------------------
// Host-path pipeline: per device, two slots used alternately, one stream each.
//  - in:  the caller's keys are copied into the slot's pinned staging buffer by the copy
//         pool (8+ threads: ~119 GB/s, tools/host_probe.hip) while the previous chunk's
//         H2D DMA runs, then DMA'd at the PCIe rate (57.5 GB/s).  Handing the runtime the
//         caller's pageable buffer instead makes it pin the whole allocation on every call
//         (~40 ms per 512 MiB, rocprofv3 --sys-trace of tools/host_trace.py).
//  - out: fixed-length keys: the kernel stores the hashes straight into the slot's pinned
//         output buffer over PCIe (a wave writes whole lines), so no D2H copy queues behind
//         the next chunk's H2D on the DMA engine; CSR keys (hashes stored in length-sorted
//         order, partial lines) come back with a D2H copy.  The pool then copies them to
//         the caller when the slot is reused or the call ends.
// ---------------------------------------------------------------------------
struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* h_in = nullptr;   // pinned input bytes
  uint64_t* h_off = nullptr; // pinned offsets (CSR)
  uint64_t* h_out = nullptr; // pinned h1 (+h2) results
  uint64_t* h_out_dev = nullptr; // the same buffer as a device pointer (kernel stores)
  uint8_t* d_in = nullptr;
  uint64_t* d_off = nullptr;
  uint64_t* d_out = nullptr;
  uint64_t cap_in = 0, cap_keys = 0;
  bool busy = false;
  // pending result copy-out
  uint64_t first = 0, count = 0;
  bool want_h2 = false;
};

struct HostCtx {
  std::mutex mu;
  Slot slot[2];
};

HostCtx g_ctx[64];

int slot_reserve(Slot& s, uint64_t bytes, uint64_t keys) {
  hipError_t e;
  if (!s.stream) {
    if ((e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess)
      return fail(K2H_AMD_EHIP, "hipStreamCreate", e);
    if ((e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming)) != hipSuccess)
      return fail(K2H_AMD_EHIP, "hipEventCreate", e);
  }
  if (bytes > s.cap_in) {
    if (s.h_in) (void)hipHostFree(s.h_in);
    if (s.d_in) (void)hipFree(s.d_in);
    s.h_in = nullptr;
    s.d_in = nullptr;
    s.cap_in = 0;
    if (hipHostMalloc((void**)&s.h_in, bytes, hipHostMallocDefault) != hipSuccess ||
        hipMalloc((void**)&s.d_in, bytes) != hipSuccess)
      return fail(K2H_AMD_ENOMEM, "staging allocation (bytes)");
    s.cap_in = bytes;
  }
  if (keys > s.cap_keys) {
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_out) (void)hipFree(s.d_out);
    s.h_off = nullptr;
    s.h_out = nullptr;
    s.h_out_dev = nullptr;
    s.d_off = nullptr;
    s.d_out = nullptr;
    s.cap_keys = 0;
    if (hipHostMalloc((void**)&s.h_off, (keys + 1) * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&s.h_out, keys * 16, hipHostMallocDefault) != hipSuccess ||
        hipMalloc((void**)&s.d_off, (keys + 1) * 8) != hipSuccess || hipMalloc((void**)&s.d_out, keys * 16) != hipSuccess)
      return fail(K2H_AMD_ENOMEM, "staging allocation (keys)");
    if (hipHostGetDevicePointer((void**)&s.h_out_dev, s.h_out, 0) != hipSuccess) s.h_out_dev = nullptr;
    s.cap_keys = keys;
  }
  return K2H_AMD_OK;
}

// Wait for a slot's previous chunk and copy its results out of pinned memory.
int slot_drain(Slot& s, uint64_t* h1, uint64_t* h2) {
  if (!s.busy) return K2H_AMD_OK;
  hipError_t e = hipEventSynchronize(s.done);
  s.busy = false;
  if (e != hipSuccess) return fail(K2H_AMD_EHIP, "chunk completion", e);
  pool().copy(h1 + s.first, s.h_out, s.count * 8);
  if (s.want_h2 && h2) pool().copy(h2 + s.first, s.h_out + s.count, s.count * 8);
  return K2H_AMD_OK;
}

// Forget a slot's pending chunk without copying it anywhere: waits for the device work that
// still writes into the slot's buffers.  Every host call starts by discarding both slots,
// and every error return discards them too, so a chunk left behind by a failed call can
// never be drained into a later caller's output.
void slot_discard(Slot& s) {
  if (s.busy && s.done) (void)hipEventSynchronize(s.done);
  s.busy = false;
}

struct SlotsGuard {  // discards both slots on entry and on every return path
  HostCtx& c;
  explicit SlotsGuard(HostCtx& ctx) : c(ctx) {
    slot_discard(c.slot[0]);
    slot_discard(c.slot[1]);
  }
  ~SlotsGuard() {
    slot_discard(c.slot[0]);
    slot_discard(c.slot[1]);
  }
};

constexpr uint64_t kChunkBytes = 64ull << 20;  // 64 MiB of key bytes per pipeline chunk
constexpr uint64_t kChunkKeysMax = 4ull << 20;

// Makes `device` current for the duration of a host-pointer call and restores the caller's
// current device on every return path (a torch process must not see its current
// device change under it).
class DeviceGuard {
 public:
  int enter(int device) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) return fail(K2H_AMD_ENODEV, "no HIP device", e);
    if (device < 0 || device >= count || device >= 64) return fail(K2H_AMD_EINVAL, "device index out of range");
    if (int rc = gate_device(device)) return rc;
    if ((e = hipGetDevice(&prev_)) != hipSuccess) return fail(K2H_AMD_EHIP, "hipGetDevice", e);
    if (prev_ != device && (e = hipSetDevice(device)) != hipSuccess) return fail(K2H_AMD_EHIP, "hipSetDevice", e);
    set_ = prev_ != device;
    return K2H_AMD_OK;
  }
  ~DeviceGuard() {
    if (set_) (void)hipSetDevice(prev_);
  }

 private:
  int prev_ = -1;
  bool set_ = false;
};

}  // namespace

extern "C" {

__attribute__((visibility("default"))) int k2h_amd_hash_fixed(const void* keys, uint64_t key_len, uint64_t n,
                                                              uint64_t* h1, uint64_t* h2, uint32_t flags,
                                                              void* stream) {
  if (n == 0) return K2H_AMD_OK;
  if (!h1) return fail(K2H_AMD_EINVAL, "h1 is NULL");
  if (key_len && n > UINT64_MAX / key_len) return fail(K2H_AMD_EINVAL, "n * key_len overflows");
  K2H_GATE();
  hipError_t e = k2h::launch_fixed(keys, key_len, n, seed_for(flags), h1, h2, (hipStream_t)stream);
  if (e != hipSuccess) return fail(K2H_AMD_EHIP, "launch_fixed", e);
  return K2H_AMD_OK;
}

__attribute__((visibility("default"))) int k2h_amd_hash_csr(const void* bytes, const uint64_t* offsets, uint64_t n,
                                                            uint64_t* h1, uint64_t* h2, uint32_t flags,
                                                            void* stream) {
  if (n == 0) return K2H_AMD_OK;
  if (!h1 || !offsets) return fail(K2H_AMD_EINVAL, "h1/offsets is NULL");
  K2H_GATE();
  hipError_t e = k2h::launch_csr(bytes, offsets, n, seed_for(flags), h1, h2, (hipStream_t)stream);
  if (e != hipSuccess) return fail(K2H_AMD_EHIP, "launch_csr", e);
  return K2H_AMD_OK;
}

}  // extern "C"

namespace {
int bucket_params(uint64_t cur_mask, uint64_t collision_mask, uint64_t* kindex, uint64_t* ckindex,
                  k2h::BucketParams& bp) {
  int bits = 0;
  for (uint64_t m = cur_mask; m; m >>= 1) ++bits;  // GetMaskBitCount, lib/k2hshm.cc:85-90
  if (kindex && bits > k2h::kKindexPosShift)
    return fail(K2H_AMD_EINVAL, "cur_mask wider than 58 bits cannot be packed into kindex");
  int cbits = 0;
  for (uint64_t m = collision_mask; m; m >>= 1) ++cbits;
  bp.cur_mask = cur_mask;
  bp.collision_mask = collision_mask;
  bp.cshift = (uint32_t)cbits;
  bp.kindex = kindex;
  bp.ckindex = ckindex;
  return K2H_AMD_OK;
}
}  // namespace

extern "C" {

__attribute__((visibility("default"))) int k2h_amd_bucket_index(const uint64_t* h1, uint64_t n, uint64_t cur_mask,
                                                                uint64_t collision_mask, uint64_t* kindex,
                                                                uint64_t* ckindex, void* stream) {
  if (n == 0 || (!kindex && !ckindex)) return K2H_AMD_OK;
  if (!h1) return fail(K2H_AMD_EINVAL, "h1 is NULL");
  k2h::BucketParams bp;
  int rc = bucket_params(cur_mask, collision_mask, kindex, ckindex, bp);
  if (rc) return rc;
  K2H_GATE();
  hipError_t e = k2h::launch_bucket_index(h1, n, bp, (hipStream_t)stream);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_bucket_index", e);
}

__attribute__((visibility("default"))) int k2h_amd_hash_fixed_index(const void* keys, uint64_t key_len, uint64_t n,
                                                                    uint64_t* h1, uint64_t* h2, uint32_t flags,
                                                                    uint64_t cur_mask, uint64_t collision_mask,
                                                                    uint64_t* kindex, uint64_t* ckindex,
                                                                    void* stream) {
  if (n == 0) return K2H_AMD_OK;
  if (!h1) return fail(K2H_AMD_EINVAL, "h1 is NULL");
  if (key_len && n > UINT64_MAX / key_len) return fail(K2H_AMD_EINVAL, "n * key_len overflows");
  k2h::BucketParams bp;
  int rc = bucket_params(cur_mask, collision_mask, kindex, ckindex, bp);
  if (rc) return rc;
  K2H_GATE();
  hipError_t e =
      k2h::launch_fixed(keys, key_len, n, seed_for(flags), h1, h2, (hipStream_t)stream, &bp);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_fixed (index)", e);
}

__attribute__((visibility("default"))) int k2h_amd_hash_csr_index(const void* bytes, const uint64_t* offsets,
                                                                  uint64_t n, uint64_t* h1, uint64_t* h2,
                                                                  uint32_t flags, uint64_t cur_mask,
                                                                  uint64_t collision_mask, uint64_t* kindex,
                                                                  uint64_t* ckindex, void* stream) {
  if (n == 0) return K2H_AMD_OK;
  if (!h1 || !offsets) return fail(K2H_AMD_EINVAL, "h1/offsets is NULL");
  k2h::BucketParams bp;
  int rc = bucket_params(cur_mask, collision_mask, kindex, ckindex, bp);
  if (rc) return rc;
  K2H_GATE();
  hipError_t e = k2h::launch_csr(bytes, offsets, n, seed_for(flags), h1, h2, (hipStream_t)stream, &bp);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_csr (index)", e);
}

// Table forms with a NULL bitmap (every entry assigned) run the stateless epilogue; what
// that epilogue cannot express is filled here: found = 1 (0 when cur_mask is 0), and for
// cur_mask 0 kindex = K2H_AMD_KINDEX_NONE -- GetKIndex returns NULL then
// (lib/k2hshm.cc:882-907), the same as the bitmap form -- so the epilogue
// does not write kindex in that case.
static int null_bitmap_fill(const k2h_amd_table* table, uint64_t n, uint64_t* kindex, uint8_t* found,
                            k2h::BucketParams& bp, void* stream) {
  if (table->assigned) return K2H_AMD_OK;
  if (found) {
    hipError_t e = hipMemsetAsync(found, table->cur_mask ? 1 : 0, n, (hipStream_t)stream);
    if (e != hipSuccess) return fail(K2H_AMD_EHIP, "found fill", e);
  }
  if (kindex && table->cur_mask == 0) {
    hipError_t e = hipMemsetAsync(kindex, 0xFF, n * sizeof(uint64_t), (hipStream_t)stream);
    if (e != hipSuccess) return fail(K2H_AMD_EHIP, "kindex fill", e);
    bp.kindex = nullptr;
  }
  return K2H_AMD_OK;
}

__attribute__((visibility("default"))) int k2h_amd_bucket_index_table(const uint64_t* h1, uint64_t n,
                                                                      const k2h_amd_table* table, uint64_t* kindex,
                                                                      uint64_t* ckindex, uint8_t* found, void* stream) {
  if (!table) return fail(K2H_AMD_EINVAL, "table is NULL");
  if (n == 0 || (!kindex && !ckindex && !found)) return K2H_AMD_OK;
  if (!h1) return fail(K2H_AMD_EINVAL, "h1 is NULL");
  k2h::BucketParams bp;
  int rc = bucket_params(table->cur_mask, table->collision_mask, kindex, ckindex, bp);
  if (rc) return rc;
  bp.assigned = table->assigned;
  bp.found = table->assigned ? found : nullptr;
  K2H_GATE();
  if ((rc = null_bitmap_fill(table, n, kindex, found, bp, stream))) return rc;
  hipError_t e = k2h::launch_bucket_index(h1, n, bp, (hipStream_t)stream);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_bucket_index (table)", e);
}

__attribute__((visibility("default"))) int k2h_amd_hash_fixed_index_table(
    const void* keys, uint64_t key_len, uint64_t n, uint64_t* h1, uint64_t* h2, uint32_t flags,
    const k2h_amd_table* table, uint64_t* kindex, uint64_t* ckindex, uint8_t* found, void* stream) {
  if (!table) return fail(K2H_AMD_EINVAL, "table is NULL");
  if (n == 0) return K2H_AMD_OK;
  if (!h1) return fail(K2H_AMD_EINVAL, "h1 is NULL");
  if (key_len && n > UINT64_MAX / key_len) return fail(K2H_AMD_EINVAL, "n * key_len overflows");
  k2h::BucketParams bp;
  int rc = bucket_params(table->cur_mask, table->collision_mask, kindex, ckindex, bp);
  if (rc) return rc;
  bp.assigned = table->assigned;
  bp.found = table->assigned ? found : nullptr;
  K2H_GATE();
  if ((rc = null_bitmap_fill(table, n, kindex, found, bp, stream))) return rc;
  hipError_t e = k2h::launch_fixed(keys, key_len, n, seed_for(flags), h1, h2, (hipStream_t)stream, &bp);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_fixed (table index)", e);
}

__attribute__((visibility("default"))) int k2h_amd_hash_csr_index_table(
    const void* bytes, const uint64_t* offsets, uint64_t n, uint64_t* h1, uint64_t* h2, uint32_t flags,
    const k2h_amd_table* table, uint64_t* kindex, uint64_t* ckindex, uint8_t* found, void* stream) {
  if (!table) return fail(K2H_AMD_EINVAL, "table is NULL");
  if (n == 0) return K2H_AMD_OK;
  if (!h1 || !offsets) return fail(K2H_AMD_EINVAL, "h1/offsets is NULL");
  k2h::BucketParams bp;
  int rc = bucket_params(table->cur_mask, table->collision_mask, kindex, ckindex, bp);
  if (rc) return rc;
  bp.assigned = table->assigned;
  bp.found = table->assigned ? found : nullptr;
  K2H_GATE();
  if ((rc = null_bitmap_fill(table, n, kindex, found, bp, stream))) return rc;
  hipError_t e = k2h::launch_csr(bytes, offsets, n, seed_for(flags), h1, h2, (hipStream_t)stream, &bp);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_csr (table index)", e);
}

__attribute__((visibility("default"))) int k2h_amd_hash_fixed_host(const void* keys, uint64_t key_len, uint64_t n,
                                                                   uint64_t* h1, uint64_t* h2, uint32_t flags,
                                                                   int device) {
  if (n == 0) return K2H_AMD_OK;
  if (!h1) return fail(K2H_AMD_EINVAL, "h1 is NULL");
  if (key_len && n > UINT64_MAX / key_len) return fail(K2H_AMD_EINVAL, "n * key_len overflows");
  if (!keys || key_len == 0) {
    memset(h1, 0, n * 8);
    if (h2) memset(h2, 0, n * 8);
    return K2H_AMD_OK;
  }
  DeviceGuard dg;
  int rc = dg.enter(device);
  if (rc) return rc;
  HostCtx& c = g_ctx[device];
  std::lock_guard<std::mutex> lk(c.mu);
  SlotsGuard sg(c);
  uint64_t per = kChunkBytes / key_len;
  if (per == 0) per = 1;
  if (per > kChunkKeysMax) per = kChunkKeysMax;
  const uint8_t* src = (const uint8_t*)keys;
  int k = 0;
  for (uint64_t first = 0; first < n; first += per, k ^= 1) {
    uint64_t cnt = n - first < per ? n - first : per;
    Slot& s = c.slot[k];
    if ((rc = slot_drain(s, h1, h2))) return rc;
    if ((rc = slot_reserve(s, per * key_len, per))) return rc;
    pool().copy(s.h_in, src + first * key_len, cnt * key_len);
    hipError_t e = hipMemcpyAsync(s.d_in, s.h_in, cnt * key_len, hipMemcpyHostToDevice, s.stream);
    uint64_t* out = s.h_out_dev ? s.h_out_dev : s.d_out;  // kernel stores over PCIe when mapped
    if (e == hipSuccess)
      e = k2h::launch_fixed(s.d_in, key_len, cnt, seed_for(flags), out, h2 ? out + cnt : nullptr, s.stream);
    if (e == hipSuccess && !s.h_out_dev)
      e = hipMemcpyAsync(s.h_out, s.d_out, cnt * (h2 ? 16 : 8), hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
    if (e != hipSuccess) return fail(K2H_AMD_EHIP, "fixed host chunk", e);
    s.busy = true;
    s.first = first;
    s.count = cnt;
    s.want_h2 = h2 != nullptr;
  }
  for (int j = 0; j < 2; ++j)
    if ((rc = slot_drain(c.slot[j], h1, h2))) return rc;
  return K2H_AMD_OK;
}

__attribute__((visibility("default"))) int k2h_amd_hash_csr_host(const void* bytes, const uint64_t* offsets,
                                                                 uint64_t n, uint64_t* h1, uint64_t* h2,
                                                                 uint32_t flags, int device) {
  if (n == 0) return K2H_AMD_OK;
  if (!h1 || !offsets) return fail(K2H_AMD_EINVAL, "h1/offsets is NULL");
  if (!bytes) {
    memset(h1, 0, n * 8);
    if (h2) memset(h2, 0, n * 8);
    return K2H_AMD_OK;
  }
  DeviceGuard dg;
  int rc = dg.enter(device);
  if (rc) return rc;
  HostCtx& c = g_ctx[device];
  std::lock_guard<std::mutex> lk(c.mu);
  SlotsGuard sg(c);
  const uint8_t* src = (const uint8_t*)bytes;
  int k = 0;
  uint64_t first = 0;
  while (first < n) {
    // the longest run of keys from `first` within the byte budget and the key cap (>= 1
    // key), found by a linear walk that checks every offset pair on the way: a decrease
    // ends the call with EINVAL before any of this chunk's work is queued (the GPU still
    // works on the previous chunk meanwhile), and no search runs over unchecked offsets
    // (ADVICE r2).  Byte counts are differences of checked, non-decreasing offsets, so
    // nothing wraps.
    const uint64_t cap = n - first < kChunkKeysMax ? n : first + kChunkKeysMax;
    if (offsets[first + 1] < offsets[first]) return fail(K2H_AMD_EINVAL, "offsets not non-decreasing");
    uint64_t last = first + 1;
    while (last < cap) {
      const uint64_t a = offsets[last], b = offsets[last + 1];
      if (b < a) return fail(K2H_AMD_EINVAL, "offsets not non-decreasing");
      if (b - offsets[first] > kChunkBytes) break;
      ++last;
    }
    uint64_t cnt = last - first;
    uint64_t nb = offsets[last] - offsets[first];
    Slot& s = c.slot[k];
    if ((rc = slot_drain(s, h1, h2))) return rc;
    if ((rc = slot_reserve(s, nb > kChunkBytes ? nb : kChunkBytes, kChunkKeysMax))) return rc;
    // the kernel takes the caller's offsets as they are, relative to a byte base placed
    // offsets[first] bytes before the chunk (no rebasing pass on the CPU)
    pool().copy(s.h_in, src + offsets[first], nb);
    pool().copy(s.h_off, offsets + first, (cnt + 1) * 8);
    hipError_t e = nb ? hipMemcpyAsync(s.d_in, s.h_in, nb, hipMemcpyHostToDevice, s.stream) : hipSuccess;
    if (e == hipSuccess) e = hipMemcpyAsync(s.d_off, s.h_off, (cnt + 1) * 8, hipMemcpyHostToDevice, s.stream);
    if (e == hipSuccess)
      e = k2h::launch_csr((const uint8_t*)s.d_in - offsets[first], s.d_off, cnt, seed_for(flags), s.d_out,
                          h2 ? s.d_out + cnt : nullptr, s.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s.h_out, s.d_out, cnt * (h2 ? 16 : 8), hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
    if (e != hipSuccess) return fail(K2H_AMD_EHIP, "csr host chunk", e);
    s.busy = true;
    s.first = first;
    s.count = cnt;
    s.want_h2 = h2 != nullptr;
    first = last;
    k ^= 1;
  }
  for (int j = 0; j < 2; ++j)
    if ((rc = slot_drain(c.slot[j], h1, h2))) return rc;
  return K2H_AMD_OK;
}

__attribute__((visibility("default"))) int k2h_amd_hash_ranges(const void* base, const uint64_t* starts,
                                                               const uint64_t* lens, uint64_t n, uint64_t* h1,
                                                               uint64_t* h2, uint32_t flags, void* stream) {
  if (n == 0) return K2H_AMD_OK;
  if (!h1 || !starts || !lens || !base) return fail(K2H_AMD_EINVAL, "NULL base/starts/lens/h1");
  K2H_GATE();
  hipError_t e = k2h::launch_ranges(base, starts, lens, n, seed_for(flags), (flags & K2H_AMD_FLAG_CSTR) != 0, h1, h2,
                                    (hipStream_t)stream);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_ranges", e);
}

// k2himport inputs in device memory (include/k2hash_amd.h section 5)
__attribute__((visibility("default"))) int k2h_amd_import_scan_device(const void* file, uint64_t size, int format,
                                                                      k2h_amd_import_rec* recs, uint64_t cap,
                                                                      uint64_t* count, void* stream) {
  if (!count || (size && !file) || (format != K2H_AMD_IMPORT_TSV && format != K2H_AMD_IMPORT_MDBM))
    return fail(K2H_AMD_EINVAL, "import_scan_device: NULL count/file or bad format");
  if (size) K2H_GATE();  // an empty file has no records and needs no device
  hipError_t e = hipSuccess;
  int rc = k2h::launch_import_scan(file, size, format, recs, cap, count, (hipStream_t)stream, &e);
  if (rc == K2H_AMD_EHIP) return fail(rc, "launch_import_scan", e);
  return rc == K2H_AMD_OK ? rc : fail(rc, "import_scan_device: not a mdbm file, or more records than cap");
}

__attribute__((visibility("default"))) int k2h_amd_import_scan_prehash_device(
    const void* file, uint64_t size, int format, k2h_amd_import_rec* recs, uint64_t cap, uint64_t* count, uint64_t* h1,
    uint64_t* h2, uint32_t flags, void* stream) {
  if (!count || (size && !file) || (format != K2H_AMD_IMPORT_TSV && format != K2H_AMD_IMPORT_MDBM))
    return fail(K2H_AMD_EINVAL, "import_scan_prehash_device: NULL count/file or bad format");
  if (recs && cap && !h1) return fail(K2H_AMD_EINVAL, "import_scan_prehash_device: NULL h1");
  if (size) K2H_GATE();  // an empty file has no records and needs no device
  hipError_t e = hipSuccess;
  int rc = k2h::launch_import_scan(file, size, format, recs, cap, count, (hipStream_t)stream, &e, h1, h2,
                                   seed_for(flags));
  if (rc == K2H_AMD_EHIP) return fail(rc, "launch_import_scan", e);
  return rc == K2H_AMD_OK ? rc : fail(rc, "import_scan_prehash_device: not a mdbm file, or more records than cap");
}

__attribute__((visibility("default"))) int k2h_amd_import_prehash(const void* file, uint64_t size,
                                                                  const k2h_amd_import_rec* recs, uint64_t n, uint64_t* h1, uint64_t* h2,
                                                                  uint32_t flags, void* stream) {
  if (n == 0) return K2H_AMD_OK;
  if (!file || !recs || !h1) return fail(K2H_AMD_EINVAL, "import_prehash: NULL file/recs/h1");
  K2H_GATE();
  hipError_t e = k2h::launch_import_prehash(file, size, recs, n, seed_for(flags), h1, h2, (hipStream_t)stream);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_import_prehash", e);
}

// ---------------------------------------------------------------------------
// RALLEDATA producer (include/k2hash_amd.h section 4)
// ---------------------------------------------------------------------------
__attribute__((visibility("default"))) uint64_t k2h_amd_ralledata_size(uint64_t n, uint64_t key_bytes,
                                                                       uint64_t val_bytes, uint64_t skey_bytes,
                                                                       uint64_t attr_bytes) {
  return 80ull * n + key_bytes + val_bytes + skey_bytes + attr_bytes;
}

__attribute__((visibility("default"))) int k2h_amd_build_ralledata(
    const void* keys, const uint64_t* key_off, const void* vals, const uint64_t* val_off, const void* skeys,
    const uint64_t* skey_off, const void* attrs, const uint64_t* attr_off, uint64_t n, void* out, uint64_t* blob_off,
    uint32_t flags, void* stream) {
  if (!key_off) return fail(K2H_AMD_EINVAL, "key_off is NULL");
  if (n && !out) return fail(K2H_AMD_EINVAL, "out is NULL");
  if ((val_off && !vals) || (skey_off && !skeys) || (attr_off && !attrs))
    return fail(K2H_AMD_EINVAL, "segment offsets without segment bytes");
  K2H_GATE();
  k2h::RalleInputs in;
  in.keys = (const uint8_t*)keys;
  in.koff = key_off;
  in.vals = (const uint8_t*)vals;
  in.voff = val_off;
  in.skeys = (const uint8_t*)skeys;
  in.soff = skey_off;
  in.attrs = (const uint8_t*)attrs;
  in.aoff = attr_off;
  hipError_t e = k2h::launch_ralledata(in, n, seed_for(flags), (uint8_t*)out, blob_off, (hipStream_t)stream);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "launch_ralledata", e);
}

// Host form: stage each segment's byte range and offsets on `device`, build there, copy
// the blobs (and offsets) back.  One shot, not pipelined.
__attribute__((visibility("default"))) int k2h_amd_build_ralledata_host(
    const void* keys, const uint64_t* key_off, const void* vals, const uint64_t* val_off, const void* skeys,
    const uint64_t* skey_off, const void* attrs, const uint64_t* attr_off, uint64_t n, void* out, uint64_t* blob_off,
    uint32_t flags, int device) {
  if (!key_off) return fail(K2H_AMD_EINVAL, "key_off is NULL");
  if (n == 0) {
    if (blob_off) blob_off[0] = 0;
    return K2H_AMD_OK;
  }
  if (!out) return fail(K2H_AMD_EINVAL, "out is NULL");
  const void* src[4] = {keys, vals, skeys, attrs};
  const uint64_t* off[4] = {key_off, val_off, skey_off, attr_off};
  uint64_t total = 80ull * n;
  for (int s = 0; s < 4; ++s) {
    if (!off[s]) continue;
    if (!src[s] && off[s][n] != off[s][0]) return fail(K2H_AMD_EINVAL, "segment offsets without segment bytes");
    for (uint64_t i = 0; i < n; ++i)
      if (off[s][i + 1] < off[s][i]) return fail(K2H_AMD_EINVAL, "offsets not non-decreasing");
    total += off[s][n] - off[s][0];
  }
  DeviceGuard dg;
  int rc = dg.enter(device);
  if (rc) return rc;
  hipStream_t st;
  hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  if (e != hipSuccess) return fail(K2H_AMD_EHIP, "hipStreamCreate", e);
  void* dbuf[4] = {nullptr, nullptr, nullptr, nullptr};
  uint64_t* doff[4] = {nullptr, nullptr, nullptr, nullptr};
  uint8_t* dout = nullptr;
  uint64_t* dblob = nullptr;
  k2h::RalleInputs in;
  const uint8_t** bp[4] = {&in.keys, &in.vals, &in.skeys, &in.attrs};
  const uint64_t** op[4] = {&in.koff, &in.voff, &in.soff, &in.aoff};
  for (int s = 0; s < 4 && e == hipSuccess; ++s) {
    if (!off[s]) continue;
    uint64_t lo = off[s][0], len = off[s][n] - lo;
    e = hipMallocAsync((void**)&doff[s], (n + 1) * 8, st);
    if (e == hipSuccess) e = hipMemcpyAsync(doff[s], off[s], (n + 1) * 8, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMallocAsync(&dbuf[s], len ? len : 1, st);
    if (e == hipSuccess && len) e = hipMemcpyAsync(dbuf[s], (const uint8_t*)src[s] + lo, len, hipMemcpyHostToDevice, st);
    *bp[s] = (const uint8_t*)dbuf[s] - lo;  // kernel indexes with the caller's raw offsets
    *op[s] = doff[s];
  }
  if (e == hipSuccess) e = hipMallocAsync((void**)&dout, total, st);
  if (e == hipSuccess && blob_off) e = hipMallocAsync((void**)&dblob, (n + 1) * 8, st);
  if (e == hipSuccess) e = k2h::launch_ralledata(in, n, seed_for(flags), dout, dblob, st);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, total, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && blob_off) e = hipMemcpyAsync(blob_off, dblob, (n + 1) * 8, hipMemcpyDeviceToHost, st);
  for (int s = 0; s < 4; ++s) {
    if (dbuf[s]) (void)hipFreeAsync(dbuf[s], st);
    if (doff[s]) (void)hipFreeAsync(doff[s], st);
  }
  if (dout) (void)hipFreeAsync(dout, st);
  if (dblob) (void)hipFreeAsync(dblob, st);
  hipError_t f = hipStreamSynchronize(st);
  (void)hipStreamDestroy(st);
  if (e == hipSuccess) e = f;
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "build_ralledata_host", e);
}

__attribute__((visibility("default"))) const char* k2h_amd_version(void) {
  return "k2hash_amd 0.1 (FNV-1A BUILTIN, gfx950 HIP batch kernels)";
}

__attribute__((visibility("default"))) const char* k2h_amd_strerror(int code) {
  static const char* names[] = {"ok", "invalid argument", "HIP runtime error", "out of memory", "no device"};
  if (code == 0) return names[0];
  if (g_err[0]) return g_err;
  if (code < 0 && code >= -4) return names[-code];
  return "unknown error";
}


__attribute__((visibility("default"))) int k2h_amd_synth_bytes(void* out, uint64_t nbytes, uint64_t seed,
                                                               uint64_t byte_off, void* stream) {
  if (nbytes && !out) return fail(K2H_AMD_EINVAL, "out is NULL");
  K2H_GATE();
  hipError_t e = k2h::launch_synth_bytes((uint8_t*)out, nbytes, seed, byte_off, (hipStream_t)stream);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "synth_bytes", e);
}

__attribute__((visibility("default"))) int k2h_amd_synth_lengths(uint32_t* lens, uint64_t n, uint64_t seed,
                                                                 uint64_t first_key, uint32_t min_len,
                                                                 uint32_t max_len, void* stream) {
  if (n && !lens) return fail(K2H_AMD_EINVAL, "lens is NULL");
  if (max_len < min_len) return fail(K2H_AMD_EINVAL, "max_len < min_len");
  K2H_GATE();
  hipError_t e = k2h::launch_synth_lengths(lens, n, seed, first_key, min_len, max_len, (hipStream_t)stream);
  return e == hipSuccess ? K2H_AMD_OK : fail(K2H_AMD_EHIP, "synth_lengths", e);
}

}  // extern "C"
