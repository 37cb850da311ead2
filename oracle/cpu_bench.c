/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU-baseline harness for bench.py's `cpu_baseline` leg.  Times the REFERENCE's
 * own k2h_hash / k2h_second_hash (oracle/_ref/libk2hfunc_ref.so, resolved with
 * dlopen/dlsym as K2HashDynLib::Load does, lib/k2hashfunc.cc:142-151) -- or, when
 * that build is absent, the C restatement in fnv_oracle.c ("port") -- on the
 * host cores of the GPU box.
 *
 *   cpu_bench_fixed      scalar calls over the exact fixed-length workload the
 *                        GPU hashes (one contiguous shard per thread).
 *   cpu_bench_k2hbench   restatement of k2hbench's per-operation hash path
 *                        (tests/k2hbench.cc:878-983, `-type rw`): per loop the key
 *                        "KEY-%016X" + NUL (tests/k2hbench.cc:44, 946-953) is hashed
 *                        (h1 + h2) 4x for Set (lib/k2hshm.cc:2106-2107, 2151,
 *                        2184-2185) and 1x for Get (lib/k2hshm.cc:1230-1231).
 *                        libk2hash itself (and so k2hbench) is unbuildable here:
 *                        it needs libfullock (configure.ac:297-312).
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef uint64_t (*hash_fn)(const void*, size_t);

uint64_t oracle_k2h_hash(const void* ptr, size_t length, int variant);
uint64_t oracle_k2h_second_hash(const void* ptr, size_t length, int variant);

static uint64_t port_h1(const void* p, size_t n) { return oracle_k2h_hash(p, n, 0); }
static uint64_t port_h2(const void* p, size_t n) { return oracle_k2h_second_hash(p, n, 0); }

static int resolve(const char* so, hash_fn* h1, hash_fn* h2) {
  if (!so || !*so) {
    *h1 = port_h1;
    *h2 = port_h2;
    return 0;
  }
  void* lib = dlopen(so, RTLD_LAZY);
  if (!lib) return -1;
  *h1 = (hash_fn)dlsym(lib, "k2h_hash");
  *h2 = (hash_fn)dlsym(lib, "k2h_second_hash");
  return (*h1 && *h2) ? 0 : -1;
}

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

struct fixed_job {
  hash_fn h1, h2;
  const uint8_t* keys;
  uint64_t key_len, first, count;
  int passes, want_h2;
  uint64_t digest;
  pthread_barrier_t *ready, *go;
};

static void* fixed_worker(void* a) {
  struct fixed_job* j = (struct fixed_job*)a;
  uint64_t d = 0;
  pthread_barrier_wait(j->ready); /* started and parked: thread creation is outside the clock */
  pthread_barrier_wait(j->go);
  for (int p = 0; p < j->passes; ++p) {
    const uint8_t* k = j->keys + j->first * j->key_len;
    for (uint64_t i = 0; i < j->count; ++i, k += j->key_len) {
      d ^= j->h1(k, j->key_len);
      if (j->want_h2) d ^= j->h2(k, j->key_len) * 3;
    }
  }
  j->digest = d;
  return NULL;
}

/* Returns wall seconds over all threads from the release of the parked workers to the last
 * join (`passes` passes over each thread's shard), or < 0 on error.  *digest = xor of
 * per-thread digests. */
double cpu_bench_fixed(const char* so, const uint8_t* keys, uint64_t key_len, uint64_t n, int threads, int passes,
                       int want_h2, uint64_t* digest) {
  hash_fn h1, h2;
  if (resolve(so, &h1, &h2)) return -1.0;
  if (threads < 1) threads = 1;
  struct fixed_job* jobs = (struct fixed_job*)calloc((size_t)threads, sizeof *jobs);
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof *th);
  pthread_barrier_t ready, go;
  pthread_barrier_init(&ready, NULL, (unsigned)threads + 1);
  pthread_barrier_init(&go, NULL, (unsigned)threads + 1);
  for (int t = 0; t < threads; ++t) {
    uint64_t a = n * (uint64_t)t / (uint64_t)threads, b = n * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t] = (struct fixed_job){h1, h2, keys, key_len, a, b - a, passes, want_h2, 0, &ready, &go};
    pthread_create(&th[t], NULL, fixed_worker, &jobs[t]);
  }
  pthread_barrier_wait(&ready);
  double t0 = now();
  pthread_barrier_wait(&go);
  uint64_t d = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    d ^= jobs[t].digest;
  }
  double dt = now() - t0;
  pthread_barrier_destroy(&ready);
  pthread_barrier_destroy(&go);
  free(jobs);
  free(th);
  if (digest) *digest = d;
  return dt;
}

struct bench_job {
  hash_fn h1, h2;
  int loops, dcount, start;
  double seconds;
  uint64_t digest;
  pthread_barrier_t* bar;
};

static void* bench_worker(void* a) {
  struct bench_job* j = (struct bench_job*)a;
  char key[48]; /* KEY_BUFF_LENGTH, tests/k2hbench.cc:46 */
  uint64_t d = 0;
  int keynum = j->start;
  pthread_barrier_wait(j->bar);
  double t0 = now();
  for (int cnt = 0; cnt < j->loops; ++cnt) {
    int len = snprintf(key, sizeof key, "KEY-%016X", keynum) + 1; /* char* callers hash strlen+1 */
    if (j->dcount <= ++keynum) keynum = 0;
    for (int r = 0; r < 5; ++r) { /* Set: 4x (h1+h2), Get: 1x (h1+h2) */
      d += j->h1(key, (size_t)len);
      d += j->h2(key, (size_t)len);
    }
  }
  j->seconds = now() - t0;
  j->digest = d;
  return NULL;
}

/* Returns the slowest thread's seconds (k2hbench times each thread, tests/k2hbench.cc:937-976). */
double cpu_bench_k2hbench(const char* so, int loops, int dcount, int threads, uint64_t* digest) {
  hash_fn h1, h2;
  if (resolve(so, &h1, &h2)) return -1.0;
  if (threads < 1) threads = 1;
  if (dcount < 1) dcount = 1;
  struct bench_job* jobs = (struct bench_job*)calloc((size_t)threads, sizeof *jobs);
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof *th);
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)threads);
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (struct bench_job){h1, h2, loops, dcount, (int)((t * 7919u) % (unsigned)dcount), 0.0, 0, &bar};
    pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
  }
  double worst = 0.0;
  uint64_t d = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].seconds > worst) worst = jobs[t].seconds;
    d ^= jobs[t].digest;
  }
  pthread_barrier_destroy(&bar);
  free(jobs);
  free(th);
  if (digest) *digest = d;
  return worst;
}

struct csr_job {
  hash_fn h1, h2;
  const uint8_t* bytes;
  const uint64_t* off;
  uint64_t first, count;
  int passes, want_h2;
  uint64_t digest;
  pthread_barrier_t *ready, *go;
};

static void* csr_worker(void* a) {
  struct csr_job* j = (struct csr_job*)a;
  uint64_t d = 0;
  pthread_barrier_wait(j->ready);
  pthread_barrier_wait(j->go);
  for (int p = 0; p < j->passes; ++p) {
    uint64_t x = 0;
    for (uint64_t i = j->first; i < j->first + j->count; ++i) {
      const uint8_t* k = j->bytes + j->off[i];
      const size_t len = (size_t)(j->off[i + 1] - j->off[i]);
      x ^= j->h1(k, len);
      if (j->want_h2) x ^= j->h2(k, len) * 3;
    }
    if (p == 0) d = x; /* digest of one pass (xor of h1 over the shard) */
  }
  j->digest = d;
  return NULL;
}

/* CSR keys (bytes + n+1 offsets): the exact config-3 input, one contiguous shard of about
 * equal BYTES per thread (cut on key boundaries).  Returns wall seconds from the release
 * of the parked workers to the last join over `passes` passes; *digest = xor of h1 over
 * the n keys (one pass). */
double cpu_bench_csr(const char* so, const uint8_t* bytes, const uint64_t* off, uint64_t n, int threads, int passes,
                     int want_h2, uint64_t* digest) {
  hash_fn h1, h2;
  if (resolve(so, &h1, &h2)) return -1.0;
  if (threads < 1) threads = 1;
  struct csr_job* jobs = (struct csr_job*)calloc((size_t)threads, sizeof *jobs);
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof *th);
  pthread_barrier_t ready, go;
  pthread_barrier_init(&ready, NULL, (unsigned)threads + 1);
  pthread_barrier_init(&go, NULL, (unsigned)threads + 1);
  const uint64_t total = off[n] - off[0];
  uint64_t a = 0;
  for (int t = 0; t < threads; ++t) {
    /* first key whose start is at or past the t+1-th byte quantile */
    uint64_t want = off[0] + total / (uint64_t)threads * (uint64_t)(t + 1), lo = a, hi = n;
    if (t + 1 == threads) lo = n;
    while (lo < hi) {
      uint64_t mid = lo + (hi - lo) / 2;
      if (off[mid] < want) lo = mid + 1;
      else hi = mid;
    }
    jobs[t] = (struct csr_job){h1, h2, bytes, off, a, lo - a, passes, want_h2, 0, &ready, &go};
    a = lo;
    pthread_create(&th[t], NULL, csr_worker, &jobs[t]);
  }
  pthread_barrier_wait(&ready);
  double t0 = now();
  pthread_barrier_wait(&go);
  uint64_t d = 0;
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    d ^= jobs[t].digest;
  }
  double dt = now() - t0;
  pthread_barrier_destroy(&ready);
  pthread_barrier_destroy(&go);
  free(jobs);
  free(th);
  if (digest) *digest = d;
  return dt;
}
