/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Golden-fixture generator.  Runs the REFERENCE's own hash functions, compiled
 * from /root/reference/lib/k2hashfunc.cc into oracle/_ref/ by oracle/Makefile,
 * resolved with dlopen/dlsym exactly as K2HashDynLib::Load does
 * (lib/k2hashfunc.cc:142-151), and writes:
 *
 *   tests/golden/vectors.json  known-answer vectors: the SURVEY.md 8(a) table,
 *                              seeded random keys of every length 0..300 plus
 *                              long keys, k2hbench keys "KEY-%016X\0"
 *                              (tests/k2hbench.cc:44,946-953) and uniq keys
 *                              "KEY-%016X-%016X\0" (tests/k2hbench.cc:45,947),
 *                              for the default and the STD::FNV build.
 *   tests/golden/digests.json  order-sensitive digests (oracle_digest) of h1/h2
 *                              over the full-size synthetic workloads of
 *                              BASELINE.json configs 2-5.
 *
 * usage: gen_golden <ref.so> <ref_stdfnv.so> <out_dir> [quick]
 * Inputs come from the generator in fnv_oracle.c (linked in); hashes come only
 * from the reference library.
 */
#include <dlfcn.h>
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef uint64_t (*hash_fn)(const void*, size_t);
typedef const char* (*ver_fn)(void);

void oracle_gen_bytes(uint64_t seed, uint64_t byte_off, size_t nbytes, uint8_t* out);
void oracle_gen_offsets(uint64_t seed, uint64_t first_key, size_t n, uint32_t min_len,
                        uint32_t max_len, uint64_t base, uint64_t* offsets);
uint64_t oracle_splitmix_word(uint64_t seed, uint64_t j);

#define SEED_BYTES 0x6B32686173680001ULL
#define SEED_LENS 0x6B32686173680002ULL
#define SEED_VEC 0x6B32686173680003ULL

struct ref {
  hash_fn h1, h2;
  ver_fn ver;
};

static struct ref load_ref(const char* path) {
  struct ref r;
  void* so = dlopen(path, RTLD_LAZY);
  if (!so) {
    fprintf(stderr, "dlopen %s: %s\n", path, dlerror());
    exit(2);
  }
  r.h1 = (hash_fn)dlsym(so, "k2h_hash");
  r.h2 = (hash_fn)dlsym(so, "k2h_second_hash");
  r.ver = (ver_fn)dlsym(so, "k2h_hash_version");
  if (!r.h1 || !r.h2 || !r.ver) {
    fprintf(stderr, "dlsym failed in %s\n", path);
    exit(2);
  }
  return r;
}

static void put_hex(FILE* f, const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  fputc('"', f);
  for (size_t i = 0; i < n; ++i) {
    fputc(d[p[i] >> 4], f);
    fputc(d[p[i] & 15], f);
  }
  fputc('"', f);
}

static int first_vec;
static void emit(FILE* f, const char* tag, const uint8_t* p, size_t n, struct ref* r) {
  uint64_t a = r->h1(p, n), b = r->h2(p, n);
  fprintf(f, "%s\n    {\"tag\": \"%s\", \"len\": %zu, \"key\": ", first_vec ? "" : ",", tag, n);
  put_hex(f, p, n);
  fprintf(f, ", \"h1\": \"%016" PRIx64 "\", \"h2\": \"%016" PRIx64 "\"}", a, b);
  first_vec = 0;
}

static void emit_vectors(FILE* f, struct ref* r, int full) {
  uint8_t buf[8192];
  first_vec = 1;
  fprintf(f, "[");
  /* SURVEY.md 8(a) table */
  emit(f, "empty", (const uint8_t*)"", 0, r);
  emit(f, "a", (const uint8_t*)"a", 1, r);
  emit(f, "ab", (const uint8_t*)"ab", 2, r);
  emit(f, "k2hexttest", (const uint8_t*)"0123456789", 10, r); /* tests/k2hexttest.cc:166-175 */
  emit(f, "dsave key1", (const uint8_t*)"key1", 5, r);        /* tests/test_linetool_dsave.cmd:29-50 */
  emit(f, "dsave key27", (const uint8_t*)"key27", 6, r);
  {
    static const uint8_t b80[] = {0x80}, b00[] = {0x00}, mix4[] = {0x80, 0xff, 0x7f, 0x00};
    emit(f, "0x80", b80, 1, r);
    emit(f, "0x00", b00, 1, r);
    emit(f, "80ff7f00", mix4, 4, r);
  }
  memset(buf, 0, 32);
  emit(f, "32x00", buf, 32, r);
  memset(buf, 0xff, 32);
  emit(f, "32xff", buf, 32, r);
  memset(buf, 0x80, 64);
  emit(f, "64x80", buf, 64, r);
  for (int i = 0; i < 256; ++i) buf[i] = (uint8_t)i;
  emit(f, "bytes00..ff", buf, 256, r);
  for (int i = 0; i < 4096; ++i) buf[i] = (uint8_t)((i * 131 + 7) & 0xff);
  emit(f, "i*131+7 x4096", buf, 4096, r);
  /* seeded random keys, every length 0..300 (full byte range: half the
   * bytes take the sign-extension path) */
  for (size_t len = 0; len <= (full ? 300u : 64u); ++len) {
    oracle_gen_bytes(SEED_VEC, len * 1000, len, buf);
    emit(f, "rand", buf, len, r);
  }
  if (!full) {
    fprintf(f, "\n  ]");
    return;
  }
  /* high-bit-only keys (every byte >= 0x80) */
  for (size_t len = 1; len <= 40; ++len) {
    oracle_gen_bytes(SEED_VEC ^ 0xff, len * 1000, len, buf);
    for (size_t i = 0; i < len; ++i) buf[i] |= 0x80;
    emit(f, "rand-high", buf, len, r);
  }
  /* long keys */
  static const size_t longs[] = {511, 512, 513, 1000, 1023, 1024, 1025, 2047, 4095, 4096, 4097, 8000};
  for (size_t j = 0; j < sizeof(longs) / sizeof(longs[0]); ++j) {
    oracle_gen_bytes(SEED_VEC, 7000000 + j * 10000, longs[j], buf);
    emit(f, "rand-long", buf, longs[j], r);
  }
  /* k2hbench keys: sprintf("KEY-%016X") + NUL, tests/k2hbench.cc:44, 946-953 */
  for (int i = 0; i < 1000; ++i) {
    char k[64];
    int n = snprintf(k, sizeof k, "KEY-%016X", i);
    emit(f, "k2hbench", (const uint8_t*)k, (size_t)n + 1, r);
  }
  /* uniq keys: "KEY-%016X-%016X" + NUL, tests/k2hbench.cc:45, 947 */
  for (int i = 0; i < 50; ++i) {
    char k[64];
    int n = snprintf(k, sizeof k, "KEY-%016X-%016X", 1234, i);
    emit(f, "k2hbench-uniq", (const uint8_t*)k, (size_t)n + 1, r);
  }
  fprintf(f, "\n  ]");
}

/* ---------------- digests over the full-size workloads ---------------- */
struct job {
  struct ref* r;
  int kind; /* 0 fixed, 1 csr */
  uint64_t key_len, first, count;
  uint32_t min_len, max_len;
  uint64_t d1[3], d2[3];
};

static void* run_job(void* arg) {
  struct job* j = (struct job*)arg;
  uint8_t* buf = (uint8_t*)malloc(1 << 16);
  uint64_t x1 = 0, s1 = 0, w1 = 0, x2 = 0, s2 = 0, w2 = 0;
  uint64_t off = 0;
  if (j->kind == 1) {
    /* absolute start offset of key `first`: sum of the preceding lengths */
    uint64_t span = (uint64_t)(j->max_len - j->min_len) + 1;
    for (uint64_t i = 0; i < j->first; ++i) off += j->min_len + oracle_splitmix_word(SEED_LENS, i) % span;
  }
  for (uint64_t t = 0; t < j->count; ++t) {
    uint64_t i = j->first + t, len, start;
    if (j->kind == 0) {
      len = j->key_len;
      start = i * j->key_len;
    } else {
      uint64_t span = (uint64_t)(j->max_len - j->min_len) + 1;
      len = j->min_len + oracle_splitmix_word(SEED_LENS, i) % span;
      start = off;
      off += len;
    }
    oracle_gen_bytes(SEED_BYTES, start, len, buf);
    uint64_t a = j->r->h1(buf, len), b = j->r->h2(buf, len);
    x1 ^= a; s1 += a; w1 += a * (2 * i + 1);
    x2 ^= b; s2 += b; w2 += b * (2 * i + 1);
  }
  j->d1[0] = x1; j->d1[1] = s1; j->d1[2] = w1;
  j->d2[0] = x2; j->d2[1] = s2; j->d2[2] = w2;
  free(buf);
  return NULL;
}

/* digest of keys [0, n) computed in `chunks` pieces (each reported), threads in parallel */
static void digest_config(FILE* f, const char* name, struct ref* r, int kind, uint64_t key_len,
                          uint64_t n, uint32_t min_len, uint32_t max_len, int chunks, int first) {
  int T = chunks;
  struct job* jobs = (struct job*)calloc((size_t)T, sizeof(struct job));
  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  for (int c = 0; c < T; ++c) {
    jobs[c].r = r; jobs[c].kind = kind; jobs[c].key_len = key_len;
    jobs[c].first = n / (uint64_t)T * (uint64_t)c;
    jobs[c].count = n / (uint64_t)T;
    jobs[c].min_len = min_len; jobs[c].max_len = max_len;
    pthread_create(&th[c], NULL, run_job, &jobs[c]);
  }
  for (int c = 0; c < T; ++c) pthread_join(th[c], NULL);
  uint64_t t1[3] = {0, 0, 0}, t2[3] = {0, 0, 0};
  fprintf(f, "%s\n    \"%s\": {\"kind\": \"%s\", \"n\": %" PRIu64 ", \"key_len\": %" PRIu64
             ", \"min_len\": %u, \"max_len\": %u, \"seed_bytes\": \"%016llx\", \"seed_lens\": \"%016llx\", \"chunks\": [",
          first ? "" : ",", name, kind ? "csr" : "fixed", n, key_len, min_len, max_len,
          (unsigned long long)SEED_BYTES, (unsigned long long)SEED_LENS);
  for (int c = 0; c < T; ++c) {
    fprintf(f, "%s{\"first\": %" PRIu64 ", \"count\": %" PRIu64 ", \"h1\": [\"%016" PRIx64 "\", \"%016" PRIx64
               "\", \"%016" PRIx64 "\"], \"h2\": [\"%016" PRIx64 "\", \"%016" PRIx64 "\", \"%016" PRIx64 "\"]}",
            c ? ", " : "", jobs[c].first, jobs[c].count, jobs[c].d1[0], jobs[c].d1[1], jobs[c].d1[2],
            jobs[c].d2[0], jobs[c].d2[1], jobs[c].d2[2]);
    t1[0] ^= jobs[c].d1[0]; t1[1] += jobs[c].d1[1]; t1[2] += jobs[c].d1[2];
    t2[0] ^= jobs[c].d2[0]; t2[1] += jobs[c].d2[1]; t2[2] += jobs[c].d2[2];
  }
  fprintf(f, "], \"h1\": [\"%016" PRIx64 "\", \"%016" PRIx64 "\", \"%016" PRIx64 "\"], \"h2\": [\"%016" PRIx64
             "\", \"%016" PRIx64 "\", \"%016" PRIx64 "\"]}",
          t1[0], t1[1], t1[2], t2[0], t2[1], t2[2]);
  fflush(f);
  free(jobs);
  free(th);
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <ref.so> <ref_stdfnv.so> <out_dir> [quick]\n", argv[0]);
    return 2;
  }
  int quick = argc > 4 && !strcmp(argv[4], "quick");
  struct ref r = load_ref(argv[1]);
  struct ref rs = load_ref(argv[2]);
  char path[4096];

  snprintf(path, sizeof path, "%s/vectors.json", argv[3]);
  FILE* f = fopen(path, "w");
  if (!f) { perror(path); return 2; }
  fprintf(f, "{\n  \"generator\": \"oracle/gen_golden.c over oracle/_ref (reference lib/k2hashfunc.cc)\",\n");
  fprintf(f, "  \"version\": \"%s\",\n  \"vectors\": ", r.ver());
  emit_vectors(f, &r, 1);
  fprintf(f, ",\n  \"std_fnv_version\": \"%s\",\n  \"std_fnv_vectors\": ", rs.ver());
  emit_vectors(f, &rs, 0);
  fprintf(f, "\n}\n");
  fclose(f);

  snprintf(path, sizeof path, "%s/digests.json", argv[3]);
  f = fopen(path, "w");
  if (!f) { perror(path); return 2; }
  fprintf(f, "{\n  \"generator\": \"oracle/gen_golden.c over oracle/_ref (reference lib/k2hashfunc.cc)\",\n");
  fprintf(f, "  \"digest\": \"[xor, wrapping sum, wrapping sum of h*(2i+1)] over keys, i = global key index\",\n");
  fprintf(f, "  \"configs\": {");
  digest_config(f, "fixed32_64K", &r, 0, 32, 1ull << 16, 0, 0, 1, 1);
  digest_config(f, "csr_8_256_64K", &r, 1, 0, 1ull << 16, 8, 256, 1, 0);
  digest_config(f, "fixed21_1M", &r, 0, 21, 1ull << 20, 0, 0, 8, 0);
  if (!quick) {
    digest_config(f, "fixed32_16M", &r, 0, 32, 1ull << 24, 0, 0, 8, 0);            /* config 2 */
    digest_config(f, "csr_8_256_64M", &r, 1, 0, 1ull << 26, 8, 256, 8, 0);         /* config 3 */
    digest_config(f, "fixed4096_1M", &r, 0, 4096, 1ull << 20, 0, 0, 8, 0);         /* config 5 */
    digest_config(f, "fixed32_1G", &r, 0, 32, 1ull << 30, 0, 0, 8, 0);             /* config 4 (8 shards) */
  }
  fprintf(f, "\n  }\n}\n");
  fclose(f);
  return 0;
}
