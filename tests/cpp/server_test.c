/*
 * server_test.c -- concurrent callers of the resident build service (mde_server_build and
 * mde_server_verify), in plain
 * C through include/mde.h, checked bit for bit against mde_build on a shared context and the C
 * oracle (oracle/mde_oracle.c, test infrastructure).
 *
 *   server_test [threads] [calls_per_thread] [lifetime_ms]      defaults: 10 40 100
 *
 * The reference builds ONE partition per VerifyEpoch (main/manager.go:1036 ->
 * RawPartitionMerkleTree, main/merkle_tree.go:86-116) on up to partition_concurrency = 10
 * workers (config/default-config.yaml:9). Every thread starts its calls at a barrier so they
 * overlap. Calls vary: bucket counts 1, 2, 30, 64, 1000 (the default) and 1024 (the service's
 * largest by default); 4096 and inputs beyond a slot's 256 KiB run on the service's context;
 * 8-byte timestamps (main/manager.go:816), variable-length values and variable offsets that
 * happen to be uniform (sent as a stride), records outside the bucket ranges, empty partitions,
 * two or three partitions in one call, full builds with and without inner nodes and digest-only
 * builds (root NULL), and the split tree (mde_server_build_levels, the device's levels up to the
 * first of at most 1 / 2 / 16 / 64 / 300 nodes); after every one-partition build, the VerifyEpoch decision step through the
 * service (mde_server_verify) against mde_verify_epochs. With a short lifetime (third argument) the launch ends and relaunches many
 * times while calls are in flight; a final phase sleeps past the lifetime between calls. Prints
 * one JSON line; exit 0 iff every output matched.
 */
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mde.h"

/* oracle/mde_oracle.c */
int oracle_build(const uint8_t* values, uint32_t stride, const uint64_t* value_off, const uint64_t* seg_rec,
                 uint32_t n_partitions, uint32_t n_buckets, uint64_t* digest, int32_t* size, int32_t* items,
                 uint8_t* root, uint8_t* nodes, int threads);

static mde_server* server;
static mde_ctx* ctx; /* per-call reference path, shared by all threads (the context locks) */
static pthread_barrier_t start;
static int n_calls = 40;
static long mismatches = 0, checked = 0, verified = 0;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;

static uint64_t rng(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void* xmalloc(size_t n) {
  void* p = calloc(1, n ? n : 1);
  if (!p) {
    fprintf(stderr, "allocation failed\n");
    exit(1);
  }
  return p;
}

static void bad(const char* what, int t, int k, uint32_t P, uint32_t B) {
  pthread_mutex_lock(&mu);
  if (mismatches < 20) fprintf(stderr, "mismatch: %s (thread %d call %d, P=%u B=%u)\n", what, t, k, P, B);
  mismatches++;
  pthread_mutex_unlock(&mu);
}

/* The VerifyEpoch decision step for the partition just built (digests d, sizes z): peers that
 * agree, differ in one bucket, are absent, are garbage, carry another bucket count (every third
 * call), and every seventh call 20 peers (beyond the service's 16: its context). The service's
 * answer == mde_verify_epochs on the shared context. */
static void verify_call(int t, int k, uint32_t B, const uint64_t* d, const int32_t* z, uint64_t* s) {
  char err[256];
  const uint64_t stride_o = mde_epoch_tree_object_max_bytes(B + 2);
  uint8_t* peers = xmalloc(2 * stride_o + 64);
  uint32_t plen[2];
  uint64_t* dp = xmalloc((B + 2) * 8ull);
  int32_t* zp = xmalloc((B + 2) * 4ull);
  memcpy(dp, d, B * 8ull);
  memcpy(zp, z, B * 4ull);
  const int32_t part = t * 100 + k;
  const int64_t epoch = 7 + (k % 2);
  if (mde_encode_epoch_tree_objects(ctx, 1, B, &part, epoch, epoch + 1, dp, zp, NULL, NULL, peers, stride_o, plen))
    exit(1);
  const uint32_t pb = (k % 3 == 2) ? B + 2 : B; /* other-shape peer */
  for (uint32_t b = B; b < pb; b++) {
    dp[b] = rng(s) % 999999u;
    zp[b] = 1;
  }
  dp[(uint32_t)k % B] = (dp[(uint32_t)k % B] + 1) % 999999u;
  if (mde_encode_epoch_tree_objects(ctx, 1, pb, &part, epoch, epoch + 1, dp, zp, NULL, NULL, peers + plen[0], stride_o,
                                    plen + 1))
    exit(1);
  const uint32_t R = (k % 7 == 6) ? 20u : (k % 2) ? 4u : 3u;
  uint64_t* off = xmalloc((R + 1) * 8ull);
  const uint32_t glen = 9; /* garbage: a truncated varint field */
  memset(peers + plen[0] + plen[1], 0xff, glen);
  off[0] = 0;
  for (uint32_t r = 0; r < R; r++) { /* agreeing, differing, absent, garbage, then agreeing again */
    const uint32_t kind = r < 4 ? r : 0;
    off[r + 1] = off[r] + (kind == 0 ? plen[0] : kind == 1 ? plen[1] : kind == 2 ? 0 : glen);
  }
  /* lay the peer bytes out in that order */
  uint8_t* blob = xmalloc(off[R] + 1);
  for (uint32_t r = 0; r < R; r++) {
    const uint32_t kind = r < 4 ? r : 0;
    const uint8_t* src = kind == 0 ? peers : kind == 1 ? peers + plen[0] : peers + plen[0] + plen[1];
    memcpy(blob + off[r], src, off[r + 1] - off[r]);
  }
  const int want_obj = k % 4 != 3;
  const uint64_t ostride = want_obj ? mde_epoch_tree_object_max_bytes(B) : 0;
  uint8_t va = 0, vb = 0;
  int32_t ca = 0, cb = 0, na = 0, nb = 0;
  int32_t *sa = xmalloc(R * 4ull), *sb = xmalloc(R * 4ull);
  int32_t *ia = xmalloc(B * 4ull), *ib = xmalloc(B * 4ull);
  uint8_t *oa = xmalloc(ostride), *ob = xmalloc(ostride);
  uint32_t la = 0, lb = 0;
  int rc = mde_server_verify(server, B, part, epoch, d, z, R, blob, off, 2, &va, &ca, ia, &na, sa,
                             want_obj ? oa : NULL, ostride, want_obj ? &la : NULL, err, sizeof err);
  if (rc) {
    fprintf(stderr, "mde_server_verify: %d %s\n", rc, err);
    exit(1);
  }
  if ((rc = mde_verify_epochs(ctx, 1, B, &part, epoch, d, z, NULL, R, blob, off, 2, &vb, &cb, ib, &nb, sb,
                              want_obj ? ob : NULL, ostride, want_obj ? &lb : NULL))) {
    fprintf(stderr, "mde_verify_epochs: %d\n", rc);
    exit(1);
  }
  if (va != vb || ca != cb || na != nb || memcmp(ia, ib, (size_t)(na > 0 ? na : 0) * 4) || memcmp(sa, sb, R * 4) ||
      la != lb || memcmp(oa, ob, la))
    bad("verify", t, k, 1, B);
  /* an even-B same-shape peer differing in one bucket: diffSet = that bucket (an odd-B object carries
   * the duplicate leaf, B + 1 buckets: the DFS then errors, as the reference's does) */
  if (pb == B && B % 2 == 0 && (na != 1 || ia[0] != (int32_t)((uint32_t)k % B))) bad("verify diff", t, k, 1, B);
  if (sa[0] != 0 || (R > 3 && sa[3] != MDE_E_DECODE)) bad("peer status", t, k, 1, B);
  pthread_mutex_lock(&mu);
  verified++;
  pthread_mutex_unlock(&mu);
  free(peers), free(dp), free(zp), free(off), free(blob), free(sa), free(sb), free(ia), free(ib), free(oa), free(ob);
}

/* One call of shape (t, k): build through the service, mde_build and the oracle; compare. */
static void one_call(int t, int k) {
  char err[256];
  uint64_t s = 0x5e77ull * 1000003u + (uint64_t)t * 7919u + (uint64_t)k;
  static const uint32_t Bs[8] = {1000, 64, 30, 1, 2, 1024, 1000, 4096};
  const uint32_t B = Bs[(t + 3 * k) % 8];
  const uint32_t P = (k % 7 == 5) ? 2u + (uint32_t)(k % 2) : 1u;
  const int kind = k % 5; /* 0,1: 8-byte; 2: variable; 3: variable but uniform (13 B); 4: empty or big */
  uint64_t n = 100 + rng(&s) % 3000;
  if (kind == 4) n = (k % 10 == 4) ? 0 : 40000; /* 40k x 8 B = 320 KB: beyond a slot */
  const uint64_t lead = (k % 3 == 1) ? 3 : 0, tail = (k % 3 == 1) ? 2 : 0;
  const uint64_t nr = n + lead + tail;
  uint64_t* voff = NULL;
  uint64_t bytes;
  uint32_t stride = 0;
  if (kind == 2 || kind == 3) {
    voff = xmalloc((nr + 1) * 8);
    for (uint64_t i = 0; i < nr; i++) voff[i + 1] = voff[i] + (kind == 3 ? 13 : rng(&s) % 41);
    bytes = voff[nr];
  } else {
    stride = 8;
    bytes = nr * 8;
  }
  uint8_t* vals = xmalloc(bytes);
  for (uint64_t i = 0; i < bytes; i++) vals[i] = (uint8_t)rng(&s);
  const uint64_t S = (uint64_t)P * B;
  uint64_t* seg = xmalloc((S + 1) * 8);
  seg[0] = lead;
  for (uint64_t b = 1; b < S; b++) seg[b] = lead + rng(&s) % (n + 1);
  seg[S] = lead + n;
  for (uint64_t i = 1; i < S; i++) /* insertion sort of the cuts */
    for (uint64_t j = i; j > 1 && seg[j] < seg[j - 1]; j--) {
      const uint64_t x = seg[j];
      seg[j] = seg[j - 1];
      seg[j - 1] = x;
    }
  mde_records rec;
  memset(&rec, 0, sizeof rec);
  rec.values = bytes ? vals : NULL;
  rec.values_bytes = bytes;
  rec.value_stride = stride;
  rec.layout = MDE_LAYOUT_SORTED;
  rec.value_off = voff;
  rec.n_records = nr;
  rec.n_partitions = P;
  rec.n_buckets = B;
  rec.seg_rec = seg;
  const uint64_t NI = mde_tree_internal_nodes(B);
  uint64_t *d1 = xmalloc(S * 8), *d2 = xmalloc(S * 8), *d3 = xmalloc(S * 8);
  int32_t *z1 = xmalloc(S * 4), *z2 = xmalloc(S * 4), *z3 = xmalloc(S * 4);
  int32_t *i1 = xmalloc(P * 4), *i2 = xmalloc(P * 4), *i3 = xmalloc(P * 4);
  uint8_t *r1 = xmalloc(P * 32), *r2 = xmalloc(P * 32), *r3 = xmalloc(P * 32);
  uint8_t *n1 = xmalloc(P * NI * 32), *n2 = xmalloc(P * NI * 32), *n3 = xmalloc(P * NI * 32);
  const int shape = (k / 2) % 3; /* 0: root + nodes; 1: root only; 2: digest-only */
  mde_tree_out o1 = {d1, z1, i1, shape < 2 ? r1 : NULL, shape == 0 ? n1 : NULL};
  mde_tree_out o2 = {d2, z2, i2, shape < 2 ? r2 : NULL, shape == 0 ? n2 : NULL};
  int rc = mde_server_build(server, &rec, &o1, err, sizeof err);
  if (rc) {
    fprintf(stderr, "mde_server_build: %d %s\n", rc, err);
    exit(1);
  }
  if ((rc = mde_build(ctx, &rec, &o2))) {
    fprintf(stderr, "mde_build: %d %s\n", rc, mde_last_error(ctx));
    exit(1);
  }
  oracle_build(vals, stride, voff, seg, P, B, d3, z3, i3, r3, n3, 1);
  if (memcmp(d1, d2, S * 8) || memcmp(d1, d3, S * 8)) bad("digest", t, k, P, B);
  if (memcmp(z1, z2, S * 4) || memcmp(z1, z3, S * 4)) bad("size", t, k, P, B);
  if (memcmp(i1, i2, P * 4) || memcmp(i1, i3, P * 4)) bad("items", t, k, P, B);
  if (shape < 2 && (memcmp(r1, r2, P * 32) || memcmp(r1, r3, P * 32))) bad("root", t, k, P, B);
  if (shape == 0 && (memcmp(n1, n2, P * NI * 32) || memcmp(n1, n3, P * NI * 32))) bad("nodes", t, k, P, B);
  /* levels 1 .. the first of at most `top` nodes (mde_server_build_levels): that prefix of every
   * partition's nodes equals the oracle's */
  {
    static const uint32_t tops[5] = {64, 1, 2, 16, 300};
    const uint32_t top = tops[k % 5];
    uint8_t* n4 = xmalloc(P * NI * 32);
    uint64_t* d4 = xmalloc(S * 8);
    int32_t* z4 = xmalloc(S * 4);
    int32_t* i4 = xmalloc(P * 4);
    mde_tree_out o4 = {d4, z4, i4, NULL, n4};
    if ((rc = mde_server_build_levels(server, &rec, &o4, top, err, sizeof err))) {
      fprintf(stderr, "mde_server_build_levels: %d %s\n", rc, err);
      exit(1);
    }
    const uint64_t pre = mde_tree_prefix_nodes(B, top);
    for (uint32_t p = 0; p < P; p++)
      if (memcmp(n4 + (uint64_t)p * NI * 32, n3 + (uint64_t)p * NI * 32, pre * 32)) bad("levels", t, k, P, B);
    if (memcmp(d4, d3, S * 8) || memcmp(z4, z3, S * 4) || memcmp(i4, i3, P * 4)) bad("levels digests", t, k, P, B);
    free(n4), free(d4), free(z4), free(i4);
  }
  if (P == 1) verify_call(t, k, B, d3, z3, &s);
  pthread_mutex_lock(&mu);
  checked++;
  pthread_mutex_unlock(&mu);
  free(vals), free(voff), free(seg), free(d1), free(d2), free(d3), free(z1), free(z2), free(z3);
  free(i1), free(i2), free(i3), free(r1), free(r2), free(r3), free(n1), free(n2), free(n3);
}

static void* worker(void* arg) {
  const int t = (int)(intptr_t)arg;
  pthread_barrier_wait(&start);
  for (int k = 0; k < n_calls; k++) one_call(t, k);
  return NULL;
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 10;
  if (argc > 2) n_calls = atoi(argv[2]);
  const char* life = argc > 3 ? argv[3] : "100";
  setenv("MDE_SERVER_LIFETIME_MS", life, 1);
  const long life_ms = atol(life);
  /* SERVER_TEST_EARLY_CTX=1: a context created before the service, used, and destroyed after it
   * (the teardown order of a process whose other contexts outlive its services) */
  mde_ctx* early = NULL;
  if (getenv("SERVER_TEST_EARLY_CTX")) {
    if (mde_create(0, &early)) {
      fprintf(stderr, "mde_create (early): failed\n");
      return 1;
    }
    uint8_t v[64] = {1, 2, 3};
    uint64_t seg[3] = {0, 4, 8};
    uint64_t dig[2];
    int32_t sz[2], it;
    uint8_t root[32];
    mde_records r;
    memset(&r, 0, sizeof r);
    r.values = v;
    r.values_bytes = sizeof v;
    r.value_stride = 8;
    r.n_records = 8;
    r.n_partitions = 1;
    r.n_buckets = 2;
    r.seg_rec = seg;
    mde_tree_out o = {dig, sz, &it, root, NULL};
    if (mde_build(early, &r, &o)) {
      fprintf(stderr, "mde_build (early): %s\n", mde_last_error(early));
      return 1;
    }
  }
  int rc = mde_server_create(0, 0, 0, &server);
  if (rc) {
    fprintf(stderr, "mde_server_create: %d\n", rc);
    return 1;
  }
  if ((rc = mde_create(0, &ctx))) {
    fprintf(stderr, "mde_create: %d\n", rc);
    return 1;
  }
  pthread_barrier_init(&start, NULL, (unsigned)threads);
  pthread_t* th = xmalloc(sizeof(pthread_t) * (size_t)threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  /* idle past the lifetime between calls: every call finds the launch ended */
  uint64_t launches0 = 0, launches1 = 0, requests = 0, on_ctx = 0;
  mde_server_stats(server, NULL, &launches0, NULL);
  for (int k = 0; k < 6; k++) {
    const long ns = (life_ms % 1000) * 1000000L + 5000000L;
    struct timespec ts = {life_ms / 1000 + ns / 1000000000L, ns % 1000000000L};
    nanosleep(&ts, NULL);
    uint64_t l0 = 0, l1 = 0;
    mde_server_stats(server, NULL, &l0, NULL);
    /* a shape the resident launch serves: one partition, B <= 1024, inputs within a slot */
    int kk = 2 * k;
    while ((threads + 3 * kk) % 8 == 7 || kk % 5 == 4 || kk % 7 == 5) kk++;
    one_call(threads, kk);
    mde_server_stats(server, NULL, &l1, NULL);
    fprintf(stderr, "idle call %d: launches %" PRIu64 " -> %" PRIu64 "\n", k, l0, l1);
  }
  mde_server_stats(server, &requests, &launches1, &on_ctx);
  fprintf(stderr, "destroying the service\n");
  mde_server_destroy(server);
  fprintf(stderr, "service destroyed\n");
  mde_destroy(ctx);
  fprintf(stderr, "context destroyed\n");
  if (early) {
    mde_destroy(early);
    fprintf(stderr, "early context destroyed\n");
  }
  const int relaunched = launches1 >= launches0 + 6;
  printf("{\"server_test\": {\"threads\": %d, \"calls\": %ld, \"verifies\": %ld, \"mismatches\": %ld, \"requests\": %" PRIu64
         ", \"launches_before_idle\": %" PRIu64 ", \"launches\": %" PRIu64 ", \"on_context\": %" PRIu64
         ", \"lifetime_ms\": %ld, \"idle_relaunches_ok\": %s}}\n",
         threads, checked, verified, mismatches, requests, launches0, launches1, on_ctx, life_ms, relaunched ? "true" : "false");
  fflush(stdout);
  return (mismatches == 0 && relaunched && checked == (long)threads * n_calls + 6) ? 0 : 1;
}
