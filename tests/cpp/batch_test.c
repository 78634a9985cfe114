/*
 * batch_test.c -- concurrent callers of the batcher (mde_batch_build / mde_batch_verify), in
 * plain C through include/mde.h, checked bit for bit against the per-call entry points
 * (mde_build, mde_verify_epochs) and the C oracle (oracle/mde_oracle.c, test infrastructure).
 *
 *   batch_test [threads] [calls_per_thread]      defaults: 10 40
 *
 * The shape is the reference's: VerifyEpoch builds ONE partition per call
 * (main/manager.go:1036 -> RawPartitionMerkleTree, main/merkle_tree.go:86-116) on
 * workers_count goroutines with partition_concurrency = 10 in flight
 * (config/default-config.yaml:7,9). Every thread starts its calls at a barrier so they overlap.
 * Each call is one partition with its own bucket count (30, 64 or the default 1000: different
 * batches), 8-byte timestamp values (main/manager.go:816) or variable-length values, records
 * outside the bucket ranges in some arenas, and the decision step against peers that agree,
 * differ in one bucket, are absent, carry another bucket count or are garbage
 * (main/manager.go:1072-1104). Prints one JSON line; exit 0 iff every output matched and calls
 * were coalesced (fewer batches than requests).
 */
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mde.h"

/* oracle/mde_oracle.c */
int oracle_build(const uint8_t* values, uint32_t stride, const uint64_t* value_off, const uint64_t* seg_rec,
                 uint32_t n_partitions, uint32_t n_buckets, uint64_t* digest, int32_t* size, int32_t* items,
                 uint8_t* root, uint8_t* nodes, int threads);
uint64_t oracle_n_internal(uint32_t n_buckets);
int32_t oracle_diff(const uint64_t* d1, uint32_t b1, const uint64_t* d2, uint32_t b2, int32_t* out, int32_t cap);

static mde_batcher* batcher;
static mde_ctx* ctx; /* per-call reference path, shared by all threads (the context locks) */
static pthread_barrier_t start;
static int n_calls = 40;
static long mismatches = 0, verify_checked = 0, builds_checked = 0;
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

static void bad(const char* what, int t, int k) {
  pthread_mutex_lock(&mu);
  if (mismatches < 20) fprintf(stderr, "mismatch: %s (thread %d call %d)\n", what, t, k);
  mismatches++;
  pthread_mutex_unlock(&mu);
}

static void* worker(void* arg) {
  const int t = (int)(intptr_t)arg;
  char err[256];
  pthread_barrier_wait(&start);
  for (int k = 0; k < n_calls; k++) {
    uint64_t s = 0x5eedull * 1000003u + (uint64_t)t * 7919u + (uint64_t)k;
    const uint32_t Bs[3] = {30, 64, 1000};
    const uint32_t B = Bs[(t + k) % 3];
    const int variable = (k % 4) == 3;
    const uint64_t n = 100 + rng(&s) % 3000;
    const uint64_t lead = (k % 5 == 4) ? 3 : 0, tail = (k % 5 == 4) ? 2 : 0; /* records in no bucket */
    const uint64_t nr = n + lead + tail;
    uint64_t* voff = NULL;
    uint64_t bytes;
    uint32_t stride = 0;
    if (variable) {
      voff = xmalloc((nr + 1) * 8);
      for (uint64_t i = 0; i < nr; i++) voff[i + 1] = voff[i] + rng(&s) % 41;
      bytes = voff[nr];
    } else {
      stride = 8;
      bytes = nr * 8;
    }
    uint8_t* vals = xmalloc(bytes);
    for (uint64_t i = 0; i < bytes; i++) vals[i] = (uint8_t)rng(&s);
    uint64_t* seg = xmalloc(((uint64_t)B + 1) * 8);
    /* bucket sizes: random cut points over [lead, lead + n), some buckets empty */
    seg[0] = lead;
    for (uint32_t b = 1; b < B; b++) seg[b] = lead + rng(&s) % (n + 1);
    seg[B] = lead + n;
    for (uint32_t i = 1; i < B; i++) /* insertion sort of the cuts */
      for (uint32_t j = i; j > 1 && seg[j] < seg[j - 1]; j--) {
        const uint64_t x = seg[j];
        seg[j] = seg[j - 1];
        seg[j - 1] = x;
      }
    mde_records rec;
    memset(&rec, 0, sizeof rec);
    rec.values = vals;
    rec.values_bytes = bytes;
    rec.value_stride = stride;
    rec.layout = MDE_LAYOUT_SORTED;
    rec.value_off = voff;
    rec.n_records = nr;
    rec.n_partitions = 1;
    rec.n_buckets = B;
    rec.seg_rec = seg;
    const uint64_t NI = mde_tree_internal_nodes(B);
    uint64_t *d1 = xmalloc(B * 8ull), *d2 = xmalloc(B * 8ull), *d3 = xmalloc(B * 8ull);
    int32_t *z1 = xmalloc(B * 4ull), *z2 = xmalloc(B * 4ull), *z3 = xmalloc(B * 4ull), i1 = 0, i2 = 0, i3 = 0;
    uint8_t r1[32], r2[32], r3[32];
    uint8_t *n1 = xmalloc(NI * 32), *n2 = xmalloc(NI * 32), *n3 = xmalloc(NI * 32);
    mde_tree_out o1 = {d1, z1, &i1, r1, n1}, o2 = {d2, z2, &i2, r2, n2};
    int rc = mde_batch_build(batcher, &rec, &o1, err, sizeof err);
    if (rc) {
      fprintf(stderr, "mde_batch_build: %d %s\n", rc, err);
      exit(1);
    }
    if ((rc = mde_build(ctx, &rec, &o2))) {
      fprintf(stderr, "mde_build: %d\n", rc);
      exit(1);
    }
    oracle_build(vals, stride, voff, seg, 1, B, d3, z3, &i3, r3, n3, 1);
    if (memcmp(d1, d2, B * 8ull) || memcmp(d1, d3, B * 8ull)) bad("digest", t, k);
    if (memcmp(z1, z2, B * 4ull) || memcmp(z1, z3, B * 4ull)) bad("size", t, k);
    if (i1 != i2 || i1 != i3) bad("items", t, k);
    if (memcmp(r1, r2, 32) || memcmp(r1, r3, 32)) bad("root", t, k);
    if (memcmp(n1, n2, NI * 32) || memcmp(n1, n3, NI * 32)) bad("nodes", t, k);
    /* digest-only builds (root = NULL: no device tree), batched and per call */
    {
      uint64_t* d4 = xmalloc(B * 8ull);
      int32_t* z4 = xmalloc(B * 4ull);
      int32_t i4 = 0;
      mde_tree_out o4 = {d4, z4, &i4, NULL, NULL};
      rc = (k & 1) ? mde_batch_build(batcher, &rec, &o4, err, sizeof err) : mde_build(ctx, &rec, &o4);
      if (rc) {
        fprintf(stderr, "digest-only build: %d %s\n", rc, err);
        exit(1);
      }
      if (memcmp(d4, d3, B * 8ull) || memcmp(z4, z3, B * 4ull) || i4 != i3) bad("digest-only", t, k);
      free(d4), free(z4);
    }

    /* VerifyEpoch decision: peers = agreeing, one bucket differing, absent, garbage, and (every
     * third call) another bucket count -- a different tree shape */
    const uint64_t stride_o = mde_epoch_tree_object_max_bytes(B + 2);
    uint8_t* peers = xmalloc(4 * stride_o + 64);
    uint32_t plen[2];
    uint64_t* dp = xmalloc((B + 2) * 8ull);
    int32_t* zp = xmalloc((B + 2) * 4ull);
    memcpy(dp, d1, B * 8ull);
    memcpy(zp, z1, B * 4ull);
    const int32_t part = t * 100 + k;
    const int64_t epoch = 7 + (k % 2);
    if ((rc = mde_encode_epoch_tree_objects(ctx, 1, B, &part, epoch, epoch + 1, dp, zp, NULL, NULL, peers, stride_o,
                                            plen)))
      exit(1);
    const uint32_t pb = (k % 3 == 2) ? B + 2 : B; /* other-shape peer */
    for (uint32_t b = B; b < pb; b++) {
      dp[b] = rng(&s) % 999999u;
      zp[b] = 1;
    }
    dp[(uint32_t)k % B] = (dp[(uint32_t)k % B] + 1) % 999999u;
    if ((rc = mde_encode_epoch_tree_objects(ctx, 1, pb, &part, epoch, epoch + 1, dp, zp, NULL, NULL,
                                            peers + plen[0], stride_o, plen + 1)))
      exit(1);
    uint64_t off[5];
    off[0] = 0;
    off[1] = plen[0];
    off[2] = off[1] + plen[1];
    off[3] = off[2];            /* absent */
    const uint32_t glen = 9;    /* garbage: a truncated varint field */
    memset(peers + off[3], 0xff, glen);
    off[4] = off[3] + glen;
    const uint32_t R = (k % 2) ? 4 : 3; /* callers of one batch with different peer counts */
    const uint32_t replicas = 2;
    uint8_t va = 0, vb = 0;
    int32_t ca = 0, cb = 0, na = 0, nb = 0, sa[4], sb[4];
    int32_t *ia = xmalloc(B * 4ull), *ib = xmalloc(B * 4ull);
    const uint64_t ostride = mde_epoch_tree_object_max_bytes(B);
    uint8_t *oa = xmalloc(ostride), *ob = xmalloc(ostride);
    uint32_t la = 0, lb = 0;
    rc = mde_batch_verify(batcher, B, part, epoch, d1, z1, R, peers, off, replicas, &va, &ca, ia, &na, sa, oa, ostride,
                          &la, err, sizeof err);
    if (rc) {
      fprintf(stderr, "mde_batch_verify: %d %s\n", rc, err);
      exit(1);
    }
    if ((rc = mde_verify_epochs(ctx, 1, B, &part, epoch, d2, z2, n2, R, peers, off, replicas, &vb, &cb, ib, &nb, sb, ob,
                                ostride, &lb))) {
      fprintf(stderr, "mde_verify_epochs: %d\n", rc);
      exit(1);
    }
    if (va != vb || ca != cb || na != nb || memcmp(ia, ib, (size_t)(na > 0 ? na : 0) * 4) ||
        memcmp(sa, sb, R * 4) || la != lb || memcmp(oa, ob, la))
      bad("verify", t, k);
    /* and the oracle's diff of the differing peer: the diffSet is its de-duplicated DFS output */
    int32_t od[4096];
    const int32_t on = oracle_diff(d3, B, dp, pb, od, 4096);
    if (pb == B) { /* DFS output: that bucket, twice when it sits under a self-paired node */
      int ok = on >= 1 && na == 1 && ia[0] == (int32_t)((uint32_t)k % B);
      for (int32_t i = 0; i < on; i++) ok &= od[i] == ia[0];
      if (!ok) bad("oracle diff", t, k);
    }
    if (sa[0] != 0 || sa[2] != MDE_E_DECODE) bad("peer status", t, k);
    pthread_mutex_lock(&mu);
    builds_checked++;
    verify_checked++;
    pthread_mutex_unlock(&mu);
    free(vals);
    free(voff);
    free(seg);
    free(d1), free(d2), free(d3), free(z1), free(z2), free(z3), free(n1), free(n2), free(n3);
    free(peers), free(dp), free(zp), free(ia), free(ib), free(oa), free(ob);
  }
  return NULL;
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 10;
  n_calls = argc > 2 ? atoi(argv[2]) : 40;
  if (T < 1 || T > 256 || n_calls < 1) return 2;
  int rc = mde_batcher_create(0, 256, 0, &batcher);
  if (rc) {
    fprintf(stderr, "mde_batcher_create: %d (%s)\n", rc, mde_strerror(rc));
    return 1;
  }
  if ((rc = mde_create(0, &ctx))) return 1;
  pthread_barrier_init(&start, NULL, (unsigned)T);
  pthread_t th[256];
  for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, (void*)(intptr_t)t);
  for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
  uint64_t batches = 0, requests = 0, partitions = 0;
  mde_batcher_stats(batcher, &batches, &requests, &partitions);
  /* a bad request fails alone, with its own message, and never poisons a batch */
  char err[256];
  mde_records badr;
  memset(&badr, 0, sizeof badr);
  uint64_t segbad[3] = {0, 5, 2};
  uint8_t v8[64] = {0};
  badr.values = v8;
  badr.values_bytes = 64;
  badr.value_stride = 8;
  badr.n_records = 8;
  badr.n_partitions = 1;
  badr.n_buckets = 2;
  badr.seg_rec = segbad;
  uint8_t rr[32];
  mde_tree_out ob = {NULL, NULL, NULL, rr, NULL};
  const int rc_bad = mde_batch_build(batcher, &badr, &ob, err, sizeof err);
  const int bad_msg = strstr(err, "nondecreasing") != NULL;
  /* nodes without root is not a digest-only build */
  uint64_t segok[3] = {0, 4, 8};
  uint8_t nn[64 * 32];
  mde_tree_out on = {NULL, NULL, NULL, NULL, nn};
  badr.seg_rec = segok;
  const int rc_nodes = mde_batch_build(batcher, &badr, &on, err, sizeof err);
  badr.seg_rec = segbad;
  const int ok_bad = rc_bad == MDE_E_INVAL && bad_msg && rc_nodes == MDE_E_INVAL;
  printf("{\"test\": \"batch_test\", \"threads\": %d, \"calls_per_thread\": %d, \"builds_checked\": %ld, "
         "\"verifies_checked\": %ld, \"mismatches\": %ld, \"batches\": %" PRIu64 ", \"requests\": %" PRIu64
         ", \"partitions\": %" PRIu64 ", \"mean_requests_per_batch\": %.2f, \"bad_request_rejected\": %s}\n",
         T, n_calls, builds_checked, verify_checked, mismatches, batches, requests, partitions,
         batches ? (double)requests / (double)batches : 0.0, ok_bad ? "true" : "false");
  mde_batcher_destroy(batcher);
  mde_destroy(ctx);
  return (mismatches == 0 && ok_bad && (T == 1 || batches < requests)) ? 0 : 3;
}
