/*
 * batch_bench.c -- the production call shape, timed from plain C through include/mde.h.
 *
 * The reference builds ONE partition per VerifyEpoch (main/manager.go:1036 ->
 * RawPartitionMerkleTree, main/merkle_tree.go:86-116), whose hashed values are 8-byte LE
 * timestamps (main/manager.go:816), at partition_buckets = 1000 by default, on up to
 * partition_concurrency = 10 workers out of workers_count = 100 (config/default-config.yaml:7-10).
 * This program puts three ways of serving that shape side by side:
 *   cpu     -- the C restatement of the reference's build (oracle/mde_oracle.c oracle_build, one
 *              thread per call: per bucket, per record Add then % 999999, then the SHA-256 tree),
 *              on P concurrent threads like P goroutines (Badger iteration excluded: an upper
 *              bound on the reference's rate);
 *   percall -- P threads calling the synchronous mde_build on one shared context (one device round
 *              trip per partition: the round-2 shim);
 *   batched -- P threads calling mde_batch_build on one batcher (group commit: concurrent calls
 *              share one H2D copy, one build and one D2H copy).
 * and the same for the decision step (mde_verify_epochs per call vs mde_batch_verify, two peers:
 * one agreeing, one differing in a bucket). Reports per-call latency (median, p90) and aggregate
 * partitions per second; every batched output is compared with the C oracle.
 *
 *   batch_bench [seconds_per_case]   default 0.4
 * One JSON line per case.
 */
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mde.h"

int oracle_build(const uint8_t* values, uint32_t stride, const uint64_t* value_off, const uint64_t* seg_rec,
                 uint32_t n_partitions, uint32_t n_buckets, uint64_t* digest, int32_t* size, int32_t* items,
                 uint8_t* root, uint8_t* nodes, int threads);

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void* xmalloc(size_t n) {
  void* p = calloc(1, n ? n : 1);
  if (!p) {
    fprintf(stderr, "allocation failed\n");
    exit(1);
  }
  return p;
}

static uint64_t rng(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

enum { CPU = 0, PERCALL = 1, BATCHED = 2, V_PERCALL = 3, V_BATCHED = 4 };
static const char* kModes[] = {"cpu", "percall", "batched", "verify_percall", "verify_batched"};

/* One partition-epoch of 8-byte timestamps, records spread evenly over B buckets, plus its
 * outputs and (for the decision step) its nodes and two peer objects. */
typedef struct {
  uint64_t n;
  uint32_t B;
  uint8_t* vals;
  uint64_t* seg;
  uint64_t *dig, *dig_ref;
  int32_t *size, items;
  uint8_t root[32], *nodes;
  uint8_t* peers;
  uint64_t off[3];
  int32_t* ids;
  uint8_t* obj;
} part_t;

static mde_ctx* ctx;
static mde_batcher* batcher;
static pthread_barrier_t bar;
static double g_seconds = 0.4;
static long g_bad = 0;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;

static void make_part(part_t* p, uint64_t n, uint32_t B, uint64_t seed) {
  memset(p, 0, sizeof *p);
  p->n = n;
  p->B = B;
  p->vals = xmalloc(n * 8);
  uint64_t ts = 1700000000ull + seed * 1000003ull;
  for (uint64_t i = 0; i < n; i++) { /* LE64 write timestamps */
    ts += 1 + rng(&seed) % 7;
    memcpy(p->vals + i * 8, &ts, 8);
  }
  p->seg = xmalloc(((uint64_t)B + 1) * 8);
  for (uint32_t b = 0; b <= B; b++) p->seg[b] = n * b / B;
  p->dig = xmalloc((uint64_t)B * 8);
  p->dig_ref = xmalloc((uint64_t)B * 8);
  p->size = xmalloc((uint64_t)B * 4);
  p->nodes = xmalloc(mde_tree_internal_nodes(B) * 32);
  p->ids = xmalloc((uint64_t)B * 4);
  p->obj = xmalloc(mde_epoch_tree_object_max_bytes(B));
  int32_t items;
  uint8_t root[32];
  oracle_build(p->vals, 8, NULL, p->seg, 1, B, p->dig_ref, p->size, &items, root, NULL, 1);
}

static void make_peers(part_t* p) {
  const uint64_t st = mde_epoch_tree_object_max_bytes(p->B);
  p->peers = xmalloc(2 * st);
  uint32_t len[2];
  const int32_t part = 3;
  mde_encode_epoch_tree_objects(ctx, 1, p->B, &part, 9, 10, p->dig_ref, p->size, NULL, NULL, p->peers, st, len);
  uint64_t* d2 = xmalloc((uint64_t)p->B * 8);
  memcpy(d2, p->dig_ref, (uint64_t)p->B * 8);
  d2[p->B / 2] = (d2[p->B / 2] + 1) % 999999u;
  mde_encode_epoch_tree_objects(ctx, 1, p->B, &part, 9, 10, d2, p->size, NULL, NULL, p->peers + len[0], st, len + 1);
  free(d2);
  p->off[0] = 0;
  p->off[1] = len[0];
  p->off[2] = (uint64_t)len[0] + len[1];
  /* the local tree's nodes, for the per-call mde_verify_epochs */
  uint8_t root[32];
  mde_tree_from_digests(ctx, 1, p->B, p->dig_ref, root, p->nodes);
}

typedef struct {
  int mode;
  part_t* parts; /* this thread's partitions (rotated through) */
  int n_parts;
  double* lat;
  int cap, n;
} job_t;

static int call(int mode, part_t* p) {
  char err[256];
  mde_records r;
  memset(&r, 0, sizeof r);
  r.values = p->vals;
  r.values_bytes = p->n * 8;
  r.value_stride = 8;
  r.layout = MDE_LAYOUT_SORTED;
  r.n_records = p->n;
  r.n_partitions = 1;
  r.n_buckets = p->B;
  r.seg_rec = p->seg;
  mde_tree_out o = {p->dig, p->size, &p->items, p->root, NULL};
  uint8_t valid;
  int32_t vc, dc, st[2];
  uint32_t olen;
  const int32_t part = 3;
  const uint64_t ost = mde_epoch_tree_object_max_bytes(p->B);
  switch (mode) {
    case CPU:
      return oracle_build(p->vals, 8, NULL, p->seg, 1, p->B, p->dig, p->size, &p->items, p->root, NULL, 1);
    case PERCALL:
      return mde_build(ctx, &r, &o);
    case BATCHED:
      return mde_batch_build(batcher, &r, &o, err, sizeof err);
    case V_PERCALL:
      return mde_verify_epochs(ctx, 1, p->B, &part, 9, p->dig_ref, p->size, p->nodes, 2, p->peers, p->off, 2, &valid,
                               &vc, p->ids, &dc, st, p->obj, ost, &olen);
    default: {
      const int rc = mde_batch_verify(batcher, p->B, part, 9, p->dig_ref, p->size, 2, p->peers, p->off, 2, &valid,
                                      &vc, p->ids, &dc, st, p->obj, ost, &olen, err, sizeof err);
      if (!rc && (vc != 1 || dc != 1 || p->ids[0] != (int32_t)(p->B / 2) || valid)) return -100;
      return rc;
    }
  }
}

static void* worker(void* arg) {
  job_t* j = arg;
  pthread_barrier_wait(&bar);
  const double t_end = now_s() + g_seconds;
  int k = 0;
  while (j->n < j->cap) {
    part_t* p = &j->parts[k++ % j->n_parts];
    const double a = now_s();
    const int rc = call(j->mode, p);
    const double b = now_s();
    if (rc) {
      fprintf(stderr, "%s failed: %d\n", kModes[j->mode], rc);
      exit(1);
    }
    if (j->mode <= BATCHED && memcmp(p->dig, p->dig_ref, (uint64_t)p->B * 8)) {
      pthread_mutex_lock(&mu);
      g_bad++;
      pthread_mutex_unlock(&mu);
    }
    j->lat[j->n++] = b - a;
    if (b >= t_end) break;
  }
  return NULL;
}

static int cmpd(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

/* P threads x calls of `mode` for g_seconds; prints one JSON line. */
static void run_case(int mode, int P, uint64_t n, uint32_t B, part_t* parts, int n_parts_per_thread) {
  job_t* jobs = xmalloc(sizeof(job_t) * (size_t)P);
  pthread_t* th = xmalloc(sizeof(pthread_t) * (size_t)P);
  pthread_barrier_init(&bar, NULL, (unsigned)P + 1);
  for (int t = 0; t < P; t++) {
    jobs[t].mode = mode;
    jobs[t].parts = parts + (size_t)t * n_parts_per_thread;
    jobs[t].n_parts = n_parts_per_thread;
    jobs[t].cap = 200000;
    jobs[t].lat = xmalloc(sizeof(double) * (size_t)jobs[t].cap);
    jobs[t].n = 0;
    pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  uint64_t b0 = 0, r0 = 0, p0 = 0, b1 = 0, r1 = 0, p1 = 0;
  mde_batcher_stats(batcher, &b0, &r0, &p0);
  pthread_barrier_wait(&bar);
  const double t0 = now_s();
  for (int t = 0; t < P; t++) pthread_join(th[t], NULL);
  const double wall = now_s() - t0;
  mde_batcher_stats(batcher, &b1, &r1, &p1);
  long total = 0;
  for (int t = 0; t < P; t++) total += jobs[t].n;
  double* all = xmalloc(sizeof(double) * (size_t)total);
  long m = 0;
  for (int t = 0; t < P; t++) {
    memcpy(all + m, jobs[t].lat, sizeof(double) * (size_t)jobs[t].n);
    m += jobs[t].n;
    free(jobs[t].lat);
  }
  qsort(all, (size_t)total, sizeof(double), cmpd);
  const double batches = (double)(b1 - b0);
  printf("{\"case\": \"%s\", \"callers\": %d, \"records\": %" PRIu64 ", \"value_len\": 8, \"n_buckets\": %u, "
         "\"calls\": %ld, \"wall_s\": %.4f, \"partitions_per_s\": %.1f, \"latency_median_us\": %.1f, "
         "\"latency_p90_us\": %.1f",
         kModes[mode], P, n, B, total, wall, (double)total / wall, all[total / 2] * 1e6, all[total * 9 / 10] * 1e6);
  if ((mode == BATCHED || mode == V_BATCHED) && batches > 0)
    printf(", \"mean_requests_per_batch\": %.2f", (double)(r1 - r0) / batches);
  printf("}\n");
  fflush(stdout);
  free(all);
  free(jobs);
  free(th);
  pthread_barrier_destroy(&bar);
}

int main(int argc, char** argv) {
  g_seconds = argc > 1 ? atof(argv[1]) : 0.4;
  int rc = mde_create(0, &ctx);
  if (rc) {
    fprintf(stderr, "mde_create: %d (%s)\n", rc, mde_strerror(rc));
    return 1;
  }
  if ((rc = mde_batcher_create(0, 256, 0, &batcher))) return 1;
  /* batch_bench SECONDS B CALLERS [MODE]: only the concurrent cases of that shape (for kernel traces) */
  if (argc > 3) {
    const uint32_t B = (uint32_t)atoi(argv[2]);
    const int P = atoi(argv[3]);
    part_t* parts = xmalloc(sizeof(part_t) * (size_t)P * 4);
    for (int i = 0; i < P * 4; i++) {
      make_part(&parts[i], 1000, B, 100 + (uint64_t)i);
      make_peers(&parts[i]);
    }
    /* optional 4th argument: one mode by name */
    for (int mode = CPU; mode <= V_BATCHED; mode++)
      if (argc <= 4 || !strcmp(argv[4], kModes[mode])) run_case(mode, P, 1000, B, parts, 4);
    printf("{\"batched_outputs_equal_oracle\": %s}\n", g_bad ? "false" : "true");
    mde_batcher_destroy(batcher);
    mde_destroy(ctx);
    return g_bad ? 3 : 0;
  }
  /* single-call shapes: CPU oracle (1 thread) beside the synchronous device call */
  const uint64_t ns[3] = {1000, 10000, 100000};
  const uint32_t Bs[2] = {64, 1000};
  for (int bi = 0; bi < 2; bi++)
    for (int ni = 0; ni < 3; ni++) {
      part_t p;
      make_part(&p, ns[ni], Bs[bi], 1 + ni);
      run_case(CPU, 1, ns[ni], Bs[bi], &p, 1);
      run_case(PERCALL, 1, ns[ni], Bs[bi], &p, 1);
      run_case(BATCHED, 1, ns[ni], Bs[bi], &p, 1);
    }
  /* concurrent callers: P threads, 4 distinct partitions each, 1,000 timestamps per partition */
  const int Ps[3] = {1, 10, 100};
  for (int bi = 0; bi < 2; bi++)
    for (int pi = 0; pi < 3; pi++) {
      const int P = Ps[pi];
      part_t* parts = xmalloc(sizeof(part_t) * (size_t)P * 4);
      for (int i = 0; i < P * 4; i++) {
        make_part(&parts[i], 1000, Bs[bi], 100 + (uint64_t)i);
        make_peers(&parts[i]);
      }
      for (int mode = CPU; mode <= V_BATCHED; mode++) run_case(mode, P, 1000, Bs[bi], parts, 4);
      for (int i = 0; i < P * 4; i++) {
        part_t* p = &parts[i];
        free(p->vals), free(p->seg), free(p->dig), free(p->dig_ref), free(p->size), free(p->nodes), free(p->ids);
        free(p->obj), free(p->peers);
      }
      free(parts);
    }
  printf("{\"batched_outputs_equal_oracle\": %s}\n", g_bad ? "false" : "true");
  mde_batcher_destroy(batcher);
  mde_destroy(ctx);
  return g_bad ? 3 : 0;
}
