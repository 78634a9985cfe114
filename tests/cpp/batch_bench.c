/*
 * batch_bench.c -- the production call shape, timed from plain C through include/mde.h, as the
 * Go caller sees it (host-side steps of the cgo shim included).
 *
 * The reference builds ONE partition per VerifyEpoch (main/manager.go:1036 ->
 * RawPartitionMerkleTree, main/merkle_tree.go:86-116), whose hashed values are 8-byte LE
 * timestamps (main/manager.go:816), at partition_buckets = 1000 by default, on up to
 * partition_concurrency = 10 workers out of workers_count = 100 (config/default-config.yaml:7-10).
 * Every case below returns what the Go caller holds afterwards -- a merkletree-shaped node graph
 * (oracle/mde_oracle.c oracle_graph_*, one allocation per tree like NewTree's nodes) -- so the rows
 * compare like for like. Badger iteration is excluded from every row (it is the same in all).
 *
 * Build (RawPartitionMerkleTree):
 *   cpu            the reference path restated in C: per bucket, per record Add then % 999999
 *                  (oracle_bucket_digests), then NewTree (oracle_graph_build: SHA-256 of every
 *                  internal node, on the SHA extensions when the CPU has them, as Go's
 *                  crypto/sha256 does on amd64);
 *   shim           the cgo shim (integration/go/merkle_gpu.go): mde_batch_build with the nodes
 *                  output (digests + SHA-256 tree on the device), then the tree assembled from the
 *                  device's node hashes (oracle_graph_from_nodes: no host hashing);
 *   shim_hosttree  the hybrid: mde_batch_build digest-only (root = NULL: no device tree), then
 *                  NewTree on the host over the device digests (oracle_graph_build);
 *   device_call    mde_batch_build alone (digests + root), no tree object: the ABI call only;
 *   percall        synchronous mde_build (nodes) on one shared context + tree assembly;
 *   server         mde_server_build (the resident build service: a persistent launch polling
 *                  request slots in pinned memory, no launch / copy / event per call) with the
 *                  nodes output, then the tree assembled from the node hashes;
 *   server_hosttree  mde_server_build digest-only, then NewTree on the host;
 *   server_levels  mde_server_build_levels: digests and the tree's levels down to the first of at
 *                  most 64 nodes on the device, the top levels hashed on the host (the shim's
 *                  memo misses, hashed with crypto/sha256).
 * The build rows report host_compressions_per_call: the SHA-256 compressions the caller ran on the
 * host (0 where every node hash comes from the device: shim, server, percall).
 * VerifyEpoch decision step (main/manager.go:1072-1104; two peers, one agreeing, one differing):
 *   cpu_verify     per peer: EpochTreeObjectToMerkleTree (decode the 8-byte bucket hashes, NewTree)
 *                  and DifferentMerkleTreeBuckets against the local tree; validCount / diffSet fold;
 *   verify_batched the shim's verifyEpochDecision: proto.Marshal of the peer objects (a C encoder
 *                  here) + mde_batch_verify;
 *   verify_server  the same through the resident service (mde_server_verify).
 * DifferentMerkleTreeBuckets of two trees the caller already holds (one pair per call):
 *   diff_host      the reference's DFS over the two node graphs (oracle_graph_diff);
 *   diff_device    mde_diff with both trees' nodes (one shared context);
 *   diff_digests   mde_diff_digests (the round-3 shim: both trees rebuilt on the device).
 * Reports per-call latency (median, p90) and aggregate calls per second; every output is checked
 * against the C oracle (digests, roots, diff lists, decisions).
 *
 *   batch_bench [seconds_per_case]                   every shape (default 0.4 s per case)
 *   batch_bench SECONDS B CALLERS [CASE]             only the concurrent cases of that shape
 * One JSON line per case; the last line says whether every checked output equalled the oracle.
 */
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mde.h"

/* oracle/mde_oracle.c (test infrastructure: the checker and the CPU rows) */
typedef struct oracle_graph oracle_graph;
int oracle_build(const uint8_t* values, uint32_t stride, const uint64_t* value_off, const uint64_t* seg_rec,
                 uint32_t n_partitions, uint32_t n_buckets, uint64_t* digest, int32_t* size, int32_t* items,
                 uint8_t* root, uint8_t* nodes, int threads);
int oracle_bucket_digests(const uint8_t* values, uint32_t stride, const uint64_t* value_off, const uint64_t* seg_rec,
                          uint32_t n_partitions, uint32_t n_buckets, uint64_t* digest, int32_t* size, int32_t* items);
int oracle_tree(const uint64_t* digest, uint32_t n_buckets, uint8_t* nodes, uint8_t* root);
int32_t oracle_diff(const uint64_t* d1, uint32_t b1, const uint64_t* d2, uint32_t b2, int32_t* out, int32_t cap);
oracle_graph* oracle_graph_build(const uint64_t* digest, uint32_t n_buckets);
oracle_graph* oracle_graph_from_nodes(const uint64_t* digest, uint32_t n_buckets, const uint8_t* nodes);
const uint8_t* oracle_graph_root(const oracle_graph* g);
int32_t oracle_graph_diff(const oracle_graph* a, const oracle_graph* b, int32_t* out, int32_t cap);
void oracle_graph_free(oracle_graph* g);
int oracle_sha_ni(void);
void oracle_sha256(const uint8_t* msg, uint64_t len, uint8_t out[32]);

/* The shim's top levels (mdeTree with mde_server_build_levels): levels above the first one of at
 * most top nodes, hashed on the host, node = SHA256(left || right), an odd level's last node
 * paired with itself -- merkletree v0.2.0's rule, on the CPU's SHA extensions like crypto/sha256. */
static uint64_t g_host_comp; /* host SHA-256 compressions of the current case (atomic adds) */

static void count_comp(uint64_t c) { __atomic_fetch_add(&g_host_comp, c, __ATOMIC_RELAXED); }

/* compressions of a whole host tree (NewTree): one per 16-byte level-1 message, two above */
static uint64_t tree_comp(uint32_t B) {
  const uint64_t n1 = (B + 1) / 2;
  return 2 * mde_tree_internal_nodes(B) - n1;
}

static void finish_top_levels(uint32_t B, uint32_t top, uint8_t* nodes) {
  uint32_t n = (B + 1) / 2;
  uint64_t off = 0;
  while (n > top && n > 1) { /* levels the device wrote */
    off += n;
    n = (n + 1) / 2;
  }
  while (n > 1) {
    const uint32_t m = (n + 1) / 2;
    uint8_t msg[64];
    for (uint32_t j = 0; j < m; j++) {
      const uint32_t l = 2 * j, r = 2 * j + 1 < n ? 2 * j + 1 : 2 * j;
      memcpy(msg, nodes + (off + l) * 32, 32);
      memcpy(msg + 32, nodes + (off + r) * 32, 32);
      oracle_sha256(msg, 64, nodes + (off + n + j) * 32);
    }
    count_comp(2ull * m);
    off += n;
    n = m;
  }
}

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

enum {
  CPU,
  SHIM,
  SHIM_HOSTTREE,
  DEVICE_CALL,
  PERCALL,
  SERVER,
  SERVER_HOSTTREE,
  SERVER_LEVELS,
  CPU_VERIFY,
  V_BATCHED,
  V_SERVER,
  DIFF_HOST,
  DIFF_DEVICE,
  DIFF_DIGESTS,
  N_CASES
};
static const char* kCases[] = {"cpu",          "shim",       "shim_hosttree",  "device_call", "percall",
                               "server",       "server_hosttree", "server_levels", "cpu_verify", "verify_batched", "verify_server", "diff_host",
                               "diff_device",  "diff_digests"};

/* One partition-epoch of 8-byte timestamps, records spread evenly over B buckets; the oracle's
 * outputs for it; two peers (agreeing, differing at bucket B/2) as decoded objects (the 8-byte
 * bucket hashes gRPC hands VerifyEpoch) and as trees (for the diff rows). */
typedef struct {
  uint64_t n;
  uint32_t B, NI;
  uint8_t* vals;
  uint64_t* seg;
  uint64_t *dig, *dig_ref;
  int32_t *size, *size_ref, items;
  uint8_t root[32], root_ref[32], *nodes, *nodes_ref;
  oracle_graph* tree;       /* the local tree (myTree) */
  uint8_t* peer_hash[2];    /* [B*8] LE64 bucket hashes of peer r */
  uint64_t* peer_dig[2];    /* the same as digests (the device diff rows) */
  uint8_t* peer_nodes[2];   /* peer r's internal nodes */
  oracle_graph* peer_tree[2];
  int32_t* diff_ref;        /* oracle_diff(local, peer 1) */
  int32_t n_diff_ref;
  uint8_t* wire;            /* marshal scratch */
  int32_t* ids;
  uint8_t* obj;
} part_t;

static mde_ctx* ctx;
static mde_batcher* batcher;
static mde_server* server;
static uint32_t g_top = 64; /* server_levels: MDE_TOP_NODES overrides (sweep) */
static pthread_barrier_t bar;
static double g_seconds = 0.4;
static long g_bad = 0;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;

static void bad(const char* what, const part_t* p) {
  pthread_mutex_lock(&mu);
  if (g_bad++ < 10) fprintf(stderr, "mismatch: %s (B=%u n=%" PRIu64 ")\n", what, p->B, p->n);
  pthread_mutex_unlock(&mu);
}

static void make_part(part_t* p, uint64_t n, uint32_t B, uint64_t seed) {
  memset(p, 0, sizeof *p);
  p->n = n;
  p->B = B;
  p->NI = (uint32_t)mde_tree_internal_nodes(B);
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
  p->size_ref = xmalloc((uint64_t)B * 4);
  p->nodes = xmalloc((uint64_t)p->NI * 32);
  p->nodes_ref = xmalloc((uint64_t)p->NI * 32);
  p->ids = xmalloc((uint64_t)B * 8);
  p->obj = xmalloc(mde_epoch_tree_object_max_bytes(B));
  p->wire = xmalloc(2 * (mde_epoch_tree_object_max_bytes(B) + 64));
  int32_t items;
  oracle_build(p->vals, 8, NULL, p->seg, 1, B, p->dig_ref, p->size_ref, &items, p->root_ref, p->nodes_ref, 1);
  p->tree = oracle_graph_build(p->dig_ref, B);
  for (int r = 0; r < 2; r++) {
    p->peer_dig[r] = xmalloc((uint64_t)B * 8);
    memcpy(p->peer_dig[r], p->dig_ref, (uint64_t)B * 8);
    if (r == 1) p->peer_dig[r][B / 2] = (p->peer_dig[r][B / 2] + 1) % 999999u;
    p->peer_hash[r] = xmalloc((uint64_t)B * 8);
    memcpy(p->peer_hash[r], p->peer_dig[r], (uint64_t)B * 8); /* little-endian host: LE64 bytes */
    p->peer_nodes[r] = xmalloc((uint64_t)p->NI * 32);
    uint8_t root[32];
    oracle_tree(p->peer_dig[r], B, p->peer_nodes[r], root);
    p->peer_tree[r] = oracle_graph_build(p->peer_dig[r], B);
  }
  p->diff_ref = xmalloc((uint64_t)B * 8);
  p->n_diff_ref = oracle_diff(p->dig_ref, B, p->peer_dig[1], B, p->diff_ref, (int32_t)(2 * B));
}

static void free_part(part_t* p) {
  free(p->vals), free(p->seg), free(p->dig), free(p->dig_ref), free(p->size), free(p->size_ref);
  free(p->nodes), free(p->nodes_ref), free(p->ids), free(p->obj), free(p->wire), free(p->diff_ref);
  oracle_graph_free(p->tree);
  for (int r = 0; r < 2; r++) {
    free(p->peer_dig[r]), free(p->peer_hash[r]), free(p->peer_nodes[r]);
    oracle_graph_free(p->peer_tree[r]);
  }
}

/* ---- proto.Marshal of an EpochTreeObject (datap/data.proto:60-68), as the shim re-encodes the
 * peer objects gRPC already decoded (integration/go/merkle_gpu.go verifyEpochDecision). */
static uint8_t* put_varint(uint8_t* o, uint64_t v) {
  while (v >= 0x80) {
    *o++ = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  *o++ = (uint8_t)v;
  return o;
}

static uint64_t marshal_object(uint8_t* out, int32_t partition, int64_t lo, int64_t hi, const uint8_t* hashes,
                               const int32_t* sizes, uint32_t B) {
  uint8_t* o = out;
  if (partition) o = put_varint(put_varint(o, 0x08), (uint64_t)(int64_t)partition);
  if (lo) o = put_varint(put_varint(o, 0x10), (uint64_t)lo);
  if (hi) o = put_varint(put_varint(o, 0x18), (uint64_t)hi);
  for (uint32_t b = 0; b < B; b++) {
    *o++ = 0x22;
    *o++ = 8;
    memcpy(o, hashes + (uint64_t)b * 8, 8);
    o += 8;
  }
  uint64_t plen = 0;
  uint8_t tmp[16];
  for (uint32_t b = 0; b < B; b++) plen += (uint64_t)(put_varint(tmp, (uint64_t)(int64_t)sizes[b]) - tmp);
  if (B) {
    o = put_varint(put_varint(o, 0x2a), plen);
    for (uint32_t b = 0; b < B; b++) o = put_varint(o, (uint64_t)(int64_t)sizes[b]);
  }
  return (uint64_t)(o - out);
}

/* ---- the cases */
typedef struct {
  int mode;
  part_t* parts; /* this thread's partitions (rotated through) */
  int n_parts;
  double* lat;
  int cap, n;
} job_t;

static mde_records records_of(const part_t* p) {
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
  return r;
}

static void check_tree(const part_t* p, const oracle_graph* g, const char* what) {
  if (!g || memcmp(oracle_graph_root(g), p->root_ref, 32) || memcmp(p->dig, p->dig_ref, (uint64_t)p->B * 8))
    bad(what, p);
}

static int call(int mode, part_t* p) {
  char err[256];
  mde_records r = records_of(p);
  const uint32_t B = p->B;
  const int32_t part = 3;
  const uint64_t ost = mde_epoch_tree_object_max_bytes(B);
  int rc = 0;
  switch (mode) {
    case CPU: {
      oracle_bucket_digests(p->vals, 8, NULL, p->seg, 1, B, p->dig, p->size, &p->items);
      oracle_graph* g = oracle_graph_build(p->dig, B);
      count_comp(tree_comp(B));
      check_tree(p, g, "cpu");
      oracle_graph_free(g);
      return 0;
    }
    case SHIM:
    case PERCALL: {
      mde_tree_out o = {p->dig, p->size, &p->items, p->root, p->nodes};
      rc = mode == SHIM ? mde_batch_build(batcher, &r, &o, err, sizeof err) : mde_build(ctx, &r, &o);
      if (rc) return rc;
      oracle_graph* g = oracle_graph_from_nodes(p->dig, B, p->nodes);
      check_tree(p, g, kCases[mode]);
      if (memcmp(p->root, p->root_ref, 32)) bad("device root", p);
      oracle_graph_free(g);
      return 0;
    }
    case SHIM_HOSTTREE: {
      mde_tree_out o = {p->dig, p->size, &p->items, NULL, NULL};
      if ((rc = mde_batch_build(batcher, &r, &o, err, sizeof err))) return rc;
      oracle_graph* g = oracle_graph_build(p->dig, B);
      count_comp(tree_comp(B));
      check_tree(p, g, "shim_hosttree");
      oracle_graph_free(g);
      return 0;
    }
    case SERVER: {
      mde_tree_out o = {p->dig, p->size, &p->items, p->root, p->nodes};
      if ((rc = mde_server_build(server, &r, &o, err, sizeof err))) return rc;
      oracle_graph* g = oracle_graph_from_nodes(p->dig, B, p->nodes);
      check_tree(p, g, "server");
      if (memcmp(p->root, p->root_ref, 32)) bad("server root", p);
      oracle_graph_free(g);
      return 0;
    }
    case SERVER_HOSTTREE: {
      mde_tree_out o = {p->dig, p->size, &p->items, NULL, NULL};
      if ((rc = mde_server_build(server, &r, &o, err, sizeof err))) return rc;
      oracle_graph* g = oracle_graph_build(p->dig, B);
      count_comp(tree_comp(B));
      check_tree(p, g, "server_hosttree");
      oracle_graph_free(g);
      return 0;
    }
    case SERVER_LEVELS: { /* device: digests + levels up to <= 64 nodes; host: the top levels */
      mde_tree_out o = {p->dig, p->size, &p->items, NULL, p->nodes};
      if ((rc = mde_server_build_levels(server, &r, &o, g_top, err, sizeof err))) return rc;
      finish_top_levels(B, g_top, p->nodes);
      oracle_graph* g = oracle_graph_from_nodes(p->dig, B, p->nodes);
      check_tree(p, g, "server_levels");
      oracle_graph_free(g);
      return 0;
    }
    case DEVICE_CALL: {
      mde_tree_out o = {p->dig, p->size, &p->items, p->root, NULL};
      if ((rc = mde_batch_build(batcher, &r, &o, err, sizeof err))) return rc;
      if (memcmp(p->root, p->root_ref, 32) || memcmp(p->dig, p->dig_ref, (uint64_t)B * 8)) bad("device_call", p);
      return 0;
    }
    case CPU_VERIFY: {
      /* per peer: decode (utils.DecodeBytesToInt64) + NewTree + DFS; fold (manager.go:1072-1104) */
      int valid_count = 0, n_ids = 0;
      uint8_t* in_set = (uint8_t*)calloc(B, 1);
      for (int k = 0; k < 2; k++) {
        for (uint32_t b = 0; b < B; b++) memcpy(&p->dig[b], p->peer_hash[k] + (uint64_t)b * 8, 8);
        oracle_graph* g = oracle_graph_build(p->dig, B);
        const int32_t nd = oracle_graph_diff(p->tree, g, p->ids, (int32_t)(2 * B));
        oracle_graph_free(g);
        if (nd < 0) continue;
        if (nd == 0) valid_count++;
        for (int32_t i = 0; i < nd; i++) in_set[p->ids[i]] = 1;
      }
      for (uint32_t b = 0; b < B; b++)
        if (in_set[b]) p->ids[n_ids++] = (int32_t)b;
      free(in_set);
      if (valid_count != 1 || n_ids != 1 || p->ids[0] != (int32_t)(B / 2)) bad("cpu_verify", p);
      return 0;
    }
    case V_BATCHED: {
      uint64_t off[3] = {0, 0, 0};
      for (int k = 0; k < 2; k++)
        off[k + 1] = off[k] + marshal_object(p->wire + off[k], part, 9, 10, p->peer_hash[k], p->size_ref, B);
      uint8_t valid;
      int32_t vc, dc, st[2];
      uint32_t olen;
      rc = mde_batch_verify(batcher, B, part, 9, p->dig_ref, p->size_ref, 2, p->wire, off, 2, &valid, &vc, p->ids, &dc,
                            st, p->obj, ost, &olen, err, sizeof err);
      if (!rc && (vc != 1 || dc != 1 || p->ids[0] != (int32_t)(B / 2) || valid)) bad("verify_batched", p);
      return rc;
    }
    case V_SERVER: {
      uint64_t off[3] = {0, 0, 0};
      for (int k = 0; k < 2; k++)
        off[k + 1] = off[k] + marshal_object(p->wire + off[k], part, 9, 10, p->peer_hash[k], p->size_ref, B);
      uint8_t valid;
      int32_t vc, dc, st[2];
      uint32_t olen;
      rc = mde_server_verify(server, B, part, 9, p->dig_ref, p->size_ref, 2, p->wire, off, 2, &valid, &vc, p->ids, &dc,
                             st, p->obj, ost, &olen, err, sizeof err);
      if (!rc && (vc != 1 || dc != 1 || p->ids[0] != (int32_t)(B / 2) || valid)) bad("verify_server", p);
      return rc;
    }
    case DIFF_HOST: {
      const int32_t nd = oracle_graph_diff(p->tree, p->peer_tree[1], p->ids, (int32_t)(2 * B));
      if (nd != p->n_diff_ref || memcmp(p->ids, p->diff_ref, (uint64_t)nd * 4)) bad("diff_host", p);
      return 0;
    }
    case DIFF_DEVICE:
    case DIFF_DIGESTS: {
      const uint64_t cap = mde_diff_capacity(B, B);
      int32_t cnt = 0;
      rc = mode == DIFF_DEVICE ? mde_diff(ctx, 1, B, p->dig_ref, p->nodes_ref, B, p->peer_dig[1], p->peer_nodes[1],
                                          p->ids, cap, &cnt)
                               : mde_diff_digests(ctx, 1, B, p->dig_ref, B, p->peer_dig[1], p->ids, cap, &cnt);
      if (!rc && (cnt != p->n_diff_ref || memcmp(p->ids, p->diff_ref, (uint64_t)cnt * 4))) bad(kCases[mode], p);
      return rc;
    }
  }
  return MDE_E_INVAL;
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
      fprintf(stderr, "%s failed: %d\n", kCases[j->mode], rc);
      exit(1);
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
  uint64_t b0 = 0, r0 = 0, p0 = 0, b1 = 0, r1 = 0, p1 = 0, sc0 = 0, sc1 = 0;
  mde_batcher_stats(batcher, &b0, &r0, &p0);
  mde_server_stats(server, NULL, NULL, &sc0);
  __atomic_store_n(&g_host_comp, 0, __ATOMIC_RELAXED);
  pthread_barrier_wait(&bar);
  const double t0 = now_s();
  for (int t = 0; t < P; t++) pthread_join(th[t], NULL);
  const double wall = now_s() - t0;
  mde_batcher_stats(batcher, &b1, &r1, &p1);
  mde_server_stats(server, NULL, NULL, &sc1);
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
         "\"calls\": %ld, \"wall_s\": %.4f, \"calls_per_s\": %.1f, \"latency_median_us\": %.1f, "
         "\"latency_p90_us\": %.1f",
         kCases[mode], P, n, B, total, wall, (double)total / wall, all[total / 2] * 1e6, all[total * 9 / 10] * 1e6);
  if ((mode == SHIM || mode == SHIM_HOSTTREE || mode == DEVICE_CALL || mode == V_BATCHED) && batches > 0)
    printf(", \"mean_requests_per_batch\": %.2f", (double)(r1 - r0) / batches);
  if (mode == SERVER || mode == SERVER_HOSTTREE || mode == SERVER_LEVELS || mode == V_SERVER) printf(", \"server_calls_on_context\": %" PRIu64, sc1 - sc0);
  if (mode <= SERVER_LEVELS)  /* the build rows: SHA-256 compressions the caller ran on the host per call */
    printf(", \"host_compressions_per_call\": %.1f", total ? (double)__atomic_load_n(&g_host_comp, __ATOMIC_RELAXED) / (double)total : 0.0);
  printf("}\n");
  fflush(stdout);
  free(all);
  free(jobs);
  free(th);
  pthread_barrier_destroy(&bar);
}

static int case_by_name(const char* s) {
  for (int m = 0; m < N_CASES; m++)
    if (!strcmp(s, kCases[m])) return m;
  return -1;
}

/* concurrent callers: P threads, 4 distinct partitions each, 1,000 timestamps per partition */
static void run_shape(uint32_t B, int P, int only) {
  part_t* parts = xmalloc(sizeof(part_t) * (size_t)P * 4);
  for (int i = 0; i < P * 4; i++) make_part(&parts[i], 1000, B, 100 + (uint64_t)i);
  for (int mode = 0; mode < N_CASES; mode++)
    if (only < 0 || mode == only) run_case(mode, P, 1000, B, parts, 4);
  for (int i = 0; i < P * 4; i++) free_part(&parts[i]);
  free(parts);
}

int main(int argc, char** argv) {
  g_seconds = argc > 1 ? atof(argv[1]) : 0.4;
  int rc = mde_create(0, &ctx);
  if (rc) {
    fprintf(stderr, "mde_create: %d (%s)\n", rc, mde_strerror(rc));
    return 1;
  }
  /* MDE_BATCH_WAIT_US: the batcher's collection window (0 = none, the shim's setting) */
  if (getenv("MDE_TOP_NODES")) g_top = (uint32_t)atoi(getenv("MDE_TOP_NODES"));
  const char* wait_env = getenv("MDE_BATCH_WAIT_US");
  const uint32_t wait_us = wait_env ? (uint32_t)atoi(wait_env) : 0u;
  /* MDE_SERVER_SLOTS: the service's request slots (0 = its default, 16); the service first
   * (include/mde.h teardown contract) */
  const uint32_t slots = getenv("MDE_SERVER_SLOTS") ? (uint32_t)atoi(getenv("MDE_SERVER_SLOTS")) : 0u;
  if ((rc = mde_server_create(0, slots, 0, &server))) {
    fprintf(stderr, "mde_server_create: %d\n", rc);
    return 1;
  }
  if ((rc = mde_batcher_create(0, 256, wait_us, &batcher))) return 1;
  printf("{\"host_sha_extensions\": %s, \"batcher_wait_us\": %u, \"server_slots\": %u}\n", oracle_sha_ni() ? "true" : "false",
         wait_us, mde_server_slots(server));
  if (argc > 3) {
    const int only = argc > 4 ? case_by_name(argv[4]) : -1;
    if (argc > 4 && only < 0) {
      fprintf(stderr, "unknown case %s\n", argv[4]);
      return 2;
    }
    run_shape((uint32_t)atoi(argv[2]), atoi(argv[3]), only);
  } else {
    /* single-call shapes: one caller, growing partitions, build rows only */
    const uint64_t ns[3] = {1000, 10000, 100000};
    const uint32_t Bs[2] = {64, 1000};
    for (int bi = 0; bi < 2; bi++)
      for (int ni = 0; ni < 3; ni++) {
        part_t p;
        make_part(&p, ns[ni], Bs[bi], 1 + ni);
        for (int mode = CPU; mode <= SERVER_LEVELS; mode++) run_case(mode, 1, ns[ni], Bs[bi], &p, 1);
        free_part(&p);
      }
    const int Ps[3] = {1, 10, 100};
    for (int bi = 0; bi < 2; bi++)
      for (int pi = 0; pi < 3; pi++) run_shape(Bs[bi], Ps[pi], -1);
  }
  printf("{\"outputs_equal_oracle\": %s}\n", g_bad ? "false" : "true");
  mde_batcher_destroy(batcher);
  mde_server_destroy(server);
  mde_destroy(ctx);
  return g_bad ? 3 : 0;
}
