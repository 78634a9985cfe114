/*
 * cabi_bench.c -- the C4 Merkle build driven from plain C through include/mde.h only: no PyTorch,
 * no HIP headers. What a cgo / C host sees: the same device-resident
 * workload bench.py measures, built with mde_build_pipelined_async, timed with the host clock.
 *
 *   cabi_bench [n_keys] [n_partitions] [value_len] [n_buckets] [steps] [warmup]
 *   defaults: 10000000 1024 1024 64 20 3 (BASELINE config 4, round-robin partitions)
 *
 * Workload: record gid's partition = gid % P, bucket =
 * BE64(SHA256("k%016x" % gid)[:8]) % B (mde_synth_tags_async on device), records ordered by
 * (partition, bucket) with a host counting sort (the LSM order, layout A), values generated on
 * device (mde_synth_values_async). Parity gates before timing: the device roots equal
 * mde_tree_from_digests of the device digests, and sampled buckets' digests equal the byte sums of
 * their records copied back to the host, mod 999999. Prints one JSON line.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mde.h"

#define CHECK(call)                                                                        \
  do {                                                                                     \
    int rc_ = (call);                                                                      \
    if (rc_) {                                                                             \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,            \
              ctx ? mde_last_error(ctx) : mde_strerror(rc_));                              \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p) {
    fprintf(stderr, "host allocation of %zu bytes failed\n", n);
    exit(1);
  }
  return p;
}

typedef struct {
  uint64_t *digest;
  int32_t *size, *items;
  uint8_t *root, *nodes;
  mde_tree_out out;
} out_set;

static mde_ctx* ctx = NULL;

static void* dalloc(uint64_t bytes) {
  void* p = NULL;
  CHECK(mde_dev_alloc(ctx, bytes ? bytes : 16, &p));
  return p;
}

static void make_outs(out_set* o, uint32_t P, uint32_t B) {
  o->digest = dalloc((uint64_t)P * B * 8);
  o->size = dalloc((uint64_t)P * B * 4);
  o->items = dalloc((uint64_t)P * 4);
  o->root = dalloc((uint64_t)P * 32);
  o->nodes = dalloc((uint64_t)P * mde_tree_internal_nodes(B) * 32);
  o->out.digest = o->digest;
  o->out.size = o->size;
  o->out.items = o->items;
  o->out.root = o->root;
  o->out.nodes = o->nodes;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : 10000000ull;
  const uint32_t P = argc > 2 ? (uint32_t)atoi(argv[2]) : 1024u;
  const uint32_t V = argc > 3 ? (uint32_t)atoi(argv[3]) : 1024u;
  const uint32_t B = argc > 4 ? (uint32_t)atoi(argv[4]) : 64u;
  const int steps = argc > 5 ? atoi(argv[5]) : 20;
  const int warmup = argc > 6 ? atoi(argv[6]) : 3;
  if (!n || !P || !V || !B || steps < 1 || warmup < 0) {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  CHECK(mde_create(0, &ctx));
  int cus = 0;
  char arch[64] = {0};
  CHECK(mde_device_info(ctx, &cus, arch, sizeof arch));

  /* tags on device, counting sort by (partition, bucket) on the host */
  uint64_t* gids = xmalloc(n * 8);
  for (uint64_t i = 0; i < n; i++) gids[i] = i;
  uint64_t* d_gids = dalloc(n * 8);
  uint32_t *d_part = dalloc(n * 4), *d_bkt = dalloc(n * 4);
  CHECK(mde_memcpy_h2d(ctx, d_gids, gids, n * 8));
  CHECK(mde_synth_tags_async(ctx, d_gids, n, P, B, 1, 0, d_part, d_bkt));
  CHECK(mde_synchronize(ctx));
  uint32_t *part = xmalloc(n * 4), *bkt = xmalloc(n * 4);
  CHECK(mde_memcpy_d2h(ctx, part, d_part, n * 4));
  CHECK(mde_memcpy_d2h(ctx, bkt, d_bkt, n * 4));
  const uint64_t S = (uint64_t)P * B;
  uint64_t* seg = calloc(S + 1, 8);
  if (!seg) return 1;
  for (uint64_t i = 0; i < n; i++) seg[(uint64_t)part[i] * B + bkt[i] + 1]++;
  for (uint64_t s = 0; s < S; s++) seg[s + 1] += seg[s];
  uint64_t* fill = xmalloc(S * 8);
  memcpy(fill, seg, S * 8);
  uint64_t* sorted = xmalloc(n * 8);
  for (uint64_t i = 0; i < n; i++) sorted[fill[(uint64_t)part[i] * B + bkt[i]]++] = gids[i];
  free(fill);
  free(part);
  free(bkt);
  CHECK(mde_memcpy_h2d(ctx, d_gids, sorted, n * 8));
  uint64_t* d_seg = dalloc((S + 1) * 8);
  CHECK(mde_memcpy_h2d(ctx, d_seg, seg, (S + 1) * 8));
  const uint64_t bytes = n * (uint64_t)V;
  uint8_t* d_vals = dalloc(bytes);
  CHECK(mde_synth_values_async(ctx, d_vals, d_gids, n, V, 0x4D445354ull));
  CHECK(mde_synchronize(ctx));
  CHECK(mde_dev_free(ctx, d_part));
  CHECK(mde_dev_free(ctx, d_bkt));
  CHECK(mde_dev_free(ctx, d_gids));
  free(gids);
  free(sorted);

  mde_records rec;
  memset(&rec, 0, sizeof rec);
  rec.values = d_vals;
  rec.values_bytes = bytes;
  rec.value_stride = V;
  rec.layout = MDE_LAYOUT_SORTED;
  rec.n_records = n;
  rec.n_partitions = P;
  rec.n_buckets = B;
  rec.seg_rec = d_seg;
  out_set outs[2];
  make_outs(&outs[0], P, B);
  make_outs(&outs[1], P, B);

  /* parity gates (standalone build) */
  CHECK(mde_build_async(ctx, &rec, &outs[0].out));
  CHECK(mde_synchronize(ctx));
  uint64_t* dig = xmalloc(S * 8);
  uint8_t *root = xmalloc((size_t)P * 32), *root2 = xmalloc((size_t)P * 32);
  CHECK(mde_memcpy_d2h(ctx, dig, outs[0].digest, S * 8));
  CHECK(mde_memcpy_d2h(ctx, root, outs[0].root, (uint64_t)P * 32));
  CHECK(mde_tree_from_digests(ctx, P, B, dig, root2, NULL));
  int ok_tree = memcmp(root, root2, (size_t)P * 32) == 0;
  int ok_sum = 1;
  for (int k = 0; k < 16; k++) {
    const uint64_t s = (uint64_t)k * 7919u % S;
    const uint64_t len = (seg[s + 1] - seg[s]) * V;
    uint8_t* buf = xmalloc(len);
    if (len) CHECK(mde_memcpy_d2h(ctx, buf, d_vals + seg[s] * V, len));
    uint64_t sum = 0;
    for (uint64_t j = 0; j < len; j++) sum += buf[j];
    free(buf);
    ok_sum &= (sum % MDE_HASH_MOD) == dig[s];
  }

  /* timed run of pipelined builds: each call digests one build and builds the previous trees */
  for (int i = 0; i < warmup; i++) CHECK(mde_build_pipelined_async(ctx, &rec, &outs[i & 1].out));
  CHECK(mde_build_pipeline_drain_async(ctx));
  CHECK(mde_synchronize(ctx));
  const double t0 = now_s();
  for (int i = 0; i < steps; i++) CHECK(mde_build_pipelined_async(ctx, &rec, &outs[i & 1].out));
  CHECK(mde_build_pipeline_drain_async(ctx));
  CHECK(mde_synchronize(ctx));
  const double dt = now_s() - t0;

  /* the last timed build's roots equal the standalone build's */
  CHECK(mde_memcpy_d2h(ctx, root2, outs[(steps - 1) & 1].root, (uint64_t)P * 32));
  int ok_run = memcmp(root, root2, (size_t)P * 32) == 0;
  const double ms = dt * 1e3 / steps;
  printf("{\"metric\": \"Merkle-tree build GiB/s (device-resident KV bytes hashed/s)\", \"host\": \"C via "
         "include/mde.h (no PyTorch)\", \"value\": %.3f, \"unit\": \"GiB/s\", \"ms_per_step\": %.5f, "
         "\"steps\": %d, \"warmup\": %d, \"frac_of_8TBps\": %.4f, \"device\": \"%s\", \"cus\": %d, "
         "\"config\": {\"n_keys\": %" PRIu64 ", \"n_partitions\": %u, \"value_len\": %u, \"n_buckets\": %u, "
         "\"bytes_hashed_per_step\": %" PRIu64 "}, \"parity\": {\"roots_equal_tree_of_digests\": %s, "
         "\"sampled_bucket_sums\": %s, \"timed_run_roots_equal_standalone\": %s}}\n",
         (double)bytes / 1073741824.0 / (ms * 1e-3), ms, steps, warmup, (double)bytes / (ms * 1e-3) / 8e12,
         arch, cus, n, P, V, B, bytes, ok_tree ? "true" : "false", ok_sum ? "true" : "false",
         ok_run ? "true" : "false");
  free(dig);
  free(root);
  free(root2);
  free(seg);

  /* Call latency of the synchronous host-buffer entry point at the production shape: ONE
   * partition per call (VerifyEpoch -> RawPartitionMerkleTree, main/manager.go:1036), values =
   * 8-byte LE timestamps (main/manager.go:816), B = n_buckets; host arena -> H2D -> digest ->
   * tree -> D2H of digests, sizes, items, root. Median of 200 calls per record count. */
  for (int k = 0; k < 3; k++) {
    const uint64_t nr = k == 0 ? 1000u : k == 1 ? 10000u : 100000u;
    uint8_t* hv = xmalloc(nr * 8);
    for (uint64_t i = 0; i < nr * 8; i++) hv[i] = (uint8_t)(i * 131u + 7u);
    uint64_t* hs = xmalloc(((uint64_t)B + 1) * 8);
    for (uint32_t b = 0; b <= B; b++) hs[b] = nr * b / B;
    uint64_t* hd = xmalloc((uint64_t)B * 8);
    int32_t *hz = xmalloc((uint64_t)B * 4), hi = 0;
    uint8_t hr[32];
    mde_records r1;
    memset(&r1, 0, sizeof r1);
    r1.values = hv;
    r1.values_bytes = nr * 8;
    r1.value_stride = 8;
    r1.layout = MDE_LAYOUT_SORTED;
    r1.n_records = nr;
    r1.n_partitions = 1;
    r1.n_buckets = B;
    r1.seg_rec = hs;
    mde_tree_out o1 = {hd, hz, &hi, hr, NULL};
    double lat[200];
    for (int i = 0; i < 210; i++) {
      const double a = now_s();
      CHECK(mde_build(ctx, &r1, &o1));
      if (i >= 10) lat[i - 10] = now_s() - a;
    }
    for (int i = 1; i < 200; i++)  /* insertion sort: 200 samples */
      for (int j = i; j > 0 && lat[j] < lat[j - 1]; j--) {
        const double t = lat[j];
        lat[j] = lat[j - 1];
        lat[j - 1] = t;
      }
    printf("{\"latency\": \"mde_build (host buffers, synchronous), 1 partition\", \"records\": %" PRIu64
           ", \"value_len\": 8, \"n_buckets\": %u, \"median_us\": %.1f, \"p10_us\": %.1f, \"p90_us\": %.1f}\n",
           nr, B, lat[100] * 1e6, lat[20] * 1e6, lat[180] * 1e6);
    free(hv);
    free(hs);
    free(hd);
    free(hz);
  }

  /* One whole VerifyEpoch's device work for one partition, from C: RawPartitionMerkleTree
   * (mde_build with the nodes output, 1,000 records) then the decision step (mde_verify_epochs)
   * against two peer objects -- one agreeing, one with a single differing bucket -- persisting the
   * object (main/manager.go:1036-1118). Median of 200 of each call. */
  {
    const uint64_t nr = 1000;
    const uint64_t NI = mde_tree_internal_nodes(B);
    uint8_t* hv = xmalloc(nr * 8);
    for (uint64_t i = 0; i < nr * 8; i++) hv[i] = (uint8_t)(i * 131u + 7u);
    uint64_t* hs = xmalloc(((uint64_t)B + 1) * 8);
    for (uint32_t b = 0; b <= B; b++) hs[b] = nr * b / B;
    uint64_t* hd = xmalloc((uint64_t)B * 8);
    uint64_t* hd2 = xmalloc((uint64_t)B * 8);
    int32_t *hz = xmalloc((uint64_t)B * 4), hi = 0;
    uint8_t hr[32];
    uint8_t* hn = xmalloc(NI * 32);
    mde_records r1;
    memset(&r1, 0, sizeof r1);
    r1.values = hv;
    r1.values_bytes = nr * 8;
    r1.value_stride = 8;
    r1.layout = MDE_LAYOUT_SORTED;
    r1.n_records = nr;
    r1.n_partitions = 1;
    r1.n_buckets = B;
    r1.seg_rec = hs;
    mde_tree_out o1 = {hd, hz, &hi, hr, hn};
    CHECK(mde_build(ctx, &r1, &o1));
    /* peer objects: this tree's object, and one with bucket 0 perturbed */
    const uint64_t stride = mde_epoch_tree_object_max_bytes(B);
    uint8_t* peers = xmalloc(2 * stride);
    uint32_t plen[2];
    memcpy(hd2, hd, (size_t)B * 8);
    hd2[0] = (hd2[0] + 1) % 999999u;
    const int32_t part = 7;
    CHECK(mde_encode_epoch_tree_objects(ctx, 1, B, &part, 5, 6, hd, hz, NULL, NULL, peers, stride, plen));
    CHECK(mde_encode_epoch_tree_objects(ctx, 1, B, &part, 5, 6, hd2, hz, NULL, NULL, peers + plen[0], stride,
                                        plen + 1));
    const uint64_t poff[3] = {0, plen[0], (uint64_t)plen[0] + plen[1]};
    uint8_t valid = 0;
    int32_t vc = 0, dc = 0, st[2];
    int32_t* ids = xmalloc((uint64_t)B * 4);
    uint8_t* obj = xmalloc(stride);
    uint32_t olen = 0;
    double lb[200], lv[200];
    for (int i = 0; i < 210; i++) {
      const double a = now_s();
      CHECK(mde_build(ctx, &r1, &o1));
      const double m = now_s();
      CHECK(mde_verify_epochs(ctx, 1, B, &part, 5, hd, hz, hn, 2, peers, poff, 2, &valid, &vc, ids, &dc, st, obj,
                              stride, &olen));
      if (i >= 10) {
        lb[i - 10] = m - a;
        lv[i - 10] = now_s() - m;
      }
    }
    const int ok_verify = vc == 1 && dc == 1 && ids[0] == 0 && st[0] == 0 && st[1] == 1 && !valid && olen > 0;
    for (int i = 1; i < 200; i++)
      for (int j = i; j > 0 && lb[j] < lb[j - 1]; j--) {
        const double t = lb[j];
        lb[j] = lb[j - 1];
        lb[j - 1] = t;
      }
    for (int i = 1; i < 200; i++)
      for (int j = i; j > 0 && lv[j] < lv[j - 1]; j--) {
        const double t = lv[j];
        lv[j] = lv[j - 1];
        lv[j - 1] = t;
      }
    printf("{\"latency\": \"VerifyEpoch device work, 1 partition: mde_build (nodes out) + mde_verify_epochs (2 peers)\", "
           "\"records\": %" PRIu64 ", \"n_buckets\": %u, \"build_median_us\": %.1f, \"verify_median_us\": %.1f, "
           "\"verify_p10_us\": %.1f, \"verify_p90_us\": %.1f, \"verify_ok\": %s}\n",
           nr, B, lb[100] * 1e6, lv[100] * 1e6, lv[20] * 1e6, lv[180] * 1e6, ok_verify ? "true" : "false");
    free(hv);
    free(hs);
    free(hd);
    free(hd2);
    free(hz);
    free(hn);
    free(peers);
    free(ids);
    free(obj);
    if (!ok_verify) ok_run = 0;
  }
  mde_destroy(ctx);
  return ok_tree && ok_sum && ok_run ? 0 : 3;
}
