/*
 * group_cabi.c -- the multi-GPU path (mde_group) driven from plain C through include/mde.h only: no
 * PyTorch, no HIP headers. What one MyDataStore node process would do with its GPUs (a Go node is
 * one process): partition p on member p % G, each member's shard
 * generated and kept on its device, a run of pipelined group builds whose roots land straight in
 * the members' send slabs, and one overlapped all-gather of the slabs per build (RCCL, or device
 * copies when a device is listed twice), timed with the host clock.
 *
 *   group_cabi [n_keys] [n_partitions] [value_len] [n_buckets] [steps] [warmup] [members] [rehearse]
 *   defaults: 10000000 1024 1024 64 20 3 <every gfx950 GPU> 0
 *   rehearse = 1: every member on the first GPU (the group logic on a one-GPU box)
 *
 * Workload: BASELINE config 4's (cabi_bench.c): partition = gid % P, bucket from SHA-256 of the key
 * (mde_synth_tags_async), records of each member's partitions sorted by (local partition, bucket)
 * on the host, values generated on the member's device. Parity gates: the gathered slabs of the
 * last timed build equal every member's own roots (and are the same on every member), and equal
 * the slabs of a standalone group build + gather; member 0's roots equal mde_tree_from_digests of
 * its digests. Prints one JSON line; exit 0 when every gate holds.
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mde.h"

static mde_group* grp = NULL;

#define CHECK(call)                                                                                       \
  do {                                                                                                    \
    int rc_ = (call);                                                                                     \
    if (rc_) {                                                                                            \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,                           \
              grp ? mde_group_last_error(grp) : mde_strerror(rc_));                                       \
      exit(1);                                                                                            \
    }                                                                                                     \
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

static void* dalloc(mde_ctx* c, uint64_t bytes) {
  void* p = NULL;
  CHECK(mde_dev_alloc(c, bytes ? bytes : 16, &p));
  return p;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : 10000000ull;
  const uint32_t P = argc > 2 ? (uint32_t)atoi(argv[2]) : 1024u;
  const uint32_t V = argc > 3 ? (uint32_t)atoi(argv[3]) : 1024u;
  const uint32_t B = argc > 4 ? (uint32_t)atoi(argv[4]) : 64u;
  const int steps = argc > 5 ? atoi(argv[5]) : 20;
  const int warmup = argc > 6 ? atoi(argv[6]) : 3;
  int G = argc > 7 ? atoi(argv[7]) : 0;
  const int rehearse = argc > 8 ? atoi(argv[8]) : 0;
  int ordinals[64];
  const int n_dev = mde_device_list(ordinals, 64);
  if (n_dev <= 0) {
    fprintf(stderr, "mde_device_list: no gfx950 device (%d)\n", n_dev);
    return 1;
  }
  if (G <= 0) G = rehearse ? 1 : n_dev;
  if (!n || !P || !V || !B || steps < 1 || warmup < 0 || G > 64 || (!rehearse && G > n_dev)) {
    fprintf(stderr, "bad arguments (%d gfx950 devices)\n", n_dev);
    return 2;
  }
  int devs[64];
  for (int i = 0; i < G; i++) devs[i] = rehearse ? ordinals[0] : ordinals[i];
  CHECK(mde_group_create(devs, (uint32_t)G, &grp));
  const uint32_t slab = (P + (uint32_t)G - 1) / (uint32_t)G;  /* partitions per member, rounded up */
  const uint64_t slab_bytes = (uint64_t)slab * 32;

  /* tags on member 0's device for every record, then each member's shard sorted on the host */
  mde_ctx* c0 = mde_group_ctx(grp, 0);
  uint64_t* gids = xmalloc(n * 8);
  for (uint64_t i = 0; i < n; i++) gids[i] = i;
  uint64_t* d_gids = dalloc(c0, n * 8);
  uint32_t *d_part = dalloc(c0, n * 4), *d_bkt = dalloc(c0, n * 4);
  CHECK(mde_memcpy_h2d(c0, d_gids, gids, n * 8));
  CHECK(mde_synth_tags_async(c0, d_gids, n, P, B, 1, 0, d_part, d_bkt));
  CHECK(mde_synchronize(c0));
  uint32_t *part = xmalloc(n * 4), *bkt = xmalloc(n * 4);
  CHECK(mde_memcpy_d2h(c0, part, d_part, n * 4));
  CHECK(mde_memcpy_d2h(c0, bkt, d_bkt, n * 4));
  CHECK(mde_dev_free(c0, d_gids));
  CHECK(mde_dev_free(c0, d_part));
  CHECK(mde_dev_free(c0, d_bkt));

  mde_records* recs = calloc((size_t)G, sizeof(mde_records));
  mde_tree_out* outs[2][2];  /* [output set][0: pipelined run, 1: spare] per member */
  uint64_t** digest[2];
  uint8_t** send[2];
  uint8_t** recv[2];
  for (int k = 0; k < 2; k++) {
    outs[k][0] = calloc((size_t)G, sizeof(mde_tree_out));
    outs[k][1] = calloc((size_t)G, sizeof(mde_tree_out));
    digest[k] = calloc((size_t)G, sizeof(uint64_t*));
    send[k] = calloc((size_t)G, sizeof(uint8_t*));
    recv[k] = calloc((size_t)G, sizeof(uint8_t*));
  }
  uint64_t bytes_total = 0;
  for (int i = 0; i < G; i++) {
    mde_ctx* c = mde_group_ctx(grp, (uint32_t)i);
    const uint32_t Pl = mde_group_partitions(grp, P, (uint32_t)i);
    const uint64_t S = (uint64_t)Pl * B;
    uint64_t* seg = calloc(S + 1, 8);
    uint64_t nl = 0;
    for (uint64_t r = 0; r < n; r++)
      if (part[r] % (uint32_t)G == (uint32_t)i) {
        seg[(uint64_t)(part[r] / (uint32_t)G) * B + bkt[r] + 1]++;
        nl++;
      }
    for (uint64_t s = 0; s < S; s++) seg[s + 1] += seg[s];
    uint64_t* fill = xmalloc((S ? S : 1) * 8);
    memcpy(fill, seg, S * 8);
    uint64_t* sorted = xmalloc((nl ? nl : 1) * 8);
    for (uint64_t r = 0; r < n; r++)
      if (part[r] % (uint32_t)G == (uint32_t)i) sorted[fill[(uint64_t)(part[r] / (uint32_t)G) * B + bkt[r]]++] = gids[r];
    free(fill);
    uint64_t* dg = dalloc(c, nl * 8);
    if (nl) CHECK(mde_memcpy_h2d(c, dg, sorted, nl * 8));
    uint64_t* d_seg = dalloc(c, (S + 1) * 8);
    CHECK(mde_memcpy_h2d(c, d_seg, seg, (S + 1) * 8));
    uint8_t* d_vals = dalloc(c, nl * V);
    if (nl) CHECK(mde_synth_values_async(c, d_vals, dg, nl, V, 0x4D445354ull));
    CHECK(mde_synchronize(c));
    CHECK(mde_dev_free(c, dg));
    free(sorted);
    free(seg);
    mde_records* r = &recs[i];
    r->values = d_vals;
    r->values_bytes = nl * V;
    r->value_stride = V;
    r->layout = MDE_LAYOUT_SORTED;
    r->n_records = nl;
    r->n_partitions = Pl;
    r->n_buckets = B;
    r->seg_rec = d_seg;
    bytes_total += nl * V;
    for (int k = 0; k < 2; k++) {
      send[k][i] = dalloc(c, slab_bytes);
      recv[k][i] = dalloc(c, (uint64_t)G * slab_bytes);
      for (int j = 0; j < 2; j++) {
        mde_tree_out* o = &outs[k][j][i];
        uint64_t* d = dalloc(c, (S ? S : 1) * 8);
        if (j == 0) digest[k][i] = d;
        o->digest = d;
        o->size = dalloc(c, (S ? S : 1) * 4);
        o->items = dalloc(c, (uint64_t)(Pl ? Pl : 1) * 4);
        o->root = j == 0 ? send[k][i] : dalloc(c, slab_bytes);  /* the run's roots go straight into its slab */
        o->nodes = dalloc(c, (uint64_t)(Pl ? Pl : 1) * mde_tree_internal_nodes(B) * 32);
      }
    }
  }
  free(part);
  free(bkt);
  free(gids);

  /* Build L owns output set L % 2 (its roots: send slab set L % 2); launch L + 1 writes its trees,
   * and the gather of build L goes out on the side streams right after that launch. The next write
   * of set L % 2 is launch L + 3 (build L + 2's trees), so the context streams wait for gather L's
   * ticket just before it. */
  uint64_t ticket[2] = {0, 0};
  double t0 = 0.0;
  for (int phase = 0; phase < 2; phase++) {
    const int K = phase ? steps : (warmup ? warmup : 1);
    CHECK(mde_group_synchronize(grp));
    ticket[0] = ticket[1] = 0;
    if (phase) t0 = now_s();
    for (int L = 0; L < K; L++) {
      /* launch L completes build L - 1 into set (L - 1) % 2: gather L - 3 (same set) must be done */
      if (L >= 1 && ticket[(L - 1) & 1]) {
        CHECK(mde_group_gather_wait_async(grp, ticket[(L - 1) & 1]));
        ticket[(L - 1) & 1] = 0;
      }
      CHECK(mde_group_build_pipelined_async(grp, recs, outs[L & 1][0]));
      if (L >= 1)
        CHECK(mde_group_gather_overlapped_async(grp, (const void* const*)send[(L - 1) & 1], (void* const*)recv[(L - 1) & 1],
                                                slab_bytes, &ticket[(L - 1) & 1]));
    }
    if (K >= 2 && ticket[(K - 1) & 1]) {
      CHECK(mde_group_gather_wait_async(grp, ticket[(K - 1) & 1]));
      ticket[(K - 1) & 1] = 0;
    }
    CHECK(mde_group_build_pipeline_drain_async(grp));
    CHECK(mde_group_gather_overlapped_async(grp, (const void* const*)send[(K - 1) & 1], (void* const*)recv[(K - 1) & 1],
                                            slab_bytes, &ticket[(K - 1) & 1]));
    CHECK(mde_group_synchronize(grp));
  }
  const double dt = now_s() - t0;
  const int last = (steps - 1) & 1;

  /* gates: the last build's gathered slabs == every member's own slab, on every member */
  uint8_t* got0 = xmalloc((size_t)G * slab_bytes);
  uint8_t* got = xmalloc((size_t)G * slab_bytes);
  uint8_t* own = xmalloc(slab_bytes);
  CHECK(mde_memcpy_d2h(mde_group_ctx(grp, 0), got0, recv[last][0], (uint64_t)G * slab_bytes));
  int ok_gather = 1, ok_same = 1;
  for (int i = 0; i < G; i++) {
    mde_ctx* c = mde_group_ctx(grp, (uint32_t)i);
    CHECK(mde_memcpy_d2h(c, own, send[last][i], slab_bytes));
    ok_gather &= memcmp(got0 + (uint64_t)i * slab_bytes, own, slab_bytes) == 0;
    CHECK(mde_memcpy_d2h(c, got, recv[last][i], (uint64_t)G * slab_bytes));
    ok_same &= memcmp(got, got0, (size_t)G * slab_bytes) == 0;
  }
  /* a standalone group build into the spare sets, its roots copied into send set 0, one gather */
  CHECK(mde_group_build_async(grp, recs, outs[0][1]));
  CHECK(mde_group_synchronize(grp));
  for (int i = 0; i < G; i++) {
    mde_ctx* c = mde_group_ctx(grp, (uint32_t)i);
    CHECK(mde_memcpy_d2h(c, own, outs[0][1][i].root, slab_bytes));
    CHECK(mde_memcpy_h2d(c, send[0][i], own, slab_bytes));
  }
  CHECK(mde_group_gather_async(grp, (const void* const*)send[0], (void* const*)recv[0], slab_bytes));
  CHECK(mde_group_synchronize(grp));
  CHECK(mde_memcpy_d2h(mde_group_ctx(grp, 0), got, recv[0][0], (uint64_t)G * slab_bytes));
  /* only the rows of real partitions are compared (a member with fewer partitions pads its slab) */
  int ok_standalone = 1;
  for (int i = 0; i < G; i++) {
    const uint64_t rows = (uint64_t)mde_group_partitions(grp, P, (uint32_t)i) * 32;
    ok_standalone &= memcmp(got + (uint64_t)i * slab_bytes, got0 + (uint64_t)i * slab_bytes, rows) == 0;
  }
  /* member 0: its roots are the tree of its digests */
  const uint32_t P0 = mde_group_partitions(grp, P, 0);
  uint64_t* dig = xmalloc((uint64_t)P0 * B * 8);
  uint8_t* r2 = xmalloc((uint64_t)P0 * 32);
  CHECK(mde_memcpy_d2h(c0, dig, outs[0][1][0].digest, (uint64_t)P0 * B * 8));
  CHECK(mde_tree_from_digests(c0, P0, B, dig, r2, NULL));
  const int ok_tree = memcmp(r2, got, (size_t)P0 * 32) == 0;

  const double ms = dt * 1e3 / steps;
  printf("{\"metric\": \"Merkle-tree build GiB/s (device-resident KV bytes hashed/s)\", \"host\": \"C via include/mde.h "
         "(no PyTorch), mde_group\", \"value\": %.3f, \"unit\": \"GiB/s\", \"ms_per_step\": %.5f, \"steps\": %d, "
         "\"warmup\": %d, \"members\": %d, \"devices_distinct\": %d, \"gather\": \"%s\", \"config\": {\"n_keys\": %" PRIu64
         ", \"n_partitions\": %u, \"value_len\": %u, \"n_buckets\": %u, \"bytes_hashed_per_step\": %" PRIu64 "}, "
         "\"parity\": {\"gathered_slabs_hold_every_members_roots\": %s, \"every_member_received_the_same_slabs\": %s, "
         "\"run_equals_standalone_group_build\": %s, \"member0_roots_equal_tree_of_digests\": %s}}\n",
         (double)bytes_total / 1073741824.0 / (ms * 1e-3), ms, steps, warmup, G, rehearse ? 1 : G,
         mde_group_gather_kind(grp), n, P, V, B, bytes_total, ok_gather ? "true" : "false", ok_same ? "true" : "false",
         ok_standalone ? "true" : "false", ok_tree ? "true" : "false");
  free(got0);
  free(got);
  free(own);
  free(dig);
  free(r2);
  mde_group_destroy(grp);
  return ok_gather && ok_same && ok_standalone && ok_tree ? 0 : 3;
}
