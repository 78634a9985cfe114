/*
 * shim_replay.c -- the Go shim's exact call sequences (integration/go/merkle_gpu.go) replayed in
 * plain C through include/mde.h, on scenarios read from a file; the results go to stdout and the
 * pytest driver (tests/test_integration.py) compares them with the oracle's restatement of the
 * reference (oracle/oracle.py: raw_partition_merkle_tree, different_merkle_tree_buckets,
 * verify_epoch). The shim cannot be compiled here (no Go toolchain); this program makes the same
 * ABI calls with the same argument shapes:
 *
 *   build B n           RawPartitionMerkleTree (main/merkle_tree.go:86-116): the shim walks the
 *                       B bucket ranges and appends every value to ONE arena, record by record:
 *                       value_off grows by each value's length, seg_rec by the record count per
 *                       bucket, n_partitions = 1, value_stride = 0 (variable-length values); an
 *                       empty arena gets one padding byte. B > 64: -> mde_server_build_levels
 *                       (the shim's mdeResident: the device's levels down to <= 64 nodes, the
 *                       levels above hashed on the host; mde_batch_build with the whole tree when
 *                       "batcher" is argv[2]) with the nodes output, then the shim's mdeNewTree:
 *                       merkletree v0.2.0's own construction (NewTreeWithHashStrategy, mirrored
 *                       below as mt_new_tree) with the memoising strategy mdeMemoHash: every node
 *                       message the device hashed is looked up in mdeMemo, every other one is
 *                       hashed with SHA-256 (counted: the host compressions of the call). B <= 64
 *                       (mdeHostTreeMaxBuckets): a digest-only build (root = nodes = NULL), then
 *                       NewTree on the host over the device digests (no memo: every node hashed).
 *                       The memo is then offered a tampered tree (one bucket digest + 1): its root
 *                       must be the SHA-256 tree of the tampered digests -- a miss is hashed, the
 *                       memo never answers for bytes the device did not hash.
 *   diff Ba Bb          DifferentMerkleTreeBuckets (main/merkle_tree.go:159-216), which the shim no
 *                       longer replaces: the reference's DFS over two trees of the shim's shape --
 *                       mdeTree over mde_tree_from_digests' nodes (a tree rebuilt from an odd-B
 *                       object has B+1 leaves, no duplicate) -- mirrored below.
 *   verify B p E rc R   VerifyEpoch's peer loop (main/manager.go:1072-1104): the local tree's
 *                       digests and sizes, R peer objects as wire bytes (absent = empty range)
 *                       -> mde_server_verify (mde_batch_verify with "batcher").
 *
 * Input: whitespace-separated tokens; values and peer objects as hex strings ("-" = empty).
 *   build B n  <bucket of each record, nondecreasing>  <hex value of each record>
 *   diff Ba Bb <Ba digests> <Bb digests>
 *   verify B p E rc R <B digests> <B sizes> <R hex objects>
 * Output, one line per op:
 *   build <digests> ; <sizes> ; <items> ; <Root.Hash hex> ; <leaf count> <SHA-256 of the pre-order
 *         walk: every node's Hash, and each leaf's bucketId as LE32> ; <host compressions>
 *         <tampered tree's root == the SHA-256 tree of the tampered digests (1/0)>
 *   diff <count> <ids>            (count = MDE_E_TREE where the reference errors)
 *   verify <valid> <validCount> ; <diffSet> ; <peer statuses> ; <object hex>
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mde.h"

void oracle_sha256(const uint8_t* msg, uint64_t len, uint8_t out[32]); /* checker's SHA-256 */
/* stands in for merkletree.NewTree's hashing where the shim builds the tree on the host */
int oracle_tree(const uint64_t* digest, uint32_t n_buckets, uint8_t* nodes, uint8_t* root);
#define HOST_TREE_MAX_BUCKETS 64  /* merkle_gpu.go mdeHostTreeMaxBuckets */
#define TOP_NODES 64              /* merkle_gpu.go mdeTopNodes */

/* ---- merkletree v0.2.0's node graph (leaf Hash = LE64(digest), a duplicate of the last leaf when B
 * is odd -- same Hash, same content --, level nodes pairing (2j, 2j+1) with the last of an odd level
 * paired with itself). */
typedef struct snode {
  struct snode *left, *right;
  const uint8_t* hash;
  uint32_t hlen;
  int32_t bucket; /* leaf content's bucketId; -1 for internal nodes (C == nil) */
} snode;

typedef struct {
  snode* pool;
  snode* root;
  uint32_t n_leafs;
  uint8_t* leaf_hash;
  uint8_t* node_hash; /* mt_new_tree: the internal nodes' hashes */
} stree;

static void* xmalloc(size_t n);

/* ---- the shim's mdeMemo / mdeMemoHash (integration/go/merkle_gpu.go): the k-th hasher merkletree's
 * construction takes answers with device node k's hash when the message written to it is exactly
 * node k's message (its children's hashes as the device hashed them), else runs SHA-256 (counted:
 * the host compressions of the call). */
typedef struct {
  uint8_t* leaf;         /* [n0 * 8] LE64 leaf hashes (+ the odd-B duplicate) */
  uint32_t n0;
  const uint8_t* nodes;  /* the device's node hashes, level 1 .. root */
  uint64_t have;         /* how many of them the device wrote */
  uint32_t lvl[40], n_lvl;
  uint64_t next;         /* the node the construction hashes next */
  uint64_t compressions;
} memo_t;

static memo_t memo_build(const uint64_t* digest, uint32_t B, const uint8_t* nodes, uint64_t have) {
  memo_t m;
  memset(&m, 0, sizeof m);
  m.n0 = B + (B & 1u);
  m.leaf = xmalloc((size_t)m.n0 * 8);
  for (uint32_t i = 0; i < B; i++)
    for (int k = 0; k < 8; k++) m.leaf[(size_t)i * 8 + k] = (uint8_t)(digest[i] >> (8 * k));
  if (B & 1u) memcpy(m.leaf + (size_t)B * 8, m.leaf + (size_t)(B - 1) * 8, 8);
  m.nodes = nodes;
  m.have = have;
  for (uint32_t n = m.n0; n > 1;) {
    n = (n + 1) / 2;
    m.lvl[m.n_lvl++] = n;
  }
  return m;
}

/* node k's message as the device hashed it; 0 when k is past the device's nodes */
static uint32_t memo_message(const memo_t* m, uint64_t k, uint8_t msg[64]) {
  if (k >= m->have) return 0;
  uint64_t off = 0, below = m->n0;
  int64_t prev = -1;
  for (uint32_t i = 0; i < m->n_lvl; i++) {
    const uint64_t n = m->lvl[i];
    if (k < off + n) {
      const uint64_t j = k - off, li = 2 * j, ri = 2 * j + 1 < below ? 2 * j + 1 : 2 * j;
      if (prev < 0) {
        memcpy(msg, m->leaf + li * 8, 8);
        memcpy(msg + 8, m->leaf + ri * 8, 8);
        return 16;
      }
      memcpy(msg, m->nodes + ((uint64_t)prev + li) * 32, 32);
      memcpy(msg + 32, m->nodes + ((uint64_t)prev + ri) * 32, 32);
      return 64;
    }
    prev = (int64_t)off;
    below = n;
    off += n;
  }
  return 0;
}

/* mdeMemoHash.Sum for the construction's next node; memo == NULL: plain NewTree */
static void strategy_sum(memo_t* m, const uint8_t* msg, uint32_t n, uint8_t out[32], uint64_t* compressions) {
  if (m) {
    const uint64_t k = m->next++;
    uint8_t want[64];
    const uint32_t wn = memo_message(m, k, want);
    if (wn && wn == n && !memcmp(want, msg, n)) {
      memcpy(out, m->nodes + k * 32, 32);
      return;
    }
  }
  *compressions += (n + 8) / 64 + 1;
  oracle_sha256(msg, n, out);
}

/* merkletree.NewTreeWithHashStrategy (v0.2.0 buildWithContent + buildIntermediate), the strategy
 * being strategy_sum over `memo` */
static stree mt_new_tree(const uint64_t* digest, uint32_t B, memo_t* memo, uint64_t* compressions) {
  stree t;
  const uint32_t n0 = B + (B & 1u);
  t.pool = xmalloc(sizeof(snode) * (2 * (size_t)n0 + 64)); /* every level rounds up: < 2 n0 + depth */
  t.leaf_hash = xmalloc((size_t)B * 8);
  t.node_hash = xmalloc(mde_tree_internal_nodes(B) * 32);
  t.n_leafs = n0;
  snode* level = t.pool;
  for (uint32_t i = 0; i < B; i++) {
    for (int k = 0; k < 8; k++) t.leaf_hash[(size_t)i * 8 + k] = (uint8_t)(digest[i] >> (8 * k));
    level[i] = (snode){NULL, NULL, t.leaf_hash + (size_t)i * 8, 8, (int32_t)i};
  }
  if (B & 1u) level[B] = level[B - 1]; /* merkletree's duplicate leaf */
  uint32_t n = n0;
  snode* next = level + n0;
  uint64_t off = 0;
  while (n > 1) {
    const uint32_t m = (n + 1) / 2;
    for (uint32_t j = 0; j < m; j++) {
      snode* l = &level[2 * j];
      snode* r = 2 * j + 1 < n ? &level[2 * j + 1] : l;
      uint8_t msg[64];
      memcpy(msg, l->hash, l->hlen);
      memcpy(msg + l->hlen, r->hash, r->hlen);
      uint8_t* h = t.node_hash + (off + j) * 32;
      strategy_sum(memo, msg, l->hlen + r->hlen, h, compressions);
      next[j] = (snode){l, r, h, 32, -1};
    }
    off += m;
    level = next;
    next += m;
    n = m;
  }
  t.root = level;
  return t;
}

/* The reference's DFS (below) over two trees rebuilt from digests: node hashes the device built
 * (mde_tree_from_digests), in the same graph. */
static stree mde_tree(const uint64_t* digest, uint32_t B, const uint8_t* nodes) {
  memo_t m = memo_build(digest, B, nodes, mde_tree_internal_nodes(B));
  uint64_t c = 0;
  stree t = mt_new_tree(digest, B, &m, &c);
  free(m.leaf);
  if (c) {
    fprintf(stderr, "tree from device nodes needed %llu host compressions\n", (unsigned long long)c);
    exit(1);
  }
  return t;
}

/* DifferentMerkleTreeBucketsDFS (main/merkle_tree.go:163-216): 0, or -1 where it errors. */
static int ref_dfs(const snode* a, const snode* b, int32_t* out, int32_t* n) {
  if (!a && !b) return 0;
  if (!a || !b) return -1;
  if (a->hlen == b->hlen && !memcmp(a->hash, b->hash, a->hlen)) return 0;
  if (!a->left && !a->right) {
    if (a->bucket < 0 || b->bucket < 0 || a->bucket != b->bucket) return -1;
    out[(*n)++] = a->bucket;
    return 0;
  }
  if (ref_dfs(a->left, b->left, out, n)) return -1;
  return ref_dfs(a->right, b->right, out, n);
}

static void walk(const snode* x, uint8_t** buf, uint64_t* len, uint64_t* cap) {
  if (*len + 40 > *cap) {
    *cap = *cap * 2 + 4096;
    *buf = realloc(*buf, *cap);
    if (!*buf) exit(1);
  }
  memcpy(*buf + *len, x->hash, x->hlen);
  *len += x->hlen;
  if (!x->left && !x->right) {
    memcpy(*buf + *len, &x->bucket, 4);
    *len += 4;
    return;
  }
  walk(x->left, buf, len, cap);
  walk(x->right, buf, len, cap);
}

static void* xmalloc(size_t n) {
  void* p = calloc(1, n ? n : 1);
  if (!p) {
    fprintf(stderr, "allocation failed\n");
    exit(1);
  }
  return p;
}

static char tok[1 << 22];

static const char* next(FILE* f) {
  if (fscanf(f, "%4194303s", tok) != 1) return NULL;
  return tok;
}

static uint64_t num(FILE* f) {
  const char* t = next(f);
  if (!t) {
    fprintf(stderr, "truncated input\n");
    exit(2);
  }
  return strtoull(t, NULL, 10);
}

/* hex token -> bytes appended at *buf (capacity grown as needed); returns the length */
static uint64_t hex(FILE* f, uint8_t** buf, uint64_t* len, uint64_t* cap) {
  const char* t = next(f);
  if (!t) exit(2);
  if (!strcmp(t, "-")) return 0;
  const uint64_t n = strlen(t) / 2;
  if (*len + n > *cap) {
    *cap = (*len + n) * 2 + 64;
    *buf = realloc(*buf, *cap);
    if (!*buf) exit(1);
  }
  for (uint64_t i = 0; i < n; i++) {
    unsigned v;
    sscanf(t + 2 * i, "%2x", &v);
    (*buf)[*len + i] = (uint8_t)v;
  }
  *len += n;
  return n;
}

static void print_hex(const uint8_t* p, uint64_t n) {
  for (uint64_t i = 0; i < n; i++) printf("%02x", p[i]);
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "r");
  if (!f) return 2;
  /* the shim's mdeResident: the resident service (default), or "batcher" as the second argument */
  const int resident = !(argc > 2 && !strcmp(argv[2], "batcher"));
  mde_batcher* batcher = NULL;
  mde_server* server = NULL;
  mde_ctx* ctx = NULL;
  /* the service first (include/mde.h teardown contract: services created before, destroyed after,
   * every other context of the device), as merkle_gpu.go's mdeEngine does */
  int rc = mde_server_create(0, 16, 1024, &server);
  if (!rc) rc = mde_batcher_create(0, 256, 0, &batcher);
  if (rc || (rc = mde_create(0, &ctx))) {
    fprintf(stderr, "create: %d (%s)\n", rc, mde_strerror(rc));
    return 1;
  }
  char err[512];
  const char* op;
  while ((op = next(f))) {
    if (!strcmp(op, "build")) {
      const uint32_t B = (uint32_t)num(f);
      const uint64_t n = num(f);
      uint64_t* bucket = xmalloc(n * 8);
      for (uint64_t i = 0; i < n; i++) bucket[i] = num(f);
      /* the shim's loop: for each bucket, for each record of its range, append the value */
      uint8_t* values = NULL;
      uint64_t vlen = 0, vcap = 0;
      uint64_t* value_off = xmalloc((n + 1) * 8);
      uint64_t* seg_rec = xmalloc(((uint64_t)B + 1) * 8);
      uint64_t r = 0;
      seg_rec[0] = 0;
      for (uint32_t b = 0; b < B; b++) {
        while (r < n && bucket[r] == b) {
          hex(f, &values, &vlen, &vcap);
          value_off[++r] = vlen;
        }
        seg_rec[b + 1] = r;
      }
      if (vlen == 0) { /* values = append(values, 0): never a zero-length arena */
        values = realloc(values, 1);
        values[0] = 0;
        vlen = 1;
      }
      mde_records rec;
      memset(&rec, 0, sizeof rec);
      rec.values = values;
      rec.values_bytes = vlen;
      rec.value_off = value_off;
      rec.n_records = r;
      rec.n_partitions = 1;
      rec.n_buckets = B;
      rec.seg_rec = seg_rec;
      uint64_t* digest = xmalloc((uint64_t)B * 8);
      int32_t* size = xmalloc((uint64_t)B * 4);
      int32_t items = 0;
      uint8_t root[32];
      uint8_t* nodes = xmalloc(mde_tree_internal_nodes(B) * 32);
      const int host_tree = B <= HOST_TREE_MAX_BUCKETS;
      mde_tree_out out = {digest, size, &items, host_tree ? NULL : root, host_tree ? NULL : nodes};
      if (resident && !host_tree) { /* merkle_gpu.go: the device's levels down to <= mdeTopNodes */
        out.root = NULL;
        rc = mde_server_build_levels(server, &rec, &out, TOP_NODES, err, sizeof err);
      } else {
        rc = resident ? mde_server_build(server, &rec, &out, err, sizeof err)
                      : mde_batch_build(batcher, &rec, &out, err, sizeof err);
      }
      if (rc) {
        fprintf(stderr, "build: %d %s\n", rc, err);
        return 1;
      }
      /* mdeNewTree: merkletree's construction over the memo of the device's nodes (the first
       * `have`: every node through the batcher, the levels down to <= mdeTopNodes nodes through the
       * service); or plain NewTree over the device digests (B <= mdeHostTreeMaxBuckets) */
      const uint64_t have = host_tree ? 0 : resident ? mde_tree_prefix_nodes(B, TOP_NODES) : mde_tree_internal_nodes(B);
      memo_t memo = memo_build(digest, B, nodes, have);
      uint64_t compressions = 0;
      stree t = mt_new_tree(digest, B, host_tree ? NULL : &memo, &compressions);
      /* the memo offered a tampered tree: one bucket's digest + 1 */
      uint64_t* tampered = xmalloc((uint64_t)B * 8);
      memcpy(tampered, digest, (uint64_t)B * 8);
      tampered[B / 2] = (tampered[B / 2] + 1) % MDE_HASH_MOD;
      uint64_t tc = 0;
      memo.next = 0; /* a second construction over the same memo */
      stree tt = mt_new_tree(tampered, B, &memo, &tc);
      uint8_t troot[32];
      oracle_tree(tampered, B, NULL, troot);
      const int tamper_ok = !memcmp(troot, tt.root->hash, 32) && tc > 0;
      uint8_t* wb = NULL;
      uint64_t wl = 0, wc = 0;
      walk(t.root, &wb, &wl, &wc);
      uint8_t wsig[32];
      oracle_sha256(wb, wl, wsig);
      printf("build");
      for (uint32_t b = 0; b < B; b++) printf(" %" PRIu64, digest[b]);
      printf(" ;");
      for (uint32_t b = 0; b < B; b++) printf(" %d", size[b]);
      printf(" ; %d ; ", items);
      print_hex(t.root->hash, 32);
      printf(" ; %u ", t.n_leafs);
      print_hex(wsig, 32);
      printf(" ; %" PRIu64 " %d\n", compressions, tamper_ok);
      if (!host_tree && !resident && memcmp(root, t.root->hash, 32)) { /* split levels: no device root */
        fprintf(stderr, "device root differs from the assembled tree's root\n");
        return 1;
      }
      free(wb), free(t.pool), free(t.leaf_hash), free(t.node_hash), free(nodes);
      free(tt.pool), free(tt.leaf_hash), free(tt.node_hash), free(tampered), free(memo.leaf);
      free(bucket), free(values), free(value_off), free(seg_rec), free(digest), free(size);
    } else if (!strcmp(op, "diff")) {
      const uint32_t Ba = (uint32_t)num(f), Bb = (uint32_t)num(f);
      uint64_t* da = xmalloc((uint64_t)Ba * 8);
      uint64_t* db = xmalloc((uint64_t)Bb * 8);
      for (uint32_t i = 0; i < Ba; i++) da[i] = num(f);
      for (uint32_t i = 0; i < Bb; i++) db[i] = num(f);
      uint8_t ra[32], rb[32];
      uint8_t* na = xmalloc(mde_tree_internal_nodes(Ba) * 32);
      uint8_t* nb = xmalloc(mde_tree_internal_nodes(Bb) * 32);
      if ((rc = mde_tree_from_digests(ctx, 1, Ba, da, ra, na)) || (rc = mde_tree_from_digests(ctx, 1, Bb, db, rb, nb))) {
        fprintf(stderr, "mde_tree_from_digests: %d %s\n", rc, mde_last_error(ctx));
        return 1;
      }
      stree ta = mde_tree(da, Ba, na), tb = mde_tree(db, Bb, nb);
      int32_t* ids = xmalloc(((uint64_t)Ba + Bb + 2) * 8);
      int32_t count = 0;
      if (ref_dfs(ta.root, tb.root, ids, &count)) count = MDE_E_TREE;
      printf("diff %d", count);
      for (int32_t i = 0; i < count; i++) printf(" %d", ids[i]);
      printf("\n");
      free(ta.pool), free(ta.leaf_hash), free(ta.node_hash), free(tb.pool), free(tb.leaf_hash), free(tb.node_hash);
      free(na), free(nb);
      free(da), free(db), free(ids);
    } else if (!strcmp(op, "verify")) {
      const uint32_t B = (uint32_t)num(f);
      const int32_t part = (int32_t)num(f);
      const int64_t epoch = (int64_t)num(f);
      const uint32_t replicas = (uint32_t)num(f), R = (uint32_t)num(f);
      uint64_t* digest = xmalloc((uint64_t)B * 8);
      int32_t* size = xmalloc((uint64_t)B * 4);
      for (uint32_t i = 0; i < B; i++) digest[i] = num(f);
      for (uint32_t i = 0; i < B; i++) size[i] = (int32_t)num(f);
      uint8_t* blob = NULL;
      uint64_t blen = 0, bcap = 0;
      uint64_t* off = xmalloc(((uint64_t)R + 1) * 8);
      for (uint32_t i = 0; i < R; i++) { /* proto.Marshal of each peer object, concatenated */
        hex(f, &blob, &blen, &bcap);
        off[i + 1] = blen;
      }
      blob = realloc(blob, blen + 1); /* blob = append(blob, 0) */
      const uint64_t stride = mde_epoch_tree_object_max_bytes(B);
      uint8_t* obj = xmalloc(stride);
      int32_t* ids = xmalloc((uint64_t)B * 4);
      int32_t* status = xmalloc(((uint64_t)R + 1) * 4);
      uint8_t valid = 0;
      int32_t vc = 0, dc = 0;
      uint32_t olen = 0;
      rc = resident ? mde_server_verify(server, B, part, epoch, digest, size, R, blob, off, replicas, &valid, &vc, ids,
                                        &dc, status, obj, stride, &olen, err, sizeof err)
                    : mde_batch_verify(batcher, B, part, epoch, digest, size, R, blob, off, replicas, &valid, &vc, ids,
                                       &dc, status, obj, stride, &olen, err, sizeof err);
      if (rc) {
        fprintf(stderr, "verify: %d %s\n", rc, err);
        return 1;
      }
      printf("verify %d %d ;", valid, vc);
      for (int32_t i = 0; i < dc; i++) printf(" %d", ids[i]);
      printf(" ;");
      for (uint32_t i = 0; i < R; i++) printf(" %d", status[i]);
      printf(" ; ");
      print_hex(obj, olen);
      printf("\n");
      free(digest), free(size), free(blob), free(off), free(obj), free(ids), free(status);
    } else {
      fprintf(stderr, "unknown op %s\n", op);
      return 2;
    }
  }
  fclose(f);
  mde_batcher_destroy(batcher);
  mde_server_destroy(server);
  mde_destroy(ctx);
  return 0;
}
