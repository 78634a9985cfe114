/* oracle_asan.c -- the C oracle (oracle/mde_oracle.c, test infrastructure) under AddressSanitizer
 * and UndefinedBehaviorSanitizer on the host: the checker every GPU parity test trusts must not
 * read out of bounds or overflow on the shapes those tests feed it. Built and run by
 * tests/test_oracle_sanitized.py (gcc -fsanitize=address,undefined, CPU only).
 *
 * Over seeded random shapes (P partitions, B buckets incl. odd B and B = 1, zero-heavy and skewed
 * counts, fixed strides incl. 1 and odd, variable lengths incl. empty values):
 *   - oracle_build with 1 and 3 threads agree;
 *   - oracle_tree over the build's digests gives the build's root and nodes;
 *   - oracle_graph_build and oracle_graph_from_nodes give the same root; a tree with one digest
 *     changed diffs to exactly that bucket (reference DFS duplicates allowed, every id that bucket);
 *   - oracle_layout_a sorts random tags into valid segments;
 * plus the SHA-256 ("abc") and XXH64 (empty input) known answers. Prints "ok" and exits 0. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_sha256(const uint8_t* msg, uint64_t len, uint8_t out[32]);
uint64_t oracle_xxh64(const uint8_t* p, uint64_t len, uint64_t seed);
int oracle_layout_a(const uint32_t* part, const uint32_t* bucket, uint64_t n, uint32_t n_partitions,
                    uint32_t n_buckets, uint64_t* order, uint64_t* seg_rec);
uint64_t oracle_n_internal(uint32_t n_buckets);
int oracle_tree(const uint64_t* digest, uint32_t n_buckets, uint8_t* nodes, uint8_t* root);
int oracle_build(const uint8_t* values, uint32_t stride, const uint64_t* value_off, const uint64_t* seg_rec,
                 uint32_t n_partitions, uint32_t n_buckets, uint64_t* digest, int32_t* size, int32_t* items,
                 uint8_t* root, uint8_t* nodes, int threads);
typedef struct oracle_graph oracle_graph;
oracle_graph* oracle_graph_build(const uint64_t* digest, uint32_t n_buckets);
oracle_graph* oracle_graph_from_nodes(const uint64_t* digest, uint32_t n_buckets, const uint8_t* nodes);
const uint8_t* oracle_graph_root(const oracle_graph* g);
int32_t oracle_graph_diff(const oracle_graph* a, const oracle_graph* b, int32_t* out, int32_t cap);
void oracle_graph_free(oracle_graph* g);

static uint64_t rng_state = 0x4D445354u;
static uint64_t rnd(void) { /* splitmix64 */
  uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static uint32_t below(uint32_t n) { return (uint32_t)(rnd() % n); }

#define CHECK(cond, ...)                    \
  do {                                      \
    if (!(cond)) {                          \
      fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);         \
      fprintf(stderr, "\n");                \
      exit(1);                              \
    }                                       \
  } while (0)

static void known_answers(void) {
  static const uint8_t abc[32] = {0xba, 0x78, 0x16, 0xbf, 0x8f, 0x01, 0xcf, 0xea, 0x41, 0x41, 0x40,
                                  0xde, 0x5d, 0xae, 0x22, 0x23, 0xb0, 0x03, 0x61, 0xa3, 0x96, 0x17,
                                  0x7a, 0x9c, 0xb4, 0x10, 0xff, 0x61, 0xf2, 0x00, 0x15, 0xad};
  uint8_t h[32];
  oracle_sha256((const uint8_t*)"abc", 3, h);
  CHECK(!memcmp(h, abc, 32), "sha256(abc)");
  CHECK(oracle_xxh64((const uint8_t*)"", 0, 0) == 0xEF46DB3751D8E999ull, "xxh64('')");
}

static void one_case(int c) {
  static const uint32_t Bs[] = {1, 2, 3, 7, 30, 64, 65, 100, 257, 1000};
  static const uint32_t strides[] = {1, 3, 8, 13, 16, 64, 100, 1024};
  const uint32_t P = 1 + below(5), B = Bs[below(sizeof Bs / sizeof Bs[0])];
  const uint64_t S = (uint64_t)P * B;
  uint64_t* seg = (uint64_t*)calloc(S + 1, 8);
  for (uint64_t s = 0; s < S; s++) {
    const uint32_t mode = c % 3;
    uint64_t k = mode == 0 ? (below(5) == 0 ? below(6) : 0) : mode == 1 ? below(12) : (below(40) == 0 ? 100 + below(400) : below(3));
    seg[s + 1] = seg[s] + k;
  }
  const uint64_t n = seg[S];
  const int var = below(3) == 0;
  const uint32_t stride = var ? 0 : strides[below(sizeof strides / sizeof strides[0])];
  uint64_t* voff = NULL;
  uint64_t bytes = n * stride;
  if (var) {
    voff = (uint64_t*)malloc((n + 1) * 8);
    voff[0] = 0;
    for (uint64_t i = 0; i < n; i++) voff[i + 1] = voff[i] + below(4) * below(90); /* empty values too */
    bytes = voff[n];
  }
  uint8_t* vals = (uint8_t*)malloc(bytes ? bytes : 1);
  for (uint64_t i = 0; i < bytes; i++) vals[i] = (uint8_t)rnd();
  const uint64_t NI = oracle_n_internal(B);
  uint64_t *d1 = (uint64_t*)malloc(S * 8), *d3 = (uint64_t*)malloc(S * 8);
  int32_t *s1 = (int32_t*)malloc(S * 4), *s3 = (int32_t*)malloc(S * 4);
  int32_t *i1 = (int32_t*)malloc(P * 4), *i3 = (int32_t*)malloc(P * 4);
  uint8_t *r1 = (uint8_t*)malloc(P * 32), *r3 = (uint8_t*)malloc(P * 32);
  uint8_t *n1 = (uint8_t*)malloc(P * NI * 32 + 1), *n3 = (uint8_t*)malloc(P * NI * 32 + 1);
  CHECK(oracle_build(vals, stride, voff, seg, P, B, d1, s1, i1, r1, n1, 1) == 0, "build");
  CHECK(oracle_build(vals, stride, voff, seg, P, B, d3, s3, i3, r3, n3, 3) == 0, "build threads");
  CHECK(!memcmp(d1, d3, S * 8) && !memcmp(s1, s3, S * 4) && !memcmp(i1, i3, P * 4) && !memcmp(r1, r3, P * 32) &&
            !memcmp(n1, n3, P * NI * 32),
        "case %d: thread counts disagree", c);
  for (uint32_t p = 0; p < P; p++) {
    uint8_t root[32];
    uint8_t* nodes = (uint8_t*)malloc(NI * 32 + 1);
    CHECK(oracle_tree(d1 + (uint64_t)p * B, B, nodes, root) == 0, "tree");
    CHECK(!memcmp(root, r1 + p * 32, 32) && !memcmp(nodes, n1 + (uint64_t)p * NI * 32, NI * 32),
          "case %d: tree != build", c);
    oracle_graph* g = oracle_graph_build(d1 + (uint64_t)p * B, B);
    oracle_graph* h = oracle_graph_from_nodes(d1 + (uint64_t)p * B, B, nodes);
    CHECK(g && h && !memcmp(oracle_graph_root(g), root, 32) && !memcmp(oracle_graph_root(h), root, 32),
          "case %d: graph roots", c);
    uint64_t* d2 = (uint64_t*)malloc(B * 8);
    memcpy(d2, d1 + (uint64_t)p * B, B * 8);
    const uint32_t b = below(B);
    d2[b] = (d2[b] + 1) % 999999;
    oracle_graph* g2 = oracle_graph_build(d2, B);
    int32_t ids[4096];
    const int32_t k = oracle_graph_diff(g, g2, ids, 4096);
    CHECK(k >= 1, "case %d: diff found nothing (%d)", c, k);
    for (int32_t j = 0; j < k; j++) CHECK(ids[j] == (int32_t)b, "case %d: diff id %d, want %u", c, ids[j], b);
    CHECK(oracle_graph_diff(g, h, ids, 4096) == 0, "case %d: equal trees differ", c);
    oracle_graph_free(g);
    oracle_graph_free(h);
    oracle_graph_free(g2);
    free(d2);
    free(nodes);
  }
  /* layout A over random tags */
  const uint64_t m = 1 + below(3000);
  uint32_t *pt = (uint32_t*)malloc(m * 4), *bk = (uint32_t*)malloc(m * 4);
  for (uint64_t i = 0; i < m; i++) {
    pt[i] = below(P);
    bk[i] = below(B);
  }
  uint64_t* order = (uint64_t*)malloc(m * 8);
  uint64_t* sg = (uint64_t*)malloc((S + 1) * 8);
  CHECK(oracle_layout_a(pt, bk, m, P, B, order, sg) == 0, "layout_a");
  CHECK(sg[0] == 0 && sg[S] == m, "layout_a bounds");
  for (uint64_t s = 0; s < S; s++)
    for (uint64_t r = sg[s]; r < sg[s + 1]; r++)
      CHECK((uint64_t)pt[order[r]] * B + bk[order[r]] == s, "case %d: layout_a slot", c);
  free(pt); free(bk); free(order); free(sg);
  free(d1); free(d3); free(s1); free(s3); free(i1); free(i3); free(r1); free(r3); free(n1); free(n3);
  free(vals); free(voff); free(seg);
}

int main(int argc, char** argv) {
  const int cases = argc > 1 ? atoi(argv[1]) : 120;
  known_answers();
  for (int c = 0; c < cases; c++) one_case(c);
  printf("ok %d cases\n", cases);
  return 0;
}
