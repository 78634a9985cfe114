/*
 * mde_oracle.c -- CPU restatement of the reference anti-entropy Merkle path.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the HIP engine and the "port" CPU baseline timed
 * by bench.py. Nothing in mydatastore_amd/ links, loads or calls this file. Parity status is
 * described in oracle/oracle.py's header (absolute tree bytes: relationally pinned only).
 *
 * Reference shape (paths relative to the reference root):
 *   CustomHash.Add            main/merkle_tree.go:25-32   value = (value + sum(bytes)) % 999999
 *   MerkleBucket.CalculateHash main/merkle_tree.go:64-71  leaf = LE64(value) (utils/utils.go:67-74)
 *   RawPartitionMerkleTree    main/merkle_tree.go:86-116  per bucket, per record Add; size++
 *   merkletree.NewTree        cbergoon/merkletree v0.2.0  SHA256(L||R), dup last leaf if odd,
 *                                                         odd level: last node pairs with itself
 *   DifferentMerkleTreeBucketsDFS main/merkle_tree.go:163-216
 *   getKeyBucket              main/manager.go:773-778     BE64(SHA256(key)[:8]) % B
 *   FindPartitionID           hashring/hashring.go:108-110 XXH64(key, 0) % P
 * SHA-256 is written from FIPS 180-4, XXH64 from the published xxHash specification.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define HASH_MOD 999999ULL

/* ------------------------------------------------------------------ SHA-256 (FIPS 180-4) */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static inline uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void sha256_block(uint32_t st[8], const uint8_t blk[64]) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) |
           ((uint32_t)blk[4 * i + 2] << 8) | (uint32_t)blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = h + (ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* The same compression with the x86 SHA extensions, as Go's crypto/sha256 uses them on amd64
 * when the CPU has them (the reference is Go 1.20, main/go.mod:3): the CPU baseline then hashes
 * at the rate the reference's own SHA-256 calls would. Chosen at run time (CPUID leaf 7, EBX bit
 * 29); MDE_ORACLE_SHA=portable forces the portable path above (the two are compared in
 * tests/test_oracle.py). */
#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
__attribute__((target("sha,sse4.1,ssse3"))) static void sha256_block_ni(uint32_t st[8], const uint8_t blk[64]) {
  const __m128i mask = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
  __m128i tmp = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&st[0]), 0xB1); /* CDAB */
  __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)&st[4]), 0x1B);  /* EFGH */
  __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);                                        /* ABEF */
  s1 = _mm_blend_epi16(s1, tmp, 0xF0);                                             /* CDGH */
  const __m128i abef = s0, cdgh = s1;
  __m128i w[4];
  for (int g = 0; g < 16; g++) { /* four rounds per group */
    __m128i m;
    if (g < 4) {
      m = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(blk + 16 * g)), mask);
    } else {
      const __m128i a = w[g & 3], b = w[(g + 1) & 3], c = w[(g + 2) & 3], d = w[(g + 3) & 3];
      m = _mm_sha256msg2_epu32(_mm_add_epi32(_mm_sha256msg1_epu32(a, b), _mm_alignr_epi8(d, c, 4)), d);
    }
    w[g & 3] = m;
    __m128i k = _mm_add_epi32(m, _mm_loadu_si128((const __m128i*)&K256[4 * g]));
    s1 = _mm_sha256rnds2_epu32(s1, s0, k);
    s0 = _mm_sha256rnds2_epu32(s0, s1, _mm_shuffle_epi32(k, 0x0E));
  }
  s0 = _mm_add_epi32(s0, abef);
  s1 = _mm_add_epi32(s1, cdgh);
  tmp = _mm_shuffle_epi32(s0, 0x1B);                   /* FEBA */
  s1 = _mm_shuffle_epi32(s1, 0xB1);                    /* DCHG */
  _mm_storeu_si128((__m128i*)&st[0], _mm_blend_epi16(tmp, s1, 0xF0)); /* DCBA */
  _mm_storeu_si128((__m128i*)&st[4], _mm_alignr_epi8(s1, tmp, 8));    /* HGFE */
}

static int sha_ni_usable(void) {
  static int v = -1;
  if (v < 0) {
    unsigned a, b, c, d;
    const char* e = getenv("MDE_ORACLE_SHA");
    v = !(e && !strcmp(e, "portable")) && __get_cpuid_count(7, 0, &a, &b, &c, &d) && ((b >> 29) & 1u);
  }
  return v;
}
#endif

static void sha256_compress(uint32_t st[8], const uint8_t blk[64]) {
#if defined(__x86_64__)
  if (sha_ni_usable()) {
    sha256_block_ni(st, blk);
    return;
  }
#endif
  sha256_block(st, blk);
}

/* 1 when oracle_sha256 runs on the SHA extensions (reported with the CPU baseline). */
int oracle_sha_ni(void) {
#if defined(__x86_64__)
  return sha_ni_usable();
#else
  return 0;
#endif
}

void oracle_sha256(const uint8_t* msg, uint64_t len, uint8_t out[32]) {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint64_t i = 0;
  for (; i + 64 <= len; i += 64) sha256_compress(st, msg + i);
  uint8_t tail[128];
  uint64_t rem = len - i;
  memset(tail, 0, sizeof tail);
  memcpy(tail, msg + i, rem);
  tail[rem] = 0x80;
  uint64_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = len * 8;
  for (int k = 0; k < 8; k++) tail[tl - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha256_compress(st, tail);
  if (tl == 128) sha256_compress(st, tail + 64);
  for (int k = 0; k < 8; k++) {
    out[4 * k] = (uint8_t)(st[k] >> 24); out[4 * k + 1] = (uint8_t)(st[k] >> 16);
    out[4 * k + 2] = (uint8_t)(st[k] >> 8); out[4 * k + 3] = (uint8_t)st[k];
  }
}

/* ------------------------------------------------------------------ XXH64 (xxHash spec) */
#define P64_1 0x9E3779B185EBCA87ULL
#define P64_2 0xC2B2AE3D27D4EB4FULL
#define P64_3 0x165667B19E3779F9ULL
#define P64_4 0x85EBCA77C2B2AE63ULL
#define P64_5 0x27D4EB2F165667C5ULL
static inline uint64_t rol64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * P64_2; acc = rol64(acc, 31); return acc * P64_1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t v) {
  acc ^= xround(0, v); return acc * P64_1 + P64_4;
}

uint64_t oracle_xxh64(const uint8_t* p, uint64_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8));
      v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rol64(v1, 1) + rol64(v2, 7) + rol64(v3, 12) + rol64(v4, 18);
    h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
  } else {
    h = seed + P64_5;
  }
  h += len;
  while (p + 8 <= end) { h ^= xround(0, rd64(p)); h = rol64(h, 27) * P64_1 + P64_4; p += 8; }
  if (p + 4 <= end) { h ^= (uint64_t)rd32(p) * P64_1; h = rol64(h, 23) * P64_2 + P64_3; p += 4; }
  while (p < end) { h ^= (*p) * P64_5; h = rol64(h, 11) * P64_1; p++; }
  h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32;
  return h;
}

/* ------------------------------------------------------------------ write-time tagging */
uint32_t oracle_key_bucket(const uint8_t* key, uint64_t len, uint32_t n_buckets) {
  uint8_t d[32];
  oracle_sha256(key, len, d);
  uint64_t be = 0;
  for (int i = 0; i < 8; i++) be = (be << 8) | d[i];
  return (uint32_t)(be % n_buckets);
}

uint32_t oracle_find_partition(const uint8_t* key, uint64_t len, uint32_t n_partitions) {
  return (uint32_t)(oracle_xxh64(key, len, 0) % n_partitions);
}

/* ------------------------------------------------------------------ synthetic workload */
static inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* dst[i*value_len ..] = value bytes of record gids[i] (SURVEY.md section 8d generator). */
void oracle_synth_values(uint8_t* dst, const uint64_t* gids, uint64_t n, uint32_t value_len,
                         uint64_t seed) {
  for (uint64_t i = 0; i < n; i++) {
    uint8_t* o = dst + i * (uint64_t)value_len;
    for (uint32_t w = 0; w * 8 < value_len; w++) {
      uint64_t x = splitmix64(seed ^ ((gids[i] << 20) + w));
      uint32_t nb = value_len - w * 8 < 8 ? value_len - w * 8 : 8;
      for (uint32_t k = 0; k < nb; k++) o[w * 8 + k] = (uint8_t)(x >> (8 * k));
    }
  }
}

/* part_mode: 0 = block (gid / kpp), 1 = mod (gid % P), 2 = hash (FindPartitionID).
 * Outputs: part[n], bucket[n] for keys "k%016x" % gid. */
void oracle_synth_tags(const uint64_t* gids, uint64_t n, uint32_t n_partitions, uint32_t n_buckets,
                       int part_mode, uint64_t keys_per_partition, uint32_t* part, uint32_t* bucket) {
  char key[32];
  for (uint64_t i = 0; i < n; i++) {
    int kl = snprintf(key, sizeof key, "k%016llx", (unsigned long long)gids[i]);
    bucket[i] = oracle_key_bucket((const uint8_t*)key, (uint64_t)kl, n_buckets);
    if (part_mode == 0) part[i] = (uint32_t)(gids[i] / keys_per_partition);
    else if (part_mode == 1) part[i] = (uint32_t)(gids[i] % n_partitions);
    else part[i] = oracle_find_partition((const uint8_t*)key, (uint64_t)kl, n_partitions);
  }
}

/* Layout A (LSM order): stable counting sort by (partition, bucket).
 * order[n] = input index of the record at each sorted slot; seg_rec[P*B+1] boundaries. */
int oracle_layout_a(const uint32_t* part, const uint32_t* bucket, uint64_t n, uint32_t n_partitions,
                    uint32_t n_buckets, uint64_t* order, uint64_t* seg_rec) {
  uint64_t S = (uint64_t)n_partitions * n_buckets;
  memset(seg_rec, 0, (S + 1) * sizeof(uint64_t));
  for (uint64_t i = 0; i < n; i++) {
    if (part[i] >= n_partitions || bucket[i] >= n_buckets) return -1;
    seg_rec[(uint64_t)part[i] * n_buckets + bucket[i] + 1]++;
  }
  for (uint64_t s = 0; s < S; s++) seg_rec[s + 1] += seg_rec[s];
  uint64_t* cur = (uint64_t*)malloc(S * sizeof(uint64_t));
  if (!cur) return -2;
  memcpy(cur, seg_rec, S * sizeof(uint64_t));
  for (uint64_t i = 0; i < n; i++) order[cur[(uint64_t)part[i] * n_buckets + bucket[i]]++] = i;
  free(cur);
  return 0;
}

/* ------------------------------------------------------------------ bucket digests */
/* Reference shape: per partition, per bucket, per record CustomHash.Add then size++.
 * value_stride != 0: record r = values[r*stride, (r+1)*stride); else value_off[N+1]. */
static void digests_partition(const uint8_t* values, uint32_t stride, const uint64_t* value_off,
                              const uint64_t* seg_rec, uint32_t p, uint32_t n_buckets,
                              uint64_t* digest, int32_t* size, int32_t* items) {
  int32_t it = 0;
  for (uint32_t b = 0; b < n_buckets; b++) {
    uint64_t s = (uint64_t)p * n_buckets + b;
    int64_t value = 0;                       /* CustomHash{value int64} */
    int32_t sz = 0;
    for (uint64_t r = seg_rec[s]; r < seg_rec[s + 1]; r++) {
      uint64_t lo = stride ? r * stride : value_off[r];
      uint64_t hi = stride ? lo + stride : value_off[r + 1];
      int64_t sum = 0;
      for (uint64_t j = lo; j < hi; j++) sum += values[j];
      value += sum;
      value = value % (int64_t)HASH_MOD;
      sz++;
    }
    digest[s] = (uint64_t)value;
    size[s] = sz;
    it += sz;
    if (b == n_buckets - 1 && (n_buckets & 1)) it += sz;  /* tree.Leafs includes the dup leaf */
  }
  if (items) items[p] = it;
}

int oracle_bucket_digests(const uint8_t* values, uint32_t stride, const uint64_t* value_off,
                          const uint64_t* seg_rec, uint32_t n_partitions, uint32_t n_buckets,
                          uint64_t* digest, int32_t* size, int32_t* items) {
  for (uint32_t p = 0; p < n_partitions; p++)
    digests_partition(values, stride, value_off, seg_rec, p, n_buckets, digest, size, items);
  return 0;
}

/* ------------------------------------------------------------------ tree (array form) */
uint32_t oracle_level_count(uint32_t n_buckets, uint32_t* sizes /* may be NULL, cap 64 */) {
  uint32_t n = n_buckets + (n_buckets & 1), lv = 0;
  if (sizes) sizes[lv] = n;
  while (n > 1) { n = (n + 1) / 2; lv++; if (sizes) sizes[lv] = n; }
  return lv + 1;
}

uint64_t oracle_n_internal(uint32_t n_buckets) {
  uint32_t sz[64];
  uint32_t L = oracle_level_count(n_buckets, sz);
  uint64_t t = 0;
  for (uint32_t k = 1; k < L; k++) t += sz[k];
  return t;
}

/* nodes: internal nodes level 1..root, 32 bytes each (may be NULL); root: 32 bytes. */
int oracle_tree(const uint64_t* digest, uint32_t n_buckets, uint8_t* nodes, uint8_t* root) {
  if (n_buckets == 0) return -1;
  uint32_t n0 = n_buckets + (n_buckets & 1);
  uint8_t* cur = (uint8_t*)malloc((size_t)n0 * 32);
  uint8_t* nxt = (uint8_t*)malloc((size_t)n0 * 32);
  if (!cur || !nxt) { free(cur); free(nxt); return -2; }
  uint32_t hl = 8;                                      /* leaf hash = 8 bytes LE */
  for (uint32_t i = 0; i < n0; i++) {
    uint64_t d = digest[i < n_buckets ? i : n_buckets - 1];
    for (int k = 0; k < 8; k++) cur[i * 32 + k] = (uint8_t)(d >> (8 * k));
  }
  uint32_t n = n0;
  uint64_t off = 0;
  uint8_t msg[64];
  while (n > 1) {
    uint32_t m = (n + 1) / 2;
    for (uint32_t j = 0; j < m; j++) {
      uint32_t l = 2 * j, r = (2 * j + 1 < n) ? 2 * j + 1 : 2 * j;
      memcpy(msg, cur + l * 32, hl);
      memcpy(msg + hl, cur + r * 32, hl);
      oracle_sha256(msg, 2 * hl, nxt + j * 32);
    }
    if (nodes) memcpy(nodes + off * 32, nxt, (size_t)m * 32);
    off += m;
    uint8_t* t = cur; cur = nxt; nxt = t;
    n = m;
    hl = 32;
  }
  memcpy(root, cur, 32);
  free(cur); free(nxt);
  return 0;
}

/* ------------------------------------------------------------------ full build */
typedef struct {
  const uint8_t* values; uint32_t stride; const uint64_t* value_off; const uint64_t* seg_rec;
  uint32_t n_partitions, n_buckets; uint64_t* digest; int32_t* size; int32_t* items;
  uint8_t* root; uint8_t* nodes; uint64_t n_int; uint32_t p_begin, p_step;
} build_job;

static void* build_worker(void* arg) {
  build_job* j = (build_job*)arg;
  for (uint32_t p = j->p_begin; p < j->n_partitions; p += j->p_step) {
    digests_partition(j->values, j->stride, j->value_off, j->seg_rec, p, j->n_buckets, j->digest,
                      j->size, j->items);
    oracle_tree(j->digest + (uint64_t)p * j->n_buckets, j->n_buckets,
                j->nodes ? j->nodes + (uint64_t)p * j->n_int * 32 : NULL, j->root + (uint64_t)p * 32);
  }
  return NULL;
}

/* RawPartitionMerkleTree over P partitions, `threads` partitions in flight (mirrors
 * PARTITION_CONCURRENCY verify workers, main/consistency_controller.go:79-81). */
int oracle_build(const uint8_t* values, uint32_t stride, const uint64_t* value_off,
                 const uint64_t* seg_rec, uint32_t n_partitions, uint32_t n_buckets,
                 uint64_t* digest, int32_t* size, int32_t* items, uint8_t* root, uint8_t* nodes,
                 int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  build_job jobs[256];
  pthread_t tids[256];
  uint64_t n_int = oracle_n_internal(n_buckets);
  for (int t = 0; t < threads; t++) {
    build_job j = {values, stride, value_off, seg_rec, n_partitions, n_buckets, digest, size, items,
                   root, nodes, n_int, (uint32_t)t, (uint32_t)threads};
    jobs[t] = j;
  }
  if (threads == 1) { build_worker(&jobs[0]); return 0; }
  for (int t = 0; t < threads; t++) pthread_create(&tids[t], NULL, build_worker, &jobs[t]);
  for (int t = 0; t < threads; t++) pthread_join(tids[t], NULL);
  return 0;
}

/* ------------------------------------------------------------------ DFS diff (pointer form) */
typedef struct onode {
  struct onode *left, *right;
  uint8_t hash[32];
  uint32_t hlen;
  int32_t bucket_id;   /* leaf content (MerkleBucket.bucketId); -1 = internal (C == nil) */
} onode;

/* Builds merkletree.NewTree's node graph from digests; returns root, *pool to free. */
static onode* build_nodes(const uint64_t* digest, uint32_t n_buckets, onode** pool) {
  uint32_t sz[64];
  uint32_t L = oracle_level_count(n_buckets, sz);
  uint64_t total = 0;
  for (uint32_t k = 0; k < L; k++) total += sz[k];
  onode* all = (onode*)calloc(total, sizeof(onode));
  if (!all) return NULL;
  *pool = all;
  onode* lvl = all;
  for (uint32_t i = 0; i < sz[0]; i++) {
    uint32_t src = i < n_buckets ? i : n_buckets - 1;     /* dup leaf: same hash, same content */
    for (int k = 0; k < 8; k++) lvl[i].hash[k] = (uint8_t)(digest[src] >> (8 * k));
    lvl[i].hlen = 8;
    lvl[i].bucket_id = (int32_t)src;
  }
  for (uint32_t k = 1; k < L; k++) {
    onode* up = lvl + sz[k - 1];
    for (uint32_t j = 0; j < sz[k]; j++) {
      onode* l = &lvl[2 * j];
      onode* r = (2 * j + 1 < sz[k - 1]) ? &lvl[2 * j + 1] : &lvl[2 * j];
      uint8_t msg[64];
      memcpy(msg, l->hash, l->hlen);
      memcpy(msg + l->hlen, r->hash, r->hlen);
      oracle_sha256(msg, l->hlen + r->hlen, up[j].hash);
      up[j].hlen = 32;
      up[j].left = l; up[j].right = r;
      up[j].bucket_id = -1;
    }
    lvl = up;
  }
  return lvl;   /* level L-1 has exactly one node: the root */
}

/* Returns 0 ok, -1 error (nil node / bucket-id mismatch / bad content), -2 out of capacity. */
static int dfs(const onode* a, const onode* b, int32_t* out, int32_t cap, int32_t* n) {
  if (!a && !b) return 0;
  if (!a || !b) return -1;
  if (a->hlen == b->hlen && memcmp(a->hash, b->hash, a->hlen) == 0) return 0;
  if (!a->left && !a->right) {
    if (a->bucket_id < 0 || b->bucket_id < 0) return -1;
    if (a->bucket_id != b->bucket_id) return -1;
    if (*n >= cap) return -2;
    out[(*n)++] = a->bucket_id;
    return 0;
  }
  int rc = dfs(a->left, b->left, out, cap, n);
  if (rc) return rc;
  return dfs(a->right, b->right, out, cap, n);
}

/* DifferentMerkleTreeBuckets(tree(d1), tree(d2)): returns count >= 0, or -1 error, -2 capacity. */
int32_t oracle_diff(const uint64_t* d1, uint32_t b1, const uint64_t* d2, uint32_t b2, int32_t* out,
                    int32_t cap) {
  onode *p1 = NULL, *p2 = NULL;
  onode* r1 = build_nodes(d1, b1, &p1);
  onode* r2 = build_nodes(d2, b2, &p2);
  int32_t n = 0;
  int rc = (r1 && r2) ? dfs(r1, r2, out, cap, &n) : -2;
  free(p1); free(p2);
  return rc ? rc : n;
}

/* ------------------------------------------------------------------ trees as node graphs */
/* A merkletree.MerkleTree-shaped node graph (what a Go caller holds after NewTree), for timing the
 * host-side steps of the production call shape (tests/cpp/batch_bench.c):
 *   oracle_graph_build      -- merkletree.NewTree from digests (SHA-256 of every internal node);
 *   oracle_graph_from_nodes -- the same graph assembled from node hashes computed elsewhere (the
 *                              Go shim's tree from the device's nodes: no hashing);
 *   oracle_graph_diff       -- DifferentMerkleTreeBucketsDFS over two graphs (main/merkle_tree.go:163-216),
 *                              the reference's own diff of two trees it already holds. */
typedef struct oracle_graph {
  onode* pool;
  onode* root;
} oracle_graph;

oracle_graph* oracle_graph_build(const uint64_t* digest, uint32_t n_buckets) {
  oracle_graph* g = (oracle_graph*)calloc(1, sizeof *g);
  if (!g || !n_buckets) { free(g); return NULL; }
  g->root = build_nodes(digest, n_buckets, &g->pool);
  if (!g->root) { free(g); return NULL; }
  return g;
}

oracle_graph* oracle_graph_from_nodes(const uint64_t* digest, uint32_t n_buckets, const uint8_t* nodes) {
  if (!n_buckets || !nodes) return NULL;
  uint32_t sz[64];
  uint32_t L = oracle_level_count(n_buckets, sz);
  uint64_t total = 0;
  for (uint32_t k = 0; k < L; k++) total += sz[k];
  oracle_graph* g = (oracle_graph*)calloc(1, sizeof *g);
  onode* all = (onode*)calloc(total, sizeof(onode));
  if (!g || !all) { free(g); free(all); return NULL; }
  onode* lvl = all;
  for (uint32_t i = 0; i < sz[0]; i++) {
    uint32_t src = i < n_buckets ? i : n_buckets - 1;
    for (int k = 0; k < 8; k++) lvl[i].hash[k] = (uint8_t)(digest[src] >> (8 * k));
    lvl[i].hlen = 8;
    lvl[i].bucket_id = (int32_t)src;
  }
  uint64_t off = 0;
  for (uint32_t k = 1; k < L; k++) {
    onode* up = lvl + sz[k - 1];
    for (uint32_t j = 0; j < sz[k]; j++) {
      memcpy(up[j].hash, nodes + (off + j) * 32, 32);
      up[j].hlen = 32;
      up[j].left = &lvl[2 * j];
      up[j].right = (2 * j + 1 < sz[k - 1]) ? &lvl[2 * j + 1] : &lvl[2 * j];
      up[j].bucket_id = -1;
    }
    off += sz[k];
    lvl = up;
  }
  g->pool = all;
  g->root = lvl;
  return g;
}

/* root hash (32 bytes) of a graph */
const uint8_t* oracle_graph_root(const oracle_graph* g) { return g->root->hash; }

int32_t oracle_graph_diff(const oracle_graph* a, const oracle_graph* b, int32_t* out, int32_t cap) {
  int32_t n = 0;
  int rc = dfs(a->root, b->root, out, cap, &n);
  return rc ? rc : n;
}

void oracle_graph_free(oracle_graph* g) {
  if (!g) return;
  free(g->pool);
  free(g);
}
