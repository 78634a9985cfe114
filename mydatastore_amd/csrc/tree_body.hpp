// tree_body.hpp -- bucket digests -> leaves -> SHA-256 Merkle tree, as a workgroup-level device
// function shared by tree_kernel (tree.hip) and the fused build-step kernel (digest.hip).
//
// Reference semantics:
//   digest = byte-sum % 999999 (CustomHash, main/merkle_tree.go:19-32); size = record count
//   (:91,107,111); items = sum of sizes as int32 (MerkleTreeToPartitionEpochObject, :121-134);
//   leaf bytes = LE64(digest) (MerkleBucket.CalculateHash :64-71, utils/utils.go:67-74);
//   cbergoon/merkletree v0.2.0 NewTree (:115,156): odd leaf count -> duplicate the last leaf;
//   node = SHA256(left || right); the last node of an odd level pairs with itself; the node made
//   from a 2-node level is the root.
// Output node layout: internal nodes level 1 .. root, 32 bytes each (big-endian digest bytes).
//
// Levels live in LDS (ping-pong, <= 96 KiB at B = 4096); larger B reads the previous level back
// from the global node array (same workgroup, ordered by __syncthreads()).
#pragma once
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {

__device__ __forceinline__ void load_node(const uint32_t* src, uint32_t h[8]) {
  const u32x4* s = reinterpret_cast<const u32x4*>(src);
  const u32x4 a = s[0], b = s[1];
  h[0] = bswap(a.x); h[1] = bswap(a.y); h[2] = bswap(a.z); h[3] = bswap(a.w);
  h[4] = bswap(b.x); h[5] = bswap(b.y); h[6] = bswap(b.z); h[7] = bswap(b.w);
}

__device__ __forceinline__ void store_node(uint32_t* dst, const uint32_t st[8]) {
  u32x4* d = reinterpret_cast<u32x4*>(dst);
  d[0] = u32x4{bswap(st[0]), bswap(st[1]), bswap(st[2]), bswap(st[3])};
  d[1] = u32x4{bswap(st[4]), bswap(st[5]), bswap(st[6]), bswap(st[7])};
}

// One lane's half of a node from the two-lane padding block: A lanes words 0..3, E lanes 4..7.
__device__ __forceinline__ void store_half_node(uint32_t* dst, const uint32_t v[4], bool is_a) {
  reinterpret_cast<u32x4*>(dst)[is_a ? 0 : 1] = u32x4{bswap(v[0]), bswap(v[1]), bswap(v[2]), bswap(v[3])};
}

// Leaf b of partition p: digest, and (when building from byte sums) its size/digest outputs.
__device__ __forceinline__ uint64_t tree_leaf(const TreeLaunch& a, uint64_t s, uint32_t& items, uint32_t& sz_out) {
  uint64_t v;
  if (a.sums_in) {
    v = (uint64_t)(a.sums_in[s - a.sums_base] % kHashMod);
    if (a.sums_clear) a.sums_clear[s - a.sums_base] = 0ull;
  } else {
    v = a.digest_in[s];
  }
  if (a.digest_out) a.digest_out[s] = v;
  if (a.seg_rec || a.counts_in) {
    uint32_t sz;  // int32 wrap like Go
    if (a.seg_rec) {
      sz = (uint32_t)(a.seg_rec[s + 1] - a.seg_rec[s]);
    } else {
      sz = a.counts_in[s - a.sums_base];
      a.counts_in[s - a.sums_base] = 0u;
    }
    if (a.size_out) a.size_out[s] = (int32_t)sz;
    items += sz;
    sz_out = sz;
  }
  return v;
}

// Digest-only build (mde_tree_out.root == NULL): the leaf outputs of partition p -- digest, size
// and its share of items -- over `width` lanes (this thread is `lane`), with no SHA-256 tree. The
// caller reduces the returned items over the lanes. The duplicate leaf of an odd B counts its
// size twice, as the tree.Leafs walk does (main/merkle_tree.go:121-134).
__device__ __forceinline__ uint32_t leaves_items(const TreeLaunch& a, uint32_t p, uint32_t lane, uint32_t width) {
  uint32_t items = 0;
  const uint64_t s0 = (uint64_t)p * a.B;
  for (uint32_t b = lane; b < a.B; b += width) {
    uint32_t sz = 0;
    tree_leaf(a, s0 + b, items, sz);
    if (b == a.B - 1 && (a.B & 1u)) items += sz;
  }
  return items;
}

__device__ __forceinline__ uint32_t wave_add_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One wave per partition: partitions wave0, wave0 + waves, ... below a.P (leaves_items + items).
__device__ __forceinline__ void leaves_waves(const TreeLaunch& a, uint32_t wave0, uint32_t waves, uint32_t p_end) {
  const uint32_t lane = threadIdx.x % 64;
  for (uint32_t p = wave0; p < p_end && p < a.P; p += waves) {
    const uint32_t items = wave_add_u32(leaves_items(a, p, lane, 64));
    if (lane == 0 && a.items_out) a.items_out[p] = (int32_t)items;
  }
}

// One workgroup (`block` = its index among the tree workgroups) builds threads / G trees with its
// first `threads` threads (a multiple of 64): a "group" of G threads per partition. Waves past
// `threads` leave at once, before any barrier (s_barrier waits only for waves still running).
// Every group of a workgroup runs the same level count, so the per-level __syncthreads() is
// uniform.
template <bool kLds>
__device__ __forceinline__ void tree_body(const TreeLaunch& a, uint32_t G, uint32_t lds_words, uint32_t block,
                                          uint32_t* lds, uint32_t threads) {
  if (threadIdx.x >= threads) return;
  const uint32_t groups = threads / G;
  const uint32_t gi = threadIdx.x / G, tid = threadIdx.x % G;
  const uint32_t p = block * groups + gi;
  // Every group runs the level loop of the widest tree (a.B) so that __syncthreads() stays
  // uniform; a group whose own tree (n_in) is narrower idles once it reaches its root.
  const int32_t bt = (a.n_in && p < a.P) ? a.n_in[p] : (int32_t)a.B;
  const bool live = p < a.P && bt > 0 && (uint32_t)bt <= a.B;
  const uint32_t B = live ? (uint32_t)bt : a.B;
  const uint32_t n1 = (B + 1) / 2;  // level-1 nodes (leaf count incl. dup / 2)
  const uint32_t n1_max = (a.B + 1) / 2;
  const uint64_t s0 = (uint64_t)p * a.B;
  uint32_t* node_base = (a.nodes_out && live)
                            ? reinterpret_cast<uint32_t*>(a.nodes_out + (uint64_t)p * a.n_int * 32)
                            : nullptr;
  uint32_t* region = lds + (uint64_t)gi * lds_words;
  uint32_t* counter = region;  // region[0]: items accumulator
  uint32_t* buf0 = kLds ? region + 4 : node_base;
  uint32_t* buf1 = kLds ? region + 4 + (uint64_t)n1_max * 8 : nullptr;
  if (tid == 0) counter[0] = 0;
  __syncthreads();

  // Leaves + level 1.
  uint32_t items = 0;
  if (live) {
    for (uint32_t j = tid; j < n1; j += G) {
      const uint32_t bl = 2 * j, br = (2 * j + 1 < B) ? 2 * j + 1 : 2 * j;
      uint32_t szl = 0, szr = 0;
      const uint64_t dl = tree_leaf(a, s0 + bl, items, szl);
      const uint64_t dr = (br != bl) ? tree_leaf(a, s0 + br, items, szr) : dl;
      if (br == bl) items += szl;  // odd B: the duplicate leaf's size counts again (tree.Leafs walk)
      uint32_t st[8];
      sha256_leaf_pair(dl, dr, st);
      store_node(buf0 + (uint64_t)j * 8, st);
      if (kLds && node_base) store_node(node_base + (uint64_t)j * 8, st);
    }
  }
  if (items) atomicAdd(counter, items);

  // Upper levels.
  uint32_t n_max = n1_max;
  uint32_t n = n1;
  uint64_t level_off = 0;  // node index of the current level's first node in node_base
  uint32_t* cur = buf0;
  uint32_t* nxt = kLds ? buf1 : (node_base ? node_base + (uint64_t)n1 * 8 : nullptr);
  const uint32_t stop = a.top_nodes ? a.top_nodes : 1u;  // uniform B when top_nodes is set
  while (n_max > stop) {
    __syncthreads();
    n_max = (n_max + 1) / 2;
    if (n <= stop) continue;  // this group's tree is complete
    const uint32_t m = (n + 1) / 2;
    if (live) {
      for (uint32_t j = tid; j < m; j += G) {
        const uint32_t l = 2 * j, r = (2 * j + 1 < n) ? 2 * j + 1 : 2 * j;
        uint32_t hl[8], hr[8], st[8];
        load_node(cur + (uint64_t)l * 8, hl);
        load_node(cur + (uint64_t)r * 8, hr);
        sha256_node_pair(hl, hr, st);
        store_node(nxt + (uint64_t)j * 8, st);
        if (kLds && node_base) store_node(node_base + (level_off + n + j) * 8, st);
      }
    }
    level_off += n;
    n = m;
    if (kLds) {
      uint32_t* t = cur; cur = nxt; nxt = t;
    } else if (node_base) {
      cur = nxt;
      nxt = node_base + (level_off + n) * 8;
    }
  }
  __syncthreads();
  if (live) {
    if (tid < 8) reinterpret_cast<uint32_t*>(a.root_out + (uint64_t)p * 32)[tid] = cur[tid];
    if (tid == 0 && a.items_out) a.items_out[p] = (int32_t)counter[0];
  }
}

// Throughput shape for the fused build step: ONE wave builds the trees of Q consecutive
// partitions (same B, byte-sum input), level by level, with the level's Q x n nodes spread over
// the 64 lanes. tree_body's shape (64/G partitions per wave, G = level-1 width) leaves most lanes
// idle above level 1 -- 11 compression rounds per 2 partitions at B = 64 -- where this one takes
// 26 rounds per 16 partitions: 3.4x fewer wave-instructions for the same trees, at a longer
// critical path (26 vs 11 rounds) that the co-running HBM stream hides. Waves past the first
// leave at once. LDS: [Q] item counters, then two level buffers of Q x n1 and Q x ceil(n1/2)
// nodes (packed_tree_lds_words).
__host__ __device__ inline uint32_t packed_tree_lds_words(uint32_t B, uint32_t Q) {
  const uint32_t n1 = (B + 1) / 2;
  return 16u + Q * (n1 + (n1 + 1) / 2) * 8u;
}

__device__ __forceinline__ void tree_body_packed(const TreeLaunch& a, uint32_t Q, uint32_t block, uint32_t* lds) {
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t B = a.B;
  const uint32_t p0 = block * Q;
  if (p0 >= a.P) return;
  const uint32_t nq = min(Q, a.P - p0);
  const uint32_t n1 = (B + 1) / 2;
  uint32_t* cnt = lds;
  uint32_t* cur = lds + 16;
  uint32_t* nxt = cur + (uint64_t)Q * n1 * 8;
  for (uint32_t i = lane; i < Q; i += 64) cnt[i] = 0;
  __syncthreads();

  // Leaves + level 1: item i = (partition q, node j).
  for (uint32_t i = lane; i < nq * n1; i += 64) {
    const uint32_t q = i / n1, j = i - q * n1;
    const uint64_t s0 = (uint64_t)(p0 + q) * B;
    const uint32_t bl = 2 * j, br = (2 * j + 1 < B) ? 2 * j + 1 : 2 * j;
    uint32_t items = 0, szl = 0, szr = 0;
    const uint64_t dl = tree_leaf(a, s0 + bl, items, szl);
    const uint64_t dr = (br != bl) ? tree_leaf(a, s0 + br, items, szr) : dl;
    if (br == bl) items += szl;  // odd B: the duplicate leaf's size counts again (tree.Leafs walk)
    if (items) atomicAdd(cnt + q, items);
    uint32_t st[8];
    sha256_leaf_pair(dl, dr, st);
    store_node(cur + ((uint64_t)q * n1 + j) * 8, st);
    if (a.nodes_out)
      store_node(reinterpret_cast<uint32_t*>(a.nodes_out + ((uint64_t)(p0 + q) * a.n_int + j) * 32), st);
  }
  __syncthreads();

  // Upper levels.
  uint32_t n = n1;
  uint64_t level_off = 0;
  while (n > 1) {
    const uint32_t m = (n + 1) / 2;
    for (uint32_t i = lane; i < nq * m; i += 64) {
      const uint32_t q = i / m, j = i - q * m;
      const uint32_t l = 2 * j, r = (2 * j + 1 < n) ? 2 * j + 1 : 2 * j;
      uint32_t hl[8], hr[8], st[8];
      load_node(cur + ((uint64_t)q * n + l) * 8, hl);
      load_node(cur + ((uint64_t)q * n + r) * 8, hr);
      sha256_node_pair(hl, hr, st);
      store_node(nxt + ((uint64_t)q * m + j) * 8, st);
      if (a.nodes_out)
        store_node(reinterpret_cast<uint32_t*>(a.nodes_out + ((uint64_t)(p0 + q) * a.n_int + level_off + n + j) * 32),
                   st);
    }
    level_off += n;
    n = m;
    uint32_t* t = cur; cur = nxt; nxt = t;
    __syncthreads();
  }
  for (uint32_t i = lane; i < nq * 8; i += 64) {
    const uint32_t q = i / 8, w = i % 8;
    reinterpret_cast<uint32_t*>(a.root_out + (uint64_t)(p0 + q) * 32)[w] = cur[(uint64_t)q * 8 + w];
  }
  if (a.items_out)
    for (uint32_t i = lane; i < nq; i += 64) a.items_out[p0 + i] = (int32_t)cnt[i];
}

// Pair shape for wide trees (level 1 > 64 nodes) with one B for every partition (byte-sum or
// digest input, no n_in): a 256-thread workgroup builds partitions 2*block and 2*block+1, 128
// threads (two waves) each, until a level has <= 64 nodes; then ONE wave finishes both trees,
// their nodes spread over its 64 lanes. tree_body's shape runs those top levels (six at
// B = 1,000) one wave per partition with 32 lanes or fewer busy: 12 of its 34 wave-compressions
// per partition at B = 1,000, here 6, for the same critical path (24 dependent compressions).
// Level 1 never reaches LDS: a thread hashes the two level-1 nodes under its level-2 node and
// that node from registers, which halves the LDS (two trees in 24 KiB at B <= 1,024).
// Used by the standalone tree kernel for >= 512 partitions (tree.hip launch_tree); in the fused
// build step it measured no better than tree_body's two-wave trees (digest.hip plan_step_trees).
// LDS per partition: a 4-word counter slot, then level buffers of n2 and ceil(n2 / 2) nodes.
__host__ __device__ inline uint32_t pair_tree_region_words(uint32_t B) {
  const uint32_t n1 = (B + 1) / 2, n2 = (n1 + 1) / 2;
  return 4u + (n2 + (n2 + 1) / 2) * 8u;
}
__host__ __device__ inline uint32_t pair_tree_lds_words(uint32_t B) { return 2u * pair_tree_region_words(B); }

// Level-1 node j of a tree over B leaves (leaves 2j, 2j+1; the odd last leaf pairs with itself).
__device__ __forceinline__ void tree_level1(const TreeLaunch& a, uint64_t s0, uint32_t B, uint32_t j,
                                            uint32_t& items, uint32_t st[8]) {
  const uint32_t bl = 2 * j, br = (2 * j + 1 < B) ? 2 * j + 1 : 2 * j;
  uint32_t szl = 0, szr = 0;
  const uint64_t dl = tree_leaf(a, s0 + bl, items, szl);
  const uint64_t dr = (br != bl) ? tree_leaf(a, s0 + br, items, szr) : dl;
  if (br == bl) items += szl;  // odd B: the duplicate leaf's size counts again (tree.Leafs walk)
  sha256_leaf_pair(dl, dr, st);
}

constexpr uint32_t kPairTreeThreads = 128;  // threads per partition in the wide phase

__device__ __forceinline__ void tree_body_pair(const TreeLaunch& a, uint32_t block, uint32_t* lds) {
  const uint32_t half = threadIdx.x / kPairTreeThreads, tid = threadIdx.x % kPairTreeThreads;
  const uint32_t p0 = block * 2u;
  const uint32_t p = p0 + half;
  const bool live = p < a.P;
  const uint32_t B = a.B;
  const uint32_t n1 = (B + 1) / 2, n2 = (n1 + 1) / 2;
  const uint32_t rw = pair_tree_region_words(B);
  uint32_t* region = lds + half * rw;
  uint32_t* cur = region + 4;
  uint32_t* nxt = cur + (uint64_t)n2 * 8;
  uint32_t* node_base = (a.nodes_out && live)
                            ? reinterpret_cast<uint32_t*>(a.nodes_out + (uint64_t)p * a.n_int * 32)
                            : nullptr;
  if (tid == 0) region[0] = 0;
  __syncthreads();

  // Leaves, level 1 and level 2 in registers.
  uint32_t items = 0;
  if (live) {
    const uint64_t s0 = (uint64_t)p * B;
    for (uint32_t j = tid; j < n2; j += kPairTreeThreads) {
      const uint32_t l = 2 * j, r = (2 * j + 1 < n1) ? 2 * j + 1 : 2 * j;
      uint32_t hl[8], hr[8], st[8];
      tree_level1(a, s0, B, l, items, hl);
      if (node_base) store_node(node_base + (uint64_t)l * 8, hl);
      if (r != l) {
        tree_level1(a, s0, B, r, items, hr);
        if (node_base) store_node(node_base + (uint64_t)r * 8, hr);
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) hr[k] = hl[k];
      }
      sha256_node_pair(hl, hr, st);
      store_node(cur + (uint64_t)j * 8, st);
      if (node_base) store_node(node_base + (uint64_t)(n1 + j) * 8, st);
    }
  }
  if (items) atomicAdd(region, items);

  // Wide levels, two waves per partition, down to a level of <= 64 nodes.
  uint32_t n = n2;
  uint64_t level_off = n1;  // node index of the current level's first node
  while (n > 64) {
    __syncthreads();
    const uint32_t m = (n + 1) / 2;
    if (live) {
      for (uint32_t j = tid; j < m; j += kPairTreeThreads) {
        const uint32_t l = 2 * j, r = (2 * j + 1 < n) ? 2 * j + 1 : 2 * j;
        uint32_t hl[8], hr[8], st[8];
        load_node(cur + (uint64_t)l * 8, hl);
        load_node(cur + (uint64_t)r * 8, hr);
        sha256_node_pair(hl, hr, st);
        store_node(nxt + (uint64_t)j * 8, st);
        if (node_base) store_node(node_base + (level_off + n + j) * 8, st);
      }
    }
    level_off += n;
    n = m;
    uint32_t* t = cur; cur = nxt; nxt = t;
  }
  __syncthreads();

  // Top levels: wave 0 finishes both trees (the other waves leave; s_barrier counts live waves).
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x;
  const uint32_t nq = p0 >= a.P ? 0u : min(2u, a.P - p0);
  while (n > 1) {
    const uint32_t m = (n + 1) / 2;
    for (uint32_t i = lane; i < nq * m; i += 64) {
      const uint32_t q = i >= m ? 1u : 0u, j = i - q * m;
      const uint32_t l = 2 * j, r = (2 * j + 1 < n) ? 2 * j + 1 : 2 * j;
      const uint32_t* c = cur + q * rw;
      uint32_t hl[8], hr[8], st[8];
      load_node(c + (uint64_t)l * 8, hl);
      load_node(c + (uint64_t)r * 8, hr);
      sha256_node_pair(hl, hr, st);
      store_node(nxt + q * rw + (uint64_t)j * 8, st);
      if (a.nodes_out)
        store_node(reinterpret_cast<uint32_t*>(a.nodes_out + ((uint64_t)(p0 + q) * a.n_int + level_off + n + j) * 32),
                   st);
    }
    level_off += n;
    n = m;
    uint32_t* t = cur; cur = nxt; nxt = t;
    __syncthreads();
  }
  for (uint32_t i = lane; i < nq * 8; i += 64) {
    const uint32_t q = i / 8, w = i % 8;
    reinterpret_cast<uint32_t*>(a.root_out + (uint64_t)(p0 + q) * 32)[w] = cur[q * rw + w];
  }
  if (a.items_out)
    for (uint32_t i = lane; i < nq; i += 64) a.items_out[p0 + i] = (int32_t)lds[i * rw];
}

// Latency form of tree_body for launches with few partitions (the one-partition calls of
// VerifyEpoch, small batches), same outputs. The workgroup is 2 x `half` threads and its upper half
// mirrors the lower half: on every level whose nodes fit the lower half, lower thread x hashes its
// node's rounds while upper thread x + half computes that node's message schedule
// (sha256_node_duo_main / _sched: 64 + 14 x 64 instead of ~2,340 instructions on the critical
// path of each level). Partitions: G <= half -> half / G per workgroup, held by the lower half;
// G = 2 x half (a wide tree, level 1 > 64 nodes) -> one per workgroup, whose levels wider than
// `half` nodes (and level 1) run over all threads as in tree_body. Threads from 2 x half on leave
// at once. Uniform B (no n_in), levels in LDS. kw: duo_kw_bytes(half) of LDS, touched only on
// split levels (it may overlay level-buffer space those levels do not use, duo_step_kw_word).
__host__ __device__ inline uint32_t duo_kw_bytes(uint32_t half) { return 8u * 16u * half; }

__device__ __forceinline__ void tree_body_duo(const TreeLaunch& a, uint32_t G, uint32_t lds_words, uint32_t block,
                                              uint32_t* lds, uint32_t half, u32x4* kw) {
  if (threadIdx.x >= 2 * half) return;
  const uint32_t x = threadIdx.x;
  const bool wide = G > half;
  const bool upper = x >= half;
  const uint32_t xm = upper ? x - half : x;  // the lower thread this one is (or mirrors)
  const uint32_t groups = wide ? 1u : half / G;
  const uint32_t gi = wide ? 0u : xm / G;
  const uint32_t tid = wide ? xm : xm % G;    // node slot within the group on split levels
  const uint32_t p = block * groups + gi;
  const bool live = p < a.P;
  const uint32_t B = a.B;
  const uint32_t n1 = (B + 1) / 2;
  const uint64_t s0 = (uint64_t)p * B;
  uint32_t* node_base = (a.nodes_out && live)
                            ? reinterpret_cast<uint32_t*>(a.nodes_out + (uint64_t)p * a.n_int * 32)
                            : nullptr;
  uint32_t* region = lds + (uint64_t)gi * lds_words;
  uint32_t* counter = region;
  uint32_t* cur = region + 4;
  uint32_t* nxt = region + 4 + (uint64_t)n1 * 8;
  if (!upper && tid == 0) counter[0] = 0;
  __syncthreads();

  // Leaves + level 1: the lower half (a wide tree: every thread).
  uint32_t items = 0;
  if (live && (wide || !upper)) {
    const uint32_t j0 = wide ? x : tid, step = wide ? 2u * half : G;
    for (uint32_t j = j0; j < n1; j += step) {
      uint32_t st[8];
      tree_level1(a, s0, B, j, items, st);
      store_node(cur + (uint64_t)j * 8, st);
      if (node_base) store_node(node_base + (uint64_t)j * 8, st);
    }
  }
  if (items) atomicAdd(counter, items);

  uint32_t n = n1;
  uint64_t level_off = 0;
  const uint32_t stop = a.top_nodes ? a.top_nodes : 1u;
  while (n > stop) {
    __syncthreads();
    const uint32_t m = (n + 1) / 2;
    if (wide && m > half) {  // a wide level: every thread hashes whole nodes
      if (live) {
        for (uint32_t j = x; j < m; j += 2u * half) {
          const uint32_t l = 2 * j, r = (2 * j + 1 < n) ? 2 * j + 1 : 2 * j;
          uint32_t hl[8], hr[8], st[8];
          load_node(cur + (uint64_t)l * 8, hl);
          load_node(cur + (uint64_t)r * 8, hr);
          sha256_node_pair(hl, hr, st);
          store_node(nxt + (uint64_t)j * 8, st);
          if (node_base) store_node(node_base + (level_off + n + j) * 8, st);
        }
      }
    } else {  // split level: no lane skips the three barriers inside the duo functions
      // two lanes per node when they fit (the padding block then runs in the two-lane form)
      const bool pair = 2u * m <= (wide ? half : G);
      const uint32_t slot = pair ? tid >> 1 : tid;
      const bool is_a = pair && (tid & 1u);
      const uint32_t j = slot < m ? slot : 0u;
      const uint32_t l = 2 * j, r = (2 * j + 1 < n) ? 2 * j + 1 : 2 * j;
      uint32_t hl[8], hr[8];
      load_node(cur + (uint64_t)l * 8, hl);
      load_node(cur + (uint64_t)r * 8, hr);
      if (!upper) {
        uint32_t st[8];
        if (pair) {
          sha256_node_duo_main<true>(hl, hr, st, kw + xm, half, is_a);
          if (live && slot < m) {
            store_half_node(nxt + (uint64_t)j * 8, st, is_a);
            if (node_base) store_half_node(node_base + (level_off + n + j) * 8, st, is_a);
          }
        } else {
          sha256_node_duo_main(hl, hr, st, kw + xm, half);
          if (live && slot < m) {
            store_node(nxt + (uint64_t)j * 8, st);
            if (node_base) store_node(node_base + (level_off + n + j) * 8, st);
          }
        }
      } else {
        sha256_node_duo_sched(hl, hr, kw + xm, half);
      }
    }
    level_off += n;
    n = m;
    uint32_t* t = cur; cur = nxt; nxt = t;
  }
  __syncthreads();
  if (live && !upper) {
    if (tid < 8) reinterpret_cast<uint32_t*>(a.root_out + (uint64_t)p * 32)[tid] = cur[tid];
    if (tid == 0 && a.items_out) a.items_out[p] = (int32_t)counter[0];
  }
}

// LDS words of one tree_body group for B buckets (counter slot + the two level buffers).
__host__ __device__ inline uint32_t tree_lds_words(uint32_t B) {
  const uint32_t n1 = (B + 1) / 2;
  return 4u + (n1 + (n1 + 1) / 2) * 8u;
}

// A tree workgroup of a fused build step (plan_step_trees): Q > 0 -> its first wave builds Q
// partitions (tree_body_packed); Q == 0 -> its first kStepTreeWideThreads threads (two waves)
// build one partition (tree_body; the other waves leave at once); Q == kStepTreeWholeWG -> the
// whole workgroup builds one partition (tree_body_duo, half = 128).
__device__ __forceinline__ void step_trees(const TreeLaunch& t, uint32_t Q, uint32_t block, uint32_t* lds) {
  if (Q == kStepTreeWholeWG)  // few wide trees: all 256 threads per partition, the upper 128 as helpers
    tree_body_duo(t, 2u * kStepTreeWideThreads, tree_lds_words(t.B), block, lds, kStepTreeWideThreads,
                  reinterpret_cast<u32x4*>(lds + t.duo_kw_word));
  else if (Q)
    tree_body_packed(t, Q, block, lds);
  else {
    if (t.duo_kw_word)  // the second wave computes the first's message schedules on its <= 64-node levels
      tree_body_duo(t, kStepTreeWideThreads, tree_lds_words(t.B), block, lds, kStepTreeWideThreads / 2,
                    reinterpret_cast<u32x4*>(lds + t.duo_kw_word));
    else
      tree_body<true>(t, kStepTreeWideThreads, tree_lds_words(t.B), block, lds, kStepTreeWideThreads);
  }
}

}  // namespace mde
