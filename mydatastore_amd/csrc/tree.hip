// tree.hip -- bucket digests -> leaves -> SHA-256 Merkle tree (standalone launch).
//
// The per-workgroup tree builder (reference semantics, node layout) is tree_body() in
// tree_body.hpp, shared with the fused build-step kernel in digest.hip.
#include <stdlib.h>

#include "tree_body.hpp"


namespace mde {
namespace {

template <bool kLds>
__global__ __launch_bounds__(256) void tree_kernel(TreeLaunch a, uint32_t G, uint32_t lds_words) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  tree_body<kLds>(a, G, lds_words, blockIdx.x, lds, blockDim.x);
}

// Latency form (tree_body_duo): the upper half of the workgroup computes the lower half's message
// schedules. `half` = 128 for wide trees (G = 256), else 64 (one wave of groups + its mirror).
__global__ __launch_bounds__(256) void tree_duo_kernel(TreeLaunch a, uint32_t G, uint32_t lds_words, uint32_t half,
                                                       uint32_t kw_word) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  tree_body_duo(a, G, lds_words, blockIdx.x, lds, half, reinterpret_cast<u32x4*>(lds + kw_word));
}

// Two wide trees per workgroup (tree_body_pair): used for many partitions, where the trees are
// bound by wave-instructions rather than by their critical path.
__global__ __launch_bounds__(256) void tree_pair_kernel(TreeLaunch a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  tree_body_pair(a, blockIdx.x, lds);
}

// Digest-only build (root_out == NULL): digest, size and items of each partition, no tree; one
// wave per partition.
__global__ __launch_bounds__(256) void leaves_kernel(TreeLaunch a) {
  const uint32_t p = blockIdx.x * 4u + threadIdx.x / 64u;
  leaves_waves(a, p, 1u << 30, p + 1);
}

}  // namespace

uint32_t tree_levels(uint32_t B, uint32_t* sizes) {
  uint32_t n = B + (B & 1u), lv = 0;
  if (sizes) sizes[0] = n;
  while (n > 1) {
    n = (n + 1) / 2;
    lv++;
    if (sizes) sizes[lv] = n;
  }
  return lv + 1;
}

uint64_t tree_internal(uint32_t B) {
  uint32_t sz[64];
  const uint32_t L = tree_levels(B, sz);
  uint64_t t = 0;
  for (uint32_t k = 1; k < L; k++) t += sz[k];
  return t;
}

bool tree_geometry(uint32_t B, TreeGeometry* g) {
  // Tree building is latency-bound (11 dependent SHA-256 compressions at B = 64) and several tree
  // waves on one CU slow each other down, so use as few waves as possible: a group of G lanes per
  // partition, G = the level-1 width rounded up to a power of two, 64/G partitions per wave, one
  // wave per workgroup (so workgroups spread over CUs). Wide trees (level 1 > 64) get a whole
  // 256-thread workgroup each.
  const uint32_t n1 = (B + 1) / 2;
  uint32_t G = 8, threads = 64;
  if (n1 > 64) {
    G = threads = 256;
  } else {
    while (G < n1) G <<= 1;
  }
  g->G = G;
  g->threads = threads;
  g->groups = threads / G;
  g->lds = B <= kTreeLdsMaxBuckets;
  // per group: 16-byte counter slot + level 1 + level 2 (ping-pong), 16-byte aligned
  g->words = g->lds ? 4 + (n1 + (n1 + 1) / 2) * 8 : 4u;
  g->lds_bytes = g->words * 4 * g->groups;
  return g->lds;
}

bool tree_duo_enabled() {
  static const bool on = [] {
    const char* e = getenv("MDE_TREE_DUO");
    return !(e && e[0] == '0');
  }();
  return on;
}

hipError_t launch_tree(const TreeLaunch& a, hipStream_t st) {
  if (a.P == 0) return hipSuccess;
  if (!a.root_out) {  // digest-only build
    hipLaunchKernelGGL(leaves_kernel, dim3((a.P + 3) / 4), dim3(256), 0, st, a);
    return hipGetLastError();
  }
  // Wide trees of many partitions: two per workgroup. 1,024 partitions at B = 1,000: 142 -> 119.5 us
  // (-16 %); at 128 partitions the 4-wave tree_body's shorter critical path wins, 61.5 vs 73 us
  // (profiles/r02an_pair_trees.jsonl, `tree_us`).
  if ((a.B + 1) / 2 > 64 && !a.n_in && a.P >= kTreePairMinPartitions && pair_tree_lds_words(a.B) * 4u <= kTreePairLdsMax) {
    hipLaunchKernelGGL(tree_pair_kernel, dim3((a.P + 1) / 2), dim3(256), pair_tree_lds_words(a.B) * 4u, st, a);
    return hipGetLastError();
  }
  TreeGeometry g;
  const bool lds = tree_geometry(a.B, &g);
  const uint32_t blocks = (a.P + g.groups - 1) / g.groups;
  // Split-schedule form: the same partitions per workgroup (a wide tree: one; else one wave of
  // groups) with a mirror half of schedule helpers, for launches of few workgroups.
  if (lds && !a.n_in && tree_duo_enabled() && ((g.G == g.threads && g.threads == 256) || blocks <= kDuoMaxBlocks)) {
    const uint32_t half = g.threads == 256 ? 128u : 64u;
    const uint32_t kw_word = (g.groups * g.words + 3u) & ~3u;
    hipLaunchKernelGGL(tree_duo_kernel, dim3(blocks), dim3(2 * half), kw_word * 4u + duo_kw_bytes(half), st, a, g.G,
                       g.words, half, kw_word);
    return hipGetLastError();
  }
  if (lds) {
    hipLaunchKernelGGL(tree_kernel<true>, dim3(blocks), dim3(g.threads), g.lds_bytes, st, a, g.G, g.words);
  } else {
    if (!a.nodes_out) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tree_kernel<false>, dim3(blocks), dim3(g.threads), g.lds_bytes, st, a, g.G, g.words);
  }
  return hipGetLastError();
}

}  // namespace mde
