// tree.hip -- bucket digests -> leaves -> SHA-256 Merkle tree, one workgroup per partition.
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
#include "mde_device.hpp"
#include "mde_internal.hpp"


namespace mde {
namespace {

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

// Leaf b of partition p: digest, and (when building from byte sums) its size/digest outputs.
__device__ __forceinline__ uint64_t leaf(const TreeLaunch& a, uint64_t s, uint32_t& items, uint32_t& sz_out) {
  uint64_t v;
  if (a.sums_in) {
    v = (uint64_t)(a.sums_in[s] % kHashMod);
    if (a.sums_clear) a.sums_clear[s] = 0ull;
  } else {
    v = a.digest_in[s];
  }
  if (a.digest_out) a.digest_out[s] = v;
  if (a.seg_rec || a.counts_in) {
    uint32_t sz;  // int32 wrap like Go
    if (a.seg_rec) {
      sz = (uint32_t)(a.seg_rec[s + 1] - a.seg_rec[s]);
    } else {
      sz = a.counts_in[s];
      a.counts_in[s] = 0u;
    }
    if (a.size_out) a.size_out[s] = (int32_t)sz;
    items += sz;
    sz_out = sz;
  }
  return v;
}

// A "group" of G threads builds one partition's tree (see launch_tree for the choice of G). Every
// group of a workgroup has the same B, hence the same level count, so the per-level
// __syncthreads() is uniform.
template <bool kLds>
__global__ __launch_bounds__(256) void tree_kernel(TreeLaunch a, uint32_t G, uint32_t lds_words) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t groups = blockDim.x / G;
  const uint32_t gi = threadIdx.x / G, tid = threadIdx.x % G;
  const uint32_t p = blockIdx.x * groups + gi;
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
      const uint64_t dl = leaf(a, s0 + bl, items, szl);
      const uint64_t dr = (br != bl) ? leaf(a, s0 + br, items, szr) : dl;
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
  while (n_max > 1) {
    __syncthreads();
    n_max = (n_max + 1) / 2;
    if (n <= 1) continue;  // this group's tree is complete
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

hipError_t launch_tree(const TreeLaunch& a, hipStream_t st) {
  if (a.P == 0) return hipSuccess;
  // Tree building is latency-bound (11 dependent SHA-256 compressions at B = 64) and several tree
  // waves on one CU slow each other down, so use as few waves as possible: a group of G lanes per
  // partition, G = the level-1 width rounded up to a power of two, 64/G partitions per wave, one
  // wave per workgroup (so workgroups spread over CUs). Wide trees (level 1 > 64) get a whole
  // 256-thread workgroup each.
  const uint32_t n1 = (a.B + 1) / 2;
  uint32_t G = 8, threads = 64;
  if (n1 > 64) {
    G = threads = 256;
  } else {
    while (G < n1) G <<= 1;
  }
  const uint32_t groups = threads / G;
  const uint32_t blocks = (a.P + groups - 1) / groups;
  if (a.B <= kTreeLdsMaxBuckets) {
    // per group: 16-byte counter slot + level 1 + level 2 (ping-pong), 16-byte aligned
    const uint32_t words = 4 + (n1 + (n1 + 1) / 2) * 8;
    hipLaunchKernelGGL(tree_kernel<true>, dim3(blocks), dim3(threads), (size_t)words * 4 * groups,
                       st, a, G, words);
  } else {
    if (!a.nodes_out) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tree_kernel<false>, dim3(blocks), dim3(threads), 16 * groups, st, a, G, 4u);
  }
  return hipGetLastError();
}

}  // namespace mde
