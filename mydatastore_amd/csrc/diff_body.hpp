// diff_body.hpp -- DifferentMerkleTreeBuckets for ONE tree pair, as a workgroup-level device
// function shared by diff_kernel (diff.hip) and the fused verify kernel (verify.hip).
//
// Reference: main/merkle_tree.go:159-216. The recursive DFS compares node hashes, prunes equal
// subtrees, emits a differing leaf's bucketId (error if the two ids differ), and otherwise
// recurses Left then Right. In merkletree v0.2.0 a self-paired node has Left == Right, so a
// differing self-paired node emits its subtree twice (e.g. "...,27,28,29,28,29" at B = 30).
//
// Every node has exactly two child edges, so the DFS visits the 2^D root-to-depth-D paths of the
// tree DAG in order of the path's bit string (left = 0). Path v emits iff every node pair along
// it differs; its leaf is found by descending child(i, bit) = 2i+bit, clamped to 2i where 2i+1
// falls off an odd level. All paths are evaluated in parallel and the emitting ones written with a
// block-wide prefix sum, which reproduces the DFS output order (duplicates included) without
// recursion. Trees of different depth: the first all-differing path reaches a leaf/inner pair,
// which the reference reports as an error (nil child, or leaf content missing).
//
// Leaf-only form (kLeafOnly): when both trees have the same shape (equal leaf count after the odd
// duplicate, hence equal level sizes), every inner node is SHA-256 of the leaf sequence below it,
// so a node pair differs exactly when some leaf pair below differs (up to a SHA-256 collision).
// A path is then all-differing iff its leaf pair differs, and the diff needs the digests only --
// no peer tree has to be built. The emitted ids, their order, duplicates and the bucketId check
// are the same as the node-compare form.
#pragma once
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {

constexpr int kDiffThreads = 256;
constexpr int kDiffMaxLevels = 40;

struct DiffShape {
  uint32_t sizes[kDiffMaxLevels];  // level 0 = leaves incl. dup, L-1 = root
  uint64_t off[kDiffMaxLevels];    // node index of level k's first node (k >= 1) in the nodes array
  uint32_t L;
};

__device__ inline void make_diff_shape(uint32_t B, DiffShape& s) {
  uint32_t n = B + (B & 1u), lv = 0;
  s.sizes[0] = n;
  s.off[0] = 0;
  uint64_t acc = 0;
  while (n > 1) {
    n = (n + 1) / 2;
    lv++;
    s.sizes[lv] = n;
    s.off[lv] = acc;
    acc += n;
  }
  s.L = lv + 1;
}

__device__ __forceinline__ uint64_t diff_internal_nodes(uint32_t B) {
  uint32_t n = B + (B & 1u);
  uint64_t t = 0;
  while (n > 1) { n = (n + 1) / 2; t += n; }
  return t;
}

// Compare node (level la, index ia) of tree A with (lb, ib) of tree B. Leaves are 8-byte LE
// digests, inner nodes 32-byte hashes; different lengths never compare equal (bytes.Equal).
__device__ __forceinline__ bool node_differs(uint32_t la, uint32_t ia, const DiffShape& sa, uint32_t Ba,
                                             const uint64_t* da, const uint8_t* na, uint32_t lb, uint32_t ib,
                                             const DiffShape& sb, uint32_t Bb, const uint64_t* db,
                                             const uint8_t* nb) {
  if ((la == 0) != (lb == 0)) return true;
  if (la == 0) return da[min(ia, Ba - 1)] != db[min(ib, Bb - 1)];
  const u32x4* pa = reinterpret_cast<const u32x4*>(na + (sa.off[la] + ia) * 32);
  const u32x4* pb = reinterpret_cast<const u32x4*>(nb + (sb.off[lb] + ib) * 32);
  const u32x4 x0 = pa[0] ^ pb[0], x1 = pa[1] ^ pb[1];
  return (x0.x | x0.y | x0.z | x0.w | x1.x | x1.y | x1.z | x1.w) != 0u;
}

// Shared state of one diff_body call (LDS).
struct DiffLds {
  DiffShape sa, sb;
  uint32_t wave_tot[kDiffThreads / 64];
  uint32_t err;
};

// Pair pr of `a`, by all kDiffThreads threads of the workgroup (uniform: contains barriers).
template <bool kLeafOnly>
__device__ __forceinline__ void diff_body(const DiffLaunch& a, uint32_t pr, DiffLds& s) {
  // Verify mode: the peer tree's own bucket count; a peer object that gave no tree is reported,
  // not diffed (uniform across the block, so the early return is safe).
  const int32_t bt = a.nb_in ? a.nb_in[pr] : (int32_t)a.Bb;
  if (bt <= 0 || (uint32_t)bt > a.Bb) {
    // capacity: more leaves than fit the local depth -> the DFS would fail (MDE_E_TREE)
    if (threadIdx.x == 0) a.out_count[pr] = bt == -5 ? -4 : -6;
    return;
  }
  const uint32_t Bb = (uint32_t)bt;
  const uint32_t ai = a.a_div ? pr / a.a_div : pr;
  if (threadIdx.x == 0) {
    make_diff_shape(a.Ba, s.sa);
    make_diff_shape(Bb, s.sb);
    s.err = 0;
  }
  __syncthreads();
  const uint64_t* da = a.da + (uint64_t)ai * a.Ba;
  const uint64_t* db = a.db + (uint64_t)pr * a.Bb;
  const uint8_t* na = kLeafOnly ? nullptr : a.na + (uint64_t)ai * diff_internal_nodes(a.Ba) * 32;
  const uint8_t* nb = kLeafOnly ? nullptr : a.nb + (uint64_t)pr * diff_internal_nodes(a.Bb) * 32;
  int32_t* out = a.out_ids + (uint64_t)pr * a.out_stride;

  const uint32_t Da = s.sa.L - 1, Db = s.sb.L - 1;
  const uint32_t Dm = min(Da, Db);
  const uint64_t n_paths = 1ull << Dm;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint64_t base = 0;

  for (uint64_t t0 = 0; t0 < n_paths; t0 += kDiffThreads) {
    const uint64_t v = t0 + threadIdx.x;
    bool emit = false;
    int32_t id = 0;
    if (v < n_paths) {
      uint32_t ia = 0, ib = 0;
      bool alive = true;
      for (uint32_t d = 0; d <= Dm; d++) {
        const uint32_t la = Da - d, lb = Db - d;
        if ((!kLeafOnly || d == Dm) && !node_differs(la, ia, s.sa, a.Ba, da, na, lb, ib, s.sb, Bb, db, nb)) {
          alive = false;
          break;
        }
        if (d == Dm) break;
        const uint32_t bit = (uint32_t)(v >> (Dm - 1 - d)) & 1u;
        const uint32_t ca = 2 * ia + bit, cb = 2 * ib + bit;
        ia = ca < s.sa.sizes[la - 1] ? ca : 2 * ia;
        ib = cb < s.sb.sizes[lb - 1] ? cb : 2 * ib;
      }
      if (alive) {
        if (Da != Db) {
          atomicOr(&s.err, 1u);  // leaf vs inner node: nil child / missing content
        } else {
          const uint32_t ida = min(ia, a.Ba - 1), idb = min(ib, Bb - 1);
          if (ida != idb) atomicOr(&s.err, 1u);  // "bucketIds dont match"
          emit = true;
          id = (int32_t)ida;
        }
      }
    }
    const uint64_t bal = __ballot(emit);
    const uint32_t before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) s.wave_tot[wid] = __popcll(bal);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int w = 0; w < kDiffThreads / 64; w++) {
      off += (w < wid) ? s.wave_tot[w] : 0u;
      tot += s.wave_tot[w];
    }
    if (emit && base + off + before < a.out_stride) out[base + off + before] = id;
    base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int32_t c = (int32_t)base;
    if (s.err) c = -4;                     // MDE_E_TREE
    else if (base > a.out_stride) c = -5;  // MDE_E_CAPACITY
    a.out_count[pr] = c;
  }
}

}  // namespace mde
