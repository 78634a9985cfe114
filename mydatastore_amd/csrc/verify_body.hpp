// verify_body.hpp -- the decision step of Manager.VerifyEpoch (main/manager.go:1072-1118) for one
// partition, as workgroup-level device functions: the fold (verify_body) and the whole fused
// step (verify_fused_body: decode the peer objects, rebuild other-shape peer trees, diff, fold,
// encode). Used by verify.hip's kernels and by the resident build service (digest.hip
// server_kernel). See verify.hip for the reference semantics.
#pragma once
#include "diff_body.hpp"
#include "tree_body.hpp"
#include "wire_body.hpp"

namespace mde {

constexpr int kVerifyThreads = 256;  // one workgroup per partition
constexpr uint32_t kVerifyWords = kVerifyMaxBuckets / 32;
constexpr uint32_t kVerifyFusedWords = kVerifyFusedMaxCap / 32;
constexpr uint32_t kVerifyStageMaxBytes = 24u * 1024u;  // per wave: a whole object up to B = 1024 (20.5 KB)

// Partition p's fold by all 256 threads (uniform: contains barriers). bits: >= ceil(B/32) words.
__device__ __forceinline__ void verify_body(const VerifyLaunch& a, uint32_t p, uint32_t* bits, uint32_t* wave_tot) {
  const uint32_t t = threadIdx.x;
  const uint32_t W = (a.B + 31) / 32;
  for (uint32_t w = t; w < W; w += kVerifyThreads) bits[w] = 0;
  __syncthreads();
  int32_t valid_count = 0;
  bool valid_diff = false;
  for (uint32_t r = 0; r < a.R; r++) {
    const uint64_t i = (uint64_t)p * a.R + r;
    const int32_t n = a.peer_status[i];
    if (n < 0) continue;  // EpochTreeObjectToMerkleTree / DifferentMerkleTreeBuckets error
    if (n == 0) {
      valid_count++;
    } else if (a.peer_valid[i]) {
      valid_diff = true;
    }
    const int32_t* ids = a.peer_ids + i * a.ids_stride;
    for (uint32_t j = t; j < (uint32_t)n; j += kVerifyThreads) {
      const uint32_t id = (uint32_t)ids[j];
      if (id < a.B) atomicOr(&bits[id >> 5], 1u << (id & 31));
    }
  }
  __syncthreads();
  // Ascending compaction: thread t owns words [t*per, (t+1)*per).
  const uint32_t per = (W + kVerifyThreads - 1) / kVerifyThreads;
  const uint32_t w0 = min(t * per, W), w1 = min(w0 + per, W);
  uint32_t mine = 0;
  for (uint32_t w = w0; w < w1; w++) mine += __popc(bits[w]);
  const int lane = t & 63, wid = t >> 6;
  uint32_t incl = mine;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(incl, o);
    if (lane >= o) incl += x;
  }
  if (lane == 63) wave_tot[wid] = incl;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < kVerifyThreads / 64; w++) {
    base += w < wid ? wave_tot[w] : 0u;
    total += wave_tot[w];
  }
  uint32_t pos = base + incl - mine;
  int32_t* out = a.diff_ids + (uint64_t)p * a.B;
  for (uint32_t w = w0; w < w1; w++) {
    uint32_t m = bits[w];
    while (m) {
      const uint32_t b = __ffs(m) - 1;
      m &= m - 1;
      out[pos++] = (int32_t)(w * 32 + b);
    }
  }
  if (t == 0) {
    const uint8_t v = (valid_count >= (int32_t)a.replica_count || valid_diff) ? 1 : 0;
    a.diff_count[p] = (int32_t)total;
    a.valid_count[p] = valid_count;
    a.valid[p] = v;
    if (a.valid_out) a.valid_out[p] = v;
  }
  if (a.status_out)
    for (uint32_t r = t; r < a.R; r += kVerifyThreads) a.status_out[(uint64_t)p * a.R + r] = a.peer_status[(uint64_t)p * a.R + r];
}


// The fused step's static LDS (the dynamic part, `dyn`, holds the object stages, then tree levels).
struct VerifyShared {
  uint32_t bits[kVerifyFusedMaxCap / 32];
  uint32_t wave_tot[4];
  DiffLds ds;
  int32_t tree_n[kVerifyFusedMaxPeers];
  uint32_t need_tree;
  uint32_t enc_red[16];
  uint32_t gstack[4][kWireGroupDepth];
};

// Partition p's whole decision step by all 256 threads of the workgroup (uniform: every barrier
// is reached by every thread, so a resident workgroup can run it once per request; server.cpp).
template <bool kDeep>
__device__ __forceinline__ void verify_fused_body(const VerifyFusedLaunch& f, uint32_t p, uint32_t G, uint32_t words,
                                                  uint32_t stage_bytes, uint32_t* dyn, VerifyShared& sh) {
  uint32_t* bits = sh.bits;
  uint32_t* wave_tot = sh.wave_tot;
  DiffLds& ds = sh.ds;
  int32_t* tree_n = sh.tree_n;
  uint32_t& need_tree = sh.need_tree;
  uint32_t* enc_red = sh.enc_red;
  auto& gstack = sh.gstack;
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t R = f.fold.R, B = f.fold.B, cap = f.dec.cap;
  const uint64_t i0 = (uint64_t)p * R;

  // 1. EpochTreeObjectToMerkleTree, decode half: wave w takes peers w, w + 4, ...
  uint8_t* stage = reinterpret_cast<uint8_t*>(dyn) + (uint64_t)wid * stage_bytes;
  for (uint32_t r0 = 0; r0 < R; r0 += kVerifyThreads / 64) {
    const uint32_t r = r0 + wid;
    const uint8_t* obj = nullptr;
    const uint8_t* staged = nullptr;
    uint64_t n = 0;
    if (r < R) {
      const uint64_t o0 = f.dec.off[i0 + r];
      n = f.dec.off[i0 + r + 1] - o0;
      obj = f.dec.bytes + o0;
      // kDeep: 16 loads per lane in flight (a 11 KB object in 3 rounds instead of 6)
      if (n + 4 <= stage_bytes) staged = stage_object<kDeep ? 16 : 8>(obj, n, stage, lane);
    }
    __syncthreads();
    if (r < R) {
      // two call sites, so the staged one reads LDS (ds_read) rather than through flat loads
      // kDeep (B > 64): 256 canonical bucket entries per step instead of 64
      if (staged)
        decode_object<kDeep ? 4 : 1>(f.dec, (uint32_t)(i0 + r), staged, n, lane, gstack[wid]);
      else
        decode_object<kDeep ? 4 : 1>(f.dec, (uint32_t)(i0 + r), obj, n, lane, gstack[wid]);
    }
    __syncthreads();
  }

  // 2. Rebuild only the peer trees whose shape (leaf count incl. the odd duplicate) differs from
  // the local tree's; same-shape peers are diffed on their leaves.
  const uint32_t leaves = B + (B & 1u);
  if (threadIdx.x == 0) need_tree = 0;
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < R; r += kVerifyThreads) {
    const int32_t nb = f.dec.n_buckets[i0 + r];
    const bool other = nb > 0 && (uint32_t)nb + ((uint32_t)nb & 1u) != leaves;
    tree_n[r] = other ? nb : 0;
    if (other) need_tree = 1;
  }
  __syncthreads();
  if (need_tree && f.local.P) {  // the local tree, only now that an other-shape peer needs its nodes
    TreeLaunch t = f.local;
    t.P = 1;
    t.digest_in += (uint64_t)p * B;
    t.nodes_out += (uint64_t)p * t.n_int * 32;
    t.root_out += (uint64_t)p * 32;
    tree_body<true>(t, G, words, 0, dyn, kVerifyThreads);  // G, words: the geometry of cap >= B
    __threadfence();
    __syncthreads();
  }
  if (need_tree) {
    TreeLaunch t = f.tree;
    t.P = R;
    t.digest_in += i0 * cap;
    t.nodes_out += i0 * t.n_int * 32;
    t.root_out += i0 * 32;
    t.n_in = tree_n;
    const uint32_t groups = kVerifyThreads / G;
    for (uint32_t blk = 0; blk * groups < R; blk++) tree_body<true>(t, G, words, blk, dyn, kVerifyThreads);
  }

  // 3. DifferentMerkleTreeBuckets(myTree, otherTree) per peer.
  // 3a. Same-shape peers: one wave per peer, lane v of step k walks path 64k + v, and the wave's
  // ballots give the DFS output order directly (diff_body's leaf-only rule, without its
  // block-wide prefix sums and barriers). kDeep (B > 64): 512 paths per register batch, every
  // digest load of a batch issued before its first id store (on gfx9 one vmcnt counter covers
  // loads and stores, so a load behind stores waits for them). The B <= 64 instantiation keeps the
  // one-step form, and with it the register count and occupancy of the common case.
  if (threadIdx.x == 0) make_diff_shape(B, ds.sa);
  __syncthreads();
  const uint32_t D = ds.sa.L - 1;
  const bool wave_diff = kDeep ? D <= 10 : D <= 6;
  if (wave_diff) {
    constexpr uint32_t kPathBatch = kDeep ? 8 : 1;
    const uint32_t n_paths = 1u << D;
    uint32_t lvl[10];  // lvl[d]: size of the level a path's step d descends into (from LDS once)
#pragma unroll
    for (uint32_t d = 0; d < 10; d++) lvl[d] = d < D ? ds.sa.sizes[D - 1 - d] : 0u;
    for (uint32_t r = wid; r < R; r += kVerifyThreads / 64) {
      if (tree_n[r] != 0) continue;
      const uint64_t i = i0 + r;
      const int32_t bt = f.dec.n_buckets[i];
      if (bt <= 0 || (uint32_t)bt > cap) {
        if (lane == 0) f.diff.out_count[i] = bt == -5 ? -4 : -6;
        continue;
      }
      const uint64_t* da = f.diff.da + (uint64_t)p * B;
      const uint64_t* db = f.diff.db + i * cap;
      int32_t* out = f.diff.out_ids + i * f.diff.out_stride;
      uint32_t base = 0;
      bool bad = false;
      for (uint32_t c0 = 0; c0 < n_paths; c0 += 64 * kPathBatch) {
        uint32_t leaf[kPathBatch];
        uint64_t xa[kPathBatch], xb[kPathBatch];
        // wave-uniform exits: the last batch of a tree runs only the steps it has
#pragma unroll
        for (uint32_t k = 0; k < kPathBatch; k++) {
          if (c0 + k * 64 >= n_paths) break;
          const uint32_t v = c0 + k * 64 + lane;
          uint32_t ia = 0;
#pragma unroll
          for (uint32_t d = 0; d < 10; d++) {
            if (d >= D) break;
            const uint32_t ca = 2 * ia + ((v >> (D - 1 - d)) & 1u);
            ia = ca < lvl[d] ? ca : 2 * ia;
          }
          leaf[k] = ia;
          const bool in = v < n_paths;
          xa[k] = in ? da[min(ia, B - 1)] : 0ull;
          xb[k] = in ? db[min(ia, (uint32_t)bt - 1)] : 0ull;
        }
#pragma unroll
        for (uint32_t k = 0; k < kPathBatch; k++) {
          if (c0 + k * 64 >= n_paths) break;
          const uint32_t v = c0 + k * 64 + lane;
          const uint32_t ida = min(leaf[k], B - 1), idb = min(leaf[k], (uint32_t)bt - 1);
          const bool emit = v < n_paths && xa[k] != xb[k];
          const uint64_t bal = __ballot(emit);
          bad |= __ballot(emit && ida != idb) != 0;  // "bucketIds dont match"
          const uint32_t at = base + __popcll(bal & ((1ull << lane) - 1ull));
          if (emit && at < f.diff.out_stride) out[at] = (int32_t)ida;
          base += __popcll(bal);
        }
      }
      if (lane == 0) f.diff.out_count[i] = bad ? -4 : base > f.diff.out_stride ? -5 : (int32_t)base;
    }
  }
  __syncthreads();
  // 3b. The rest: other-shape peers (node hashes), and same-shape peers of deeper trees.
  for (uint32_t r = 0; r < R; r++) {
    if (tree_n[r] == 0) {
      if (!wave_diff) diff_body<true>(f.diff, (uint32_t)(i0 + r), ds);
    } else {
      diff_body<false>(f.diff, (uint32_t)(i0 + r), ds);
    }
  }
  __syncthreads();

  // 4. validCount / validDiff / diffSet.
  verify_body(f.fold, p, bits, wave_tot);

  // 5. The object VerifyEpoch persists.
  if (f.enc.n) {
    __syncthreads();
    if (kDeep) {
      encode_object_block(f.enc, p, threadIdx.x, kVerifyThreads, enc_red);  // B > 64: all four waves
    } else if (wid == 0) {
      encode_object(f.enc, p, lane);
    }
  }
}

}  // namespace mde
