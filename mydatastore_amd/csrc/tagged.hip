// tagged.hip -- bucket digests for layout B: records grouped by partition, in arrival order,
// each carrying its bucket tag.
//
// Reference: the bucket of a record is fixed at write time (Manager.getKeyBucket,
// main/manager.go:773-778) and the build folds CustomHash.Add over each bucket's records
// (main/merkle_tree.go:90-113). Layout A needs the records sorted by bucket; layout B bins them
// into the B leaf buckets inside the kernel, so the unit of work is a record, not a bucket:
//   * equal contiguous byte ranges per wave (one per resident wave), 16-byte nontemporal loads,
//     the next step's loads issued before the current step is reduced (register double buffer);
//   * each lane byte-sums (v_sad_u8) the part of its 16 bytes that belongs to each record it
//     touches (one record unless a boundary falls inside the vector) -- the record index comes
//     from a float reciprocal of the wave-relative offset, corrected to exact;
//   * no cross-lane reduction per record: every lane owns a private slot in the wave's LDS bins
//     (sum bins laid out [bucket][lane slot], u32) and adds its partial sum to
//     bins[tag(record)][slot] with one conflict-free ds_add; the lane holding a record's first
//     byte adds 1 to that bucket's record count;
//   * when the wave leaves a partition it folds the lane slots of each bucket (rotated so the 64
//     lanes hit 64 banks), adds them to the global u64 sums / u32 counts and clears the bins.
// Slots per bucket: 64 up to B = 64, halving as B doubles (<= 32 KiB of bins per wave); lanes
// sharing a slot serialize on the LDS atomic. B > 4096 adds straight to global memory.
// Exactness: a wave covers <= 8 MiB, so any u32 slot holds <= 255 * 8 MiB < 2^32.
// Fixed-length values only (0 < value_stride <= 2^30).
#include "mde_device.hpp"
#include "mde_internal.hpp"
#include "tree_body.hpp"

#include <algorithm>

namespace mde {
namespace {

constexpr int kThreads = 128;  // 2 waves: 4 workgroups per CU fit their LDS bins
constexpr int kU = 8;                       // 16-byte loads per lane per step
constexpr uint64_t kStep = 1024ull * kU;    // 8 KiB per wave step

__device__ __forceinline__ uint32_t byte_mask(int lo, int hi) {
  const uint32_t mh = hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
  const uint32_t ml = lo >= 4 ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
  return hi > lo ? (mh & ~ml) : 0u;
}

// Byte sum of bytes [a, b) of the 16-byte vector v (0 <= a <= b <= 16).
__device__ __forceinline__ uint32_t masked_sum16(u32x4 v, int a, int b) {
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int lo = min(max(a - 4 * k, 0), 4), hi = min(max(b - 4 * k, 0), 4);
    acc = __builtin_amdgcn_sad_u8(v[k] & byte_mask(lo, hi), 0u, acc);
  }
  return acc;
}

__device__ __forceinline__ uint32_t full_sum16(u32x4 v) {
  uint32_t acc = __builtin_amdgcn_sad_u8(v[0], 0u, 0u);
  acc = __builtin_amdgcn_sad_u8(v[1], 0u, acc);
  acc = __builtin_amdgcn_sad_u8(v[2], 0u, acc);
  return __builtin_amdgcn_sad_u8(v[3], 0u, acc);
}

// Partition of record r (linear walk from q; only taken for records past the wave's partition).
__device__ __forceinline__ uint32_t part_of(const TaggedLaunch& a, uint64_t r, uint32_t q) {
  while (q + 1 < a.P && a.part_rec[q + 1] <= r) q++;
  return q;
}

struct WaveBins {
  uint32_t* sum;  // [B][lrep] (nullptr: global only)
  uint32_t* cnt;  // [B]
};

__device__ void flush_bins(const TaggedLaunch& a, const WaveBins& w, uint32_t q, int lane) {
  if (!w.sum) return;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t L = a.lrep;
  for (uint32_t b = lane; b < a.B; b += 64) {
    uint32_t* row = w.sum + (uint64_t)b * L;
    unsigned long long s = 0;
    for (uint32_t j = 0; j < L; j++) {
      const uint32_t k = (j + (uint32_t)lane) & (L - 1);  // rotate: lanes hit different banks
      s += row[k];
      row[k] = 0;
    }
    const uint32_t c = w.cnt[b];
    w.cnt[b] = 0;
    if (s) atomicAdd(a.sums + (uint64_t)q * a.B + b, s);
    if (c) atomicAdd(a.counts + (uint64_t)q * a.B + b, c);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ void load_step(u32x4 (&v)[kU], const u32x4* lane_base, uint64_t p,
                                          uint64_t end, int lane) {
#pragma unroll
  for (int u = 0; u < kU; u++) {
    const uint64_t x = p + (uint64_t)u * 1024u + (uint64_t)lane * 16u;
    v[u] = x < end ? __builtin_nontemporal_load(lane_base + (p >> 4) + u * 64) : u32x4{0u, 0u, 0u, 0u};
  }
}

// `block` = this workgroup's index among the digest workgroups of the launch.
__device__ __forceinline__ void tagged_body(const TaggedLaunch& a, uint32_t block, uint32_t* smem) {
  // As in the layout-A digest: co-running SHA-256 tree waves (fused step, or a tree kernel on a
  // second stream) take the issue slots the binning waves leave, not the other way round.
  __builtin_amdgcn_s_setprio(2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t L = a.lrep;
  WaveBins w{nullptr, nullptr};
  if (a.use_lds) {
    const uint64_t words = (uint64_t)a.B * L + a.B;
    w.sum = smem + (uint64_t)wid * words;
    w.cnt = w.sum + (uint64_t)a.B * L;
    for (uint64_t j = lane; j < words; j += 64) w.sum[j] = 0;
  }
  const uint32_t wave = block * (kThreads / 64) + wid;
  if (wave >= a.n_waves) return;
  const uint64_t V = a.stride;
  const uint64_t r_lo = a.part_rec[0], r_hi = a.part_rec[a.P];
  const uint64_t valid_lo = a.shift + r_lo * V, last = a.shift + r_hi * V;
  const uint64_t first = valid_lo & ~15ull;
  const uint64_t beg = first + (uint64_t)wave * a.wave_bytes;
  if (beg >= last) return;
  const uint64_t end = min(beg + a.wave_bytes, last);
  const uint64_t start = max(beg, valid_lo);
  // The wave's first record (exact, double reciprocal), then wave-relative offsets (< 2^24 + V)
  // divide in float with a one-step correction.
  uint64_t r0;
  {
    const uint64_t rel = start - a.shift;
    r0 = (uint64_t)((double)rel * a.inv_stride);
    while (r0 * V > rel) r0--;
    while ((r0 + 1) * V <= rel) r0++;
  }
  const uint64_t pos0 = a.shift + r0 * V;
  auto rec_at = [&](uint64_t pos) -> uint64_t {
    const uint32_t rel = (uint32_t)(pos - pos0);
    uint32_t q = (uint32_t)((float)rel * a.inv_stride_f);
    while ((uint64_t)q * V > rel) q--;
    while ((uint64_t)(q + 1) * V <= rel) q++;
    return r0 + q;
  };
  // partition of the wave's first record (64-ary search over part_rec)
  uint32_t q = 0;
  {
    uint32_t lo = 0, hi = a.P;
    while (hi - lo > 1) {
      const uint32_t n = hi - lo, step = (n + 63u) / 64u;
      const uint32_t idx = lo + (uint32_t)lane * step;
      const int c = __popcll(__ballot(idx < hi && a.part_rec[idx] <= r0));
      if (c == 0) break;
      lo = lo + (uint32_t)(c - 1) * step;
      hi = min(lo + step, hi);
    }
    q = lo;
    while (q + 1 < a.P && a.part_rec[q + 1] <= r0) q++;  // skip empty partitions
  }
  uint64_t q_end = a.part_rec[q + 1];  // first record past partition q
  const u32x4* lane_base = reinterpret_cast<const u32x4*>(a.base) + lane;
  const uint32_t slot = (uint32_t)lane & (L - 1);

  // Tags travel with the data: the loads of a step also fetch the tags of its first 64 records
  // (one coalesced u16 per lane), read back with a lane shuffle. A tag load issued next to the
  // record's own use would make the wait for it (vmcnt counts in order) also wait for the
  // prefetched next step.
  const bool straddles = ((V | a.shift) & 15u) != 0;  // record boundaries inside a 16-byte vector
  const uint32_t vsh = V >= kStep / 64 && (V & (V - 1)) == 0 ? (uint32_t)__builtin_ctzll(V) : 0u;
  const uint32_t vmask = (uint32_t)V - 1u;
  const bool fast_ok = vsh != 0 && !straddles && w.sum != nullptr && start == beg;
  // one record per 1 KiB row (records of 2^k >= 1 KiB starting on the wave's row grid), shared slots
  const bool rows_ok = fast_ok && vsh >= 10 && L < 64 && ((beg - pos0) & 1023u) == 0;
  // Small records (8 or 16 bytes: production values are 8-byte timestamps,
  // main/manager.go:816), each vector holding 16 / V whole records: every lane bins its own
  // records, whose tags it prefetches with the step (16 / V u16 loads per vector).
  const uint32_t ssh = (V == 8 || V == 16) ? (uint32_t)__builtin_ctzll(V) : 0u;
  const bool small = ssh != 0 && (a.shift & (V - 1)) == 0 && w.sum != nullptr && start == beg;
  const uint64_t r_last = r_hi - 1;
  auto load_tags = [&](uint64_t p, uint64_t& r_first) -> uint32_t {
    r_first = rec_at(max(p, start));
    return a.tag[min(r_first + (uint64_t)lane, r_last)];
  };
  constexpr int kR = 2;  // tags per vector kept per lane (16 / V <= 2)
  auto load_small_tags = [&](uint64_t p, uint32_t (&t)[kU][kR]) {
    const uint32_t per = 16u >> ssh;
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint64_t rv = r0 + (((p - pos0) + (uint64_t)u * 1024u + (uint64_t)lane * 16u) >> ssh);
#pragma unroll
      for (int j = 0; j < kR; j++)
        t[u][j] = (uint32_t)j < per ? (uint32_t)a.tag[min(rv + (uint64_t)j, r_last)] : 0u;
    }
  };
  u32x4 cur[kU], nxt[kU];
  uint32_t ctag[kU][kR], ntag[kU][kR];
  uint64_t cur_r0 = 0, nxt_r0 = 0;
  uint32_t cur_tags = 0, nxt_tags = 0;
  if (small)
    load_small_tags(beg, ctag);
  else
    cur_tags = load_tags(beg, cur_r0);
  load_step(cur, lane_base, beg, end, lane);
  for (uint64_t p = beg; p < end; p += kStep) {
    const uint64_t pn = p + kStep;
    if (pn < end) {
      if (small)
        load_small_tags(pn, ntag);
      else
        nxt_tags = load_tags(pn, nxt_r0);
      load_step(nxt, lane_base, pn, end, lane);
    }
    // Small-record step: the whole step inside [start, end) and inside partition q; per vector
    // 16 / V byte sums of V bytes (v_sad_u8 per dword), each binned with its own tag.
    if (small && pn <= end && r0 + ((pn - 1 - pos0) >> ssh) < q_end) {
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t d0 = __builtin_amdgcn_sad_u8(cur[u].x, 0u, 0u), d1 = __builtin_amdgcn_sad_u8(cur[u].y, 0u, 0u);
        const uint32_t d2 = __builtin_amdgcn_sad_u8(cur[u].z, 0u, 0u), d3 = __builtin_amdgcn_sad_u8(cur[u].w, 0u, 0u);
        uint32_t sj[kR];
        if (ssh == 4) {
          sj[0] = d0 + d1 + d2 + d3;
          sj[1] = 0u;
        } else {
          sj[0] = d0 + d1;
          sj[1] = d2 + d3;
        }
#pragma unroll
        for (int j = 0; j < kR; j++) {
          if ((uint32_t)j >= (16u >> ssh)) break;
          const uint32_t b = min(ctag[u][j], a.B - 1);
          atomicAdd(w.sum + b * L + slot, sj[j]);
          atomicAdd(w.cnt + b, 1u);
        }
      }
    } else if (rows_ok && pn <= end && r0 + ((pn - 1 - pos0) >> vsh) < q_end) {
      // Records of >= 1 KiB with fewer than 64 bin slots per bucket (B > 64; 4 at the reference's
      // default B = 1,000): one 1 KiB row of the step lies in ONE record, so the 64 lanes' ds_adds
      // of a row all hit that bucket's L slots -- 64/L-way on one address (SQ_LDS_BANK_CONFLICT
      // 142.6 M vs 0.05 M at B = 64, profiles/r03f_sq_counters.json). Instead the 8 rows are
      // reduced together: exchanges across lane bits 5, 4 and 3 leave lane l holding 1/8 of row
      // l >> 3 (8 partials per row, one per lane bit 0-2 class); DPP folds those to L partials;
      // then ONE ds_add puts every row's partials in its bucket's distinct slots, and one adds
      // the record counts.
      uint32_t f[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) f[u] = full_sum16(cur[u]);
      const bool b5 = (lane & 32) != 0, b4 = (lane & 16) != 0, b3 = (lane & 8) != 0;
      uint32_t g[4], h[2];
#pragma unroll
      for (int j = 0; j < 4; j++) {  // bit 5: keep rows 4*b5 + j, give the partner the other half
        const uint32_t send = b5 ? f[j] : f[j + 4], keep = b5 ? f[j + 4] : f[j];
        g[j] = keep + (uint32_t)__shfl_xor((int)send, 32);
      }
#pragma unroll
      for (int j = 0; j < 2; j++) {  // bit 4
        const uint32_t send = b4 ? g[j] : g[j + 2], keep = b4 ? g[j + 2] : g[j];
        h[j] = keep + (uint32_t)__shfl_xor((int)send, 16);
      }
      const uint32_t send = b3 ? h[0] : h[1];  // bit 3: within a 16-lane row, row_ror:8 = lane ^ 8
      uint32_t x = (b3 ? h[1] : h[0]) + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, 0x128, 0xf, 0xf, true);
      if (L < 8) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xf, 0xf, true);  // j ~ 7 - j
      if (L < 4) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4e, 0xf, 0xf, true);   // j ~ j ^ 2
      if (L < 2) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xb1, 0xf, 0xf, true);   // j ~ j ^ 1
      const uint32_t r = (uint32_t)lane >> 3, j = (uint32_t)lane & 7u;
      const uint32_t xr = (uint32_t)(p - pos0) + r * 1024u;
      const uint32_t k = (xr >> vsh) - (uint32_t)(cur_r0 - r0);  // < 64
      const uint32_t b = min((uint32_t)__shfl((int)cur_tags, (int)k), a.B - 1);
      if (j < L) atomicAdd(w.sum + b * L + j, x);
      if (j == 0 && (xr & vmask) == 0) atomicAdd(w.cnt + b, 1u);
    } else if (fast_ok && pn <= end && r0 + ((pn - 1 - pos0) >> vsh) < q_end) {
      // Fast step (wave-uniform): power-of-two records of >= kStep/64 B on 16-byte boundaries, the
      // whole step inside [start, end) and inside partition q. Every vector then lies in one
      // record, the record index is a shift, and a step holds <= 64 records (tags by shuffle):
      // per vector 4 v_sad_u8 + one ds_add, in 32-bit arithmetic.
      const uint32_t xr0 = (uint32_t)(p - pos0) + (uint32_t)lane * 16u;
      const uint32_t k0 = (uint32_t)(cur_r0 - r0);
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t xr = xr0 + (uint32_t)u * 1024u;
        const uint32_t k = (xr >> vsh) - k0;  // < 64
        const uint32_t b = min((uint32_t)__shfl((int)cur_tags, (int)k), a.B - 1);
        atomicAdd(w.sum + b * L + slot, full_sum16(cur[u]));
        if ((xr & vmask) == 0) atomicAdd(w.cnt + b, 1u);
      }
    } else {
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint64_t x = p + (uint64_t)u * 1024u + (uint64_t)lane * 16u;
      const uint64_t lo = max(x, start), hi = min(x + 16, end);
      const bool act = lo < hi;
      uint64_t r = rec_at(act ? lo : start);
      const uint32_t k = (uint32_t)min<uint64_t>(r - cur_r0, 64);  // r >= cur_r0 for active lanes
      // shuffles stay outside divergent code (bpermute reads inactive lanes as 0)
      const uint32_t t0 = (uint32_t)__shfl((int)cur_tags, (int)min(k, 63u));
      const uint32_t t1 = straddles ? (uint32_t)__shfl((int)cur_tags, (int)min(k + 1, 63u)) : 0u;
      if (!act) continue;
      uint64_t rs = a.shift + r * V;
      for (uint32_t j = 0;; j++, r++) {  // one record unless a boundary falls inside
        const uint64_t c0 = j ? rs : lo;
        if (c0 >= hi) break;
        const uint64_t re = rs + V, c1 = min(hi, re);
        const uint32_t s = (c0 == x && c1 == x + 16) ? full_sum16(cur[u])
                                                      : masked_sum16(cur[u], (int)(c0 - x), (int)(c1 - x));
        const uint32_t cnt = rs >= lo ? 1u : 0u;  // this lane holds the record's first byte
        // (small-record mode prefetches per-lane tags, not the step's first 64: load directly)
        const uint32_t tg = (!small && j == 0 && k < 64) ? t0 : (!small && j == 1 && k + 1 < 64) ? t1 : (uint32_t)a.tag[r];
        const uint32_t b = min(tg, a.B - 1);  // bad tags never fault (the host API rejects them)
        if (w.sum && r < q_end) {
          if (s) atomicAdd(w.sum + (uint64_t)b * L + slot, s);
          if (cnt) atomicAdd(w.cnt + b, 1u);
        } else {
          const uint64_t idx = (uint64_t)part_of(a, r, q) * a.B + b;
          if (s) atomicAdd(a.sums + idx, (unsigned long long)s);
          if (cnt) atomicAdd(a.counts + idx, 1u);
        }
        rs = re;
      }
    }
    }
    // leave partitions the next step no longer touches
    while (q + 1 < a.P && pn < end && a.shift + q_end * V <= pn) {
      flush_bins(a, w, q, lane);
      q++;
      q_end = a.part_rec[q + 1];
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      cur[u] = nxt[u];
#pragma unroll
      for (int j = 0; j < kR; j++) ctag[u][j] = ntag[u][j];
    }
    cur_tags = nxt_tags;
    cur_r0 = nxt_r0;
  }
  flush_bins(a, w, q, lane);
}

__global__ __launch_bounds__(kThreads) void tagged_digest_kernel(TaggedLaunch a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  tagged_body(a, blockIdx.x, smem);
}

// Fused build step for layout B (see build_step_kernel in digest.hip): the binning workgroups
// come first, then tree_blocks workgroups build the previous build's trees (step_trees). Both
// roles share one LDS reservation, the bins of two waves (33 KiB at B = 64), so four binning
// workgroups fill a CU's LDS: tree workgroups placed first would each
// hold back a binning workgroup until the tree is done (measured: 1.584 vs 1.551 ms at C4 with
// the trees last); placed last they start in LDS left over and in the first slots that free up.
__global__ __launch_bounds__(kThreads) void tagged_step_kernel(TaggedLaunch a, TreeLaunch t, uint32_t tree_blocks,
                                                               uint32_t Q) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t digest_blocks = gridDim.x - tree_blocks;
  if (blockIdx.x >= digest_blocks) {
    step_trees(t, Q, blockIdx.x - digest_blocks, smem);
    return;
  }
  tagged_body(a, blockIdx.x, smem);
}

size_t prepare_tagged(TaggedLaunch& a) {  // launcher-set fields; returns the bins' LDS bytes
  a.use_lds = a.B <= kTaggedLdsMaxBuckets ? 1 : 0;
  // bins of one workgroup <= 64 KiB: (kThreads/64) * B * (L + 1) * 4 bytes
  uint32_t L = 64;
  while (L > 1 && (uint64_t)a.B * (L + 1) * (kThreads / 64) * 4 > 65536) L >>= 1;
  // Records of 2^k >= 1 KiB on 16-byte boundaries take the row-reduced fast step (tagged_body
  // rows_ok), which folds each row to L partials itself: one slot per bucket is enough there, and
  // the bins shrink so that the fused step's tree workgroups still fit beside four binning
  // workgroups (at B = 1,000: 16 instead of 40 KiB per workgroup; with 40 KiB the CU's LDS was
  // full and the trees ran only after the binning, +139 vs +68 us over the digest in layout A).
  if (L < 64 && a.stride >= 1024 && (a.stride & (a.stride - 1)) == 0 && ((a.stride | a.shift) & 15) == 0) L = 1;
  a.lrep = L;
  a.inv_stride_f = 1.0f / (float)a.stride;
  return a.use_lds ? (size_t)(kThreads / 64) * ((size_t)a.B * L + a.B) * 4 : 0;
}

}  // namespace

void plan_tagged(uint64_t bytes, int cus, int waves_per_cu, uint64_t* wave_bytes, uint32_t* n_waves) {
  const uint64_t target = (uint64_t)(cus > 0 ? cus : 256) * (uint64_t)(waves_per_cu > 0 ? waves_per_cu : 8);
  uint64_t wb = (bytes + target - 1) / target;
  wb = (wb + kStep - 1) / kStep * kStep;
  if (wb < 2 * kStep) wb = 2 * kStep;
  if (wb > (8ull << 20)) wb = 8ull << 20;  // u32 bin slots stay exact; float offsets stay < 2^24
  *wave_bytes = wb;
  *n_waves = (uint32_t)((bytes + 16 + wb - 1) / wb);
}

hipError_t launch_tagged_digest(TaggedLaunch& a, hipStream_t st) {
  if (a.n_waves == 0) return hipSuccess;
  const size_t lds = prepare_tagged(a);
  const uint32_t blocks = (a.n_waves + (kThreads / 64) - 1) / (kThreads / 64);
  hipLaunchKernelGGL(tagged_digest_kernel, dim3(blocks), dim3(kThreads), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_tagged_step(TaggedLaunch& a, const TreeLaunch* t, hipStream_t st) {
  const size_t bins = a.n_waves ? prepare_tagged(a) : 0;
  uint32_t tree_blocks = 0, Q = 0, kw_word = 0;
  size_t lds = bins;
  if (t && t->P) {
    if (!build_step_fusable(t->B) || !t->sums_in || t->n_in) return hipErrorInvalidValue;
    uint32_t tree_lds = 0;
    // stream bytes 0: layout B keeps the packed / two-wave forms (its bins already take 33 KiB
    // per binning workgroup; the whole-workgroup trees' 40 KB would cut its residency)
    plan_step_trees(t->B, t->P, &Q, &tree_blocks, &tree_lds, &kw_word, 0);
    lds = std::max<size_t>(lds, (size_t)tree_lds);
  }
  const uint32_t blocks = (a.n_waves + (kThreads / 64) - 1) / (kThreads / 64);
  if (tree_blocks + blocks == 0) return hipSuccess;
  TreeLaunch tl = t ? *t : TreeLaunch{};
  tl.duo_kw_word = kw_word;
  hipLaunchKernelGGL(tagged_step_kernel, dim3(tree_blocks + blocks), dim3(kThreads), lds, st, a, tl, tree_blocks, Q);
  return hipGetLastError();
}

}  // namespace mde
