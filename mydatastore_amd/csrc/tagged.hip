// tagged.hip -- bucket digests for layout B: records grouped by partition, in arrival order,
// each carrying its bucket tag.
//
// Reference: the bucket of a record is fixed at write time (Manager.getKeyBucket,
// main/manager.go:773-778) and the build folds CustomHash.Add over each bucket's records
// (main/merkle_tree.go:90-113). Layout A needs the records sorted by bucket; layout B hashes them
// into the B leaf buckets inside the kernel:
//   * equal contiguous byte ranges per wave (one per resident wave), 16-byte nontemporal loads;
//   * each lane byte-sums (v_sad_u8) the part of its 16 bytes that belongs to the first record
//     it touches; a record spilling into the vector's tail goes straight to its bin;
//   * records are contiguous runs of lanes, so a key-segmented inclusive scan over the wave
//     (6 shuffle steps) leaves each run's total on its last lane, which does ONE LDS atomic into
//     the wave's private bucket bins (u64 byte sum + u32 record count per bucket);
//   * when the wave passes a partition boundary it flushes its bins to global u64/u32 atomics
//     (B per partition per wave) and clears them. B > 1024 bins skip LDS and add globally.
// Fixed-length values only (value_stride > 0).
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {
namespace {

constexpr int kThreads = 256;
constexpr int kU = 4;                       // 16-byte loads per lane per step
constexpr uint64_t kStep = 1024ull * kU;    // 4 KiB per wave step

__device__ __forceinline__ uint32_t byte_mask(int lo, int hi) {
  const uint32_t mh = hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
  const uint32_t ml = lo >= 4 ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
  return hi > lo ? (mh & ~ml) : 0u;
}

__device__ __forceinline__ uint32_t masked_sum16(u32x4 v, int64_t a, int64_t b) {
  const int ia = (int)min<int64_t>(max<int64_t>(a, 0), 16);
  const int ib = (int)min<int64_t>(max<int64_t>(b, 0), 16);
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int lo = min(max(ia - 4 * k, 0), 4), hi = min(max(ib - 4 * k, 0), 4);
    acc = __builtin_amdgcn_sad_u8(v[k] & byte_mask(lo, hi), 0u, acc);
  }
  return acc;
}

struct Bins {
  unsigned long long* sum;  // LDS, B entries (nullptr: global only)
  uint32_t* cnt;
};

// Partition of record r (linear walk from q; only taken for records past the wave's partition).
__device__ __forceinline__ uint32_t part_of(const TaggedLaunch& a, uint64_t r, uint32_t q) {
  while (q + 1 < a.P && a.part_rec[q + 1] <= r) q++;
  return q;
}

__device__ __forceinline__ void add_bin(const TaggedLaunch& a, const Bins& bins, uint32_t q,
                                        uint64_t q_end, uint64_t r, uint32_t s, uint32_t c) {
  if (!s && !c) return;
  const uint32_t b = a.tag[r];
  if (bins.sum && r < q_end) {
    if (s) atomicAdd(bins.sum + b, (unsigned long long)s);
    if (c) atomicAdd(bins.cnt + b, c);
  } else {
    const uint64_t idx = (uint64_t)part_of(a, r, q) * a.B + b;
    if (s) atomicAdd(a.sums + idx, (unsigned long long)s);
    if (c) atomicAdd(a.counts + idx, c);
  }
}

__device__ void flush_bins(const TaggedLaunch& a, const Bins& bins, uint32_t q, int lane) {
  if (!bins.sum) return;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (uint32_t j = lane; j < a.B; j += 64) {
    const unsigned long long s = bins.sum[j];
    const uint32_t c = bins.cnt[j];
    if (s) atomicAdd(a.sums + (uint64_t)q * a.B + j, s);
    if (c) atomicAdd(a.counts + (uint64_t)q * a.B + j, c);
    bins.sum[j] = 0;
    bins.cnt[j] = 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__global__ __launch_bounds__(kThreads) void tagged_digest_kernel(TaggedLaunch a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  Bins bins{nullptr, nullptr};
  if (a.use_lds) {
    bins.sum = reinterpret_cast<unsigned long long*>(smem) + (uint64_t)wid * a.B;
    bins.cnt = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned long long*>(smem) + 4ull * a.B) +
               (uint64_t)wid * a.B;
    for (uint32_t j = lane; j < a.B; j += 64) { bins.sum[j] = 0; bins.cnt[j] = 0; }
  }
  const uint32_t wave = blockIdx.x * (kThreads / 64) + wid;
  if (wave >= a.n_waves) return;
  const uint64_t V = a.stride;
  const uint64_t r_lo = a.part_rec[0], r_hi = a.part_rec[a.P];
  const uint64_t valid_lo = a.shift + r_lo * V, last = a.shift + r_hi * V;
  const uint64_t first = valid_lo & ~15ull;
  const uint64_t beg = first + (uint64_t)wave * a.wave_bytes;
  if (beg >= last) return;
  const uint64_t end = min(beg + a.wave_bytes, last);
  auto rec_of = [&](uint64_t pos) -> uint64_t {  // record containing byte position pos
    const uint64_t rel = pos - a.shift;
    uint64_t r = (uint64_t)((double)rel * a.inv_stride);
    while (r * V > rel) r--;
    while ((r + 1) * V <= rel) r++;
    return r;
  };
  // partition of the wave's first byte (64-ary search over part_rec)
  uint64_t r_first = rec_of(max(beg, valid_lo));
  uint32_t q = 0;
  {
    uint32_t lo = 0, hi = a.P;
    while (hi - lo > 1) {
      const uint32_t n = hi - lo, step = (n + 63u) / 64u;
      const uint32_t idx = lo + (uint32_t)lane * step;
      const int c = __popcll(__ballot(idx < hi && a.part_rec[idx] <= r_first));
      if (c == 0) break;
      lo = lo + (uint32_t)(c - 1) * step;
      hi = min(lo + step, hi);
    }
    q = lo;
    while (q + 1 < a.P && a.part_rec[q + 1] <= r_first) q++;  // skip empty partitions
  }
  uint64_t q_end = a.part_rec[q + 1];  // first record past partition q
  const u32x4* lane_base = reinterpret_cast<const u32x4*>(a.base) + lane;

  for (uint64_t p = beg; p < end; p += kStep) {
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint64_t x = p + (uint64_t)u * 1024u + (uint64_t)lane * 16u;
      v[u] = x < end ? __builtin_nontemporal_load(lane_base + (p >> 4) + u * 64) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint64_t x = p + (uint64_t)u * 1024u + (uint64_t)lane * 16u;
      const uint64_t lo = max(x, max(beg, valid_lo)), hi = min(x + 16, end);
      uint32_t key = 0xffffffffu, s_a = 0;
      if (lo < hi) {
        const uint64_t ra = rec_of(lo), rb = rec_of(hi - 1);
        const uint64_t ra_end = a.shift + (ra + 1) * V;
        s_a = masked_sum16(v[u], (int64_t)lo - (int64_t)x, (int64_t)min(hi, ra_end) - (int64_t)x);
        key = (uint32_t)(ra - r_first);
        // records starting inside [lo, hi) are counted here; tail records are summed here
        if (a.shift + ra * V >= lo) add_bin(a, bins, q, q_end, ra, 0u, 1u);
        for (uint64_t r = ra + 1; r <= rb; r++) {
          const uint64_t rs = a.shift + r * V, re = rs + V;
          const uint32_t s = masked_sum16(v[u], (int64_t)rs - (int64_t)x, (int64_t)min(hi, re) - (int64_t)x);
          add_bin(a, bins, q, q_end, r, s, 1u);
        }
      }
      // key-segmented inclusive scan: runs of equal keys are contiguous lanes
      uint32_t tot = s_a;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ot = __shfl_up(tot, o), ok = __shfl_up(key, o);
        if (lane >= o && ok == key) tot += ot;
      }
      const uint32_t next_key = __shfl_down(key, 1);
      const bool tail = lane == 63 || next_key != key;
      if (tail && key != 0xffffffffu) add_bin(a, bins, q, q_end, r_first + key, tot, 0u);
    }
    // leave partitions the next step no longer touches
    const uint64_t pn = p + kStep;
    while (q + 1 < a.P && pn < end && a.shift + q_end * V <= pn) {
      flush_bins(a, bins, q, lane);
      q++;
      q_end = a.part_rec[q + 1];
    }
  }
  flush_bins(a, bins, q, lane);
}

}  // namespace

void plan_tagged(uint64_t bytes, int cus, int blocks_per_cu, uint64_t* wave_bytes, uint32_t* n_waves) {
  const uint64_t target = (uint64_t)(cus > 0 ? cus : 256) * (uint64_t)(blocks_per_cu > 0 ? blocks_per_cu : 2) *
                          (kThreads / 64);
  uint64_t wb = (bytes + target - 1) / target;
  wb = (wb + kStep - 1) / kStep * kStep;
  if (wb < 2 * kStep) wb = 2 * kStep;
  if (wb > (8ull << 20)) wb = 8ull << 20;
  *wave_bytes = wb;
  *n_waves = (uint32_t)((bytes + 16 + wb - 1) / wb);
}

hipError_t launch_tagged_digest(TaggedLaunch& a, hipStream_t st) {
  if (a.n_waves == 0) return hipSuccess;
  a.use_lds = a.B <= kTaggedLdsMaxBuckets ? 1 : 0;
  const size_t lds = a.use_lds ? (size_t)(kThreads / 64) * a.B * 12 : 0;
  const uint32_t blocks = (a.n_waves + (kThreads / 64) - 1) / (kThreads / 64);
  hipLaunchKernelGGL(tagged_digest_kernel, dim3(blocks), dim3(kThreads), lds, st, a);
  return hipGetLastError();
}

}  // namespace mde
