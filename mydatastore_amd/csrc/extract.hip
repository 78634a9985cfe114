// extract.hip -- out-of-sync range extract on device.
//
// Reference: StreamBucketsTask (main/manager.go:445-487) walks, for each requested bucket of a
// partition, the range [epoch_p_b_{lo}_, epoch_p_b_{hi}_) and emits every record; VerifyEpoch
// requests the de-duplicated diff set (utils.Int32Set, main/manager.go:1073,1086,1114). In layout A
// a bucket's records are one contiguous run, so the extract is a segmented gather: per partition
// the records of the requested buckets, duplicates removed, in ascending bucket order and LSM
// record order (the reference's bucket order is Go map iteration order, i.e. unspecified).
//
// Three launches, all device-side: count (one workgroup per partition: LDS bitmap of requested
// buckets, record/byte totals), scan (one workgroup: exclusive prefix sums + capacity check),
// copy (one workgroup per partition: record indices, value byte offsets and the value bytes,
// 16-byte vector copies when source and destination allow it).
//
// Layout B (records in write order with bucket tags): the same record set, found by testing every
// record's tag against the bitmap (a stream compaction over the partition, 2 bytes of tag read
// per record) and emitted in arrival order -- a bucket's records are not contiguous there, and
// the reference's order within a bucket is LSM key order, which write order does not carry.
//
// Request-order mode (ExtractLaunch::ordered, mde_stream_buckets): StreamBucketsTask's own list
// contract (main/manager.go:447-485) -- the ids are walked in the order given, a repeated id streams
// its bucket's records again, an id outside [0, B) streams nothing (no record carries it), and an
// empty list (counts[p] == 0) means every bucket 0..B-1 (:448-452). Layout A only. The count
// kernel sums the runs of the requests; the copy kernel scans the requests 64 at a time and copies
// each run in turn with the whole workgroup, as extract_copy_kernel does for marked buckets.
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {
namespace {

constexpr int kThreads = 256;
constexpr uint32_t kBitmapWords = kExtractMaxBuckets / 32;

__device__ void load_bitmap(const ExtractLaunch& a, uint32_t p, uint32_t* bm) {
  for (uint32_t w = threadIdx.x; w < (a.B + 31) / 32; w += kThreads) bm[w] = 0;
  __syncthreads();
  const int32_t n = a.counts[p];
  const int32_t* ids = a.ids + (uint64_t)p * a.ids_stride;
  for (int32_t i = threadIdx.x; i < n; i += kThreads) {
    const int32_t b = ids[i];
    if (b >= 0 && (uint32_t)b < a.B) atomicOr(&bm[b >> 5], 1u << (b & 31));
  }
  __syncthreads();
}

__device__ __forceinline__ bool marked(const uint32_t* bm, uint32_t b) { return (bm[b >> 5] >> (b & 31)) & 1u; }

// Request-order mode: how many requests partition p has, and the i-th one's bucket id.
__device__ __forceinline__ uint32_t n_requests(const ExtractLaunch& a, uint32_t p) {
  const int32_t n = a.counts[p];
  return n < 0 ? 0u : n == 0 ? a.B : (uint32_t)n;
}
__device__ __forceinline__ int32_t request_id(const ExtractLaunch& a, uint32_t p, uint32_t i) {
  return a.counts[p] == 0 ? (int32_t)i : a.ids[(uint64_t)p * a.ids_stride + i];
}

// Copies bucket bs's run (records r0..r1, their value bytes) to out_rec[rb..], out_values[bb..]
// with the whole workgroup.
__device__ void copy_run(const ExtractLaunch& a, uint32_t bs, uint64_t rb, uint64_t bb) {
  const uint64_t r0 = a.seg.seg_rec[bs], r1 = a.seg.seg_rec[bs + 1];
  const uint64_t src0 = segpos(a.seg, bs) - a.seg.shift, src1 = segpos(a.seg, bs + 1) - a.seg.shift;
  for (uint64_t r = r0 + threadIdx.x; r < r1; r += kThreads) {
    a.out_rec[rb + (r - r0)] = r;
    if (a.out_value_off) a.out_value_off[rb + (r - r0)] = bb + (recpos(a.seg, r) - src0);
  }
  if (a.out_values) {
    const uint8_t* src = a.values + src0;
    uint8_t* dst = a.out_values + bb;
    const uint64_t len = src1 - src0;
    if ((((uintptr_t)src | (uintptr_t)dst | len) & 15u) == 0) {
      const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
      u32x4* d4 = reinterpret_cast<u32x4*>(dst);
      for (uint64_t i = threadIdx.x; i < len / 16; i += kThreads) d4[i] = __builtin_nontemporal_load(s4 + i);
    } else {
      for (uint64_t i = threadIdx.x; i < len; i += kThreads) dst[i] = src[i];
    }
  }
}

__global__ __launch_bounds__(kThreads) void extract_count_kernel(ExtractLaunch a) {
  __shared__ uint32_t bm[kBitmapWords];
  __shared__ unsigned long long tot[2];
  const uint32_t p = blockIdx.x;
  if (threadIdx.x == 0) { tot[0] = 0; tot[1] = 0; }
  unsigned long long nr = 0, nb = 0;
  if (a.ordered) {  // request order: every request's run, repeats included
    __syncthreads();  // tot[] is zero before any thread adds to it
    const uint32_t n = n_requests(a, p);
    for (uint32_t i = threadIdx.x; i < n; i += kThreads) {
      const int32_t b = request_id(a, p, i);
      if (b < 0 || (uint32_t)b >= a.B) continue;
      const uint32_t s = p * a.B + (uint32_t)b;
      nr += a.seg.seg_rec[s + 1] - a.seg.seg_rec[s];
      nb += segpos(a.seg, s + 1) - segpos(a.seg, s);
    }
  } else if (a.tag) {  // layout B: test every record's tag
    load_bitmap(a, p, bm);
    for (uint64_t r = a.part_rec[p] + threadIdx.x; r < a.part_rec[p + 1]; r += kThreads)
      nr += marked(bm, min((uint32_t)a.tag[r], a.B - 1)) ? 1u : 0u;
    nb = nr * a.stride;
  } else {
    load_bitmap(a, p, bm);
    for (uint32_t b = threadIdx.x; b < a.B; b += kThreads) {
      if (!marked(bm, b)) continue;
      const uint32_t s = p * a.B + b;
      nr += a.seg.seg_rec[s + 1] - a.seg.seg_rec[s];
      nb += segpos(a.seg, s + 1) - segpos(a.seg, s);
    }
  }
  if (nr) atomicAdd(&tot[0], nr);
  if (nb) atomicAdd(&tot[1], nb);
  __syncthreads();
  if (threadIdx.x == 0) {
    a.scratch[p] = tot[0];
    a.scratch[(a.P + 1) + p] = tot[1];
  }
}

// Exclusive scans of the per-partition record and byte counts (one workgroup).
__global__ __launch_bounds__(kThreads) void extract_scan_kernel(ExtractLaunch a) {
  __shared__ unsigned long long carry[2];
  __shared__ unsigned long long part[2][kThreads];
  if (threadIdx.x == 0) { carry[0] = 0; carry[1] = 0; }
  __syncthreads();
  for (uint32_t base = 0; base < a.P; base += kThreads) {
    const uint32_t i = base + threadIdx.x;
    part[0][threadIdx.x] = i < a.P ? a.scratch[i] : 0;
    part[1][threadIdx.x] = i < a.P ? a.scratch[(a.P + 1) + i] : 0;
    __syncthreads();
    for (uint32_t o = 1; o < kThreads; o <<= 1) {  // Hillis-Steele inclusive scan
      unsigned long long x0 = threadIdx.x >= o ? part[0][threadIdx.x - o] : 0;
      unsigned long long x1 = threadIdx.x >= o ? part[1][threadIdx.x - o] : 0;
      __syncthreads();
      part[0][threadIdx.x] += x0;
      part[1][threadIdx.x] += x1;
      __syncthreads();
    }
    if (i < a.P) {
      const unsigned long long inc0 = part[0][threadIdx.x], inc1 = part[1][threadIdx.x];
      const unsigned long long own0 = a.scratch[i], own1 = a.scratch[(a.P + 1) + i];
      a.part_off[i] = carry[0] + inc0 - own0;
      a.scratch[2 * (a.P + 1) + i] = carry[1] + inc1 - own1;  // byte base
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      carry[0] += part[0][kThreads - 1];
      carry[1] += part[1][kThreads - 1];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.part_off[a.P] = carry[0];
    a.scratch[2 * (a.P + 1) + a.P] = carry[1];
    const bool over = carry[0] > a.rec_cap || (a.out_values && carry[1] > a.bytes_cap);
    *a.status = over ? -5 /* MDE_E_CAPACITY */ : 0;
  }
}

// Layout B copy: chunks of kThreads records in arrival order, a block prefix sum over the
// "requested" flags places them; each wave then copies the values of every 4th selected record.
__global__ __launch_bounds__(kThreads) void extract_copy_tagged_kernel(ExtractLaunch a) {
  __shared__ uint32_t bm[kBitmapWords];
  __shared__ uint32_t wave_tot[kThreads / 64];
  __shared__ uint64_t sel[kThreads];
  const uint32_t p = blockIdx.x;
  if (*a.status != 0) return;  // capacity exceeded: nothing is written
  load_bitmap(a, p, bm);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint64_t V = a.stride;
  uint64_t rb = a.part_off[p];
  const uint64_t bb0 = a.scratch[2 * (a.P + 1) + p], rb0 = rb;
  for (uint64_t c0 = a.part_rec[p]; c0 < a.part_rec[p + 1]; c0 += kThreads) {
    const uint64_t r = c0 + threadIdx.x;
    const bool m = r < a.part_rec[p + 1] && marked(bm, min((uint32_t)a.tag[r], a.B - 1));
    const uint64_t bal = __ballot(m);
    if (lane == 0) wave_tot[wid] = __popcll(bal);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (int w = 0; w < kThreads / 64; w++) {
      off += w < wid ? wave_tot[w] : 0u;
      tot += wave_tot[w];
    }
    const uint32_t pos = off + __popcll(bal & ((1ull << lane) - 1ull));
    if (m) {
      sel[pos] = r;
      a.out_rec[rb + pos] = r;
      if (a.out_value_off) a.out_value_off[rb + pos] = bb0 + (rb + pos - rb0) * V;
    }
    __syncthreads();
    if (a.out_values) {
      for (uint32_t k = wid; k < tot; k += kThreads / 64) {
        const uint8_t* src = a.values + sel[k] * V;
        uint8_t* dst = a.out_values + bb0 + (rb + k - rb0) * V;
        if ((((uintptr_t)src | (uintptr_t)dst | V) & 15u) == 0) {
          const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
          u32x4* d4 = reinterpret_cast<u32x4*>(dst);
          for (uint64_t i = lane; i < V / 16; i += 64) d4[i] = __builtin_nontemporal_load(s4 + i);
        } else {
          for (uint64_t i = lane; i < V; i += 64) dst[i] = src[i];
        }
      }
    }
    rb += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0 && p == a.P - 1 && a.out_value_off)
    a.out_value_off[a.part_off[a.P]] = a.scratch[2 * (a.P + 1) + a.P];
}

__global__ __launch_bounds__(kThreads) void extract_copy_kernel(ExtractLaunch a) {
  __shared__ uint32_t bm[kBitmapWords];
  __shared__ unsigned long long run[2];
  const uint32_t p = blockIdx.x;
  if (*a.status != 0) return;  // capacity exceeded: nothing is written
  if (threadIdx.x == 0) { run[0] = a.part_off[p]; run[1] = a.scratch[2 * (a.P + 1) + p]; }
  load_bitmap(a, p, bm);
  const int lane = threadIdx.x & 63;
  for (uint32_t b0 = 0; b0 < a.B; b0 += 64) {
    // one wave scans 64 buckets: offsets of the marked ones
    const uint32_t b = b0 + lane;
    const bool m = b < a.B && marked(bm, b);
    const uint32_t s = p * a.B + (b < a.B ? b : 0);
    unsigned long long nr = m ? a.seg.seg_rec[s + 1] - a.seg.seg_rec[s] : 0;
    unsigned long long nb = m ? segpos(a.seg, s + 1) - segpos(a.seg, s) : 0;
    unsigned long long er = nr, eb = nb;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long xr = __shfl_up(er, o), xb = __shfl_up(eb, o);
      if (lane >= o) { er += xr; eb += xb; }
    }
    const unsigned long long r_base = run[0] + er - nr, b_base = run[1] + eb - nb;
    __syncthreads();
    if (threadIdx.x == 63) { run[0] += er; run[1] += eb; }
    // copy each marked bucket of this 64-bucket window with the whole workgroup
    unsigned long long ball = __ballot(m);
    while (ball) {
      const int k = __ffsll((long long)ball) - 1;
      ball &= ball - 1;
      // every wave computed the same window scan, so all 256 threads copy this bucket together
      copy_run(a, p * a.B + b0 + k, __shfl(r_base, k), __shfl(b_base, k));
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && p == a.P - 1 && a.out_value_off) a.out_value_off[a.part_off[a.P]] = run[1];
}

// Request order: requests i0..i0+63 per round; lane i's run lands after the runs of the requests
// before it (a wave scan, computed identically by every wave), then the workgroup copies the
// non-empty runs in request order.
__global__ __launch_bounds__(kThreads) void extract_copy_ordered_kernel(ExtractLaunch a) {
  __shared__ unsigned long long run[2];
  const uint32_t p = blockIdx.x;
  if (*a.status != 0) return;  // capacity exceeded: nothing is written
  if (threadIdx.x == 0) { run[0] = a.part_off[p]; run[1] = a.scratch[2 * (a.P + 1) + p]; }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t n = n_requests(a, p);
  for (uint32_t i0 = 0; i0 < n; i0 += 64) {
    const uint32_t i = i0 + lane;
    const int32_t b = i < n ? request_id(a, p, i) : -1;
    const bool in = b >= 0 && (uint32_t)b < a.B;
    const uint32_t s = p * a.B + (in ? (uint32_t)b : 0u);
    unsigned long long nr = in ? a.seg.seg_rec[s + 1] - a.seg.seg_rec[s] : 0;
    unsigned long long nb = in ? segpos(a.seg, s + 1) - segpos(a.seg, s) : 0;
    unsigned long long er = nr, eb = nb;  // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned long long xr = __shfl_up(er, o), xb = __shfl_up(eb, o);
      if (lane >= o) { er += xr; eb += xb; }
    }
    const unsigned long long r_base = run[0] + er - nr, b_base = run[1] + eb - nb;
    __syncthreads();
    if (threadIdx.x == 63) { run[0] += er; run[1] += eb; }
    unsigned long long ball = __ballot(nr != 0);
    while (ball) {
      const int k = __ffsll((long long)ball) - 1;
      ball &= ball - 1;
      copy_run(a, __shfl(s, k), __shfl(r_base, k), __shfl(b_base, k));
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && p == a.P - 1 && a.out_value_off) a.out_value_off[a.part_off[a.P]] = run[1];
}

}  // namespace

hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st) {
  if (a.P == 0) return hipSuccess;
  hipLaunchKernelGGL(extract_count_kernel, dim3(a.P), dim3(kThreads), 0, st, a);
  hipLaunchKernelGGL(extract_scan_kernel, dim3(1), dim3(kThreads), 0, st, a);
  if (a.ordered)
    hipLaunchKernelGGL(extract_copy_ordered_kernel, dim3(a.P), dim3(kThreads), 0, st, a);
  else if (a.tag)
    hipLaunchKernelGGL(extract_copy_tagged_kernel, dim3(a.P), dim3(kThreads), 0, st, a);
  else
    hipLaunchKernelGGL(extract_copy_kernel, dim3(a.P), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace mde
