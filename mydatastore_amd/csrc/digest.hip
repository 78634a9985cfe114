// digest.hip -- bucket digest kernel (the HBM-bound hot loop of RawPartitionMerkleTree).
//
// Reference: main/merkle_tree.go:90-113 walks every bucket's records and folds
// CustomHash.Add (:25-32): value = (value + sum(bytes)) % 999999. Non-negative modular addition
// is associative, so a bucket's digest is (sum of all its value bytes) % 999999; this kernel
// produces the exact u64 byte sum per bucket and the tree kernel applies the modulus.
//
// Layout A: values form one contiguous arena ordered by (partition, bucket) -- the order the
// reference's per-bucket LSM range scans yield -- so bucket s is the byte range
// [segpos(s), segpos(s+1)). The arena is split into equal contiguous ranges, one per wave
// (64 lanes); a wave streams its range in 8 KiB steps (8 x 16-B nontemporal loads per lane,
// 1 KiB per wave-instruction, fully coalesced), byte-sums each dword with v_sad_u8 into a u32
// lane accumulator, and tracks the bucket it is in with wave-uniform scalar state. A step that
// lies wholly inside one bucket takes the fast path (loads + 32 v_sad_u8 per lane); a step that
// crosses bucket boundaries is split with byte masks. When the wave leaves a bucket it reduces
// its lanes (6 shuffles) and issues ONE u64 atomic add for that bucket: no LDS, no barriers,
// at most (#buckets touched) atomics per wave.
//
// Algorithmic bytes per launch: sum of value lengths.
#include "mde.h"
#include "mde_device.hpp"
#include "mde_internal.hpp"
#include "tree_body.hpp"
#include "verify_body.hpp"
#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstring>


namespace mde {
namespace {

constexpr int kThreads = 256;
constexpr uint64_t kMaxStepBytes = 16ull * 1024ull;  // wave ranges are multiples of this (4 steps)
constexpr uint64_t kMaxWaveBytes = 256ull << 20;    // largest contiguous range per wave

// Largest s in [lo, S) with segpos(s) <= x (lo if none). 64-ary search: one vector load and one
// ballot per round, log64(S) rounds. Must be called by all 64 lanes.
__device__ __forceinline__ uint32_t seg_search(const SegDesc& d, uint32_t lo, uint64_t x, int lane) {
  uint32_t hi = d.S;
  while (hi - lo > 1) {
    const uint32_t n = hi - lo;
    const uint32_t step = (n + 63u) / 64u;
    const uint32_t idx = lo + (uint32_t)lane * step;
    const bool pred = idx < hi && segpos(d, idx) <= x;
    const int c = __popcll(__ballot(pred));
    if (c == 0) return lo;
    lo = lo + (uint32_t)(c - 1) * step;
    hi = min(lo + step, hi);
  }
  return lo;
}

// Next bucket after s that contains position x == segpos(s+1) (skips empty buckets).
__device__ __forceinline__ uint32_t seg_next(const SegDesc& d, uint32_t s, uint64_t x, int lane) {
  const uint32_t idx = s + 1u + (uint32_t)lane;
  const bool pred = idx < d.S && segpos(d, idx) <= x;
  const int c = __popcll(__ballot(pred));
  if (c < 64) return s + (uint32_t)c;
  return seg_search(d, s + 64u, x, lane);
}

// Register window over the bucket starts: lane i holds segpos(base + i) (~0 past S), so the 63
// buckets base .. base + 62 have their bounds in registers. A bucket boundary inside the window is
// then a ballot and two readlanes instead of two dependent seg_rec round trips (seg_next + the
// new bucket's bounds); the window reloads once per 63 buckets.
struct SegWindow {
  uint32_t base;
  uint64_t start;  // this lane's segpos(base + lane)
  __device__ __forceinline__ void load(const SegDesc& d, uint32_t b, int lane) {
    base = b;
    const uint32_t idx = b + (uint32_t)lane;
    start = idx <= d.S ? segpos(d, idx) : ~0ull;
  }
};

// The bucket holding position x (segpos(lo) <= x < segpos(S)), with a register window loaded over
// it (win.base <= s <= win.base + 31), for a wave's first step. The 64-ary search costs log64(S)
// dependent seg_rec round trips -- 4 at the reference's default B = 1,000 over 1,024 partitions --
// plus the window's, each 1-2 us on a loaded HBM, while every wave of the launch waits: the fixed
// cost of a short launch (13.5 us of a 139 us production-shape digest, tools/size_probe.py). Layout
// A positions grow with the bucket index and buckets hold similar byte counts, so an interpolated
// guess from the arena bounds [first, last), one 64-lane sample every 32 buckets around it, and the
// window at the sampled bracket take two round trips; a guess off by more than ~1,000 buckets
// falls back to the search.
__device__ __forceinline__ uint32_t seg_start(const SegDesc& d, uint32_t lo, uint64_t x, uint64_t first, uint64_t last,
                                              int lane, SegWindow& win) {
  const uint32_t S = d.S;
  if (S - lo > 64u && last > first && x >= first) {
    const double f = (double)(x - first) / (double)(last - first);
    const int64_t i0 = (int64_t)(f * (double)S) - 32 * 32;
    const int64_t idx = i0 + 32 * (int64_t)lane;
    // monotone in the lane: samples below lo lie at or before x, samples past S after it
    const bool pred = idx < (int64_t)lo ? true : (idx >= (int64_t)S ? false : segpos(d, (uint32_t)idx) <= x);
    const int c = __popcll(__ballot(pred));
    if (c > 0 && c < 64) {
      const int64_t b = i0 + 32 * (int64_t)(c - 1);
      const uint32_t base = b < (int64_t)lo ? lo : (uint32_t)b;
      win.load(d, base, lane);
      // n = 0 only at lo (x before the first record, e.g. the 16-byte-rounded first wave):
      // bucket lo, as seg_search answers
      const int n = __popcll(__ballot(win.start <= x));
      if (n < 64) return base + (uint32_t)(n > 0 ? n - 1 : 0);
      // 64 bucket starts at or before x (a run of empty buckets): search on from the window's end
      const uint32_t s = seg_search(d, base + 63u, x, lane);
      win.load(d, s, lane);
      return s;
    }
  }
  const uint32_t s = seg_search(d, lo, x, lane);
  win.load(d, s, lane);
  return s;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t byte_mask(int lo, int hi) {  // bytes [lo, hi) of a dword
  const uint32_t mh = hi >= 4 ? 0xffffffffu : ((1u << (8 * hi)) - 1u);
  const uint32_t ml = lo >= 4 ? 0xffffffffu : ((1u << (8 * lo)) - 1u);
  return hi > lo ? (mh & ~ml) : 0u;
}

// Sum of bytes [a, b) (clamped to [0, 16]) of one 16-byte vector.
__device__ __forceinline__ uint32_t masked_sum16(u32x4 v, int64_t a, int64_t b, uint32_t acc) {
  const int ia = (int)min<int64_t>(max<int64_t>(a, 0), 16);
  const int ib = (int)min<int64_t>(max<int64_t>(b, 0), 16);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int lo = min(max(ia - 4 * k, 0), 4), hi = min(max(ib - 4 * k, 0), 4);
    acc = __builtin_amdgcn_sad_u8(v[k] & byte_mask(lo, hi), 0u, acc);
  }
  return acc;
}

__device__ __forceinline__ void flush(unsigned long long* sums, uint32_t s, uint32_t acc) {
  unsigned long long v = acc;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(sums + s, v);
}

template <int U, bool NT>
__device__ __forceinline__ void load_step(u32x4 (&v)[U], const u32x4* src, uint64_t p, uint64_t end,
                                          int lane, bool full) {
  if (full) {
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(src + u * 64) : src[u * 64];
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t x = p + (uint64_t)u * 1024u + (uint64_t)lane * 16u;
      v[u] = x < end ? (NT ? __builtin_nontemporal_load(src + u * 64) : src[u * 64]) : u32x4{0u, 0u, 0u, 0u};
    }
  }
}

// Streams the arena range [beg, end) of one wave: U = 16-byte loads per lane per step (step = U
// KiB per wave); NT = nontemporal loads; PIPE = issue the next step's loads before reducing the
// current one (register double buffer); PIPE = 2 also issues the first step's loads before the
// bucket search (from bucket s_lo on), so the wave's first HBM round trip overlaps the search's
// dependent seg_rec loads. Returns the last bucket the range touched.
template <int U, bool NT, int PIPE>
__device__ __forceinline__ uint32_t digest_range(const DigestLaunch& a, uint64_t beg, uint64_t end, uint32_t s_lo,
                                                 int lane) {
  constexpr uint64_t kStep = 1024ull * U;
  const SegDesc& d = a.seg;
  const u32x4* lane_base = reinterpret_cast<const u32x4*>(d.base) + lane;
  u32x4 cur[U];
  if (PIPE == 2) load_step<U, NT>(cur, lane_base + (beg >> 4), beg, end, lane, beg + kStep <= end);
  uint32_t s = seg_search(d, s_lo, beg, lane);
  uint64_t sb = segpos(d, s), se = segpos(d, s + 1);
  uint32_t acc = 0;
  if (PIPE == 1) load_step<U, NT>(cur, lane_base + (beg >> 4), beg, end, lane, beg + kStep <= end);
  for (uint64_t p = beg; p < end; p += kStep) {
    u32x4 v[U];
    const bool full = p + kStep <= end;
    if (PIPE) {
      const uint64_t pn = p + kStep;
      u32x4 nxt[U];
      if (pn < end) load_step<U, NT>(nxt, lane_base + (pn >> 4), pn, end, lane, pn + kStep <= end);
#pragma unroll
      for (int u = 0; u < U; u++) { v[u] = cur[u]; cur[u] = nxt[u]; }
    } else {
      load_step<U, NT>(v, lane_base + (p >> 4), p, end, lane, full);
    }
    if (full && sb <= p && p + kStep <= se) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
      }
    } else {
      const uint64_t q = min(p + kStep, end);
      for (;;) {
        const uint64_t lo = max(sb, p), hi = min(se, q);
        if (lo < hi) {
#pragma unroll
          for (int u = 0; u < U; u++) {
            const int64_t x = (int64_t)(p + (uint64_t)u * 1024u + (uint64_t)lane * 16u);
            acc = masked_sum16(v[u], (int64_t)lo - x, (int64_t)hi - x, acc);
          }
        }
        if (se >= q) break;
        flush(a.sums, s, acc);
        acc = 0;
        s = seg_next(d, s, se, lane);
        sb = segpos(d, s);
        se = segpos(d, s + 1);
      }
    }
  }
  flush(a.sums, s, acc);
  return s;
}

// Inclusive prefix sum over the 64 lanes (lane order), exact when the total fits 32 bits: DPP
// row shifts within each row of 16 lanes, then row_bcast:15 / row_bcast:31 across rows (gfx9).
// Call with all 64 lanes active.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Sum of the 64 lanes' u32 values, exact when it fits 32 bits: DPP within each row of 16 lanes
// (no LDS round trips), then the four row sums by readlane. Call with all 64 lanes active.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, true);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, true);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, true);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// digest_range for many short buckets (the reference's default B = 1000 puts a bucket boundary
// every few KiB):
//   * a true register double buffer: the loop is unrolled by two over buffers A and B and every
//     step issues its U loads unconditionally (addresses past `end` clamp to the last vector), so
//     the compiler's vmcnt bookkeeping waits for the current buffer only and the next step's
//     loads stay in flight across the reduction (digest_range's single-buffer swap makes hipcc
//     wait for both before the register moves);
//   * the bucket bounds come from a SegWindow: no dependent seg_rec loads per boundary;
//   * a step that crosses boundaries byte-sums each vector once and attributes whole vectors to
//     buckets by two compares (only a vector holding a boundary takes byte masks);
//   * a finished bucket's sum is a DPP wave reduction (u64 shuffles when this wave streamed more
//     than 16 MiB of it), parked in the window lane of that bucket; the window's sums go out as
//     ONE coalesced atomic per 63 buckets, not one atomic (and its vmcnt stall) per bucket.
// Bytes past `end` are loaded but never counted: whole-vector sums are used only for vectors
// inside [lo, hi) and the vector holding `end` is masked.
template <int U, bool NT>
__device__ __forceinline__ void load_step_clamped(u32x4 (&v)[U], const u32x4* base16, uint64_t p, uint64_t lastvec,
                                                  int lane) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint64_t x = min(p + (uint64_t)u * 1024u + (uint64_t)lane * 16u, lastvec);
    v[u] = NT ? __builtin_nontemporal_load(base16 + (x >> 4)) : base16[x >> 4];
  }
}

template <int U, bool NT, int PIPE, bool A8>
__device__ __forceinline__ uint32_t digest_range_win(const DigestLaunch& a, uint64_t beg, uint64_t end, uint32_t s_lo,
                                                     int lane) {
  constexpr uint64_t kStep = 1024ull * U;
  const SegDesc& d = a.seg;
  const u32x4* base16 = reinterpret_cast<const u32x4*>(d.base);
  const uint64_t lastvec = (end - 1) & ~15ull;  // the vector holding the range's last byte
  u32x4 va[U], vb[U];
  load_step_clamped<U, NT>(va, base16, beg, lastvec, lane);
  uint32_t s = seg_search(d, s_lo, beg, lane);
  SegWindow win;
  win.load(d, s, lane);
  uint64_t sb = readlane64(win.start, 0), se = readlane64(win.start, 1);
  uint64_t wsum = 0;     // this lane's window bucket (win.base + lane): its finished sum
  uint64_t bfrom = beg;  // where this wave entered bucket s
  uint32_t acc = 0;

  // the bucket being left: its sum into its window lane
  auto retire = [&](uint64_t upto) {
    uint64_t v;
    if (upto - bfrom <= (16ull << 20)) {
      v = wave_sum_u32(acc);  // <= 255 x 16 MiB < 2^32
    } else {
      v = acc;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    }
    if ((uint32_t)lane == s - win.base) wsum = v;
    acc = 0;
  };
  auto window_out = [&]() {  // one coalesced atomic for the window's finished buckets
    if (wsum) atomicAdd(a.sums + win.base + (uint32_t)lane, (unsigned long long)wsum);
    wsum = 0;
  };
  auto process = [&](const u32x4 (&v)[U], uint64_t p) {
    if (p + kStep <= end && sb <= p && p + kStep <= se) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
      }
      return;
    }
    uint32_t fs[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint32_t t = __builtin_amdgcn_sad_u8(v[u].x, 0u, 0u);
      t = __builtin_amdgcn_sad_u8(v[u].y, 0u, t);
      t = __builtin_amdgcn_sad_u8(v[u].z, 0u, t);
      fs[u] = __builtin_amdgcn_sad_u8(v[u].w, 0u, t);
    }
    const uint64_t q = min(p + kStep, end);
    // Two or more bucket starts inside the step (buckets of a few hundred bytes, e.g. 8-byte
    // timestamps at B = 1,000): segmented sums by a prefix scan instead of one pass per bucket.
    // E[u] = bytes of the step before vector (u, lane) in address order; window lane i reads
    // F(y_i) = bytes before its bucket's start y_i (clamped to the step), so bucket i's bytes in
    // the step are F(y_{i+1}) - F(y_i): one scan, a few shuffles and one reduction per step,
    // whatever the number of buckets.
    if (__popcll(__ballot(win.start > p && win.start < q)) >= 2) {
      uint32_t E[U];
      uint32_t total = 0;
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t incl = wave_incl_scan_u32(fs[u]);
        E[u] = total + incl - fs[u];
        total += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      }
      const uint32_t qrel = (uint32_t)(q - p);
      for (;;) {
        const uint64_t st = win.start;
        const uint32_t y = st <= p ? 0u : (st >= q ? qrel : (uint32_t)(st - p));
        const uint32_t vi = y >> 4, ui = vi >> 6, li = vi & 63u, boff = y & 15u;
        uint32_t e = 0;
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t eu = (uint32_t)__shfl((int)E[u], (int)li);
          e = ui == (uint32_t)u ? eu : e;
        }
        if (__ballot(boff != 0u)) {  // some bucket starts inside a vector: add its leading bytes
          if (A8 && !__ballot(boff & 7u)) {
            // every such start 8 bytes in (8-byte records): the vector's first two dwords, summed
            // at the owner lane. Standalone digest kernel only (A8): in the fused step's kernel
            // the extra registers (95 -> 99 VGPRs) cost 64-byte values at B = 1,000 ~5 % per
            // build, and there the trees, not the digest, bound 8-byte values at B = 1,000.
            uint32_t h = 0;
#pragma unroll
            for (int u = 0; u < U; u++) {
              const uint32_t lo8 = __builtin_amdgcn_sad_u8(v[u].y, 0u, __builtin_amdgcn_sad_u8(v[u].x, 0u, 0u));
              const uint32_t hu = (uint32_t)__shfl((int)lo8, (int)li);
              h = ui == (uint32_t)u ? hu : h;
            }
            e += boff ? h : 0u;
          } else {
            u32x4 w = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int u = 0; u < U; u++) {
              const u32x4 g = {(uint32_t)__shfl((int)v[u].x, (int)li), (uint32_t)__shfl((int)v[u].y, (int)li),
                               (uint32_t)__shfl((int)v[u].z, (int)li), (uint32_t)__shfl((int)v[u].w, (int)li)};
              if (ui == (uint32_t)u) w = g;
            }
            e = masked_sum16(w, 0, (int64_t)boff, e);
          }
        }
        const uint32_t F = vi >= (uint32_t)(kStep / 16) ? total : e;
        const uint32_t c = (uint32_t)__shfl_down((int)F, 1) - F;  // bucket base + lane, lanes 0..62
        const uint32_t k = s - win.base;
        const uint32_t cnt = (uint32_t)__popcll(__ballot(st < q));
        const uint32_t ck = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)k);
        if (lane == 0) acc += ck;
        if (cnt == 64u) {  // the step runs past the window: buckets k..62 all end inside it
          retire(readlane64(st, k + 1u));
          if ((uint32_t)lane > k && lane < 63) wsum = c;
          window_out();
          win.load(d, win.base + 63u, lane);
          s = win.base;
          sb = readlane64(win.start, 0);
          se = readlane64(win.start, 1);
          bfrom = sb;
          continue;
        }
        const uint32_t m = cnt - 1u;  // the last bucket starting before q: it runs on past q
        if (m > k) {
          retire(readlane64(st, k + 1u));
          if ((uint32_t)lane > k && (uint32_t)lane < m) wsum = c;
          s = win.base + m;
          sb = readlane64(st, m);
          se = readlane64(st, m + 1u);
          bfrom = sb;
          const uint32_t cm = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)m);
          acc = lane == 0 ? cm : 0u;
        }
        return;
      }
    }
    for (;;) {
      const uint64_t lo = max(sb, p), hi = min(se, q);
      if (lo < hi) {
        const int a32 = (int)(lo - p), b32 = (int)(hi - p);  // within [0, kStep]
#pragma unroll
        for (int u = 0; u < U; u++) {
          const int off = u * 1024 + lane * 16;
          const bool inside = off >= a32 && off + 16 <= b32;
          acc += inside ? fs[u] : 0u;
          if (!inside && off < b32 && off + 16 > a32)  // this vector holds a boundary
            acc = masked_sum16(v[u], (int64_t)(a32 - off), (int64_t)(b32 - off), acc);
        }
      }
      if (se >= q) break;
      retire(se);
      bfrom = se;
      // the bucket holding position se (empty buckets skipped), through the window
      uint32_t c = (uint32_t)__popcll(__ballot(win.start <= se));
      while (c == 64u) {  // past the window: its sums go out, the next 63 buckets come in
        window_out();
        win.load(d, win.base + 63u, lane);
        c = (uint32_t)__popcll(__ballot(win.start <= se));
      }
      s = win.base + c - 1u;
      sb = readlane64(win.start, c - 1u);
      se = readlane64(win.start, c);
    }
  };

  for (uint64_t p = beg;; p += 2 * kStep) {
    load_step_clamped<U, NT>(vb, base16, p + kStep, lastvec, lane);  // always issued (see above)
    process(va, p);
    if (p + kStep >= end) break;
    load_step_clamped<U, NT>(va, base16, p + 2 * kStep, lastvec, lane);
    process(vb, p + kStep);
    if (p + 2 * kStep >= end) break;
  }
  retire(min(se, end));
  window_out();
  return s;
}

// digest_range for fixed 8-byte records (the production epoch-index value is the LE64 write
// timestamp, main/manager.go:816) with short buckets (the reference's default B = 1,000 puts a
// bucket start every ~100 records): the prefix scan runs in RECORD space, once per 4 KiB step.
//   * each lane byte-sums its 8 records (two per 16-byte vector of each of the 4 coalesced 1 KiB
//     rows) and writes the 8 sums to LDS at their record index; the wave reads them back
//     transposed -- lane l gets records 8l .. 8l+7 of the step -- so ONE wave scan of the lane
//     totals plus a 7-add local scan give every record's prefix (LDS XOR-swizzled so the row
//     writes and the transposed ds_read_b128 are conflict-free);
//   * each lane writes its 8 exclusive local prefixes back (and its lane prefix), so the window
//     lane of every bucket starting in the step reads F(start) = bytes of the step before it with
//     two ds_read_b32 -- bucket i's bytes in the step are F(y_{i+1}) - F(y_i), as in
//     digest_range_win's scan path;
//   * a step inside one bucket just byte-sums into the lane accumulators.
// Needs value_stride == 8 and an 8-byte-aligned arena start (segpos multiples of 8).
// LDS swizzle (XOR inside 16-byte chunks): the row writes (lane l: words 128u + 2l, +1) and the
// transposed ds_read_b128 (lane l: its 8 records) both conflict-free.
constexpr int kRec8Rows = 4;  // 1 KiB rows per step
__device__ __forceinline__ uint32_t rec8_swz(uint32_t w) { return w ^ (((w >> 6) & 1u) << 2); }
__host__ __device__ constexpr uint32_t rec8_sums_words() { return 128u * kRec8Rows + 16u; }  // + word 512 = 0
__host__ __device__ constexpr uint32_t rec8_wave_words() { return rec8_sums_words() + 80u; }  // + 65 lane prefixes
__host__ __device__ constexpr uint32_t rec8_lds_bytes() { return rec8_wave_words() * 4u * (kThreads / 64); }

template <bool NT>
__device__ __forceinline__ void load_rec8(u32x4 (&v)[kRec8Rows], __amdgpu_buffer_rsrc_t rs, uint32_t off, int lane) {
#pragma unroll
  for (int u = 0; u < kRec8Rows; u++)
    v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(u * 64 + lane) * 16u,
                                                                          off, NT ? 2 : 0));
}

// The rec8 stream's bookkeeping (r06, VERDICT r05 item 3: the VALU per 4 KiB step):
//   * the window holds each bucket start as a 32-bit record slot relative to the wave's range
//     (int32: < 0 before it, clamped far past it), so a step's slot of every start is one
//     subtract and one med3 -- no 64-bit compares, subtracts or shifts per step;
//   * the step position, the current bucket, its bounds, the window base and the bucket's running
//     sum are wave-uniform scalars, and finished buckets park 32-bit step sums in their window lane
//     (a bucket wholly inside one step holds < 2^32 bytes); only the bucket the wave carries
//     across steps needs 64 bits, and it is a scalar;
//   * the record-space prefix scan is as described above; only the window lanes of the buckets a
//     step touches use its result.
// Counted in the ISA (gfx950): 58 VALU per scan step for the bookkeeping and the scan (the round-5
// form: ~117 with the per-load readfirstlane loops), plus the 4 loads' readfirstlane loops (below).
// The wave's range stays in VGPRs (it derives from threadIdx.x >> 6), so each of the 4 loads per
// step is a one-iteration readfirstlane loop (6 VALU). Measured with the range in SGPRs as well
// (no loops, 58 VALU per step): the digest alone 136-138 us either way, but the fused production
// step SLOWER, 176-180 vs 166-167 us per build, the tree waves 154-155 vs 139-143 us each
// (profiles/r06/r06c_rec8_timeline.jsonl, r06e_rec8_ab.jsonl; the same as round 3's SGPR-range
// probe): what the co-resident SHA-256 waves lose is not the stream's VALU count.
template <bool NT>
__device__ __forceinline__ uint32_t digest_range_rec8(const DigestLaunch& a, uint64_t beg_v, uint64_t end_v,
                                                       uint32_t s_lo, int lane, uint32_t* lds, uint64_t first,
                                                       uint64_t last) {
  constexpr int ROWS = kRec8Rows;
  constexpr uint32_t kRecs = 128u * ROWS;        // record slots per step
  constexpr uint32_t kLaneRecs = 2u * ROWS;      // record slots per lane after the transpose
  constexpr uint32_t kFoldSteps = 16384 / ROWS;  // fast steps per lane fold: exact in 32 bits
  constexpr int32_t kFar = 0x3fffffff;           // a start past every slot of the range
  const SegDesc& d = a.seg;
  uint32_t* R = lds;                             // record sums, then exclusive local prefixes (swizzled)
  uint32_t* E = lds + rec8_sums_words();        // lane exclusive prefixes; E[64] = the step's total
  const uint64_t beg = beg_v, end = end_v;
  const uint64_t span = ((end - beg) + 15) & ~15ull;                      // <= kMaxWaveBytes
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(d.base + beg), (short)0, (int)span, 0x00020000);
  u32x4 va[ROWS], vb[ROWS];
  load_rec8<NT>(va, rs, 0, lane);  // the first step's loads before the bucket search
  if (lane == 0) R[kRecs] = 0;           // F(kRecs) = E[64] + 0
  // the window as record slots of the range: lane i = bucket base + i
  auto rel_of = [&](uint64_t st) -> int32_t {
    return st < beg ? -1 : (int32_t)min<uint64_t>((st - beg) >> 3, (uint64_t)kFar);
  };
  uint32_t base;
  int32_t rel;
  auto win_load = [&](uint32_t b) {
    base = b;
    const uint32_t idx = b + (uint32_t)lane;
    rel = idx <= d.S ? rel_of(segpos(d, idx)) : kFar;
  };
  {
    SegWindow w0;
    const uint32_t s0 = seg_start(d, s_lo, beg, first, last, lane, w0);
    base = __builtin_amdgcn_readfirstlane(w0.base);
    rel = rel_of(w0.start);
    s_lo = __builtin_amdgcn_readfirstlane(s0);
  }
  uint32_t s = s_lo;  // the bucket the wave is in (uniform)
  int32_t sbr = __builtin_amdgcn_readlane(rel, (int)(s - base));        // its first slot
  int32_t ser = __builtin_amdgcn_readlane(rel, (int)(s - base + 1u));   // the next bucket's
  uint32_t wlo = 0, whi = 0;   // this lane's window bucket (base + lane): its finished sum
  uint32_t acc = 0;            // lane accumulator of whole steps inside bucket s
  uint32_t acc_steps = 0;      // uniform: fast steps in acc
  uint64_t accs = 0;           // uniform: bucket s's bytes folded out of acc and from scan steps
  uint32_t* const wrow = R + rec8_swz(2u * (uint32_t)lane);
  uint32_t* rd[ROWS / 2];
#pragma unroll
  for (int j = 0; j < ROWS / 2; j++) rd[j] = R + rec8_swz(kLaneRecs * (uint32_t)lane + 4u * j);

  auto fold = [&]() {
    if (acc_steps) accs += wave_sum_u32(acc);
    acc = 0;
    acc_steps = 0;
  };
  auto window_out = [&]() {  // one coalesced atomic for the window's finished buckets
    const uint64_t w = ((uint64_t)whi << 32) | wlo;
    if (w) atomicAdd(a.sums + base + (uint32_t)lane, (unsigned long long)w);
    wlo = whi = 0;
  };
  // P = the step's first slot in the range, kq = its slots (< kRecs only on the range's last step)
  auto process = [&](const u32x4 (&v)[ROWS], int32_t P, uint32_t kq) {
    if (kq == kRecs && sbr <= P && P + (int32_t)kRecs <= ser) {  // the whole step inside bucket s
#pragma unroll
      for (int u = 0; u < ROWS; u++) {
        acc = __builtin_amdgcn_sad_u8(v[u].x, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].y, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].z, 0u, acc);
        acc = __builtin_amdgcn_sad_u8(v[u].w, 0u, acc);
      }
      if (++acc_steps == kFoldSteps) fold();
      return;
    }
#pragma unroll
    for (int u = 0; u < ROWS; u++) {
      const uint32_t r0 = __builtin_amdgcn_sad_u8(v[u].y, 0u, __builtin_amdgcn_sad_u8(v[u].x, 0u, 0u));
      const uint32_t r1 = __builtin_amdgcn_sad_u8(v[u].w, 0u, __builtin_amdgcn_sad_u8(v[u].z, 0u, 0u));
      *reinterpret_cast<uint2*>(wrow + 128u * u) = make_uint2(r0, r1);
    }
    uint32_t c[kLaneRecs + 1];
    c[0] = 0u;
#pragma unroll
    for (int j = 0; j < ROWS / 2; j++) {
      const uint4 x = *reinterpret_cast<const uint4*>(rd[j]);
      c[4 * j + 1] = c[4 * j] + x.x;
      c[4 * j + 2] = c[4 * j + 1] + x.y;
      c[4 * j + 3] = c[4 * j + 2] + x.z;
      c[4 * j + 4] = c[4 * j + 3] + x.w;
    }
    const uint32_t tot = c[kLaneRecs];
    const uint32_t incl = wave_incl_scan_u32(tot);
#pragma unroll
    for (int j = 0; j < ROWS / 2; j++)
      *reinterpret_cast<uint4*>(rd[j]) = make_uint4(c[4 * j], c[4 * j + 1], c[4 * j + 2], c[4 * j + 3]);
    E[lane] = incl - tot;
    if (lane == 63) E[64] = incl;
    for (;;) {
      const int32_t t = rel - P;  // this lane's bucket start, as a slot of the step
      const uint32_t k = (uint32_t)min(max(t, 0), (int32_t)kq);  // clamped to [0, kq] (v_med3_i32)
      const uint32_t F = R[rec8_swz(k)] + E[k / kLaneRecs];
      // lane i: bucket base + i's bytes in the step (lanes 0..62), F of the next lane (wave_shl:1)
      const uint32_t cb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)F, 0x130, 0xf, 0xf, true) - F;
      const uint32_t k0 = s - base;
      const uint32_t cnt = (uint32_t)__popcll(__ballot(t < (int32_t)kq));  // starts before the step's end
      accs += (uint32_t)__builtin_amdgcn_readlane((int)cb, (int)k0);
      const uint32_t m = cnt - 1u;  // the last bucket starting before the step's end
      if (cnt == 64u || m > k0) {
        // bucket k0 is finished, and every bucket between it and m lies inside this step
        fold();
        const uint32_t hi_end = cnt == 64u ? 63u : m;
        if ((uint32_t)lane == k0) {
          wlo = (uint32_t)accs;
          whi = (uint32_t)(accs >> 32);
        } else if ((uint32_t)lane > k0 && (uint32_t)lane < hi_end) {
          wlo = cb;
        }
        if (cnt == 64u) {  // the step runs past the window: its sums go out, the next 63 come in
          window_out();
          win_load(base + 63u);
          s = base;
          accs = 0;
          sbr = __builtin_amdgcn_readlane(rel, 0);
          ser = __builtin_amdgcn_readlane(rel, 1);
          continue;
        }
        s = base + m;
        sbr = __builtin_amdgcn_readlane(rel, (int)m);
        ser = __builtin_amdgcn_readlane(rel, (int)(m + 1u));
        accs = (uint32_t)__builtin_amdgcn_readlane((int)cb, (int)m);
      }
      return;
    }
  };

  const uint32_t nslots = (uint32_t)((end - beg + 7) >> 3);
  for (uint32_t P = 0;; P += 2 * kRecs) {
    load_rec8<NT>(vb, rs, (P + kRecs) * 8u, lane);  // always issued (bounded by the range)
    process(va, (int32_t)P, min(kRecs, nslots - P));
    if (P + kRecs >= nslots) break;
    load_rec8<NT>(va, rs, (P + 2 * kRecs) * 8u, lane);
    process(vb, (int32_t)(P + kRecs), min(kRecs, nslots - P - kRecs));
    if (P + 2 * kRecs >= nslots) break;
  }
  fold();
  if ((uint32_t)lane == s - base) {
    wlo = (uint32_t)accs;
    whi = (uint32_t)(accs >> 32);
  }
  window_out();
  return s;
}

// One contiguous range of wave_bytes per wave. `block` = this workgroup's index among the digest
// workgroups of the launch.
template <int U, bool NT, int PIPE, int PRIO = 0, bool WIN = false, bool A8 = false, bool REC8 = false>
__device__ __forceinline__ void digest_body(const DigestLaunch& a, uint32_t block, uint32_t* lds = nullptr) {
  // Streaming waves issue little VALU; when tree waves (back-to-back SHA-256 VALU) share the CU,
  // a raised priority keeps the loads flowing and the SHA waves take the slack.
  if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  const int lane = threadIdx.x & 63;
  const uint32_t wave = block * (kThreads / 64) + (threadIdx.x >> 6);
  if (wave >= a.n_waves) return;
  const SegDesc& d = a.seg;
  const uint64_t first = segpos(d, 0) & ~15ull;
  const uint64_t last = segpos(d, d.S);
  const uint64_t beg = first + (uint64_t)wave * a.wave_bytes;
  if (beg >= last) return;
  if (REC8)
    digest_range_rec8<NT>(a, beg, min(beg + a.wave_bytes, last), 0u, lane,
                          lds + (threadIdx.x >> 6) * rec8_wave_words(), first, last);
  else if (WIN)
    digest_range_win<U, NT, PIPE, A8>(a, beg, min(beg + a.wave_bytes, last), 0u, lane);
  else
    digest_range<U, NT, PIPE>(a, beg, min(beg + a.wave_bytes, last), 0u, lane);
}

// Interleaved pieces (DigestLaunch::pieces): the wave streams `pieces` ranges of wave_bytes,
// piece_stride apart, so the whole grid sweeps the arena front to back together. Each piece is a
// digest_range (its own bucket search, from the previous piece's last bucket on, and flush).
template <int U, bool NT, int PIPE, int PRIO = 0, bool WIN = false, bool A8 = false, bool REC8 = false>
__device__ __forceinline__ void digest_body_pieces(const DigestLaunch& a, uint32_t block, uint32_t* lds = nullptr) {
  if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  const int lane = threadIdx.x & 63;
  const uint32_t wave = block * (kThreads / 64) + (threadIdx.x >> 6);
  if (wave >= a.n_waves) return;
  const SegDesc& d = a.seg;
  const uint64_t first = segpos(d, 0) & ~15ull;
  const uint64_t last = segpos(d, d.S);
  uint32_t s = 0;
  uint64_t beg = first + (uint64_t)wave * a.wave_bytes;
  for (uint32_t j = 0; j < a.pieces && beg < last; j++, beg += a.piece_stride)
    s = REC8  ? digest_range_rec8<NT>(a, beg, min(beg + a.wave_bytes, last), s, lane,
                                      lds + (threadIdx.x >> 6) * rec8_wave_words(), first, last)
        : WIN ? digest_range_win<U, NT, PIPE, A8>(a, beg, min(beg + a.wave_bytes, last), s, lane)
              : digest_range<U, NT, PIPE>(a, beg, min(beg + a.wave_bytes, last), s, lane);
}

// MODE: 0 = one static range per wave, 2 = interleaved pieces; 3 and 4 = 0 and 2 with the bucket
// bounds in a register window (SegWindow); 5 and 6 = 0 and 2 for fixed 8-byte records with the
// prefix scan in record space (digest_range_rec8; LDS: rec8_lds_bytes).
__host__ __device__ constexpr bool mode_rec8(int mode) { return mode == 5 || mode == 6; }
__host__ __device__ constexpr bool mode_pieces(int mode) { return mode == 2 || mode == 4 || mode == 6; }
template <int U, bool NT, int PIPE, int PRIO, int MODE, bool A8>
__device__ __forceinline__ void digest_dispatch(const DigestLaunch& a, uint32_t block, uint32_t* lds) {
  if (mode_pieces(MODE))
    digest_body_pieces<U, NT, PIPE, PRIO, MODE == 4, A8, mode_rec8(MODE)>(a, block, lds);
  else
    digest_body<U, NT, PIPE, PRIO, MODE == 3, A8, mode_rec8(MODE)>(a, block, lds);
}

template <int U, bool NT, int PIPE, int PRIO = 0, int MODE = 0>
__global__ __launch_bounds__(kThreads) void bucket_digest_kernel(DigestLaunch a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  digest_dispatch<U, NT, PIPE, PRIO, MODE, true>(a, blockIdx.x, lds);
}

// Fused build step (software pipelining of consecutive builds in ONE launch): workgroups
// [0, tree_blocks) build the trees of the PREVIOUS build from its byte sums (tree_body, LDS
// levels), the rest stream THIS build's arena into the other scratch slot (digest_body). The
// latency-bound SHA-256 tree waves co-run with the HBM-bound streaming waves inside one dispatch,
// so a run of builds on one stream pays neither a second kernel boundary per build nor a
// cross-stream event wait. A tree workgroup keeps the standalone tree kernel's shape (one live
// wave per workgroup up to B = 128, the rest exit at once), so the SHA waves spread over many
// CUs instead of crowding a few; tree workgroups come first so the dispatcher places them before
// the streaming grid (sized to be fully resident) fills the remaining slots.
template <int U, bool NT, int PIPE, int PRIO = 0, int MODE = 0>
__global__ __launch_bounds__(kThreads) void build_step_kernel(DigestLaunch a, TreeLaunch t, uint32_t tree_blocks,
                                                              uint32_t Q) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  if (blockIdx.x < tree_blocks) {
    step_trees(t, Q, blockIdx.x, lds);
    return;
  }
  digest_dispatch<U, NT, PIPE, PRIO, MODE, false>(a, blockIdx.x - tree_blocks, lds);
}

// First LDS word of the small build's bucket sums (after `groups` tree regions, 16-byte aligned).
__host__ __device__ __forceinline__ uint32_t small_build_sums_word(uint32_t groups, uint32_t words) {
  return (groups * words + 3u) & ~3u;
}
// Partitions per small-build workgroup: 256 / G, or in the split-schedule form 128 / G (a wide
// tree, G = 256: one).
__host__ __device__ __forceinline__ uint32_t small_build_groups(uint32_t G, bool duo) {
  const uint32_t half = (uint32_t)kThreads / 2;
  return duo ? (G > half ? 1u : half / G) : (uint32_t)kThreads / G;
}
// First LDS word of the split-schedule K+W slots (after the bucket sums, 16-byte aligned).
__host__ __device__ __forceinline__ uint32_t small_build_kw_word(uint32_t groups, uint32_t words, uint32_t B) {
  return (small_build_sums_word(groups, words) + groups * B * 2u + 3u) & ~3u;
}

// One-launch build of small arenas (the synchronous one-partition calls of VerifyEpoch, and the
// batcher's many small partitions, mde_batch_build). Workgroup b owns partitions
// [b * groups, (b + 1) * groups) (groups = 256 / G trees per workgroup, tree_body's shape): digest
// phase bucket-parallel over ITS partitions' buckets -- thread i sums bucket i's bytes with 16-byte
// loads (a wave walking the bucket boundaries of a small arena in order pays one dependent seg_rec
// load per bucket, which is what bounds the streaming kernel there) -- then, after a device-scope
// fence and a barrier, the same workgroup builds those partitions' trees with tree_body. Every
// bucket is summed by exactly one workgroup, so no cross-workgroup synchronisation is needed; it
// saves the second launch of the digest + tree pair.
// kDuo: the trees run split-schedule (tree_body_duo, the latency form) with the workgroup's upper
// half as schedule helpers, so a workgroup holds half as many partitions of B <= 128 buckets.
// The body is a device function: the resident build service (server_kernel) runs it once per
// request in a workgroup that stays resident between requests -- every barrier inside is reached
// by all kThreads threads (no early exits), so the workgroup can loop.
template <bool kDuo>
__device__ __forceinline__ void small_build_body(const SegDesc& d, const TreeLaunch& t, uint32_t G, uint32_t words,
                                                 uint32_t blk, uint32_t* lds) {
  const u32x4* base = reinterpret_cast<const u32x4*>(d.base);
  const uint32_t groups = small_build_groups(G, kDuo);
  const uint32_t s_beg = min(blk * groups * t.B, d.S), s_end = min((blk + 1) * groups * t.B, d.S);
  const uint32_t nb = s_end - s_beg;
  // this workgroup's bucket sums live in LDS after the tree levels (no global atomics, no fence)
  unsigned long long* sums = reinterpret_cast<unsigned long long*>(lds + small_build_sums_word(groups, words));
  for (uint32_t i = threadIdx.x; i < nb; i += kThreads) sums[i] = 0ull;
  __syncthreads();
  // K threads per bucket (K = 256 / nb rounded down to a power of two, >= 1), each taking every
  // K-th 16-byte vector of the bucket, four loads in flight
  uint32_t K = 1;
  while (K * 2 * nb <= (uint32_t)kThreads) K *= 2;
  const uint32_t j = threadIdx.x % K;
  for (uint32_t s = s_beg + threadIdx.x / K; s < s_end; s += kThreads / K) {
    const uint64_t lo = segpos(d, s), hi = segpos(d, s + 1);
    const int64_t l = (int64_t)lo, h = (int64_t)hi;
    uint32_t acc = 0;
    uint64_t x = (lo & ~15ull) + 16ull * j;
    for (; x + 48ull * K < hi; x += 64ull * K) {
      const u32x4 v0 = __builtin_nontemporal_load(base + (x >> 4));
      const u32x4 v1 = __builtin_nontemporal_load(base + ((x + 16ull * K) >> 4));
      const u32x4 v2 = __builtin_nontemporal_load(base + ((x + 32ull * K) >> 4));
      const u32x4 v3 = __builtin_nontemporal_load(base + ((x + 48ull * K) >> 4));
      acc = masked_sum16(v0, l - (int64_t)x, h - (int64_t)x, acc);
      acc = masked_sum16(v1, l - (int64_t)(x + 16ull * K), h - (int64_t)(x + 16ull * K), acc);
      acc = masked_sum16(v2, l - (int64_t)(x + 32ull * K), h - (int64_t)(x + 32ull * K), acc);
      acc = masked_sum16(v3, l - (int64_t)(x + 48ull * K), h - (int64_t)(x + 48ull * K), acc);
    }
    for (; x < hi; x += 16ull * K)
      acc = masked_sum16(__builtin_nontemporal_load(base + (x >> 4)), l - (int64_t)x, h - (int64_t)x, acc);
    if (acc) atomicAdd(sums + (s - s_beg), (unsigned long long)acc);
  }
  __syncthreads();
  TreeLaunch tl = t;
  tl.sums_in = sums;
  tl.sums_clear = nullptr;
  tl.sums_base = s_beg;
  if (!t.root_out) {  // digest-only build: the leaf outputs of this workgroup's partitions, no tree
    const uint32_t p0 = blk * groups;
    leaves_waves(tl, p0 + threadIdx.x / 64u, (uint32_t)kThreads / 64u, p0 + groups);
    return;
  }
  if (kDuo) {
    u32x4* kw = reinterpret_cast<u32x4*>(lds + small_build_kw_word(groups, words, t.B));
    tree_body_duo(tl, G, words, blk, lds, (uint32_t)kThreads / 2, kw);
  } else {
    tree_body<true>(tl, G, words, blk, lds, kThreads);
  }
}

template <bool kDuo>
__global__ __launch_bounds__(kThreads) void small_build_kernel(SegDesc d, TreeLaunch t, uint32_t G, uint32_t words) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  small_build_body<kDuo>(d, t, G, words, blockIdx.x, lds);
}

constexpr uint64_t kServerExit = ~0ull - 1ull;
constexpr uint64_t kServerFinal = 1ull << 62;  // served after closing: the last request of this workgroup

// The resident build service (mde_server, server.cpp): workgroup blockIdx.x serves slot
// blockIdx.x -- a one-partition RawPartitionMerkleTree call, or one VerifyEpoch decision step
// (verify_fused_body), without a kernel launch, a copy command or an event per call. Thread 0 polls the slot's `req` word in coherent pinned host
// memory (a relaxed system-scope load: a read over PCIe, no cache invalidation per poll), the
// workgroup copies the posted request into LDS with per-lane vector loads (never the scalar cache:
// the slot is rewritten for every request), optionally stages its inputs into device memory (one
// PCIe round trip for all of them instead of one per dependent load), runs small_build_body
// (outputs stored straight into the slot's pinned out region), makes every thread's stores
// visible at system scope and publishes `done`. Exit: the host's kServerStop, or the lifetime --
// then thread 0 sets `closed`, fences (seq_cst, system) and reads `req` once more, so a request
// posted concurrently is either served here or seen by its host as closed (server.cpp relaunches).
// Every wave reaches the exit: the decision is thread 0's, broadcast through LDS behind a barrier.
__global__ __launch_bounds__(kThreads) void server_kernel(ServerSlot* slots, uint64_t lifetime) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  constexpr uint32_t kReqWords = (uint32_t)(sizeof(ServerReq) / 4);
  static_assert(sizeof(ServerReq) % 4 == 0, "request in whole words");
  __shared__ uint64_t cmd;
  __shared__ __attribute__((aligned(16))) uint32_t req[kReqWords];  // raw words (TreeLaunch has initializers)
  __shared__ VerifyShared vsh;  // the decision step's static LDS
  ServerSlot* s = slots + blockIdx.x;
  const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + lifetime;
  uint64_t served = 0;
  if (threadIdx.x == 0) served = __hip_atomic_load(&s->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    if (threadIdx.x == 0) {
      uint64_t c;
      for (;;) {
        const uint64_t r = __hip_atomic_load(&s->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (r == kServerStop) {
          c = kServerExit;
          break;
        }
        if (r != served) {
          c = r;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() > t_end) {
          __hip_atomic_store(&s->closed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __atomic_thread_fence(__ATOMIC_SEQ_CST);  // system scope: closed is visible before req is re-read
          const uint64_t r2 = __hip_atomic_load(&s->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          c = (r2 != served && r2 != kServerStop) ? (r2 | kServerFinal) : kServerExit;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
      cmd = c;
    }
    __syncthreads();
    const uint64_t c = cmd;
    if (c == kServerExit) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system scope: the request's bytes, posted before req
    for (uint32_t w = threadIdx.x; w < kReqWords; w += (uint32_t)kThreads)
      req[w] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(&s->r) + w, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    const char* rq = reinterpret_cast<const char*>(req);
#define MDE_REQ_FIELD(x) ({ decltype(ServerReq::x) v_; __builtin_memcpy(&v_, rq + offsetof(ServerReq, x), sizeof v_); v_; })
    if (MDE_REQ_FIELD(stage)) {  // the inputs into device memory: every load in flight at once
      const u32x4* src = reinterpret_cast<const u32x4*>(MDE_REQ_FIELD(src));
      u32x4* dst = reinterpret_cast<u32x4*>(MDE_REQ_FIELD(dev_in));
      const uint32_t n = (uint32_t)(MDE_REQ_FIELD(stage_bytes) / 16u);
      constexpr uint32_t kU = 8;
      for (uint32_t i0 = 0; i0 < n; i0 += kU * (uint32_t)kThreads) {
        u32x4 v[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
          const uint32_t i = i0 + u * (uint32_t)kThreads + threadIdx.x;
          if (i < n) v[u] = src[i];
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
          const uint32_t i = i0 + u * (uint32_t)kThreads + threadIdx.x;
          if (i < n) dst[i] = v[u];
        }
      }
      __threadfence_block();
      __syncthreads();
    }
    // the descriptors are read in place from LDS (the bodies take references): held in registers,
    // a decision step's ~0.6 KB descriptor alone would take ~160 VGPRs
    if (MDE_REQ_FIELD(kind) == 1) {  // VerifyEpoch's decision step for one partition
      const VerifyFusedLaunch& v = *reinterpret_cast<const VerifyFusedLaunch*>(rq + offsetof(ServerReq, v));
      const uint32_t vg = MDE_REQ_FIELD(v_G), vw = MDE_REQ_FIELD(v_words), vs = MDE_REQ_FIELD(v_stage);
      if (MDE_REQ_FIELD(v_deep))
        verify_fused_body<true>(v, 0, vg, vw, vs, lds, vsh);
      else
        verify_fused_body<false>(v, 0, vg, vw, vs, lds, vsh);
    } else {
      const SegDesc& d = *reinterpret_cast<const SegDesc*>(rq + offsetof(ServerReq, d));
      const TreeLaunch& t = *reinterpret_cast<const TreeLaunch*>(rq + offsetof(ServerReq, t));
      const uint32_t g = MDE_REQ_FIELD(G), w = MDE_REQ_FIELD(words);
      if (MDE_REQ_FIELD(duo))
        small_build_body<true>(d, t, g, w, 0, lds);
      else
        small_build_body<false>(d, t, g, w, 0, lds);
    }
#undef MDE_REQ_FIELD
    __threadfence_system();  // this thread's output stores, before done
    __syncthreads();
    if (threadIdx.x == 0) {
      served = c & ~kServerFinal;
      __hip_atomic_store(&s->done, served, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (c & kServerFinal) return;
  }
}

typedef void (*DigestKernel)(DigestLaunch);
typedef void (*StepKernel)(DigestLaunch, TreeLaunch, uint32_t, uint32_t);
struct Variant {
  int id;
  DigestKernel fn;
  StepKernel step;
  int mode;
};

#define MDE_VARIANT(ID, MODE) \
  { ID, bucket_digest_kernel<4, true, 2, 2, MODE>, build_step_kernel<4, true, 2, 2, MODE>, MODE }

// Kernel variants (the tuning knob mde_set_tuning's digest_variant = id; plan_digest picks one per
// build). Every variant: 4 KiB steps (4 x 16-byte nontemporal loads per lane), the next step's
// loads issued before the current one is reduced and the first step's before the bucket search,
// issue priority 2. Round 1-5 variants measured and rejected (other unrolls and cache policies,
// tail stealing, 8 KiB rec8 steps, other priorities; DESIGN.md sections 4.1, 4.9) were removed in
// round 6; the ids of the shipped ones are unchanged.
const Variant kVariants[] = {
    MDE_VARIANT(11, 0),  // one static range per wave (byte sums per 16-byte vector)
    MDE_VARIANT(12, 2),  // 11 with interleaved pieces (large shares)
    MDE_VARIANT(13, 3),  // register window over the bucket bounds + prefix-scan steps (short buckets)
    MDE_VARIANT(14, 4),  // 13 with interleaved pieces
    MDE_VARIANT(15, 5),  // fixed 8-byte records: record-space prefix scan (the production value)
    MDE_VARIANT(16, 6),  // 15 with interleaved pieces
};
#undef MDE_VARIANT


const Variant& variant(int v) {
  for (const Variant& x : kVariants)
    if (x.id == v) return x;
  return kVariants[0];
}

}  // namespace

bool bucket_digest_variant_valid(int v) {
  for (const Variant& x : kVariants)
    if (x.id == v) return true;
  return false;
}


// LDS of one small-build workgroup: tree regions, bucket sums and counts, and in the split-schedule
// form the K+W ring.
size_t small_build_lds(const TreeGeometry& g, uint32_t B, bool duo) {
  const uint32_t groups = small_build_groups(g.G, duo);
  return duo ? (size_t)small_build_kw_word(groups, g.words, B) * 4u + duo_kw_bytes((uint32_t)kThreads / 2)
             : (size_t)small_build_sums_word(groups, g.words) * 4u + (size_t)groups * B * 8u;
}
constexpr size_t kSmallBuildLdsMax = 160u * 1024u;  // one gfx950 CU

// Split-schedule trees (latency form) unless that would take more than kDuoMaxBlocks
// workgroups (a wide tree has one workgroup per partition either way; narrower trees pack half as
// many partitions per workgroup) or more LDS than a CU has (B = 4,096: the plain form).
bool small_build_duo(const TreeGeometry& g, uint32_t P, uint32_t B) {
  const uint32_t groups_duo = small_build_groups(g.G, true);
  const uint32_t blocks_duo = (P + groups_duo - 1) / groups_duo;
  return tree_duo_enabled() && (g.G > (uint32_t)kThreads / 2 || blocks_duo <= kDuoMaxBlocks) &&
         small_build_lds(g, B, true) <= kSmallBuildLdsMax;
}

// The one-launch build serves arenas of at most kSmallBuildMaxBytes per workgroup on average:
// one workgroup streams its partitions' bytes alone (~0.1 TB/s), so larger arenas go to the
// full-chip digest kernel + tree kernel instead.
bool small_build_fits(uint64_t bytes, uint32_t P, uint32_t B) {
  TreeGeometry g;
  if (!tree_geometry(B, &g) || g.G > (uint32_t)kThreads || P < 1) return false;
  const bool duo = small_build_duo(g, P, B);
  if (small_build_lds(g, B, duo) > kSmallBuildLdsMax) return false;
  const uint32_t groups = small_build_groups(g.G, duo);
  const uint64_t blocks = (P + (uint64_t)groups - 1) / groups;
  return bytes <= kSmallBuildMaxBytes * blocks;
}

hipError_t launch_small_build(const SegDesc& d, const TreeLaunch& t, hipStream_t st) {
  TreeGeometry g;
  tree_geometry(t.B, &g);
  const bool duo = small_build_duo(g, t.P, t.B);
  const uint32_t groups = small_build_groups(g.G, duo);
  const uint32_t blocks = (t.P + groups - 1) / groups;
  const size_t lds = small_build_lds(g, t.B, duo);
  if (duo)
    hipLaunchKernelGGL(small_build_kernel<true>, dim3(blocks), dim3(kThreads), lds, st, d, t, g.G, g.words);
  else
    hipLaunchKernelGGL(small_build_kernel<false>, dim3(blocks), dim3(kThreads), lds, st, d, t, g.G, g.words);
  return hipGetLastError();
}

// Static LDS of server_kernel (the command word and the request copy), below the dynamic LDS.
constexpr size_t kServerStaticLds = sizeof(ServerReq) + sizeof(VerifyShared) + 64u;

bool server_plan(uint32_t P, uint32_t B, size_t lds_bytes, uint32_t* G, uint32_t* words, uint32_t* duo) {
  TreeGeometry g;
  if (P < 1 || B < 1 || !tree_geometry(B, &g) || g.G > (uint32_t)kThreads) return false;
  // one workgroup: the split-schedule form when its LDS fits the service's launch (kDuoMaxBlocks
  // does not bind for one workgroup), else the plain form
  bool d = tree_duo_enabled() && small_build_lds(g, B, true) <= lds_bytes;
  if (P > small_build_groups(g.G, d)) d = false;
  if (P > small_build_groups(g.G, d) || small_build_lds(g, B, d) > lds_bytes) return false;
  *G = g.G;
  *words = g.words;
  *duo = d ? 1u : 0u;
  return true;
}

size_t server_lds_bytes(uint32_t max_buckets) {
  uint32_t vg, vw, vs;
  size_t m = verify_fused_lds(mde_verify_peer_capacity(max_buckets), &vg, &vw, &vs);
  for (uint32_t B = 1; B <= max_buckets; B++) {
    TreeGeometry g;
    if (!tree_geometry(B, &g) || g.G > (uint32_t)kThreads) continue;
    size_t need = small_build_lds(g, B, tree_duo_enabled());
    if (need + kServerStaticLds > kSmallBuildLdsMax) need = small_build_lds(g, B, false);
    if (need + kServerStaticLds <= kSmallBuildLdsMax) m = std::max(m, need);
  }
  return (m + 15u) & ~size_t(15);
}

hipError_t launch_server(ServerSlot* slots, uint32_t n_slots, uint64_t lifetime_ticks, size_t lds_bytes,
                         hipStream_t st) {
  if (lds_bytes + kServerStaticLds > kSmallBuildLdsMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(server_kernel, dim3(n_slots), dim3(kThreads), lds_bytes, st, slots, lifetime_ticks);
  return hipGetLastError();
}

bool bucket_digest_pieces(int v) { return mode_pieces(variant(v).mode); }
bool bucket_digest_rec8(int v) { return mode_rec8(variant(v).mode); }
uint32_t bucket_digest_rec8_lds_bytes(int v) { return bucket_digest_rec8(v) ? rec8_lds_bytes() : 0u; }
int bucket_digest_pieces_sibling(int v) {  // the same kernel with interleaved pieces
  switch (v) {
    case 11: return 12;
    case 13: return 14;
    case 15: return 16;
    default: return v;
  }
}

int bucket_digest_blocks_per_cu(int v, int cap) {
  int blocks = 0;
  const size_t lds = bucket_digest_rec8_lds_bytes(v);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, variant(v).fn, kThreads, lds) != hipSuccess ||
      blocks <= 0)
    blocks = 4;
  if (cap > 0 && cap < blocks) blocks = cap;
  return blocks;
}

// One contiguous range per resident wave: every wave of the grid is co-resident and all ranges
// are equal, so the launch has no tail of late waves.
void plan_bucket_digest(uint64_t bytes, int cus, int blocks_per_cu, int oversub, uint64_t piece_bytes,
                        uint64_t* wave_bytes, uint32_t* n_waves, uint32_t* pieces) {
  const uint64_t target_waves = (uint64_t)(cus > 0 ? cus : 256) *
                                (uint64_t)(blocks_per_cu > 0 ? blocks_per_cu : 4) * (kThreads / 64) *
                                (uint64_t)(oversub > 0 ? oversub : 1);
  uint64_t wb = (bytes + target_waves - 1) / target_waves;
  *pieces = 1;
  if (piece_bytes && oversub <= 1 && wb >= 2 * piece_bytes) {
    // Interleaved pieces: every resident wave takes k pieces of ~piece_bytes, piece j of wave w at
    // (j * n_waves + w) * wave_bytes, so the whole grid sweeps the arena front to back together.
    // Pieces are 1 KiB multiples (one wave-instruction), so the largest share exceeds the mean by
    // at most k KiB; each piece switch costs one bucket search and one flush.
    const uint64_t k = (wb + piece_bytes / 2) / piece_bytes;
    uint64_t c = (bytes + 16 + target_waves * k - 1) / (target_waves * k);
    c = (c + 1023) / 1024 * 1024;
    if (c <= kMaxWaveBytes) {
      *wave_bytes = c;
      *n_waves = (uint32_t)target_waves;
      *pieces = (uint32_t)k;
      return;
    }
  }
  if (wb > kMaxStepBytes) {
    wb = (wb + kMaxStepBytes - 1) / kMaxStepBytes * kMaxStepBytes;
    if (wb < 2 * kMaxStepBytes) wb = 2 * kMaxStepBytes;
  } else {
    // Small arenas (under 32 MiB at 2,048 waves): short ranges (16-byte multiples, >= 256 B) over
    // the whole grid. Each bucket boundary a wave crosses is one dependent seg_rec load (~1-2 us),
    // so one wave walking all 64 buckets of an 8 KB one-partition build took ~60 us; spread over
    // 32 waves it takes two or three such loads per wave.
    wb = (wb + 15) / 16 * 16;
    if (wb < 256) wb = 256;
  }
  // A lane reads wave_bytes / 64 bytes of its range, so its u32 accumulator holds at most
  // 255 * wave_bytes / 64 (< 2^30 at the cap): exact. The cap sits far above every resident
  // grid's range (64 GiB over 2,048 waves = 32 MiB), so big arenas keep one range per resident
  // wave instead of queueing extra rounds of waves (C3 with an 8 MiB cap: 3.8 rounds, a tail).
  if (wb > kMaxWaveBytes) wb = kMaxWaveBytes;
  *wave_bytes = wb;
  *n_waves = (uint32_t)((bytes + 16 + wb - 1) / wb);
}

hipError_t launch_bucket_digest(const DigestLaunch& a, hipStream_t st) {
  if (a.n_waves == 0) return hipSuccess;
  const uint32_t blocks = (a.n_waves + (kThreads / 64) - 1) / (kThreads / 64);
  // With an oversubscribed grid, residency is capped by reserving LDS the kernel never touches:
  // 160 KiB / lds_bytes workgroups fit per CU, and the dispatcher hands the remaining workgroups
  // to whichever CU frees a slot first (load balance around CUs slowed by co-running kernels).
  hipLaunchKernelGGL(variant(a.variant).fn, dim3(blocks), dim3(kThreads), a.lds_bytes, st, a);
  return hipGetLastError();
}

// Partitions per tree wave in the fused step: up to 8, as many as the LDS budget holds. A packed
// tree wave's critical path grows with Q (B = 64: 8.4 node-hash passes at Q = 8, 13.8 at Q = 16);
// on small arenas it outlasts the stream: 800 MB of 8-byte values at B = 64 took 137-141 us per
// fused build at Q = 2-8 vs 165-167 at Q = 16, C4 and its N = 8 shard unchanged within noise
// (profiles/r02af_treeq.jsonl).
uint32_t build_step_tree_q(uint32_t B) {
  const uint32_t n1 = (B + 1) / 2;
  const uint32_t per = (n1 + (n1 + 1) / 2) * 8u * 4u;  // bytes of level buffers per partition
  const uint32_t q = (kStepTreeLdsMax - 64u) / per;
  return q > 8u ? 8u : q;
}

bool build_step_fusable(uint32_t B) { return B >= 1 && build_step_tree_q(B) >= 1; }

// Where the split-schedule trees of a fused step keep their K+W ring: after the level buffers when
// that fits kStepTreeLdsMax, else over level-1 buffer space that levels of <= 64 nodes never touch
// (they read at most 128 nodes of either level buffer); 0 = no room (plain tree_body).
uint32_t duo_step_kw_word(uint32_t B, uint32_t* lds_bytes) {
  if (!tree_duo_enabled()) return 0;
  const uint32_t words = tree_lds_words(B), kw_words = duo_kw_bytes(kStepTreeWideThreads / 2) / 4u;
  const uint32_t app = (words + 3u) & ~3u;
  if ((app + kw_words) * 4u <= kStepTreeLdsMax) {
    *lds_bytes = std::max<uint32_t>(*lds_bytes, (app + kw_words) * 4u);
    return app;
  }
  const uint32_t n1 = (B + 1) / 2;
  return n1 * 8u >= 128u * 8u + kw_words ? 4u + 128u * 8u : 0u;
}

void plan_step_trees(uint32_t B, uint32_t P, uint32_t* Q, uint32_t* blocks, uint32_t* lds_bytes, uint32_t* duo_kw_word,
                     uint64_t stream_bytes) {
  *duo_kw_word = 0;
  // One packed tree wave per partition (Q = 1, B > 128) has a critical path of 34 dependent
  // compressions at B = 1,000; two waves per partition (tree_body over 128 threads) cut it to 24.
  // With many partitions the trees, not the stream, bound a small arena: 800 MB of 8-byte values
  // at B = 1,000 over 1,024 partitions went 248 -> 234 us per fused build, C4 at B = 1,000 and
  // 64-byte values unchanged; with few partitions the packed wave hides behind the stream (the
  // N = 8 shard at B = 1,000, 128 partitions: 218 vs 221 us), hence the partition threshold
  // (profiles/r02ak_half.jsonl). Four waves per partition measured worse at C4 (1,645 vs
  // 1,615 us; r02af_treewide.jsonl).
  // r02, rejected: the pair shape of the standalone tree kernel (tree_body_pair: two partitions
  // per workgroup, 28 instead of 34 wave-compressions per partition at B = 1,000, the same
  // critical path). Beside the stream it bought nothing: 8-byte values at B = 1,000 230-233 vs
  // 233 us per fused build, 64-byte values 269-271 vs 266-267, C4 at B = 1,000 within noise
  // (profiles/r02an_pair_trees.jsonl). Stopping every tree at its first level of <= 64 nodes
  // (a probe, wrong roots) took 8-byte values to 193-197 us: the top levels' six dependent node
  // hashes, not their instruction count, hold the step.
  const uint32_t q = build_step_tree_q(B);
  // r06: few wide trees beside a short stream -- the whole workgroup per partition (tree_body_duo,
  // 128 hashing + 128 schedule threads: ~16 dependent compression-equivalents at B = 1,000 against
  // ~34 for the packed wave and ~24 for the two-wave form). Same process, alternating, warm
  // (profiles/r06/r06g_tree_forms.jsonl, r06h_tree_forms.jsonl; packed / two-wave / whole, us per
  // fused build): 8-byte values at B = 1,000 over 128 partitions (the production shape's N = 8
  // shard, 100 MB) 112 / 71 / 61, 256 partitions 126 / 86 / 69, 512 partitions 172 / 128 / 103;
  // 64-byte values over 128 partitions 120 / 80 / 69. Where the stream outlasts every tree form
  // (C4 at B = 1,000 on its N = 8 shard, 1.28 GB: 213-214 / 217 / 216-217; B = 300 within noise)
  // the packed wave's smaller footprint stays; 1,024 partitions keep the two-wave form (whole:
  // 211 vs 166). The rule: whole for at most kStepTreeWideMinPartitions partitions when the stream
  // is under kStepTreeWholeMaxBytes (~120 us at 6.5 TB/s, the packed trees' critical path).
  const bool whole_fits = P <= kStepTreeWideMinPartitions && stream_bytes && stream_bytes < kStepTreeWholeMaxBytes;
  if (q == 1 && (B + 1) / 2 > 64 && tree_duo_enabled() && whole_fits) {
    *Q = kStepTreeWholeWG;
    *blocks = P;
    const uint32_t words = (tree_lds_words(B) + 3u) & ~3u;
    *duo_kw_word = words;
    *lds_bytes = words * 4u + duo_kw_bytes(kStepTreeWideThreads);
    return;
  }
  if (q == 1 && (B + 1) / 2 > 64 && P >= kStepTreeWideMinPartitions) {
    *Q = 0;
    *blocks = P;
    *lds_bytes = tree_lds_words(B) * 4u;
    *duo_kw_word = duo_step_kw_word(B, lds_bytes);
    return;
  }
  *Q = q;
  *blocks = q ? (P + q - 1) / q : 0;
  *lds_bytes = packed_tree_lds_words(B, q) * 4u;
}

hipError_t launch_build_step(const DigestLaunch& a, const TreeLaunch* t, hipStream_t st) {
  uint32_t tree_blocks = 0, Q = 0, lds = a.lds_bytes, kw_word = 0;
  if (t && t->P) {
    // every partition of a fused step has t->B buckets (no per-tree n_in)
    if (!build_step_fusable(t->B) || !t->sums_in || t->n_in) return hipErrorInvalidValue;
    uint32_t tree_lds = 0;
    plan_step_trees(t->B, t->P, &Q, &tree_blocks, &tree_lds, &kw_word,
                    a.wave_bytes * a.n_waves * (uint64_t)(a.pieces ? a.pieces : 1u));
    // every workgroup of the dispatch reserves the tree waves' LDS; kStepTreeLdsMax keeps the
    // streaming grid fully resident (the whole-workgroup form's 40 KB leaves 3 per CU: at most
    // 512 tree workgroups beside the 2-per-CU stream, the short streams that form is chosen for)
    lds = std::max<uint32_t>(lds, tree_lds);
  }
  const uint32_t digest_blocks = (a.n_waves + (kThreads / 64) - 1) / (kThreads / 64);
  if (tree_blocks + digest_blocks == 0) return hipSuccess;
  TreeLaunch tl = t ? *t : TreeLaunch{};
  tl.duo_kw_word = kw_word;
  hipLaunchKernelGGL(variant(a.variant).step, dim3(tree_blocks + digest_blocks), dim3(kThreads), lds, st, a, tl,
                     tree_blocks, Q);
  return hipGetLastError();
}

}  // namespace mde
