// wire_body.hpp -- EpochTreeObject protobuf encode/decode of ONE object, as device functions
// shared by the standalone wire kernels (wire.hip) and the fused verify kernel (verify.hip).
//
// Reference: VerifyEpoch persists and serves proto.Marshal(MerkleTreeToPartitionEpochObject(...))
// (main/manager.go:1041-1056, rpc/server.go:170-187) and peers decode it back into a tree
// (EpochTreeObjectToMerkleTree, main/merkle_tree.go:140-157). Message (datap/data.proto:60-68):
//   1 int32 partition | 2 int64 lower_epoch | 3 int64 upper_epoch | 4 repeated bytes buckets
//   5 repeated int32 buckets_size (packed) | 6 bool valid | 7 int32 items
// proto3 encoding as protobuf-go emits it: fields in number order, zero scalars omitted, each
// bucket a length-delimited 8-byte LE64 digest, sizes one packed run of varints, negative int32
// sign-extended to a 10-byte varint. Leaves follow tree.Leafs: an odd B repeats the last bucket.
#pragma once
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {

__device__ __forceinline__ uint32_t varint_len(uint64_t v) {
  uint32_t n = 1;
  while (v >= 0x80) { v >>= 7; n++; }
  return n;
}

__device__ __forceinline__ uint32_t put_varint(uint8_t* p, uint64_t v) {
  uint32_t n = 0;
  while (v >= 0x80) { p[n++] = (uint8_t)(v | 0x80); v >>= 7; }
  p[n++] = (uint8_t)v;
  return n;
}

__device__ __forceinline__ uint64_t sx32(int32_t v) { return (uint64_t)(int64_t)v; }

// Object i by one wave (lane = 0..63); no barriers, so a fused kernel may call it from one wave.
__device__ __forceinline__ void encode_object(const WireEncodeLaunch& a, uint32_t i, uint32_t lane) {
  const uint32_t B = a.B, L = B + (B & 1u);
  const uint64_t* dg = a.digest + (uint64_t)i * B;
  const int32_t* sz = a.size + (uint64_t)i * B;
  uint8_t* out = a.out + (uint64_t)i * a.out_stride;
  const int32_t part = a.partition ? a.partition[i] : 0;
  const bool valid = a.valid && a.valid[i];
  // items: given, or the tree.Leafs sum (duplicate leaf counted again), int32 wrap
  int32_t items;
  if (a.items) {
    items = a.items[i];
  } else {
    uint32_t acc = 0;
    for (uint32_t j = lane; j < L; j += 64) acc += (uint32_t)sz[min(j, B - 1)];
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    items = (int32_t)acc;
  }
  // header (lane 0) -- identical length computation in every lane
  uint32_t hdr = 0;
  if (part) hdr += 1 + varint_len(sx32(part));
  if (a.lower) hdr += 1 + varint_len((uint64_t)a.lower);
  if (a.upper) hdr += 1 + varint_len((uint64_t)a.upper);
  if (lane == 0) {
    uint32_t q = 0;
    if (part) { out[q++] = 0x08; q += put_varint(out + q, sx32(part)); }
    if (a.lower) { out[q++] = 0x10; q += put_varint(out + q, (uint64_t)a.lower); }
    if (a.upper) { out[q++] = 0x18; q += put_varint(out + q, (uint64_t)a.upper); }
  }
  // buckets: L entries of [0x22, 0x08, LE64]
  for (uint32_t j = lane; j < L; j += 64) {
    uint8_t* e = out + hdr + (uint64_t)j * 10;
    const uint64_t d = dg[min(j, B - 1)];
    e[0] = 0x22;
    e[1] = 0x08;
#pragma unroll
    for (int k = 0; k < 8; k++) e[2 + k] = (uint8_t)(d >> (8 * k));
  }
  uint32_t q = hdr + L * 10;
  // buckets_size: packed varints
  uint32_t plen = 0;
  for (uint32_t j = lane; j < L; j += 64) plen += varint_len(sx32(sz[min(j, B - 1)]));
  for (int o = 32; o > 0; o >>= 1) plen += __shfl_xor(plen, o);
  if (L) {
    if (lane == 0) {
      out[q] = 0x2a;
      put_varint(out + q + 1, plen);
    }
    q += 1 + varint_len(plen);
    uint32_t base = q;
    for (uint32_t j0 = 0; j0 < L; j0 += 64) {
      const uint32_t j = j0 + lane;
      const uint32_t len = j < L ? varint_len(sx32(sz[min(j, B - 1)])) : 0;
      uint32_t incl = len;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o);
        if ((int)lane >= o) incl += x;
      }
      if (j < L) put_varint(out + base + incl - len, sx32(sz[min(j, B - 1)]));
      base += __shfl(incl, 63);
    }
    q += plen;
  }
  if (lane == 0) {
    if (valid) { out[q] = 0x30; out[q + 1] = 0x01; }
    uint32_t t = q + (valid ? 2 : 0);
    if (items) { out[t++] = 0x38; t += put_varint(out + t, sx32(items)); }
    a.out_len[i] = t;
  }
}

// Object i by a whole workgroup of nt threads (a multiple of 64, nt / 64 <= 8 waves; thread t):
// the same bytes as encode_object, with the per-entry work spread over every wave. The one-wave
// form is instruction-latency bound at large B (a dependent chain of shuffles, varint loops and
// ten byte stores per 64 entries: ~13 us at B = 1,000). Uniform: contains barriers. red: >= 16
// words of LDS.
__device__ __forceinline__ void encode_object_block(const WireEncodeLaunch& a, uint32_t i, uint32_t t,
                                                    uint32_t nt, uint32_t* red) {
  const uint32_t B = a.B, L = B + (B & 1u);
  const uint32_t lane = t & 63, wid = t >> 6, nw = nt >> 6;
  const uint64_t* dg = a.digest + (uint64_t)i * B;
  const int32_t* sz = a.size + (uint64_t)i * B;
  uint8_t* out = a.out + (uint64_t)i * a.out_stride;
  const int32_t part = a.partition ? a.partition[i] : 0;
  const bool valid = a.valid && a.valid[i];
  // items (tree.Leafs sum, int32 wrap) and the packed length of buckets_size
  uint32_t acc = 0, plen = 0;
  for (uint32_t j = t; j < L; j += nt) {
    const int32_t v = sz[min(j, B - 1)];
    acc += (uint32_t)v;
    plen += varint_len(sx32(v));
  }
  for (int o = 32; o > 0; o >>= 1) {
    acc += __shfl_xor(acc, o);
    plen += __shfl_xor(plen, o);
  }
  if (lane == 0) {
    red[wid] = acc;
    red[8 + wid] = plen;
  }
  __syncthreads();
  acc = 0;
  plen = 0;
  for (uint32_t w = 0; w < nw; w++) {
    acc += red[w];
    plen += red[8 + w];
  }
  __syncthreads();  // red is reused by the size scan below
  const int32_t items = a.items ? a.items[i] : (int32_t)acc;
  uint32_t hdr = 0;
  if (part) hdr += 1 + varint_len(sx32(part));
  if (a.lower) hdr += 1 + varint_len((uint64_t)a.lower);
  if (a.upper) hdr += 1 + varint_len((uint64_t)a.upper);
  if (t == 0) {
    uint32_t q = 0;
    if (part) { out[q++] = 0x08; q += put_varint(out + q, sx32(part)); }
    if (a.lower) { out[q++] = 0x10; q += put_varint(out + q, (uint64_t)a.lower); }
    if (a.upper) { out[q++] = 0x18; q += put_varint(out + q, (uint64_t)a.upper); }
  }
  for (uint32_t j = t; j < L; j += nt) {
    uint8_t* e = out + hdr + (uint64_t)j * 10;
    const uint64_t d = dg[min(j, B - 1)];
    e[0] = 0x22;
    e[1] = 0x08;
#pragma unroll
    for (int k = 0; k < 8; k++) e[2 + k] = (uint8_t)(d >> (8 * k));
  }
  uint32_t q = hdr + L * 10;
  if (L) {
    if (t == 0) {
      out[q] = 0x2a;
      put_varint(out + q + 1, plen);
    }
    q += 1 + varint_len(plen);
    uint32_t base = q;
    for (uint32_t j0 = 0; j0 < L; j0 += nt) {  // block-wide prefix sum of the varint lengths
      const uint32_t j = j0 + t;
      const int32_t v = j < L ? sz[min(j, B - 1)] : 0;
      const uint32_t len = j < L ? varint_len(sx32(v)) : 0;
      uint32_t incl = len;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o);
        if ((int)lane >= o) incl += x;
      }
      if (lane == 63) red[wid] = incl;
      __syncthreads();
      uint32_t before = 0, tot = 0;
      for (uint32_t w = 0; w < nw; w++) {
        before += w < wid ? red[w] : 0u;
        tot += red[w];
      }
      if (j < L) put_varint(out + base + before + incl - len, sx32(v));
      base += tot;
      __syncthreads();
    }
    q += plen;
  }
  if (t == 0) {
    if (valid) { out[q] = 0x30; out[q + 1] = 0x01; }
    uint32_t e = q + (valid ? 2 : 0);
    if (items) { out[e++] = 0x38; e += put_varint(out + e, sx32(items)); }
    a.out_len[i] = e;
  }
}

// Copy the n bytes at src into LDS at dst + (src & 3) with 4-byte loads (kBatch per lane in flight)
// for the aligned interior and byte loads for the <= 3 + 3 edge bytes; nothing outside
// [src, src + n) is read. One wave; returns the staged copy of src.
template <uint32_t kBatch = 8>
__device__ __forceinline__ const uint8_t* stage_object(const uint8_t* src, uint64_t n, uint8_t* dst, uint32_t lane) {
  const uint64_t s = reinterpret_cast<uint64_t>(src), e = s + n, base = s & ~3ull;
  const uint64_t wa = (s + 3) & ~3ull, wb = e & ~3ull;
  if (wa < wb) {
    const uint32_t nw = (uint32_t)((wb - wa) >> 2);
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(wa);
    uint32_t* lw = reinterpret_cast<uint32_t*>(dst + (wa - base));
    for (uint32_t k0 = 0; k0 < nw; k0 += kBatch * 64) {
      uint32_t v[kBatch];
#pragma unroll
      for (uint32_t u = 0; u < kBatch; u++) {
        const uint32_t k = k0 + u * 64 + lane;
        v[u] = k < nw ? gw[k] : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < kBatch; u++) {
        const uint32_t k = k0 + u * 64 + lane;
        if (k < nw) lw[k] = v[u];
      }
    }
    if (lane < wa - s) dst[s - base + lane] = src[lane];
    if (lane < e - wb) dst[wb - base + lane] = reinterpret_cast<const uint8_t*>(wb)[lane];
  } else {
    for (uint32_t k = lane; k < n; k += 64) dst[s - base + k] = src[k];
  }
  return dst + (s - base);
}

// Decoder cursor. Every lane of the wave holds the same cursor and reads the same bytes (LDS
// broadcast when the object is staged there), so control flow stays wave-uniform and the lanes
// are free for the two runs that dominate an object: the bucket entries and the packed sizes.
struct Cursor {
  const uint8_t* p;
  uint64_t n, pos;
  bool ok;
  // protowire.ConsumeVarint: at most 10 bytes, the 10th 0 or 1 (else errCodeOverflow).
  __device__ __forceinline__ uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 63; s += 7) {
      if (pos >= n) { ok = false; return 0; }
      const uint8_t b = p[pos++];
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    if (pos >= n) { ok = false; return 0; }
    const uint8_t b = p[pos++];
    if (b > 1) { ok = false; return 0; }
    return v | ((uint64_t)b << 63);
  }
  // Advance by len bytes; fails (without wrapping) past the end.
  __device__ __forceinline__ void skip(uint64_t len) {
    if (len > n - pos) { ok = false; return; }
    pos += len;
  }
};

// protowire.consumeFieldValueD for an unknown group (start tag `num` already read): nested
// fields are skipped by wire type until the end tag of the same number; inner tags need a number
// in [1, MaxInt32]. protobuf-go enters a group only while its depth budget
// (protowire.DefaultRecursionLimit = 10,000, one less per level) is >= 0, so up to 10,001 levels
// nest and the 10,002nd fails.
// The open groups' numbers live in gstack, a ring of the kWireGroupDepth deepest levels
// (wave-uniform LDS): level k at gstack[(k - 1) % kWireGroupDepth], valid for levels
// [lo, depth]. Every level's number is also written through to `deep` (level k at deep[k - 1]),
// the object's spill area in global memory (wire_deep_slot: half an entry per object byte, as a
// level takes at least a start and an end tag byte), so an end tag below lo reads its number
// back in one load: the skip stays linear however the depth oscillates (a hostile peer object
// nested past 64 levels that repeatedly dips below the ring and climbs again). Without a spill
// area (an async call whose objects exceed the context's reserved scratch) an end tag below lo
// refills the ring by rescanning the group from its first byte: the last start tag seen at level k
// before the end tag is the open level-k group. Objects nested no deeper than the ring never
// touch either.
constexpr uint32_t kWireGroupDepth = 64;
constexpr uint32_t kWireGroupMaxNest = 10001;
__device__ __forceinline__ void group_refill(const Cursor& c, uint64_t start, uint64_t stop, uint32_t depth,
                                             uint32_t num, uint32_t* gstack) {
  const uint32_t lo = depth > kWireGroupDepth ? depth - kWireGroupDepth + 1 : 1u;
  if (lo == 1) gstack[0] = num;  // level 1's start tag precedes `start`
  // bytes [start, stop) were parsed once (well formed); the last is the end tag being matched,
  // which only lowers d
  Cursor r{c.p, stop, start, true};
  uint32_t d = 1;
  while (r.pos < stop) {
    const uint64_t key = r.varint();
    const uint32_t w = (uint32_t)(key & 7);
    if (w == 3) {
      if (++d >= lo && d <= depth) gstack[(d - 1) % kWireGroupDepth] = (uint32_t)(key >> 3);
    } else if (w == 4) {
      d--;
    } else if (w == 0) {
      r.varint();
    } else if (w == 1) {
      r.pos += 8;
    } else if (w == 5) {
      r.pos += 4;
    } else {
      const uint64_t len = r.varint();
      r.pos += len;
    }
  }
}

// The spill area's reads and writes are lane 0's vector memory operations (relaxed atomics:
// read-your-writes within the lane), broadcast to the wave.
// A level deeper than half the object's bytes can never be closed (each open level still needs
// an end tag byte), so such an object fails whatever happens next: levels past the area's
// n / 2 + 1 entries are not spilled, and an end tag for one of them fails the object at once.
__device__ __forceinline__ void deep_put(uint32_t* deep, uint32_t levels, uint32_t level, uint32_t v, uint32_t lane) {
  if (deep && level <= levels && lane == 0)
    __hip_atomic_store(deep + (level - 1), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t deep_get(uint32_t* deep, uint32_t level, uint32_t lane) {
  uint32_t v = 0;
  if (lane == 0) v = __hip_atomic_load(deep + (level - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint32_t)__shfl((int)v, 0);
}

__device__ __forceinline__ void skip_group(Cursor& c, uint64_t num, uint32_t* gstack, uint32_t* deep, uint32_t lane) {
  const uint64_t start = c.pos;  // first byte inside the outermost group (level 1)
  const uint32_t levels = (uint32_t)min<uint64_t>(c.n / 2 + 1, kWireGroupMaxNest);  // spilled levels
  uint32_t depth = 1, lo = 1;    // invariant: lo <= depth + 1 (lo = depth + 1: no ring level valid)
  gstack[0] = (uint32_t)num;
  deep_put(deep, levels, 1, (uint32_t)num, lane);
  while (c.ok) {
    const uint64_t key = c.varint();
    if (!c.ok) return;
    const uint64_t n2 = key >> 3;
    const uint32_t w = (uint32_t)(key & 7);
    if (n2 < 1 || n2 > 0x7FFFFFFFull) { c.ok = false; return; }
    if (w == 4) {
      uint32_t open;
      if (depth >= lo) {
        open = gstack[(depth - 1) % kWireGroupDepth];
      } else if (deep) {  // this level's number left the ring: read it back from the spill area
        if (depth > levels) { c.ok = false; return; }  // unclosable (see deep_put)
        open = deep_get(deep, depth, lane);
        lo = depth;  // after the pop below, the ring holds no level
      } else {  // no spill area: rescan up to this end tag
        group_refill(c, start, c.pos, depth, (uint32_t)num, gstack);
        lo = depth > kWireGroupDepth ? depth - kWireGroupDepth + 1 : 1u;
        open = gstack[(depth - 1) % kWireGroupDepth];
      }
      if ((uint32_t)n2 != open) { c.ok = false; return; }
      if (--depth == 0) return;
      continue;
    }
    if (w == 3) {
      if (depth == kWireGroupMaxNest) { c.ok = false; return; }  // errCodeRecursion
      gstack[depth++ % kWireGroupDepth] = (uint32_t)n2;
      deep_put(deep, levels, depth, (uint32_t)n2, lane);
      if (depth - lo >= kWireGroupDepth) lo = depth - kWireGroupDepth + 1;
      continue;
    }
    if (w == 0) { c.varint(); continue; }
    if (w == 1) { c.skip(8); continue; }
    if (w == 5) { c.skip(4); continue; }
    if (w == 2) { const uint64_t len = c.varint(); if (c.ok) c.skip(len); continue; }
    c.ok = false;  // reserved wire types 6, 7
  }
}

// Object i's spill area in a.deep (entries [(off[i] - off[0]) / 2 + i, + n / 2 + 1): disjoint per
// object, n / 2 + 1 entries >= its deepest level), or nullptr when a.deep does not cover it.
__device__ __forceinline__ uint32_t* wire_deep_slot(const WireDecodeLaunch& a, uint32_t i, uint64_t n) {
  if (!a.deep) return nullptr;
  const uint64_t base = (a.off[i] - a.off[0]) / 2 + i;
  return base + n / 2 + 1 <= a.deep_cap ? a.deep + base : nullptr;
}

// Object i by ALL 64 lanes of one wave (lane = 0..63), parsing the n bytes at p (the object in
// a.bytes, or a copy staged in LDS). Same results as a one-field-at-a-time walk:
//   * a run of canonical bucket entries [0x22 0x08 LE64] is checked and extracted 64 x kWin
//     entries at a time (kWin per lane; ballots: the run ends at the first entry that is not
//     canonical, which then goes through the generic path); entries past cap are counted, not
//     stored, and the object then fails with MDE_E_CAPACITY unless it has a decode error;
//   * a packed sizes run is split at its varint terminators 64 bytes at a time (ballot; element
//     index = terminators before it); a varint longer than 10 bytes, with a 10th byte above 1, or
//     crossing the run's end is a decode error, as it is for the serial walk.
// Errors follow protobuf-go v1.30's proto.Unmarshal (main/go.mod:15; the restatement is
// oracle/wire_pb.py unmarshal): varint overflow, field numbers outside [1, 2^29-1], truncation,
// stray end groups, reserved wire types. Unknown fields are skipped, groups included.
template <uint32_t kWin = 1>
__device__ __forceinline__ void decode_object(const WireDecodeLaunch& a, uint32_t i, const uint8_t* p, uint64_t n,
                                              uint32_t lane, uint32_t* gstack) {
  Cursor c{p, n, 0, true};
  int32_t part = 0, items = 0;
  int64_t lower = 0, upper = 0;
  uint8_t valid = 0;
  uint32_t nb = 0, ns = 0;
  int32_t err = 0;
  const uint32_t cap = a.cap;
  uint64_t* dg = a.digest + (uint64_t)i * cap;
  int32_t* sz = a.size + (uint64_t)i * cap;
  while (c.ok && c.pos < c.n && !err) {
    if (c.p[c.pos] == 0x22 && c.n - c.pos >= 10 && c.p[c.pos + 1] == 0x08) {
      bool good[kWin];
#pragma unroll
      for (uint32_t u = 0; u < kWin; u++) {
        const uint64_t q = c.pos + 10ull * (u * 64 + lane);
        good[u] = q + 10 <= c.n && c.p[q] == 0x22 && c.p[q + 1] == 0x08;
      }
      uint32_t run = 0;  // >= 1: the first entry is canonical
#pragma unroll
      for (uint32_t u = 0; u < kWin; u++) {
        const uint64_t bad = ~__ballot(good[u]);
        if (bad) {
          run = u * 64 + (uint32_t)__builtin_ctzll(bad);
          break;
        }
        run = (u + 1) * 64;
      }
#pragma unroll
      for (uint32_t u = 0; u < kWin; u++) {
        const uint32_t e = u * 64 + lane;
        if (e < run && nb + e < cap) {
          const uint64_t q = c.pos + 10ull * e;
          uint64_t v = 0;
#pragma unroll
          for (int k = 7; k >= 0; k--) v = (v << 8) | c.p[q + 2 + k];
          dg[nb + e] = v;
        }
      }
      nb += run;
      c.pos += 10ull * run;
      continue;
    }
    const uint64_t key = c.varint();
    if (!c.ok) break;
    if ((key >> 3) < 1 || (key >> 3) > 0x1FFFFFFFull) { c.ok = false; break; }  // MaxValidNumber
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (field == 1 && wt == 0) { part = (int32_t)c.varint(); continue; }
    if (field == 2 && wt == 0) { lower = (int64_t)c.varint(); continue; }
    if (field == 3 && wt == 0) { upper = (int64_t)c.varint(); continue; }
    if (field == 6 && wt == 0) { valid = c.varint() != 0; continue; }
    if (field == 7 && wt == 0) { items = (int32_t)c.varint(); continue; }
    if (field == 4 && wt == 2) {  // a non-canonical entry (e.g. a length other than 8)
      const uint64_t len = c.varint();
      if (!c.ok || len > c.n - c.pos) { c.ok = false; break; }
      if (len != 8) { err = -6; break; }  // DecodeBytesToInt64 (utils/utils.go:80-82)
      if (nb < cap) {
        uint64_t v = 0;
        for (int k = 7; k >= 0; k--) v = (v << 8) | c.p[c.pos + k];
        if (lane == 0) dg[nb] = v;
      }
      nb++;
      c.pos += len;
      continue;
    }
    if (field == 5 && wt == 2) {  // packed
      const uint64_t len = c.varint();
      if (!c.ok || len > c.n - c.pos) { c.ok = false; break; }
      const uint64_t end = c.pos + len;
      if (kWin > 1) {  // 64 x kWin bytes per step; byte e = 64u + lane of the window
        while (c.pos < end) {
          uint8_t bv[kWin];
          uint64_t T[kWin];
          uint32_t last = 0, any = 0;
#pragma unroll
          for (uint32_t u = 0; u < kWin; u++) {
            const uint64_t q = c.pos + u * 64 + lane;
            bv[u] = q < end ? c.p[q] : (uint8_t)0x80;
            T[u] = __ballot(!(bv[u] & 0x80));
            if (T[u]) {
              last = u * 64 + 63 - (uint32_t)__builtin_clzll(T[u]);
              any = 1;
            }
          }
          if (!any) { c.ok = false; break; }  // > 64 x kWin bytes, or crosses the run's end
          bool too_long = false;
          uint32_t prev_end = 0, cnt = 0;  // (last terminator before word u) + 1; terminators before it
#pragma unroll
          for (uint32_t u = 0; u < kWin; u++) {
            const uint32_t e = u * 64 + lane;
            const bool term = !(bv[u] & 0x80);
            const uint64_t below = T[u] & ((1ull << lane) - 1ull);
            const uint32_t start = below ? u * 64 + 64u - (uint32_t)__builtin_clzll(below) : prev_end;
            too_long |= term && (e - start >= 10u || (e - start == 9u && bv[u] > 1));
            if (term && !too_long) {
              uint64_t v = 0;
              for (uint32_t k = start; k <= e; k++) v |= (uint64_t)(c.p[c.pos + k] & 0x7f) << (7 * (k - start));
              const uint32_t idx = ns + cnt + (uint32_t)__popcll(below);
              if (idx < cap) sz[idx] = (int32_t)v;
            }
            if (T[u]) prev_end = u * 64 + 64u - (uint32_t)__builtin_clzll(T[u]);
            cnt += (uint32_t)__popcll(T[u]);
          }
          // an object with an over-long varint fails whole; the sizes written before it are
          // scratch that no caller reads for a failed object
          if (__ballot(too_long)) { c.ok = false; break; }
          ns += cnt;
          c.pos += last + 1;
        }
        continue;
      }
      while (c.pos < end) {
        const uint64_t q = c.pos + lane;
        const uint8_t b = q < end ? c.p[q] : (uint8_t)0x80;
        const bool term = !(b & 0x80);
        const uint64_t T = __ballot(term);
        if (!T) { c.ok = false; break; }  // > 64 bytes, or crosses the run's end
        const uint64_t below = T & ((1ull << lane) - 1ull);
        const uint32_t start = below ? 64u - (uint32_t)__builtin_clzll(below) : 0u;
        const bool too_long = term && (lane - start >= 10u || (lane - start == 9u && b > 1));
        if (__ballot(too_long)) { c.ok = false; break; }
        if (term) {
          uint64_t v = 0;
          for (uint32_t k = start; k <= lane; k++) v |= (uint64_t)(c.p[c.pos + k] & 0x7f) << (7 * (k - start));
          const uint32_t idx = ns + (uint32_t)__popcll(below);
          if (idx < cap) sz[idx] = (int32_t)v;
        }
        ns += (uint32_t)__popcll(T);
        c.pos += 64u - (uint32_t)__builtin_clzll(T);
      }
      continue;
    }
    if (field == 5 && wt == 0) {  // unpacked element (parsers must accept both)
      const int32_t v = (int32_t)c.varint();
      if (lane == 0 && ns < cap) sz[ns] = v;
      ns++;
      continue;
    }
    // unknown field: skip by wire type
    if (wt == 0) { c.varint(); continue; }
    if (wt == 1) { c.skip(8); continue; }
    if (wt == 5) { c.skip(4); continue; }
    if (wt == 2) { const uint64_t len = c.varint(); if (c.ok) c.skip(len); continue; }
    if (wt == 3) { skip_group(c, key >> 3, gstack, wire_deep_slot(a, i, n), lane); continue; }
    c.ok = false;  // a stray end group, reserved wire types 6, 7
  }
  if (!c.ok && !err) err = -6;
  // More buckets than fit: reported only for an object Go would unmarshal (a later wire error
  // makes the whole object a decode error), after the scan that checked the rest of it.
  if (!err && nb > cap) err = -5;
  // sizes default to 0 when BucketsSize is shorter (main/merkle_tree.go:147-152)
  for (uint32_t j = ns + lane; j < nb && j < cap; j += 64) sz[j] = 0;
  if (lane == 0) {
    if (a.partition) a.partition[i] = part;
    if (a.lower) a.lower[i] = lower;
    if (a.upper) a.upper[i] = upper;
    if (a.valid) a.valid[i] = valid;
    if (a.items) a.items[i] = items;
    a.n_buckets[i] = err ? err : (int32_t)nb;
  }
}

}  // namespace mde
