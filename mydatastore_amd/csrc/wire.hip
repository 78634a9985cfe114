// wire.hip -- EpochTreeObject protobuf wire bytes on device.
//
// Reference: VerifyEpoch persists and serves proto.Marshal(MerkleTreeToPartitionEpochObject(...))
// (main/manager.go:1041-1056, rpc/server.go:170-187) and peers decode it back into a tree
// (EpochTreeObjectToMerkleTree, main/merkle_tree.go:140-157). Message (datap/data.proto:60-68):
//   1 int32 partition | 2 int64 lower_epoch | 3 int64 upper_epoch | 4 repeated bytes buckets
//   5 repeated int32 buckets_size (packed) | 6 bool valid | 7 int32 items
// proto3 encoding as protobuf-go emits it: fields in number order, zero scalars omitted, each
// bucket a length-delimited 8-byte LE64 digest, sizes one packed run of varints, negative int32
// sign-extended to a 10-byte varint. Leaves follow tree.Leafs: an odd B repeats the last bucket.
//
// Encode: one wave per object, lanes write the 10-byte bucket entries and the size varints at
// offsets from a wave prefix sum. Decode: one wave per object, lane 0 parses (varint walk) --
// objects are ~1 KiB, the parallelism is across objects.
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {
namespace {

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

__global__ __launch_bounds__(64) void encode_kernel(WireEncodeLaunch a) {
  const uint32_t i = blockIdx.x, lane = threadIdx.x;
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

struct Cursor {
  const uint8_t* p;
  uint64_t n, pos;
  bool ok;
  __device__ uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (pos >= n) { ok = false; return 0; }
      const uint8_t b = p[pos++];
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    ok = false;
    return 0;
  }
};

__global__ __launch_bounds__(64) void decode_kernel(WireDecodeLaunch a) {
  const uint32_t i = blockIdx.x;
  if (threadIdx.x != 0) return;
  Cursor c{a.bytes + a.off[i], a.off[i + 1] - a.off[i], 0, true};
  int32_t part = 0, items = 0;
  int64_t lower = 0, upper = 0;
  uint8_t valid = 0;
  uint32_t nb = 0, ns = 0;
  int32_t err = 0;
  uint64_t* dg = a.digest + (uint64_t)i * a.cap;
  int32_t* sz = a.size + (uint64_t)i * a.cap;
  while (c.ok && c.pos < c.n && !err) {
    const uint64_t key = c.varint();
    if (!c.ok) break;
    const uint32_t field = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (field == 1 && wt == 0) { part = (int32_t)c.varint(); continue; }
    if (field == 2 && wt == 0) { lower = (int64_t)c.varint(); continue; }
    if (field == 3 && wt == 0) { upper = (int64_t)c.varint(); continue; }
    if (field == 6 && wt == 0) { valid = c.varint() != 0; continue; }
    if (field == 7 && wt == 0) { items = (int32_t)c.varint(); continue; }
    if (field == 4 && wt == 2) {
      const uint64_t len = c.varint();
      if (!c.ok || c.pos + len > c.n) { c.ok = false; break; }
      if (len != 8) { err = -6; break; }  // DecodeBytesToInt64 (utils/utils.go:80-82)
      if (nb >= a.cap) { err = -5; break; }
      uint64_t v = 0;
      for (int k = 7; k >= 0; k--) v = (v << 8) | c.p[c.pos + k];
      dg[nb++] = v;
      c.pos += len;
      continue;
    }
    if (field == 5 && wt == 2) {  // packed
      const uint64_t len = c.varint();
      if (!c.ok || c.pos + len > c.n) { c.ok = false; break; }
      const uint64_t end = c.pos + len;
      while (c.ok && c.pos < end) {
        const int32_t v = (int32_t)c.varint();
        if (ns < a.cap) sz[ns] = v;
        ns++;
      }
      if (c.pos != end) c.ok = false;
      continue;
    }
    if (field == 5 && wt == 0) {  // unpacked element (parsers must accept both)
      const int32_t v = (int32_t)c.varint();
      if (ns < a.cap) sz[ns] = v;
      ns++;
      continue;
    }
    // unknown field: skip by wire type
    if (wt == 0) { c.varint(); continue; }
    if (wt == 1) { c.pos += 8; if (c.pos > c.n) c.ok = false; continue; }
    if (wt == 5) { c.pos += 4; if (c.pos > c.n) c.ok = false; continue; }
    if (wt == 2) { const uint64_t len = c.varint(); c.pos += len; if (c.pos > c.n) c.ok = false; continue; }
    c.ok = false;
  }
  if (!c.ok && !err) err = -6;
  // sizes default to 0 when BucketsSize is shorter (main/merkle_tree.go:147-152)
  for (uint32_t j = ns; j < nb && j < a.cap; j++) sz[j] = 0;
  if (a.partition) a.partition[i] = part;
  if (a.lower) a.lower[i] = lower;
  if (a.upper) a.upper[i] = upper;
  if (a.valid) a.valid[i] = valid;
  if (a.items) a.items[i] = items;
  a.n_buckets[i] = err ? err : (int32_t)nb;
}

}  // namespace

hipError_t launch_wire_encode(const WireEncodeLaunch& a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(encode_kernel, dim3(a.n), dim3(64), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_wire_decode(const WireDecodeLaunch& a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(decode_kernel, dim3(a.n), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace mde
