// tag.hip -- write-time key tagging and the synthetic workload generator (device side).
//
// Tagging: the reference computes, per written key,
//   bucket    = BE64(SHA256(key)[0:8]) % PartitionBuckets   (Manager.getKeyBucket, main/manager.go:773-778)
//   partition = XXH64(key, seed 0) % PartitionCount          (Hashring.FindPartitionID,
//               hashring/hashring.go:89-93,108-110 -> buraksezer/consistent v0.10.0)
// and bakes both into the epoch index key (main/indexs.go:13-20), which fixes the bucket a record
// is summed into. One thread per key; integer/bit work only.
//
// Synthetic workload: key(gid) = "k%016x" % gid (17 bytes);
// value word w of record gid = splitmix64(seed ^ (gid * 2^20 + w)), stored little-endian.
#include "mde_device.hpp"
#include "mde_internal.hpp"

namespace mde {
namespace {

constexpr int kThreads = 256;

// SHA-256 of key bytes [p, p+len) read from global memory -> first 8 digest bytes, big-endian.
__device__ uint64_t sha256_prefix64(const uint8_t* p, uint64_t len) {
  uint32_t st[8];
  sha256_init(st);
  const uint64_t nblk = (len + 9 + 63) / 64;
  for (uint64_t blk = 0; blk < nblk; blk++) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
      uint32_t word = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint64_t pos = blk * 64 + 4 * t + k;
        const uint32_t byte = pos < len ? p[pos] : (pos == len ? 0x80u : 0u);
        word = (word << 8) | byte;
      }
      w[t] = word;
    }
    if (blk == nblk - 1) {
      w[14] = (uint32_t)((len * 8) >> 32);
      w[15] = (uint32_t)(len * 8);
    }
    sha256_compress(st, w);
  }
  return ((uint64_t)st[0] << 32) | st[1];
}

__device__ __forceinline__ uint64_t rd64le(const uint8_t* p) {
  uint64_t v = 0;
#pragma unroll
  for (int k = 7; k >= 0; k--) v = (v << 8) | p[k];
  return v;
}

__device__ uint64_t xxh64(const uint8_t* p, uint64_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xx_round(v1, rd64le(p));
      v2 = xx_round(v2, rd64le(p + 8));
      v3 = xx_round(v3, rd64le(p + 16));
      v4 = xx_round(v4, rd64le(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xx_merge(h, v1); h = xx_merge(h, v2); h = xx_merge(h, v3); h = xx_merge(h, v4);
  } else {
    h = seed + XP5;
  }
  h += len;
  while (p + 8 <= end) { h ^= xx_round(0, rd64le(p)); h = rotl64(h, 27) * XP1 + XP4; p += 8; }
  if (p + 4 <= end) {
    const uint32_t v = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    h ^= (uint64_t)v * XP1;
    h = rotl64(h, 23) * XP2 + XP3;
    p += 4;
  }
  while (p < end) { h ^= (*p) * XP5; h = rotl64(h, 11) * XP1; p++; }
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
  return h;
}

__global__ __launch_bounds__(kThreads) void tag_keys_kernel(const uint8_t* keys, const uint64_t* key_off,
                                                            uint64_t n, uint32_t B, uint32_t P,
                                                            uint32_t* bucket, uint32_t* partition) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kThreads) {
    const uint8_t* k = keys + key_off[i];
    const uint64_t len = key_off[i + 1] - key_off[i];
    if (bucket) bucket[i] = (uint32_t)(sha256_prefix64(k, len) % B);
    if (partition) partition[i] = (uint32_t)(xxh64(k, len, 0) % P);
  }
}

// "k%016x" % gid as big-endian SHA words + the XXH64 of those 17 bytes.
__device__ __forceinline__ uint32_t hexc(uint64_t gid, int nib) {  // nib 0 = most significant
  const uint32_t v = (uint32_t)(gid >> (60 - 4 * nib)) & 15u;
  return v < 10 ? 0x30u + v : 0x57u + v;
}

__global__ __launch_bounds__(kThreads) void synth_tags_kernel(const uint64_t* gids, uint64_t n, uint32_t P,
                                                              uint32_t B, int mode, uint64_t kpp,
                                                              uint32_t* part, uint32_t* bucket) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kThreads) {
    const uint64_t gid = gids[i];
    uint32_t c[20];
    c[0] = 0x6bu;  // 'k'
#pragma unroll
    for (int j = 0; j < 16; j++) c[1 + j] = hexc(gid, j);
    c[17] = 0x80u;
    c[18] = 0u;
    c[19] = 0u;
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 5; t++) w[t] = (c[4 * t] << 24) | (c[4 * t + 1] << 16) | (c[4 * t + 2] << 8) | c[4 * t + 3];
#pragma unroll
    for (int t = 5; t < 15; t++) w[t] = 0u;
    w[15] = 17u * 8u;
    uint32_t st[8];
    sha256_init(st);
    sha256_compress(st, w);
    bucket[i] = (uint32_t)((((uint64_t)st[0] << 32) | st[1]) % B);
    uint32_t pid;
    if (mode == 0) {
      pid = (uint32_t)(gid / kpp);
    } else if (mode == 1) {
      pid = (uint32_t)(gid % P);
    } else {
      uint64_t lo = 0, hi = 0;
#pragma unroll
      for (int k = 7; k >= 0; k--) { lo = (lo << 8) | c[k]; hi = (hi << 8) | c[8 + k]; }
      uint64_t h = XP5 + 17u;
      h ^= xx_round(0, lo); h = rotl64(h, 27) * XP1 + XP4;
      h ^= xx_round(0, hi); h = rotl64(h, 27) * XP1 + XP4;
      h ^= (uint64_t)c[16] * XP5; h = rotl64(h, 11) * XP1;
      h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
      pid = (uint32_t)(h % P);
    }
    part[i] = pid;
  }
}

__global__ __launch_bounds__(kThreads) void synth_values_kernel(uint8_t* dst, const uint64_t* gids, uint64_t n,
                                                                uint32_t len, uint64_t seed) {
  const uint64_t words = (len + 7) / 8;
  const uint64_t total = n * words;
  for (uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * kThreads) {
    const uint64_t i = t / words, w = t - i * words;
    const uint64_t x = splitmix64(seed ^ ((gids[i] << 20) + w));
    uint8_t* o = dst + i * len + w * 8;
    if ((len & 7u) == 0 && (((uintptr_t)dst) & 7u) == 0) {
      *reinterpret_cast<uint64_t*>(o) = x;
    } else {
      const uint32_t nb = (uint32_t)min<uint64_t>(8, len - w * 8);
      for (uint32_t k = 0; k < nb; k++) o[k] = (uint8_t)(x >> (8 * k));
    }
  }
}

uint32_t grid_for(uint64_t work) {
  uint64_t g = (work + kThreads - 1) / kThreads;
  if (g > 65536) g = 65536;
  return (uint32_t)(g ? g : 1);
}

}  // namespace

hipError_t launch_tag_keys(const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint32_t B,
                           uint32_t P, uint32_t* bucket, uint32_t* partition, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(tag_keys_kernel, dim3(grid_for(n)), dim3(kThreads), 0, st, keys, key_off, n,
                     B, P, bucket, partition);
  return hipGetLastError();
}

hipError_t launch_synth_tags(const uint64_t* gids, uint64_t n, uint32_t P, uint32_t B, int mode,
                             uint64_t kpp, uint32_t* part, uint32_t* bucket, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(synth_tags_kernel, dim3(grid_for(n)), dim3(kThreads), 0, st, gids, n, P, B,
                     mode, kpp, part, bucket);
  return hipGetLastError();
}

hipError_t launch_synth_values(uint8_t* dst, const uint64_t* gids, uint64_t n, uint32_t len,
                               uint64_t seed, hipStream_t st) {
  if (n == 0 || len == 0) return hipSuccess;
  hipLaunchKernelGGL(synth_values_kernel, dim3(grid_for(n * ((len + 7) / 8))), dim3(kThreads), 0,
                     st, dst, gids, n, len, seed);
  return hipGetLastError();
}

}  // namespace mde
