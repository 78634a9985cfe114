// mde_device.hpp -- device-side primitives shared by the gfx950 kernels.
//
// SHA-256 (FIPS 180-4) specialised for the three message shapes the Merkle path hashes:
//   * level-1 nodes: SHA256(LE64(d_l) || LE64(d_r)) -- one 16-byte message, one block
//     (leaf bytes: MerkleBucket.CalculateHash, main/merkle_tree.go:64-71 -> utils/utils.go:67-74);
//   * upper nodes:   SHA256(h_l || h_r) -- 64-byte message, data block + constant padding block
//     (cbergoon/merkletree v0.2.0 buildIntermediate);
//   * keys:          SHA256(key) of any length (getKeyBucket, main/manager.go:773-778).
// Integer/bit operations only (v_alignbit for rotates, v_perm for byte swaps) -- no MFMA.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mde {

// CustomHash modulus, main/merkle_tree.go:19.
constexpr uint64_t kHashMod = 999999ull;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr uint32_t kSha256K(int i) {
  constexpr uint32_t K[64] = {
      0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
      0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
      0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
      0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
      0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
      0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
      0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
      0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
      0xc67178f2};
  return K[i];
}

__host__ __device__ constexpr uint32_t c_ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// Message schedule of the constant padding block of a 64-byte message
// (W0 = 0x80000000, W1..W14 = 0, W15 = 512 bits), pre-added to K: KW[i] = K[i] + W[i].
struct PadSchedule {
  uint32_t kw[64];
  constexpr PadSchedule() : kw() {
    uint32_t w[64] = {};
    w[0] = 0x80000000u;
    w[15] = 512u;
    for (int i = 16; i < 64; i++) {
      uint32_t s0 = c_ror(w[i - 15], 7) ^ c_ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      uint32_t s1 = c_ror(w[i - 2], 17) ^ c_ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    for (int i = 0; i < 64; i++) kw[i] = kSha256K(i) + w[i];
  }
};

__device__ __forceinline__ uint32_t ror(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void sha256_init(uint32_t st[8]) {
  st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
  st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

// gfx950 v_bitop3_b32: any 3-input boolean function in one instruction. Truth-table immediates
// for inputs (a, b, c) = (0xF0, 0xCC, 0xAA): xor3 = 0x96, ch = a ? b : c = 0xCA, maj = 0xE8.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
  return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

#define MDE_SHA_ROUND(a, b, c, d, e, f, g, h, kw)                                       \
  do {                                                                                \
    uint32_t t1_ = (h) + (kw) + ch((e), (f), (g)) + xor3(ror((e), 6), ror((e), 11), ror((e), 25)); \
    uint32_t t2_ = xor3(ror((a), 2), ror((a), 13), ror((a), 22)) + maj((a), (b), (c));  \
    (d) += t1_;                                                                       \
    (h) = t1_ + t2_;                                                                  \
  } while (0)

// Round constants in constant memory; the round loops index them with a wave-uniform counter,
// so they are read with scalar loads (one s_load_dwordx16 per 16 rounds).
__device__ static constexpr uint32_t kK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
__device__ static constexpr PadSchedule kPad{};

#define MDE_SHA_8ROUNDS(KW)                                \
  MDE_SHA_ROUND(a, b, c, d, e, f, g, h, KW(0));            \
  MDE_SHA_ROUND(h, a, b, c, d, e, f, g, KW(1));            \
  MDE_SHA_ROUND(g, h, a, b, c, d, e, f, KW(2));            \
  MDE_SHA_ROUND(f, g, h, a, b, c, d, e, KW(3));            \
  MDE_SHA_ROUND(e, f, g, h, a, b, c, d, KW(4));            \
  MDE_SHA_ROUND(d, e, f, g, h, a, b, c, KW(5));            \
  MDE_SHA_ROUND(c, d, e, f, g, h, a, b, KW(6));            \
  MDE_SHA_ROUND(b, c, d, e, f, g, h, a, KW(7))

__device__ __forceinline__ void sha_sched16(uint32_t w[16]) {
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t x15 = w[(j + 1) & 15], x2 = w[(j + 14) & 15];
    w[j] += xor3(ror(x15, 7), ror(x15, 18), x15 >> 3) + w[(j + 9) & 15] +
            xor3(ror(x2, 17), ror(x2, 19), x2 >> 10);
  }
}

// One compression of a 16-word big-endian message block (w is clobbered). Compact form: a loop of
// four 16-round bodies (the schedule for rounds 16..63 is computed 16 words at a time), which keeps
// the code ~6x smaller than a full unroll -- several trees in flight on one CU no longer thrash the
// instruction cache.
__device__ __forceinline__ void sha256_compress(uint32_t st[8], uint32_t w[16]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int i = 0; i < 64; i += 16) {
    if (i) sha_sched16(w);
#define MDE_KW_LO(j) (kK[i + (j)] + w[(j)])
#define MDE_KW_HI(j) (kK[i + 8 + (j)] + w[8 + (j)])
    MDE_SHA_8ROUNDS(MDE_KW_LO);
    MDE_SHA_8ROUNDS(MDE_KW_HI);
#undef MDE_KW_LO
#undef MDE_KW_HI
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// Compression of the constant padding block of a 64-byte message (schedule folded into KW).
__device__ __forceinline__ void sha256_compress_pad64(uint32_t st[8]) {
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll 1
  for (int i = 0; i < 64; i += 8) {
#define MDE_KW_PAD(j) (kPad.kw[i + (j)])
    MDE_SHA_8ROUNDS(MDE_KW_PAD);
#undef MDE_KW_PAD
  }
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// ---- Two-lane padding block (latency form) ----
// A lane pair (even lane "E" = the e..h chain, odd lane "A" = the a..d chain) runs one padding-
// block compression with 11 instructions per round instead of 14: both chains' big sigma and
// Ch / Maj come from the same instructions (per-lane rotate amounts; Maj(a,b,c) = Ch(~(a^b), b, c)),
// and two DPP quad permutes exchange T1 and d. Per round, with P = Sigma + Ch|Maj + KW (A: KW = 0):
//   E: Q = P + h = T1;  A: P = T2;  new e = T1 + d (d: the A lane's x3),  new a = T1 + T2.
// v: this lane's four state words (E: st[4..7], A: st[0..3]) in, its four hash words out.
#define MDE_SHA2_ROUND(a, b, c, d, kw)                                                            \
  do {                                                                                            \
    const uint32_t dd_ = (uint32_t)__builtin_amdgcn_mov_dpp((int)(d), 0xF5, 0xF, 0xF, true);      \
    const uint32_t s_ = xor3(__builtin_amdgcn_alignbit((a), (a), r1), __builtin_amdgcn_alignbit((a), (a), r2), \
                             __builtin_amdgcn_alignbit((a), (a), r3));                             \
    const uint32_t f_ = ch(__builtin_amdgcn_bitop3_b32((a), (b), m, 0xD2), (b), (c));             \
    const uint32_t p_ = s_ + f_ + (kw);                                                           \
    const uint32_t q_ = p_ + (d);                                                                 \
    const uint32_t r_ = is_a ? p_ : dd_;                                                          \
    (d) = (uint32_t)__builtin_amdgcn_mov_dpp((int)q_, 0xA0, 0xF, 0xF, true) + r_;                 \
  } while (0)
#define MDE_SHA2_4ROUNDS(KW)                 \
  MDE_SHA2_ROUND(x0, x1, x2, x3, KW(0));     \
  MDE_SHA2_ROUND(x3, x0, x1, x2, KW(1));     \
  MDE_SHA2_ROUND(x2, x3, x0, x1, KW(2));     \
  MDE_SHA2_ROUND(x1, x2, x3, x0, KW(3))

__device__ __forceinline__ void sha256_pad64_pair(uint32_t v[4], bool is_a) {
  const uint32_t r1 = is_a ? 2u : 6u, r2 = is_a ? 13u : 11u, r3 = is_a ? 22u : 25u, m = is_a ? ~0u : 0u;
  uint32_t me = ~m;  // E lanes add the round constant, A lanes add 0 (one v_and per round)
  asm volatile("" : "+v"(me));  // keep the AND: a known select costs a v_mov + v_cndmask
  uint32_t x0 = v[0], x1 = v[1], x2 = v[2], x3 = v[3];
#pragma unroll 1
  for (int i = 0; i < 64; i += 8) {
#define MDE_KW_PAD2(j) (kPad.kw[i + (j)] & me)
#define MDE_KW_PAD2B(j) (kPad.kw[i + 4 + (j)] & me)
    MDE_SHA2_4ROUNDS(MDE_KW_PAD2);
    MDE_SHA2_4ROUNDS(MDE_KW_PAD2B);
#undef MDE_KW_PAD2
#undef MDE_KW_PAD2B
  }
  v[0] += x0; v[1] += x1; v[2] += x2; v[3] += x3;
}

// ---- Split-schedule node hash (latency form, tree_body_duo) ----
// One wave issues at most one VALU instruction per ~4.6 cycles, so a lone dependent chain costs its
// instruction count: the data block of SHA256(hl || hr) is 64 rounds of ~15 instructions plus 48
// schedule words of ~10. Here a compute thread runs only the rounds; its mirror thread, in another
// wave of the workgroup, computes W16..63 (pre-added to K) and hands them over through LDS in three
// 16-word chunks, each published behind a workgroup barrier four rounds before the compute thread
// needs it (the LDS read latency hides under those four rounds). Both sides execute exactly three
// barriers per node, so every wave of the workgroup must call one side or the other the same
// number of times. kw: this thread's slot of a [8][stride] u32x4 ring of two chunks (chunk c of 16
// words = slots 4 (c % 2) .. +3): the helper writes chunk c + 2 only after the barrier that
// follows the compute side's reads of chunk c (a barrier waits for the wave's LDS reads).
#define MDE_SHA_4A(KW)                                     \
  MDE_SHA_ROUND(a, b, c, d, e, f, g, h, KW(0));            \
  MDE_SHA_ROUND(h, a, b, c, d, e, f, g, KW(1));            \
  MDE_SHA_ROUND(g, h, a, b, c, d, e, f, KW(2));            \
  MDE_SHA_ROUND(f, g, h, a, b, c, d, e, KW(3))
#define MDE_SHA_4B(KW)                                     \
  MDE_SHA_ROUND(e, f, g, h, a, b, c, d, KW(0));            \
  MDE_SHA_ROUND(d, e, f, g, h, a, b, c, KW(1));            \
  MDE_SHA_ROUND(c, d, e, f, g, h, a, b, KW(2));            \
  MDE_SHA_ROUND(b, c, d, e, f, g, h, a, KW(3))

// kPair: the node's lane pair runs the data block redundantly, then the padding block in the
// two-lane form; st[0..3] then holds this lane's four hash words (A: words 0..3, E: 4..7).
template <bool kPair = false>
__device__ __forceinline__ void sha256_node_duo_main(const uint32_t hl[8], const uint32_t hr[8], uint32_t st[8],
                                                     const u32x4* kw, uint32_t stride, bool is_a = false) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { w[i] = hl[i]; w[8 + i] = hr[i]; }
  sha256_init(st);
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#define MDE_KWM0(j) (kK[0 + (j)] + w[0 + (j)])
#define MDE_KWM4(j) (kK[4 + (j)] + w[4 + (j)])
#define MDE_KWM8(j) (kK[8 + (j)] + w[8 + (j)])
#define MDE_KWM12(j) (kK[12 + (j)] + w[12 + (j)])
#define MDE_KWV0(j) (v0[(j)])
#define MDE_KWV1(j) (v1[(j)])
#define MDE_KWV2(j) (v2[(j)])
#define MDE_KWP3(j) (p3[(j)])
  MDE_SHA_4A(MDE_KWM0);
  MDE_SHA_4B(MDE_KWM4);
  MDE_SHA_4A(MDE_KWM8);
  u32x4 p3 = {0u, 0u, 0u, 0u};  // K+W of the previous chunk's last four rounds
#pragma unroll
  for (int cn = 0; cn < 3; cn++) {
    __syncthreads();  // chunk cn = K+W of rounds 16(cn+1) .. 16(cn+1)+15 is in LDS
    const int r = 4 * (cn & 1);
    const u32x4 v0 = kw[(r + 0) * stride], v1 = kw[(r + 1) * stride];
    const u32x4 v2 = kw[(r + 2) * stride], v3 = kw[(r + 3) * stride];
    if (cn == 0) {
      MDE_SHA_4B(MDE_KWM12);
    } else {
      MDE_SHA_4B(MDE_KWP3);
    }
    MDE_SHA_4A(MDE_KWV0);
    MDE_SHA_4B(MDE_KWV1);
    MDE_SHA_4A(MDE_KWV2);
    p3 = v3;
  }
  MDE_SHA_4B(MDE_KWP3);
#undef MDE_KWM0
#undef MDE_KWM4
#undef MDE_KWM8
#undef MDE_KWM12
#undef MDE_KWV0
#undef MDE_KWV1
#undef MDE_KWV2
#undef MDE_KWP3
  st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
  if (kPair) {  // this lane's half of the state through the two-lane padding block (st[0..3] out)
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = is_a ? st[k] : st[4 + k];
    sha256_pad64_pair(v, is_a);
#pragma unroll
    for (int k = 0; k < 4; k++) st[k] = v[k];
  } else {
    sha256_compress_pad64(st);
  }
}

// The mirror side: the message schedule of the same node, published chunk by chunk.
__device__ __forceinline__ void sha256_node_duo_sched(const uint32_t hl[8], const uint32_t hr[8], u32x4* kw,
                                                      uint32_t stride) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { w[i] = hl[i]; w[8 + i] = hr[i]; }
#pragma unroll
  for (int cn = 0; cn < 3; cn++) {
    sha_sched16(w);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int r = 16 * (cn + 1) + 4 * q;
      kw[(4 * (cn & 1) + q) * stride] = u32x4{kK[r] + w[4 * q], kK[r + 1] + w[4 * q + 1], kK[r + 2] + w[4 * q + 2],
                                        kK[r + 3] + w[4 * q + 3]};
    }
    __syncthreads();
  }
}

// Level-1 node: SHA256(LE64(dl) || LE64(dr)) -> state words (big-endian digest words).
__device__ __forceinline__ void sha256_leaf_pair(uint64_t dl, uint64_t dr, uint32_t st[8]) {
  uint32_t w[16];
  w[0] = bswap((uint32_t)dl);
  w[1] = bswap((uint32_t)(dl >> 32));
  w[2] = bswap((uint32_t)dr);
  w[3] = bswap((uint32_t)(dr >> 32));
  w[4] = 0x80000000u;
#pragma unroll
  for (int i = 5; i < 15; i++) w[i] = 0;
  w[15] = 128u;
  sha256_init(st);
  sha256_compress(st, w);
}

// Upper node: SHA256(hl || hr) where hl, hr are 8-word digests (state-word form).
__device__ __forceinline__ void sha256_node_pair(const uint32_t hl[8], const uint32_t hr[8],
                                                 uint32_t st[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) { w[i] = hl[i]; w[8 + i] = hr[i]; }
  sha256_init(st);
  sha256_compress(st, w);
  sha256_compress_pad64(st);
}

// ------------------------------------------------------------------ XXH64 (xxHash spec)
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ULL, XP2 = 0xC2B2AE3D27D4EB4FULL,
                   XP3 = 0x165667B19E3779F9ULL, XP4 = 0x85EBCA77C2B2AE63ULL,
                   XP5 = 0x27D4EB2F165667C5ULL;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xx_round(uint64_t acc, uint64_t in) {
  acc += in * XP2;
  acc = rotl64(acc, 31);
  return acc * XP1;
}
__device__ __forceinline__ uint64_t xx_merge(uint64_t acc, uint64_t v) {
  acc ^= xx_round(0, v);
  return acc * XP1 + XP4;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

}  // namespace mde
