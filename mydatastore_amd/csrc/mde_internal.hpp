// mde_internal.hpp -- host-side launch interfaces between the C ABI (mde_api.cpp) and the
// gfx950 kernels (*.hip). Not installed; the public surface is include/mde.h.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mde {

// Segment s = bucket (p, b), s = p*B + b; its bytes are [segpos(s), segpos(s+1)) of the arena,
// segpos(s) = shift + (stride ? seg_rec[s]*stride : value_off[seg_rec[s]]).
struct SegDesc {
  const uint8_t* base;        // values rounded down to 16 B
  uint64_t shift;             // values - base (0..15)
  uint32_t stride;            // fixed value length, or 0
  const uint64_t* value_off;  // variable-length offsets (stride == 0)
  const uint64_t* seg_rec;    // [S+1]
  uint32_t S;                 // P*B
  uint64_t n_records;         // record indices are clamped to this ...
  uint64_t end;               // ... and positions to shift + values_bytes: bad input never faults
};

// Byte position of bucket s's first value (clamped: bad input never faults).
__host__ __device__ __forceinline__ uint64_t segpos(const SegDesc& d, uint32_t s) {
  const uint64_t r0 = d.seg_rec[s];
  const uint64_t r = r0 < d.n_records ? r0 : d.n_records;
  const uint64_t p = d.shift + (d.stride ? r * (uint64_t)d.stride : d.value_off[r]);
  return p < d.end ? p : d.end;
}
// Byte offset of record r's value relative to the arena start (no clamping).
__host__ __device__ __forceinline__ uint64_t recpos(const SegDesc& d, uint64_t r) {
  return d.stride ? r * (uint64_t)d.stride : d.value_off[r];
}

struct DigestLaunch {
  SegDesc seg;
  unsigned long long* sums;   // [S] u64 accumulators (zero on entry)
  uint64_t wave_bytes;        // contiguous bytes per wave (multiple of the 16 KiB max step)
  uint32_t n_waves;
  int variant;                // kernel variant id (digest.hip kVariants)
  uint32_t lds_bytes;         // residency cap for oversubscribed grids (0 = none)
  // Interleaved pieces (static variants): wave w streams `pieces` ranges of wave_bytes each,
  // [first + (j * n_waves + w) * wave_bytes, +wave_bytes) for j < pieces; piece_stride =
  // n_waves * wave_bytes. pieces = 1 is one contiguous range per wave.
  uint32_t pieces;
  uint64_t piece_stride;
};
hipError_t launch_bucket_digest(const DigestLaunch& a, hipStream_t st);
// Waves and wave range for an arena of `bytes` on a device with `cus` CUs.
// piece_bytes > 0 cuts each resident wave's share into pieces of about that size, interleaved
// across the grid (DigestLaunch::pieces); 0 keeps one contiguous range per wave.
void plan_bucket_digest(uint64_t bytes, int cus, int blocks_per_cu, int oversub, uint64_t piece_bytes,
                        uint64_t* wave_bytes, uint32_t* n_waves, uint32_t* pieces);
int bucket_digest_blocks_per_cu(int variant, int cap);
bool bucket_digest_variant_valid(int variant);
bool bucket_digest_pieces(int variant);  // interleaved-pieces variant (DigestLaunch::pieces)
int bucket_digest_pieces_sibling(int variant);  // its interleaved-pieces form (itself if none)
bool bucket_digest_rec8(int variant);  // fixed 8-byte records, record-space scan (needs LDS)
uint32_t bucket_digest_rec8_lds_bytes(int variant);

struct TaggedLaunch {
  const uint8_t* base;        // values rounded down to 16 B
  uint64_t shift;             // values - base
  uint32_t stride;            // fixed value length (> 0)
  double inv_stride;
  const uint64_t* part_rec;   // [P+1] record ranges of the partitions
  const uint16_t* tag;        // [n_records] bucket of each record
  uint32_t P, B;
  unsigned long long* sums;   // [P*B]
  uint32_t* counts;           // [P*B]
  uint64_t wave_bytes;
  uint32_t n_waves;
  int use_lds;                // set by the launcher: B <= kTaggedLdsMaxBuckets
  uint32_t lrep;              // set by the launcher: LDS bin slots per bucket (power of two)
  float inv_stride_f;         // set by the launcher
};
constexpr uint32_t kTaggedLdsMaxBuckets = 4096;
void plan_tagged(uint64_t bytes, int cus, int waves_per_cu, uint64_t* wave_bytes, uint32_t* n_waves);
hipError_t launch_tagged_digest(TaggedLaunch& a, hipStream_t st);
struct TreeLaunch;
// Fused build step for layout B (tagged.hip): this build's binning + the previous build's trees.
hipError_t launch_tagged_step(TaggedLaunch& a, const TreeLaunch* t, hipStream_t st);

struct TreeLaunch {
  uint32_t P, B;
  const unsigned long long* sums_in;  // [P*B] byte sums (digest = sum % 999999), or
  const uint64_t* digest_in;          // [P*B] digests (tree-from-digests mode)
  unsigned long long* sums_clear;     // zeroed after read (may be null)
  const uint64_t* seg_rec;            // [P*B+1] for sizes (may be null)
  uint32_t* counts_in;                // [P*B] sizes when seg_rec is null (layout B); cleared
  uint64_t* digest_out;               // [P*B] (may be null)
  int32_t* size_out;                  // [P*B]
  int32_t* items_out;                 // [P]
  uint8_t* root_out;                  // [P*32]
  uint8_t* nodes_out;                 // [P*n_int*32]; required when B > kTreeLdsMaxBuckets
  uint64_t n_int;
  // Tree-from-digests with a per-tree bucket count (decoded peer objects): tree p has
  // n_in[p] <= B buckets at digest_in + p*B (n_in[p] <= 0: no tree, nothing written); its nodes
  // use its own shape at stride n_int (= tree_internal(B)). Null: every tree has B buckets.
  const int32_t* n_in;
  // sums_in / sums_clear hold buckets [sums_base, ...) (the one-launch small build keeps each
  // workgroup's bucket sums in LDS)
  uint64_t sums_base = 0;
  // Fused build step, one partition per tree workgroup (Q = 0): LDS word of the split-schedule
  // K+W ring (tree_body_duo), 0 = plain tree_body. Set by the step launchers (plan_step_trees).
  uint32_t duo_kw_word = 0;
  // tree_body / tree_body_duo: stop at the first level of at most top_nodes nodes (0: the root).
  // nodes_out then holds levels 1 .. that level and root_out that level's first node; the caller
  // hashes the few top levels itself (mde_server_build_levels: a one-partition call's dependent
  // top levels, where a CPU core's SHA extensions beat the device's dependent chain).
  uint32_t top_nodes = 0;
};
constexpr uint32_t kTreeLdsMaxBuckets = 4096;
constexpr uint32_t kTreePairLdsMax = 64u * 1024u;  // standalone pair-shape trees (B <= 2,728)
constexpr uint32_t kTreePairMinPartitions = 512;
hipError_t launch_tree(const TreeLaunch& a, hipStream_t st);
// Split-schedule trees (tree_body_duo) for launches of at most kDuoMaxBlocks workgroups (wide
// trees: always); MDE_TREE_DUO=0 in the environment turns them off (A/B switch).
constexpr uint32_t kDuoMaxBlocks = 256;
bool tree_duo_enabled();
struct TreeGeometry {
  uint32_t G, threads, groups, words, lds_bytes;
  bool lds;  // levels in LDS (B <= kTreeLdsMaxBuckets)
};
// Group width / live threads per workgroup / LDS of the tree builder for B buckets; false when B
// is too large for LDS levels (the standalone kernel then needs nodes_out).
bool tree_geometry(uint32_t B, TreeGeometry* g);

// Fused build step (digest.hip): ONE launch digests `a` (this build) and, when t != null, builds
// the trees of the previous build from its byte sums `t` (another scratch slot), Q partitions per
// tree wave (tree_body_packed). Fusable when one partition's level buffers fit the LDS budget
// that keeps the streaming grid fully resident (B <= 1024 always does).
constexpr uint32_t kStepTreeLdsMax = 24u * 1024u + 64u;
bool build_step_fusable(uint32_t B);
uint32_t build_step_tree_q(uint32_t B);  // partitions per packed tree wave
// The tree workgroups of a fused step for P partitions of B buckets: Q partitions per packed tree
// wave (Q >= 1), or Q = 0 for one partition per two-wave group (kStepTreeWideThreads threads of
// tree_body); blocks = tree workgroups, lds_bytes = their LDS.
constexpr uint32_t kStepTreeWideThreads = 128;
constexpr uint32_t kStepTreeWideMinPartitions = 512;
// Q value: one partition per whole tree workgroup (tree_body_duo over 256 threads, half = 128) --
// the latency form for builds of few wide trees (plan_step_trees).
constexpr uint32_t kStepTreeWholeWG = 0xffffffffu;
// duo_kw_word: see TreeLaunch::duo_kw_word (may raise lds_bytes within kStepTreeLdsMax).
// stream_bytes: the build's arena bytes (0 = unknown: no whole-workgroup form).
void plan_step_trees(uint32_t B, uint32_t P, uint32_t* Q, uint32_t* blocks, uint32_t* lds_bytes, uint32_t* duo_kw_word,
                     uint64_t stream_bytes);
constexpr uint64_t kStepTreeWholeMaxBytes = 768ull << 20;
hipError_t launch_build_step(const DigestLaunch& a, const TreeLaunch* t, hipStream_t st);
// One-launch build of a small layout-A arena (digest.hip small_build_kernel): each workgroup sums
// its partitions' buckets into LDS and builds their trees from there (t.sums_in is not used).
constexpr uint64_t kSmallBuildMaxBytes = 96u * 1024u;
bool small_build_fits(uint64_t bytes, uint32_t P, uint32_t B);
hipError_t launch_small_build(const SegDesc& d, const TreeLaunch& t, hipStream_t st);

struct DiffLaunch {
  uint32_t n_pairs;
  uint32_t Ba, Bb;
  const uint64_t* da;
  const uint8_t* na;
  const uint64_t* db;
  const uint8_t* nb;
  int32_t* out_ids;
  uint64_t out_stride;
  int32_t* out_count;
  // Verify mode (all zero/null for plain pairwise diffs): pair i compares A tree i / a_div with
  // B tree i, whose bucket count is nb_in[i] (<= Bb; <= 0 means the peer tree could not be built:
  // out_count[i] = nb_in[i] or MDE_E_DECODE); B trees sit at stride Bb digests and
  // tree_internal(Bb) nodes, each laid out by its own shape.
  uint32_t a_div;
  const int32_t* nb_in;
};
hipError_t launch_diff(const DiffLaunch& a, hipStream_t st);

struct ExtractLaunch {
  SegDesc seg;
  const uint8_t* values;      // unaligned arena start (= seg.base + seg.shift)
  uint32_t P, B;
  const int32_t* ids;         // [P * ids_stride] bucket ids (e.g. diff output)
  uint64_t ids_stride;
  const int32_t* counts;      // [P] ids per partition (< 0: nothing)
  uint64_t* part_off;         // [P+1] record offsets into out_rec
  uint64_t* out_rec;          // [rec_cap]
  uint64_t rec_cap;
  uint8_t* out_values;        // [bytes_cap] (may be null)
  uint64_t* out_value_off;    // [rec_cap + 1] (may be null)
  uint64_t bytes_cap;
  int32_t* status;            // MDE_OK or MDE_E_CAPACITY
  uint64_t* scratch;          // [3 * (P + 1)] device scratch
  // layout B (tag != null): records of partition p are part_rec[p] .. part_rec[p+1], fixed stride
  const uint16_t* tag;
  const uint64_t* part_rec;
  uint32_t stride;
  // request order (mde_stream_buckets, layout A): ids walked as given, repeats streamed again, ids
  // outside [0, B) stream nothing, counts[p] == 0 means every bucket
  bool ordered;
};
constexpr uint32_t kExtractMaxBuckets = 1u << 16;
hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st);

struct WireEncodeLaunch {
  uint32_t n, B;
  const int32_t* partition;  // [n] (may be null: 0)
  int64_t lower, upper;
  const uint64_t* digest;    // [n*B]
  const int32_t* size;       // [n*B]
  const uint8_t* valid;      // [n] (may be null: false)
  const int32_t* items;      // [n] (may be null: sum over tree.Leafs)
  uint8_t* out;              // [n*out_stride]
  uint64_t out_stride;
  uint32_t* out_len;         // [n]
};
struct WireDecodeLaunch {
  uint32_t n;
  const uint8_t* bytes;
  const uint64_t* off;       // [n+1]
  uint32_t cap;              // bucket capacity per object
  int32_t* partition;
  int64_t* lower;
  int64_t* upper;
  uint64_t* digest;          // [n*cap]
  int32_t* size;             // [n*cap]
  uint8_t* valid;
  int32_t* items;
  int32_t* n_buckets;        // [n] bucket count, or MDE_E_DECODE / MDE_E_CAPACITY
  // Spill area of deeply nested unknown groups (wire_body.hpp skip_group): object i uses entries
  // [(off[i] - off[0]) / 2 + i, + len_i / 2 + 1); nullptr / too small = rescan fallback.
  uint32_t* deep = nullptr;
  uint64_t deep_cap = 0;     // entries
};
// Entries a decode of n objects of `bytes` bytes in all needs in WireDecodeLaunch::deep.
inline uint64_t wire_deep_entries(uint64_t n, uint64_t bytes) { return bytes / 2 + 2 * n + 2; }
inline uint64_t wire_max_bytes(uint32_t B) { return 57 + 20ull * (B + (B & 1u)); }
hipError_t launch_wire_encode(const WireEncodeLaunch& a, hipStream_t st);
hipError_t launch_wire_decode(const WireDecodeLaunch& a, hipStream_t st);

// VerifyEpoch's per-partition fold over its R peer diffs (main/manager.go:1072-1103).
struct VerifyLaunch {
  uint32_t P, R, B;
  const int32_t* peer_status;  // [P*R] diff length (>= 0) or a skipped peer (< 0)
  const int32_t* peer_ids;     // [P*R*ids_stride] diff ids
  uint64_t ids_stride;
  const uint8_t* peer_valid;   // [P*R] decoded EpochTreeObject.valid
  uint32_t replica_count;
  uint8_t* valid;              // [P] (read again by the encoder: device memory)
  int32_t* valid_count;        // [P]
  int32_t* diff_ids;           // [P*B] ascending, de-duplicated (utils.Int32Set)
  int32_t* diff_count;         // [P]
  // the caller's copies, stored once at the end of the fold (so they may live in pinned host
  // memory, no D2H copy): valid, and peer_status (may be null)
  uint8_t* valid_out = nullptr;
  int32_t* status_out = nullptr;
};
constexpr uint32_t kVerifyMaxBuckets = 1u << 16;
hipError_t launch_verify(const VerifyLaunch& a, hipStream_t st);

// The whole decision step in ONE launch, one workgroup per partition (verify.hip): decode the R
// peer objects (staged through LDS), rebuild only the peer trees whose shape differs from the
// local tree, diff (leaf-only for same-shape peers, diff_body.hpp), fold, encode. Used when
// R <= kVerifyFusedMaxPeers and the peer capacity is <= kVerifyFusedMaxCap; the five-launch chain
// otherwise. The member launches carry the scratch pointers of the chain (tree.n_in is set
// in-kernel per partition).
constexpr uint32_t kVerifyFusedMaxPeers = 64;
constexpr uint32_t kVerifyFusedMaxCap = 1024;
struct VerifyFusedLaunch {
  WireDecodeLaunch dec;  // n = P*R
  TreeLaunch tree;       // P = R per partition, B = cap; digest_in/nodes_out/root_out at partition 0
  DiffLaunch diff;       // n_pairs = P*R, a_div = R
  VerifyLaunch fold;
  WireEncodeLaunch enc;  // enc.n = 0: no object
  // local.P != 0: the local trees were given as digests only; partition p builds its own tree
  // (local.digest_in + p*B -> local.nodes_out + p*n_int*32) when one of its peers has another
  // shape (the only diff that reads local nodes). local.nodes_out == diff.na.
  TreeLaunch local;
};
bool verify_fused_fits(uint32_t R, uint32_t cap);
hipError_t launch_verify_fused(const VerifyFusedLaunch& a, hipStream_t st);
// Dynamic LDS of one fused decision-step workgroup for peer capacity `cap`, and its geometry.
size_t verify_fused_lds(uint32_t cap, uint32_t* G, uint32_t* words, uint32_t* stage_bytes);

// Resident build service (server.cpp, mde_server_* in include/mde.h): a persistent launch whose
// workgroup i serves request slot i. The slots live in coherent pinned host memory, mapped into
// the device's address space; the host posts a request by writing `r` and then `req` (release),
// the workgroup polls `req`, runs the one-launch small build on it (small_build_body) and stores
// `done` = `req` after its outputs (system-scope release). `closed` is set by a workgroup that
// stops polling at the end of its lifetime (it then checks `req` once more), so a host that posts
// and then reads `closed` == 1 knows its request may not be seen and relaunches the service.
// kind 0: a build (d, t: small_build_body); kind 1: a VerifyEpoch decision step of one partition
// (v: verify_fused_body with the geometry v_G / v_words / v_stage, v_deep for B > 64).
struct ServerReq {
  uint32_t kind;
  uint32_t stage;     // copy the request's inputs into dev_in first (1) or read them in place
  const uint8_t* src;  // stage: [src, src + stage_bytes) -> dev_in, 16-byte multiples
  uint8_t* dev_in;
  uint64_t stage_bytes;
  SegDesc d;
  TreeLaunch t;
  uint32_t G, words;  // tree_geometry(t.B)
  uint32_t duo;       // small_build_duo: split-schedule trees
  uint32_t v_G, v_words, v_stage, v_deep;
  VerifyFusedLaunch v;
};
struct alignas(128) ServerSlot {
  uint64_t req;          // host: sequence number of the posted request; kServerStop: exit
  uint64_t pad0[15];
  uint64_t done;         // device: sequence number of the last request served
  uint32_t closed;       // device: the workgroup has stopped polling this slot
  uint32_t pad1[29];
  ServerReq r;           // host: the posted request
};
constexpr uint64_t kServerStop = ~0ull;
// LDS of the service's workgroups for builds and decision steps of up to max_buckets buckets (0:
// none fit).
size_t server_lds_bytes(uint32_t max_buckets);
// The request plan of one build of P partitions x B buckets in one service workgroup: false when
// it does not fit (more partitions than one workgroup holds, or B beyond the LDS).
bool server_plan(uint32_t P, uint32_t B, size_t lds_bytes, uint32_t* G, uint32_t* words, uint32_t* duo);
// n_slots workgroups, each polling slots[i] (device address) until s_memrealtime passes its start
// + lifetime ticks (100 MHz) or it reads kServerStop.
hipError_t launch_server(ServerSlot* slots, uint32_t n_slots, uint64_t lifetime_ticks, size_t lds_bytes,
                         hipStream_t st);


hipError_t launch_tag_keys(const uint8_t* keys, const uint64_t* key_off, uint64_t n, uint32_t B,
                           uint32_t P, uint32_t* bucket, uint32_t* partition, hipStream_t st);
hipError_t launch_synth_tags(const uint64_t* gids, uint64_t n, uint32_t P, uint32_t B, int mode,
                             uint64_t kpp, uint32_t* part, uint32_t* bucket, hipStream_t st);
hipError_t launch_synth_values(uint8_t* dst, const uint64_t* gids, uint64_t n, uint32_t len,
                               uint64_t seed, hipStream_t st);

// Tree geometry helpers (host).
uint32_t tree_levels(uint32_t B, uint32_t* sizes /* cap 64, may be null */);
uint64_t tree_internal(uint32_t B);

}  // namespace mde
