/*
 * mde.h -- MI355X anti-entropy Merkle engine, C ABI (the drop-in boundary).
 *
 * Replaces the hot path of andrew-delph/MyDataStore main/merkle_tree.go. Paths below are relative
 * to the reference root. The reference has no Go `interface` for this path; it is four concrete
 * functions called from Manager.VerifyEpoch (main/manager.go:1036,1041,1076,1081):
 *
 *   RawPartitionMerkleTree(partitionId, lowerEpoch, upperEpoch)      main/merkle_tree.go:86-116
 *       -> mde_build / mde_build_async (many partitions per call)
 *   MerkleTreeToPartitionEpochObject(tree, p, lo, hi)                main/merkle_tree.go:118-138
 *       -> the digest/size/items outputs of mde_build (wire object assembly stays in the caller)
 *   EpochTreeObjectToMerkleTree(obj)                                 main/merkle_tree.go:140-157
 *       -> mde_tree_from_digests / _async
 *   DifferentMerkleTreeBuckets(tree1, tree2)                         main/merkle_tree.go:159-216
 *       -> mde_diff / mde_diff_async
 *
 * and their caller's decision step, Manager.VerifyEpoch (main/manager.go:998-1118: build ->
 * persist -> decode peer objects -> diff -> valid / diffSet) -> mde_verify_epochs / _async.
 *
 * plus the write-time tagging the records carry (main/manager.go:773-778 getKeyBucket,
 * hashring/hashring.go:108-110 FindPartitionID) -> mde_tag_keys_async.
 *
 * Conventions
 *  - Plain pointers and sizes only. `*_async` entry points take DEVICE pointers and enqueue on the
 *    context's stream (mde_set_stream); the others take HOST pointers and are synchronous.
 *  - Return 0 (MDE_OK) or a negative MDE_E_* code; never abort or throw across the ABI. The Go
 *    shim maps codes to errors.Errorf. Every entry point locks its context, so one context may be
 *    shared by many threads. The message of the last failed call on a context: mde_last_error_copy
 *    (copied under the context lock -- use it when the context is shared), or mde_last_error (a
 *    pointer into the context, valid until the next call on it: single-threaded use only).
 *  - Host input buffers are read only during the call and never retained (cgo pointer rules).
 *    Outputs are caller-allocated. A synchronous call returns only after every copy and launch
 *    it issued has finished, a failing call too: the caller may reuse or free its buffers as soon
 *    as it returns.
 */
#ifndef MDE_H_
#define MDE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDE_ABI_VERSION 1

#define MDE_OK 0
#define MDE_E_INVAL -1    /* bad argument (null pointer, zero buckets, inconsistent sizes) */
#define MDE_E_NOMEM -2    /* host or device allocation failed */
#define MDE_E_DEVICE -3   /* HIP runtime / kernel failure, or no usable gfx950 device */
#define MDE_E_TREE -4     /* diff: node/bucket-id mismatch (main/merkle_tree.go:168-170,194-196) */
#define MDE_E_CAPACITY -5 /* caller-supplied output too small */
#define MDE_E_DECODE -6   /* bucket hash not 8 bytes (utils/utils.go:80-82) */

/* CustomHash modulus, main/merkle_tree.go:19. */
#define MDE_HASH_MOD 999999ULL

typedef struct mde_ctx mde_ctx;

/* The records of P partitions in layout A (the order the reference's LSM range scans yield them,
 * main/merkle_tree.go:90-113): a contiguous value arena, records sorted by (partition, bucket).
 * Bucket s = p*n_buckets + b holds records seg_rec[s] .. seg_rec[s+1]-1 -- exactly the records
 * the iterator over [epoch_p_b_{lo}_, epoch_p_b_{hi}_) yields (main/indexs.go:13-20). */
typedef struct mde_records {
  const uint8_t* values;     /* value arena: the bytes CustomHash.Add consumes */
  uint64_t values_bytes;     /* arena size in bytes */
  uint32_t value_stride;     /* > 0: record r = values[r*stride, (r+1)*stride) */
  uint32_t layout;           /* MDE_LAYOUT_SORTED (A) or MDE_LAYOUT_TAGGED (B) */
  const uint64_t* value_off; /* value_stride == 0: [n_records+1] byte offsets into values */
  uint64_t n_records;
  uint32_t n_partitions;
  uint32_t n_buckets;        /* PartitionBuckets (config/config.go:20); any value >= 1 */
  const uint64_t* seg_rec;   /* layout A: [n_partitions*n_buckets + 1], nondecreasing, <= n_records */
  /* Layout B: records grouped by partition in arrival order, each with its bucket tag (the
   * getKeyBucket value, main/manager.go:773-778); the engine bins them into buckets itself.
   * Fixed-length values (value_stride > 0), n_buckets <= 65536. */
  const uint16_t* bucket_tag; /* [n_records] */
  const uint64_t* part_rec;   /* [n_partitions + 1] record ranges, nondecreasing, <= n_records */
} mde_records;

#define MDE_LAYOUT_SORTED 0u /* layout A: sorted by (partition, bucket); seg_rec */
#define MDE_LAYOUT_TAGGED 1u /* layout B: grouped by partition; bucket_tag + part_rec */

/* Per-partition results. Any pointer may be NULL except root. */
typedef struct mde_tree_out {
  uint64_t* digest; /* [P*B] CustomHash value of each bucket, in [0, 999999) */
  int32_t* size;    /* [P*B] MerkleBucket.size (record count, int32) */
  int32_t* items;   /* [P]   EpochTreeObject.items: sum of sizes over tree.Leafs -- the duplicate
                       leaf of an odd B counts twice (main/merkle_tree.go:122-134); int32 wrap */
  uint8_t* root;    /* [P*32] tree.MerkleRoot() */
  uint8_t* nodes;   /* [P*mde_tree_internal_nodes(B)*32] internal node hashes, level 1 .. root */
} mde_tree_out;

int mde_abi_version(void);
const char* mde_strerror(int code);
/* Visible gfx950 devices (0 without a usable GPU); a node's Go shim spreads partitions over them.
 * mde_device_list writes the HIP ordinals of the first `cap` of them (the ones mde_create and
 * mde_group_create take; another GPU model visible at a lower index is skipped) and returns how
 * many there are. */
int mde_device_count(void);
int mde_device_list(int* ordinals, int cap);

/* Context: one HIP device, one stream, device scratch. */
int mde_create(int device, mde_ctx** out);
void mde_destroy(mde_ctx* ctx);
const char* mde_last_error(mde_ctx* ctx);
/* Copy the last error message of ctx into buf (at most cap-1 bytes + NUL) under the context
 * lock; returns the message's full length. Safe while other threads use the context. To pair a
 * failed call with its own message on a shared context, the caller serialises call + copy (the
 * Go shim holds a mutex across both: calls on one context are serialised by its lock anyway). */
uint64_t mde_last_error_copy(mde_ctx* ctx, char* buf, uint64_t cap);
/* Launch stream for *_async calls and internal copies. A new context uses its own stream (a
 * blocking stream: ordered after work on the null stream). NULL selects the null stream, which
 * is torch's default stream. */
int mde_set_stream(mde_ctx* ctx, void* hip_stream);
int mde_use_own_stream(mde_ctx* ctx);
void* mde_get_stream(mde_ctx* ctx);
int mde_synchronize(mde_ctx* ctx);
int mde_device_info(mde_ctx* ctx, int* cu_count, char* arch_name, int arch_cap);
/* Tuning hook for benchmarks: digest-kernel variant, resident workgroups per CU, and grid
 * oversubscription (-1 = the built-in defaults: the variant is then chosen per build -- the
 * register-window kernel when buckets average under 64 KiB, e.g. the reference's default
 * B = 1000 -- with interleaved pieces for large shares). Results are identical for every setting;
 * only speed changes. */
int mde_set_tuning(mde_ctx* ctx, int digest_variant, int digest_blocks_per_cu, int digest_oversub);
/* Work accounting since the context was created: builds enqueued on it (mde_build[_async],
 * mde_build_pipelined_async, each chunk of mde_build_streamed), their partitions and value bytes.
 * On a group member's context (mde_group_ctx) it shows which GPU built what. */
int mde_ctx_stats(mde_ctx* ctx, uint64_t* builds, uint64_t* partitions, uint64_t* value_bytes);
/* Tuning hook: layout-A digest work split. 0 = one contiguous range per resident wave; N > 0 =
 * with the interleaved-pieces digest variant, each wave's share cut into pieces of about N bytes,
 * interleaved across the grid so all waves sweep the arena front to back together (used when a
 * share is at least 2N bytes); UINT64_MAX (default) = automatic: shares of 4 MiB or more are cut
 * into 5 pieces. Results are identical for every setting. */
int mde_set_digest_piece_bytes(mde_ctx* ctx, uint64_t piece_bytes);
/* Launch shape of mde_verify_epochs[_async]: 0 (default) = one fused launch whenever
 * n_peers <= 64 and mde_verify_peer_capacity(n_buckets) <= 1024, else the five-launch chain;
 * 1 = always the chain. Results are identical; only latency changes. */
int mde_set_verify_mode(mde_ctx* ctx, int mode);

/* Tree geometry (merkletree v0.2.0 shape: dup last leaf if odd, self-pair odd levels). */
uint32_t mde_tree_depth(uint32_t n_buckets);          /* internal levels, root included */
uint64_t mde_tree_internal_nodes(uint32_t n_buckets); /* nodes per tree in mde_tree_out.nodes */
/* Nodes of levels 1 .. L, L = the first level of at most top_nodes nodes (top_nodes <= 1: every
 * level, = mde_tree_internal_nodes): what mde_server_build_levels writes per partition. */
uint64_t mde_tree_prefix_nodes(uint32_t n_buckets, uint32_t top_nodes);
uint64_t mde_diff_capacity(uint32_t n_buckets_a, uint32_t n_buckets_b); /* max ids one diff emits */

/* RawPartitionMerkleTree for P partitions: bucket digests + sizes + SHA-256 tree on device.
 * Host pointers; synchronous (H2D, build, D2H). */
int mde_build(mde_ctx* ctx, const mde_records* rec, const mde_tree_out* out);
/* Same, device pointers, enqueued on the context stream (inputs resident in HBM). */
int mde_build_async(mde_ctx* ctx, const mde_records* rec, const mde_tree_out* out);
/* Host ingest path: same contract as mde_build, but the arena is
 * streamed to the device in chunks of whole partitions (about chunk_bytes each; 0 = 256 MiB)
 * through a two-slot device ring -- the copy of chunk k+1 overlaps the build of chunk k on a
 * second stream -- so device memory stays bounded and arenas larger than HBM work. Pass pinned
 * host memory (hipHostMalloc / hipHostRegister) for the copies to be asynchronous. */
int mde_build_streamed(mde_ctx* ctx, const mde_records* rec, const mde_tree_out* out,
                       uint64_t chunk_bytes);
/* The two stages of mde_build_async, for stage timing: bucket byte-sum kernel, then the
 * digest/size/tree kernel. mde_build_async == mde_digest_async + mde_tree_async. */
int mde_digest_async(mde_ctx* ctx, const mde_records* rec);
int mde_tree_async(mde_ctx* ctx, const mde_records* rec, const mde_tree_out* out);
/* Throughput mode for a run of builds (successive epochs, replicas or partition batches of
 * RawPartitionMerkleTree, main/merkle_tree.go:86-116), software-pipelined on the context stream:
 * each call enqueues ONE launch that streams rec's arena into a free scratch slot and, in the
 * same dispatch, builds the trees of the previous pipelined call into that call's outputs. So the
 * outputs of call i are complete (in stream order) after call i+1 or after
 * mde_build_pipeline_drain_async; rec's device arrays (seg_rec / part_rec, bucket_tag) and the
 * outputs of call i must stay valid until then. Results are identical to mde_build_async. Uses
 * scratch of its own: the other entry points may be interleaved freely. Both layouts fuse when
 * the previous build's tree levels fit the fused launch's 24 KiB LDS budget (n_buckets <= 1024
 * always does); wider trees run as a separate tree launch on the same stream. */
int mde_build_pipelined_async(mde_ctx* ctx, const mde_records* rec, const mde_tree_out* out);
int mde_build_pipeline_drain_async(mde_ctx* ctx);

/* EpochTreeObjectToMerkleTree for n_trees trees of n_buckets leaves each: digests -> nodes.
 * `buckets` are the 8-byte LE bucket hashes exactly as carried on the wire (EpochTreeObject
 * .buckets); each must be 8 bytes, mirroring utils.DecodeBytesToInt64. */
int mde_tree_from_digests(mde_ctx* ctx, uint32_t n_trees, uint32_t n_buckets,
                          const uint64_t* digest, uint8_t* root, uint8_t* nodes);
int mde_tree_from_digests_async(mde_ctx* ctx, uint32_t n_trees, uint32_t n_buckets,
                                const uint64_t* digest, uint8_t* root, uint8_t* nodes);
int mde_decode_bucket_hashes(const uint8_t* const* hashes, const uint32_t* lens, uint32_t n,
                             uint64_t* digest_out);

/* DifferentMerkleTreeBuckets for n_pairs tree pairs (tree i of A vs tree i of B): bucket ids in
 * the reference's DFS order, duplicates included (a differing self-paired node emits its subtree
 * twice). Tree inputs are (digest[n_buckets], nodes[mde_tree_internal_nodes*32]) per tree.
 * out_ids: [n_pairs * out_stride] with out_stride >= mde_diff_capacity(b_a, b_b);
 * out_count[i] = number of ids, or MDE_E_TREE where the reference returns an error. */
int mde_diff(mde_ctx* ctx, uint32_t n_pairs, uint32_t n_buckets_a, const uint64_t* digest_a,
             const uint8_t* nodes_a, uint32_t n_buckets_b, const uint64_t* digest_b,
             const uint8_t* nodes_b, int32_t* out_ids, uint64_t out_stride, int32_t* out_count);
int mde_diff_async(mde_ctx* ctx, uint32_t n_pairs, uint32_t n_buckets_a, const uint64_t* digest_a,
                   const uint8_t* nodes_a, uint32_t n_buckets_b, const uint64_t* digest_b,
                   const uint8_t* nodes_b, int32_t* out_ids, uint64_t out_stride,
                   int32_t* out_count);

/* Convenience for callers that hold only bucket digests (e.g. the Go shim, whose trees are
 * *merkletree.MerkleTree): builds both trees on device and diffs them. Host pointers, synchronous.
 * Same output contract as mde_diff. */
int mde_diff_digests(mde_ctx* ctx, uint32_t n_pairs, uint32_t n_buckets_a, const uint64_t* digest_a,
                     uint32_t n_buckets_b, const uint64_t* digest_b, int32_t* out_ids,
                     uint64_t out_stride, int32_t* out_count);

/* Out-of-sync range extract (StreamBucketsTask, main/manager.go:445-487): for partition p, the
 * records of the buckets ids[p*ids_stride .. +counts[p]) (duplicates removed -- VerifyEpoch's
 * Int32Set, main/manager.go:1086; counts[p] < 0 extracts nothing), in ascending bucket order and
 * LSM record order. Feed it mde_diff's output directly. n_buckets <= 65536.
 * Layout B records (MDE_LAYOUT_TAGGED): the same record set, in arrival order (a bucket's records
 * are not contiguous there).
 * part_off[P+1]: record offsets of each partition in out_rec / out_value_off;
 * out_rec[rec_cap]: source record indices; out_values[bytes_cap] (optional): the value bytes,
 * concatenated; out_value_off[rec_cap+1] (optional): byte offset of each extracted value in
 * out_values. *status = MDE_OK, or MDE_E_CAPACITY (then nothing is written past part_off). */
int mde_extract_async(mde_ctx* ctx, const mde_records* rec, const int32_t* ids, uint64_t ids_stride,
                      const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                      uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap,
                      int32_t* status);
/* Host-pointer version; returns MDE_E_CAPACITY when the outputs are too small. */
int mde_extract(mde_ctx* ctx, const mde_records* rec, const int32_t* ids, uint64_t ids_stride,
                const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap);

/* StreamBucketsTask's own list contract (main/manager.go:447-485; replaces the loop over
 * task.Buckets): for partition p the requested ids ids[p*ids_stride .. +counts[p]) are walked IN
 * THE ORDER GIVEN -- a repeated id streams its bucket's records again, an id outside [0, n_buckets)
 * streams nothing (no record carries it) -- and counts[p] == 0 streams every bucket 0..B-1 (the
 * task's empty list, :448-452); counts[p] < 0 streams nothing. Within a bucket, LSM record order.
 * Layout A only (MDE_E_INVAL for MDE_LAYOUT_TAGGED). Outputs as mde_extract; rec_cap / bytes_cap
 * must cover the repeats. mde_extract stays the deduplicated ascending form for VerifyEpoch's
 * diff set (already an Int32Set, :1086), whose order the reference leaves to Go's map iteration. */
int mde_stream_buckets_async(mde_ctx* ctx, const mde_records* rec, const int32_t* ids, uint64_t ids_stride,
                             const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                             uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap,
                             int32_t* status);
int mde_stream_buckets(mde_ctx* ctx, const mde_records* rec, const int32_t* ids, uint64_t ids_stride,
                       const int32_t* counts, uint64_t* part_off, uint64_t* out_rec, uint64_t rec_cap,
                       uint8_t* out_values, uint64_t* out_value_off, uint64_t bytes_cap);

/* EpochTreeObject wire bytes (datap/data.proto:60-68), exactly as proto.Marshal emits them for
 * MerkleTreeToPartitionEpochObject's object (main/merkle_tree.go:118-138, main/manager.go:1045):
 * leaves follow tree.Leafs (an odd B repeats the last bucket), zero scalars omitted, sizes packed.
 * Object i is written at out + i*out_stride (out_stride >= mde_epoch_tree_object_max_bytes(B)),
 * its length in out_len[i]. partition/valid/items may be NULL (0 / false / the tree.Leafs sum).
 * n_buckets = 0 encodes objects without buckets (scalars only; digest/size may then be NULL), as
 * proto.Marshal does for an RpcEpochTreeObject built field by field (main/manager_test.go:245). */
uint64_t mde_epoch_tree_object_max_bytes(uint32_t n_buckets);
int mde_encode_epoch_tree_objects_async(mde_ctx* ctx, uint32_t n, uint32_t n_buckets,
                                        const int32_t* partition, int64_t lower_epoch,
                                        int64_t upper_epoch, const uint64_t* digest,
                                        const int32_t* size, const uint8_t* valid,
                                        const int32_t* items, uint8_t* out, uint64_t out_stride,
                                        uint32_t* out_len);
int mde_encode_epoch_tree_objects(mde_ctx* ctx, uint32_t n, uint32_t n_buckets,
                                  const int32_t* partition, int64_t lower_epoch, int64_t upper_epoch,
                                  const uint64_t* digest, const int32_t* size, const uint8_t* valid,
                                  const int32_t* items, uint8_t* out, uint64_t out_stride,
                                  uint32_t* out_len);
/* Decode n objects (object i = bytes[off[i] .. off[i+1])) into up to `cap` buckets each:
 * n_buckets[i] = number of bucket hashes (the tree's leaf count for EpochTreeObjectToMerkleTree),
 * or MDE_E_DECODE (malformed, or a bucket hash that is not 8 bytes) / MDE_E_CAPACITY. Missing
 * sizes read as 0 (main/merkle_tree.go:147-152). Any output except n_buckets may be NULL. */
int mde_decode_epoch_tree_objects_async(mde_ctx* ctx, uint32_t n, const uint8_t* bytes,
                                        const uint64_t* off, uint32_t cap, int32_t* partition,
                                        int64_t* lower_epoch, int64_t* upper_epoch,
                                        uint64_t* digest, int32_t* size, uint8_t* valid,
                                        int32_t* items, int32_t* n_buckets);
int mde_decode_epoch_tree_objects(mde_ctx* ctx, uint32_t n, const uint8_t* bytes,
                                  const uint64_t* off, uint32_t cap, int32_t* partition,
                                  int64_t* lower_epoch, int64_t* upper_epoch, uint64_t* digest,
                                  int32_t* size, uint8_t* valid, int32_t* items, int32_t* n_buckets);

/* Manager.VerifyEpoch (main/manager.go:1036-1118) for n_partitions partitions of epoch E, given
 * this node's trees (digest/size/nodes from mde_build with the nodes output, n_buckets each; nodes
 * may be NULL: a partition then builds its own tree on the device, only if one of its peers has
 * another shape -- the one diff that reads inner nodes) and
 * n_peers peer EpochTreeObject wire objects per partition (what EpochTreeObjectRequest returned):
 * object (p, r) = peer_bytes[peer_off[p*n_peers+r] .. peer_off[p*n_peers+r+1]); an empty range is
 * an absent peer. Each peer object is decoded and rebuilt (EpochTreeObjectToMerkleTree) and diffed
 * against the local tree (DifferentMerkleTreeBuckets(myTree, otherTree)); a peer whose object or
 * diff fails is skipped, as the reference does (logrus.Error; continue).
 * Outputs per partition p:
 *   valid[p]       = validCount >= replica_count || a non-empty diff against a Valid peer object
 *   valid_count[p] = number of peers whose diff is empty
 *   diff_ids[p*n_buckets ..], diff_count[p] = diffSet (utils.Int32Set of every successful diff),
 *                    ascending -- the bucket list PoliteStreamRequest asks for when !valid
 *   peer_status[p*n_peers+r] (optional) = the peer's diff length, MDE_E_DECODE (no tree from the
 *                    object) or MDE_E_TREE (DifferentMerkleTreeBuckets error)
 *   object_out (optional) = the EpochTreeObject VerifyEpoch persists for index
 *                    epochtree_{p}_{E}: MerkleTreeToPartitionEpochObject(myTree, p, E, E+1) with
 *                    Valid = valid[p], at object_out + p*object_stride (length object_len[p]).
 * partition may be NULL (0). n_buckets <= 65536. A peer object with more than
 * mde_verify_peer_capacity(n_buckets) buckets builds a deeper tree, which the reference's diff
 * always rejects; it is reported as MDE_E_TREE without being rebuilt. Every output is stored
 * exactly once and never read back by the call (the _async form may point them at pinned host
 * memory mapped into the device address space). */
uint32_t mde_verify_peer_capacity(uint32_t n_buckets);
/* Unknown groups nested deeper than 64 levels (a hostile peer object) spill their group numbers
 * to a per-context device area, so decoding stays linear in the object bytes however the nesting
 * oscillates. The host-buffer calls size it exactly; the *_async decode / verify calls use what
 * the context holds (by default enough for 8 MiB of objects per call; past that a deep object
 * falls back to rescanning its outer group). Reserve room for `n_objects` objects of
 * `object_bytes` bytes in all before such a call to keep every object linear. */
int mde_reserve_decode_scratch(mde_ctx* ctx, uint64_t n_objects, uint64_t object_bytes);
int mde_verify_epochs_async(mde_ctx* ctx, uint32_t n_partitions, uint32_t n_buckets,
                            const int32_t* partition, int64_t epoch, const uint64_t* digest,
                            const int32_t* size, const uint8_t* nodes, uint32_t n_peers,
                            const uint8_t* peer_bytes, const uint64_t* peer_off,
                            uint32_t replica_count, uint8_t* valid, int32_t* valid_count,
                            int32_t* diff_ids, int32_t* diff_count, int32_t* peer_status,
                            uint8_t* object_out, uint64_t object_stride, uint32_t* object_len);
int mde_verify_epochs(mde_ctx* ctx, uint32_t n_partitions, uint32_t n_buckets,
                      const int32_t* partition, int64_t epoch, const uint64_t* digest,
                      const int32_t* size, const uint8_t* nodes, uint32_t n_peers,
                      const uint8_t* peer_bytes, const uint64_t* peer_off, uint32_t replica_count,
                      uint8_t* valid, int32_t* valid_count, int32_t* diff_ids, int32_t* diff_count,
                      int32_t* peer_status, uint8_t* object_out, uint64_t object_stride,
                      uint32_t* object_len);

/* Device groups: one process driving the G GPUs of a node (a Go node is one process). Partition p
 * lives on device p % G (the in-node analogue of the reference's partition sharding over nodes,
 * hashring/hashring.go:126-154); every device builds its own partitions, and the one exchange step
 * -- the per-partition roots -- is ONE all-gather of fixed-size root slabs: RCCL over xGMI on
 * communicators created once by mde_group_create (ncclCommInitAll), or device copies when a device
 * is listed more than once (several contexts on one GPU) -- mde_group_gather_kind says which.
 * Shard i holds partitions i, i + G, i + 2G, ... (mde_group_partitions of them), in that order. */
typedef struct mde_group mde_group;
int mde_group_create(const int* devices, uint32_t n_devices, mde_group** out);
void mde_group_destroy(mde_group* group);
uint32_t mde_group_size(const mde_group* group);
mde_ctx* mde_group_ctx(mde_group* group, uint32_t i);
const char* mde_group_gather_kind(const mde_group* group); /* "rccl all_gather" or "device copies (why)" */
uint32_t mde_group_partitions(const mde_group* group, uint32_t n_partitions, uint32_t i);
const char* mde_group_last_error(const mde_group* group);
/* mde_last_error_copy for a group (its calls are serialised by a group lock). */
uint64_t mde_group_last_error_copy(mde_group* group, char* buf, uint64_t cap);
/* RawPartitionMerkleTree for P partitions over the group (host pointers, synchronous); same
 * contract and results as mde_build: each device receives its partitions' records (one copy per
 * partition range), builds them, the root slabs (ceil(P/G) roots each) are all-gathered, and the
 * outputs land in the caller's arrays in partition order. root == NULL: digest-only, no gather. */
int mde_multi_build(mde_group* group, const mde_records* rec, const mde_tree_out* out);
/* Host ingest over the group (arenas larger than HBM, nothing resident): partition p on device
 * p % G as everywhere else in the group API (mde_group_partitions); each device streams its
 * partitions in chunks of ~chunk_bytes (0: 256 MiB) through a two-slot device ring, one host copy
 * per partition range, concurrently with the other devices. Same contract and results as
 * mde_multi_build. */
int mde_multi_build_streamed(mde_group* group, const mde_records* rec, const mde_tree_out* out,
                             uint64_t chunk_bytes);
/* Device-resident use, each call enqueued on every device's context stream (mde_group_ctx,
 * mde_set_stream): shard[i] / shard_out[i] hold device-i pointers (shard i's partitions, layout as
 * in mde_build_async); a shard with n_partitions == 0 is skipped. */
int mde_group_build_async(mde_group* group, const mde_records* shard, const mde_tree_out* shard_out);
int mde_group_build_pipelined_async(mde_group* group, const mde_records* shard, const mde_tree_out* shard_out);
int mde_group_build_pipeline_drain_async(mde_group* group);
/* The exchange step: device i contributes `bytes` from send[i] (device i memory); recv[i] (device
 * i memory, G x bytes) receives every device's slab, slab r = device r's. */
int mde_group_gather_async(mde_group* group, const void* const* send, void* const* recv, uint64_t bytes);
/* The same exchange step overlapped with the next builds: each device's gather waits for the work
 * already enqueued on the context streams (the producers of the send slabs) and runs on a side
 * stream of that device, so the builds enqueued next on the context streams overlap it. *ticket
 * (may be NULL) names it for mde_group_gather_wait_async, which makes every context stream wait
 * until that gather has read every send slab and filled every recv -- call it before rewriting a
 * send slab or reading a recv buffer in stream order. mde_group_synchronize also waits for it. */
int mde_group_gather_overlapped_async(mde_group* group, const void* const* send, void* const* recv, uint64_t bytes,
                                      uint64_t* ticket);
int mde_group_gather_wait_async(mde_group* group, uint64_t ticket);
int mde_group_synchronize(mde_group* group);
/* BASELINE config 5 over the group (both replicas of a partition on the same device, so the
 * compare and the extract are device-local): DifferentMerkleTreeBuckets
 * (main/merkle_tree.go:159-216) of shard i's tree pairs on device i -- mde_diff_async's arguments,
 * device-i pointers; n_pairs == 0 skips the device -- and StreamBucketsTask's range walk
 * (main/manager.go:445-487) of shard i's records of the differing buckets -- mde_extract_async's
 * arguments. Enqueued on every device's context stream. */
typedef struct mde_diff_args {
  uint32_t n_pairs, n_buckets_a, n_buckets_b;
  const uint64_t* digest_a;
  const uint8_t* nodes_a;
  const uint64_t* digest_b;
  const uint8_t* nodes_b;
  int32_t* out_ids;
  uint64_t out_stride;
  int32_t* out_count;
} mde_diff_args;
typedef struct mde_extract_args {
  const int32_t* ids;
  uint64_t ids_stride;
  const int32_t* counts;
  uint64_t* part_off;
  uint64_t* out_rec;
  uint64_t rec_cap;
  uint8_t* out_values;     /* optional */
  uint64_t* out_value_off; /* optional */
  uint64_t bytes_cap;
  int32_t* status;
} mde_extract_args;
int mde_group_diff_async(mde_group* group, const mde_diff_args* shard);
int mde_group_extract_async(mde_group* group, const mde_records* shard, const mde_extract_args* shard_args);

/* Request coalescing for the production call shape (one partition per call). The reference runs
 * RawPartitionMerkleTree and the VerifyEpoch decision for ONE (partition, epoch) per call, on any
 * of workers_count = 100 goroutines with up to partition_concurrency = 10 in flight
 * (config/default-config.yaml:7,9; main/manager.go:68,166-170,489-497,998-1118). A batcher owns
 * its own contexts on `device` and merges concurrent calls by group commit: a caller's request
 * joins the queue; the first caller to find no batch running takes every compatible queued
 * request (same kind and n_buckets; verify: same epoch and replica_count, objects wanted or not;
 * at most max_partitions partitions; after waiting up to max_wait_us for more, 0 = no wait) and
 * runs them as ONE H2D copy + ONE build (or verify) launch + ONE D2H copy; requests arriving
 * meanwhile form the next batch (up to mde_batcher_contexts() batches in flight). A build batch
 * holds at most 2^32 buckets in all. Every call is synchronous and thread-safe, returns exactly what
 * the per-call entry point returns for its own inputs, and writes its own error message into
 * err (err_cap bytes, NUL-terminated; may be NULL) -- no shared last-error state, so the Go shim
 * needs no lock. Inputs are host pointers, read only during the call (cgo pointer rules).
 * mde_batcher_destroy must not race with calls in flight. */
typedef struct mde_batcher mde_batcher;
int mde_batcher_create(int device, uint32_t max_partitions, uint32_t max_wait_us, mde_batcher** out);
void mde_batcher_destroy(mde_batcher* b);
/* A batcher keeps up to mde_batcher_contexts() batches in flight, each on its own context (own
 * stream and scratch), so small batches run concurrently on the device; mde_batcher_ctx(b, i)
 * gives context i (tuning, device info). */
uint32_t mde_batcher_contexts(const mde_batcher* b);
mde_ctx* mde_batcher_ctx(mde_batcher* b, uint32_t i);
/* batches run, requests served and partitions built since creation */
int mde_batcher_stats(mde_batcher* b, uint64_t* batches, uint64_t* requests, uint64_t* partitions);
/* RawPartitionMerkleTree (main/merkle_tree.go:86-116) for the caller's partitions: mde_build's
 * contract for layout A records (fixed or variable-length values); records outside
 * [seg_rec[0], seg_rec[P*B]) are not read. */
int mde_batch_build(mde_batcher* b, const mde_records* rec, const mde_tree_out* out, char* err,
                    uint64_t err_cap);
/* The VerifyEpoch decision step (main/manager.go:1072-1104) for ONE partition: mde_verify_epochs
 * with n_partitions = 1, whose local tree is given by its bucket digests (and sizes, required for
 * object_out); its inner nodes (EpochTreeObjectToMerkleTree of the local object) are built on the
 * device inside the verify launch, and only when a peer of another shape needs them. n_peers may
 * differ between callers of one batch. */
int mde_batch_verify(mde_batcher* b, uint32_t n_buckets, int32_t partition, int64_t epoch,
                     const uint64_t* digest, const int32_t* size, uint32_t n_peers,
                     const uint8_t* peer_bytes, const uint64_t* peer_off, uint32_t replica_count,
                     uint8_t* valid, int32_t* valid_count, int32_t* diff_ids, int32_t* diff_count,
                     int32_t* peer_status, uint8_t* object_out, uint64_t object_stride,
                     uint32_t* object_len, char* err, uint64_t err_cap);

/* Resident build service for the one-partition calls (RawPartitionMerkleTree,
 * main/merkle_tree.go:86-116, called once per VerifyEpoch, main/manager.go:1036). A persistent
 * launch keeps one workgroup per request slot resident on `device`, polling the slot in coherent
 * pinned host memory: a call packs its records into a free slot and spins until the slot's
 * workgroup has built them (the one-launch small build: bucket digests, then the SHA-256 tree, or
 * no tree when out->root is NULL) into the slot's pinned outputs -- no kernel launch, copy command
 * or event per call. The launch ends itself after MDE_SERVER_LIFETIME_MS (default 100) and the
 * next call relaunches it, so an idle process holds no GPU work. n_slots = 0: 16 (at most 256);
 * max_buckets = 0: 1024 (at most 4096), which sizes the launch's LDS. mde_server_build has
 * mde_batch_build's contract (layout A, host pointers read only during the call, its own error
 * message in err); a request one workgroup cannot take (more partitions than it holds, more than
 * 256 KiB of packed inputs, n_buckets > max_buckets) runs as mde_build on the service's own
 * context. Thread-safe; mde_server_destroy must not race with calls in flight.
 * Teardown: the launch runs on a CU-masked stream (a hardware queue of its own). By default that
 * stream is never destroyed -- mde_server_destroy parks it for the next service on the device --
 * because destroying a masked stream hung the runtime when a stream created before it was destroyed
 * after it. With MDE_SERVER_CUMASK=1 (destroy it with the service) create the
 * service before, and destroy it after, every other context of the device. */
typedef struct mde_server mde_server;
int mde_server_create(int device, uint32_t n_slots, uint32_t max_buckets, mde_server** out);
void mde_server_destroy(mde_server* s);
uint32_t mde_server_slots(const mde_server* s);
int mde_server_build(mde_server* s, const mde_records* rec, const mde_tree_out* out, char* err,
                     uint64_t err_cap);
/* RawPartitionMerkleTree split between the device and the caller: digests, sizes, items and the
 * tree's levels 1 .. L (L = the first level of at most top_nodes nodes; out->nodes required, at
 * the usual stride of mde_tree_internal_nodes(B) per partition, of which the first
 * mde_tree_prefix_nodes(B, top_nodes) hold the tree's nodes; the nodes past that prefix are
 * unspecified -- a call run on the service's context writes every level, one served resident
 * leaves them untouched; out->root is not written). The caller hashes
 * the few top levels (node = SHA256(left || right), the last node of an odd level paired with
 * itself): a tree's dependent top levels cost a CPU core ~40 ns per compression on its SHA
 * extensions against ~2 us on the device. The Go shim assembles the tree from these nodes and
 * hashes its top levels with crypto/sha256. */
int mde_server_build_levels(mde_server* s, const mde_records* rec, const mde_tree_out* out, uint32_t top_nodes,
                            char* err, uint64_t err_cap);
/* The VerifyEpoch decision step (main/manager.go:1072-1104) for ONE partition, served the same
 * way (the fused decision step of mde_verify_epochs in the slot's workgroup): mde_batch_verify's
 * contract. More than 16 peers, more than 256 KiB of packed inputs or n_buckets > max_buckets run
 * as mde_verify_epochs on the service's context. */
int mde_server_verify(mde_server* s, uint32_t n_buckets, int32_t partition, int64_t epoch,
                      const uint64_t* digest, const int32_t* size, uint32_t n_peers,
                      const uint8_t* peer_bytes, const uint64_t* peer_off, uint32_t replica_count,
                      uint8_t* valid, int32_t* valid_count, int32_t* diff_ids, int32_t* diff_count,
                      int32_t* peer_status, uint8_t* object_out, uint64_t object_stride,
                      uint32_t* object_len, char* err, uint64_t err_cap);
/* calls served, launches made (1 + relaunches after a lifetime ended) and calls run on the
 * service's context */
int mde_server_stats(mde_server* s, uint64_t* requests, uint64_t* launches, uint64_t* on_context);
/* 1 while the resident launch serves calls; 0 once it is out of service -- a launch failed, a
 * request timed out (30 s), or mde_server_disable -- after which every call runs as mde_build /
 * mde_verify_epochs on the service's context (same results, a launch per call), so one transient
 * stall does not fail later calls. mde_server_disable takes the resident launch out of service
 * (e.g. to give its CUs back to bulk builds): the resident workgroups of idle slots exit at once,
 * a slot serving a call exits when that call returns; `why` is kept for diagnostics. */
int mde_server_usable(mde_server* s);
int mde_server_disable(mde_server* s, const char* why);

/* Write-time tagging of raw keys (device): bucket = BE64(SHA256(key)[:8]) % n_buckets
 * (main/manager.go:773-778), partition = XXH64(key, 0) % n_partitions (hashring.go:108-110).
 * key i = keys[key_off[i] .. key_off[i+1]). Either output may be NULL. */
int mde_tag_keys_async(mde_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                       uint32_t n_buckets, uint32_t n_partitions, uint32_t* bucket,
                       uint32_t* partition);
int mde_tag_keys(mde_ctx* ctx, const uint8_t* keys, const uint64_t* key_off, uint64_t n,
                 uint32_t n_buckets, uint32_t n_partitions, uint32_t* bucket, uint32_t* partition);

/* Synthetic workload, device side, for benches and tests:
 * key of record gid = "k%016x" % gid; value word w = splitmix64(seed ^ (gid*2^20 + w)), LE bytes.
 * part_mode: 0 = gid / keys_per_partition, 1 = gid % P, 2 = FindPartitionID(key). */
int mde_synth_tags_async(mde_ctx* ctx, const uint64_t* gids, uint64_t n, uint32_t n_partitions,
                         uint32_t n_buckets, int part_mode, uint64_t keys_per_partition,
                         uint32_t* partition, uint32_t* bucket);
int mde_synth_values_async(mde_ctx* ctx, uint8_t* dst, const uint64_t* gids, uint64_t n,
                           uint32_t value_len, uint64_t seed);

/* Plain device memory helpers for callers without a device allocator of their own. */
int mde_dev_alloc(mde_ctx* ctx, uint64_t bytes, void** ptr);
int mde_dev_free(mde_ctx* ctx, void* ptr);
int mde_memcpy_h2d(mde_ctx* ctx, void* dst, const void* src, uint64_t bytes);
int mde_memcpy_d2h(mde_ctx* ctx, void* dst, const void* src, uint64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* MDE_H_ */
