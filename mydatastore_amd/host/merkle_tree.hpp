// merkle_tree.hpp -- C++ host mirror of andrew-delph/MyDataStore main/merkle_tree.go over the
// MI355X engine's C ABI (include/mde.h).
//
// The reference is Go and no Go toolchain exists in this image, so the host side of the drop-in
// is this C++ layer with the reference's names, argument meaning and error behaviour (errors are
// returned, never thrown, like Go's (value, error)). All hashing -- bucket byte-sums, SHA-256 tree
// nodes, key tagging, tree diffs -- runs in the engine's gfx950 kernels; this layer only moves
// bytes and mirrors the object shapes:
//
//   RawPartitionMerkleTree            main/merkle_tree.go:86-116   -> mde_build
//   MerkleTreeToPartitionEpochObject  main/merkle_tree.go:118-138  (leaf walk, host)
//   EpochTreeObjectToMerkleTree       main/merkle_tree.go:140-157  -> mde_tree_from_digests
//   DifferentMerkleTreeBuckets        main/merkle_tree.go:159-216  -> mde_diff
//   Manager.VerifyEpoch               main/manager.go:998-1118     -> mde_verify_epochs
//   Manager.GetEpochTreeLastValid     main/manager.go:838-867      -> mde_decode_epoch_tree_objects
//   CustomHash / MerkleBucket         main/merkle_tree.go:21-84
//   merkletree.MerkleTree / Node      cbergoon/merkletree v0.2.0 (Root, Leafs, MerkleRoot, Left,
//                                     Right, Hash, C)
// plus the slice of the storage/index layer the build reads (storage/storage.go:12-34,
// main/indexs.go:13-61, storage/index.go:41-110) and Manager.SetValue/GetValue
// (main/manager.go:773-836) so the reference's Merkle tests port one to one.
#pragma once

#include <stdint.h>

#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "mde.h"

namespace mds {

using Bytes = std::vector<uint8_t>;
using Error = std::string;  // empty == nil

constexpr int64_t hashMod = 999999;  // main/merkle_tree.go:19
constexpr int epochLength = 10;      // main/indexs.go:11

// ---------------------------------------------------------------- engine context (RAII)
class Engine {
 public:
  explicit Engine(int device = 0);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;
  bool ok() const { return ctx_ != nullptr; }
  const Error& init_error() const { return init_err_; }
  mde_ctx* ctx() const { return ctx_; }
  Error error(int rc) const;  // message for an MDE_E_* code

 private:
  mde_ctx* ctx_ = nullptr;
  Error init_err_;
};

// ---------------------------------------------------------------- utils/utils.go:67-89
Bytes EncodeInt64ToBytes(int64_t v);
Error DecodeBytesToInt64(const Bytes& b, int64_t* out);

// ---------------------------------------------------------------- main/merkle_tree.go:21-84
struct CustomHash {
  int64_t value = 0;
  int64_t Hash() const { return value; }
};

struct MerkleBucket {
  int32_t bucketId = 0;
  CustomHash hasher;
  int32_t size = 0;
  Bytes CalculateHash() const { return EncodeInt64ToBytes(hasher.Hash()); }
};

// ---------------------------------------------------------------- merkletree v0.2.0 shapes
struct Node {
  Node* Left = nullptr;
  Node* Right = nullptr;
  Bytes Hash;
  const MerkleBucket* C = nullptr;  // leaf content; nullptr for inner nodes
  bool leaf = false;
  bool dup = false;
};

class MerkleTree {
 public:
  MerkleTree() = default;
  MerkleTree(const MerkleTree&) = delete;  // nodes point into this object's own storage
  MerkleTree& operator=(const MerkleTree&) = delete;
  MerkleTree(MerkleTree&&) = default;      // deque moves keep element addresses
  MerkleTree& operator=(MerkleTree&&) = default;

  Node* Root = nullptr;
  std::vector<Node*> Leafs;  // includes the duplicate leaf when the bucket count is odd
  Bytes MerkleRoot() const { return Root ? Root->Hash : Bytes(); }

  uint32_t n_buckets() const { return (uint32_t)digests_.size(); }
  const std::vector<uint64_t>& digests() const { return digests_; }
  const Bytes& nodes() const { return nodes_; }  // internal nodes, level 1 .. root

  // Assemble the node graph from the engine's outputs (no hashing here).
  static MerkleTree FromDevice(std::vector<uint64_t> digests, std::vector<int32_t> sizes, Bytes nodes);

 private:
  std::vector<uint64_t> digests_;
  Bytes nodes_;
  std::deque<MerkleBucket> buckets_;
  std::deque<Node> pool_;
};

// ---------------------------------------------------------------- datap/data.proto:60-68
struct EpochTreeObject {
  int32_t Partition = 0;
  int64_t LowerEpoch = 0;
  int64_t UpperEpoch = 0;
  std::vector<Bytes> Buckets;
  std::vector<int32_t> BucketsSize;
  bool Valid = false;
  int32_t Items = 0;
};

// proto.Marshal / proto.Unmarshal of the object (main/manager.go:1045,1025), on the device.
Error MarshalEpochTreeObject(Engine& eng, const EpochTreeObject& obj, Bytes* out);
Error UnmarshalEpochTreeObject(Engine& eng, const Bytes& data, EpochTreeObject* out);

Error MerkleTreeToPartitionEpochObject(const MerkleTree& tree, int partitionId, int64_t lowerEpoch,
                                       int64_t upperEpoch, EpochTreeObject* out);
Error EpochTreeObjectToMerkleTree(Engine& eng, const EpochTreeObject& obj, MerkleTree* out);
Error DifferentMerkleTreeBuckets(Engine& eng, const MerkleTree& t1, const MerkleTree& t2,
                                 std::vector<int32_t>* out);

// ---------------------------------------------------------------- index keys
struct Column {
  std::string name, value;
  int length = -1;  // >= 0: OrderedColumn (zero-padded to length)
};
class Index {
 public:
  explicit Index(const std::string& name) { cols_.push_back({"name", name, -1}); }
  Index& AddColumn(const Column& c) { cols_.push_back(c); return *this; }
  Error Build(std::string* out) const;
  Error Parse(const std::string& s, std::map<std::string, std::string>* out) const;

 private:
  std::vector<Column> cols_;
};
inline Column CreateUnorderedColumn(const std::string& n, const std::string& v) { return {n, v, -1}; }
inline Column CreateOrderedColumn(const std::string& n, const std::string& v, int len) { return {n, v, len}; }

Error BuildEpochIndex(int partition, uint64_t bucket, int64_t epoch, const std::string& key, std::string* out);
Error ParseEpochIndex(const std::string& s, int* partition, uint64_t* bucket, int64_t* epoch, std::string* key);
Error BuildKeyIndex(const std::string& key, std::string* out);
Error BuildEpochTreeObjectIndex(int partition, int64_t epoch, std::string* out);

// ---------------------------------------------------------------- storage.Storage slice
// storage/badger_storage.go:79-130. Forward: Seek(Start), then ascending keys until one is
// >= Limit. Reverse (reverse = true): Seek(Limit) -- the largest key <= Limit -- then descending
// keys; IsDone still tests only key >= Limit, so a reverse scan is NOT bounded below by Start
// (it walks on into smaller keys, e.g. other partitions' objects) and a key equal to Limit ends
// it at once. Reproduced as the reference behaves.
class Iterator {
 public:
  Iterator(const std::map<std::string, Bytes>* m, const std::string& start, const std::string& limit,
           bool reverse = false);
  bool IsDone() const;
  bool Next();
  const std::string& Key() const { return it_->first; }
  Bytes Value() const { return it_->second; }  // a copy, like Badger's ValueCopy

 private:
  const std::map<std::string, Bytes>* m_;
  std::map<std::string, Bytes>::const_iterator it_;
  std::string limit_;
  bool reverse_ = false;
  bool valid_ = true;
};

class MemStorage {  // ordered KV with Badger iterator semantics (storage/badger_storage.go:79-130)
 public:
  void Put(const std::string& k, const Bytes& v) { kv_[k] = v; }
  bool Get(const std::string& k, Bytes* v) const;
  Iterator NewIterator(const std::string& start, const std::string& limit, bool reverse = false) const {
    return Iterator(&kv_, start, limit, reverse);
  }
  size_t size() const { return kv_.size(); }

 private:
  std::map<std::string, Bytes> kv_;
};

struct Value {  // rpc.RpcValue
  std::string Key, Val;
  int64_t Epoch = 0;
  int64_t UnixTimestamp = 0;
};

// ---------------------------------------------------------------- Manager slice
class Manager {
 public:
  Manager(Engine& eng, int partitionCount, int partitionBuckets)
      : eng_(eng), partitionCount_(partitionCount), partitionBuckets_(partitionBuckets) {}

  Error SetValue(const Value& v);                       // main/manager.go:780-818
  Error GetValue(const std::string& key, Value* out);   // main/manager.go:820-836
  // main/merkle_tree.go:86-116, on the device.
  Error RawPartitionMerkleTree(int partitionId, int64_t lowerEpoch, int64_t upperEpoch, MerkleTree* out);
  // Batched form: one engine call for many partitions (what a coalescing caller uses).
  Error RawPartitionMerkleTrees(const std::vector<int>& partitionIds, int64_t lowerEpoch,
                                int64_t upperEpoch, std::vector<MerkleTree>* out);
  // Tagging through the engine (getKeyBucket main/manager.go:773-778, FindPartitionID).
  Error KeyTags(const std::string& key, uint64_t* bucket, int* partition);

  // StreamBucketsTask (main/manager.go:445-487): every record (key, epoch, timestamp) of the
  // listed buckets of a partition in [LowerEpoch, UpperEpoch); an empty list means all buckets.
  // The range scans fill one arena and the device (mde_stream_buckets) gathers the records in the
  // task's own order: the buckets as listed, a repeated bucket streamed again, an id outside
  // [0, PartitionBuckets) streaming nothing, LSM order inside a bucket.
  Error StreamBuckets(int PartitionId, const std::vector<int32_t>& Buckets, int64_t LowerEpoch,
                      int64_t UpperEpoch, std::vector<Value>* out);

  // Manager.VerifyEpoch (main/manager.go:998-1118) without the network: peerObjects are the wire
  // bytes EpochTreeObjectRequest (:729-771) returned for this partition and epoch. Returns nil
  // when the epoch object is (or already was) valid, else the reference's "validCount= ..." error;
  // *out carries the decision and diffSet.List() (ascending), the bucket list
  // PoliteStreamRequest would ask for. The object persisted under epochtree_{p}_{E} is the one the
  // reference leaves there.
  struct VerifyResult {
    bool Valid = false;
    bool AlreadyValid = false;  // stored object already valid: early return (:1020-1027)
    int ValidCount = 0;
    int Trees = 0;              // peer objects considered
    std::vector<int32_t> DiffSet;
  };
  Error VerifyEpoch(int PartitionId, int64_t Epoch, const std::vector<Bytes>& peerObjects, int replicaCount,
                    VerifyResult* out);
  // Batched: one build and one verify call for many partitions of the same epoch.
  Error VerifyEpochs(const std::vector<int>& partitionIds, int64_t Epoch,
                     const std::vector<std::vector<Bytes>>& peerObjects, int replicaCount,
                     std::vector<VerifyResult>* out, std::vector<Error>* errs);

  // Manager.GetEpochTreeLastValid (main/manager.go:838-867): the newest stored EpochTreeObject
  // with Valid set, scanning epochtree_{p}_ keys downward from CurrentEpoch (reverse iterator,
  // with its unbounded-below quirk); none found -> {Partition: p, LowerEpoch: -1, UpperEpoch: -1}.
  // The stored objects are decoded by the engine's wire decoder.
  Error GetEpochTreeLastValid(int32_t partitionId, EpochTreeObject* out);
  int64_t CurrentEpoch = 0;

  MemStorage& db() { return db_; }
  int PartitionBuckets() const { return partitionBuckets_; }

 private:
  // The per-bucket range scans of main/merkle_tree.go:90-113 for several partitions, copied into
  // one layout-A arena (values, value_off, seg_rec); keys (optional) receives each record's
  // epoch-index key.
  Error ScanArena(const std::vector<int>& partitionIds, int64_t lowerEpoch, int64_t upperEpoch, Bytes* arena,
                  std::vector<uint64_t>* value_off, std::vector<uint64_t>* seg_rec,
                  std::vector<std::string>* keys) const;

  Engine& eng_;
  int partitionCount_, partitionBuckets_;
  MemStorage db_;
};

}  // namespace mds
