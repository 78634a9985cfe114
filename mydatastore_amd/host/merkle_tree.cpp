// merkle_tree.cpp -- see merkle_tree.hpp. Host-side object plumbing only; every hash is computed
// by the engine (libmde.so).
#include "merkle_tree.hpp"

#include <algorithm>

#include <cstdio>
#include <cstring>

namespace mds {

// ---------------------------------------------------------------- Engine
Engine::Engine(int device) {
  int rc = mde_create(device, &ctx_);
  if (rc != MDE_OK) {
    ctx_ = nullptr;
    init_err_ = std::string("mde_create failed: ") + mde_strerror(rc);
  }
}

Engine::~Engine() {
  if (ctx_) mde_destroy(ctx_);
}

Error Engine::error(int rc) const {
  char m[512] = {0};
  if (ctx_) mde_last_error_copy(ctx_, m, sizeof m);
  return std::string(mde_strerror(rc)) + (*m ? std::string(": ") + m : std::string());
}

// ---------------------------------------------------------------- utils/utils.go:67-89
Bytes EncodeInt64ToBytes(int64_t v) {
  Bytes b(8);
  const uint64_t u = (uint64_t)v;
  for (int k = 0; k < 8; k++) b[k] = (uint8_t)(u >> (8 * k));
  return b;
}

Error DecodeBytesToInt64(const Bytes& b, int64_t* out) {
  if (b.size() != 8) return "byte slice should be 8 bytes long for int64 decoding";
  uint64_t u = 0;
  for (int k = 7; k >= 0; k--) u = (u << 8) | b[k];
  *out = (int64_t)u;
  return "";
}

// ---------------------------------------------------------------- MerkleTree
MerkleTree MerkleTree::FromDevice(std::vector<uint64_t> digests, std::vector<int32_t> sizes, Bytes nodes) {
  MerkleTree t;
  const uint32_t B = (uint32_t)digests.size();
  t.digests_ = std::move(digests);
  t.nodes_ = std::move(nodes);
  for (uint32_t b = 0; b < B; b++) {
    MerkleBucket mb;
    mb.bucketId = (int32_t)b;
    mb.hasher.value = (int64_t)t.digests_[b];
    mb.size = b < sizes.size() ? sizes[b] : 0;
    t.buckets_.push_back(mb);
  }
  // level 0: leaves (+ duplicate of the last leaf when B is odd -- merkletree buildWithContent)
  std::vector<Node*> level;
  for (uint32_t b = 0; b < B; b++) {
    t.pool_.push_back(Node{nullptr, nullptr, t.buckets_[b].CalculateHash(), &t.buckets_[b], true, false});
    level.push_back(&t.pool_.back());
  }
  if (B % 2 == 1) {
    t.pool_.push_back(Node{nullptr, nullptr, level.back()->Hash, level.back()->C, true, true});
    level.push_back(&t.pool_.back());
  }
  t.Leafs = level;
  // inner levels: hashes come from the device's node array (level 1 .. root, 32 B each)
  uint64_t off = 0;
  while (level.size() > 1) {
    std::vector<Node*> up;
    const size_t n = level.size(), m = (n + 1) / 2;
    for (size_t j = 0; j < m; j++) {
      Node nd;
      nd.Left = level[2 * j];
      nd.Right = (2 * j + 1 < n) ? level[2 * j + 1] : level[2 * j];
      if ((off + j + 1) * 32 <= t.nodes_.size())
        nd.Hash.assign(t.nodes_.begin() + (off + j) * 32, t.nodes_.begin() + (off + j + 1) * 32);
      t.pool_.push_back(nd);
      up.push_back(&t.pool_.back());
    }
    off += m;
    level.swap(up);
  }
  t.Root = level.empty() ? nullptr : level[0];
  return t;
}

// ---------------------------------------------------------------- main/merkle_tree.go:118-157
Error MerkleTreeToPartitionEpochObject(const MerkleTree& tree, int partitionId, int64_t lowerEpoch,
                                       int64_t upperEpoch, EpochTreeObject* out) {
  EpochTreeObject o;
  uint32_t items = 0;
  for (const Node* leaf : tree.Leafs) {
    if (!leaf->C) return "failed to decode MerkleBucket";
    o.Buckets.push_back(leaf->C->CalculateHash());
    o.BucketsSize.push_back(leaf->C->size);
    items += (uint32_t)leaf->C->size;  // int32 arithmetic wraps like Go
  }
  o.Partition = partitionId;
  o.LowerEpoch = lowerEpoch;
  o.UpperEpoch = upperEpoch;
  o.Items = (int32_t)items;
  *out = std::move(o);
  return "";
}

Error EpochTreeObjectToMerkleTree(Engine& eng, const EpochTreeObject& obj, MerkleTree* out) {
  const uint32_t B = (uint32_t)obj.Buckets.size();
  if (B == 0) return "error: cannot construct tree with no content";
  std::vector<const uint8_t*> ptrs(B);
  std::vector<uint32_t> lens(B);
  for (uint32_t i = 0; i < B; i++) {
    ptrs[i] = obj.Buckets[i].data();
    lens[i] = (uint32_t)obj.Buckets[i].size();
  }
  std::vector<uint64_t> digests(B);
  int rc = mde_decode_bucket_hashes(ptrs.data(), lens.data(), B, digests.data());
  if (rc != MDE_OK) return "byte slice should be 8 bytes long for int64 decoding";
  std::vector<int32_t> sizes(B, 0);
  for (uint32_t i = 0; i < B && i < obj.BucketsSize.size(); i++) sizes[i] = obj.BucketsSize[i];
  Bytes root(32), nodes(mde_tree_internal_nodes(B) * 32);
  rc = mde_tree_from_digests(eng.ctx(), 1, B, digests.data(), root.data(), nodes.data());
  if (rc != MDE_OK) return eng.error(rc);
  *out = MerkleTree::FromDevice(std::move(digests), std::move(sizes), std::move(nodes));
  return "";
}

Error DifferentMerkleTreeBuckets(Engine& eng, const MerkleTree& t1, const MerkleTree& t2,
                                 std::vector<int32_t>* out) {
  if (!t1.Root && !t2.Root) { out->clear(); return ""; }
  if (!t1.Root || !t2.Root) return "a merkletree.Node is nil";
  const uint64_t cap = mde_diff_capacity(t1.n_buckets(), t2.n_buckets());
  std::vector<int32_t> ids(cap);
  int32_t count = 0;
  int rc = mde_diff(eng.ctx(), 1, t1.n_buckets(), t1.digests().data(), t1.nodes().data(),
                    t2.n_buckets(), t2.digests().data(), t2.nodes().data(), ids.data(), cap, &count);
  if (rc != MDE_OK) return eng.error(rc);
  if (count == MDE_E_TREE) return "bucketIds dont match (or a merkletree.Node is nil)";
  if (count < 0) return std::string("diff failed: ") + mde_strerror(count);
  ids.resize((size_t)count);
  *out = std::move(ids);
  return "";
}

Error MarshalEpochTreeObject(Engine& eng, const EpochTreeObject& obj, Bytes* out) {
  const uint32_t L = (uint32_t)obj.Buckets.size();  // 0: an object without buckets (scalars only)
  std::vector<uint64_t> digest(L + 1);
  std::vector<int32_t> size(L + 1, 0);
  for (uint32_t i = 0; i < L; i++) {
    int64_t v;
    Error e = DecodeBytesToInt64(obj.Buckets[i], &v);
    if (!e.empty()) return e;
    digest[i] = (uint64_t)v;
    if (i < obj.BucketsSize.size()) size[i] = obj.BucketsSize[i];
  }
  // The object holds tree.Leafs, whose count is always even (merkletree duplicates the last leaf
  // of an odd B), so its L leaves are encoded as B = L buckets with no further duplicate.
  const uint8_t valid = obj.Valid ? 1 : 0;
  const int32_t part = obj.Partition, items = obj.Items;
  const uint32_t B = L;
  if (L % 2 == 1) return "EpochTreeObject with an odd leaf count cannot come from a merkletree";
  const uint64_t stride = mde_epoch_tree_object_max_bytes(B);
  Bytes buf(stride);
  uint32_t len = 0;
  int rc = mde_encode_epoch_tree_objects(eng.ctx(), 1, B, &part, obj.LowerEpoch, obj.UpperEpoch,
                                         digest.data(), size.data(), &valid, &items, buf.data(),
                                         stride, &len);
  if (rc != MDE_OK) return eng.error(rc);
  buf.resize(len);
  *out = std::move(buf);
  return "";
}

Error UnmarshalEpochTreeObject(Engine& eng, const Bytes& data, EpochTreeObject* out) {
  const uint64_t off[2] = {0, data.size()};
  const uint32_t cap = (uint32_t)(data.size() / 10 + 1);
  std::vector<uint64_t> digest(cap);
  std::vector<int32_t> size(cap);
  int32_t part = 0, items = 0, nb = 0;
  int64_t lo = 0, hi = 0;
  uint8_t valid = 0;
  const uint8_t dummy = 0;
  int rc = mde_decode_epoch_tree_objects(eng.ctx(), 1, data.empty() ? &dummy : data.data(), off, cap,
                                         &part, &lo, &hi, digest.data(), size.data(), &valid, &items, &nb);
  if (rc != MDE_OK) return eng.error(rc);
  if (nb < 0) return std::string("proto: cannot parse EpochTreeObject: ") + mde_strerror(nb);
  EpochTreeObject o;
  o.Partition = part;
  o.LowerEpoch = lo;
  o.UpperEpoch = hi;
  o.Valid = valid != 0;
  o.Items = items;
  for (int32_t i = 0; i < nb; i++) {
    o.Buckets.push_back(EncodeInt64ToBytes((int64_t)digest[i]));
    o.BucketsSize.push_back(size[i]);
  }
  *out = std::move(o);
  return "";
}

// ---------------------------------------------------------------- index keys
Error Index::Build(std::string* out) const {
  std::string s;
  for (size_t i = 0; i < cols_.size(); i++) {
    std::string v = cols_[i].value;
    if (cols_[i].length >= 0) {
      if ((int)v.size() > cols_[i].length) return "index value invalid length " + std::to_string(v.size());
      v = std::string(cols_[i].length - v.size(), '0') + v;
    }
    if (i) s += "_";
    s += v;
  }
  *out = s;
  return "";
}

Error Index::Parse(const std::string& s, std::map<std::string, std::string>* out) const {
  std::vector<std::string> parts;
  size_t start = 0;
  for (;;) {
    size_t p = s.find('_', start);
    parts.push_back(s.substr(start, p == std::string::npos ? std::string::npos : p - start));
    if (p == std::string::npos) break;
    start = p + 1;
  }
  if (parts.size() != cols_.size())
    return "index columns #" + std::to_string(cols_.size() + 1) + " and parts #" + std::to_string(parts.size()) + " not equal";
  out->clear();
  for (size_t i = cols_.size(); i-- > 0;) {
    std::string v = parts[i];
    if (cols_[i].length >= 0) {
      size_t nz = v.find_first_not_of('0');
      v = nz == std::string::npos ? "0" : v.substr(nz);
    }
    (*out)[cols_[i].name] = v;
  }
  return "";
}

Error BuildEpochIndex(int partition, uint64_t bucket, int64_t epoch, const std::string& key, std::string* out) {
  return Index("epoch")
      .AddColumn(CreateUnorderedColumn("parition", std::to_string(partition)))
      .AddColumn(CreateUnorderedColumn("bucket", std::to_string(bucket)))
      .AddColumn(CreateOrderedColumn("epoch", std::to_string(epoch), epochLength))
      .AddColumn(CreateUnorderedColumn("key", key))
      .Build(out);
}

Error ParseEpochIndex(const std::string& s, int* partition, uint64_t* bucket, int64_t* epoch, std::string* key) {
  std::map<std::string, std::string> m;
  Error e = Index("epoch")
                .AddColumn(CreateUnorderedColumn("parition", "1"))
                .AddColumn(CreateUnorderedColumn("bucket", "1"))
                .AddColumn(CreateOrderedColumn("epoch", "1", epochLength))
                .AddColumn(CreateUnorderedColumn("key", "1"))
                .Parse(s, &m);
  if (!e.empty()) return e;
  if (m["name"] != "epoch") return "index name is wrong";
  try {
    *partition = std::stoi(m["parition"]);
    *bucket = std::stoull(m["bucket"]);
    *epoch = std::stoll(m["epoch"]);
  } catch (...) {
    return "invalid syntax";
  }
  *key = m["key"];
  return "";
}

Error BuildKeyIndex(const std::string& key, std::string* out) {
  return Index("item").AddColumn(CreateUnorderedColumn("key", key)).Build(out);
}

Error BuildEpochTreeObjectIndex(int partition, int64_t epoch, std::string* out) {
  return Index("epochtree")
      .AddColumn(CreateUnorderedColumn("partition", std::to_string(partition)))
      .AddColumn(CreateOrderedColumn("epoch", std::to_string(epoch), epochLength))
      .Build(out);
}

// ---------------------------------------------------------------- storage slice
Iterator::Iterator(const std::map<std::string, Bytes>* m, const std::string& start, const std::string& limit,
                   bool reverse)
    : m_(m), limit_(limit), reverse_(reverse) {
  if (!reverse) {
    it_ = m->lower_bound(start);
  } else {  // badger reverse Seek(Limit): the largest key <= Limit
    it_ = m->upper_bound(limit);
    if (it_ == m->begin()) valid_ = false;
    else --it_;
  }
}

bool Iterator::IsDone() const { return !valid_ || it_ == m_->end() || it_->first.compare(limit_) >= 0; }

bool Iterator::Next() {
  if (!reverse_) {
    ++it_;
  } else if (valid_) {
    if (it_ == m_->begin()) valid_ = false;
    else --it_;
  }
  return !IsDone();
}

bool MemStorage::Get(const std::string& k, Bytes* v) const {
  auto it = kv_.find(k);
  if (it == kv_.end()) return false;
  *v = it->second;
  return true;
}

// ---------------------------------------------------------------- Manager slice
Error Manager::GetEpochTreeLastValid(int32_t partitionId, EpochTreeObject* out) {
  std::string index1, index2;
  Error e = BuildEpochTreeObjectIndex(partitionId, 0, &index1);
  if (!e.empty()) return "BuildEpochTreeObjectIndex: " + e;
  e = BuildEpochTreeObjectIndex(partitionId, CurrentEpoch, &index2);
  if (!e.empty()) return "BuildEpochTreeObjectIndex: " + e;
  for (Iterator it = db_.NewIterator(index1, index2, true); !it.IsDone(); it.Next()) {
    EpochTreeObject obj;
    e = UnmarshalEpochTreeObject(eng_, it.Value(), &obj);
    if (!e.empty()) return "RpcEpochTreeObject Unmarshal: " + e;
    if (obj.Valid) {
      *out = std::move(obj);
      return "";
    }
  }
  EpochTreeObject none;
  none.Partition = partitionId;
  none.LowerEpoch = -1;
  none.UpperEpoch = -1;
  *out = std::move(none);
  return "";
}

Error Manager::KeyTags(const std::string& key, uint64_t* bucket, int* partition) {
  const uint64_t off[2] = {0, key.size()};
  uint32_t b = 0, p = 0;
  int rc = mde_tag_keys(eng_.ctx(), reinterpret_cast<const uint8_t*>(key.data()), off, 1,
                        (uint32_t)partitionBuckets_, (uint32_t)partitionCount_, &b, &p);
  if (rc != MDE_OK) return eng_.error(rc);
  *bucket = b;
  *partition = (int)p;
  return "";
}

static Bytes encode_item(const Value& v) {  // item_{key} record: epoch, timestamp, value bytes
  Bytes b = EncodeInt64ToBytes(v.Epoch), t = EncodeInt64ToBytes(v.UnixTimestamp);
  b.insert(b.end(), t.begin(), t.end());
  b.insert(b.end(), v.Val.begin(), v.Val.end());
  return b;
}

static void decode_item(const std::string& key, const Bytes& b, Value* v) {
  v->Key = key;
  DecodeBytesToInt64(Bytes(b.begin(), b.begin() + 8), &v->Epoch);
  DecodeBytesToInt64(Bytes(b.begin() + 8, b.begin() + 16), &v->UnixTimestamp);
  v->Val.assign(b.begin() + 16, b.end());
}

Error Manager::SetValue(const Value& v) {
  uint64_t bucket;
  int partition;
  Error e = KeyTags(v.Key, &bucket, &partition);
  if (!e.empty()) return e;
  std::string epochIndex, keyIndex;
  if (!(e = BuildEpochIndex(partition, bucket, v.Epoch, v.Key, &epochIndex)).empty()) return e;
  if (!(e = BuildKeyIndex(v.Key, &keyIndex)).empty()) return e;
  Bytes existing;
  if (db_.Get(keyIndex, &existing)) {
    Value ev;
    decode_item(v.Key, existing, &ev);
    if (ev.Epoch >= v.Epoch && ev.UnixTimestamp > v.UnixTimestamp) return "a newer value already exists";
  }
  db_.Put(keyIndex, encode_item(v));
  db_.Put(epochIndex, EncodeInt64ToBytes(v.UnixTimestamp));
  return "";
}

Error Manager::GetValue(const std::string& key, Value* out) {
  std::string keyIndex;
  Error e = BuildKeyIndex(key, &keyIndex);
  if (!e.empty()) return e;
  Bytes b;
  if (!db_.Get(keyIndex, &b)) return "KEY_NOT_FOUND";
  decode_item(key, b, out);
  return "";
}

Error Manager::ScanArena(const std::vector<int>& partitionIds, int64_t lowerEpoch, int64_t upperEpoch,
                         Bytes* arena, std::vector<uint64_t>* value_off, std::vector<uint64_t>* seg_rec,
                         std::vector<std::string>* keys) const {
  // Ingest: the per-bucket range scans of main/merkle_tree.go:90-113 copy each record's value into
  // one contiguous arena (layout A); seg_rec marks the bucket boundaries.
  const uint32_t B = (uint32_t)partitionBuckets_;
  arena->clear();
  *value_off = {0};
  *seg_rec = {0};
  if (keys) keys->clear();
  for (int p : partitionIds) {
    for (uint32_t b = 0; b < B; b++) {
      std::string i1, i2;
      Error e = BuildEpochIndex(p, b, lowerEpoch, "", &i1);
      if (!e.empty()) return e;
      if (!(e = BuildEpochIndex(p, b, upperEpoch, "", &i2)).empty()) return e;
      for (Iterator it = db_.NewIterator(i1, i2); !it.IsDone(); it.Next()) {
        const Bytes v = it.Value();
        arena->insert(arena->end(), v.begin(), v.end());
        value_off->push_back(arena->size());
        if (keys) keys->push_back(it.Key());
      }
      seg_rec->push_back(value_off->size() - 1);
    }
  }
  if (arena->empty()) arena->push_back(0);  // keep a valid pointer for an all-empty build
  return "";
}

Error Manager::StreamBuckets(int PartitionId, const std::vector<int32_t>& Buckets, int64_t LowerEpoch,
                             int64_t UpperEpoch, std::vector<Value>* out) {
  out->clear();
  const uint32_t B = (uint32_t)partitionBuckets_;
  Bytes arena;
  std::vector<uint64_t> value_off, seg_rec;
  std::vector<std::string> keys;
  Error e = ScanArena({PartitionId}, LowerEpoch, UpperEpoch, &arena, &value_off, &seg_rec, &keys);
  if (!e.empty()) return e;
  mde_records rec{};
  rec.values = arena.data();
  rec.values_bytes = arena.size();
  rec.value_off = value_off.data();
  rec.n_records = value_off.size() - 1;
  rec.n_partitions = 1;
  rec.n_buckets = B;
  rec.seg_rec = seg_rec.data();
  // the task's list as given (main/manager.go:447-453): an empty list is every bucket (count 0),
  // a repeat streams its bucket again, an id outside [0, B) streams nothing -- the capacities
  // cover every request's run
  uint64_t need_rec = 0, need_bytes = 0;
  for (uint32_t i = 0; i < (Buckets.empty() ? B : (uint32_t)Buckets.size()); i++) {
    const int64_t b = Buckets.empty() ? (int64_t)i : (int64_t)Buckets[i];
    if (b < 0 || b >= (int64_t)B) continue;
    need_rec += seg_rec[b + 1] - seg_rec[b];
    need_bytes += value_off[seg_rec[b + 1]] - value_off[seg_rec[b]];
  }
  const uint64_t cap = need_rec ? need_rec : 1, bcap = need_bytes ? need_bytes : 1;
  const int32_t count = (int32_t)Buckets.size();
  const int32_t none = 0;
  std::vector<uint64_t> part_off(2), out_rec(cap), out_voff(cap + 1);
  Bytes out_vals(bcap);
  int rc = mde_stream_buckets(eng_.ctx(), &rec, Buckets.empty() ? &none : Buckets.data(), Buckets.size(), &count,
                              part_off.data(), out_rec.data(), cap, out_vals.data(), out_voff.data(), bcap);
  if (rc != MDE_OK) return eng_.error(rc);
  for (uint64_t i = 0; i < part_off[1]; i++) {
    int p;
    uint64_t b;
    Value v;
    if (!(e = ParseEpochIndex(keys[out_rec[i]], &p, &b, &v.Epoch, &v.Key)).empty()) return e;
    const Bytes ts(out_vals.begin() + out_voff[i], out_vals.begin() + out_voff[i + 1]);
    if (!(e = DecodeBytesToInt64(ts, &v.UnixTimestamp)).empty()) return e;
    out->push_back(v);
  }
  return "";
}

Error Manager::RawPartitionMerkleTree(int partitionId, int64_t lowerEpoch, int64_t upperEpoch, MerkleTree* out) {
  std::vector<MerkleTree> trees;
  Error e = RawPartitionMerkleTrees({partitionId}, lowerEpoch, upperEpoch, &trees);
  if (!e.empty()) return e;
  *out = std::move(trees[0]);
  return "";
}

Error Manager::RawPartitionMerkleTrees(const std::vector<int>& partitionIds, int64_t lowerEpoch,
                                       int64_t upperEpoch, std::vector<MerkleTree>* out) {
  const uint32_t B = (uint32_t)partitionBuckets_, P = (uint32_t)partitionIds.size();
  Bytes arena;
  std::vector<uint64_t> value_off, seg_rec;
  Error se = ScanArena(partitionIds, lowerEpoch, upperEpoch, &arena, &value_off, &seg_rec, nullptr);
  if (!se.empty()) return se;
  mde_records rec{};
  rec.values = arena.data();
  rec.values_bytes = arena.size();
  rec.value_stride = 0;
  rec.value_off = value_off.data();
  rec.n_records = value_off.size() - 1;
  rec.n_partitions = P;
  rec.n_buckets = B;
  rec.seg_rec = seg_rec.data();
  const uint64_t NI = mde_tree_internal_nodes(B);
  std::vector<uint64_t> digest((size_t)P * B);
  std::vector<int32_t> size((size_t)P * B), items(P);
  Bytes root((size_t)P * 32), nodes((size_t)P * NI * 32);
  mde_tree_out o{digest.data(), size.data(), items.data(), root.data(), nodes.data()};
  int rc = mde_build(eng_.ctx(), &rec, &o);
  if (rc != MDE_OK) return eng_.error(rc);
  out->clear();
  for (uint32_t i = 0; i < P; i++) {
    out->push_back(MerkleTree::FromDevice(
        std::vector<uint64_t>(digest.begin() + (size_t)i * B, digest.begin() + (size_t)(i + 1) * B),
        std::vector<int32_t>(size.begin() + (size_t)i * B, size.begin() + (size_t)(i + 1) * B),
        Bytes(nodes.begin() + (size_t)i * NI * 32, nodes.begin() + (size_t)(i + 1) * NI * 32)));
  }
  return "";
}

Error Manager::VerifyEpoch(int PartitionId, int64_t Epoch, const std::vector<Bytes>& peerObjects,
                           int replicaCount, VerifyResult* out) {
  std::vector<VerifyResult> res;
  std::vector<Error> errs;
  Error e = VerifyEpochs({PartitionId}, Epoch, {peerObjects}, replicaCount, &res, &errs);
  if (!e.empty()) return e;
  *out = res[0];
  return errs[0];
}

Error Manager::VerifyEpochs(const std::vector<int>& partitionIds, int64_t Epoch,
                            const std::vector<std::vector<Bytes>>& peerObjects, int replicaCount,
                            std::vector<VerifyResult>* out, std::vector<Error>* errs) {
  const size_t N = partitionIds.size();
  if (peerObjects.size() != N) return "one peer list per partition";
  out->assign(N, VerifyResult{});
  errs->assign(N, "");
  if (Epoch < 0) return "";  // :1006-1008
  // Early return when the stored object is already valid (:1015-1027).
  std::vector<int> todo_parts;
  std::vector<size_t> todo;
  std::vector<std::string> index(N);
  for (size_t i = 0; i < N; i++) {
    Error e = BuildEpochTreeObjectIndex(partitionIds[i], Epoch, &index[i]);
    if (!e.empty()) return e;
    Bytes stored;
    EpochTreeObject obj;
    if (db_.Get(index[i], &stored) && UnmarshalEpochTreeObject(eng_, stored, &obj).empty() && obj.Valid) {
      (*out)[i].Valid = (*out)[i].AlreadyValid = true;
      continue;
    }
    todo.push_back(i);
    todo_parts.push_back(partitionIds[i]);
  }
  if (todo.empty()) return "";
  // myTree = RawPartitionMerkleTree(p, E, E+1) for every partition at once (:1036).
  std::vector<MerkleTree> trees;
  Error e = RawPartitionMerkleTrees(todo_parts, Epoch, Epoch + 1, &trees);
  if (!e.empty()) return e;
  const uint32_t P = (uint32_t)todo.size(), B = (uint32_t)partitionBuckets_;
  const uint64_t NI = mde_tree_internal_nodes(B);
  size_t R = 0;
  for (size_t i : todo) R = std::max(R, peerObjects[i].size());
  std::vector<uint64_t> digest((size_t)P * B);
  std::vector<int32_t> size((size_t)P * B), part(P);
  Bytes nodes((size_t)P * NI * 32), blob;
  std::vector<uint64_t> off{0};
  for (uint32_t k = 0; k < P; k++) {
    const MerkleTree& t = trees[k];
    std::copy(t.digests().begin(), t.digests().end(), digest.begin() + (size_t)k * B);
    for (uint32_t b = 0; b < B; b++) size[(size_t)k * B + b] = t.Leafs[b]->C->size;
    std::copy(t.nodes().begin(), t.nodes().end(), nodes.begin() + (size_t)k * NI * 32);
    part[k] = todo_parts[k];
    const std::vector<Bytes>& peers = peerObjects[todo[k]];
    for (size_t r = 0; r < R; r++) {  // a missing peer is an empty object: it yields no tree
      if (r < peers.size()) blob.insert(blob.end(), peers[r].begin(), peers[r].end());
      off.push_back(blob.size());
    }
  }
  std::vector<uint8_t> valid(P);
  std::vector<int32_t> vcount(P), ids((size_t)P * B), dcount(P), status((size_t)P * R + 1);
  const uint64_t stride = mde_epoch_tree_object_max_bytes(B);
  Bytes objs((size_t)P * stride);
  std::vector<uint32_t> olen(P);
  int rc = mde_verify_epochs(eng_.ctx(), P, B, part.data(), Epoch, digest.data(), size.data(), nodes.data(),
                             (uint32_t)R, blob.data(), off.data(), (uint32_t)replicaCount, valid.data(),
                             vcount.data(), ids.data(), dcount.data(), status.data(), objs.data(), stride,
                             olen.data());
  if (rc != MDE_OK) return eng_.error(rc);
  for (uint32_t k = 0; k < P; k++) {
    VerifyResult& v = (*out)[todo[k]];
    v.Valid = valid[k] != 0;
    v.ValidCount = vcount[k];
    v.Trees = (int)peerObjects[todo[k]].size();
    v.DiffSet.assign(ids.begin() + (size_t)k * B, ids.begin() + (size_t)k * B + dcount[k]);
    // persist the epoch object (:1049, :1102): Valid set when verified
    db_.Put(index[todo[k]], Bytes(objs.begin() + (size_t)k * stride, objs.begin() + (size_t)k * stride + olen[k]));
    if (!v.Valid)
      (*errs)[todo[k]] = "validCount= " + std::to_string(v.ValidCount) + "<" + std::to_string(replicaCount) +
                         " Epoch " + std::to_string(Epoch) + " trees " + std::to_string(v.Trees) +
                         " diffSet= " + std::to_string(v.DiffSet.size());
  }
  return "";
}

}  // namespace mds
