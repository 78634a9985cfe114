// test_merkle_tree.cpp -- C++ port of the reference's tests for the Merkle path, run against the
// host mirror (mydatastore_amd/host) over the MI355X engine:
//   TestMerkleTreeRaw   main/merkle_tree_test.go:15-185 (N = 100 and the -test.short N = 10)
//   TestIndexManager    main/indexs_test.go:9-41
//   TestIndexStorage    storage/index_test.go:9-40
//   TestManagerStorage  main/manager_test.go:30-115 (range-iteration counts)
//   TestGetEpochTreeLastValidObjectTask  main/manager_test.go:213-301
// Prints "ROOT <name> <hex>" lines (checked against tests/golden by tests/test_cpp_port.py) and
// exits non-zero on the first failed assertion.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "merkle_tree.hpp"

using namespace mds;

static int failures = 0;
#define CHECK(cond, msg)                                                            \
  do {                                                                              \
    if (!(cond)) {                                                                  \
      std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, msg, #cond); \
      failures++;                                                                   \
    }                                                                               \
  } while (0)
#define CHECK_OK(err)                                                                       \
  do {                                                                                      \
    Error e_ = (err);                                                                       \
    if (!e_.empty()) {                                                                      \
      std::fprintf(stderr, "FAIL %s:%d: error: %s\n", __FILE__, __LINE__, e_.c_str());      \
      failures++;                                                                           \
    }                                                                                       \
  } while (0)

static std::string hex(const Bytes& b) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (uint8_t x : b) { s += d[x >> 4]; s += d[x & 15]; }
  return s;
}

static std::string ids(const std::vector<int32_t>& v) {
  std::string s;
  for (size_t i = 0; i < v.size(); i++) s += (i ? "," : "") + std::to_string(v[i]);
  return s;
}

static void TestMerkleTreeRaw(Engine& eng, int writeValuesNum) {
  Manager manager(eng, /*PartitionCount=*/1, /*PartitionBuckets=*/30);
  int64_t timestamp = 0;
  for (int i = 0; i < writeValuesNum; i++) {  // write to epoch 1
    timestamp++;
    Value v{"key" + std::to_string(i), "val" + std::to_string(i), 1, timestamp};
    CHECK_OK(manager.SetValue(v));
    Value got;
    CHECK_OK(manager.GetValue(v.Key, &got));
    CHECK(got.Val == v.Val, "get value is wrong");
  }
  for (int i = 0; i < writeValuesNum; i++) {  // write to epoch 2
    timestamp++;
    Value v{"keyz" + std::to_string(i), "valz" + std::to_string(i), 2, timestamp};
    CHECK_OK(manager.SetValue(v));
    Value got;
    CHECK_OK(manager.GetValue(v.Key, &got));
    CHECK(got.Val == v.Val, "get value is wrong");
  }
  MerkleTree tree1, tree2, tree3;
  CHECK_OK(manager.RawPartitionMerkleTree(0, 0, 3, &tree1));
  CHECK_OK(manager.RawPartitionMerkleTree(0, 1, 3, &tree2));
  CHECK_OK(manager.RawPartitionMerkleTree(0, 2, 3, &tree3));

  CHECK(tree1.Leafs.size() == 30, "confirm leafs num is the same as PartitionBuckets");
  CHECK(tree2.Leafs.size() == 30, "confirm leafs num is the same as PartitionBuckets");
  CHECK(tree3.Leafs.size() == 30, "confirm leafs num is the same as PartitionBuckets");
  CHECK(tree1.MerkleRoot() == tree2.MerkleRoot(), "hash should be the same");
  CHECK(tree1.MerkleRoot() != tree3.MerkleRoot(), "hash should be different");
  CHECK(tree2.MerkleRoot() != tree3.MerkleRoot(), "hash should be different");
  for (const MerkleTree* t : {&tree1, &tree2, &tree3})
    for (size_t i = 0; i < t->Leafs.size(); i++)
      CHECK(t->Leafs[i]->C && t->Leafs[i]->C->bucketId == (int32_t)i, "wrong bucket id");

  EpochTreeObject obj1, obj2, obj3;
  CHECK_OK(MerkleTreeToPartitionEpochObject(tree1, 0, 0, 3, &obj1));
  CHECK_OK(MerkleTreeToPartitionEpochObject(tree2, 0, 1, 3, &obj2));
  CHECK_OK(MerkleTreeToPartitionEpochObject(tree3, 0, 2, 3, &obj3));
  MerkleTree stree1, stree2, stree3;
  CHECK_OK(EpochTreeObjectToMerkleTree(eng, obj1, &stree1));
  CHECK_OK(EpochTreeObjectToMerkleTree(eng, obj2, &stree2));
  CHECK_OK(EpochTreeObjectToMerkleTree(eng, obj3, &stree3));
  CHECK(tree1.MerkleRoot() == stree1.MerkleRoot(), "hash should be the same");
  CHECK(tree2.MerkleRoot() == stree2.MerkleRoot(), "hash should be the same");
  CHECK(tree3.MerkleRoot() == stree3.MerkleRoot(), "hash should be the same");

  std::vector<int32_t> diff1, diff2, diff3, diff4, diff5;
  CHECK_OK(DifferentMerkleTreeBuckets(eng, tree1, tree2, &diff1));
  CHECK_OK(DifferentMerkleTreeBuckets(eng, tree2, tree1, &diff2));
  CHECK_OK(DifferentMerkleTreeBuckets(eng, tree1, tree3, &diff3));
  CHECK_OK(DifferentMerkleTreeBuckets(eng, tree1, stree1, &diff4));
  CHECK_OK(DifferentMerkleTreeBuckets(eng, tree1, stree3, &diff5));
  CHECK(diff1 == diff2, "diff should be the same");
  CHECK(diff1.empty(), "should be no diff");
  CHECK(diff1 == diff4, "diff should be the same");
  CHECK(!diff3.empty(), "there should be a diff");
  CHECK(!diff5.empty(), "there should be a diff");
  CHECK(diff3 == diff5, "diff vs the round-tripped tree equals diff vs the tree");

  // proto.Marshal / Unmarshal round trip on the device (main/manager.go:1045, :1025)
  Bytes wire1;
  CHECK_OK(MarshalEpochTreeObject(eng, obj1, &wire1));
  EpochTreeObject back;
  CHECK_OK(UnmarshalEpochTreeObject(eng, wire1, &back));
  CHECK(back.Buckets == obj1.Buckets && back.BucketsSize == obj1.BucketsSize && back.Items == obj1.Items &&
            back.LowerEpoch == 0 && back.UpperEpoch == 3 && !back.Valid, "wire round trip");

  const std::string n = std::to_string(writeValuesNum);
  std::printf("WIRE n%s_0_3 %s\n", n.c_str(), hex(wire1).c_str());
  std::printf("ROOT n%s_0_3 %s\nROOT n%s_1_3 %s\nROOT n%s_2_3 %s\nDIFF n%s_t1_t3 %s\nITEMS n%s_0_3 %d\n",
              n.c_str(), hex(tree1.MerkleRoot()).c_str(), n.c_str(), hex(tree2.MerkleRoot()).c_str(),
              n.c_str(), hex(tree3.MerkleRoot()).c_str(), n.c_str(), ids(diff3).c_str(), n.c_str(),
              obj1.Items);

  // Batched build (one engine call for the partition) agrees with the single build.
  std::vector<MerkleTree> batch;
  CHECK_OK(manager.RawPartitionMerkleTrees({0, 0}, 0, 3, &batch));
  CHECK(batch.size() == 2 && batch[0].MerkleRoot() == tree1.MerkleRoot() &&
            batch[1].MerkleRoot() == tree1.MerkleRoot(), "batched build root");
}

static void TestIndexManager() {
  std::string index1;
  CHECK_OK(BuildEpochIndex(1, 2, 3, "zz", &index1));
  CHECK(index1 == "epoch_1_2_0000000003_zz", "equal index");
  int p;
  uint64_t b;
  int64_t e;
  std::string k;
  CHECK_OK(ParseEpochIndex(index1, &p, &b, &e, &k));
  CHECK(p == 1 && b == 2 && e == 3 && k == "zz", "parsed fields");
  std::string index2;
  CHECK_OK(BuildEpochTreeObjectIndex(1, 2, &index2));
  CHECK(index2 == "epochtree_1_0000000002", "equal index");
}

static void TestIndexStorage() {
  std::string index;
  CHECK_OK(Index("test")
               .AddColumn(CreateUnorderedColumn("partition", "part1"))
               .AddColumn(CreateUnorderedColumn("bucket", "bucket1"))
               .AddColumn(CreateOrderedColumn("epoch", "1", 4))
               .AddColumn(CreateUnorderedColumn("key", "mykey"))
               .Build(&index));
  CHECK(index == "test_part1_bucket1_0001_mykey", "index should be equal");
  Index index2 = Index("zzz");
  index2.AddColumn(CreateUnorderedColumn("partition", "part1"))
      .AddColumn(CreateUnorderedColumn("bucket", "bucket1"))
      .AddColumn(CreateOrderedColumn("epoch", "100", 4))
      .AddColumn(CreateUnorderedColumn("key", "mykey"));
  std::string s2;
  CHECK_OK(index2.Build(&s2));
  CHECK(s2 == "zzz_part1_bucket1_0100_mykey", "index2 should be equal");
  std::map<std::string, std::string> m;
  CHECK_OK(index2.Parse(s2, &m));
  CHECK(m["name"] == "zzz" && m["partition"] == "part1" && m["bucket"] == "bucket1" &&
            m["epoch"] == "100" && m["key"] == "mykey", "parsed columns");
  std::string bad;
  CHECK(!Index("x").AddColumn(CreateOrderedColumn("e", "12345", 4)).Build(&bad).empty(),
        "too-long ordered column is an error");
}

static void TestManagerStorage(Engine& eng, int writeValuesNum) {
  Manager manager(eng, 1, 1);
  for (int i = 0; i < writeValuesNum; i++)
    CHECK_OK(manager.SetValue({"key" + std::to_string(i), "val" + std::to_string(i), 1, 0}));
  for (int i = 0; i < writeValuesNum; i++)
    CHECK_OK(manager.SetValue({"keyz" + std::to_string(i), "valz" + std::to_string(i), 2, 0}));
  std::string i1, i2, i3;
  CHECK_OK(BuildEpochIndex(0, 0, 1, "", &i1));
  CHECK_OK(BuildEpochIndex(0, 0, 2, "", &i2));
  CHECK_OK(BuildEpochIndex(0, 0, 3, "", &i3));
  int count = 0;
  for (Iterator it = manager.db().NewIterator(i1, i2); !it.IsDone(); it.Next()) count++;
  CHECK(count == writeValuesNum, "Should have iterated all inserted keys");
  count = 0;
  for (Iterator it = manager.db().NewIterator(i1, i3); !it.IsDone(); it.Next()) count++;
  CHECK(count == 2 * writeValuesNum, "Should have iterated all inserted keys");
  // B = 1: a single-bucket tree (leaf + its duplicate)
  MerkleTree t;
  CHECK_OK(manager.RawPartitionMerkleTree(0, 1, 3, &t));
  CHECK(t.Leafs.size() == 2 && t.Leafs[1]->dup && t.Leafs[0]->C->size == 2 * writeValuesNum, "B = 1 tree");
  // a newer value in an older-or-equal epoch is rejected (main/manager.go:807-809)
  CHECK_OK(manager.SetValue({"kk", "a", 5, 100}));
  CHECK(!manager.SetValue({"kk", "b", 5, 50}).empty(), "a newer value already exists");
}

// Manager.VerifyEpoch (main/manager.go:998-1118) with the peer fetch replaced by the objects
// three replicas would serve: A and B hold the same writes, C misses some and has others.
// Prints "VERIFY <case> <valid> <validCount> <diffSet>" for tests/test_cpp_port.py to check
// against the oracle.
static Bytes EpochObjectBytes(Engine& eng, Manager& m, int p, int64_t e) {
  MerkleTree t;
  EpochTreeObject o;
  Bytes w;
  CHECK_OK(m.RawPartitionMerkleTree(p, e, e + 1, &t));
  CHECK_OK(MerkleTreeToPartitionEpochObject(t, p, e, e + 1, &o));
  CHECK_OK(MarshalEpochTreeObject(eng, o, &w));
  return w;
}

static void TestVerifyEpoch(Engine& eng) {
  Manager a(eng, 1, 16), b(eng, 1, 16), c(eng, 1, 16);
  for (int i = 0; i < 40; i++) {
    Value v{"key" + std::to_string(i), "val" + std::to_string(i), 1, i + 1};
    CHECK_OK(a.SetValue(v));
    CHECK_OK(b.SetValue(v));
    if (i < 35) CHECK_OK(c.SetValue(v));
  }
  for (int i = 0; i < 3; i++) CHECK_OK(c.SetValue({"other" + std::to_string(i), "x", 1, 100 + i}));
  const Bytes oa = EpochObjectBytes(eng, a, 0, 1), ob = EpochObjectBytes(eng, b, 0, 1),
              oc = EpochObjectBytes(eng, c, 0, 1);
  auto show = [](const char* name, const Manager::VerifyResult& r) {
    std::printf("VERIFY %s %d %d %s\n", name, r.Valid ? 1 : 0, r.ValidCount, ids(r.DiffSet).c_str());
  };
  Manager::VerifyResult r;
  Error e = a.VerifyEpoch(0, 1, {oa, ob, oc}, 3, &r);  // 2 agreeing trees < ReplicaCount 3
  CHECK(!e.empty() && !r.Valid && r.ValidCount == 2 && !r.DiffSet.empty(), "not verified");
  show("a_r3", r);
  Bytes stored;
  EpochTreeObject so;
  std::string idx;
  CHECK_OK(BuildEpochTreeObjectIndex(0, 1, &idx));
  CHECK(a.db().Get(idx, &stored), "epoch object persisted");
  CHECK_OK(UnmarshalEpochTreeObject(eng, stored, &so));
  CHECK(!so.Valid && so.LowerEpoch == 1 && so.UpperEpoch == 2, "persisted object is not valid");
  CHECK_OK(a.VerifyEpoch(0, 1, {oa, ob, oc}, 2, &r));  // now enough agreeing trees
  CHECK(r.Valid && !r.AlreadyValid && r.ValidCount == 2, "verified");
  show("a_r2", r);
  CHECK(a.db().Get(idx, &stored), "epoch object persisted");
  CHECK_OK(UnmarshalEpochTreeObject(eng, stored, &so));
  CHECK(so.Valid, "persisted object is valid");
  CHECK_OK(a.VerifyEpoch(0, 1, {}, 3, &r));  // stored object valid: early return
  CHECK(r.Valid && r.AlreadyValid, "already valid");
  // C disagrees with a peer object that is marked valid -> validDiff
  CHECK_OK(c.VerifyEpoch(0, 1, {oc, stored, Bytes{0xff}}, 3, &r));
  CHECK(r.Valid && r.ValidCount == 1, "valid by a differing valid tree");
  show("c_vd", r);
  // batched form over partitions of one epoch (the only partition here, twice)
  std::vector<Manager::VerifyResult> rs;
  std::vector<Error> es;
  CHECK_OK(b.VerifyEpochs({0}, 1, {{oa, oc}}, 2, &rs, &es));
  CHECK(rs.size() == 1 && !rs[0].Valid && !es[0].empty(), "batched verify");
  show("b_r2", rs[0]);
}

// TestStreamBucketsTask (main/manager_test.go:117-211): all buckets of epochs [0,2) stream the N
// epoch-1 records, [0,3) all 2N; a bucket subset streams exactly that subset's records.
static void TestStreamBucketsTask(Engine& eng, int writeValuesNum) {
  Manager manager(eng, 1, 100);
  for (int i = 0; i < writeValuesNum; i++)
    CHECK_OK(manager.SetValue({"key" + std::to_string(i), "val" + std::to_string(i), 1, 0}));
  for (int i = 0; i < writeValuesNum; i++)
    CHECK_OK(manager.SetValue({"keyz" + std::to_string(i), "valz" + std::to_string(i), 2, 0}));
  std::vector<Value> items;
  CHECK_OK(manager.StreamBuckets(0, {}, 0, 2, &items));
  CHECK((int)items.size() == writeValuesNum, "itemCount is wrong");
  for (const Value& v : items) CHECK(v.Epoch == 1 && v.Key.rfind("key", 0) == 0, "epoch-1 records");
  CHECK_OK(manager.StreamBuckets(0, {}, 0, 3, &items));
  CHECK((int)items.size() == 2 * writeValuesNum, "itemCount is wrong");
  // a list with a repeat and an out-of-range id, streamed as the task walks it
  // (main/manager.go:453-485): b1's records, bucket 99's, b0's, b1's again, nothing for 1000
  uint64_t b0 = 0, b1 = 0;
  int p0;
  CHECK_OK(manager.KeyTags(items.front().Key, &b0, &p0));
  CHECK_OK(manager.KeyTags(items.back().Key, &b1, &p0));
  std::vector<Value> sub;
  CHECK_OK(manager.StreamBuckets(0, {(int32_t)b1, 99, (int32_t)b0, (int32_t)b1, 1000}, 0, 3, &sub));
  std::vector<Value> want;
  for (uint64_t req : {b1, (uint64_t)99, b0, b1})
    for (const Value& v : items) {  // items: all buckets, ascending, LSM order inside each
      uint64_t b;
      int p;
      CHECK_OK(manager.KeyTags(v.Key, &b, &p));
      if (b == req) want.push_back(v);
    }
  CHECK(!want.empty(), "the list holds records");
  CHECK(sub.size() == want.size(), "request-order stream size");
  for (size_t i = 0; i < want.size() && i < sub.size(); i++)
    CHECK(sub[i].Key == want[i].Key && sub[i].Epoch == want[i].Epoch &&
              sub[i].UnixTimestamp == want[i].UnixTimestamp,
          "request-order stream: b1, 99, b0, b1 (repeats streamed again)");
  size_t nb1 = 0;
  for (const Value& v : sub) {
    uint64_t b;
    int p;
    CHECK_OK(manager.KeyTags(v.Key, &b, &p));
    nb1 += b == b1;
  }
  size_t once = 0;
  for (const Value& v : items) {
    uint64_t b;
    int p;
    CHECK_OK(manager.KeyTags(v.Key, &b, &p));
    once += b == b1;
  }
  CHECK(nb1 == (2 + (b1 == b0) + (b1 == 99)) * once, "b1 streamed once per request");
  const size_t wantN = want.size();
  std::printf("STREAMSEQ n%d %llu %llu", writeValuesNum, (unsigned long long)b0, (unsigned long long)b1);
  for (const Value& v : sub) std::printf(" %s:%lld:%lld", v.Key.c_str(), (long long)v.Epoch, (long long)v.UnixTimestamp);
  std::printf("\n");
  std::printf("STREAM n%d %zu %zu %zu\n", writeValuesNum, items.size(), sub.size(), wantN);
}

// TestGetEpochTreeLastValidObjectTask (main/manager_test.go:213-301): no stored object -> the
// LowerEpoch -1 object; objects at epochs 1 (valid), 2 (valid), 3 (not valid) -> epoch 2. Plus the
// reverse iterator's unbounded-below quirk: partition 2, with no objects of its own, finds
// partition 1's newest valid object ("epochtree_1_..." < "epochtree_2_...").
static void TestGetEpochTreeLastValid(Engine& eng) {
  Manager manager(eng, 200, 100);
  manager.CurrentEpoch = 100;
  const int writePartition = 1;
  EpochTreeObject got;
  CHECK_OK(manager.GetEpochTreeLastValid(writePartition, &got));
  CHECK(got.LowerEpoch == -1 && got.UpperEpoch == -1 && !got.Valid && got.Partition == writePartition,
        "no stored object: LowerEpoch -1");
  const struct { int64_t epoch; bool valid; } objs[] = {{1, true}, {2, true}, {3, false}};
  for (const auto& o : objs) {
    EpochTreeObject obj;
    obj.Partition = writePartition;
    obj.LowerEpoch = o.epoch;
    obj.Valid = o.valid;
    Bytes data;
    std::string index;
    CHECK_OK(MarshalEpochTreeObject(eng, obj, &data));
    CHECK_OK(BuildEpochTreeObjectIndex(writePartition, obj.LowerEpoch, &index));
    manager.db().Put(index, data);
  }
  CHECK_OK(manager.GetEpochTreeLastValid(writePartition, &got));
  CHECK(got.LowerEpoch == 2 && got.Valid, "the correct object was returned");
  CHECK_OK(manager.GetEpochTreeLastValid(2, &got));
  CHECK(got.LowerEpoch == 2 && got.Partition == 1, "reverse scan walks below its Start bound");
  manager.CurrentEpoch = 3;  // Seek(Limit) lands on epochtree_1_0000000003 == Limit: done at once
  CHECK_OK(manager.GetEpochTreeLastValid(writePartition, &got));
  CHECK(got.LowerEpoch == -1, "a key equal to Limit ends the reverse scan");
}

int main() {
  Engine eng(0);
  if (!eng.ok()) {
    std::fprintf(stderr, "engine unavailable: %s\n", eng.init_error().c_str());
    return 2;
  }
  TestMerkleTreeRaw(eng, 100);
  TestMerkleTreeRaw(eng, 10);
  TestIndexManager();
  TestIndexStorage();
  TestManagerStorage(eng, 100);
  TestVerifyEpoch(eng);
  TestGetEpochTreeLastValid(eng);
  TestStreamBucketsTask(eng, 100);
  TestStreamBucketsTask(eng, 10);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("PASS\n");
  return 0;
}
