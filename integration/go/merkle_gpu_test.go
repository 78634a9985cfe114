// merkle_gpu_test.go -- the parity pin a maintainer with Go and a gfx950 GPU can run:
//
//	go test ./main -run TestMde -v            (N = 100 writes per epoch)
//	go test ./main -run TestMde -v -short     (N = 10)
//	go test ./main -run TestMde -v -tags mde_nohashstrategy
//
// It writes the reference's own TestMerkleTreeRaw scenario (main/merkle_tree_test.go:15-75: B = 30,
// "key%d" at epoch 1 and "keyz%d" at epoch 2, timestamps 1..2N) and checks, for the ranges [0,3),
// [1,3) and [2,3), through every path the shim has (the resident service or the batcher; device
// tree or host tree):
//   - the shim's tree equals the reference's construction over the same store, node by node
//     (mdeRefTree restates main/merkle_tree.go:86-116 with the reference's own CustomHash,
//     MerkleBucket and merkletree.NewTree);
//   - the roots equal what this repository's oracle predicts (tests/golden/testmerkletreeraw_n*.json;
//     tests/test_integration.py keeps the constants below equal to those fixtures). The oracle's
//     tree bytes are otherwise unpinned (DESIGN.md section 1): this is the test that pins them;
//   - DifferentMerkleTreeBuckets over the shim's trees gives the predicted diff lists.
// Skipped when no gfx950 GPU is visible. Not compiled in this repository (no Go toolchain).
package main

import (
	"bytes"
	"encoding/hex"
	"fmt"
	"reflect"
	"sync"
	"testing"

	"github.com/cbergoon/merkletree"

	"github.com/andrew-delph/my-key-store/config"
	"github.com/andrew-delph/my-key-store/rpc"
)

// the oracle's predicted roots (hex) of [0,3), [1,3), [2,3) and diff [0,3) vs [2,3), by N
var mdePredicted = map[int]struct {
	roots [3]string
	diff  []int32
}{
	10: {[3]string{
		"5d5f2fb4daa3b70c53ecd56bee99ce02676fbd6b0826706e1fa0c9d7a0186b44",
		"5d5f2fb4daa3b70c53ecd56bee99ce02676fbd6b0826706e1fa0c9d7a0186b44",
		"e2b93610ede015c33c922a1dd00d647f6731373b597b3eb76704446743e8c984"},
		[]int32{3, 6, 9, 11, 12, 22, 23, 27}},
	100: {[3]string{
		"2cb892f8455313dccedb990e7d071816c13c8bb728137c887d2d7c0a3438c7a7",
		"2cb892f8455313dccedb990e7d071816c13c8bb728137c887d2d7c0a3438c7a7",
		"03f02578452d8b229a02a12399d47e105ddbe15ed3e89cb2a2e5ad30e1eacae1"},
		[]int32{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 21, 22, 23, 24,
			25, 26, 27, 28, 29, 28, 29}},
}

var mdeTestMetrics sync.Once

// mdeRefTree -- main/merkle_tree.go:86-116 over the same store: per bucket, the epoch-index range
// scan, CustomHash.Add of every value, the record count; then merkletree.NewTree.
func mdeRefTree(manager *Manager, partitionId int, lowerEpoch, upperEpoch int64) (*merkletree.MerkleTree, error) {
	B := manager.config.Manager.PartitionBuckets
	cs := make([]merkletree.Content, B)
	for b := 0; b < B; b++ {
		lo, err := BuildEpochIndex(partitionId, uint64(b), lowerEpoch, "")
		if err != nil {
			return nil, err
		}
		hi, err := BuildEpochIndex(partitionId, uint64(b), upperEpoch, "")
		if err != nil {
			return nil, err
		}
		leaf := &MerkleBucket{bucketId: int32(b), hasher: &CustomHash{}}
		it := manager.db.NewIterator([]byte(lo), []byte(hi), false)
		for ; !it.IsDone(); it.Next() {
			leaf.hasher.Add(it.Value())
			leaf.size++
		}
		it.Release()
		cs[b] = leaf
	}
	return merkletree.NewTree(cs)
}

// mdeSameTree: equal roots and leaf lists, and the same node graph (hashes, shape, leaf contents).
func mdeSameTree(t *testing.T, what string, got, want *merkletree.MerkleTree) {
	t.Helper()
	if !bytes.Equal(got.MerkleRoot(), want.MerkleRoot()) {
		t.Fatalf("%s: root %x, reference %x", what, got.MerkleRoot(), want.MerkleRoot())
	}
	if len(got.Leafs) != len(want.Leafs) {
		t.Fatalf("%s: %d leaves, reference %d", what, len(got.Leafs), len(want.Leafs))
	}
	var walk func(g, w *merkletree.Node, path string)
	walk = func(g, w *merkletree.Node, path string) {
		if (g == nil) != (w == nil) {
			t.Fatalf("%s: node %s present on one side only", what, path)
		}
		if g == nil {
			return
		}
		if !bytes.Equal(g.Hash, w.Hash) {
			t.Fatalf("%s: node %s hash %x, reference %x", what, path, g.Hash, w.Hash)
		}
		if (g.Left == nil) != (w.Left == nil) {
			t.Fatalf("%s: node %s is a leaf on one side only", what, path)
		}
		if g.Left == nil { // a leaf: the bucket behind it
			gb, ok1 := g.C.(*MerkleBucket)
			wb, ok2 := w.C.(*MerkleBucket)
			if !ok1 || !ok2 {
				t.Fatalf("%s: leaf %s content %v / %v", what, path, reflect.TypeOf(g.C), reflect.TypeOf(w.C))
			}
			if gb.bucketId != wb.bucketId || gb.size != wb.size || gb.hasher.Hash() != wb.hasher.Hash() {
				t.Fatalf("%s: leaf %s bucket (%d, %d, %d), reference (%d, %d, %d)", what, path,
					gb.bucketId, gb.size, gb.hasher.Hash(), wb.bucketId, wb.size, wb.hasher.Hash())
			}
			return
		}
		walk(g.Left, w.Left, path+"L")
		walk(g.Right, w.Right, path+"R")
	}
	walk(got.Root, want.Root, "root:")
}

func TestMdeRawPartitionMerkleTreeMatchesReference(t *testing.T) {
	if _, err := mdeEngine(0); err != nil {
		t.Skipf("no MI355X engine: %v", err)
	}
	mdeTestMetrics.Do(func() { initMetrics("mde_gpu_test") })
	n := 100
	if testing.Short() {
		n = 10
	}
	c := config.GetConfig()
	c.Storage.DataPath = t.TempDir()
	c.Manager.PartitionCount = 1
	c.Manager.PartitionBuckets = 30
	manager := NewManager(c)
	ts := int64(0)
	for _, w := range []struct {
		key, val string
		epoch    int64
	}{{"key", "val", 1}, {"keyz", "valz", 2}} { // epoch 1 first, as the reference test writes them
		for i := 0; i < n; i++ {
			ts++
			v := &rpc.RpcValue{Key: fmt.Sprintf("%s%d", w.key, i), Value: fmt.Sprintf("%s%d", w.val, i),
				Epoch: w.epoch, UnixTimestamp: ts}
			if err := manager.SetValue(v); err != nil {
				t.Fatal(err)
			}
		}
	}
	pred := mdePredicted[n]
	ranges := [3][2]int64{{0, 3}, {1, 3}, {2, 3}}
	saved := [2]bool{mdeResident, mdeHostTree}
	defer func() { mdeResident, mdeHostTree = saved[0], saved[1] }()
	for _, resident := range []bool{true, false} {
		for _, hostTree := range []bool{false, true} {
			mdeResident, mdeHostTree = resident, hostTree
			path := fmt.Sprintf("resident=%v hostTree=%v hashStrategy=%v", resident, hostTree, mdeHashStrategy)
			var trees [3]*merkletree.MerkleTree
			for k, r := range ranges {
				got, err := manager.RawPartitionMerkleTree(0, r[0], r[1])
				if err != nil {
					t.Fatalf("%s [%d,%d): %v", path, r[0], r[1], err)
				}
				want, err := mdeRefTree(&manager, 0, r[0], r[1])
				if err != nil {
					t.Fatal(err)
				}
				what := fmt.Sprintf("%s [%d,%d)", path, r[0], r[1])
				mdeSameTree(t, what, got, want)
				if h := hex.EncodeToString(got.MerkleRoot()); h != pred.roots[k] {
					t.Errorf("%s: root %s, oracle predicted %s", what, h, pred.roots[k])
				}
				if ok, err := got.VerifyTree(); err != nil || !ok {
					t.Errorf("%s: VerifyTree = %v, %v", what, ok, err)
				}
				trees[k] = got
			}
			diff, err := DifferentMerkleTreeBuckets(trees[0], trees[2])
			if err != nil {
				t.Fatal(err)
			}
			if !reflect.DeepEqual(diff, pred.diff) {
				t.Errorf("%s: diff [0,3) vs [2,3) %v, oracle predicted %v", path, diff, pred.diff)
			}
		}
	}
}
