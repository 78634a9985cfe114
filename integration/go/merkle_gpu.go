// merkle_gpu.go -- cgo shim: drop-in for the hot path of main/merkle_tree.go (MyDataStore).
//
// Copy into the reference's main/ package and delete RawPartitionMerkleTree and
// DifferentMerkleTreeBuckets from merkle_tree.go (INTEGRATION.md section 2); VerifyEpoch may then
// replace its peer loop (main/manager.go:1072-1104) with verifyEpochDecision. It binds only what
// include/mde.h declares (tests/test_integration.py checks every C.* name against the header).
// Not compiled in this repository: the image has no Go toolchain (DESIGN.md section 1).
package main

/*
#cgo CFLAGS: -I${SRCDIR}/../mi355x/include
#cgo LDFLAGS: -L${SRCDIR}/../mi355x/mydatastore_amd -lmde -Wl,-rpath,${SRCDIR}/../mi355x/mydatastore_amd
#include <stdlib.h>
#include "mde.h"
*/
import "C"

import (
	"bytes"
	"sync"
	"unsafe"

	"github.com/cbergoon/merkletree"
	"github.com/pkg/errors"
	"google.golang.org/protobuf/proto"

	"github.com/andrew-delph/my-key-store/rpc"
)

var (
	mdeOnce sync.Once
	// mdeBatcher serves RawPartitionMerkleTree and verifyEpochDecision: VerifyEpoch runs one
	// partition per call on a pool of worker goroutines (main/manager.go:166-170,491), up to
	// PartitionConcurrency at once (config/default-config.yaml:9); the batcher coalesces the calls
	// in flight into one device build / verify (group commit, mde_batch_build / mde_batch_verify).
	// Each call gets its own error message back in its own buffer, so no lock is needed.
	mdeBatcher *C.mde_batcher
	// mdeCtx serves the unbatched calls (DifferentMerkleTreeBuckets). mdeMu pairs each call with
	// its own error message; it costs no concurrency, since the context lock serialises calls on
	// one context anyway.
	mdeCtx *C.mde_ctx
	mdeErr error
	mdeMu  sync.Mutex
)

// mdeCall runs one engine call on mdeCtx and, when it fails, returns ITS message (copied under
// the context lock by mde_last_error_copy while mdeMu is still held).
func mdeCall(ctx *C.mde_ctx, name string, call func() C.int) error {
	mdeMu.Lock()
	defer mdeMu.Unlock()
	if rc := call(); rc != C.MDE_OK {
		var buf [512]C.char
		C.mde_last_error_copy(ctx, &buf[0], C.uint64_t(len(buf)))
		return errors.Errorf("%s: %s", name, C.GoString(&buf[0]))
	}
	return nil
}

func mdeEngine() (*C.mde_batcher, *C.mde_ctx, error) {
	mdeOnce.Do(func() {
		var b *C.mde_batcher
		// at most 256 partitions per batch, no wait window: a batch is whatever queued while the
		// previous batches ran
		if rc := C.mde_batcher_create(0, 256, 0, &b); rc != C.MDE_OK {
			mdeErr = errors.Errorf("mde_batcher_create: %s", C.GoString(C.mde_strerror(rc)))
			return
		}
		var ctx *C.mde_ctx
		if rc := C.mde_create(0, &ctx); rc != C.MDE_OK {
			mdeErr = errors.Errorf("mde_create: %s", C.GoString(C.mde_strerror(rc)))
			return
		}
		mdeBatcher, mdeCtx = b, ctx
	})
	return mdeBatcher, mdeCtx, mdeErr
}

func cU64(v []uint64) unsafe.Pointer { return C.CBytes(unsafe.Slice((*byte)(unsafe.Pointer(&v[0])), len(v)*8)) }

// RawPartitionMerkleTree -- drop-in for main/merkle_tree.go:86-116. The per-bucket range scans are
// unchanged; the values go into one arena that the MI355X engine reduces (bucket digests + SHA-256
// tree on device), batched with the other partitions' calls in flight.
func (manager *Manager) RawPartitionMerkleTree(partitionId int, lowerEpoch, upperEpoch int64) (*merkletree.MerkleTree, error) {
	batcher, _, err := mdeEngine()
	if err != nil {
		return nil, err
	}
	B := manager.config.Manager.PartitionBuckets
	values := make([]byte, 0, 1<<16)
	valueOff := []uint64{0}
	segRec := []uint64{0}
	for i := 0; i < B; i++ {
		index1, err := BuildEpochIndex(partitionId, uint64(i), lowerEpoch, "")
		if err != nil {
			return nil, err
		}
		index2, err := BuildEpochIndex(partitionId, uint64(i), upperEpoch, "")
		if err != nil {
			return nil, err
		}
		it := manager.db.NewIterator([]byte(index1), []byte(index2), false)
		for !it.IsDone() {
			values = append(values, it.Value()...)
			valueOff = append(valueOff, uint64(len(values)))
			it.Next()
		}
		it.Release()
		segRec = append(segRec, uint64(len(valueOff)-1))
	}
	if len(values) == 0 {
		values = append(values, 0)
	}
	cValues, cOff, cSeg := C.CBytes(values), cU64(valueOff), cU64(segRec)
	defer C.free(cValues)
	defer C.free(cOff)
	defer C.free(cSeg)
	cDigest := C.malloc(C.size_t(8 * B))
	cSize := C.malloc(C.size_t(4 * B))
	cItems := C.malloc(4)
	cRoot := C.malloc(32)
	defer C.free(cDigest)
	defer C.free(cSize)
	defer C.free(cItems)
	defer C.free(cRoot)
	rec := C.mde_records{
		values: (*C.uint8_t)(cValues), values_bytes: C.uint64_t(len(values)),
		value_off: (*C.uint64_t)(cOff), n_records: C.uint64_t(len(valueOff) - 1),
		n_partitions: 1, n_buckets: C.uint32_t(B), seg_rec: (*C.uint64_t)(cSeg),
	}
	out := C.mde_tree_out{digest: (*C.uint64_t)(cDigest), size: (*C.int32_t)(cSize),
		items: (*C.int32_t)(cItems), root: (*C.uint8_t)(cRoot)}
	var errBuf [512]C.char
	if rc := C.mde_batch_build(batcher, &rec, &out, &errBuf[0], C.uint64_t(len(errBuf))); rc != C.MDE_OK {
		return nil, errors.Errorf("mde_batch_build: %s", C.GoString(&errBuf[0]))
	}
	digest := unsafe.Slice((*uint64)(cDigest), B)
	size := unsafe.Slice((*int32)(cSize), B)
	// Rebuild the reference's tree type from the device digests so every caller keeps its types;
	// merkletree.NewTree costs B-1 host SHA-256s, and the device root cross-checks it.
	bucketList := make([]merkletree.Content, B)
	for i := 0; i < B; i++ {
		bucketList[i] = &MerkleBucket{bucketId: int32(i), hasher: &CustomHash{value: int64(digest[i])}, size: size[i]}
	}
	tree, err := merkletree.NewTree(bucketList)
	if err != nil {
		return nil, err
	}
	if !bytes.Equal(tree.MerkleRoot(), C.GoBytes(cRoot, 32)) {
		return nil, errors.New("device root differs from merkletree root")
	}
	return tree, nil
}

// DifferentMerkleTreeBuckets -- drop-in for main/merkle_tree.go:159-161 (DFS order, duplicates).
func DifferentMerkleTreeBuckets(tree1 *merkletree.MerkleTree, tree2 *merkletree.MerkleTree) ([]int32, error) {
	_, ctx, err := mdeEngine()
	if err != nil {
		return nil, err
	}
	digests := func(t *merkletree.MerkleTree) ([]uint64, error) {
		n := len(t.Leafs)
		if n > 1 && t.Leafs[n-1].C == t.Leafs[n-2].C { // merkletree's duplicate of the last leaf
			n--
		}
		d := make([]uint64, n)
		for i := 0; i < n; i++ {
			b, ok := t.Leafs[i].C.(*MerkleBucket)
			if !ok {
				return nil, errors.New("failed to decode MerkleBucket")
			}
			d[i] = uint64(b.hasher.Hash())
		}
		return d, nil
	}
	d1, err := digests(tree1)
	if err != nil {
		return nil, err
	}
	d2, err := digests(tree2)
	if err != nil {
		return nil, err
	}
	capIds := C.mde_diff_capacity(C.uint32_t(len(d1)), C.uint32_t(len(d2)))
	cA, cB := cU64(d1), cU64(d2)
	defer C.free(cA)
	defer C.free(cB)
	cIds := C.malloc(C.size_t(4 * capIds))
	cCount := C.malloc(4)
	defer C.free(cIds)
	defer C.free(cCount)
	if err := mdeCall(ctx, "mde_diff", func() C.int {
		return C.mde_diff_digests(ctx, 1, C.uint32_t(len(d1)), (*C.uint64_t)(cA), C.uint32_t(len(d2)),
			(*C.uint64_t)(cB), (*C.int32_t)(cIds), capIds, (*C.int32_t)(cCount))
	}); err != nil {
		return nil, err
	}
	n := *(*int32)(cCount)
	if n == C.MDE_E_TREE {
		return nil, errors.New("bucketIds dont match (or a merkletree.Node is nil)")
	}
	out := make([]int32, n)
	copy(out, unsafe.Slice((*int32)(cIds), n))
	return out, nil
}

// verifyEpochDecision -- the decision step of Manager.VerifyEpoch (main/manager.go:1072-1104) in
// one mde_batch_verify call, batched with the other partitions' decisions in flight: every peer
// object is decoded, rebuilt and diffed against myTree on the device (myTree's own nodes are built
// there from its digests); failed peers are skipped (the reference logs and continues);
// validCount, validDiff and diffSet fold as the reference does. Returns valid (validCount >=
// replicaCount || validDiff), validCount, diffSet (ascending) and the EpochTreeObject to persist
// (Valid set) as wire bytes. VerifyEpoch keeps its own flow: on valid it stores data, otherwise it
// calls PoliteStreamRequest(partitionId, epoch, epoch+1, diffSet).
func verifyEpochDecision(myTree *merkletree.MerkleTree, partitionId int, epoch int64,
	epochTreeObjects []*rpc.RpcEpochTreeObject, replicaCount int) (bool, int, []int32, []byte, error) {
	batcher, _, err := mdeEngine()
	if err != nil {
		return false, 0, nil, nil, err
	}
	// the local tree as bucket digests + sizes (tree.Leafs without merkletree's odd duplicate)
	n := len(myTree.Leafs)
	if n > 1 && myTree.Leafs[n-1].C == myTree.Leafs[n-2].C {
		n--
	}
	B := n
	digest := make([]uint64, B)
	size := make([]int32, B)
	for i := 0; i < B; i++ {
		b, ok := myTree.Leafs[i].C.(*MerkleBucket)
		if !ok {
			return false, 0, nil, nil, errors.New("failed to decode MerkleBucket")
		}
		digest[i] = uint64(b.hasher.Hash())
		size[i] = b.size
	}
	cDigest := cU64(digest)
	defer C.free(cDigest)
	cSize := C.CBytes(unsafe.Slice((*byte)(unsafe.Pointer(&size[0])), B*4))
	defer C.free(cSize)
	// peer objects back to wire bytes (gRPC already unmarshalled them); a nil object is absent
	R := len(epochTreeObjects)
	var blob []byte
	off := make([]uint64, R+1)
	for r, obj := range epochTreeObjects {
		if obj != nil {
			b, err := proto.Marshal(obj)
			if err != nil {
				return false, 0, nil, nil, err
			}
			blob = append(blob, b...)
		}
		off[r+1] = uint64(len(blob))
	}
	blob = append(blob, 0) // never a zero-length allocation
	cBlob := C.CBytes(blob)
	cOff := cU64(off)
	defer C.free(cBlob)
	defer C.free(cOff)
	stride := C.mde_epoch_tree_object_max_bytes(C.uint32_t(B))
	cObj := C.malloc(C.size_t(stride))
	cIds := C.malloc(C.size_t(4 * B))
	cStatus := C.malloc(C.size_t(4 * (R + 1)))
	cOut := C.malloc(16) // valid (u8), validCount, diffCount, objectLen
	defer C.free(cObj)
	defer C.free(cIds)
	defer C.free(cStatus)
	defer C.free(cOut)
	outs := unsafe.Slice((*int32)(cOut), 4)
	var errBuf [512]C.char
	if rc := C.mde_batch_verify(batcher, C.uint32_t(B), C.int32_t(partitionId), C.int64_t(epoch),
		(*C.uint64_t)(cDigest), (*C.int32_t)(cSize), C.uint32_t(R), (*C.uint8_t)(cBlob), (*C.uint64_t)(cOff),
		C.uint32_t(replicaCount), (*C.uint8_t)(unsafe.Pointer(&outs[0])), (*C.int32_t)(unsafe.Pointer(&outs[1])),
		(*C.int32_t)(cIds), (*C.int32_t)(unsafe.Pointer(&outs[2])), (*C.int32_t)(cStatus), (*C.uint8_t)(cObj),
		stride, (*C.uint32_t)(unsafe.Pointer(&outs[3])), &errBuf[0], C.uint64_t(len(errBuf))); rc != C.MDE_OK {
		return false, 0, nil, nil, errors.Errorf("mde_batch_verify: %s", C.GoString(&errBuf[0]))
	}
	valid := *(*uint8)(unsafe.Pointer(&outs[0])) != 0
	diffSet := make([]int32, outs[2])
	copy(diffSet, unsafe.Slice((*int32)(cIds), outs[2]))
	return valid, int(outs[1]), diffSet, C.GoBytes(cObj, C.int(outs[3])), nil
}
