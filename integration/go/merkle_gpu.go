// merkle_gpu.go -- cgo shim: drop-in for the hot path of main/merkle_tree.go (MyDataStore).
//
// Copy into the reference's main/ package and delete RawPartitionMerkleTree from merkle_tree.go
// (INTEGRATION.md section 2); VerifyEpoch may then replace its peer loop (main/manager.go:1072-1104)
// with verifyEpochDecision. DifferentMerkleTreeBuckets stays the reference's own DFS: it compares
// node hashes the trees already hold (<= 2B-1 byte compares, no hashing), which no device round
// trip beats for one pair (tests/cpp/batch_bench.c diff_host / diff_device). It binds only what
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
	"log"
	"sync"
	"sync/atomic"
	"unsafe"

	"github.com/cbergoon/merkletree"
	"github.com/pkg/errors"
	"google.golang.org/protobuf/proto"

	"github.com/andrew-delph/my-key-store/rpc"
)

var (
	mdeOnce sync.Once
	// mdeBatchers serve RawPartitionMerkleTree and verifyEpochDecision, one per GPU of the node:
	// partition p goes to GPU p % G, the in-node analogue of the ring's partition sharding
	// (hashring/hashring.go:126-154; the same placement as mde_group / mde_multi_build, which a
	// caller building many partitions at once uses instead). VerifyEpoch runs one partition per
	// call on a pool of worker goroutines (main/manager.go:166-170,491), up to
	// PartitionConcurrency at once (config/default-config.yaml:9); each batcher coalesces the calls
	// in flight into one device build / verify (group commit, mde_batch_build / mde_batch_verify).
	// Each call gets its own error message back in its own buffer, so no lock is needed.
	mdeBatchers []*C.mde_batcher
	// mdeServers: the resident build service of each GPU (mde_server_build / mde_server_verify): a
	// persistent launch polling request slots in pinned memory serves each call without a kernel
	// launch, copy command or event (INTEGRATION.md section 3). mdeResident picks it over the
	// batcher for RawPartitionMerkleTree and verifyEpochDecision.
	mdeServers  []*C.mde_server
	mdeResident = true
	mdeErr      error
	// mdeHostTree: build every returned tree with plain merkletree.NewTree over the device digests
	// (a digest-only device build; B-1 host SHA-256s per call). Either way the tree is merkletree's
	// own (mdeNewTree): MerkleRoot(), VerifyTree(), VerifyContent() and RebuildTree() all work on it.
	// Built with -tags mde_nohashstrategy (merkletree without NewTreeWithHashStrategy,
	// merkle_gpu_nomemo.go) every tree is a host tree whatever this says (mdeHashStrategy = false).
	mdeHostTree = false
	// mdeHostCompressions counts the SHA-256 compressions this process ran on the host for the
	// trees it returned (the memo's misses, or every node of a host tree); batch_bench reports the
	// same count per call (tests/cpp/batch_bench.c).
	mdeHostCompressions uint64
)

// mdeHostTreeMaxBuckets: at most this many buckets, the tree is NewTree's on the host over a
// digest-only device build. A tree is a chain of dependent SHA-256 compressions: the CPU's SHA
// extensions (which crypto/sha256 uses on amd64) run B = 64's 94 compressions in ~5 us, while the
// device's share of the split tree (mde_server_build_levels) only starts paying above that:
// 16.9 vs 18.4 us per call at B = 64, equal at 96, 26.0 vs 22.7 at 128, 27.8 vs 35.8 at 256 and
// 48 vs 109 at 1,000 (profiles/r04/r04thr_hosttree_vs_levels.jsonl, INTEGRATION.md section 3).
const mdeHostTreeMaxBuckets = 64

// mdeEngine returns the batcher of the GPU that holds partitionId.
func mdeEngine(partitionId int) (*C.mde_batcher, error) {
	mdeOnce.Do(func() {
		n := int(C.mde_device_list(nil, 0))
		if n < 1 {
			mdeErr = errors.New("mde: no gfx950 GPU visible")
			return
		}
		// the HIP ordinals of the gfx950 devices (another GPU model may sit at a lower index)
		ords := make([]C.int, n)
		C.mde_device_list(&ords[0], C.int(n))
		for _, d := range ords {
			var b *C.mde_batcher
			var sv *C.mde_server
			// the service first (include/mde.h: services are created before, and destroyed after,
			// every other context of the device); 16 request slots (>= partition_concurrency),
			// buckets up to 1,024 in the resident launch
			if rc := C.mde_server_create(d, 16, 1024, &sv); rc != C.MDE_OK {
				log.Printf("mde: GPU %d skipped: mde_server_create: %s", int(d), C.GoString(C.mde_strerror(rc)))
				continue
			}
			// at most 256 partitions per batch, no wait window: a batch is whatever queued while the
			// previous batches ran
			if rc := C.mde_batcher_create(d, 256, 0, &b); rc != C.MDE_OK {
				log.Printf("mde: GPU %d skipped: mde_batcher_create: %s", int(d), C.GoString(C.mde_strerror(rc)))
				C.mde_server_destroy(sv)
				continue
			}
			mdeBatchers = append(mdeBatchers, b)
			mdeServers = append(mdeServers, sv)
		}
		if len(mdeBatchers) == 0 {
			mdeErr = errors.New("mde: no gfx950 GPU could be set up")
		}
	})
	if mdeErr != nil {
		return nil, mdeErr
	}
	return mdeBatchers[partitionId%len(mdeBatchers)], nil
}

// mdeServer returns the resident build service of the GPU that holds partitionId.
func mdeServer(partitionId int) (*C.mde_server, error) {
	if _, err := mdeEngine(partitionId); err != nil {
		return nil, err
	}
	return mdeServers[partitionId%len(mdeServers)], nil
}

// mdeTopNodes: with the resident service the device builds a tree's levels down to the first of at
// most this many nodes (mde_server_build_levels) and the host hashes the few levels above it: a
// tree's dependent top levels cost a core ~40 ns per compression on the SHA extensions
// crypto/sha256 uses, the device ~2 us (INTEGRATION.md section 3).
const mdeTopNodes = 64

// mdeTreeCompressions -- SHA-256 compressions of merkletree.NewTree over B buckets: one per 16-byte
// level-1 message, two per 64-byte message above (the odd-B duplicate leaf included).
func mdeTreeCompressions(B int) uint64 {
	n, c := B+B%2, uint64(0)
	for lvl := 1; n > 1; lvl++ {
		n = (n + 1) / 2
		if lvl == 1 {
			c += uint64(n)
		} else {
			c += 2 * uint64(n)
		}
	}
	return c
}

func cU64(v []uint64) unsafe.Pointer { return C.CBytes(unsafe.Slice((*byte)(unsafe.Pointer(&v[0])), len(v)*8)) }

// RawPartitionMerkleTree -- drop-in for main/merkle_tree.go:86-116. The per-bucket range scans are
// unchanged; the values go into one arena that the MI355X engine reduces, batched with the other
// partitions' calls in flight: bucket digests always on the device; for B > mdeHostTreeMaxBuckets
// the SHA-256 tree too, returned as its node hashes, from which merkletree's own construction takes
// every node the device built (mdeNewTree).
func (manager *Manager) RawPartitionMerkleTree(partitionId int, lowerEpoch, upperEpoch int64) (*merkletree.MerkleTree, error) {
	batcher, err := mdeEngine(partitionId)
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
	nodeBytes := 32 * int(C.mde_tree_internal_nodes(C.uint32_t(B)))
	cDigest := C.malloc(C.size_t(8 * B))
	cSize := C.malloc(C.size_t(4 * B))
	cItems := C.malloc(4)
	cRoot := C.malloc(32)
	cNodes := C.malloc(C.size_t(nodeBytes))
	defer C.free(cDigest)
	defer C.free(cSize)
	defer C.free(cItems)
	defer C.free(cRoot)
	defer C.free(cNodes)
	rec := C.mde_records{
		values: (*C.uint8_t)(cValues), values_bytes: C.uint64_t(len(values)),
		value_off: (*C.uint64_t)(cOff), n_records: C.uint64_t(len(valueOff) - 1),
		n_partitions: 1, n_buckets: C.uint32_t(B), seg_rec: (*C.uint64_t)(cSeg),
	}
	hostTree := mdeHostTree || !mdeHashStrategy || B <= mdeHostTreeMaxBuckets
	out := C.mde_tree_out{digest: (*C.uint64_t)(cDigest), size: (*C.int32_t)(cSize),
		items: (*C.int32_t)(cItems)}
	if !hostTree { // else a digest-only build: root and nodes stay NULL
		out.root, out.nodes = (*C.uint8_t)(cRoot), (*C.uint8_t)(cNodes)
	}
	var errBuf [512]C.char
	have := nodeBytes / 32 // device node hashes in cNodes (all of them unless the levels are split)
	if mdeResident {
		server, err := mdeServer(partitionId)
		if err != nil {
			return nil, err
		}
		if !hostTree { // the device's levels down to <= mdeTopNodes nodes; the memo misses the top ones
			out.root = nil
			if rc := C.mde_server_build_levels(server, &rec, &out, mdeTopNodes, &errBuf[0], C.uint64_t(len(errBuf))); rc != C.MDE_OK {
				return nil, errors.Errorf("mde_server_build_levels: %s", C.GoString(&errBuf[0]))
			}
			have = int(C.mde_tree_prefix_nodes(C.uint32_t(B), mdeTopNodes))
		} else if rc := C.mde_server_build(server, &rec, &out, &errBuf[0], C.uint64_t(len(errBuf))); rc != C.MDE_OK {
			return nil, errors.Errorf("mde_server_build: %s", C.GoString(&errBuf[0]))
		}
	} else if rc := C.mde_batch_build(batcher, &rec, &out, &errBuf[0], C.uint64_t(len(errBuf))); rc != C.MDE_OK {
		return nil, errors.Errorf("mde_batch_build: %s", C.GoString(&errBuf[0]))
	}
	digest := unsafe.Slice((*uint64)(cDigest), B)
	size := unsafe.Slice((*int32)(cSize), B)
	bucketList := make([]merkletree.Content, B)
	for i := 0; i < B; i++ {
		bucketList[i] = &MerkleBucket{bucketId: int32(i), hasher: &CustomHash{value: int64(digest[i])}, size: size[i]}
	}
	if !hostTree { // merkletree's construction, its node hashes from the device (the top levels of a split build hashed here)
		return mdeNewTree(bucketList, digest, unsafe.Slice((*byte)(cNodes), nodeBytes), have)
	}
	// merkletree.NewTree over the device digests (B-1 host SHA-256s: one compression per 16-byte
	// level-1 message, two per 64-byte message above)
	atomic.AddUint64(&mdeHostCompressions, mdeTreeCompressions(B))
	return merkletree.NewTree(bucketList)
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
	batcher, err := mdeEngine(partitionId)
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
	if mdeResident {
		server, err := mdeServer(partitionId)
		if err != nil {
			return false, 0, nil, nil, err
		}
		if rc := C.mde_server_verify(server, C.uint32_t(B), C.int32_t(partitionId), C.int64_t(epoch),
			(*C.uint64_t)(cDigest), (*C.int32_t)(cSize), C.uint32_t(R), (*C.uint8_t)(cBlob), (*C.uint64_t)(cOff),
			C.uint32_t(replicaCount), (*C.uint8_t)(unsafe.Pointer(&outs[0])), (*C.int32_t)(unsafe.Pointer(&outs[1])),
			(*C.int32_t)(cIds), (*C.int32_t)(unsafe.Pointer(&outs[2])), (*C.int32_t)(cStatus), (*C.uint8_t)(cObj),
			stride, (*C.uint32_t)(unsafe.Pointer(&outs[3])), &errBuf[0], C.uint64_t(len(errBuf))); rc != C.MDE_OK {
			return false, 0, nil, nil, errors.Errorf("mde_server_verify: %s", C.GoString(&errBuf[0]))
		}
	} else if rc := C.mde_batch_verify(batcher, C.uint32_t(B), C.int32_t(partitionId), C.int64_t(epoch),
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
