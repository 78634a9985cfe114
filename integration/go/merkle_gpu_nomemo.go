//go:build mde_nohashstrategy

// merkle_gpu_nomemo.go -- the shim's tree construction for a merkletree without
// NewTreeWithHashStrategy (`go build -tags mde_nohashstrategy`, INTEGRATION.md section 2). Every
// returned tree is plain merkletree.NewTree over the device's bucket digests, with the same results
// and method set as the memoised construction of merkle_gpu_memo.go and B-1 host SHA-256s per call;
// with mdeHashStrategy = false RawPartitionMerkleTree asks the device for digests only, so nothing
// here ever receives device node hashes.
package main

import (
	"sync/atomic"

	"github.com/cbergoon/merkletree"
)

// mdeHashStrategy: merkletree's construction hashes every node on the host (this file).
const mdeHashStrategy = false

// mdeNewTree -- merkle_gpu_memo.go's signature; the device's node hashes are not used.
func mdeNewTree(cs []merkletree.Content, digest []uint64, nodes []byte, have int) (*merkletree.MerkleTree, error) {
	atomic.AddUint64(&mdeHostCompressions, mdeTreeCompressions(len(digest)))
	return merkletree.NewTree(cs)
}
