//go:build !mde_nohashstrategy

// merkle_gpu_memo.go -- the shim's tree construction when the pinned cbergoon/merkletree
// (main/go.mod:6, main/go.sum:3: v0.2.0) has NewTreeWithHashStrategy: merkletree builds its own tree
// and takes each internal node's hash from the device's node hashes (mdeMemo) instead of hashing it
// on the host. This is the only file that names that constructor. If a Go build of the shim finds
// it undefined at the pinned version, build with `go build -tags mde_nohashstrategy`:
// merkle_gpu_nomemo.go then supplies mdeNewTree (same signature) as plain merkletree.NewTree and the
// shim does digest-only device builds (mdeHashStrategy = false, INTEGRATION.md section 2).
package main

import (
	"bytes"
	"crypto/sha256"
	"encoding/binary"
	"hash"
	"sync/atomic"

	"github.com/cbergoon/merkletree"
)

// mdeHashStrategy: merkletree's construction can take node hashes from the device (this file).
const mdeHashStrategy = true

// mdeMemo -- what the device already hashed, in the order merkletree asks for it. cbergoon/merkletree
// v0.2.0's construction (buildIntermediate) takes one hasher from the hash strategy per internal
// node, level 1 first, left to right within a level -- the order of mde_tree_out.nodes -- and writes
// it that node's message: left.Hash || right.Hash (two 8-byte LE64 leaves at level 1,
// main/merkle_tree.go:64-71 and utils/utils.go:67-74; two 32-byte hashes above), the duplicate of
// the last leaf when B is odd, the last node of an odd level paired with itself. The k-th hasher
// answers with device node k's hash only when the message it was written is exactly node k's
// message as the device hashed it; otherwise it runs SHA-256. A hit is therefore always the
// SHA-256 of the bytes merkletree asked about, whatever order or tree it comes from (a tampered
// leaf, another tree); the order only decides how often it hits. O(1) per node: no map, no copy
// of the device's nodes.
type mdeMemo struct {
	leaf   [][]byte // LE64 leaf hashes (+ the odd-B duplicate)
	nodes  []byte   // the device's node hashes, level 1 .. root, 32 bytes each
	have   int      // how many of them the device wrote (its levels; all of them for a whole tree)
	lvl    []int    // node count of each internal level, level 1 first
	next   int      // the node merkletree's construction hashes next
	active bool     // false once the tree exists: later hashers are plain SHA-256
}

func newMdeMemo(digest []uint64, nodes []byte, have int) *mdeMemo {
	B := len(digest)
	m := &mdeMemo{leaf: make([][]byte, B, B+1), nodes: nodes, have: have, active: true}
	for i := 0; i < B; i++ {
		m.leaf[i] = make([]byte, 8)
		binary.LittleEndian.PutUint64(m.leaf[i], digest[i])
	}
	if B%2 == 1 {
		m.leaf = append(m.leaf, m.leaf[B-1])
	}
	for n := len(m.leaf); n > 1; {
		n = (n + 1) / 2
		m.lvl = append(m.lvl, n)
	}
	return m
}

// message of device node k: its children's hashes (nil when k is past the device's nodes)
func (m *mdeMemo) message(k int) ([]byte, []byte) {
	if k >= m.have {
		return nil, nil
	}
	off, below, prev := 0, len(m.leaf), -1
	for _, n := range m.lvl {
		if k < off+n {
			j := k - off
			li, ri := 2*j, 2*j
			if 2*j+1 < below {
				ri = 2*j + 1
			}
			if prev < 0 {
				return m.leaf[li], m.leaf[ri]
			}
			return m.nodes[(prev+li)*32 : (prev+li+1)*32], m.nodes[(prev+ri)*32 : (prev+ri+1)*32]
		}
		prev, below, off = off, n, off+n
	}
	return nil, nil
}

// mdeMemoHash -- the hash.Hash the strategy hands merkletree for node k: Write buffers the node's
// message; Sum returns the device's hash of node k when the message is node k's, else SHA-256.
type mdeMemoHash struct {
	m   *mdeMemo
	k   int
	buf []byte
}

func (h *mdeMemoHash) Write(p []byte) (int, error) { h.buf = append(h.buf, p...); return len(p), nil }
func (h *mdeMemoHash) Reset()                      { h.buf = h.buf[:0] }
func (h *mdeMemoHash) Size() int                   { return sha256.Size }
func (h *mdeMemoHash) BlockSize() int              { return sha256.BlockSize }
func (h *mdeMemoHash) Sum(b []byte) []byte {
	if l, r := h.m.message(h.k); l != nil && len(h.buf) == len(l)+len(r) &&
		bytes.Equal(h.buf[:len(l)], l) && bytes.Equal(h.buf[len(l):], r) {
		return append(b, h.m.nodes[h.k*32:(h.k+1)*32]...) // a copy: merkletree appends to node hashes
	}
	atomic.AddUint64(&mdeHostCompressions, uint64(len(h.buf)+8)/64+1)
	sum := sha256.Sum256(h.buf)
	return append(b, sum[:]...)
}

// mdeNewTree -- merkletree's own tree over the buckets (digest: the bucket digests; nodes: the
// device's node hashes, level 1 .. root, of which the first `have` were written), its internal hashes taken from the memo (no
// host SHA-256 for the nodes the device built): merkletree.NewTreeWithHashStrategy runs its own
// construction (leafs, the odd-B duplicate, parents, merkleRoot), so MerkleRoot(), VerifyTree(),
// VerifyContent() and RebuildTree() behave as on a NewTree tree. Once the tree exists the memo is
// switched off: a later VerifyTree / RebuildTree hashes with real SHA-256, as the reference's trees
// do.
func mdeNewTree(cs []merkletree.Content, digest []uint64, nodes []byte, have int) (*merkletree.MerkleTree, error) {
	m := newMdeMemo(digest, nodes, have)
	t, err := merkletree.NewTreeWithHashStrategy(cs, func() hash.Hash {
		if !m.active {
			return sha256.New()
		}
		h := &mdeMemoHash{m: m, k: m.next}
		m.next++
		return h
	})
	m.active, m.nodes = false, nil
	return t, err
}
