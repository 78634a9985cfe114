"""CPU: the Go shim's memoising hash strategy (integration/go/merkle_gpu.go mdeMemo / mdeMemoHash /
mdeNewTree), mirrored in Python over a restatement of cbergoon/merkletree v0.2.0's construction
with a pluggable hash strategy (NewTreeWithHashStrategy: one hasher per internal node, level 1
first, left to right; leaf Hash = LE64(digest); an odd leaf count duplicates the last leaf; the
last node of an odd level pairs with itself). The device's node hashes stand in as the oracle's
level-order nodes (the engine's `nodes` output layout, which the -m gpu tests prove equal).

What it pins, independent of a GPU or a Go toolchain:
  * with every device node in the memo, merkletree's tree equals NewTree's and no SHA-256 runs on
    the host; with the levels down to <= 64 nodes (mde_server_build_levels), exactly the nodes
    above them are hashed;
  * a hit is only ever the SHA-256 of the bytes asked about: a tampered leaf, a tree over other
    digests, or a construction that asks for the nodes in another order all give NewTree's tree
    of what was asked, with the misses hashed for real.
"""
import hashlib
import random

import pytest

from oracle import oracle as O


class Memo:
    """mdeMemo: the k-th hasher answers with device node k's hash iff its message is node k's."""

    def __init__(self, digests, nodes, have):
        self.leaf = [O.encode_int64_to_bytes(int(d)) for d in digests]
        if len(self.leaf) % 2 == 1:
            self.leaf.append(self.leaf[-1])
        self.nodes, self.have = nodes, have  # nodes: list of 32-byte hashes, level 1 .. root
        self.lvl, n = [], len(self.leaf)
        while n > 1:
            n = (n + 1) // 2
            self.lvl.append(n)
        self.next, self.compressions = 0, 0

    def message(self, k):
        if k >= self.have:
            return None
        off, below, prev = 0, len(self.leaf), -1
        for n in self.lvl:
            if k < off + n:
                j = k - off
                li, ri = 2 * j, (2 * j + 1 if 2 * j + 1 < below else 2 * j)
                if prev < 0:
                    return self.leaf[li] + self.leaf[ri]
                return self.nodes[prev + li] + self.nodes[prev + ri]
            prev, below, off = off, n, off + n
        return None

    def hasher(self):
        k = self.next
        self.next += 1

        def sum_(msg):  # mdeMemoHash.Sum over the bytes written to it
            if msg == self.message(k):
                return self.nodes[k]
            self.compressions += (len(msg) + 8) // 64 + 1
            return hashlib.sha256(msg).digest()
        return sum_


def new_tree_with_strategy(digests, strategy, order=None):
    """merkletree v0.2.0 buildWithContent + buildIntermediate, hashing every internal node with a
    fresh hasher from `strategy`. `order` permutes which hasher each node of a level receives (the
    real construction is order=None), to check that the memo is order-independent for
    correctness."""
    nl = [O.encode_int64_to_bytes(int(d)) for d in digests]
    if len(nl) % 2 == 1:
        nl.append(nl[-1])
    levels = []
    while len(nl) > 1:
        m = (len(nl) + 1) // 2
        idx = list(range(m))
        if order is not None:
            order.shuffle(idx)
        nxt = [None] * m
        for j in idx:
            r = 2 * j + 1 if 2 * j + 1 < len(nl) else 2 * j
            nxt[j] = strategy()(nl[2 * j] + nl[r])
        levels.append(nxt)
        nl = nxt
    return levels


def device_nodes(digests):
    return [h for lv in O.tree_levels_from_digests(digests)[1:] for h in lv]


def prefix_nodes(B, top):
    """mde_tree_prefix_nodes: the nodes of levels 1 .. the first of at most `top` nodes."""
    n, total = B + (B & 1), 0
    while n > 1:
        n = (n + 1) // 2
        total += n
        if n <= top:
            break
    return total


@pytest.mark.parametrize("B", [1, 2, 3, 30, 31, 64, 65, 100, 999, 1000, 1023])
def test_memo_with_every_device_node_hashes_nothing_on_the_host(B):
    rng = random.Random(B)
    d = [rng.randrange(999999) for _ in range(B)]
    nodes = device_nodes(d)
    memo = Memo(d, nodes, len(nodes))
    got = new_tree_with_strategy(d, memo.hasher)
    assert [h for lv in got for h in lv] == nodes
    assert got[-1][0] == O.tree_from_digests(d).merkle_root()
    assert memo.compressions == 0 and memo.next == len(nodes)


@pytest.mark.parametrize("B", [65, 100, 1000, 1023, 5000])
def test_memo_of_the_device_levels_hashes_only_the_top(B):
    """mde_server_build_levels' prefix in the memo: the host hashes exactly the nodes above it,
    two compressions each (64-byte messages)."""
    rng = random.Random(7 * B)
    d = [rng.randrange(999999) for _ in range(B)]
    nodes = device_nodes(d)
    have = prefix_nodes(B, 64)
    memo = Memo(d, nodes, have)
    got = new_tree_with_strategy(d, memo.hasher)
    assert [h for lv in got for h in lv] == nodes
    assert memo.compressions == 2 * (len(nodes) - have)


@pytest.mark.parametrize("B", [31, 64, 1000])
def test_memo_never_answers_for_bytes_the_device_did_not_hash(B):
    """A tampered leaf, a tree over unrelated digests and a shuffled construction order: every
    result is the SHA-256 tree of what was actually asked; only the misses cost host hashing."""
    rng = random.Random(11 * B)
    d = [rng.randrange(999999) for _ in range(B)]
    nodes = device_nodes(d)
    t = list(d)
    t[B // 2] = (t[B // 2] + 1) % 999999
    memo = Memo(d, nodes, len(nodes))
    got = new_tree_with_strategy(t, memo.hasher)
    assert [h for lv in got for h in lv] == device_nodes(t)
    depth = len(O.level_sizes(B)) - 1
    assert memo.compressions == 1 + 2 * (depth - 1)  # the tampered leaf's path to the root
    other = [rng.randrange(999999) for _ in range(B)]
    memo = Memo(d, nodes, len(nodes))
    assert [h for lv in new_tree_with_strategy(other, memo.hasher) for h in lv] == device_nodes(other)
    memo = Memo(d, nodes, len(nodes))
    got = new_tree_with_strategy(d, memo.hasher, order=random.Random(3))
    assert [h for lv in got for h in lv] == nodes
