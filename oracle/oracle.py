"""CPU restatement of the reference anti-entropy Merkle path -- TEST INFRASTRUCTURE ONLY.

This module is the *checker*. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it. The product (``mydatastore_amd``,
``libmde.so``) never imports, links or calls anything under ``oracle/``.

Parity status
-------------
* Index-key strings, iteration-range semantics, SHA-256 (FIPS 180-4) and XXH64: pinned by the
  reference's own known-answer tests (``main/indexs_test.go:18,32``,
  ``storage/index_test.go:19,30``) and by published KATs.
* Bucket digests, tree roots and diff lists: **relationally pinned only**. The reference's
  ``main/merkle_tree_test.go:86-184`` asserts relations (leaf count, bucket-id order,
  root equalities/inequalities, round-trip equality, empty/non-empty diffs), never absolute
  bytes, and the reference cannot be built here (no Go toolchain; the third-party
  ``github.com/cbergoon/merkletree v0.2.0`` source is absent). The tree-reduce semantics below are
  restated from that pinned version's published algorithm. Absolute tree bytes are therefore
  "parity unpinned" beyond those relations.

Every function cites the reference file:line it restates (paths relative to the reference root).
"""
from __future__ import annotations

import bisect
import hashlib
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

try:  # cespare/xxhash v1.1.0 == XXH64 seed 0; the python module is the same published algorithm
    import xxhash as _xxhash
except ImportError:  # pragma: no cover - xxhash is present in this image
    _xxhash = None

# main/merkle_tree.go:19
HASH_MOD = 999999
# main/indexs.go:11
EPOCH_LENGTH = 10


class MerkleError(Exception):
    """Mirrors the Go ``error`` returns of main/merkle_tree.go."""


# ---------------------------------------------------------------------------------------------
# utils/utils.go:67-89
# ---------------------------------------------------------------------------------------------
def encode_int64_to_bytes(value: int) -> bytes:
    """utils.EncodeInt64ToBytes (utils/utils.go:67-74): binary.Write LittleEndian int64."""
    return struct.pack("<q", value)


def decode_bytes_to_int64(data: bytes) -> int:
    """utils.DecodeBytesToInt64 (utils/utils.go:77-89): errors unless exactly 8 bytes."""
    if len(data) != 8:
        raise MerkleError("byte slice should be 8 bytes long for int64 decoding")
    return struct.unpack("<q", data)[0]


# ---------------------------------------------------------------------------------------------
# main/merkle_tree.go:21-84  CustomHash / MerkleBucket
# ---------------------------------------------------------------------------------------------
class CustomHash:
    """main/merkle_tree.go:21-56."""

    def __init__(self, value: int = 0):
        self.value = value

    def add(self, b: bytes) -> None:  # :25-32
        s = sum(b)
        self.value += s
        self.value = _go_mod(self.value, HASH_MOD)

    def remove(self, b: bytes) -> None:  # :34-44
        self.value -= sum(b)
        while self.value < 0:
            self.value += HASH_MOD
        self.value = _go_mod(self.value, HASH_MOD)

    def merge(self, other: "CustomHash") -> None:  # :46-52
        self.value += other.value
        while self.value < 0:
            self.value += HASH_MOD
        self.value = _go_mod(self.value, HASH_MOD)

    def hash(self) -> int:  # :54-56
        return self.value


def _go_mod(a: int, m: int) -> int:
    """Go's % truncates toward zero (sign follows the dividend)."""
    r = abs(a) % m
    return -r if a < 0 else r


@dataclass
class MerkleBucket:
    """main/merkle_tree.go:58-84 (implements merkletree.Content)."""

    bucket_id: int
    hasher: CustomHash
    size: int = 0

    def calculate_hash(self) -> bytes:  # :64-71
        return encode_int64_to_bytes(self.hasher.hash())

    def add_item(self, b: bytes) -> None:  # :73-76
        self.hasher.add(b)


# ---------------------------------------------------------------------------------------------
# github.com/cbergoon/merkletree v0.2.0 (main/go.mod:6) -- restated semantics
# ---------------------------------------------------------------------------------------------
@dataclass(eq=False)
class Node:
    hash: bytes
    left: Optional["Node"] = None
    right: Optional["Node"] = None
    c: Optional[MerkleBucket] = None
    leaf: bool = False
    dup: bool = False


@dataclass(eq=False)
class MerkleTree:
    root: Node
    leafs: List[Node] = field(default_factory=list)

    def merkle_root(self) -> bytes:
        return self.root.hash


def new_tree(contents: Sequence[MerkleBucket]) -> MerkleTree:
    """merkletree.NewTree (v0.2.0; called at main/merkle_tree.go:115,156).

    leaf.Hash = Content.CalculateHash(); an odd leaf count appends a duplicate of the last
    leaf (same hash, same content, dup=true); every level pairs (i, i+1) and the last node of an
    odd level pairs with itself; Hash = SHA256(left.Hash || right.Hash); the node produced from a
    2-node level is the root.
    """
    if not contents:
        raise MerkleError("error: cannot construct tree with no content")
    leafs = [Node(hash=c.calculate_hash(), c=c, leaf=True) for c in contents]
    if len(leafs) % 2 == 1:
        last = leafs[-1]
        leafs.append(Node(hash=last.hash, c=last.c, leaf=True, dup=True))
    nl = leafs
    while True:
        nodes = []
        for i in range(0, len(nl), 2):
            left, right = i, i + 1
            if i + 1 == len(nl):
                right = i
            h = hashlib.sha256(nl[left].hash + nl[right].hash).digest()
            n = Node(hash=h, left=nl[left], right=nl[right])
            nodes.append(n)
            if len(nl) == 2:
                return MerkleTree(root=n, leafs=leafs)
        nl = nodes


# ---------------------------------------------------------------------------------------------
# main/merkle_tree.go:118-216
# ---------------------------------------------------------------------------------------------
@dataclass
class EpochTreeObject:
    """datap/data.proto:60-68 (rpc.RpcEpochTreeObject)."""

    partition: int
    lower_epoch: int
    upper_epoch: int
    buckets: List[bytes]
    buckets_size: List[int]
    valid: bool = False
    items: int = 0


def merkle_tree_to_partition_epoch_object(tree: MerkleTree, partition_id: int, lower: int,
                                          upper: int) -> EpochTreeObject:
    """main/merkle_tree.go:118-138 -- iterates tree.Leafs, so an odd B yields B+1 buckets."""
    hashes, sizes, items = [], [], 0
    for leaf in tree.leafs:
        if not isinstance(leaf.c, MerkleBucket):
            raise MerkleError("failed to decode MerkleBucket")
        hashes.append(leaf.c.calculate_hash())
        sizes.append(leaf.c.size)
        items = _int32(items + leaf.c.size)
    return EpochTreeObject(partition=partition_id, lower_epoch=lower, upper_epoch=upper,
                           buckets=hashes, buckets_size=sizes, items=items)


def epoch_tree_object_to_merkle_tree(obj: EpochTreeObject) -> MerkleTree:
    """main/merkle_tree.go:140-157 -- sizes default to 0 when BucketsSize is short."""
    contents = []
    for i, bh in enumerate(obj.buckets):
        v = decode_bytes_to_int64(bh)
        size = obj.buckets_size[i] if i < len(obj.buckets_size) else 0
        contents.append(MerkleBucket(bucket_id=i, hasher=CustomHash(v), size=size))
    return new_tree(contents)


def different_merkle_tree_buckets(t1: MerkleTree, t2: MerkleTree) -> List[int]:
    """main/merkle_tree.go:159-161."""
    return different_merkle_tree_buckets_dfs(t1.root, t2.root)


def different_merkle_tree_buckets_dfs(n1: Optional[Node], n2: Optional[Node]) -> List[int]:
    """main/merkle_tree.go:163-216: pre-order; equal hash prunes; a differing leaf emits its
    bucketId (error if the ids differ); otherwise recurse Left then Right. A self-paired node
    has Left is Right, so its subtree is visited (and emitted) twice."""
    if n1 is None and n2 is None:
        return []
    if n1 is None or n2 is None:
        raise MerkleError("a merkletree.Node is nil")
    out: List[int] = []
    if n1.hash != n2.hash:
        if n1.left is None and n1.right is None:
            if not isinstance(n1.c, MerkleBucket):
                raise MerkleError("failed to decode MerkleBucket")
            if not isinstance(n2.c, MerkleBucket):
                raise MerkleError("failed to decode MerkleBucket")
            if n1.c.bucket_id != n2.c.bucket_id:
                raise MerkleError("bucketIds dont match")
            out.append(n1.c.bucket_id)
        else:
            out += different_merkle_tree_buckets_dfs(n1.left, n2.left)
            out += different_merkle_tree_buckets_dfs(n1.right, n2.right)
    return out


def _int32(x: int) -> int:
    return ((x + 2**31) % 2**32) - 2**31


# ---------------------------------------------------------------------------------------------
# Index keys: main/indexs.go:13-61, storage/index.go:8-110
# ---------------------------------------------------------------------------------------------
def _ordered(value: str, length: int) -> str:
    """storage/index.go:49-56 OrderedColumn.GetValue (zero pad; error if too long)."""
    if len(value) > length:
        raise MerkleError(f"index value invalid length {len(value)}")
    return "0" * (length - len(value)) + value


def build_index(name: str, columns: Sequence[str]) -> str:
    """storage/index.go:83-97 Index.Build: name and column values joined with '_'."""
    return "_".join([name, *columns])


def build_epoch_index(partition: int, bucket: int, epoch: int, key: str) -> str:
    """main/indexs.go:13-20."""
    return build_index("epoch", [str(partition), str(bucket), _ordered(str(epoch), EPOCH_LENGTH), key])


def parse_epoch_index(index: str):
    """main/indexs.go:22-48 (+ storage/index.go:99-110 Parse, OrderedColumn.Parse 58-64)."""
    parts = index.split("_")
    if len(parts) != 5:
        raise MerkleError("index columns and parts not equal")
    if parts[0] != "epoch":
        raise MerkleError("index name is wrong")
    epoch = parts[3].lstrip("0") or "0"
    return int(parts[1]), int(parts[2]), int(epoch), parts[4]


def build_key_index(key: str) -> str:
    """main/indexs.go:50-54."""
    return build_index("item", [key])


def build_epoch_tree_object_index(partition: int, epoch: int) -> str:
    """main/indexs.go:56-61."""
    return build_index("epochtree", [str(partition), _ordered(str(epoch), EPOCH_LENGTH)])


# ---------------------------------------------------------------------------------------------
# Write-time tagging: main/manager.go:773-778, hashring/hashring.go:89-110
# ---------------------------------------------------------------------------------------------
def get_key_bucket(key: bytes, n_buckets: int) -> int:
    """Manager.getKeyBucket (main/manager.go:773-778): BE64(SHA256(key)[:8]) % B."""
    h = hashlib.sha256(key).digest()
    return int.from_bytes(h[:8], "big") % n_buckets


def xxh64(data: bytes, seed: int = 0) -> int:
    """cespare/xxhash v1.1.0 Sum64 (hashring/hashring.go:89-93) == XXH64(data, seed=0)."""
    if _xxhash is None:  # pragma: no cover
        raise RuntimeError("xxhash module missing")
    return _xxhash.xxh64_intdigest(data, seed)


def find_partition_id(key: bytes, n_partitions: int) -> int:
    """Hashring.FindPartitionID (hashring/hashring.go:108-110) -> buraksezer/consistent v0.10.0
    FindPartitionID: int(Sum64(key) % partitionCount)."""
    return xxh64(key) % n_partitions


# ---------------------------------------------------------------------------------------------
# storage.Iterator contract (storage/storage.go:20-27; Badger storage/badger_storage.go:79-130)
# ---------------------------------------------------------------------------------------------
class MemStore:
    """Ordered in-memory KV with Badger iterator semantics: Seek(start), done when key >= limit."""

    def __init__(self):
        self._keys: List[bytes] = []
        self._vals: dict = {}

    def put(self, key: bytes, value: bytes) -> None:
        if key not in self._vals:
            bisect.insort(self._keys, key)
        self._vals[key] = bytes(value)

    def get(self, key: bytes) -> Optional[bytes]:
        return self._vals.get(key)

    def iterate(self, start: bytes, limit: bytes):
        i = bisect.bisect_left(self._keys, start)
        while i < len(self._keys) and self._keys[i] < limit:
            k = self._keys[i]
            yield k, self._vals[k]
            i += 1


class Manager:
    """The slice of main/manager.go that feeds and calls the Merkle path."""

    def __init__(self, partition_count: int, partition_buckets: int):
        self.partition_count = partition_count
        self.partition_buckets = partition_buckets
        self.db = MemStore()
        self._items: dict = {}

    def set_value(self, key: str, value: str, epoch: int, unix_timestamp: int) -> None:
        """Manager.SetValue (main/manager.go:780-818): epoch index -> LE64(timestamp)."""
        kb = key.encode()
        ts_bytes = encode_int64_to_bytes(unix_timestamp)
        p = find_partition_id(kb, self.partition_count)
        b = get_key_bucket(kb, self.partition_buckets)
        epoch_index = build_epoch_index(p, b, epoch, key)
        existing = self._items.get(key)
        if existing is not None:
            e_epoch, e_ts = existing
            if e_epoch >= epoch and e_ts > unix_timestamp:
                raise MerkleError("a newer value already exists")
        self._items[key] = (epoch, unix_timestamp)
        self.db.put(build_key_index(key).encode(), value.encode())
        self.db.put(epoch_index.encode(), ts_bytes)

    def raw_partition_merkle_tree(self, partition_id: int, lower: int, upper: int) -> MerkleTree:
        """Manager.RawPartitionMerkleTree (main/merkle_tree.go:86-116)."""
        buckets = []
        for i in range(self.partition_buckets):
            bucket = MerkleBucket(bucket_id=i, hasher=CustomHash())
            lo = build_epoch_index(partition_id, i, lower, "").encode()
            hi = build_epoch_index(partition_id, i, upper, "").encode()
            size = 0
            for _, v in self.db.iterate(lo, hi):
                bucket.add_item(v)
                size += 1
            bucket.size = size
            buckets.append(bucket)
        return new_tree(buckets)

    def stream_buckets(self, partition_id: int, buckets, lower: int, upper: int):
        """StreamBucketsTask (main/manager.go:445-487): an empty list is every bucket (:448-452);
        the list is walked in the order given (:453), each bucket's range scan streamed whole
        (:454-483) -- a repeated bucket streams again, a bucket no record carries streams
        nothing. Returns [(key, epoch, timestamp)]."""
        buckets = list(buckets) if len(buckets) else list(range(self.partition_buckets))
        out = []
        for b in buckets:
            out.extend(self.bucket_records(partition_id, b, lower, upper) if b >= 0 else [])
        return out

    def bucket_records(self, partition_id: int, bucket: int, lower: int, upper: int):
        """The records one bucket's range scan yields (StreamBucketsTask main/manager.go:445-487)."""
        lo = build_epoch_index(partition_id, bucket, lower, "").encode()
        hi = build_epoch_index(partition_id, bucket, upper, "").encode()
        out = []
        for k, v in self.db.iterate(lo, hi):
            _, _, epoch, key = parse_epoch_index(k.decode())
            out.append((key, epoch, decode_bytes_to_int64(v)))
        return out


# ---------------------------------------------------------------------------------------------
# main/manager.go:1036-1118 -- VerifyEpoch's decision step
# ---------------------------------------------------------------------------------------------
VERIFY_DECODE = "decode"  # EpochTreeObjectToMerkleTree (or proto.Unmarshal) failed
VERIFY_TREE = "tree"      # DifferentMerkleTreeBuckets returned an error


def tree_from_digests(digests: Sequence[int], sizes: Optional[Sequence[int]] = None) -> MerkleTree:
    """RawPartitionMerkleTree's tree for given bucket digests/sizes (bucket i -> id i)."""
    sizes = list(sizes) if sizes is not None else [0] * len(digests)
    return new_tree([MerkleBucket(bucket_id=i, hasher=CustomHash(int(d)), size=int(sizes[i]))
                     for i, d in enumerate(digests)])


def verify_epoch(my_tree: MerkleTree, partition_id: int, epoch: int,
                 peer_objects: Sequence[Optional[bytes]], replica_count: int):
    """Manager.VerifyEpoch (main/manager.go:1036-1118) after the peer fetch: the local object
    (:1041), each peer object -> tree (:1076) -> diff against my tree (:1081), peers whose object
    or diff fails are skipped (:1077-1084), diffSet = Int32Set of all successful diffs (:1086),
    validCount / validDiff (:1088-1097), valid = validCount >= ReplicaCount || validDiff (:1100).
    A missing peer (None) contributes nothing, like an object that yields no tree.
    Returns dict(valid, valid_count, diff (sorted set), status (per peer: diff length or
    VERIFY_DECODE / VERIFY_TREE), object (the persisted EpochTreeObject wire bytes))."""
    from oracle import wire_pb

    obj = merkle_tree_to_partition_epoch_object(my_tree, partition_id, epoch, epoch + 1)
    valid_count, valid_diff, diff_set, status = 0, False, set(), []
    for raw in peer_objects:
        try:
            m = wire_pb.unmarshal(raw or b"")
            other = epoch_tree_object_to_merkle_tree(EpochTreeObject(
                partition=m.partition, lower_epoch=m.lower_epoch, upper_epoch=m.upper_epoch,
                buckets=list(m.buckets), buckets_size=list(m.buckets_size), valid=m.valid,
                items=m.items))
        except Exception:  # MerkleError / DecodeError: logrus.Error; continue
            status.append(VERIFY_DECODE)
            continue
        try:
            diff = different_merkle_tree_buckets(my_tree, other)
        except MerkleError:
            status.append(VERIFY_TREE)
            continue
        diff_set.update(diff)
        if not diff:
            valid_count += 1
        elif m.valid:
            valid_diff = True
        status.append(len(diff))
    valid = valid_count >= replica_count or valid_diff
    digests = [decode_bytes_to_int64(h) for h in obj.buckets]
    wire = wire_pb.marshal(partition_id, epoch, epoch + 1, digests, obj.buckets_size, valid=valid,
                           items=obj.items)
    return {"valid": valid, "valid_count": valid_count, "diff": sorted(diff_set), "status": status,
            "object": wire}


# ---------------------------------------------------------------------------------------------
# Array form used to check the device engine (same semantics as above, flat layout)
# ---------------------------------------------------------------------------------------------
def level_sizes(n_buckets: int) -> List[int]:
    """Node count per level: [n0 (leaves incl. dup), n1, ..., 1]."""
    n = n_buckets + (n_buckets & 1)
    sizes = [n]
    while n > 1:
        n = (n + 1) // 2
        sizes.append(n)
    return sizes


def n_internal_nodes(n_buckets: int) -> int:
    return sum(level_sizes(n_buckets)[1:])


def tree_levels_from_digests(digests: Sequence[int]) -> List[List[bytes]]:
    """Level 0 = 8-byte leaves (with dup); levels 1.. = 32-byte SHA-256 nodes; last = [root]."""
    leaves = [encode_int64_to_bytes(int(d)) for d in digests]
    if len(leaves) % 2 == 1:
        leaves.append(leaves[-1])
    levels = [leaves]
    nl = leaves
    while len(nl) > 1:
        nxt = []
        for i in range(0, len(nl), 2):
            r = i + 1 if i + 1 < len(nl) else i
            nxt.append(hashlib.sha256(nl[i] + nl[r]).digest())
        levels.append(nxt)
        nl = nxt
    return levels


def internal_nodes_blob(digests: Sequence[int]) -> bytes:
    """Internal nodes level 1..root, 32 bytes each (the engine's ``nodes`` output layout)."""
    return b"".join(b"".join(lv) for lv in tree_levels_from_digests(digests)[1:])


def diff_from_digests(d1: Sequence[int], d2: Sequence[int]) -> List[int]:
    """DifferentMerkleTreeBuckets on trees rebuilt from digest vectors."""
    t1 = new_tree([MerkleBucket(i, CustomHash(int(v))) for i, v in enumerate(d1)])
    t2 = new_tree([MerkleBucket(i, CustomHash(int(v))) for i, v in enumerate(d2)])
    return different_merkle_tree_buckets(t1, t2)


def bucket_digests(values: np.ndarray, value_off: np.ndarray, seg_rec: np.ndarray):
    """digest[s] = (sum of value bytes of records seg_rec[s]..seg_rec[s+1]) mod 999999, i.e. the
    fold of CustomHash.Add (main/merkle_tree.go:25-32) over the bucket's records, and
    size[s] = record count (main/merkle_tree.go:91,107,111). ``value_off`` is the [N+1] byte-offset
    array of a contiguous value arena (record r = values[value_off[r]:value_off[r+1]])."""
    values = np.asarray(values, dtype=np.uint8)
    csum = np.zeros(values.size + 1, dtype=np.uint64)
    np.cumsum(values, dtype=np.uint64, out=csum[1:])
    byte_lo = value_off[seg_rec[:-1]]
    byte_hi = value_off[seg_rec[1:]]
    sums = csum[byte_hi] - csum[byte_lo]
    digest = (sums % np.uint64(HASH_MOD)).astype(np.uint64)
    size = (seg_rec[1:] - seg_rec[:-1]).astype(np.int32)
    return digest, size


# ---------------------------------------------------------------------------------------------
# Synthetic workload
# ---------------------------------------------------------------------------------------------
SYNTH_SEED = 0x4D445354  # "MDST"
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z: np.ndarray) -> np.ndarray:
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def synth_value_words(gids: np.ndarray, n_words: int, seed: int = SYNTH_SEED) -> np.ndarray:
    """[len(gids), n_words] u64: word w of record gid = splitmix64(seed ^ (gid * 2^20 + w))."""
    g = np.asarray(gids, dtype=np.uint64)[:, None]
    w = np.arange(n_words, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        x = np.uint64(seed) ^ ((g << np.uint64(20)) + w)
    return splitmix64(x)


def synth_values(gids: np.ndarray, value_len: int, seed: int = SYNTH_SEED) -> np.ndarray:
    """[len(gids), value_len] u8: the little-endian bytes of the record's splitmix words."""
    n_words = (value_len + 7) // 8
    words = synth_value_words(gids, n_words, seed).astype("<u8")
    return words.view(np.uint8).reshape(len(gids), n_words * 8)[:, :value_len]


def synth_key(gid: int) -> bytes:
    return b"k%016x" % gid


def synth_tags(gids: Sequence[int], n_partitions: int, n_buckets: int, part_mode: str,
               keys_per_partition: int = 0):
    """(partition, bucket) per synthetic record. part_mode: 'block' (gid // kpp), 'mod'
    (gid % P) or 'hash' (FindPartitionID); bucket always = getKeyBucket(key)."""
    parts, bks = [], []
    for g in gids:
        k = synth_key(int(g))
        if part_mode == "block":
            p = int(g) // keys_per_partition
        elif part_mode == "mod":
            p = int(g) % n_partitions
        else:
            p = find_partition_id(k, n_partitions)
        parts.append(p)
        bks.append(get_key_bucket(k, n_buckets))
    return np.asarray(parts, dtype=np.int64), np.asarray(bks, dtype=np.int64)


def layout_a(parts: np.ndarray, bks: np.ndarray, n_partitions: int, n_buckets: int):
    """LSM order: records sorted by (partition, bucket) (stable), + seg_rec[P*B+1] boundaries."""
    comp = parts * n_buckets + bks
    order = np.argsort(comp, kind="stable")
    counts = np.bincount(comp, minlength=n_partitions * n_buckets)
    seg_rec = np.zeros(n_partitions * n_buckets + 1, dtype=np.uint64)
    np.cumsum(counts, out=seg_rec[1:])
    return order, seg_rec


# ---------------------------------------------------------------------------------------------
# StreamBucketsTask's list contract over the arena (main/manager.go:447-485): requests in the
# order given, repeats streamed again, ids outside [0, B) stream nothing, an empty list is every
# bucket. mde_stream_buckets' checker.
# ---------------------------------------------------------------------------------------------
def stream_buckets_from_arena(values, value_off, seg_rec, n_partitions, n_buckets, ids, ids_stride, counts):
    """Per partition, the requests of ids[p*ids_stride : +counts[p]] in order (counts[p] == 0:
    buckets 0..B-1; < 0: none), each bucket's records in LSM order. Returns (part_off, rec_idx,
    value_bytes, value_off_out)."""
    part_off, recs, chunks, voff = [0], [], [], [0]
    for p in range(n_partitions):
        c = int(counts[p])
        row = (range(n_buckets) if c == 0 else
               [int(x) for x in ids[p * ids_stride:p * ids_stride + max(c, 0)]])
        for b in row:
            if not 0 <= b < n_buckets:
                continue
            s = p * n_buckets + b
            for r in range(int(seg_rec[s]), int(seg_rec[s + 1])):
                recs.append(r)
                v = values[int(value_off[r]):int(value_off[r + 1])]
                chunks.append(v)
                voff.append(voff[-1] + len(v))
        part_off.append(len(recs))
    vb = np.concatenate(chunks) if chunks else np.zeros(0, np.uint8)
    return (np.asarray(part_off, np.uint64), np.asarray(recs, np.uint64), vb.astype(np.uint8),
            np.asarray(voff, np.uint64))


# ---------------------------------------------------------------------------------------------
# Out-of-sync range extract: StreamBucketsTask (main/manager.go:445-487) over the de-duplicated
# diff set (utils.Int32Set, main/manager.go:1073,1086,1114), array form
# ---------------------------------------------------------------------------------------------
def extract_from_arena(values, value_off, seg_rec, n_partitions, n_buckets, ids, ids_stride, counts):
    """Per partition: records of the requested buckets, duplicates removed, ascending bucket
    order (the reference's order is Go map order, i.e. unspecified), LSM record order within a
    bucket. Returns (part_off, rec_idx, value_bytes, value_off_out)."""
    part_off, recs, chunks, voff = [0], [], [], [0]
    for p in range(n_partitions):
        c = int(counts[p])
        row = ids[p * ids_stride:p * ids_stride + max(c, 0)]
        for b in sorted({int(x) for x in row if 0 <= int(x) < n_buckets}):
            s = p * n_buckets + b
            for r in range(int(seg_rec[s]), int(seg_rec[s + 1])):
                recs.append(r)
                v = values[int(value_off[r]):int(value_off[r + 1])]
                chunks.append(v)
                voff.append(voff[-1] + len(v))
        part_off.append(len(recs))
    vb = np.concatenate(chunks) if chunks else np.zeros(0, np.uint8)
    return (np.asarray(part_off, np.uint64), np.asarray(recs, np.uint64), vb.astype(np.uint8),
            np.asarray(voff, np.uint64))
