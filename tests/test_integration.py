"""CPU: the cgo shim (integration/go/merkle_gpu.go) binds only what include/mde.h declares.

There is no Go toolchain in this image, so the shim cannot be compiled here; this checks, by
parsing, that every C function, constant, type and struct field it names exists in the header
with the argument count the shim passes.
"""
import re
from pathlib import Path

from tests.conftest import ROOT

GO_DIR = ROOT / "integration" / "go"
GO = GO_DIR / "merkle_gpu.go"
GO_MEMO = GO_DIR / "merkle_gpu_memo.go"          # //go:build !mde_nohashstrategy
GO_NOMEMO = GO_DIR / "merkle_gpu_nomemo.go"      # //go:build mde_nohashstrategy
HEADER = ROOT / "include" / "mde.h"


GO_TEST = GO_DIR / "merkle_gpu_test.go"         # go test: the shim against the reference + oracle


def _shim_sources():
    return {p.name: p.read_text() for p in sorted(GO_DIR.glob("*.go")) if not p.name.endswith("_test.go")}


def _imports_used(code, name):
    imports = re.search(r"import \((.*?)\)", code, re.S).group(1)
    body = code[code.index(imports) + len(imports):]
    for pkg in re.findall(r'"([\w./-]+)"', imports):
        if pkg != "C":
            assert re.search(r"\b" + re.escape(pkg.rsplit("/", 1)[-1]) + r"\.", body), (name, pkg)


def _header():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    funcs = {}
    for m in re.finditer(r"\b(mde_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", text, re.S):
        args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        funcs[m.group(1)] = len(args)
    consts = set(re.findall(r"#define\s+(MDE_[A-Z0-9_]+)", text))
    types = set(re.findall(r"typedef\s+struct\s+\w+\s+(mde_\w+)\s*;", text))
    structs = {}
    for m in re.finditer(r"typedef\s+struct\s+(mde_\w+)\s*\{(.*?)\}\s*(mde_\w+)\s*;", text, re.S):
        body = re.sub(r"//.*", "", m.group(2))
        structs[m.group(3)] = set(re.findall(r"\**\s*(\w+)\s*;", body))
        types.add(m.group(3))
    return funcs, consts, types, structs


def _call_args(src, start):
    """Top-level comma count of the call whose '(' is at src[start]."""
    depth, n, i = 0, 0, start
    saw = False
    while True:
        c = src[i]
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
            if depth == 0:
                return n + 1 if saw else 0
        elif c == "," and depth == 1:
            n += 1
        elif not c.isspace() and depth >= 1:
            saw = True
        i += 1


def test_shim_names_exist_in_header():
    funcs, consts, types, structs = _header()
    src = "\n".join(_shim_sources().values())
    code = re.sub(r"//.*", "", src)
    used_funcs = set(re.findall(r"\bC\.(mde_[a-z0-9_]+)\s*\(", code))
    used_types = set(re.findall(r"\bC\.(mde_[a-z0-9_]+)\b(?!\s*\()", code))
    used_consts = set(re.findall(r"\bC\.(MDE_[A-Z0-9_]+)", code))
    assert used_funcs, "no C calls found"
    assert not used_funcs - set(funcs), used_funcs - set(funcs)
    assert not used_types - types, used_types - types
    assert not used_consts - consts, used_consts - consts
    for m in re.finditer(r"\bC\.(mde_[a-z0-9_]+)\s*\(", code):
        n = _call_args(code, m.end() - 1)
        assert n == funcs[m.group(1)], (m.group(1), n, funcs[m.group(1)])
    for m in re.finditer(r"\bC\.(mde_records|mde_tree_out)\{(.*?)\}", code, re.S):
        fields = set(re.findall(r"(\w+)\s*:", m.group(2)))
        assert fields and not fields - structs[m.group(1)], (m.group(1), fields - structs[m.group(1)])


def test_shim_reimplements_the_reference_signatures():
    """The replaced function keeps the reference's Go signature (main/merkle_tree.go:86); the
    reference's own DifferentMerkleTreeBuckets (:159-216) stays, so the shim must not redefine it
    (two definitions in package main would not compile). Every tree the shim returns is built by
    merkletree itself -- NewTree, or NewTreeWithHashStrategy fed by the memo of device node hashes
    -- never as a struct literal, whose unexported merkleRoot / leaf / dup / Tree fields would stay
    unset (MerkleRoot() nil, VerifyTree() walking into nil children)."""
    src = "\n".join(_shim_sources().values())
    code = re.sub(r"//.*", "", src)
    assert ("func (manager *Manager) RawPartitionMerkleTree(partitionId int, lowerEpoch, upperEpoch int64) "
            "(*merkletree.MerkleTree, error)") in src
    assert "func DifferentMerkleTreeBuckets(" not in code
    assert "merkletree.MerkleTree{" not in code and "merkletree.Node{" not in code
    assert "merkletree.NewTreeWithHashStrategy(cs, func() hash.Hash" in code
    assert "return merkletree.NewTree(bucketList)" in code
    # mdeMemoHash is a hash.Hash (io.Writer + Sum + Reset + Size + BlockSize)
    for method in ("Write(p []byte) (int, error)", "Sum(b []byte) []byte", "Reset()", "Size() int",
                   "BlockSize() int"):
        assert f"func (h *mdeMemoHash) {method}" in code, method
    # Sum answers from the device only for node k's exact message, and copies out (merkletree
    # appends to the hashes it gets back); the memo is switched off once the tree exists
    assert "bytes.Equal(h.buf[:len(l)], l) && bytes.Equal(h.buf[len(l):], r)" in code
    assert "return append(b, h.m.nodes[h.k*32:(h.k+1)*32]...)" in code
    assert "m.active, m.nodes = false, nil" in code


def test_shim_hash_strategy_constructor_is_build_tagged():
    """The memoised construction names merkletree.NewTreeWithHashStrategy, whose presence at the
    pinned v0.2.0 (main/go.sum:3) cannot be checked without Go. Go compiles every function of a
    file it builds, so the fallback must be a build tag, not a variable: the constructor and the
    memo live only in merkle_gpu_memo.go (//go:build !mde_nohashstrategy); merkle_gpu_nomemo.go
    (//go:build mde_nohashstrategy) defines mdeNewTree with the same signature as plain NewTree;
    each defines mdeHashStrategy, and the main file uses only mdeNewTree / mdeHashStrategy."""
    srcs = _shim_sources()
    assert set(srcs) == {GO.name, GO_MEMO.name, GO_NOMEMO.name}
    code = {n: re.sub(r"//.*", "", s) for n, s in srcs.items()}
    first = {n: s.lstrip().splitlines()[0] for n, s in srcs.items()}
    assert first[GO_MEMO.name] == "//go:build !mde_nohashstrategy"
    assert first[GO_NOMEMO.name] == "//go:build mde_nohashstrategy"
    assert not first[GO.name].startswith("//go:build")
    for n, c in code.items():
        assert ("NewTreeWithHashStrategy" in c) == (n == GO_MEMO.name), n
        assert ("mdeMemo" in c) == (n == GO_MEMO.name), n
    sig = re.compile(r"^func mdeNewTree\((.*?)\) \((.*?)\) \{", re.M)
    sigs = {n: sig.findall(c) for n, c in code.items()}
    assert sigs[GO.name] == []
    assert len(sigs[GO_MEMO.name]) == 1 and sigs[GO_MEMO.name] == sigs[GO_NOMEMO.name]
    assert "const mdeHashStrategy = true" in code[GO_MEMO.name]
    assert "const mdeHashStrategy = false" in code[GO_NOMEMO.name]
    assert "return merkletree.NewTree(cs)" in code[GO_NOMEMO.name]
    # without the constructor the device builds digests only: every tree is a host tree
    assert "hostTree := mdeHostTree || !mdeHashStrategy ||" in code[GO.name]
    assert "mdeNewTree(bucketList, digest," in code[GO.name]
    # each file imports what it uses (an unused import is a Go compile error)
    for n, c in code.items():
        _imports_used(c, n)


def test_go_parity_test_pins_the_oracle_fixtures():
    """integration/go/merkle_gpu_test.go is the test a maintainer with Go and a GPU runs to pin the
    oracle's tree bytes against the reference's own construction (merkletree v0.2.0 + Go's SHA-256):
    its predicted roots and diff lists are exactly tests/golden/testmerkletreeraw_n{10,100}.json's,
    it runs every path of the shim, and it names only the shim's and the reference's functions."""
    import json
    src = GO_TEST.read_text()
    code = re.sub(r"//.*", "", src)
    assert src.startswith("// merkle_gpu_test.go") and "package main" in code
    _imports_used(code, GO_TEST.name)
    for n in (10, 100):
        fx = json.loads((ROOT / "tests" / "golden" / f"testmerkletreeraw_n{n}.json").read_text())
        m = re.search(r"\b%d: \{\[3\]string\{(.*?)\},\s*\[\]int32\{(.*?)\}\}" % n, code, re.S)
        assert m, n
        roots = re.findall(r'"([0-9a-f]{64})"', m.group(1))
        assert roots == [fx["trees"][k]["root"] for k in ("0_3", "1_3", "2_3")], n
        assert [int(x) for x in re.findall(r"-?\d+", m.group(2))] == fx["diffs"]["t1_t3"], n
        assert fx["n_buckets"] == 30 and fx["n"] == n
    assert "c.Manager.PartitionBuckets = 30" in code and "n = 10" in code and "n := 100" in code
    # every path: resident service / batcher x device tree / host tree
    assert "for _, resident := range []bool{true, false}" in code
    assert "for _, hostTree := range []bool{false, true}" in code
    assert "manager.RawPartitionMerkleTree(0, r[0], r[1])" in code and "mdeSameTree(t, what, got, want)" in code
    # the reference's construction, restated over the same store (main/merkle_tree.go:86-116)
    assert "leaf.hasher.Add(it.Value())" in code and "return merkletree.NewTree(cs)" in code
    # no second definition of anything the shim or the reference defines
    shim = "\n".join(_shim_sources().values())
    defined = set(re.findall(r"^func (?:\([^)]*\) )?(\w+)", code, re.M))
    assert defined == {"mdeRefTree", "mdeSameTree", "TestMdeRawPartitionMerkleTreeMatchesReference"}
    assert not any(re.search(r"^func (?:\([^)]*\) )?%s\(" % d, shim, re.M) for d in defined)
    called = {"mdeEngine", "NewManager", "initMetrics", "BuildEpochIndex", "DifferentMerkleTreeBuckets"}
    for f in called:
        assert re.search(r"\b%s\(" % f, code), f
    assert re.search(r"^func mdeEngine\(", shim, re.M)
    ref = Path("/root/reference/main")
    if ref.is_dir():  # this container only: the reference's package defines the rest
        refsrc = "\n".join(p.read_text() for p in ref.glob("*.go") if not p.name.endswith("_test.go"))
        for f in called - {"mdeEngine"}:
            assert re.search(r"^func (?:\([^)]*\) )?%s\(" % f, refsrc, re.M), f
        assert re.search(r"^func \(\w+ \*Manager\) SetValue\(", refsrc, re.M)
        assert not re.search(r"^func (?:\([^)]*\) )?(mdeRefTree|mdeSameTree|mdePredicted)\b", refsrc, re.M)


# ---------------------------------------------------------------------------------------------
# The shim's call sequences, replayed from C (tests/cpp/shim_replay.c) and checked against the
# oracle's restatement of the reference functions the shim replaces.
import pytest  # noqa: E402

REPLAY = ROOT / "tests" / "cpp" / "build" / "shim_replay"


def _walk_sig(root):
    """SHA-256 of the tree's pre-order walk (shim_replay.c `walk`): every node's Hash, and each
    leaf's bucketId as LE32 -- a self-paired node's subtree is walked twice, as the DFS does."""
    import hashlib
    import struct
    out = bytearray()

    def go(n):
        out.extend(n.hash)
        if n.left is None and n.right is None:
            out.extend(struct.pack("<i", n.c.bucket_id))
            return
        go(n.left)
        go(n.right)
    go(root)
    return hashlib.sha256(bytes(out)).hexdigest()


def _levels(B):
    """Node counts of merkletree v0.2.0's internal levels for B buckets (level 1 .. root)."""
    n, out = B + (B & 1), []
    while n > 1:
        n = (n + 1) // 2
        out.append(n)
    return out


def _host_compressions(B, path):
    """SHA-256 compressions the shim runs on the host for one B-bucket tree (mdeHostCompressions):
    B <= 64 -- NewTree over the device digests, every node (one compression per 16-byte level-1
    message, two per 64-byte message above); B > 64 through the resident service -- the nodes above
    the device's levels (down to the first of at most mdeTopNodes = 64 nodes); through the batcher
    -- none, every node hash comes from the device."""
    lv = _levels(B)
    if B <= 64:
        return lv[0] + 2 * sum(lv[1:])
    if path == "batcher":
        return 0
    k = next(i for i, n in enumerate(lv) if n <= 64)
    return 2 * sum(lv[k + 1:])


def _replay_scenarios(path="resident"):
    """(input tokens, expected output line) per op, from the oracle (oracle/oracle.py)."""
    import numpy as np
    from oracle import oracle as O
    from oracle import wire_pb
    rng = np.random.default_rng(2024)
    lines, expect = [], []

    # RawPartitionMerkleTree: one partition, the arena filled record by record
    def build(B, n, lens):
        bucket = np.sort(rng.integers(0, B, n)) if n else np.zeros(0, np.int64)
        vals = [rng.integers(0, 256, int(ln), dtype=np.uint8).tobytes() for ln in lens]
        toks = ["build", str(B), str(n)] + [str(int(b)) for b in bucket] + [v.hex() or "-" for v in vals]
        lines.append(" ".join(toks))
        voff = np.zeros(n + 1, np.uint64)
        voff[1:] = np.cumsum([len(v) for v in vals])
        seg = np.searchsorted(bucket, np.arange(B + 1)).astype(np.uint64)
        arena = np.frombuffer(b"".join(vals) or b"\0", np.uint8)
        d, z = O.bucket_digests(arena, voff, seg)
        t = O.tree_from_digests(d, z)
        items = O.merkle_tree_to_partition_epoch_object(t, 0, 0, 1).items
        expect.append(f"build {' '.join(map(str, d))} ; {' '.join(map(str, z))} ; {items} ; "
                      f"{t.merkle_root().hex()} ; {len(t.leafs)} {_walk_sig(t.root)} ; "
                      f"{_host_compressions(B, path)} 1")
        return list(map(int, d)), list(map(int, z))

    build(31, 300, rng.integers(0, 41, 300))                  # variable lengths, empty values, odd B
    build(64, 1000, [8] * 1000)                                # 8-byte timestamps
    d1000, z1000 = build(1000, 5000, [8] * 5000)               # the reference's default B
    build(30, 0, [])                                           # no records: one padding byte
    d31, z31 = build(31, 200, rng.integers(1, 17, 200))
    # the memoised merkletree construction just above the host-tree cutoff, at odd and even B, and
    # past the service's 1,024-bucket launch (the service's context writes every level there)
    for B, n in ((65, 400), (100, 700), (1023, 4000), (5000, 20000)):
        build(B, n, [8] * n)

    # DifferentMerkleTreeBuckets (the reference's DFS over two trees of the shim's shape): local
    # B = 31 (merkletree duplicates the last leaf) against a tree rebuilt from an odd-B object
    # (B + 1 distinct leaves)
    def diff(local, peer_src):
        t1 = O.tree_from_digests(local)
        t2 = O.epoch_tree_object_to_merkle_tree(
            O.merkle_tree_to_partition_epoch_object(O.tree_from_digests(peer_src), 0, 0, 1))
        peer_leaves = [O.decode_bytes_to_int64(l.c.calculate_hash()) for l in t2.leafs]
        lines.append(" ".join(["diff", str(len(local)), str(len(peer_leaves))] + list(map(str, local)) +
                     list(map(str, peer_leaves))))
        try:
            ids = O.different_merkle_tree_buckets(t1, t2)
            expect.append(" ".join(["diff", str(len(ids))] + list(map(str, ids))))
        except O.MerkleError:
            expect.append("diff -4")

    diff(d31, d31)                                              # equal: the duplicate leaves agree
    p = list(d31)
    p[5] = (p[5] + 1) % 999999
    diff(d31, p)                                                # one inner bucket differs
    p = list(d31)
    p[30] = (p[30] + 7) % 999999
    diff(d31, p)                                                # the duplicated bucket differs
    p = list(d1000)
    p[999] = (p[999] + 1) % 999999
    diff(d1000, p)                                              # even B: same leaf counts

    # VerifyEpoch's decision: an agreeing odd-B object, an absent peer, a garbage peer, a differing
    # object marked Valid (validDiff), and B = 1000 with another bucket count
    def verify(d, z, peers, rc, part=7, epoch=4):
        t = O.tree_from_digests(d, z)
        lines.append(" ".join(["verify", str(len(d)), str(part), str(epoch), str(rc), str(len(peers))] +
                              list(map(str, d)) + list(map(str, z)) + [(x.hex() if x else "-") for x in peers]))
        w = O.verify_epoch(t, part, epoch, peers, rc)
        st = [O_STATUS.get(s, s) for s in w["status"]]
        expect.append(f"verify {int(w['valid'])} {w['valid_count']} ; {' '.join(map(str, w['diff']))} ; "
                      f"{' '.join(map(str, st))} ; {w['object'].hex()}")

    O_STATUS = {O.VERIFY_DECODE: -6, O.VERIFY_TREE: -4}

    def obj(d, z, valid=False):
        t = O.tree_from_digests(d, z)
        o = O.merkle_tree_to_partition_epoch_object(t, 7, 4, 5)
        return wire_pb.marshal(7, 4, 5, [O.decode_bytes_to_int64(h) for h in o.buckets], o.buckets_size,
                               valid=valid, items=o.items)

    p = list(d31)
    p[3] = (p[3] + 1) % 999999
    verify(d31, z31, [obj(d31, z31), None, b"\xff\xff\xff", obj(p, z31, valid=True)], 2)
    verify(d31, z31, [obj(d31, z31), None, b"\x0a"], 1)
    q = list(d1000)
    q[10] = (q[10] + 1) % 999999
    verify(d1000, z1000, [obj(q, z1000), obj(d1000[:998], z1000[:998]), None], 3)
    return lines, expect


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["resident", "batcher"])
def test_shim_call_sequences_replayed_from_c_match_oracle(tmp_path, path):
    """The Go shim's exact ABI call sequences (integration/go/merkle_gpu.go, which cannot be
    compiled here), replayed in C: RawPartitionMerkleTree's one-partition arena with value_off
    built record by record -> mde_server_build_levels (the shim's default; mde_batch_build for
    path="batcher") with nodes -> merkletree's own construction fed by the memo of the device's
    node hashes (mdeNewTree: Root.Hash, leaf count and the whole pre-order walk equal NewTree's;
    host compressions = the nodes above the device's levels through the service, 0 through the
    batcher, every node for B <= 64; a tampered tree misses the memo and is hashed for real) at
    B in {30, 31, 64, 65, 100, 1000, 1023, 5000};
    the reference's DFS over trees of that shape, B local leaves against B + 1 peer leaves
    (odd-B object quirk);
    verifyEpochDecision with agreeing, absent, garbage, Valid-differing and other-B peers ->
    mde_server_verify / mde_batch_verify. Every output equals the oracle's restatement of the reference
    (main/merkle_tree.go:86-216, main/manager.go:1072-1104)."""
    import subprocess
    lines, expect = _replay_scenarios(path)
    f = tmp_path / "scenarios.txt"
    f.write_text("\n".join(lines) + "\n")
    r = subprocess.run([str(REPLAY), str(f), path], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = r.stdout.strip().splitlines()
    assert len(got) == len(expect)
    for i, (g, e) in enumerate(zip(got, expect)):
        assert " ".join(g.split()) == " ".join(e.split()), (i, lines[i][:80])


def test_shim_replay_scenarios_exercise_every_branch():
    """CPU: the replay's expectations cover the branches the verdict asked for -- an error diff
    (the duplicated odd-B bucket), a non-empty diff, the padding byte of an empty arena, and absent
    (-6), garbage (-6) and other-shape peers."""
    lines, expect = _replay_scenarios()
    assert any(e == "diff -4" for e in expect)
    assert any(e.startswith("diff 1 5") for e in expect)
    assert any(e.startswith("build") and e.split(" ; ")[2] == "0" for e in expect)
    verifies = [e for e in expect if e.startswith("verify")]
    assert all("-6" in v.split(" ; ")[2] for v in verifies)
    assert verifies[0].startswith("verify 1 ")  # validDiff: a differing peer object marked Valid
