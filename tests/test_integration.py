"""CPU: the cgo shim (integration/go/merkle_gpu.go) binds only what include/mde.h declares.

There is no Go toolchain in this image, so the shim cannot be compiled here; this checks, by
parsing, that every C function, constant, type and struct field it names exists in the header
with the argument count the shim passes.
"""
import re

from tests.conftest import ROOT

GO = ROOT / "integration" / "go" / "merkle_gpu.go"
HEADER = ROOT / "include" / "mde.h"


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
    src = GO.read_text()
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
    """The two replaced functions keep the reference's Go signatures (main/merkle_tree.go:86,159)."""
    src = GO.read_text()
    assert ("func (manager *Manager) RawPartitionMerkleTree(partitionId int, lowerEpoch, upperEpoch int64) "
            "(*merkletree.MerkleTree, error)") in src
    assert ("func DifferentMerkleTreeBuckets(tree1 *merkletree.MerkleTree, tree2 *merkletree.MerkleTree) "
            "([]int32, error)") in src
