"""The C++ port of the reference's Merkle tests (tests/cpp/test_merkle_tree.cpp) over the host
mirror + engine; its printed roots and diffs must equal the golden fixtures."""
import subprocess
import sys

import pytest

from tests.conftest import ROOT

BIN = ROOT / "tests" / "cpp" / "build" / "test_merkle_tree"


def test_cpp_port_builds():
    subprocess.run([sys.executable, "-m", "mydatastore_amd._build", "-q"], cwd=ROOT, check=True)
    assert BIN.exists()
    assert (ROOT / "mydatastore_amd" / "libmde_host.so").exists()


@pytest.mark.gpu
def test_cpp_port_matches_golden(golden):
    r = subprocess.run([str(BIN)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = {(ln.split()[0], ln.split()[1]): (ln.split()[2] if len(ln.split()) > 2 else "")
             for ln in r.stdout.splitlines() if ln.startswith(("ROOT", "DIFF", "ITEMS", "WIRE"))}
    for n in (100, 10):
        fix = golden(f"testmerkletreeraw_n{n}.json")
        for key in ("0_3", "1_3", "2_3"):
            assert lines[("ROOT", f"n{n}_{key}")] == fix["trees"][key]["root"]
        assert lines[("DIFF", f"n{n}_t1_t3")] == ",".join(map(str, fix["diffs"]["t1_t3"]))
        assert int(lines[("ITEMS", f"n{n}_0_3")]) == fix["trees"]["0_3"]["items"]
        assert lines[("WIRE", f"n{n}_0_3")] == fix["trees"]["0_3"]["wire"]
    assert "PASS" in r.stdout
