"""CPU: the C-ABI library builds for gfx950, loads, and exports exactly what include/mde.h
declares. No compute calls are made here (no GPU in this container)."""
import re
import subprocess
import sys

import pytest

from tests.conftest import ROOT

HEADER = ROOT / "include" / "mde.h"


@pytest.fixture(scope="module")
def lib():
    import mydatastore_amd as mde
    if not mde.LIB_PATH.exists():
        subprocess.run([sys.executable, "-m", "mydatastore_amd._build", "-q"], cwd=ROOT, check=True)
    return mde.load_library()


def _declared():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(mde_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported(lib):
    import mydatastore_amd as mde
    declared = _declared()
    assert declared == sorted(mde.EXPORTED_SYMBOLS)
    nm = subprocess.run(["nm", "-D", "--defined-only", str(mde.LIB_PATH)], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mde_[a-z0-9_]+)$", nm, re.M))
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    for s in declared:
        getattr(lib, s)


def test_gfx950_code_object(lib):
    import mydatastore_amd as mde
    blob = mde.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx90a" not in blob and b"gfx942" not in blob


def test_geometry_matches_oracle(lib):
    from oracle import oracle as O
    import mydatastore_amd as mde
    for B in list(range(1, 70)) + [99, 100, 1000, 4096, 4097, 99999]:
        sizes = O.level_sizes(B)
        assert mde.tree_internal_nodes(B) == sum(sizes[1:]), B
        assert mde.tree_depth(B) == len(sizes) - 1, B
    assert mde.diff_capacity(30, 30) == 32 and mde.diff_capacity(64, 64) == 64
    assert mde.diff_capacity(6, 8) == 8 and mde.diff_capacity(2, 3) == 2
    assert lib.mde_abi_version() == 1
    assert lib.mde_strerror(-4) == b"merkle trees do not match in shape"


def test_no_fallback_without_gpu(lib):
    """The product fails loudly without a gfx950 device -- it never falls back to the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import mydatastore_amd as mde
    with pytest.raises(mde.MdeError) as e:
        mde.Engine(0)
    assert e.value.code == mde.MDE_E_DEVICE


def test_product_never_uses_oracle():
    """Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may touch oracle/."""
    for p in (ROOT / "mydatastore_amd").rglob("*"):
        if p.suffix in {".py", ".cpp", ".hip", ".hpp", ".h"}:
            src = p.read_text()
            assert "import oracle" not in src and "from oracle" not in src, p
            assert "liboracle" not in src or p.name == "_build.py", p


def test_last_error_copy_truncates_and_terminates(lib):
    """mde_last_error_copy / mde_group_last_error_copy: at most cap-1 bytes + NUL, full length
    returned (the shared-context-safe way to read a message)."""
    import ctypes as C
    buf = C.create_string_buffer(b"\xff" * 8, 8)
    assert lib.mde_last_error_copy(None, buf, 8) == len(b"null context")
    assert buf.raw == b"null co\0"
    assert lib.mde_last_error_copy(None, None, 0) == len(b"null context")
    big = C.create_string_buffer(64)
    assert lib.mde_group_last_error_copy(None, big, 64) == len(b"null group")
    assert big.value == b"null group"


def test_product_sources_carry_no_probe_code():
    """the product kernels compile only the variants plan_digest can select
    (ids 11..16) and no probe sites -- no preprocessor conditional on an MDE_* macro anywhere in
    the library's sources, so no stray -D can change what libmde.so computes. The per-wave
    timeline stamps live in tools/probe_stamps.patch, applied to a scratch copy by
    tools/build_probe_lib.sh; the patch must still apply to today's sources."""
    import re
    import shutil
    import subprocess
    import tempfile
    from tests.conftest import ROOT
    csrc = ROOT / "mydatastore_amd" / "csrc"
    for f in sorted(csrc.iterdir()):
        if f.suffix in (".hip", ".cpp", ".hpp"):
            bad = [ln for ln in f.read_text().splitlines() if re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b.*\bMDE_", ln)]
            assert not bad, (f.name, bad)
    digest = (csrc / "digest.hip").read_text()
    assert re.findall(r"MDE_VARIANT\((\d+),", digest) == [str(i) for i in range(11, 17)]
    if shutil.which("patch"):
        with tempfile.TemporaryDirectory() as d:
            shutil.copy(csrc / "digest.hip", d)
            r = subprocess.run(["patch", "-p1", "--dry-run", "-i", str(ROOT / "tools" / "probe_stamps.patch")],
                               cwd=d, capture_output=True, text=True)
            assert r.returncode == 0, r.stdout + r.stderr
