"""CPU: the C oracle (test infrastructure every GPU parity test trusts) under AddressSanitizer and
UndefinedBehaviorSanitizer, over seeded random shapes (tests/cpp/oracle_asan.c): builds with 1 and
3 threads agree, the array tree, both graph forms and the DFS diff agree, layout A sorts, and the
SHA-256 / XXH64 known answers hold -- with no sanitizer report."""
import subprocess

import pytest

from tests.conftest import ROOT


def test_oracle_clean_under_asan_and_ubsan(tmp_path):
    exe = tmp_path / "oracle_asan"
    cmd = ["gcc", "-O1", "-g", "-std=c11", "-D_GNU_SOURCE", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined",
           str(ROOT / "tests" / "cpp" / "oracle_asan.c"), str(ROOT / "oracle" / "mde_oracle.c"),
           "-o", str(exe), "-lpthread", "-lm"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode and "asan" in (b.stderr or "").lower():
        pytest.skip("no sanitizer runtime: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-2000:]
    r = subprocess.run([str(exe), "300"], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "PATH": "/usr/bin:/bin"})
    assert r.returncode == 0 and r.stdout.startswith("ok 300"), (r.stdout[-500:], r.stderr[-3000:])
