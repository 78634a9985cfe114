"""CPU: mde_group's per-device enqueue threads (mydatastore_amd/csrc/enq_pool.hpp, used by
csrc/group.cpp run_all) under ThreadSanitizer -- every call runs every share exactly once on its
own thread, the lowest failing share's code comes back, and workers that went to sleep between
calls are woken (a lost wake-up would hang: the timeout fails it). Host code only; the pool has no
HIP in it, so the test needs no GPU."""
import shutil
import subprocess

import pytest

from tests.conftest import ROOT

SRC = ROOT / "tests" / "cpp" / "enq_pool_test.cpp"
OUT = ROOT / "tests" / "cpp" / "build"


def _build(name, flags):
    OUT.mkdir(parents=True, exist_ok=True)
    exe = OUT / name
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-pthread", *flags, str(SRC), "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    return exe if r.returncode == 0 else None


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("sanitizer", ["thread", None])
def test_enq_pool_under_stress(sanitizer):
    exe = _build("enq_pool_test_tsan" if sanitizer else "enq_pool_test",
                 ["-fsanitize=thread"] if sanitizer else [])
    if exe is None and sanitizer:
        pytest.skip("g++ cannot build with -fsanitize=thread here")
    assert exe is not None
    env = {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66"}
    r = subprocess.run([str(exe), "1500" if sanitizer else "6000"], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert r.stdout.startswith("ok ")
