"""Build the engine's native libraries in-tree (hipcc for gfx950; gcc for the oracle).

  python -m mydatastore_amd._build            # libmde.so (+ host mirror, C++ tests, oracle)

Outputs (git-ignored, but shipped to the GPU box with the snapshot):
  mydatastore_amd/libmde.so         C ABI (include/mde.h) + gfx950 kernels
  mydatastore_amd/libmde_host.so    C++ mirror of main/merkle_tree.go over the C ABI
  tests/cpp/build/test_merkle_tree  C++ port of the reference's Merkle tests
  tests/cpp/build/cabi_bench        plain-C driver of the C ABI (C4 build, no PyTorch)
  tests/cpp/build/group_cabi        plain-C driver of the multi-GPU path (mde_group, no PyTorch)
  tests/cpp/build/batch_test        concurrent callers of the batcher vs mde_build / the C oracle
  tests/cpp/build/batch_bench       production call shape: CPU oracle vs per-call vs batched, P callers
  tests/cpp/build/shim_replay       the Go shim's call sequences replayed from C (checked by pytest)
  tests/cpp/build/server_test       concurrent callers of the resident build service vs mde_build / the C oracle
  oracle/build/liboracle.so         CPU restatement (test infrastructure only)
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
HIP_FLAGS = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall",
             "-Wno-unused-function", f"-I{ROOT / 'include'}"]

LIB = PKG / "libmde.so"
HOST_LIB = PKG / "libmde_host.so"
ORACLE_LIB = ROOT / "oracle" / "build" / "liboracle.so"
CPP_TEST = ROOT / "tests" / "cpp" / "build" / "test_merkle_tree"
C_BENCH = ROOT / "tests" / "cpp" / "build" / "cabi_bench"
GROUP_CABI = ROOT / "tests" / "cpp" / "build" / "group_cabi"
BATCH_TEST = ROOT / "tests" / "cpp" / "build" / "batch_test"
BATCH_BENCH = ROOT / "tests" / "cpp" / "build" / "batch_bench"
SHIM_REPLAY = ROOT / "tests" / "cpp" / "build" / "shim_replay"
SERVER_TEST = ROOT / "tests" / "cpp" / "build" / "server_test"


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True)


def build_engine(verbose: bool = True) -> Path:
    OBJ.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.hpp")) + [ROOT / "include" / "mde.h"]
    sources = sorted(CSRC.glob("*.hip")) + [CSRC / "mde_api.cpp", CSRC / "batch.cpp", CSRC / "group.cpp", CSRC / "server.cpp"]
    objs, jobs = [], []
    for src in sources:
        obj = OBJ / (src.stem + ".o")
        if _stale(obj, [src, *headers]):
            lang = ["-x", "hip"] if src.suffix == ".hip" else []
            jobs.append([HIPCC, *HIP_FLAGS, *lang, "-c", src, "-o", obj])
        objs.append(obj)
    # the translation units compile independently: in parallel, up to the CPU share
    # (MAX_JOBS / OMP_NUM_THREADS on a GPU box, else the cores, at most 8)
    from concurrent.futures import ThreadPoolExecutor
    share = os.environ.get("MAX_JOBS") or os.environ.get("OMP_NUM_THREADS") or str(os.cpu_count() or 1)
    workers = max(1, min(8, int(share) if share.isdigit() else 1, len(jobs) or 1))
    with ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(_run, j, verbose) for j in jobs]:
            f.result()
    if _stale(LIB, objs):
        _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-pthread", "-o", LIB, *objs, "-ldl"], verbose)
    return LIB


def build_host(verbose: bool = True) -> Path:
    hdir = PKG / "host"
    srcs = sorted(hdir.glob("*.cpp"))
    deps = [*srcs, *hdir.glob("*.hpp"), ROOT / "include" / "mde.h", LIB]
    if srcs and _stale(HOST_LIB, deps):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{ROOT / 'include'}",
              *srcs, "-o", HOST_LIB, f"-L{PKG}", "-lmde", f"-Wl,-rpath,$ORIGIN"], verbose)
    test_src = ROOT / "tests" / "cpp" / "test_merkle_tree.cpp"
    if test_src.exists() and _stale(CPP_TEST, [test_src, *deps, HOST_LIB]):
        CPP_TEST.parent.mkdir(parents=True, exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-Wall", f"-I{ROOT / 'include'}", f"-I{hdir}", test_src,
              "-o", CPP_TEST, f"-L{PKG}", "-lmde_host", "-lmde",
              f"-Wl,-rpath,{PKG}", "-Wl,-rpath,$ORIGIN/../../../mydatastore_amd"], verbose)
    for name, out in (("cabi_bench.c", C_BENCH), ("group_cabi.c", GROUP_CABI)):
        c_src = ROOT / "tests" / "cpp" / name
        if c_src.exists() and _stale(out, [c_src, ROOT / "include" / "mde.h", LIB]):
            out.parent.mkdir(parents=True, exist_ok=True)
            _run(["gcc", "-O2", "-std=c11", "-D_POSIX_C_SOURCE=199309L", "-Wall", f"-I{ROOT / 'include'}",
                  c_src, "-o", out, f"-L{PKG}", "-lmde", f"-Wl,-rpath,{PKG}",
                  "-Wl,-rpath,$ORIGIN/../../../mydatastore_amd"], verbose)
    # test programs that also link the C oracle (test infrastructure) as their checker
    for name, out in (("batch_test.c", BATCH_TEST), ("batch_bench.c", BATCH_BENCH), ("shim_replay.c", SHIM_REPLAY),
                      ("server_test.c", SERVER_TEST)):
        src = ROOT / "tests" / "cpp" / name
        if src.exists() and _stale(out, [src, ROOT / "include" / "mde.h", LIB, ORACLE_LIB]):
            out.parent.mkdir(parents=True, exist_ok=True)
            _run(["gcc", "-O2", "-std=c11", "-D_GNU_SOURCE", "-Wall", f"-I{ROOT / 'include'}", src, "-o", out,
                  f"-L{PKG}", "-lmde", f"-L{ORACLE_LIB.parent}", "-loracle", "-lpthread",
                  f"-Wl,-rpath,{PKG}", f"-Wl,-rpath,{ORACLE_LIB.parent}",
                  "-Wl,-rpath,$ORIGIN/../../../mydatastore_amd", "-Wl,-rpath,$ORIGIN/../../../oracle/build"],
                 verbose)
    return HOST_LIB


def build_oracle(verbose: bool = True) -> Path:
    src = ROOT / "oracle" / "mde_oracle.c"
    if _stale(ORACLE_LIB, [src]):
        ORACLE_LIB.parent.mkdir(parents=True, exist_ok=True)
        _run(["gcc", "-O2", "-fPIC", "-shared", "-Wall", src, "-o", ORACLE_LIB, "-lpthread"], verbose)
    return ORACLE_LIB


def build_all(verbose: bool = True) -> None:
    build_engine(verbose)
    build_oracle(verbose)
    build_host(verbose)


if __name__ == "__main__":
    build_all(verbose="-q" not in sys.argv)
