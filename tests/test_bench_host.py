"""CPU tests of bench.py's host side: the oracle sample a rank regenerates for its partitions
(tests/sample.py) equals the matching rows of the oracle's whole-workload build, the config-5
perturbation changes exactly one bucket per partition, and the CPU-share rule."""
import numpy as np
import pytest

from tests.sample import host_sample, perturb_first_record

P, B, N_KEYS, V = 12, 16, 3000, 40


def _full(co, mode):
    kpp = -(-N_KEYS // P)
    g = np.arange(N_KEYS, dtype=np.uint64)
    part, bk = co.synth_tags(g, P, B, {"block": 0, "mod": 1}[mode], kpp)
    order, seg = co.layout_a(part, bk, P, B)
    vals = co.synth_values(g[order], V, 0x4D445354)
    return co.build(vals, seg, P, B, V)


@pytest.mark.parametrize("mode", ["mod", "block"])
@pytest.mark.parametrize("sample", [[0, 1, 2], [3, 7, 11], [11], list(range(12))])
def test_host_sample_equals_whole_build_rows(coracle, mode, sample):
    full = _full(coracle, mode)
    values, seg, n, _ = host_sample(coracle, N_KEYS, P, V, B, mode, sample)
    ref = coracle.build(values, seg, n, B, V)
    ni = full["nodes"].size // P
    for i, p in enumerate(sample):
        assert np.array_equal(ref["digest"][i * B:(i + 1) * B], full["digest"][p * B:(p + 1) * B])
        assert np.array_equal(ref["size"][i * B:(i + 1) * B], full["size"][p * B:(p + 1) * B])
        assert ref["items"][i] == full["items"][p]
        assert np.array_equal(ref["root"][i * 32:(i + 1) * 32], full["root"][p * 32:(p + 1) * 32])
        assert np.array_equal(ref["nodes"][i * ni:(i + 1) * ni], full["nodes"][p * ni:(p + 1) * ni])


def test_perturbed_replica_differs_in_exactly_one_bucket(coracle):
    sample = list(range(P))
    values, seg, n, _ = host_sample(coracle, N_KEYS, P, V, B, "mod", sample)
    vb, touched = perturb_first_record(values, seg, V, B, sample)
    a = coracle.build(values, seg, n, B, V)
    b = coracle.build(vb, seg, n, B, V)
    for i in range(n):
        want = [touched[i]] if i in touched else []
        assert coracle.diff(a["digest"][i * B:(i + 1) * B], b["digest"][i * B:(i + 1) * B]) == want
        assert want == [] or touched[i] == (sample[i] * 37) % B


def test_cpu_share_rule():
    import bench
    info = {"nproc": 192, "affinity_cpus": 192, "cgroup_cpu_quota": None, "omp_num_threads": 16}
    assert bench.cpu_share(info) == 16
    assert bench.cpu_share(info, world=8) == 2
    info = {"nproc": 8, "affinity_cpus": 8, "cgroup_cpu_quota": 4.0, "omp_num_threads": None}
    assert bench.cpu_share(info) == 4
    info = {"nproc": 8, "affinity_cpus": None, "cgroup_cpu_quota": None, "omp_num_threads": None}
    assert bench.cpu_share(info) == 8
    h = bench.host_cpu_info()
    assert h["nproc"] and "cpu_model" in h


def test_group_bench_ranks_join_rank0s_barriers():
    """CPU: under torch.distributed.run the group bench's rank 0 drives every GPU and the other
    ranks only join its barriers, so their count must equal rank 0's: two around each timed run
    (the bucketed run, plus for C4 the run with one gather per build) and one at the end. Counted
    from bench.py's source, so a new barrier on one side fails here instead of hanging a launch."""
    import ast
    from tests.conftest import ROOT
    src = (ROOT / "bench.py").read_text()
    tree = ast.parse(src)
    mg = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main_group")
    timed = next(n for n in ast.walk(mg) if isinstance(n, ast.FunctionDef) and n.name == "timed")

    def barriers(node):
        return sum(1 for n in ast.walk(node) if isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute)
                   and n.func.attr == "barrier")
    per_timed = barriers(timed)
    calls_of_timed = sum(1 for n in ast.walk(mg) if isinstance(n, ast.Call) and isinstance(n.func, ast.Name)
                         and n.func.id == "timed")
    others = barriers(mg) - per_timed  # outside timed(): the non-zero ranks' loop + rank 0's final one
    assert per_timed == 2 and calls_of_timed == 2 and others == 2
    # the non-zero ranks' count: 2 per timed run + 1, the per-build run only for C4 with steps > 0
    assert "n_barriers = 2 * (2 if per_build_run else 1) + 1" in src
    assert "per_build_run = not c5 and not args.no_gather_per_build and args.steps > 0" in src
    assert "if per_build_run:\n        one = Run(1)" in src


def test_default_warmup_covers_the_clock_ramp():
    """--warmup W is taken as given; the default is >= 3 steps covering >= WARMUP_MIN_MS of device
    time, from the faster of two 3-step calibrations (the VALU-bound
    production step reads ~12 % slow after 3 warm-up builds that follow an idle spell)."""
    import argparse
    import bench
    calls = []

    def calibrate(ms_per_step):
        def f(k):
            calls.append(k)
            return k * ms_per_step
        return f
    assert bench.resolve_warmup(argparse.Namespace(warmup=5), calibrate(1.0)) == 5 and calls == []
    assert bench.resolve_warmup(argparse.Namespace(warmup=0), calibrate(1.0)) == 0 and calls == []
    c4 = bench.resolve_warmup(argparse.Namespace(warmup=None), calibrate(1.48))
    prod = bench.resolve_warmup(argparse.Namespace(warmup=None), calibrate(0.17))
    c3 = bench.resolve_warmup(argparse.Namespace(warmup=None), calibrate(12.0))
    assert calls == [3] * 6
    assert c4 * 1.48 >= bench.WARMUP_MIN_MS and (c4 - 1) * 1.48 < bench.WARMUP_MIN_MS
    assert prod * 0.17 >= bench.WARMUP_MIN_MS and c3 == 3


def test_gpurun_upload_keeps_what_the_bench_reads():
    """bench.py reads profiles/pmc_traffic.json on the GPU box for roofline.traffic; a
    .gpurunignore pattern that drops it from the upload silently nulls the field."""
    import fnmatch
    from tests.conftest import ROOT
    pats = [p.strip() for p in (ROOT / ".gpurunignore").read_text().splitlines() if p.strip()]
    for path in ("./profiles/pmc_traffic.json", "./bench.py", "./mydatastore_amd/libmde.so",
                 "./oracle/build/liboracle.so"):
        for p in pats:
            parts = path.split("/")
            prefixes = ["/".join(parts[:i]) for i in range(2, len(parts) + 1)]
            hit = (any(fnmatch.fnmatch(x, p) for x in prefixes) if p.startswith("./")
                   else any(fnmatch.fnmatch(x, p) for x in parts[1:]))
            assert not hit, (path, p)


def test_production_shape_is_measured_before_the_host_legs():
    """The N = 1 line measures the production shape first, on the warm GPU: measured after the
    end-to-end leg, the standalone digest of the bench process read 12 % slow (DESIGN.md 4.9,
    profiles/r06/r06s_*.json). Both engines keep that order: production shape, CPU baseline,
    end to end."""
    import re
    from tests.conftest import ROOT
    src = (ROOT / "bench.py").read_text()
    for start in ("def main_group(", "def main("):
        body = src[src.index(start):]
        body = body[:body.index("\ndef ", 1)] if "\ndef " in body[1:] else body
        pos = [m.start() for m in (re.search(r"= production_shape\(", body), re.search(r"= cpu_baseline\(", body),
                                   re.search(r"= end_to_end\(", body))]
        assert pos == sorted(pos), (start, pos)
