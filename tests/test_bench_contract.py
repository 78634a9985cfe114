"""The default bench line against the driver's contract (the JSON line the round-end BENCH run
parses): every required key, roofline and cpu_baseline objects of the prescribed shape, value ==
bytes hashed / ms_per_step, frac == achieved / peak, the timed build checked against the C oracle.
Runs bench.py as the driver does (no flags but a short timed region), on the GPU. One engine and
one timer over the whole scaling curve: the N = 1 line and a rehearsed N = 8 line (all eight
shards on GPU 0) come from the same group engine with the same field set, and the one-process-per-GPU
engine agrees with it at N = 1."""
import json
import subprocess
import sys

import pytest

from tests.conftest import ROOT


def _line(*args, timeout=600):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


_N1 = {}


def _default_line():
    if "d" not in _N1:
        _N1["d"] = _line("--steps", "5", "--cpu-baseline-seconds", "2", "--no-e2e", "--no-production-shape")
    return _N1["d"]


@pytest.mark.gpu
def test_default_bench_line_keeps_the_contract():
    d = _default_line()
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["warmup"] >= 3 and d["higher_is_better"] is True
    assert d["unit"] == "GiB/s" and d["dtype"] == "u8" and d["vs_baseline"] is None
    assert "workload" in d["config"] and d["config"]["workload"].startswith("C4")
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3 and 0.5 < rf["frac"] < 1.0
    assert rf["traffic"] is None or rf["traffic"] >= rf["algorithmic_bytes_per_launch"]
    assert rf["kernel_ms"] <= d["ms_per_step"] * 1.001
    total = d["config"]["bytes_hashed_per_step"]
    assert abs(d["value"] - total / 2**30 / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-3
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0
    assert d["parity"]["all_ranks_ok"] and d["parity"]["timed_build_equals_c_oracle_on_sample"]


@pytest.mark.gpu
def test_scaling_curve_one_engine_one_timer():
    """The driver's 1 -> 8 ratio divides like by like: the N = 1 line and a rehearsed N = 8 line
    (bench.py --gpus 8 --rehearse: the eight shards of the strong-scaling split on GPU 0, copy
    gather) share the engine, the timer text and the top-level field set; the one-process-per-GPU
    engine (--engine ranks) measures the same N = 1 step within 1 %."""
    d1 = _default_line()
    d8 = _line("--gpus", "8", "--rehearse", "--steps", "5", "--no-gather-per-build")
    assert d1["config"]["engine"] == d8["config"]["engine"] == "group"
    assert d1["timer"] == d8["timer"]
    assert set(d1) == set(d8), set(d1) ^ set(d8)
    assert d8["n_gpus"] == 8 and d8["cpu_baseline"] is None and d8["parity"]["all_ranks_ok"]
    assert d8["config"]["bytes_hashed_per_step"] == d1["config"]["bytes_hashed_per_step"]
    for d in (d1, d8):  # the host CPU the engine burns is on the line (enq_pool spin)
        assert 0 < d["host_timing"]["host_cpu_cores"] and d["host_timing"]["host_cpu_ms_per_step"] > 0
    short = ("--steps", "20", "--no-cpu-baseline", "--no-e2e", "--no-production-shape")
    # each engine's best of two alternating runs, so one noisy run on a shared box does not decide
    runs = [_line("--engine", "ranks", *short), _line(*short), _line("--engine", "ranks", *short), _line(*short)]
    dr = max(runs[0::2], key=lambda d: d["value"])
    dg = max(runs[1::2], key=lambda d: d["value"])
    assert dr["config"]["engine"] == "ranks" and dg["config"]["engine"] == "group"
    assert set(dr) == set(dg), set(dr) ^ set(dg)
    assert abs(dr["value"] - dg["value"]) / dg["value"] < 0.01, ([d["value"] for d in runs])
