"""The default bench line against the driver's contract (the JSON line the round-end BENCH run
parses): every required key, roofline and cpu_baseline objects of the prescribed shape, value ==
bytes hashed / ms_per_step, frac == achieved / peak, the timed build checked against the C oracle.
Runs bench.py as the driver does (no flags but a short timed region), on the GPU."""
import json
import subprocess
import sys

import pytest

from tests.conftest import ROOT


@pytest.mark.gpu
def test_default_bench_line_keeps_the_contract():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "5", "--cpu-baseline-seconds", "2",
                        "--no-e2e", "--no-production-shape"], capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
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
