"""bench.py keeps the driver's contract: one JSON line with the metric, the
roofline and (at N=1) the CPU baseline; a small, fast configuration."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("workload", ["bit131072", "byte32768"])
def test_bench_json_line(workload):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--rows", "4096",
                        "--cols", "8192", "--steps", "4", "--warmup", "1", "--no-cpu-baseline", "--no-secondary"],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in d, key
    assert d["unit"] == "GCUPS" and d["value"] > 0 and d["n_gpus"] == 1 and d["steps"] == 4
    rf = d["roofline"]
    assert rf["bound"] in ("hbm", "mfma") and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert 0 < rf["frac"] < 1.5 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert d["config"]["workload"].startswith(workload)
    assert d["live_cells"] > 0
