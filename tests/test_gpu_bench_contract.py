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


@pytest.mark.timeout(300)
def test_bench_config4_valu_roofline():
    """The roofline branch the driver's line takes: config 4's
    shape (bit 131072², the default k = 16: the chain of two pair waves per
    strip), a few steps.  The kernel is issue-bound, so the line must say bound
    "valu", with roofline.frac = traffic.json's SQ_INSTS_VALU per step × 64
    lanes ÷ the live step time ÷ the lane-op peak, and the HBM object = 0.25
    B/cell × 131072² per step ÷ the same time ÷ 8 TB/s.  Under the split
    interior (the default) the unit is the step (two half-launches + the seam
    band) and the record is traffic.json's per-step bit131072_k16_split."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
                        "--no-cpu-baseline", "--no-secondary", "--no-aged", "--no-config4", "--settle-s", "0.2"],
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["config"]["rows"] == d["config"]["cols"] == 131072 and d["config"]["gens_per_step"] == 16
    assert d["verified"] is True
    rf = d["roofline"]
    assert rf["bound"] == "valu" and rf["unit"] == "Tlane-op/s"
    assert rf["interior_split"] is True and d["config"]["interior_split"] == 2
    with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
        tr = json.load(f)["bit131072_k16_split"]
    assert tr["dispatches_per_step"] == 3
    t = rf["kernel_avg_ms"] * 1e-3
    assert t > 0 and rf["launches"] == 2 * 4
    assert abs(t - d["device_ms"] * 1e-3 / 4) < 1e-12
    peak = 256 * 4 * 32 * 2.4e9
    want = tr["valu_insts_per_launch"] * 64 / t / peak
    assert abs(rf["frac"] - want) < 1e-9 * max(1.0, want), (rf["frac"], want)
    assert abs(rf["peak"] - peak / 1e12) < 1e-9 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    hbm_want = 0.25 * 131072 * 131072 / t / 8.0e12
    assert rf["hbm"]["bytes_per_launch"] == 0.25 * 131072 * 131072
    assert abs(rf["hbm"]["frac"] - hbm_want) < 1e-9, (rf["hbm"]["frac"], hbm_want)
    assert abs(rf["traffic"] - tr["hbm_bytes_per_launch"]) < 1.0
    assert 0.2 < rf["frac"] < 1.0 and 0.2 < rf["hbm"]["frac"] < 1.0


@pytest.mark.timeout(300)
def test_bench_single_process_eight_slabs():
    """Config 5 rehearsed in one process (8 row slabs of 131072² on this GPU,
    peer copies for the halos): the line is verified across the first slab
    seam, and the clock settles on the headline board itself — a twin
    context's 16 more streams would exceed the 24 hardware queues and share
    queues with the headline's (92-107 k instead of 141-145 k)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--single-process", "--gpus", "8", "--steps",
                        "3", "--warmup", "1", "--no-cpu-baseline", "--no-secondary", "--settle-s", "0.2"],
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert d["config"]["rows"] == 8 * 131072 and d["config"]["cols"] == 131072
    assert d["verified"] is True and "hardware queues" in d["board"]
    assert d["value"] > 0 and d["n_gpus"] == 8


@pytest.mark.timeout(400)
def test_bench_two_ranks_real_rccl_same_device():
    """The driver's N>1 path (bench.py --gpus 2: spawned ranks, gloo side
    channel, max-over-ranks timing, per-rank and seam light-cone windows) with
    REAL RCCL halos, both ranks on this GPU (--same-device: one NCCL_HOSTID
    per rank, RCCL's socket transport).  The rate is no scaling number; the
    line must be verified across the seam."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device", "--steps", "4",
                        "--warmup", "2", "--no-cpu-baseline", "--no-secondary", "--settle-s", "0.2"],
                       capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert d["n_gpus"] == 2 and d["config"]["rows"] == 2 * 131072 and "same-device" in d["config"]["parallelism"]
    seams = [v for v in d["verify"] if v.get("seam")]
    assert d["verified"] is True and len(seams) == 1 and seams[0]["seam"] == 131072
    # the halo diagnostic (after verification): per-rank comm-stream time, the
    # no-exchange step, and the efficiency they explain
    h = d["halo"]
    assert len(h["per_rank"]) == 2 and all(r["steps_timed"] == 2 * (4 + 2) for r in h["per_rank"])
    assert h["exchange_ms_per_step"] > 0 and h["bands_ms_per_step"] > 0
    assert abs(h["exposed_ms_per_step"] - (h["step_ms"] - h["step_ms_no_halo"])) < 1e-9
    assert 0 < h["efficiency_vs_no_halo"] and abs(h["efficiency_vs_no_halo"] * h["step_ms"] - h["step_ms_no_halo"]) < 1e-9
