"""The PMC bookkeeping behind bench.py's `traffic` and VALU roofline
(tools/pmc_summary.py, tools/make_traffic.py) on synthetic rocprofv3 CSVs:
the gfx950 FETCH_SIZE ×2 correction, and under the split interior the
per-step record (counter sums over all dispatches ÷ (dispatches ÷ 3))."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = "void gol::bit_pair_kernel<8, 1, 4, 4>(gol::StencilArgs, gol::Sched, int, int)"


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _fake_profile(base, tag, per_dispatch):
    """per_dispatch: list of (FETCH_SIZE KiB, WRITE_SIZE KiB, SQ_INSTS_VALU) per dispatch."""
    _write(os.path.join(base, f"{tag}_kt", "run_kernel_stats.csv"),
           ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"],
           [[K, len(per_dispatch), 1000.0 * len(per_dispatch), 1000.0, 100.0]])
    for name, idx, counter in (("fetch", 0, "FETCH_SIZE"), ("write", 1, "WRITE_SIZE"), ("sq", 2, "SQ_INSTS_VALU")):
        _write(os.path.join(base, f"{tag}_{name}", "run_counter_collection.csv"),
               ["Kernel_Name", "Counter_Name", "Counter_Value"],
               [[K, counter, d[idx]] for d in per_dispatch])


def _run(base, tag, key, out, *extra):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "make_traffic.py"), base, tag, key,
                        "bit_pair_kernel", "--out", out, *extra], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return json.load(open(out))[key]


def test_per_launch_record(tmp_path):
    _fake_profile(str(tmp_path), "prof_a", [(100.0, 300.0, 1000.0), (120.0, 300.0, 1200.0)])
    rec = _run(str(tmp_path), "prof_a", "k", str(tmp_path / "t.json"))
    assert rec["fetch_kib_raw"] == 110.0 and rec["write_kib"] == 300.0
    assert rec["hbm_bytes_per_launch"] == (2 * 110.0 + 300.0) * 1024   # FETCH_SIZE counts half the reads
    assert rec["valu_insts_per_launch"] == 1100.0 and "dispatches_per_step" not in rec


def test_per_step_record_under_the_split(tmp_path):
    # two steps: (half A, half B, seam band) each
    d = [(100.0, 200.0, 900.0), (100.0, 200.0, 900.0), (4.0, 6.0, 30.0)] * 2
    _fake_profile(str(tmp_path), "prof_b", d)
    rec = _run(str(tmp_path), "prof_b", "k_split", str(tmp_path / "t.json"), "--per-step", "3")
    assert rec["dispatches_per_step"] == 3
    assert rec["fetch_kib_raw"] == 204.0 and rec["write_kib"] == 406.0
    assert rec["hbm_bytes_per_launch"] == (2 * 204.0 + 406.0) * 1024
    assert rec["valu_insts_per_launch"] == 1830.0


def test_split_dispatch_summary(tmp_path):
    """tools/split_dispatches.py on a synthetic trace: two streams of 900-µs
    half-launches, half a period out of phase, plus 60-µs seam bands."""
    rows, t = [], 0
    hdr = ["Kind", "Stream_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X"]
    for i in range(20):
        s = i * 920_000
        rows.append(["KERNEL_DISPATCH", 1, K, s, s + 900_000, 131072])
        rows.append(["KERNEL_DISPATCH", 2, K, s + 460_000, s + 1_360_000, 131072])
        rows.append(["KERNEL_DISPATCH", 3, K, s + 10_000, s + 70_000, 1280])
    _write(os.path.join(tmp_path, "prof_c_kt", "run_kernel_trace.csv"), hdr, rows)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "split_dispatches.py"),
                        str(tmp_path / "prof_c_kt")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["by_grid_size"]["131072"]["calls"] == 40 and d["by_grid_size"]["1280"]["median_us"] == 60.0
    assert d["half_launch_start_to_start_us"]["median"] == 920.0
    assert abs(d["overlap_after_start_us"]["median"] - 440.0) < 25.0
