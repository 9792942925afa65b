"""The one-process-per-rank RCCL transport of libgolhip.so on one GPU.

Real RCCL refuses two ranks on one device, so tests/rccl_shim_check.py runs
the ranks as threads over tests/shim/libfake_rccl.so (an in-process
ncclSend/ncclRecv stand-in, built by __graft_entry__.build()).  What is
exercised is the library's own RCCL-mode code: gol_create_rank, the per-rank
slab, exchange() with ranks ±1 in one group, the boundary/interior overlap and
its events — against the oracle, bit-exactly, for 2-8 ranks.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "tests", "shim", "libfake_rccl.so")


def test_rccl_transport_over_shim():
    assert os.path.exists(SHIM), "build the shim first (__graft_entry__.build())"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_shim_check.py"), SHIM],
                       capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "rccl shim transport ok" in r.stdout


@pytest.mark.timeout(420)
def test_config5_over_shim():
    """BASELINE config 5 (8 × 131072² slabs, RCCL transport) on this GPU."""
    assert os.path.exists(SHIM), "build the shim first (__graft_entry__.build())"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_shim_check.py"), SHIM, "--config5"],
                       capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "rccl shim config5 ok" in r.stdout


@pytest.mark.parametrize("override", [None, 402, 415, "split410"])
def test_schedule_trial_agrees_over_shim(override):
    """RCCL mode: every rank keeps the same k=8 chunk policy after the trial
    (ncclAllReduce MAX of the medians at a fixed k-step), 8 ranks.  override:
    one rank sets its own chunk policy while the trial records — it must still
    join the agreement (before round 5 it left the trial alone and the other
    ranks hung in the allreduce; before the first step 402 it also left at the
    trial's restart) and keep its own policy afterwards.  split410: one rank
    turns the split interior off while the trial records (the option moves its
    default and candidates): same rule."""
    assert os.path.exists(SHIM), "build the shim first (__graft_entry__.build())"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_shim_check.py"), SHIM, "--trial"]
                       + ([] if override is None else ["--override", "410", "--split"] if override == "split410"
                          else ["--override", str(override)]), capture_output=True,
                       text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "rccl shim trial ok" in r.stdout


def test_rank_schedules_have_no_race_over_shim():
    """Each rank's recorded step schedule in RCCL mode (exchange, bands, seam
    bands, interior parts), checked by happens-before (tests/sched_race.py)."""
    assert os.path.exists(SHIM), "build the shim first (__graft_entry__.build())"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_shim_check.py"), SHIM, "--sched"],
                       capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "rccl shim sched ok" in r.stdout


@pytest.mark.timeout(300)
def test_real_rccl_two_ranks_one_gpu():
    """REAL RCCL, two processes on this one GPU: each rank sets its own
    NCCL_HOSTID so RCCL takes them for two hosts (it refuses two ranks on one
    device of one host) and moves the halos over its socket transport.  The
    library's RCCL-mode path runs for real — gol_create_rank on a real
    communicator, ncclSend/ncclRecv halo groups, bands, the split interior,
    the trial's ncclAllReduce agreement — 444 k-steps, bit-exact against the
    oracle, both ranks on the same policy (tests/rccl_real2_check.py)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_real2_check.py")],
                       capture_output=True, text=True, timeout=280)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "real rccl 2-rank ok" in r.stdout


@pytest.mark.timeout(400)
def test_real_rccl_random_cases():
    """Random worlds of 2-4 rank processes on this GPU over real RCCL (socket
    transport): bit / byte layouts, depths 1-32, dead and serial-compat
    boundaries, uneven steps, split 1-3 — each against the oracle."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_real2_check.py"), "--cases", "6",
                        "--seed", "11"], capture_output=True, text=True, timeout=380)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "real rccl cases ok" in r.stdout
