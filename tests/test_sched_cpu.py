"""The runtime's stream schedules race-checked on the CPU: libgolhip's host
code built over a host-only HIP stand-in (tests/fake_hip, built by
__graft_entry__.build()) records its real step schedule — slabs 1-4, the
interior split 1-4 (toggled mid-run), overlap on/off, bit and byte layouts,
uneven depths, async window copies — and tests/sched_race.py finds any two
conflicting accesses left unordered.  Removing the fix of either round-5 race
makes this fail."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "fake_hip", "libgolhip_fakehip.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="build the host-only runtime first (__graft_entry__.build())")
def test_random_schedules_have_no_race_cpu():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sched_cpu_check.py"), "2000", "5"],
                       env=dict(os.environ, GOL_LIB=LIB), capture_output=True, text=True, timeout=600)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sched cpu ok" in r.stdout


@pytest.mark.skipif(not os.path.exists(LIB), reason="build the host-only runtime first (__graft_entry__.build())")
def test_rank_schedules_have_no_race_cpu():
    """RCCL mode (ranks as threads over the in-process RCCL stand-in, both
    built for the host): every rank's schedule — the exchange's sends and
    receives, bands, seam bands, parts, async windows — race-free."""
    shim = os.path.join(ROOT, "tests", "fake_hip", "libfake_rccl_host.so")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sched_cpu_check.py"), "150", "7"],
                       env=dict(os.environ, GOL_LIB=LIB, GOL_RCCL_SHIM=shim), capture_output=True, text=True,
                       timeout=600)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sched cpu rccl ok" in r.stdout


@pytest.mark.skipif(not os.path.exists(LIB), reason="build the host-only runtime first (__graft_entry__.build())")
def test_trial_agreement_state_machine_cpu():
    """The k = 8 trial's RCCL-mode agreement on the CPU (8 ranks as threads over
    the stand-ins): no rank left out of the ncclAllReduce — also when one rank
    sets GOL_OPT_CHUNK_ROWS before / after the trial's restart, turns the split
    off, or turns the trial off mid-trial — and all others keep one policy."""
    shim = os.path.join(ROOT, "tests", "fake_hip", "libfake_rccl_host.so")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "sched_cpu_check.py"), "--trial"],
                       env=dict(os.environ, GOL_LIB=LIB, GOL_RCCL_SHIM=shim), capture_output=True, text=True,
                       timeout=600)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sched cpu trial ok" in r.stdout


ASAN = os.path.join(ROOT, "tests", "fake_hip", "host_asan_driver")


@pytest.mark.skipif(not os.path.exists(ASAN), reason="build the host-only runtime first (__graft_entry__.build())")
def test_host_code_under_address_and_ub_sanitizers():
    """The runtime's host code under -fsanitize=address,undefined (over the
    host-only HIP stand-in, an executable of its own: no preloading): 300
    random contexts of 1-4 slabs, split toggled, uneven steps, async windows,
    the schedule trace, text, popcount, destroy — no report."""
    r = subprocess.run([ASAN, "300"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "300 contexts ok" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr


TSAN = os.path.join(ROOT, "tests", "fake_hip", "host_tsan_driver")


@pytest.mark.skipif(not os.path.exists(TSAN), reason="build the host-only runtime first (__graft_entry__.build())")
def test_rank_threads_under_thread_sanitizer():
    """Rank contexts of 2-4-rank RCCL worlds created, stepped and destroyed from
    threads at once (host stand-ins for HIP and RCCL) under ThreadSanitizer:
    no data race in the runtime's process-wide state."""
    r = subprocess.run([TSAN], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "tsan driver ok" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr
