"""bench.py host logic on CPU: the sharded leg's watchdog exits non-zero on a stuck exchange
(VERDICT r2 item 2), the CPU-baseline core choice and clock probe, the golden lookup."""
import os
import subprocess
import sys

from helpers import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_watchdog_exits_nonzero_on_a_stuck_leg():
    """A leg that never returns (a group whose render blocks forever): the watchdog runs the
    timeout callback (rank 0 prints the line) and the process exits with LEG_TIMEOUT_EXIT."""
    code = ("import sys, threading; sys.path.insert(0, %r); import bench\n"
            "class StuckGroup:\n"
            "    def render(self, *a, **k):\n"
            "        threading.Event().wait()\n"
            "g = StuckGroup()\n"
            "bench.run_leg_with_watchdog(lambda: g.render(), 0.5,\n"
            "                            lambda: print('{\"leg\": \"timed out\"}', flush=True))\n"
            "print('not reached', flush=True)\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == bench.LEG_TIMEOUT_EXIT != 0, (r.returncode, r.stderr)
    assert '{"leg": "timed out"}' in r.stdout
    assert "not reached" not in r.stdout


def test_watchdog_reports_a_failing_leg():
    """A leg that raises (an RCCL error in the sharded exchange) comes back as an error
    record, so rank 0 can still print the line; the watchdog does not fire afterwards."""
    calls = []

    def leg():
        raise RuntimeError("rc_render_sharded failed")
    r = bench.run_leg_with_watchdog(leg, 0.2, lambda: calls.append(1))
    assert r == {"error": "RuntimeError: rc_render_sharded failed"}
    import time
    time.sleep(0.4)
    assert not calls


def test_watchdog_returns_the_leg_result():
    calls = []
    assert bench.run_leg_with_watchdog(lambda: 42, 30, lambda: calls.append(1)) == 42
    assert not calls


def test_quiet_core_and_clock():
    cands = sorted(os.sched_getaffinity(0))
    c = bench.quiet_core(cands, window_s=0.05)
    assert c in cands
    mhz = bench.core_mhz(c)
    assert mhz is None or mhz > 0


def test_golden_lookup():
    assert bench.golden_md5("quadric", 4096, 4096, 6, "parity") == "3bf1c59fc7cf7e508e5b1796348e9726"
    assert bench.golden_md5("quadric", 4096, 4096, 6, "fast") == "7b6a08a014498b1c3b81df44fce9b776"
    assert bench.golden_md5("quadric", 123, 4096, 6, "parity") is None
