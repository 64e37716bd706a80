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


# ---- bench.py --gpus N without a launcher ----

def test_resolve_world():
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(8, {}) == (8, True)          # self-launch 8 ranks
    assert bench.resolve_world(None, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)   # the driver's torchrun
    for gpus, env in ((8, {"WORLD_SIZE": "2"}), (1, {"WORLD_SIZE": "2"}), (0, {})):
        try:
            bench.resolve_world(gpus, env)
        except ValueError:
            continue
        raise AssertionError((gpus, env))


def test_launch_plan_argv_and_env():
    env = {"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0", "RC_BENCH_BACKEND": "gloo"}
    argv = ["--gpus", "4", "--steps", "5"]
    plans = bench.launch_plan(4, argv, env, 29999)
    assert len(plans) == 4
    for r, (a, e) in enumerate(plans):
        assert a[0] == sys.executable and a[-4:] == argv
        assert os.path.samefile(a[a.index("-u") + 1], os.path.join(ROOT, "bench.py"))
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"]) == (str(r), str(r), "4")
        assert (e["MASTER_ADDR"], e["MASTER_PORT"]) == ("127.0.0.1", "29999")
        # the caller's environment travels (IPC mode, rehearsal backend)
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["RC_BENCH_BACKEND"] == "gloo"
    assert "RANK" not in env   # the parent's own environment is untouched


def test_worst_status():
    assert bench.worst_status([0, 0, 0]) == 0
    assert bench.worst_status([0, 3, 0]) == 3
    assert bench.worst_status([4, 3]) == 4
    assert bench.worst_status([0, -9]) == 137   # killed by SIGKILL
    assert bench.worst_status([]) == 0


def _py(code):
    return [sys.executable, "-c", code]


def test_run_ranks_relays_codes_and_kills_stuck_ranks():
    env = dict(os.environ)
    assert bench.run_ranks([(_py("pass"), env), (_py("import sys; sys.exit(0)"), env)]) == [0, 0]
    # one rank fails, the other is stuck (as in a collective with the dead rank): killed after
    # the grace period by its own PID
    import time
    t0 = time.monotonic()
    codes = bench.run_ranks([(_py("import sys; sys.exit(4)"), env),
                             (_py("import time; time.sleep(600)"), env)], grace_s=1.0)
    assert codes[0] == 4 and codes[1] == -9, codes
    assert time.monotonic() - t0 < 30
    assert bench.worst_status(codes) == 137


def test_self_launch_end_to_end_without_gpu():
    """`bench.py --gpus 2` with no launcher starts two ranks; here (no GPU) each rank stops
    with its own message before any GPU call and the parent exits with their status."""
    import torch
    if torch.cuda.device_count() > 0:   # counting devices does not initialise HIP
        import pytest
        pytest.skip("needs a box without GPUs (the ranks would start rendering)")
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "RC_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "rank 0 needs GPU 0" in r.stderr and "rank 1 needs GPU 1" in r.stderr, r.stderr
    assert "rank exit codes [2, 2]" in r.stderr


def test_gpus_must_match_the_launcher():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 2 and "--gpus 8 but the launcher started WORLD_SIZE=2" in r.stderr


def test_counter_files_exist_and_are_current():
    """every counter summary bench.py reads exists, is this round's (one
    scripts/pmc_all.sh call at HEAD) and covers the line's dominant kernel."""
    import json
    maps = list(bench.PMC_PROFILES.items()) + list(bench.PMC_HEADLINE.items())
    assert maps
    for (scene, size, depth, mode), rel in maps:
        assert os.path.basename(rel).startswith("r06s_"), rel
        with open(os.path.join(ROOT, rel)) as f:
            ks = {k.split("::")[-1].split("<")[0] for k in json.load(f)["kernels"]}
        want = "k_render" if mode == "fast" else "k_resolve"
        assert want in ks, (rel, ks)
    pmc, src = bench.pmc_kernel("k_resolve", "quadric", 4096, 6, "parity", inflight=True)
    assert src == bench.PMC_HEADLINE[("quadric", 4096, 6, "parity")] and pmc["hbm_bytes"] > 0
