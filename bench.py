#!/usr/bin/env python3
"""Benchmark: primary rays/s (= pixels/s) rendering quadric.scene at 4096x4096, bounce depth 6
(MAX_RECURSION 7, C/raycast.c:14) — BASELINE.json's metric.

A "step" is one full render of the image through the C-ABI: scene already resident in HBM,
every frame written to its own device buffer, every kernel of the mode inside the timed
region.  Parity mode (default, byte-identical to the reference): phase A + scan-order
compaction + carry-chain resolver + phase C, with two frames in flight (rc_frame_submit:
the carry resolvers of consecutive frames run side by side on one CU partition while the
pixel phases run on the other; DESIGN.md §frames in flight) — `value` is K frames' pixels
over the time to finish all K.  `single_frame` reports one frame at a time
(rc_render_device, the raycast() path; --inflight 1 makes that the measured step).
Fast mode: one render kernel per frame; cuda mode (the CUDA port's semantics) likewise.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode parity|fast] [--inflight 1|2]

Multi-GPU (torchrun, one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE from the env): every rank
joins an rc_group (the library's own RCCL communicator; rank 0's ncclUniqueId shared over
torch.distributed).
  fast:   one image row-sharded (row y -> rank y % N), rendered by rc_render_sharded: each
          rank its rows, ncclGather of the row blocks to rank 0, de-interleaved on its device
          ("strong").
  parity: the carry chain's resolver is serial, so the headline is N replicas,
          one image per GPU, no data-path collective ("weak"); the row-sharded single image
          (rank 0 receives the other ranks' DEP entries and row blocks, resolves the chain and
          shades every DEP entry; nothing returns) is timed after the timed region and
          reported as `sharded_single_image` (--shard makes it the step).

What `value` includes is stated in the line itself (`config.timed_region`); `rates` puts the
three rates side by side: frames in flight on the device (`value`), one frame at a time on the
device (`single_frame`), and the drop-in raycast() call end to end — scene upload, kernels and
the copy into the caller's fresh pageable pixmap (`end_to_end`, SURVEY.md §8d's rate).

Rank 0 prints one JSON line with `roofline` (the dominant kernel, timed live with HIP events
on its stream through rc_profile_begin/end), per-phase times and `cpu_baseline` (the reference
C/ build from oracle/_ref on one host core; N=1 only).
"""
import argparse
import importlib.util
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

# Algorithmic work: SURVEY.md §8d's per-operation weights (sphere test
# 29, plane 15, quadric 81, hit post-processing 26 per non-shadow nearest, light setup 18 per
# shadow ray, unshadowed light 70, reflect+normalize 21 per bounce, ray generation 15) applied
# to the reference's exact per-pixel work counts at each config (CPU oracle counters over the
# whole image, tests/helpers.oracle_render stats).  A carry transfer function (one DEP entry
# of the resolver) = (depth - 1) bounce levels x (every shape's test + reflect/normalize) +
# hit post-processing for its hits (quadric: 5 x (287 + 21) + 3 x 26 = 1618, the creep
# pattern hit/miss/hit/miss/hit; reflection d4: 3 x (421 + 21) + 2 x 26 = 1378).
WORK = {
    "simple:1024:0": {"render_flop_per_px": 260.1},                 # C2 (no bounce: no DEP)
    "simple:256:6": {"render_flop_per_px": 406.4, "dep_flop_per_entry": 5 * (102 + 21) + 3 * 26},
    "reflection:2048:4": {"render_flop_per_px": 930.6, "dep_flop_per_entry": 1378.0},   # C3
    "quadric:4096:6": {"render_flop_per_px": 1373.9, "dep_flop_per_entry": 1618.0},     # C4
    "quadric:8192:6": {"render_flop_per_px": 1381.7, "dep_flop_per_entry": 1618.0},     # C5
}
PEAK_FP64_TFLOPS = 78.6    # MI355X vector FP64 (MI355X_MICROARCH.md: FP32 157.3 / 2)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E
GOLDEN_MD5 = os.path.join(ROOT, "tests", "golden", "md5.json")   # the reference's own outputs
LEG_TIMEOUT_EXIT = 3       # exit status when the sharded leg's watchdog fires


def load_pkg():
    name = "raytracing_programs_amd"
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


# rocprofv3 --pmc summaries of this exact configuration at HEAD, all from one call of
# scripts/pmc_all.sh (kernel stats, VALU/wave-state and FETCH/WRITE passes per configuration ->
# scripts/pmc_summary.py): per-kernel counter means per launch.  Lone frames for parity (the
# one-frame-at-a-time schedule, phase C inside the resolver), the timed launches for fast mode.
PMC_PROFILES = {("quadric", 4096, 6, "parity"): "profiles/r06s_pmc_c4.json",
                ("reflection", 2048, 4, "parity"): "profiles/r06s_pmc_c3.json",
                ("quadric", 8192, 6, "parity"): "profiles/r06s_pmc_c5.json",
                ("quadric", 4096, 6, "fast"): "profiles/r06s_pmc_fast.json"}

# The headline's whole counter set from the same call, on the driver's command itself
# (`bench.py --timed-only --steps 20 --warmup 5`, frames in flight): valu_busy and traffic of
# the headline line's dominant kernel come from the launches it times.
PMC_HEADLINE = {("quadric", 4096, 6, "parity"): "profiles/r06s_pmc_headline.json"}


def pmc_kernel(kernel, scene, size, depth, mode, inflight=False):
    """Counter means of `kernel` from the committed PMC summary of this configuration:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch (the gfx950 correction of
    MI355X_MICROARCH.md), write_bytes = WRITE_SIZE * 1024, valu_busy; (None, None) when no
    profile covers it.  inflight: every figure from the frames-in-flight summary of the
    driver's command when one exists (PMC_HEADLINE)."""
    def find(rel):
        if not rel or not os.path.exists(os.path.join(ROOT, rel)):
            return None
        with open(os.path.join(ROOT, rel)) as f:
            prof = json.load(f)
        for name, d in prof["kernels"].items():
            if name.split("::")[-1].split("<")[0] == kernel:
                return d
        return None
    rel = PMC_PROFILES.get((scene, size, depth, mode))
    d = find(rel)
    if d is None:
        return None, None
    out = {"hbm_bytes": d.get("hbm_bytes"),
           "write_bytes": d["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in d else None,
           "valu_busy": d.get("valu_busy")}
    if inflight:
        hrel = PMC_HEADLINE.get((scene, size, depth, mode))
        h = find(hrel)
        if h is not None:   # one run: valu_busy and traffic of the frames-in-flight launches
            return {"hbm_bytes": h.get("hbm_bytes"),
                    "write_bytes": h["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in h else None,
                    "valu_busy": h.get("valu_busy"),
                    "frac_wait_any": h.get("frac_wait_any")}, hrel
    return out, rel


def end_to_end(pkg, scene, W, H, depth, mode, reps=5):
    """The drop-in path's rate: rc_render() into a host pixmap — scene
    upload, every kernel and the device-to-host copy into pageable memory, as raycast()
    runs it.  Like the reference's main (C/raycast.c:52-57: malloc, then raycast()), every
    rep gets a fresh, never-touched pixmap allocated before the timer starts, so faulting its
    pages in is timed.  Reported beside `value` (device-resident), never as it."""
    import numpy as np
    pkg.render(scene, W, H, depth=depth, mode=mode)   # warm: host buffers, scene upload
    ts, lib = [], []
    for _ in range(reps):
        out = np.empty((H, W, 3), dtype=np.uint8)
        tim = {}
        t0 = time.perf_counter()
        pkg.render(scene, W, H, depth=depth, mode=mode, timing=tim, out=out)
        ts.append(time.perf_counter() - t0)
        lib.append(tim["total_ms"])
        del out
    ts.sort()
    lib.sort()
    med = ts[len(ts) // 2]
    return {"value": round(W * H / med, 1), "unit": "rays/s", "ms": round(med * 1e3, 3),
            "lib_total_ms": round(lib[len(lib) // 2], 3),
            "note": "rc_render into a fresh pageable host pixmap (upload + kernels + D2H, the "
                    f"copy overlapped with the resolver), median of {reps}; lib_total_ms = "
                    "rc_render's own clock"}


def golden_md5(scene, W, H, depth, mode):
    """md5 of the reference's P3 output for this configuration (tests/golden/md5.json, made by
    the reference build itself), or None when the table has no such image."""
    try:
        with open(GOLDEN_MD5) as f:
            e = json.load(f).get(f"{scene}:{W}x{H}:d{depth}:{mode}")
    except OSError:
        return None
    return e["md5"] if e else None


def verify_frames(pkg, bufs, want_md5):
    """Outside the timed region: every timed frame's bytes against frame 0's (torch.equal on
    the device) and frame 0's P3 md5 against the reference's golden.  Returns (frames whose
    bytes equal frame 0's, frame 0's md5, golden match or None without a golden)."""
    import torch
    ref = bufs[0]
    equal = sum(1 for b in bufs if torch.equal(b, ref))
    md5 = pkg.p3_md5(ref.cpu().numpy())
    return equal, md5, (None if want_md5 is None else md5 == want_md5)


def run_leg_with_watchdog(leg, timeout_s, on_timeout):
    """Run leg() under a watchdog: if it has not returned after timeout_s (a stuck
    multi-process exchange), on_timeout() runs (rank 0 prints the line with the leg marked as
    timed out, so the timed result is not lost) and the process exits with LEG_TIMEOUT_EXIT —
    never 0, so the driver sees the hang.  A leg that raises returns {"error": ...} instead
    (the caller prints the line with it, then exits with LEG_TIMEOUT_EXIT as well)."""
    done = threading.Event()

    def watch():
        if done.wait(timeout_s):
            return
        try:
            on_timeout()
        finally:
            sys.stdout.flush()
            os._exit(LEG_TIMEOUT_EXIT)

    threading.Thread(target=watch, daemon=True).start()
    try:
        return leg()
    except Exception as e:  # noqa: BLE001 — reported in the line; the timed value stands
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        done.set()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _cpu_jiffies():
    """{cpu: (busy, total)} from /proc/stat."""
    out = {}
    with open("/proc/stat") as f:
        for line in f:
            if line.startswith("cpu") and line[3:4].isdigit():
                name, *v = line.split()
                v = [int(x) for x in v]
                idle = v[3] + (v[4] if len(v) > 4 else 0)
                out[int(name[3:])] = (sum(v) - idle, sum(v))
    return out


def _siblings(c):
    """The hardware threads sharing core c (SMT siblings), c included."""
    try:
        with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
            out = set()
            for part in f.read().strip().split(","):
                lo, _, hi = part.partition("-")
                out.update(range(int(lo), int(hi or lo) + 1))
            return out
    except (OSError, ValueError):
        return {c}


def quiet_core(cands, window_s=0.5):
    """The least busy core of `cands` over a short window, judged with its SMT siblings (a
    busy sibling shares the core's pipelines and caches); ties: the highest id, away from
    core 0's interrupts and housekeeping."""
    try:
        a = _cpu_jiffies()
        time.sleep(window_s)
        b = _cpu_jiffies()
    except OSError:
        return max(cands)

    def busy(c):
        if c not in a or c not in b:
            return 1.0
        dt = b[c][1] - a[c][1]
        return (b[c][0] - a[c][0]) / dt if dt > 0 else 0.0
    return min(cands, key=lambda c: (round(max(busy(x) for x in _siblings(c)), 2), -c))


def core_mhz(core):
    """Current clock of `core` (cpufreq, else /proc/cpuinfo), MHz, or None."""
    try:
        with open(f"/sys/devices/system/cpu/cpu{core}/cpufreq/scaling_cur_freq") as f:
            return round(int(f.read()) / 1000.0, 1)
    except (OSError, ValueError):
        pass
    try:
        cur = None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("processor"):
                    cur = int(line.split(":")[1])
                elif line.startswith("cpu MHz") and cur == core:
                    return round(float(line.split(":")[1]), 1)
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(scene_path, size, depth):
    """The reference itself (oracle/_ref/ref_timer_d<depth>: the C/ sources built like
    C/Makefile:4, raycast() timed alone) on one pinned host core, 3 runs; falls
    back to the CPU restatement (oracle/build) when the reference build is absent.  The core is
    the least busy of the affinity set (not core 0: interrupts and housekeeping), its clock is
    recorded before and after every run, and min and median are reported.  Above 4096^2 the
    sample is the same scene at 4096^2 (rays/s is per pixel; a full 8192^2 run takes ~40 s),
    so the leg stays at ~15-30 s."""
    n = min(size, 4096)
    ref = os.path.join(ROOT, "oracle", "_ref", f"ref_timer_d{depth}")
    if os.path.exists(ref):
        cmd, kind = [ref, str(n), str(n), scene_path], "reference"
    else:
        cmd = [os.path.join(ROOT, "oracle", "build", "oracle_raytrace"), str(n), str(n),
               scene_path, "/dev/null", str(depth)]
        kind = "port"
    runs = 3
    info = {"cpu_model": cpu_model(), "nproc": os.cpu_count()}
    try:
        core = None
        try:
            core = quiet_core(sorted(os.sched_getaffinity(0)))
            cmd = ["taskset", "-c", str(core)] + cmd
        except (AttributeError, OSError):
            pass
        res, mhz = [], []
        for _ in range(runs):
            before = core_mhz(core) if core is not None else None
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                                 check=True).stdout
            mhz.append([before, core_mhz(core) if core is not None else None])
            res.append(json.loads([l for l in out.splitlines() if l.startswith("{")][-1]))
        secs = sorted(r["seconds"] for r in res)
        med = secs[len(secs) // 2]
        # value from the fastest run: on a shared host the slower runs measure other tenants
        # (the same core at the same clock varied 4.6-5.9 s within one bench run)
        return {"value": round(n * n / secs[0], 1), "unit": "rays/s", "cores": 1, "kind": kind,
                "sample": f"full {n}x{n} {os.path.basename(scene_path)} depth {depth} render, "
                          f"raycast() only, 1 pinned core (cpu {core}), {runs} runs: min "
                          f"{secs[0]:.2f} s (value), median {med:.2f} s",
                "seconds": [round(x, 3) for x in secs],
                "value_median_time": round(n * n / med, 1),
                "core": core, "mhz_before_after": mhz, **info}
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "rays/s", "cores": 1, "kind": kind,
                "sample": f"failed: {e}", **info}


def make_group(pkg, dist, world, rank, local):
    """This rank's rc_group (one process per GPU): rank 0 makes the RCCL unique id, the job
    shares it over torch.distributed, every rank joins (ncclCommInitRank inside the library)."""
    import torch
    uid = torch.zeros(pkg.GROUP_ID_BYTES, dtype=torch.uint8, device="cuda")
    if rank == 0:
        uid.copy_(torch.frombuffer(bytearray(pkg.Group.unique_id()), dtype=torch.uint8))
    dist.broadcast(uid, 0)
    return pkg.Group.rank(world, rank, bytes(uid.cpu().tolist()), local)


def resolver_diag(d):
    """The bench line's resolver record (rc_resolver_stats_get), outside the timed region: a
    slow frame's mechanism shows here — per-frame resolver span spread, the resolver's placement
    against what a CU can hold (a register or LDS overrun halves the workgroups per CU), the
    team's rounds, and the longest bounded wait per hand-off site."""
    r = lambda v: round(v, 4)
    return {"frames": d["frames"],
            "resolve_ms": {"min": r(d["resolve_ms_min"]), "max": r(d["resolve_ms_max"]),
                           "mean": r(d["resolve_ms_mean"])} if d["resolve_ms_mean"] else None,
            "placement": {"workgroups": d["grid"], "cus": d["res_cus"],
                          "workgroups_per_cu": d["wg_per_cu"],
                          "workgroups_per_cu_max": d["wg_per_cu_max"],
                          "regs_per_lane": d["regs"], "scratch_bytes": d["scratch_bytes"],
                          "lds_bytes": d["lds_bytes"], "team_blocks": d["team_blocks"]},
            "team_rounds_max": {"scan": d["scan_rounds_max"], "coop_scan": d["cscan_rounds_max"],
                                "resolve": d["resolve_rounds_max"]},
            "spin_wait_us_max": d["spin_wait_us_max"],
            "clock_mhz": {"min": d["clock_mhz_min"], "max": d["clock_mhz_max"]}}


def free_port():
    """A TCP port free on 127.0.0.1 right now (the rendezvous of self-launched ranks)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(n, argv, env, port):
    """One (argv, env) per rank for `bench.py --gpus n` started without a launcher: the same
    script and arguments in a fresh interpreter, with the variables torchrun would set
    (RANK = LOCAL_RANK = r, WORLD_SIZE = n, rendezvous on 127.0.0.1:port).  The children are
    started before this process makes any HIP call, and never by an exec of it."""
    plans = []
    for r in range(n):
        e = dict(env)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plans.append(([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), e))
    return plans


def worst_status(codes):
    """The job's exit status from its ranks': 0 when every rank exited 0, else the largest
    failure, a rank killed by signal s counting as 128 + s (the shell's convention)."""
    norm = [(128 - c if c < 0 else c) for c in codes]
    return max(norm) if norm else 0


def run_ranks(plans, grace_s=60.0, poll_s=0.2):
    """Start every rank, wait for all of them and return their exit codes.  Rank 0's JSON line
    reaches the caller through the inherited stdout.  Once a rank has failed, the others get
    grace_s to finish (they may be blocked in a collective with the dead rank) and are then
    killed by their own PIDs."""
    procs = [subprocess.Popen(a, env=e) for a, e in plans]
    deadline = None
    try:
        while any(p.poll() is None for p in procs):
            if deadline is None and any(p.returncode not in (None, 0) for p in procs):
                deadline = time.monotonic() + grace_s
            if deadline is not None and time.monotonic() > deadline:
                for p in procs:
                    if p.poll() is None:
                        print(f"bench.py: rank pid {p.pid} still running {grace_s:.0f} s after "
                              "another rank failed; killing it", file=sys.stderr, flush=True)
                        p.kill()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    return [p.returncode for p in procs]


def resolve_world(gpus, env):
    """(world size, launch children?) for `--gpus` (None = not given) under this environment.
    Under a launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE; without one, --gpus N > 1
    means this process launches the N ranks itself.  Raises ValueError on a mismatch."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        ws = int(ws)
        if gpus is not None and gpus != ws:
            raise ValueError(f"--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks")
        return ws, False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise ValueError(f"--gpus {n}: need at least one GPU")
    return n, n > 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each); default 1, or WORLD_SIZE under a launcher.  "
                         "Without a launcher, N > 1 starts the N ranks as child processes")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="parity", choices=["parity", "fast", "cuda"],
                    help="cuda: the CUDA port's semantics (RC_MODE_CUDA, SURVEY §8 f4; pass "
                         "--depth 50 for its MAX_ITER)")
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--scene", default="quadric")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--timed-only", action="store_true",
                    help="launch nothing but the warmup and timed steps (no single-frame, "
                         "end-to-end or CPU legs): the command profiled under rocprofv3, so its "
                         "per-kernel averages are those of the timed launches")
    ap.add_argument("--inflight", type=int, default=2, choices=[1, 2],
                    help="parity frames in flight: 2 = rc_frame_submit (the next frame's pixel "
                         "phases beside this frame's resolver), 1 = one rc_render_device per step")
    ap.add_argument("--tune", action="append", default=[], metavar="FIELD=VALUE",
                    help="schedule experiment: rc_set_tuning field (repeatable; see "
                         "include/raycast_hip.h rc_tuning); the default is the product schedule")
    ap.add_argument("--force-group", action="store_true",
                    help="test aid: take the N>1 code paths (torch.distributed + rc_group over "
                         "RCCL, sharded step / leg) even with one rank")
    ap.add_argument("--shard", action="store_true",
                    help="N>1 parity: time the row-sharded single image (rc_render_sharded) as "
                         "the step instead of N replicas")
    args = ap.parse_args()

    try:
        world, spawn = resolve_world(args.gpus, os.environ)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    if spawn:   # no launcher: this process only starts the ranks (no torch, no HIP call here)
        codes = run_ranks(launch_plan(world, sys.argv[1:], os.environ, free_port()))
        if any(codes):
            print(f"bench.py: rank exit codes {codes}", file=sys.stderr, flush=True)
        sys.exit(worst_status(codes))

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("RC_BENCH_BACKEND", "nccl")   # gloo: 1-GPU rehearsal only
    ndev = torch.cuda.device_count()
    if backend != "nccl":   # rehearsal: ranks share the GPUs, so no RCCL group (replicas only)
        local %= max(1, ndev)
    elif local >= ndev:
        print(f"bench.py: rank {rank} needs GPU {local} but {ndev} are visible (one rank per "
              "GPU; RC_BENCH_BACKEND=gloo shares them for a rehearsal)", file=sys.stderr,
              flush=True)
        sys.exit(2)
    torch.cuda.set_device(local)
    # host-side collectives (timing max, verification counts): on the device over RCCL, on the
    # host over gloo
    cdev = "cuda" if backend == "nccl" else "cpu"
    multi = world > 1 or args.force_group
    if multi:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    pkg = load_pkg()
    if args.tune:
        pkg.set_tuning(**{k: int(v) for k, v in (t.split("=", 1) for t in args.tune)})
    scene_path = os.path.join(ROOT, "tests", "golden", "scenes", args.scene + ".scene")
    scene = pkg.Scene.from_file(scene_path)
    W = H = args.size
    mode = args.mode
    parity = mode == "parity" and args.depth > 0
    def join_group():
        g, err = None, None
        try:
            g = make_group(pkg, dist, world, rank, local)
        except Exception as e:  # noqa: BLE001 — reported in the line; replicas still run
            err = f"{type(e).__name__}: {e}"
        ok = torch.tensor([0 if g is None else 1], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0 and g is not None:   # every rank or none uses the group
            g.close()
            g, err = None, err or "another rank failed to join the rc_group"
        return g, err

    # the library's RCCL group before the timed steps only when the step needs it (fast mode's
    # row shards, --shard); parity replicas join it after them, inside the watchdog-bounded
    # sharded leg, so a communicator that never forms cannot cost the headline
    group, group_err = None, None
    if multi and backend == "nccl" and (mode in ("fast", "cuda") or args.shard):
        group, group_err = join_group()
    # the step: fast mode over N GPUs = one image row-sharded (strong); parity over N GPUs =
    # N replicas, one image per GPU (weak: the carry resolver is serial), or the
    # sharded single image with --shard
    sharded = group is not None and (mode in ("fast", "cuda") or args.shard)
    out = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    want_md5 = golden_md5(args.scene, W, H, args.depth, mode) if mode != "cuda" else None

    piped = parity and args.inflight == 2 and not sharded
    # every frame of the timed region gets its own output image, so that all of them can be
    # byte-checked afterwards (the sharded step's image is the root's)
    outs = None
    if not sharded:
        outs = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
                for _ in range(max(args.steps, 1))]
        torch.cuda.synchronize()
    frame_no = [0]

    def step():
        if sharded:   # synchronous: the root holds the de-interleaved image when it returns
            group.render(scene, W, H, out.data_ptr(), depth=args.depth, mode=mode)
            return
        buf = outs[frame_no[0] % len(outs)]
        frame_no[0] += 1
        if piped:
            pkg.frame_submit(scene, W, H, buf.data_ptr(), depth=args.depth, mode=mode)
        else:
            pkg.render_device(scene, W, H, buf.data_ptr(), stream.cuda_stream, depth=args.depth,
                              mode=mode)

    def drain():
        if piped:
            pkg.frames_wait(pipe_tim)
        torch.cuda.synchronize()

    pipe_tim = {}
    single = None
    side0 = None
    if piped and not args.timed_only:
        # latency and per-phase times of a lone frame (rc_render_device, the raycast() path),
        # taken before the frame pipeline's CU-partitioned streams exist
        for _ in range(2):
            pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream,
                              depth=args.depth, mode=mode)
        torch.cuda.synchronize()
        pkg.profile_begin()
        ts = time.perf_counter()
        for _ in range(5):
            pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream,
                              depth=args.depth, mode=mode)
        torch.cuda.synchronize()
        single_ms = (time.perf_counter() - ts) * 1e3 / 5
        single_phases = pkg.profile_end()
        lone = pkg.lone_frames_check()   # every lone frame's hand-off words (7 frames)
        lone_diag = pkg.resolver_stats(lone=True)
        md5 = pkg.p3_md5(out.cpu().numpy())
        single = {"ms": round(single_ms, 4), "value": round(W * H / (single_ms * 1e-3), 1),
                  "note": "one frame at a time (rc_render_device); phases_ms are its phases",
                  "verified": f"{lone['checked'] - lone['failed']}/7 hand-offs, last image md5 "
                              + ("== reference" if md5 == want_md5 else
                                 "(no golden)" if want_md5 is None else "MISMATCH"),
                  "resolver_diag": resolver_diag(lone_diag)}
        # phase C after the resolver on the whole device (side=0): the pixel kernels' own
        # time, for roofline_render (a lone frame's k_side runs beside the resolver and waits
        # for its carry-ins, so its span is not compute time)
        with pkg.tuned(side=0):
            pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream,
                              depth=args.depth, mode=mode)
            torch.cuda.synchronize()
            pkg.profile_begin()
            for _ in range(3):
                pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream,
                                  depth=args.depth, mode=mode)
            torch.cuda.synchronize()
            side0 = pkg.profile_end()
        pkg.lone_frames_check()
    for _ in range(args.warmup):
        step()
    drain()
    if parity and not piped and not sharded:
        pkg.lone_frames_check()   # the warmup frames: the timed region's count starts at 0
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    pkg.profile_begin()
    frame_no[0] = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    phases = pkg.profile_end()
    if single:
        phases = single_phases
        single["resolve_ms_in_flight"] = round(pipe_tim.get("resolve_ms", 0.0), 4)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if multi:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tmax = float(tmax.item())

    # ---- verification of the timed frames (outside the timed region) ----
    # hand-offs: every parity frame's latched carry hand-off words (rc_frames_wait /
    # rc_lone_frames_check); bytes: every frame's image against frame 0's on the device, and
    # frame 0's P3 md5 against the reference's golden
    diag = None   # the timed frames' own resolver record (rc_resolver_stats_get)
    if piped:
        hand = {"checked": int(pipe_tim.get("frames_checked", 0)),
                "failed": int(pipe_tim.get("frames_failed", 0))}
        diag = pkg.resolver_stats(lone=False)
    elif parity and not sharded:
        hand = pkg.lone_frames_check()
        diag = pkg.resolver_stats(lone=True)
    else:
        hand = None   # no carry hand-off in this mode (sharded: checked inside each call)
    if sharded:
        equal, md5, gold = (1, *verify_frames(pkg, [out], want_md5)[1:]) if rank == 0 else \
            (1, None, None)
        nframes = 1
    else:
        nframes = min(args.steps, len(outs))
        equal, md5, gold = verify_frames(pkg, outs[:nframes], want_md5)
    ok = nframes if (equal == nframes and gold is not False and
                     (hand is None or (hand["checked"] == args.steps and hand["failed"] == 0))) \
        else 0
    okt = torch.tensor([ok, nframes], dtype=torch.int64, device=cdev)
    if multi and not sharded:
        dist.all_reduce(okt)
    verified = {"frames": f"{int(okt[0])}/{int(okt[1])}",
                "bytes_equal_frame0": f"{equal}/{nframes}",
                "frame0_md5": md5,
                "frame0_vs_reference": ("equal" if gold else "MISMATCH" if gold is False
                                        else "no golden for this configuration"),
                "hand_offs": (f"{hand['checked'] - hand['failed']}/{args.steps}" if hand
                              else "n/a")}

    tim = {}
    shard_stats = group.stats() if sharded else None
    if piped:
        tim = pipe_tim
    elif sharded:
        tim = {"dep_pixels": shard_stats["dep_pixels"], "resolve_ms": shard_stats["resolve_ms"]}
        phases = {"local_ms": shard_stats["local_ms"],
                  "exchange_in_ms": shard_stats["exchange_in_ms"],
                  "resolve_ms": shard_stats["resolve_ms"], "phase_c_ms": shard_stats["phase_c_ms"],
                  "image_ms": shard_stats["image_ms"], "total_ms": shard_stats["device_ms"],
                  "render_ms": shard_stats["local_ms"] if not parity else 0.0,
                  "phase_a_ms": shard_stats["local_ms"] if parity else 0.0}
    elif not args.timed_only:
        pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream, depth=args.depth,
                          mode=mode, timing=tim)
    torch.cuda.synchronize()
    line = None
    if rank == 0:
        images = 1 if sharded else world
        value = images * W * H * args.steps / tmax
        work = WORK.get(f"{args.scene}:{args.size}:{args.depth}") if mode != "cuda" else None
        rows_here = H if not sharded else (H + world - 1) // world
        if parity:
            dom_name, dom_ms = "k_resolve", phases["resolve_ms"]
            if piped and pipe_tim.get("resolve_ms"):   # the launches of the timed region
                dom_ms = pipe_tim["resolve_ms"]
            dom_flop = (work["dep_flop_per_entry"] * tim["dep_pixels"]
                        if work and tim.get("dep_pixels") else None)
            if side0:   # phase A + phase C (k_dep_chunks after the resolver), whole device
                render_ms = side0["phase_a_ms"] + side0["phase_c_ms"]
                render_kernels = "k_phase_a + k_dep_chunks (phase C after the resolver, side=0)"
            else:
                render_ms = phases["phase_a_ms"] + phases["phase_c_ms"]
                render_kernels = "k_phase_a + phase C tail"
        else:
            dom_name, dom_ms = "k_render", phases["render_ms"]
            dom_flop = work["render_flop_per_px"] * W * rows_here if work else None
            render_ms = phases["render_ms"]
            render_kernels = "k_render"
        ach = dom_flop / (dom_ms * 1e-3) / 1e12 if dom_flop and dom_ms else None
        step_ms = tmax * 1e3 / args.steps
        # per step: the dominant kernel's algorithmic work of one image over the step time
        # (with frames in flight two resolvers overlap, so per-launch and per-step differ)
        ach_step = (dom_flop * images / world) / (step_ms * 1e-3) / 1e12 if dom_flop else None
        pmc, pmc_src = pmc_kernel(dom_name, args.scene, args.size, args.depth, mode,
                                  inflight=piped)
        store_name = "k_phase_a" if parity else "k_render"   # the framebuffer's writer
        spmc, spmc_src = pmc_kernel(store_name, args.scene, args.size, args.depth, mode)
        store_ms = phases["phase_a_ms"] if parity else phases["render_ms"]
        rach = (work["render_flop_per_px"] * W * rows_here / (render_ms * 1e-3) / 1e12
                if work and render_ms else None)
        fb_bytes = 3 * W * rows_here
        line = {
            "metric": ("primary rays/sec (= pixels/sec) at 4096x4096, quadric.scene"
                       if (args.scene, W) == ("quadric", 4096) else
                       f"primary rays/sec (= pixels/sec) at {W}x{H}, {args.scene}.scene"),
            "value": round(value, 1),
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic: the reference's own examples/" + args.scene + ".scene (no dataset)",
            "config": {"workload": f"{args.scene}.scene {W}x{H}, bounce depth {args.depth} "
                                   f"(MAX_RECURSION {args.depth + 1}), {mode} mode"
                                   + (", byte-identical to C/raycast.c" if mode == "parity" else ""),
                       "mode": mode, "width": W, "height": H, "depth": args.depth,
                       "parallelism": (f"row-cyclic shards x{world}, RCCL gather in the library "
                                       "(rc_render_sharded)" if sharded else
                                       (f"replicas x{world}" if world > 1 else "single GPU")),
                       "frames_in_flight": 2 if piped else 1,
                       "timed_region": (
                           ("device-resident: scene and output images in HBM, two parity frames "
                            "in flight (rc_frame_submit), no scene upload and no copy to the host; "
                            "the drop-in raycast() call (one image, upload + kernels + D2H into "
                            "the caller's pixmap) is `end_to_end`") if piped else
                           ("device-resident: one image per step, scene and output in HBM, no "
                            "scene upload and no copy to the host"
                            + ("; row-sharded over the group, gathered on rank 0" if sharded
                               else "")))},
            "verified": verified,
            "phases_ms": {k: round(v, 4) for k, v in phases.items() if k.endswith("_ms")},
            "tuning": ({t.split("=", 1)[0]: int(t.split("=", 1)[1]) for t in args.tune}
                       if args.tune else "default"),
            "dep_pixels": tim.get("dep_pixels"),
            "roofline": {"bound": "valu", "kernel": dom_name,
                         "kernel_ms": round(dom_ms, 4),
                         "achieved": round(ach, 4) if ach else None,
                         "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ach / PEAK_FP64_TFLOPS, 5) if ach else None,
                         "achieved_per_step": round(ach_step, 4) if ach_step else None,
                         "frac_per_step": round(ach_step / PEAK_FP64_TFLOPS, 5) if ach_step else None,
                         "traffic": pmc["hbm_bytes"] if pmc else None,
                         "traffic_unit": "bytes per launch (HBM, PMC)",
                         "valu_busy": pmc["valu_busy"] if pmc else None,
                         "frac_wait_any": pmc.get("frac_wait_any") if pmc else None,
                         "valu_busy_basis": ("all 256 CUs (a pipeline lane's resolver holds 64 of "
                                             "them: x4 for its own CUs)" if piped else
                                             "all 256 CUs"),
                         "pmc_source": pmc_src,
                         "note": ("serial carry chain: latency-bound, see DESIGN.md; frac = per "
                                  "launch, frac_per_step = one image's work over ms_per_step"
                                  if parity else "throughput kernel")},
            "roofline_render": {"bound": "valu", "kernel": render_kernels,
                                "kernel_ms": round(render_ms, 4),
                                "achieved": round(rach, 3) if rach else None,
                                "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                                "frac": round(rach / PEAK_FP64_TFLOPS, 4) if rach else None},
            # the framebuffer store (north_star): its 3 B/pixel over the writer kernel's time.
            # In parity the writer (k_phase_a) also writes the classes, writer carries and
            # DEP records; its whole PMC WRITE_SIZE is reported beside, labelled as such.
            "roofline_hbm": {"bound": "hbm", "kernel": store_name,
                             "what": "framebuffer store (3 B/pixel RGB) over the writer's time",
                             "achieved": (round(fb_bytes / (store_ms * 1e-3) / 1e9, 3)
                                          if store_ms else None),
                             "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": (round(fb_bytes / (store_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 5)
                                      if store_ms else None),
                             "framebuffer_bytes": fb_bytes,
                             "kernel_ms": round(store_ms, 4) if store_ms else None,
                             "kernel_write_bytes_pmc": spmc["write_bytes"] if spmc else None,
                             "kernel_write_gbs_pmc": (
                                 round(spmc["write_bytes"] / (store_ms * 1e-3) / 1e9, 3)
                                 if spmc and spmc.get("write_bytes") and store_ms else None),
                             "pmc_source": spmc_src},
        }
        if diag:
            line["resolver_diag"] = resolver_diag(diag)
        if single:
            line["single_frame"] = single
        if group_err:
            line["group_error"] = group_err
        if sharded:
            line["shard_stats"] = {k: (round(v, 4) if isinstance(v, float) else v)
                                   for k, v in shard_stats.items()}
        if world == 1 and not args.timed_only:
            line["end_to_end"] = end_to_end(pkg, scene, W, H, args.depth, mode)
            rates = {"value_is": ("frames_in_flight_device" if piped else "one_frame_device"),
                     "dropin_rate_is": "raycast_end_to_end (SURVEY.md §8d: upload + kernels + D2H)"}
            if piped:
                rates["frames_in_flight_device"] = {"value": round(value, 1),
                                                    "ms_per_frame": round(step_ms, 4)}
            if single:
                rates["one_frame_device"] = {"value": single["value"], "ms": single["ms"]}
            elif not piped and not sharded:
                rates["one_frame_device"] = {"value": round(value, 1), "ms": round(step_ms, 4)}
            rates["raycast_end_to_end"] = {"value": line["end_to_end"]["value"],
                                           "ms": line["end_to_end"]["ms"]}
            line["rates"] = rates
        if world == 1 and not args.no_cpu_baseline and not args.timed_only and mode != "cuda":
            line["cpu_baseline"] = cpu_baseline(scene_path, args.size, args.depth)
    # N>1 parity replicas: the sharded single image as well, reported beside (never as) value.
    # It is the only multi-process RCCL exchange of the run, so a watchdog bounds it: if it has
    # not finished in LEG_TIMEOUT_S, rank 0 prints the line with the leg marked as timed out
    # and every rank exits with LEG_TIMEOUT_EXIT.
    LEG_TIMEOUT_S = 120

    def shard_leg():
        nonlocal group, group_err
        if group is None:
            group, group_err = join_group()
            if group is None:   # every rank agreed no group formed: no collective is pending
                return {"group_error": f"no rc_group: {group_err}"}
        dist.barrier()
        group.render(scene, W, H, out.data_ptr(), depth=args.depth, mode=mode)   # warm
        dist.barrier()
        ts = time.perf_counter()
        reps = 5
        for _ in range(reps):
            group.render(scene, W, H, out.data_ptr(), depth=args.depth, mode=mode)
        dist.barrier()
        ms = (time.perf_counter() - ts) * 1e3 / reps
        st = group.stats()
        # every rank's own timeline of the last frame (rc_group_rank_stats), gathered over
        # torch.distributed outside the timed frames: where a rank's time goes
        mine = group.rank_stats(rank)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        leg = {"value": round(W * H / (ms * 1e-3), 1), "unit": "rays/s", "ms": round(ms, 4),
               "note": (f"one {W}x{H} image row-sharded over {world} GPUs (rc_render_sharded: "
                        "phase A on every rank, DEP entries and row blocks gathered to rank 0 "
                        "over RCCL, serial carry resolver there with phase C inside it); strong "
                        "scaling, capped by the resolver")
                       if world > 1 else
                       (f"one {W}x{H} image through rc_render_sharded with one rank: nothing "
                        "to exchange, the rank renders it as a lone frame" if pkg.get_tuning()[
                            "shard_lone"] else
                        f"one {W}x{H} image through rc_render_sharded's exchange with one rank "
                        "(rc_tuning.shard_lone = 0: wire records, gathers, the root's resolver)"),
               "stats": {k: (round(v, 4) if isinstance(v, float) else v)
                         for k, v in (st or {}).items()},
               "per_rank": [{k: (round(v, 4) if isinstance(v, float) else v)
                             for k, v in q.items()} if q else None for q in per_rank]}
        if rank == 0:
            m = pkg.p3_md5(out.cpu().numpy())
            leg["md5_vs_reference"] = ("equal" if m == want_md5 else "no golden"
                                       if want_md5 is None else "MISMATCH")
        return leg

    def leg_timed_out():
        if rank == 0:
            line["sharded_single_image"] = {"error": f"timed out after {LEG_TIMEOUT_S} s"}
            print(json.dumps(line), flush=True)

    shard_leg_res = None
    if (multi and backend == "nccl" and not sharded and not args.timed_only
            and group_err is None):
        shard_leg_res = run_leg_with_watchdog(shard_leg, LEG_TIMEOUT_S, leg_timed_out)
    if rank == 0:
        if shard_leg_res and "group_error" in shard_leg_res:
            line["group_error"] = shard_leg_res["group_error"]   # the replicas stand; exit 0
        elif shard_leg_res:
            line["sharded_single_image"] = shard_leg_res
        print(json.dumps(line), flush=True)
    if isinstance(shard_leg_res, dict) and "error" in shard_leg_res:
        # the exchange failed on this rank: the others may be left inside a collective, so no
        # teardown (it could block); the line is out, the status says the leg failed
        sys.stdout.flush()
        os._exit(LEG_TIMEOUT_EXIT)
    if group is not None:
        group.close()
    if multi:
        dist.destroy_process_group()
    if verified["frames"].split("/")[0] != verified["frames"].split("/")[1]:
        sys.exit(4)   # a timed frame failed its checks: the line is printed, the run fails


if __name__ == "__main__":
    main()
