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
Fast mode: one render kernel per frame.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode parity|fast] [--inflight 1|2]

Multi-GPU (torchrun, one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE from the env):
  parity: the image's scan-order carry chain is one serial dependency,
          so the path does not shard: every rank renders its own full image (replicas, no
          data-path collective) and `value` = N images' pixels / max rank time ("weak").
  fast:   rows dealt cyclically (row r -> rank r mod N), each rank renders its rows, the row
          blocks are gathered over RCCL (all_gather_into_tensor, "nccl" backend) and
          de-interleaved on rank 0 inside the timed region ("strong").

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
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

# Algorithmic work: SURVEY.md §8d's per-operation weights (sphere test
# 29, plane 15, quadric 81, hit post-processing ~26, light setup 18, unshadowed light 70,
# reflect+normalize 21, ray generation 15) applied to the exact per-pixel work counts of
# the reference at this config (oracle counters, quadric 4096^2 depth 6).
WORK = {
    "quadric:4096:6": {"render_flop_per_px": 1374.0,   # full render, every pixel
                       "dep_flop_per_entry": 1618.0},  # one carry transfer function
}
PEAK_FP64_TFLOPS = 78.6    # MI355X vector FP64 (MI355X_MICROARCH.md: FP32 157.3 / 2)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E


def load_pkg():
    name = "raytracing_programs_amd"
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def pmc_traffic(kernel, scene, size, depth, mode):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this
    exact configuration (profiles/r01_pmc_traffic_<size>.json: 2*FETCH_SIZE + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md); None when no profile covers it."""
    path = os.path.join(ROOT, "profiles", f"r01_pmc_traffic_{size}.json")
    if scene != "quadric" or depth != 6 or not os.path.exists(path):
        return None, None
    with open(path) as f:
        prof = json.load(f)
    if mode not in prof.get("config", ""):
        return None, None
    for name, d in prof["kernels"].items():
        if name.split("::")[-1].split("<")[0] == kernel and "hbm_bytes" in d:
            return d["hbm_bytes"], os.path.relpath(path, ROOT)
    return None, None


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


def cpu_baseline(scene_path, size, depth):
    """The reference itself (oracle/_ref/ref_timer_d<depth>: the C/ sources built like
    C/Makefile:4, raycast() timed alone) on the same image on one pinned host core; falls
    back to the CPU restatement (oracle/build) when the reference build is absent."""
    ref = os.path.join(ROOT, "oracle", "_ref", f"ref_timer_d{depth}")
    if os.path.exists(ref):
        cmd, kind = [ref, str(size), str(size), scene_path], "reference"
    else:
        cmd = [os.path.join(ROOT, "oracle", "build", "oracle_raytrace"), str(size), str(size),
               scene_path, "/dev/null", str(depth)]
        kind = "port"
    try:
        try:
            core = sorted(os.sched_getaffinity(0))[0]
            cmd = ["taskset", "-c", str(core)] + cmd
        except (AttributeError, OSError):
            pass
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True).stdout
        r = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
        return {"value": round(r["rays_per_s"], 1), "unit": "rays/s", "cores": 1, "kind": kind,
                "sample": f"full {size}x{size} quadric.scene depth {depth} render, raycast() "
                          f"only, 1 pinned core: {r['seconds']:.2f} s"}
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "rays/s", "cores": 1, "kind": kind, "sample": f"failed: {e}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="parity", choices=["parity", "fast"])
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
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("RC_BENCH_BACKEND", "nccl") != "nccl":   # 1-GPU rehearsal: ranks share GPUs
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        backend = os.environ.get("RC_BENCH_BACKEND", "nccl")   # gloo: 1-GPU rehearsal only
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    pkg = load_pkg()
    scene_path = os.path.join(ROOT, "tests", "golden", "scenes", args.scene + ".scene")
    scene = pkg.Scene.from_file(scene_path)
    W = H = args.size
    mode = args.mode
    sharded = world > 1 and mode == "fast"
    if sharded:
        row0, step_rows, nrows = pkg.row_shard(H, rank, world)
    else:
        row0, step_rows, nrows = 0, 1, H
    out = torch.empty((nrows, W, 3), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    if sharded:
        rows_max = (H + world - 1) // world
        gathered = torch.empty((world, rows_max, W, 3), dtype=torch.uint8, device="cuda")
        send = torch.zeros((rows_max, W, 3), dtype=torch.uint8, device="cuda")
        full = torch.empty((rows_max * world, W, 3), dtype=torch.uint8, device="cuda")

    piped = mode == "parity" and args.depth > 0 and args.inflight == 2 and not sharded
    if piped:   # every frame of the timed region gets its own output image
        outs = [torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
                for _ in range(max(args.steps, 1))]
        torch.cuda.synchronize()
    frame_no = [0]

    def step():
        if piped:
            buf = outs[frame_no[0] % len(outs)]
            frame_no[0] += 1
            pkg.frame_submit(scene, W, H, buf.data_ptr(), depth=args.depth, mode=mode)
            return
        if sharded:
            pkg.render_device(scene, W, H, send.data_ptr(), stream.cuda_stream, depth=args.depth,
                              mode=mode, row0=row0, row_step=step_rows, nrows=nrows)
            pkg.gather_rows(send, gathered, dist)
            if rank == 0:   # image row y lives on rank y % N at local row y // N
                full.copy_(pkg.deinterleave(gathered, rows_max * world))
        else:
            pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream, depth=args.depth,
                              mode=mode)

    def drain():
        if piped:
            pkg.frames_wait(pipe_tim)
        torch.cuda.synchronize()

    pipe_tim = {}
    single = None
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
        single = {"ms": round(single_ms, 4), "value": round(W * H / (single_ms * 1e-3), 1),
                  "note": "one frame at a time (rc_render_device); phases_ms are its phases"}
    for _ in range(args.warmup):
        step()
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    pkg.profile_begin()
    frame_no[0] = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    phases = pkg.profile_end()
    if single:
        phases = single_phases
        single["resolve_ms_in_flight"] = round(pipe_tim.get("resolve_ms", 0.0), 4)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tmax = float(tmax.item())

    tim = {}
    if piped:
        tim = pipe_tim
    elif not args.timed_only:
        pkg.render_device(scene, W, H, (send if sharded else out).data_ptr(), stream.cuda_stream,
                          depth=args.depth, mode=mode, row0=row0, row_step=step_rows,
                          nrows=nrows, timing=tim)
    torch.cuda.synchronize()
    if rank == 0:
        images = 1 if sharded else world
        value = images * W * H * args.steps / tmax
        work = WORK.get(f"{args.scene}:{args.size}:{args.depth}")
        parity = mode == "parity" and args.depth > 0
        if parity:
            dom_name, dom_ms = "k_resolve", phases["resolve_ms"]
            if piped and pipe_tim.get("resolve_ms"):   # the launches of the timed region
                dom_ms = pipe_tim["resolve_ms"]
            dom_flop = (work["dep_flop_per_entry"] * tim["dep_pixels"]
                        if work and tim.get("dep_pixels") else None)
            render_ms = phases["phase_a_ms"] + phases["phase_c_ms"]
        else:
            dom_name, dom_ms = "k_render", phases["render_ms"]
            dom_flop = work["render_flop_per_px"] * W * nrows if work else None
            render_ms = phases["render_ms"]
        ach = dom_flop / (dom_ms * 1e-3) / 1e12 if dom_flop and dom_ms else None
        traffic, traffic_src = pmc_traffic(dom_name, args.scene, args.size, args.depth, mode)
        rach = (work["render_flop_per_px"] * W * nrows / (render_ms * 1e-3) / 1e12
                if work and render_ms else None)
        line = {
            "metric": "primary rays/sec (= pixels/sec) at 4096x4096, quadric.scene",
            "value": round(value, 1),
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic: the reference's own examples/quadric.scene (no dataset)",
            "config": {"workload": f"{args.scene}.scene {W}x{H}, bounce depth {args.depth} "
                                   f"(MAX_RECURSION {args.depth + 1}), {mode} mode"
                                   + (", byte-identical to C/raycast.c" if mode == "parity" else ""),
                       "mode": mode, "width": W, "height": H, "depth": args.depth,
                       "parallelism": (f"rows-cyclic x{world} + RCCL all_gather" if sharded else
                                       (f"replicas x{world}" if world > 1 else "single GPU")),
                       "frames_in_flight": 2 if piped else 1},
            "phases_ms": {k: round(v, 4) for k, v in phases.items() if k.endswith("_ms")},
            "dep_pixels": tim.get("dep_pixels"),
            "roofline": {"bound": "valu", "kernel": dom_name,
                         "kernel_ms": round(dom_ms, 4),
                         "achieved": round(ach, 4) if ach else None,
                         "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(ach / PEAK_FP64_TFLOPS, 5) if ach else None,
                         "traffic": traffic,
                         "traffic_unit": "bytes per launch (HBM, PMC)",
                         "traffic_source": traffic_src,
                         "note": ("serial carry chain: latency-bound, see DESIGN.md" if parity
                                  else "throughput kernel")},
            "roofline_render": {"bound": "valu",
                                "kernel": "k_phase_a+k_phase_c" if parity else "k_render",
                                "kernel_ms": round(render_ms, 4),
                                "achieved": round(rach, 3) if rach else None,
                                "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                                "frac": round(rach / PEAK_FP64_TFLOPS, 4) if rach else None},
            "roofline_hbm": {"bound": "hbm", "kernel": "framebuffer store (3 B/pixel)",
                             "achieved": round(3 * W * nrows / (phases["total_ms"] * 1e-3) / 1e9, 3)
                             if phases["total_ms"] else None,
                             "peak": PEAK_HBM_GBS, "unit": "GB/s"},
        }
        if single:
            line["single_frame"] = single
        if world == 1 and not sharded and not args.timed_only:
            line["end_to_end"] = end_to_end(pkg, scene, W, H, args.depth, mode)
        if world == 1 and not args.no_cpu_baseline and not args.timed_only:
            line["cpu_baseline"] = cpu_baseline(scene_path, args.size, args.depth)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
