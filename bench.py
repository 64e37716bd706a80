#!/usr/bin/env python3
"""Benchmark: primary rays/s (= pixels/s) rendering quadric.scene at 4096x4096, depth 6
(MAX_RECURSION 7, C/raycast.c:14) — BASELINE.json's metric.

A "step" is one full render of the image through the C-ABI (rc_render_device): scene
already resident in HBM, output written to a device buffer, every kernel of the mode
inside the timed region (parity mode: phase A + compaction + carry resolver + phase C).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode parity|fast]

N > 1 (torchrun, one rank per GPU): rows are dealt cyclically (row r -> rank r mod N), each
rank renders its rows, and the row blocks are gathered to rank 0 over RCCL (torch.distributed
"nccl" backend) and de-interleaved there — inside the timed region.  Parity mode at N > 1
needs the whole scan-order carry chain: see DESIGN.md §multi-GPU.

Rank 0 prints one JSON line (contract in the task statement) with a `roofline` object for
the dominant kernel (timed live with HIP events) and a `cpu_baseline` object (the reference
C/ build from oracle/_ref, timed on this host on one core; N=1 only).
"""
import argparse
import importlib.util
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

# Algorithmic work per pixel (SURVEY.md §8d weights applied to the oracle's exact per-pixel
# counts at this config; derivation in DESIGN.md §roofline).
FLOP_PER_PX = {"quadric:4096:6": 1380.0}
PEAK_FP64_TFLOPS = 78.6    # MI355X vector FP64 (MI355X_MICROARCH.md: FP32 157.3 / 2)
PEAK_HBM_GBS = 8000.0


def load_pkg():
    name = "raytracing_programs_amd"
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(scene_path, size, depth):
    """The reference itself (oracle/_ref/ref_timer_d<depth>: C/ sources, gcc -O3) rendering the
    same image on one host core; falls back to the CPU restatement (oracle/build)."""
    ref = os.path.join(ROOT, "oracle", "_ref", f"ref_timer_d{depth}")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    if os.path.exists(ref):
        cmd, kind = [ref, str(size), str(size), scene_path], "reference"
    else:
        cmd = [os.path.join(ROOT, "oracle", "build", "oracle_raytrace"), str(size), str(size),
               scene_path, "/dev/null", str(depth)]
        kind = "port"
    try:
        cmd = ["taskset", "-c", "0"] + cmd
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env,
                             check=True).stdout
        line = [l for l in out.splitlines() if l.startswith("{")][-1]
        r = json.loads(line)
        return {"value": round(r["rays_per_s"], 1), "unit": "rays/s", "cores": 1, "kind": kind,
                "sample": f"full {size}x{size} quadric.scene d{depth} render, raycast() only, "
                          f"1 pinned core ({r['seconds']:.2f} s)"}
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "rays/s", "cores": 1, "kind": kind, "sample": f"failed: {e}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="parity", choices=["parity", "fast"])
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--scene", default="quadric")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    pkg = load_pkg()
    scene_path = os.path.join(ROOT, "tests", "golden", "scenes", args.scene + ".scene")
    scene = pkg.Scene.from_file(scene_path)
    W = H = args.size
    mode = args.mode
    if world > 1 and mode == "parity":
        mode = "fast"   # the carry chain is not sharded yet
    nrows = (H - rank + world - 1) // world
    out = torch.empty((nrows, W, 3), dtype=torch.uint8, device="cuda")
    gathered = (torch.empty((world, (H + world - 1) // world, W, 3), dtype=torch.uint8,
                            device="cuda") if world > 1 else None)
    full = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda") if world > 1 else None
    stream = torch.cuda.current_stream()

    def step():
        pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream, depth=args.depth,
                          mode=mode, row0=rank, row_step=world, nrows=nrows)
        if world > 1:
            send = out
            pad = gathered.shape[1] - nrows
            if pad:
                send = torch.cat([out, out.new_zeros((pad, W, 3))])
            dist.all_gather_into_tensor(gathered, send)
            if rank == 0:   # row y lives in rank y % N at local row y // N
                full.copy_(gathered.permute(1, 0, 2, 3).reshape(-1, W, 3)[:H])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tmax = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tmax = float(tmax.item())

    # live kernel timing of the dominant kernel (HIP events on its stream, inside the lib)
    tim = {}
    pkg.render_device(scene, W, H, out.data_ptr(), stream.cuda_stream, depth=args.depth,
                      mode=mode, row0=rank, row_step=world, nrows=nrows, timing=tim)
    torch.cuda.synchronize()
    if rank == 0:
        value = W * H * args.steps / tmax
        key = f"{args.scene}:{args.size}:{args.depth}"
        flop_px = FLOP_PER_PX.get(key)
        main_ms = pkg.last_kernel_ms()   # phase A (parity) or k_render (fast)
        main_px = W * nrows
        achieved = (flop_px * main_px / (main_ms * 1e-3) / 1e12) if flop_px and main_ms else None
        line = {
            "metric": "primary rays/sec (= pixels/sec) at 4096x4096, quadric.scene",
            "value": round(value, 1),
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic: the reference's own examples/quadric.scene",
            "config": {"workload": f"{args.scene}.scene {W}x{H} depth {args.depth} "
                                   f"(MAX_RECURSION {args.depth + 1}), mode {mode}",
                       "mode": mode, "width": W, "height": H, "depth": args.depth,
                       "parallelism": f"rows-cyclic x{world}"},
            "phases_ms": {k: round(v, 4) for k, v in tim.items() if k.endswith("_ms")},
            "dep_pixels": tim.get("dep_pixels"),
            "roofline": {"bound": "valu", "kernel": "k_phase_a" if mode == "parity" else "k_render",
                         "achieved": round(achieved, 3) if achieved else None,
                         "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP64_TFLOPS, 5) if achieved else None,
                         "traffic": None},
            "roofline_hbm": {"bound": "hbm", "kernel": "framebuffer store",
                             "achieved": round(3 * W * H / (tmax / args.steps) / 1e9, 3),
                             "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(3 * W * H / (tmax / args.steps) / 1e9 / PEAK_HBM_GBS, 6),
                             "traffic": None},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(scene_path, args.size, args.depth)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
