"""Repeated lone parity frames (rc_render_device, quadric 4096^2 d6) under a tuning, to
estimate how often a resolver hand-off times out (the frame then fails loudly).  Stops at the
first failure of each schedule.  Usage: python scripts/stall_stress.py FRAMES [name:k=v,k=v ...]"""
import importlib.util
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location(
    "raytracing_programs_amd", os.path.join(ROOT, "raytracing-programs_amd", "__init__.py"))
pkg = importlib.util.module_from_spec(spec)
sys.modules["raytracing_programs_amd"] = pkg
spec.loader.exec_module(pkg)

frames = int(sys.argv[1])
scheds = []
for a in sys.argv[2:] or ["default:"]:
    name, _, kv = a.partition(":")
    scheds.append((name, {k: int(v) for k, v in (p.split("=") for p in kv.split(",") if p)}))
scene = pkg.Scene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "quadric.scene"))
W = H = 4096
out = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda:0")
for name, tune in scheds:
    t0 = time.time()
    done = 0
    with pkg.tuned(**tune):
        for i in range(frames):
            try:
                pkg.render_device(scene, W, H, out.data_ptr())
                torch.cuda.synchronize()
                if pkg.lone_frames_check()["failed"]:
                    raise RuntimeError("lone_frames_check reports a failed frame")
            except RuntimeError as e:
                print(f"{name}: FAILED at frame {i} after {time.time() - t0:.1f} s: {e}", flush=True)
                break
            done += 1
            if i % 100 == 99:
                print(f"{name}: {i + 1} frames ok ({time.time() - t0:.1f} s)", flush=True)
    print(f"{name} {tune}: {done}/{frames} frames ok", flush=True)
